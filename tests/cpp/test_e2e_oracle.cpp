// test_e2e_oracle.cpp — TEST INFRASTRUCTURE (CPU, no GPU): the end-to-end host driver
// (omp-bowtie2-prime_amd/host/bt2x_align.cpp: per-read coroutine, prioritizeSATups,
// extendSeeds, reporting, MAPQ, SAM) run with the CPU oracle standing in for the three
// kernels, so the host logic can be pinned against the reference's own SAM output
// (tests/golden/*.sam.xz) on a machine without a GPU.  The product binary
// (bt2x-align) links only libbt2x.so and is checked against the same goldens on the
// GPU (tests/test_e2e.py, -m gpu).  The kernels' own parity with the oracle is
// tested separately (tests/test_gpu_parity.py).
//
//   test_e2e_oracle <index base> <reads.fq> [--dpad N] [--slots N] [-p T]
#include <chrono>
#include <csignal>
#include <sys/resource.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../omp-bowtie2-prime_amd/host/bt2x_align.hpp"
#include "../../oracle/bt2x_oracle.h"

using namespace bt2x::host;

namespace {
class OracleBackend : public Backend {
public:
	OracleBackend(const bt2x_index_desc& idx, const bt2x_scoring& sc, const RefInfo* ref = nullptr)
		: idx_(idx), sc_(sc), ref_(ref) {}
	// with a RefInfo: DP problems name their windows (BT2X_DP_REF_TEXT) as with the GPU
	// backend, and the windows are cut here
	bool ref_from_index() const override { return ref_ != nullptr; }
	// --inject-error N: the Nth DP launch throws, as a failing GPU call would (bt2x::check)
	int fail_at = 0;
	void seed_search(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& in,
	                 HostVec<bt2x_seed_out>& out) override {
		out.resize(in.size());
		if(bt2o_seed_search(&idx_, reads.data(), in.data(), (uint32_t)in.size(), 1, out.data(), nullptr) != 0)
			throw std::runtime_error("oracle seed search");
	}
	void resolve(const HostVec<bt2x_resolve_in>& in, HostVec<bt2x_resolve_out>& out) override {
		out.resize(in.size());
		if(bt2o_resolve(&idx_, in.data(), (uint32_t)in.size(), 0, out.data(), nullptr) != 0)
			throw std::runtime_error("oracle resolve");
	}
	void dp_align(const HostVec<uint8_t>& reads, const HostVec<uint8_t>& quals,
	              const HostVec<uint8_t>& refs, const HostVec<bt2x_dp_in>& in,
	              HostVec<bt2x_dp_out>& out, HostVec<bt2x_aln_rec>& recs,
	              HostVec<uint32_t>& edits) override {
		if(fail_at > 0 && ++ndp_ == fail_at) throw bt2x::Error(BT2X_E_NODEVICE, "injected backend error");
		const uint32_t n = (uint32_t)in.size();
		out.resize(n);
		const uint8_t* rf = refs.data();
		const bt2x_dp_in* pin = in.data();
		std::vector<uint8_t> win;
		std::vector<bt2x_dp_in> in2;
		if(ref_) {                                           // BitPairReference::getStretch per problem
			in2.assign(in.begin(), in.end());
			for(bt2x_dp_in& q : in2) {
				if(!(q.flags & BT2X_DP_REF_TEXT)) continue;
				const size_t o = win.size();
				win.resize(o + q.ncol);
				ref_->stretch((uint32_t)q.ref_off, q.refl, q.ncol, win.data() + o);
				q.ref_off = o;
				q.flags &= (uint8_t)~BT2X_DP_REF_TEXT;
			}
			rf = win.data();
			pin = in2.data();
		}
		uint32_t rec_cap = 4 * n + 64, edit_cap = 48 * n + 256;
		for(int attempt = 0; attempt < 2; attempt++) {
			recs.resize(rec_cap); edits.resize(edit_cap);
			uint32_t nrec = 0, ned = 0;
			const int rc = bt2o_dp_align(&sc_, reads.data(), quals.data(), rf, pin, n, out.data(),
			                             recs.data(), rec_cap, &nrec, edits.data(), edit_cap, &ned, nullptr, nullptr);
			if(rc == BT2X_E_OVERFLOW && attempt == 0) { rec_cap = nrec; edit_cap = ned; continue; }
			if(rc != 0) throw std::runtime_error("oracle dp");
			recs.resize(nrec); edits.resize(ned);
			return;
		}
	}
	// the oracle seed search, then the host restatement of the round (host_round), then
	// the oracle SA resolution: the contract of bt2x_seed_round on the CPU
	void seed_round(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& seeds,
	                const HostVec<bt2x_round_in>& in, const HostVec<bt2x_exrange>& exr, uint32_t maxelt,
	                HostVec<bt2x_round_out>& out, HostVec<bt2x_sat>& sats, HostVec<bt2x_elt>& elts,
	                HostVec<bt2x_exrange>& exr_out) override {
		HostVec<bt2x_seed_out> so;
		seed_search(reads, seeds, so);
		out.resize(in.size());
		std::vector<bt2x_sat> sv;
		std::vector<bt2x_exrange> xv;
		std::vector<bt2x_resolve_in> rows;
		RoundScratch w;
		for(size_t r = 0; r < in.size(); r++) {
			const bt2x_round_in& q = in[r];
			Rng rnd;
			rnd.last = q.rnd_last; rnd.lastOff = q.rnd_lastoff;
			const uint32_t s0 = (uint32_t)sv.size(), e0 = (uint32_t)rows.size(), x0 = (uint32_t)xv.size();
			host_round(q, seeds.data() + q.seed0, so.data() + q.seed0, exr.data() + q.exr0, maxelt, rnd, w, out[r],
			           sv, rows, xv);
			out[r].sat0 = s0; out[r].elt0 = e0; out[r].exr0 = x0;
		}
		sats.assign(sv.begin(), sv.end());
		exr_out.assign(xv.begin(), xv.end());
		HostVec<bt2x_resolve_out> ro;
		resolve(HostVec<bt2x_resolve_in>(rows.begin(), rows.end()), ro);
		elts.resize(ro.size());
		for(size_t k = 0; k < ro.size(); k++) elts[k] = bt2x_elt_pack(ro[k].toff, ro[k].tidx, ro[k].straddled);
	}
private:
	const bt2x_index_desc& idx_;
	const bt2x_scoring& sc_;
	const RefInfo* ref_;
	int ndp_ = 0;
};

// --host-timing: the second run answers every launch from the first run's recorded
// outputs (the driver is deterministic), so its wall time is the host driver's alone.
class ReplayBackend : public Backend {
public:
	explicit ReplayBackend(Backend* rec) : rec_(rec), ref_index_(rec->ref_from_index()) {}
	bool ref_from_index() const override { return ref_index_; }
	void rewind() { rec_ = nullptr; k_ = kr_ = kd_ = kn_ = 0; }
	void seed_search(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& in,
	                 HostVec<bt2x_seed_out>& out) override {
		if(rec_) { rec_->seed_search(reads, in, out); seeds_.push_back(out); } else out = seeds_[k_++];
	}
	void resolve(const HostVec<bt2x_resolve_in>& in, HostVec<bt2x_resolve_out>& out) override {
		if(rec_) { rec_->resolve(in, out); res_.push_back(out); } else out = res_[kr_++];
	}
	void dp_align(const HostVec<uint8_t>& reads, const HostVec<uint8_t>& quals,
	              const HostVec<uint8_t>& refs, const HostVec<bt2x_dp_in>& in,
	              HostVec<bt2x_dp_out>& out, HostVec<bt2x_aln_rec>& recs,
	              HostVec<uint32_t>& edits) override {
		if(rec_) { rec_->dp_align(reads, quals, refs, in, out, recs, edits); dp_.push_back({out, recs, edits}); }
		else { const auto& d = dp_[kd_++]; out = d.out; recs = d.recs; edits = d.edits; }
	}
	void seed_round(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& seeds,
	                const HostVec<bt2x_round_in>& in, const HostVec<bt2x_exrange>& exr, uint32_t maxelt,
	                HostVec<bt2x_round_out>& out, HostVec<bt2x_sat>& sats, HostVec<bt2x_elt>& elts,
	                HostVec<bt2x_exrange>& exr_out) override {
		if(rec_) {
			rec_->seed_round(reads, seeds, in, exr, maxelt, out, sats, elts, exr_out);
			rounds_.push_back({out, sats, elts, exr_out});
		} else {
			const auto& d = rounds_[kn_++];
			out = d.out; sats = d.sats; elts = d.elts; exr_out = d.exr;
		}
	}
private:
	struct Round { HostVec<bt2x_round_out> out; HostVec<bt2x_sat> sats; HostVec<bt2x_elt> elts;
	               HostVec<bt2x_exrange> exr; };
	std::vector<Round> rounds_;
	size_t kn_ = 0;
	struct Dp { HostVec<bt2x_dp_out> out; HostVec<bt2x_aln_rec> recs; HostVec<uint32_t> edits; };
	Backend* rec_;
	bool ref_index_;
	size_t k_ = 0, kr_ = 0, kd_ = 0;
	std::vector<HostVec<bt2x_seed_out>> seeds_;
	std::vector<HostVec<bt2x_resolve_out>> res_;
	std::vector<Dp> dp_;
};
}

int main(int argc, char** argv) {
	tune_malloc();
	// test_e2e_oracle <index> <reads.fq> [options], or bt2x-align's -x/-U/-S form (the
	// multi-process launcher drives it as it drives bt2x-align)
	const char* usage = "usage: test_e2e_oracle <index> <reads.fq>[,more.fq] [--dpad N] [--slots N] [-p T] [--shard i/N] "
	                    "[--no-hd] [--metrics] [-S out]\n";
	Params p;
	size_t slots = 4096;
	int threads = 4;
	bool host_timing = false, pipeline = true, gpu_round = true, hd = true, metrics = false, host_windows = false;
	int reps = 1, inject = 0, shard = 0, nshards = 1, warm_files = 0, streams = 1;
	std::string idx, fqs, outp;
	std::vector<std::string> pos;
	for(int i = 1; i < argc; i++) {
		if(const int k = parse_align_option(p, argc, argv, i)) { i += k - 1; continue; }
		const std::string a = argv[i];
		if(a == "--slots" && i + 1 < argc) slots = (size_t)std::atol(argv[++i]);
		else if(a == "-p" && i + 1 < argc) threads = std::atoi(argv[++i]);
		else if(a == "-x" && i + 1 < argc) idx = argv[++i];
		else if(a == "-U" && i + 1 < argc) fqs = argv[++i];
		else if(a == "-S" && i + 1 < argc) outp = argv[++i];
		else if(a == "--host-timing") host_timing = true;
		else if(a == "--no-pipeline") pipeline = false;
		else if(a == "--streams" && i + 1 < argc) streams = std::atoi(argv[++i]);
		else if(a == "--no-gpu-round") gpu_round = false;
		else if(a == "--no-hd") hd = false;
		else if(a == "--host-windows") host_windows = true;
		else if(a == "--metrics") metrics = true;
		// bt2x-align's bench options (bench.py drives this binary as it drives bt2x-align in the
		// CPU test of its multi-rank path): --device and --stats are accepted and ignored
		else if(a == "--device" && i + 1 < argc) ++i;
		else if(a == "--stats") {}
		else if(a == "--warmup-files" && i + 1 < argc) warm_files = std::atoi(argv[++i]);
		else if(a == "--cpus" && i + 1 < argc) {               // bt2x-align's per-rank CPU set
			try { apply_cpu_list(argv[++i]); } catch(const std::exception& e) { std::fprintf(stderr, "%s\n", e.what()); return 1; }
			std::fprintf(stderr, "BT2X_CPUS %s\n", affinity_list().c_str());
		}
		else if(a == "--reps" && i + 1 < argc) reps = std::atoi(argv[++i]);
		else if(a == "--inject-error" && i + 1 < argc) inject = std::atoi(argv[++i]);
		else if(a == "--shard" && i + 1 < argc) {
			if(std::sscanf(argv[++i], "%d/%d", &shard, &nshards) != 2) { std::fputs(usage, stderr); return 1; }
		}
		else if(a[0] != '-') pos.push_back(a);
		else { std::fprintf(stderr, "unsupported option %s\n", a.c_str()); return 1; }
	}
	if(idx.empty() && !pos.empty()) idx = pos[0];
	if(fqs.empty() && pos.size() > 1) fqs = pos[1];
	if(idx.empty() || fqs.empty()) { std::fputs(usage, stderr); return 1; }
	const std::vector<std::string> files = split_list(fqs);
	std::FILE* out = stdout;
	if(!outp.empty() && !(out = std::fopen(outp.c_str(), "wb"))) { std::fprintf(stderr, "cannot open %s\n", outp.c_str()); return 1; }
	bt2x_scoring_init(&p.sc);
	bt2x::Index index(idx.c_str(), true);
	RefInfo ref;
	ref.init(index.desc(), idx);
	// windows named by the problems and cut by the backend (the GPU backend's mode), or cut by
	// the driver (--host-windows)
	OracleBackend be(index.desc(), p.sc, host_windows ? nullptr : &ref);
	be.fail_at = inject;
	if(host_timing) {
		ReplayBackend rb(&be);
		// one aligner for the recording pass and the timed replays, as bt2x-align keeps one
		// for its --warmup-files run and the timed run (pooled read contexts, warm heap)
		Aligner al(p, ref, rb);
		al.set_pipeline(pipeline);
		al.set_gpu_round(gpu_round);
		{
			FastqReader fq(files, shard, nshards);
			std::FILE* nul = std::fopen("/dev/null", "wb");
			al.run(fq, nul, slots, threads);
			std::fclose(nul);
		}
		for(int rep = 0; rep < reps; rep++) {
		rb.rewind();
		// tools/sprof.c: profile the replay only (SPROF_SKIP=k: not the first k replays)
		const bool prof = std::getenv("SPROF_WAIT") && rep >= (std::getenv("SPROF_SKIP") ? std::atoi(std::getenv("SPROF_SKIP")) : 0);
		if(prof) std::raise(SIGUSR2);
		FastqReader fq(files, shard, nshards);
		struct rusage ru0, ru1;
		getrusage(RUSAGE_SELF, &ru0);
		const auto t0 = std::chrono::steady_clock::now();
		double t_run = 0;
		const RunStats st = al.run(fq, stdout, slots, threads, &t_run);
		const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
		getrusage(RUSAGE_SELF, &ru1);
		if(prof) std::raise(SIGUSR2);   // ... and not the teardown
		auto sec = [](const timeval& a, const timeval& b) { return (b.tv_sec - a.tv_sec) + (b.tv_usec - a.tv_usec) * 1e-6; };
		std::fprintf(stderr, "HOST_TIMING rusage user=%.3f sys=%.3f minflt=%ld vcsw=%ld\n", sec(ru0.ru_utime, ru1.ru_utime),
		             sec(ru0.ru_stime, ru1.ru_stime), ru1.ru_minflt - ru0.ru_minflt, ru1.ru_nvcsw - ru0.ru_nvcsw);
		std::fprintf(stderr, "HOST_TIMING t_alloc=%.3f t_step=%.3f t_wait=%.3f t_backend=%.3f t_gather=%.3f t_retire=%.3f t_run=%.3f\n",
		             st.t_alloc, st.t_step, st.t_wait, st.t_backend, st.t_gather, st.t_retire, t_run);
		std::fprintf(stderr, "HOST_TIMING reads=%llu wall=%.3f t_host=%.3f t_io=%.3f t_seed=%.3f t_resolve=%.3f t_dp=%.3f "
		             "launches=%llu/%llu/%llu dps=%llu dps_used=%llu\n", (unsigned long long)st.reads, t, st.t_host, st.t_io, st.t_seed,
		             st.t_resolve, st.t_dp, (unsigned long long)st.seed_launches,
		             (unsigned long long)st.resolve_launches, (unsigned long long)st.dp_launches, (unsigned long long)st.dps, (unsigned long long)st.dps_used);
		}
		return 0;
	}
	Aligner al(p, ref, be);
	al.set_pipeline(pipeline);
	al.set_gpu_round(gpu_round);
	al.set_header(hd);
	// --streams 2: the second cohort's launches on a backend of their own (bt2x-align's two
	// contexts), so the two GPU threads run concurrently
	OracleBackend be2(index.desc(), p.sc, host_windows ? nullptr : &ref);
	be2.fail_at = inject;
	if(streams >= 2) al.set_second_backend(&be2);
	RunStats st;
	uint64_t first_rdid = 0;
	double t_align = 0;
	if(warm_files < 0 || (size_t)warm_files >= files.size()) { std::fprintf(stderr, "--warmup-files must leave a file\n"); return 1; }
	try {
		uint64_t warm_records = 0;
		if(warm_files > 0) {                              // untimed, unwritten (bt2x-align --warmup-files)
			FastqReader wr(std::vector<std::string>(files.begin(), files.begin() + warm_files), shard, nshards);
			std::FILE* nul = std::fopen("/dev/null", "wb");
			al.run(wr, nul, slots, threads);
			std::fclose(nul);
			for(int k = 0; k < warm_files; k++) warm_records += FastqReader::count_file_records(files[(size_t)k]);
		}
		FastqReader fq(std::vector<std::string>(files.begin() + warm_files, files.end()), shard, nshards, warm_records);
		first_rdid = fq.first_rdid();
		const auto t0 = std::chrono::steady_clock::now();
		st = al.run(fq, out, slots, threads);
		t_align = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
	} catch(const std::exception& e) {               // as bt2x-align's main does
		std::fprintf(stderr, "test_e2e_oracle: %s\n", e.what());
		return 1;
	}
	if(out != stdout) std::fclose(out); else std::fflush(out);
	if(metrics) {                                     // bt2x-align --metrics' lines
		print_alignment_summary(st.met, stderr);
		std::string line = "BT2X_METRICS";
		for(uint64_t v : st.met.v) line += " " + std::to_string(v);
		std::string tf;
		for(double t : st.t_files) { char b[32]; std::snprintf(b, sizeof b, "%s%.4f", tf.empty() ? "" : ",", t); tf += b; }
		std::fprintf(stderr, "%s\nBT2X_TIMED reads=%llu first_rdid=%llu t_align=%.4f t_files=%s\n", line.c_str(),
		             (unsigned long long)st.reads, (unsigned long long)first_rdid, t_align, tf.c_str());
	}
	std::fprintf(stderr, "reads=%llu aligned=%llu seed_launches=%llu resolve_launches=%llu dp_launches=%llu dps=%llu "
	             "tight_recs=%llu\n",
	             (unsigned long long)st.reads, (unsigned long long)st.aligned, (unsigned long long)st.seed_launches,
	             (unsigned long long)st.resolve_launches, (unsigned long long)st.dp_launches, (unsigned long long)st.dps,
	             (unsigned long long)st.tight_recs);
	return 0;
}
