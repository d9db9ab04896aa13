// bt2x-align — the MI355X aligner's command line: the subset of bowtie2-align-l's
// options this fork honours for unpaired end-to-end alignment (bt2_search.cpp:446-643),
// FASTQ in, SAM out.  All hot-path work runs on one GPU through libbt2x (include/bt2x.h);
// there is no CPU fallback.
//
//   bt2x-align -x <index base> {-U <r1.fq>[,r2.fq,...] | -1 <m1.fq> -2 <m2.fq>} [-S out.sam] [--dpad N] [-D N] [-R N]
//              [-L N] [-i FUNC] [--score-min FUNC] [--n-ceil FUNC] [--mp MX,MN] [--np N]
//              [--rdg O,E] [--rfg O,E] [--gbar N] [--seed N] [--no-sse8] [--i16-build]
//              [--no-hd] [-p threads] [--slots N] [--device N] [--stats]
//              [--shard i/N] [--warmup-files K] [--metrics]
// --shard i/N aligns the i-th of N contiguous parts of the read stream (FastqReader); the
// N outputs concatenated in order (headers from part 0 only: --no-hd on the others) are
// the whole run's SAM.  --warmup-files K aligns the first K files of the -U list once,
// untimed and unwritten, before the timed run over the rest (bench.py); unnamed reads of
// the rest keep their numbers in the whole list.  --metrics prints
// the 27 ReportingMetrics counters (BT2X_METRICS) and the run's clock (BT2X_TIMED) for a
// launcher to sum over shards.
// --no-sse8 runs the signed 16-bit DP as the reference's -DENABLE_I16 build does
// (aligner_swsse_ee_i16.cpp); --i16-build emulates that build's default (u8 unless the
// minimum score is below -254).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include <csignal>
#include <sched.h>
#include <sys/resource.h>

#include "bt2x_align.hpp"

using namespace bt2x::host;

namespace {

// Page-locked blocks by power-of-two class, kept for reuse: pinning and unpinning cost
// milliseconds per call (0.6 s of a 1 M-read run when the launch buffers grew through
// hipHostMalloc/hipHostFree directly), so a freed block waits for the next request of
// its class instead of going back to the driver.
class PinnedCache {
public:
	static void* alloc(size_t n) { return inst().get(n); }
	static void release(void* p) { inst().put(p); }
	// one block for each later request of n bytes in `sizes`
	static void prefill(const std::vector<size_t>& sizes) {
		std::vector<void*> got;
		for(size_t n : sizes) if(void* p = inst().get(n)) got.push_back(p);
		for(void* p : got) inst().put(p);
	}
private:
	static constexpr size_t kHdr = 64;
	static PinnedCache& inst() { static PinnedCache c; return c; }
	void* get(size_t n) {
		int cls = 12;
		while(((size_t)1 << cls) < n + kHdr) cls++;
		{
			std::lock_guard<std::mutex> g(mu_);
			if(!free_[cls].empty()) { void* p = free_[cls].back(); free_[cls].pop_back(); return p; }
		}
		uint8_t* b = static_cast<uint8_t*>(bt2x_host_alloc((size_t)1 << cls));
		if(!b) return nullptr;
		*reinterpret_cast<int*>(b) = cls;
		return b + kHdr;
	}
	void put(void* p) {
		uint8_t* b = static_cast<uint8_t*>(p) - kHdr;
		const int cls = *reinterpret_cast<int*>(b);
		std::lock_guard<std::mutex> g(mu_);
		free_[cls].push_back(p);
	}
	std::mutex mu_;
	std::vector<void*> free_[64];
};

// Product backend: every request kind is one bt2x C-ABI call on the context's GPU.
class HipBackend : public Backend {
public:
	explicit HipBackend(bt2x_ctx* ctx) : ctx_(ctx) {
		uint32_t caps = 0;
		bt2x::check(bt2x_capabilities(ctx, &caps), "bt2x_capabilities");
		ref_text_ = (caps & BT2X_CAP_REF_TEXT) != 0 && !(std::getenv("BT2X_HOST_WINDOWS") && std::getenv("BT2X_HOST_WINDOWS")[0] == '1');
		const char* st = std::getenv("BT2X_READ_STORE");          // 0: reads travel with every request
		store_ = !(st && st[0] == '0');
		const char* hs = std::getenv("BT2X_HOST_SEEDS");          // 1: the driver's seed lists are sent
		dseeds_ = !(hs && hs[0] == '1');
		// 1: mismatch-only records' tails formatted by bt2x_sam_tails (off by default: measured
		// slower end to end, DESIGN.md §3 round 6 -- the host still copies every tail once more
		// out of the page-locked buffer, and that costs what formatting it saved)
		const char* gs_ = std::getenv("BT2X_GPU_SAM");
		gpu_sam_ = store_ && gs_ && gs_[0] == '1';
	}
	bool sam_tails_ok() const override { return gpu_sam_; }
	void sam_tails(const HostVec<bt2x_sam_req>& req, HostVec<char>& text, uint64_t text_bytes,
	               HostVec<uint16_t>& lens) override {
		const auto t0 = std::chrono::steady_clock::now();
		text.resize(text_bytes);
		lens.resize(req.size());
		bt2x::check(bt2x_sam_tails(ctx_, req.data(), (uint32_t)req.size(), text.data(), text_bytes, lens.data()),
		            "bt2x_sam_tails");
		gs.sam_h2d += req.size() * sizeof(bt2x_sam_req);
		gs.sam_d2h += text_bytes + req.size() * sizeof(uint16_t);
		gs.t_sam_call += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
	}
	bool read_store() const override { return store_; }
	bool device_seeds() const override { return dseeds_; }
	void store_put(const HostVec<uint8_t>& packed, const HostVec<bt2x_store_in>& in) override {
		bt2x::check(bt2x_store_reads(ctx_, packed.data(), packed.size(), in.data(), (uint32_t)in.size()), "bt2x_store_reads");
		gs.store_h2d += packed.size() + in.size() * sizeof(bt2x_store_in);
	}
	// DP windows cut on the GPU from the resident text (BT2X_DP_REF_TEXT), unless the
	// context lacks it or BT2X_HOST_WINDOWS=1 asks for host-side windows
	bool ref_from_index() const override { return ref_text_; }
	void seed_search(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& in,
	                 HostVec<bt2x_seed_out>& out) override {
		out.resize(in.size());
		bt2x::check(bt2x_seed_search(ctx_, reads.data(), reads.size(), in.data(), (uint32_t)in.size(), 1,
		                             out.data()), "bt2x_seed_search");
	}
	void resolve(const HostVec<bt2x_resolve_in>& in, HostVec<bt2x_resolve_out>& out) override {
		out.resize(in.size());
		bt2x::check(bt2x_resolve(ctx_, in.data(), (uint32_t)in.size(), 0, out.data()), "bt2x_resolve");
	}
	void seed_round(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& seeds,
	                const HostVec<bt2x_round_in>& in, const HostVec<bt2x_exrange>& exr, uint32_t maxelt,
	                HostVec<bt2x_round_out>& out, HostVec<bt2x_sat>& sats, HostVec<bt2x_elt>& elts,
	                HostVec<bt2x_exrange>& exr_out) override {
		const auto t0 = std::chrono::steady_clock::now();
		const uint32_t n = (uint32_t)in.size();
		out.resize(n);
		uint32_t nseeds = 0;                             // the GPU-instantiated seeds' array
		for(const bt2x_round_in& q : in) nseeds = std::max<uint32_t>(nseeds, (uint32_t)(q.seed0 + q.nseeds));
		// arenas sized from the last launch's use per read (grown and retried on overflow)
		uint32_t used[3] = {0, 0, 0};
		// (at least the buffers' reserved capacity: a retry re-runs the whole round)
		uint32_t cap[3] = {(uint32_t)std::max<size_t>((size_t)(sat_per_read_ * n) + 1024, sats.capacity()),
		                   (uint32_t)std::max<size_t>((size_t)(elt_per_read_ * n) + 1024, elts.capacity()),
		                   (uint32_t)std::max<size_t>(4 * (size_t)n + 256, exr_out.capacity())};
		for(int attempt = 0; attempt < 2; attempt++) {
			sats.resize(cap[0]); elts.resize(cap[1]); exr_out.resize(cap[2]);
			// (empty reads: the read store; no seeds: instantiated on the GPU -- a DumpBackend
			// over this one sends both)
			const int rc = bt2x_seed_round(ctx_, reads.empty() ? nullptr : reads.data(), reads.size(),
			                               seeds.empty() ? nullptr : seeds.data(), seeds.empty() ? nseeds : (uint32_t)seeds.size(), in.data(),
			                               n, exr.data(), (uint32_t)exr.size(), maxelt, out.data(), sats.data(), cap[0],
			                               elts.data(), cap[1], exr_out.data(), cap[2], used);
			if(rc == BT2X_E_OVERFLOW && attempt == 0) {
				for(int k = 0; k < 3; k++) cap[k] = std::max(cap[k], used[k]);
				gs.retries++;
				continue;
			}
			bt2x::check(rc, "bt2x_seed_round");
			break;
		}
		sats.resize(used[0]); elts.resize(used[1]); exr_out.resize(used[2]);
		if(n) {
			sat_per_read_ = std::max(8.0, 1.25 * used[0] / n);
			elt_per_read_ = std::max(16.0, 1.25 * used[1] / n);
		}
		gs.k_round_ms += std::max(0.0, bt2x_last_kernel_ms(ctx_, BT2X_K_ROUND));
		gs.round_h2d += reads.size() + seeds.size() * sizeof(bt2x_seed_in) + n * sizeof(bt2x_round_in) +
		                exr.size() * sizeof(bt2x_exrange);
		gs.round_d2h += n * sizeof(bt2x_round_out) + sats.size() * sizeof(bt2x_sat) +
		                elts.size() * sizeof(bt2x_elt) + exr_out.size() * sizeof(bt2x_exrange);
		gs.t_round_call += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
	}
	void dp_align(const HostVec<uint8_t>& reads, const HostVec<uint8_t>& quals,
	              const HostVec<uint8_t>& refs, const HostVec<bt2x_dp_in>& in,
	              HostVec<bt2x_dp_out>& out, HostVec<bt2x_aln_rec>& recs,
	              HostVec<uint32_t>& edits) override {
		const auto t0 = std::chrono::steady_clock::now();
		const uint32_t n = (uint32_t)in.size();
		out.resize(n);
		uint32_t rec_cap = (uint32_t)std::max<size_t>(4 * (size_t)n + 64, recs.capacity()),
		         edit_cap = (uint32_t)std::max<size_t>(48 * (size_t)n + 256, edits.capacity());
		for(int attempt = 0; attempt < 2; attempt++) {
			recs.resize(rec_cap);
			edits.resize(edit_cap);
			uint32_t nrec = 0, ned = 0;
			const int rc = bt2x_dp_align(ctx_, reads.empty() ? nullptr : reads.data(), reads.size(),
			                             quals.empty() ? nullptr : quals.data(), quals.size(),
			                             refs.data(), refs.size(), in.data(), n, out.data(), recs.data(), rec_cap,
			                             &nrec, edits.data(), edit_cap, &ned, nullptr);
			if(rc == BT2X_E_OVERFLOW && attempt == 0) { rec_cap = nrec; edit_cap = ned; gs.retries++; continue; }
			bt2x::check(rc, "bt2x_dp_align");
			recs.resize(nrec);
			edits.resize(ned);
			gs.k_dp_ms += std::max(0.0, bt2x_last_kernel_ms(ctx_, BT2X_K_DP));
			gs.dp_h2d += reads.size() + quals.size() + refs.size() + n * sizeof(bt2x_dp_in);
			gs.dp_d2h += n * sizeof(bt2x_dp_out) + nrec * sizeof(bt2x_aln_rec) + ned * sizeof(uint32_t);
			gs.t_dp_call += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
			return;
		}
	}
	struct GpuStats {                      // kernel time and bytes over PCIe, per request kind
		double k_round_ms = 0, k_dp_ms = 0, t_round_call = 0, t_dp_call = 0;
		uint64_t round_h2d = 0, round_d2h = 0, dp_h2d = 0, dp_d2h = 0, store_h2d = 0, retries = 0;
		uint64_t sam_h2d = 0, sam_d2h = 0;
		double t_sam_call = 0;
	} gs;
private:
	bt2x_ctx* ctx_;
	bool ref_text_ = false, store_ = true, dseeds_ = true, gpu_sam_ = false;
	double sat_per_read_ = 16, elt_per_read_ = 64;
};

// --dump DIR: record every GPU launch's inputs (bench.py replays them from HBM).
// File NNNNNN.<kind>: u64 count of each array, then the arrays.
class DumpBackend : public Backend {
public:
	DumpBackend(Backend& inner, const std::string& dir) : in_(inner), dir_(dir) {}
	bool ref_from_index() const override { return in_.ref_from_index(); }
	void seed_search(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& in,
	                 HostVec<bt2x_seed_out>& out) override {
		write("seed", {{reads.data(), reads.size()}, {in.data(), in.size() * sizeof(bt2x_seed_in)}});
		in_.seed_search(reads, in, out);
	}
	void resolve(const HostVec<bt2x_resolve_in>& in, HostVec<bt2x_resolve_out>& out) override {
		write("resolve", {{in.data(), in.size() * sizeof(bt2x_resolve_in)}});
		in_.resolve(in, out);
	}
	void seed_round(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& seeds,
	                const HostVec<bt2x_round_in>& in, const HostVec<bt2x_exrange>& exr, uint32_t maxelt,
	                HostVec<bt2x_round_out>& out, HostVec<bt2x_sat>& sats, HostVec<bt2x_elt>& elts,
	                HostVec<bt2x_exrange>& exr_out) override {
		in_.seed_round(reads, seeds, in, exr, maxelt, out, sats, elts, exr_out);
		const uint64_t meta[4] = {maxelt, sats.size(), elts.size(), exr_out.size()};   // arena sizes the replay needs
		write("round", {{reads.data(), reads.size()}, {seeds.data(), seeds.size() * sizeof(bt2x_seed_in)},
		                {in.data(), in.size() * sizeof(bt2x_round_in)}, {exr.data(), exr.size() * sizeof(bt2x_exrange)},
		                {meta, sizeof meta}});
	}
	void dp_align(const HostVec<uint8_t>& reads, const HostVec<uint8_t>& quals,
	              const HostVec<uint8_t>& refs, const HostVec<bt2x_dp_in>& in,
	              HostVec<bt2x_dp_out>& out, HostVec<bt2x_aln_rec>& recs,
	              HostVec<uint32_t>& edits) override {
		in_.dp_align(reads, quals, refs, in, out, recs, edits);
		const uint64_t used[2] = {recs.size(), edits.size()};      // arena sizes the replay needs
		write("dp", {{reads.data(), reads.size()}, {quals.data(), quals.size()}, {refs.data(), refs.size()},
		             {in.data(), in.size() * sizeof(bt2x_dp_in)}, {used, sizeof used}});
	}
private:
	void write(const char* kind, std::initializer_list<std::pair<const void*, size_t>> parts) {
		char name[64];
		std::snprintf(name, sizeof name, "/%06u.%s", n_++, kind);
		std::FILE* f = std::fopen((dir_ + name).c_str(), "wb");
		if(!f) throw std::runtime_error("cannot write " + dir_ + name);
		for(auto& p : parts) { const uint64_t n = p.second; std::fwrite(&n, 8, 1, f); }
		for(auto& p : parts) if(p.second) std::fwrite(p.first, 1, p.second, f);
		std::fclose(f);
	}
	Backend& in_;
	std::string dir_;
	unsigned n_ = 0;
};

// Keep the process on the NUMA node of its GPU (threads spawned later inherit the mask, and
// first-touch places their memory there): the box's CPU share is a quota over both sockets'
// CPUs, and threads drifting across sockets reached the read contexts remotely -- runs of
// the same input alternated between ~6.3 and ~8.5 us of CPU per read.  BT2X_NUMA=0 keeps
// the inherited mask; BT2X_NUMA=<node+1> picks a node.  The mask narrows only when the node
// holds at least as many allowed CPUs as the run's worker threads (-p): a cpuset split
// across sockets, or ranks sharing one node, would otherwise be squeezed onto fewer CPUs
// than threads.  Returns the decision for the BT2X_STATS line.
std::string pin_to_gpu_node(int device, int threads) {
	const char* e = std::getenv("BT2X_NUMA");
	if(e && e[0] == '0') return "off";
	int node = e ? std::atoi(e) - 1 : bt2x_device_numa_node(device);
	if(node < 0) return "nonode";
	char path[96];
	std::snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
	std::FILE* f = std::fopen(path, "r");
	if(!f) return "nonode";
	char buf[4096] = {0};
	const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
	std::fclose(f);
	buf[n] = 0;
	cpu_set_t cur, want;
	if(sched_getaffinity(0, sizeof cur, &cur) != 0) return "noaffinity";
	CPU_ZERO(&want);
	for(char* p = buf; *p && *p != '\n';) {                 // "0-63,128-191"
		char* q = nullptr;
		const long a = std::strtol(p, &q, 10);
		long b = a;
		if(*q == '-') b = std::strtol(q + 1, &q, 10);
		for(long c = a; c <= b && c < CPU_SETSIZE; c++) if(CPU_ISSET(c, &cur)) CPU_SET(c, &want);
		p = (*q == ',') ? q + 1 : q;
	}
	// BT2X_NUMA_CORES=1: one hardware thread per physical core of the node (its first SMT
	// sibling), when that still leaves a CPU per worker thread
	const char* oc = std::getenv("BT2X_NUMA_CORES");
	if(oc && oc[0] == '1') {
		cpu_set_t first;
		CPU_ZERO(&first);
		for(int c = 0; c < CPU_SETSIZE; c++) {
			if(!CPU_ISSET(c, &want)) continue;
			char sp[128];
			std::snprintf(sp, sizeof sp, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
			std::FILE* sf = std::fopen(sp, "r");
			long lo = c;
			if(sf) { if(std::fscanf(sf, "%ld", &lo) != 1) lo = c; std::fclose(sf); }
			if(lo == c) CPU_SET(c, &first);
		}
		if(CPU_COUNT(&first) >= threads) want = first;
	}
	const int have = CPU_COUNT(&want);
	char note[64];
	if(have >= 4 && have >= threads && sched_setaffinity(0, sizeof want, &want) == 0)
		std::snprintf(note, sizeof note, "node%d:%d", node, have);
	else
		std::snprintf(note, sizeof note, "kept(node%d:%d<%d)", node, have, threads);
	return note;
}

void usage() {
	std::fprintf(stderr,
	             "usage: bt2x-align -x <index> -U <r1.fq>[,r2.fq,...] [-S out.sam] [--dpad N] [-D N] [-R N] [-L N]\n"
	             "                  [-i FUNC] [--score-min FUNC] [--n-ceil FUNC] [--mp MX,MN] [--np N]\n"
	             "                  [--rdg O,E] [--rfg O,E] [--gbar N] [--seed N] [--no-sse8] [--i16-build]\n"
	             "                  [--no-hd] [-p threads] [--slots N] [--device N] [--stats]\n"
	             "                  [--shard i/N] [--warmup-files K] [--metrics] [--no-pipeline] [--streams 1|2]\n"
	             "                  [--cpus LIST]\n");
}

} // namespace

int main(int argc, char** argv) {
	tune_malloc();
	std::string idx, fq, outp, mate1, mate2;
	Params p;
	int threads = 16, device = 0;
	size_t slots = 1 << 17;                             // reads in flight: two cohorts of 65,536
	bool stats = false, pipeline = true, gpu_round = true, hd = true, metrics = false;
	// --streams 2: the second cohort on a second context (bt2x_open_shared).  One is the
	// default: the run is host-bound, and two contexts' concurrent launches each take longer
	// (C3, one box: 2.05 vs 1.87 M reads/s).  BT2X_STREAMS sets the default (A/B runs).
	int streams = 1;
	if(const char* e = std::getenv("BT2X_STREAMS")) streams = std::atoi(e);
	int shard = 0, nshards = 1, warm_files = 0;
	std::string dump, cpus;
	for(int i = 1; i < argc; i++) {
		const std::string a = argv[i];
		auto val = [&]() -> const char* {
			if(i + 1 >= argc) { usage(); std::exit(1); }
			return argv[++i];
		};
		if(const int k = parse_align_option(p, argc, argv, i)) { i += k - 1; continue; }
		if(a == "-x") idx = val();
		else if(a == "-U") fq = val();
		else if(a == "-1") mate1 = val();
		else if(a == "-2") mate2 = val();
		else if(a == "-S") outp = val();
		else if(a == "-p") threads = std::atoi(val());
		else if(a == "--slots") slots = (size_t)std::atol(val());
		else if(a == "--device") device = std::atoi(val());
		else if(a == "--stats") stats = true;
		else if(a == "--dump") dump = val();
		else if(a == "--no-pipeline") pipeline = false;
		else if(a == "--streams") streams = std::atoi(val());
		else if(a == "--no-gpu-round") gpu_round = false;
		else if(a == "--no-hd") hd = false;
		else if(a == "--metrics") metrics = true;
		else if(a == "--warmup-files") warm_files = std::atoi(val());
		else if(a == "--cpus") cpus = val();
		else if(a == "--shard") {
			if(std::sscanf(val(), "%d/%d", &shard, &nshards) != 2 || nshards < 1 || shard < 0 || shard >= nshards) {
				std::fprintf(stderr, "--shard takes i/N with 0 <= i < N\n");
				return 1;
			}
		}
		else if(a == "--end-to-end" || a == "--sensitive" || a == "--reorder" || a == "-q") {}
		else { std::fprintf(stderr, "unsupported option %s\n", a.c_str()); usage(); return 1; }
	}
	// -1/-2: this fork aligns mate 1 alone, as unpaired reads (bt2_search.cpp:1006-1007,
	// 1690-1694 -- paired alignment is compiled out), so the mate-1 files are the read stream
	if(!mate1.empty() || !mate2.empty()) {
		if(!fq.empty()) { std::fprintf(stderr, "-U with -1/-2 is not supported\n"); return 1; }
		if(split_list(mate1).size() != split_list(mate2).size()) {
			std::fprintf(stderr, "Error: %zu mate files/sequences were specified with -1, but %zu\n"
			             "mate files/sequences were specified with -2.  The same number of mate files/\n"
			             "sequences must be specified with -1 and -2.\n", split_list(mate1).size(), split_list(mate2).size());
			return 1;
		}
		fq = mate1;
	}
	if(idx.empty() || fq.empty()) { usage(); return 1; }
	// --cpus (the sharded launcher's per-rank set) replaces the NUMA-node pinning
	std::string numa;
	if(!cpus.empty()) {
		try { apply_cpu_list(cpus); } catch(const std::exception& e) { std::fprintf(stderr, "%s\n", e.what()); return 1; }
		numa = "cpus";
	} else {
		numa = pin_to_gpu_node(device, threads);
	}
	std::fprintf(stderr, "BT2X_CPUS %s\n", affinity_list().c_str());
	const std::vector<std::string> files = split_list(fq);
	if(warm_files < 0 || (size_t)warm_files >= files.size()) {
		std::fprintf(stderr, "--warmup-files must leave at least one -U file to time\n");
		return 1;
	}
	bt2x_scoring_init(&p.sc);
	if(p.multiseedLen < 1 || p.multiseedLen > 32) { std::fprintf(stderr, "-L must be in 1..32\n"); return 1; }
	try {
		// the launch buffers' page-locked blocks are pinned while the index loads (pinning
		// runs at ~1 GB/s; done launch by launch it cost ~0.5 s of a 1 M-read run)
		std::thread pin([&] {
			std::vector<size_t> sizes;
			for(int k = 0; k < 2; k++)
				for(size_t b : Aligner::launch_buffer_bytes(p, pipeline ? slots / 2 : slots))
					sizes.push_back(b + 64);                       // + host_alloc's header
			PinnedCache::prefill(sizes);
		});
		struct Join { std::thread& t; ~Join() { if(t.joinable()) t.join(); } } join_pin{pin};
		bt2x::Index index(idx.c_str(), true);
		RefInfo ref;
		ref.init(index.desc(), idx);
		bt2x::Device dev(device, index, p.sc);
		// align()'s best of a failed DP feeds only --mapq-extra's ZT:Z, which this driver does
		// not print: skip the kernels' exact-best pass (bt2x.h BT2X_OPT_EXACT_BEST)
		bt2x::check(bt2x_set_option(dev.ctx(), BT2X_OPT_EXACT_BEST, 0), "bt2x_set_option");
		HipBackend hip(dev.ctx());
		// --streams 2 (pipelined): the second cohort's launches run on a second context over the
		// same device index (its own stream), so the two cohorts' launches overlap on the GPU
		// (--dump records one launch sequence on one context)
		std::unique_ptr<bt2x_ctx, void (*)(bt2x_ctx*)> ctx2(nullptr, bt2x_close);
		std::unique_ptr<HipBackend> hip2;
		if(pipeline && streams >= 2 && dump.empty()) {
			bt2x_ctx* c2 = nullptr;
			bt2x::check(bt2x_open_shared(dev.ctx(), &c2), "bt2x_open_shared");
			ctx2.reset(c2);
			bt2x::check(bt2x_set_option(c2, BT2X_OPT_EXACT_BEST, 0), "bt2x_set_option");
			hip2.reset(new HipBackend(c2));
		}
		set_host_allocator(PinnedCache::alloc, PinnedCache::release);   // launch buffers page-locked
		std::unique_ptr<DumpBackend> dumper;
		if(!dump.empty()) dumper.reset(new DumpBackend(hip, dump));
		Backend& be = dumper ? static_cast<Backend&>(*dumper) : static_cast<Backend&>(hip);
		Aligner al(p, ref, be);
		al.set_pipeline(pipeline);
		if(hip2) al.set_second_backend(hip2.get());
		// bt2x_elt holds fewer than 2^24 - 1 reference indices: beyond that, the three-request round
		al.set_gpu_round(gpu_round && ref.nrefs() < BT2X_ELT_TIDX_NONE);
		al.set_header(hd);
		pin.join();
		if(warm_files > 0) {                           // untimed: first launches, page faults, pools
			FastqReader wr(std::vector<std::string>(files.begin(), files.begin() + warm_files), shard, nshards);
			std::FILE* null = std::fopen("/dev/null", "wb");
			if(!null) throw std::runtime_error("cannot open /dev/null");
			al.run(wr, null, slots, threads);
			std::fclose(null);
			// BT2X_GPU, like BT2X_TIMED, covers the timed files only
			hip.gs = HipBackend::GpuStats{};
			if(hip2) hip2->gs = HipBackend::GpuStats{};
		}
		// unnamed reads of the timed files are numbered after the warmup files' records, as in
		// one run over the whole -U list
		uint64_t warm_records = 0;
		for(int k = 0; k < warm_files; k++) warm_records += FastqReader::count_file_records(files[(size_t)k]);
		FastqReader reader(std::vector<std::string>(files.begin() + warm_files, files.end()), shard, nshards, warm_records);
		struct rusage ru0;
		getrusage(RUSAGE_SELF, &ru0);
		const auto t_start = std::chrono::steady_clock::now();
		std::FILE* out = outp.empty() ? stdout : std::fopen(outp.c_str(), "wb");
		if(!out) { std::fprintf(stderr, "cannot open %s\n", outp.c_str()); return 1; }
		std::vector<char> obuf(1 << 24);
		std::setvbuf(out, obuf.data(), _IOFBF, obuf.size());
		double t_run = 0;
		// development: bt2x-align-prof (tools/sprof.c linked in) with SPROF_WAIT=1 samples the
		// timed run only; SIGUSR2 toggles its sampling
		const bool sprof = std::getenv("SPROF_WAIT") != nullptr;
		if(sprof) std::raise(SIGUSR2);
		const RunStats st = al.run(reader, out, slots, threads, &t_run);
		if(sprof) std::raise(SIGUSR2);
		const double t_ret = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
		if(out != stdout) std::fclose(out); else std::fflush(out);
		const double t_align = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
		struct rusage ru_end;
		getrusage(RUSAGE_SELF, &ru_end);
		print_alignment_summary(st.met, stderr);
		if(metrics) {
			std::string line = "BT2X_METRICS";
			for(uint64_t v : st.met.v) line += " " + std::to_string(v);
			std::fprintf(stderr, "%s\n", line.c_str());
			std::string tf;
			for(double t : st.t_files) { char b[32]; std::snprintf(b, sizeof b, "%s%.4f", tf.empty() ? "" : ",", t); tf += b; }
			std::fprintf(stderr, "BT2X_TIMED reads=%llu first_rdid=%llu t_align=%.4f t_files=%s t_run=%.4f t_ret=%.4f\n",
			             (unsigned long long)st.reads, (unsigned long long)reader.first_rdid(), t_align, tf.c_str(), t_run,
			             t_ret);
		}
		if(stats) {
			// the whole process, then the alignment window alone
			struct rusage ru;
			getrusage(RUSAGE_SELF, &ru);
			auto sec = [](const timeval& t) { return t.tv_sec + t.tv_usec * 1e-6; };
			std::fprintf(stderr, "BT2X_RUSAGE user=%.3f sys=%.3f maxrss_mib=%ld minflt=%ld majflt=%ld vcsw=%ld ivcsw=%ld\n",
			             sec(ru.ru_utime), sec(ru.ru_stime), ru.ru_maxrss / 1024, ru.ru_minflt, ru.ru_majflt, ru.ru_nvcsw,
			             ru.ru_nivcsw);
			std::fprintf(stderr, "BT2X_RUSAGE_ALIGN user=%.3f sys=%.3f minflt=%ld vcsw=%ld ivcsw=%ld\n",
			             sec(ru_end.ru_utime) - sec(ru0.ru_utime), sec(ru_end.ru_stime) - sec(ru0.ru_stime),
			             ru_end.ru_minflt - ru0.ru_minflt, ru_end.ru_nvcsw - ru0.ru_nvcsw, ru_end.ru_nivcsw - ru0.ru_nivcsw);
		}
		if(stats)
			std::fprintf(stderr, "BT2X_STATS reads=%llu t_align=%.4f seed_launches=%llu seeds=%llu t_seed=%.4f "
			             "resolve_launches=%llu resolves=%llu t_resolve=%.4f dp_launches=%llu dps=%llu t_dp=%.4f "
			             "t_host=%.4f t_io=%.4f dps_used=%llu tight_recs=%llu t_backend=%.4f t_step=%.4f t_wait=%.4f t_gather=%.4f t_retire=%.4f "
			             "round_launches=%llu rounds=%llu t_round=%.4f dp_max_launch=%llu numa=%s\n", (unsigned long long)st.reads, t_align,
			             (unsigned long long)st.seed_launches, (unsigned long long)st.seeds, st.t_seed,
			             (unsigned long long)st.resolve_launches, (unsigned long long)st.resolves, st.t_resolve,
			             (unsigned long long)st.dp_launches, (unsigned long long)st.dps, st.t_dp, st.t_host, st.t_io, (unsigned long long)st.dps_used,
			             (unsigned long long)st.tight_recs, st.t_backend, st.t_step, st.t_wait, st.t_gather, st.t_retire,
			             (unsigned long long)st.round_launches, (unsigned long long)st.rounds, st.t_round,
			             (unsigned long long)st.dp_max_launch, numa.c_str());
		if(stats) {
			HipBackend::GpuStats g = hip.gs;
			if(hip2) {
				const HipBackend::GpuStats& h = hip2->gs;
				g.k_round_ms += h.k_round_ms; g.k_dp_ms += h.k_dp_ms; g.t_round_call += h.t_round_call;
				g.t_dp_call += h.t_dp_call; g.round_h2d += h.round_h2d; g.round_d2h += h.round_d2h;
				g.dp_h2d += h.dp_h2d; g.dp_d2h += h.dp_d2h; g.store_h2d += h.store_h2d; g.retries += h.retries;
				g.sam_h2d += h.sam_h2d; g.sam_d2h += h.sam_d2h; g.t_sam_call += h.t_sam_call;
			}
			std::fprintf(stderr, "BT2X_GPU k_round=%.4f t_round_call=%.4f round_h2d_mib=%.1f round_d2h_mib=%.1f "
			             "k_dp=%.4f t_dp_call=%.4f dp_h2d_mib=%.1f dp_d2h_mib=%.1f store_h2d_mib=%.1f retries=%llu "
			             "sam_h2d_mib=%.1f sam_d2h_mib=%.1f t_sam_call=%.4f sam_gpu=%llu\n",
			             g.k_round_ms * 1e-3, g.t_round_call, g.round_h2d / 1048576.0, g.round_d2h / 1048576.0, g.k_dp_ms * 1e-3,
			             g.t_dp_call, g.dp_h2d / 1048576.0, g.dp_d2h / 1048576.0, g.store_h2d / 1048576.0,
			             (unsigned long long)g.retries, g.sam_h2d / 1048576.0, g.sam_d2h / 1048576.0, g.t_sam_call,
			             (unsigned long long)st.sam_gpu);
		}
	} catch(const std::exception& e) {
		std::fprintf(stderr, "bt2x-align: %s\n", e.what());
		return 1;
	}
	return 0;
}
