// bt2x_align.cpp — the host driver of bt2x_align.hpp: per-read coroutine (the
// reference's multiseedSearchWorker phases for one read), the batching scheduler,
// reporting and SAM formatting.  Compiled without -ffast-math and with
// -ffp-contract=off: RowSampler darts and MAPQ thresholds are float/double compares
// that must round exactly like the reference's x86-64 build.
#include "bt2x_align.hpp"

#include <cctype>
#include <chrono>
#include <map>
#include <memory>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace bt2x {
namespace host {

const uint8_t kAsc2Dna[256] = {   // alphabet.cpp:142 (A/C/G/T, either case; all else N)
#define N4 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4
	N4, N4, N4, N4,
	4, 0, 4, 1, 4, 4, 4, 2, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 0, 4, 1, 4, 4, 4, 2, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4,
	N4, N4, N4, N4, N4, N4, N4, N4
#undef N4
};

// ---------------------------------------------------------------- FastqReader

FastqReader::FastqReader(const char* path) {
	fd_ = ::open(path, O_RDONLY);
	if(fd_ < 0) throw std::runtime_error(std::string("cannot open reads file ") + path);
	struct stat sb;
	if(::fstat(fd_, &sb) != 0) throw std::runtime_error(std::string("cannot stat ") + path);
	len_ = (size_t)sb.st_size;
	if(len_) {
		void* m = ::mmap(nullptr, len_, PROT_READ, MAP_PRIVATE, fd_, 0);
		if(m == MAP_FAILED) throw std::runtime_error(std::string("cannot map ") + path);
		::madvise(m, len_, MADV_SEQUENTIAL);
		map_ = (const char*)m;
	}
}

FastqReader::~FastqReader() {
	if(map_) ::munmap((void*)map_, len_);
	if(fd_ >= 0) ::close(fd_);
}

// ------------------------------------------------------------------- RefInfo

void RefInfo::init(const bt2x_index_desc& d, const std::string& base) {
	plen_.assign(d.plen, d.plen + d.npat);
	text_ = d.text2;
	if(!text_) throw std::runtime_error("RefInfo: index loaded without the packed text (.4.bt2l)");
	frags_.assign(d.npat, {});
	// rstarts: (joined offset, text id, text offset) per fragment (Ebwt::_rstarts)
	for(uint64_t k = 0; k < d.nfrag; k++) {
		const uint64_t joff = d.rstarts[3 * k], tidx = d.rstarts[3 * k + 1], toff = d.rstarts[3 * k + 2];
		const uint64_t jend = (k + 1 < d.nfrag) ? d.rstarts[3 * (k + 1)] : d.len;
		if(tidx >= d.npat) throw std::runtime_error("RefInfo: bad fragment record");
		if(jend > joff) frags_[tidx].push_back({(int64_t)toff, jend - joff, joff});
	}
	// reference names: the text after eftab in <base>.1.bt2l, one per line (bt2_io.cpp:499)
	const std::string p1 = base + ".1.bt2l";
	std::FILE* f = std::fopen(p1.c_str(), "rb");
	if(!f) throw std::runtime_error("cannot open " + p1);
	const uint64_t sideSz = 128, sideBwt = 96;
	const uint64_t numSides = (d.len / 4 + 1 + sideBwt - 1) / sideBwt;
	const uint64_t hdr = 4 + 8 + 5 * 4 + 8 + 8 * d.npat + 8 + 24 * d.nfrag;
	const uint64_t off = hdr + numSides * sideSz + 8 + 40 + 8 * d.ftab_len + 8 * d.eftab_len;
	std::fseek(f, (long)off, SEEK_SET);
	std::string cur;
	int ch;
	while((ch = std::fgetc(f)) != EOF) {
		if(ch == '\n') { names_.push_back(cur); cur.clear(); }
		else cur.push_back((char)ch);
	}
	std::fclose(f);
	if(!cur.empty()) names_.push_back(cur);
	while(names_.size() < d.npat) names_.push_back(std::to_string(names_.size()));
	names_.resize(d.npat);
}

void RefInfo::stretch(uint32_t tidx, int64_t off, size_t n, uint8_t* out) const {
	std::memset(out, 4, n);
	const std::vector<Frag>& fs = frags_[tidx];
	// fragments are in text order: start at the last one beginning at or before `off`
	size_t k = (size_t)(std::upper_bound(fs.begin(), fs.end(), off,
	                                     [](int64_t o, const Frag& f) { return o < f.toff; }) - fs.begin());
	if(k > 0) k--;
	for(; k < fs.size() && fs[k].toff < off + (int64_t)n; k++) {
		const Frag& fr = fs[k];
		const int64_t a = std::max<int64_t>(off, fr.toff);
		const int64_t b = std::min<int64_t>(off + (int64_t)n, fr.toff + (int64_t)fr.len);
		for(int64_t p = a; p < b; p++) {
			const uint64_t j = fr.joff + (uint64_t)(p - fr.toff);
			out[p - off] = (text_[j >> 2] >> ((j & 3) << 1)) & 3;
		}
	}
}

// -------------------------------------------------------------- reporting

namespace {

enum { EXIT_DID_NOT_EXIT = 1, EXIT_SHORT_CIRCUIT_k, EXIT_SHORT_CIRCUIT_M, EXIT_SHORT_CIRCUIT_TRUMPED,
       EXIT_NO_ALIGNMENTS, EXIT_WITH_ALIGNMENTS };

enum { EXTEND_EXHAUSTED_CANDIDATES = 1, EXTEND_POLICY_FULFILLED, EXTEND_PERFECT_SCORE,
       EXTEND_EXCEEDED_SOFT_LIMIT, EXTEND_EXCEEDED_HARD_LIMIT };

constexpr int64_t kMinScore = std::numeric_limits<int64_t>::min();

// AlnSinkWrap for an unpaired read (aln_sink.cpp:583-643, 1395-1445) with its
// ReportingState (aln_sink.cpp:33-210) under -k 1 -M mhits.
struct Sink {
	int64_t mhits = 50;
	std::vector<AlnRes> rs;
	int64_t best = kMinScore, best2 = kMinScore;
	uint64_t n = 0;
	bool doneUnpair = false;
	int exitUnpair = EXIT_DID_NOT_EXIT;
	bool done() const { return doneUnpair; }            // doneConcord_/doneDiscord_ are true
	bool report(const AlnRes& r) {
		n++;
		if(!doneUnpair && n > (uint64_t)mhits) { doneUnpair = true; exitUnpair = EXIT_SHORT_CIRCUIT_M; }
		rs.push_back(r);
		if(r.score > best) { best2 = best; best = r.score; }
		else if(r.score > best2) best2 = r.score;
		return done();
	}
	bool hasSecondBest() const { return best2 != kMinScore; }
};

// StackedAln (aligner_result.cpp:448-770) over the Watson-strand read.
std::string cigar_md(const Read& rd, const AlnRes& r, std::string& md) {
	const std::vector<uint8_t>& s = r.fw ? rd.fw : rd.rc;
	const std::vector<uint32_t> ed = r.fw ? r.ned : invert_poss(r.ned, rd.length());
	std::vector<char> ref, rel, rdc;
	ref.reserve(s.size() + 16); rel.reserve(s.size() + 16); rdc.reserve(s.size() + 16);
	size_t rdoff = 0;
	static const char kAcgtn[] = "ACGTN";
	// The printed edits come from the read's shared edit buffer and may step
	// past the read's end; the reference then reads stale bytes of its read buffer, which
	// only ever reach the output through left-alignment of an adjacent gap.  N stands in.
	auto at = [&](size_t i) -> int { return i < s.size() ? s[i] : 4; };
	for(uint32_t e : ed) {
		const size_t pos = e_pos(e);
		while(rdoff < pos) { const int c = at(rdoff++); ref.push_back(kAcgtn[c]); rel.push_back('='); rdc.push_back(kAcgtn[c]); }
		const uint32_t t = e_type(e);
		if(t == ET_MM) { const int c = at(rdoff++); ref.push_back(e_chr(e)); rel.push_back('X'); rdc.push_back(kAcgtn[c]); }
		else if(t == ET_REF_GAP) { const int c = at(rdoff++); ref.push_back('-'); rel.push_back('I'); rdc.push_back(kAcgtn[c]); }
		else if(t == ET_READ_GAP) { ref.push_back(e_chr(e)); rel.push_back('D'); rdc.push_back('-'); }
	}
	while(rdoff < s.size()) { const int c = s[rdoff++]; ref.push_back(kAcgtn[c]); rel.push_back('='); rdc.push_back(kAcgtn[c]); }
	// leftAlign(pastMms = false)
	const size_t ln = ref.size();
	for(size_t i = 0; i < ln; i++) {
		const char g = rel[i];
		if(g == '=' || g == 'X') continue;
		size_t glen = 1;
		for(size_t j = i + 1; j < ln; j++) { if(rel[j] != g) break; glen++; }
		if(i >= 1) {   // i == 0 would index [-1] in the reference; a gap never opens row 0
			size_t l = i - 1, r2 = l + glen;
			std::vector<char>& gp = (g == 'I') ? ref : rdc;
			const std::vector<char>& ngp = (g == 'I') ? rdc : ref;
			while(l > 0 && ngp[l] == ngp[r2]) {
				if(rel[l] == 'X') break;
				std::swap(gp[l], gp[r2]);
				std::swap(rel[l], rel[r2]);
				l--; r2--;
			}
		}
		i += glen - 1;
	}
	// CIGAR (xeq = false)
	std::string cig;
	for(size_t i = 0; i < ln; i++) {
		char op = rel[i] == 'X' || rel[i] == '=' ? 'M' : rel[i];
		size_t run = 1;
		for(; i + run < ln; run++) {
			const char op2 = rel[i + run] == 'X' || rel[i + run] == '=' ? 'M' : rel[i + run];
			if(op2 != op) break;
		}
		i += run - 1;
		cig += std::to_string(run);
		cig.push_back(op);
	}
	// MD:Z (buildMdz + writeMdz)
	md.clear();
	bool mm_last = false, rdgap_last = false, first_print = true;
	for(size_t i = 0; i < ln; i++) {
		const char op = rel[i];
		if(op == '=') {
			size_t run = 1, nins = 0;
			for(; i + run < ln; run++) {
				if(rel[i + run] == '=') {}
				else if(rel[i + run] == 'I') nins++;
				else break;
			}
			i += run - 1;
			if(run - nins > 0) {
				md += std::to_string(run - nins);
				first_print = false; mm_last = false; rdgap_last = false;
			}
		} else if(op == 'X') {
			if(rdgap_last || mm_last || first_print) md.push_back('0');
			md.push_back(ref[i]);
			first_print = false; mm_last = true; rdgap_last = false;
		} else if(op == 'D') {
			if(mm_last || first_print) md.push_back('0');
			if(!rdgap_last) md.push_back('^');
			md.push_back(ref[i]);
			first_print = false; mm_last = false; rdgap_last = true;
		}
	}
	if(mm_last || rdgap_last) md.push_back('0');
	return cig;
}

// BowtieMapq2::mapq, monotone (end-to-end) branch, unpaired (unique.h:187-330).
int64_t mapq_v2(const Params& p, size_t rdlen, int64_t best, bool hasSecbest, int64_t secbestIn) {
	const int64_t scPer = 0;
	const int64_t scMin = p.scoreMin.f<int64_t>((float)rdlen);
	int64_t secbest = scMin - 1;
	const int64_t diff = std::max<int64_t>(1, scPer - scMin);
	int64_t ret = 0;
	const int64_t bestOver = best - scMin;
	if(!hasSecbest) {
		if     (bestOver >= diff * (double)0.8f) ret = 42;
		else if(bestOver >= diff * (double)0.7f) ret = 40;
		else if(bestOver >= diff * (double)0.6f) ret = 24;
		else if(bestOver >= diff * (double)0.5f) ret = 23;
		else if(bestOver >= diff * (double)0.4f) ret = 8;
		else if(bestOver >= diff * (double)0.3f) ret = 3;
		else                                     ret = 0;
	} else {
		secbest = secbestIn;
		const int64_t bestdiff = std::labs(std::labs((long)best) - std::labs((long)secbest));
		if(bestdiff >= diff * (double)0.9f) ret = bestOver == diff ? 39 : 33;
		else if(bestdiff >= diff * (double)0.8f) ret = bestOver == diff ? 38 : 27;
		else if(bestdiff >= diff * (double)0.7f) ret = bestOver == diff ? 37 : 26;
		else if(bestdiff >= diff * (double)0.6f) ret = bestOver == diff ? 36 : 22;
		else if(bestdiff >= diff * (double)0.5f) {
			if(bestOver == diff) ret = 35;
			else if(bestOver >= diff * (double)0.84f) ret = 25;
			else if(bestOver >= diff * (double)0.68f) ret = 16;
			else ret = 5;
		} else if(bestdiff >= diff * (double)0.4f) {
			if(bestOver == diff) ret = 34;
			else if(bestOver >= diff * (double)0.84f) ret = 21;
			else if(bestOver >= diff * (double)0.68f) ret = 14;
			else ret = 4;
		} else if(bestdiff >= diff * (double)0.3f) {
			if(bestOver == diff) ret = 32;
			else if(bestOver >= diff * (double)0.88f) ret = 18;
			else if(bestOver >= diff * (double)0.67f) ret = 15;
			else ret = 3;
		} else if(bestdiff >= diff * (double)0.2f) {
			if(bestOver == diff) ret = 31;
			else if(bestOver >= diff * (double)0.88f) ret = 17;
			else if(bestOver >= diff * (double)0.67f) ret = 11;
			else ret = 0;
		} else if(bestdiff >= diff * (double)0.1f) {
			if(bestOver == diff) ret = 30;
			else if(bestOver >= diff * (double)0.88f) ret = 12;
			else if(bestOver >= diff * (double)0.67f) ret = 7;
			else ret = 0;
		} else if(bestdiff > 0) {
			ret = bestOver >= diff * (double)0.67f ? 6 : 2;
		} else {
			ret = bestOver >= diff * (double)0.67f ? 1 : 0;
		}
	}
	return ret;
}

void append_name(std::string& o, const std::string& name) {   // SamConfig::printReadName
	size_t n = std::min<size_t>(name.size(), 255);
	for(size_t i = 0; i < n; i++) {
		if(std::isspace((unsigned char)name[i])) break;
		o.push_back(name[i]);
	}
}

void append_refname(std::string& o, const std::string& name) {   // SamConfig::printRefName
	for(char ch : name) { if(std::isspace((unsigned char)ch)) break; o.push_back(ch); }
}

void append_seq(std::string& o, const std::vector<uint8_t>& s) {
	if(s.empty()) { o.push_back('*'); return; }
	for(uint8_t c : s) o.push_back("ACGTN"[c]);
}

// AlnSinkWrap::finishRead, unpaired branch (aln_sink.cpp:643-1384) -> one SAM record
// (AlnSinkSam::appendMate, aln_sink.cpp:1889-2090; tags per sam.cpp:121-730).
std::string finish_read(const Params& p, const RefInfo& ref, const Read& rd, Sink& sk, Rng& rnd,
                        const std::vector<uint32_t>& edbuf, bool* aligned, bool* rep) {
	// ReportingState::finish + getReport
	if(!sk.doneUnpair) { sk.doneUnpair = true; sk.exitUnpair = sk.n > 0 ? EXIT_WITH_ALIGNMENTS : EXIT_NO_ALIGNMENTS; }
	uint64_t nunpair = 0;
	bool unpairMax = false;
	if(sk.n > 0) {
		if(sk.exitUnpair == EXIT_SHORT_CIRCUIT_M) { unpairMax = true; nunpair = 1; }
		else if(sk.exitUnpair == EXIT_WITH_ALIGNMENTS) nunpair = std::min<uint64_t>(sk.n, 1);
	}
	std::string o;
	append_name(o, rd.name);
	if(nunpair == 0) {
		*aligned = false; *rep = unpairMax;
		o += "\t4\t*\t0\t0\t*\t*\t0\t0\t";
		append_seq(o, rd.fw);
		o.push_back('\t');
		o += rd.qual.empty() ? std::string("*") : rd.qual;
		o += "\tYT:Z:UU\tYF:Z:LN\n";
		return o;
	}
	// selectByScore (aln_sink.cpp:1477-1640): sort by score desc (ties by index desc),
	// shuffle equal-score streaks with the read's RNG
	const size_t sz = sk.rs.size();
	std::vector<std::pair<int64_t, size_t>> buf(sz);
	for(size_t i = 0; i < sz; i++) buf[i] = {sk.rs[i].score, i};
	std::stable_sort(buf.begin(), buf.end());
	std::reverse(buf.begin(), buf.end());
	auto shuffle = [&](size_t begin, size_t num) {
		if(num < 2) return;
		size_t left = num;
		for(size_t i = begin; i < begin + num - 1; i++) {
			const size_t rndi = rnd.nextSizeT() % left;
			if(rndi > 0) std::swap(buf[i], buf[i + rndi]);
			left--;
		}
	};
	size_t streak = 0;
	for(size_t i = 1; i < buf.size(); i++) {
		if(buf[i].first == buf[i - 1].first) { if(streak == 0) streak = 1; streak++; }
		else { if(streak > 1) shuffle(i - streak, streak); streak = 0; }
	}
	if(streak > 1) shuffle(buf.size() - streak, streak);
	// Every reported AlnRes shares the read's edit buffer (DList copies keep the source's
	// storage pointer, ds.h:979-1040): the record shows its first ned().size() entries as
	// they stand now.
	AlnRes r = sk.rs[buf[0].second];
	const size_t nshow = r.ned.size();
	r.ned.assign(edbuf.begin(), edbuf.begin() + (long)std::min(nshow, edbuf.size()));
	const int64_t bestU = r.score;
	const bool hasSec = buf.size() > 1;
	const int64_t secU = hasSec ? sk.rs[buf[1].second].score : 0;
	*aligned = true; *rep = unpairMax;
	// record
	o.push_back('\t');
	o += r.fw ? "0" : "16";
	o.push_back('\t');
	append_refname(o, ref.name((size_t)r.refid));
	o.push_back('\t');
	o += std::to_string(r.refoff + 1);
	o.push_back('\t');
	o += std::to_string(mapq_v2(p, rd.length(), bestU, hasSec, secU));
	o.push_back('\t');
	std::string md;
	o += cigar_md(rd, r, md);
	o += "\t*\t0\t0\t";
	append_seq(o, r.fw ? rd.fw : rd.rc);
	o.push_back('\t');
	o += (r.fw ? rd.qual : rd.qualRev);
	o += "\tAS:i:" + std::to_string(r.score);
	if(hasSec) o += "\tXS:i:" + std::to_string(secU);
	o += "\tXN:i:" + std::to_string(r.refns);
	size_t num_mm = 0, num_go = 0, num_gx = 0;
	const std::vector<uint32_t>& ned = r.ned;
	for(size_t i = 0; i < ned.size(); i++) {
		const uint32_t t = e_type(ned[i]);
		if(t == ET_MM) num_mm++;
		else if(t == ET_READ_GAP) {
			num_go++; num_gx++;
			while(i < ned.size() - 1 && e_pos(ned[i + 1]) == e_pos(ned[i]) && e_type(ned[i + 1]) == ET_READ_GAP) { i++; num_gx++; }
		} else if(t == ET_REF_GAP) {
			num_go++; num_gx++;
			while(i < ned.size() - 1 && e_pos(ned[i + 1]) == e_pos(ned[i]) + 1 && e_type(ned[i + 1]) == ET_REF_GAP) { i++; num_gx++; }
		}
	}
	o += "\tXM:i:" + std::to_string(num_mm);
	o += "\tXO:i:" + std::to_string(num_go);
	o += "\tXG:i:" + std::to_string(num_gx);
	o += "\tNM:i:" + std::to_string(ned.size());
	o += "\tMD:Z:" + md;
	o += "\tYT:Z:UU\tYF:Z:LN\n";
	return o;
}

struct SatPos {                     // SATupleAndPos (aligner_sw_driver.h:118-180)
	uint64_t topf = 0, size = 0;    // SATuple: BW top and #elements (offs.size())
	uint64_t key = 0;               // identity of the cache entry (its BW top)
	uint8_t nlex = 0;
	uint64_t origSz = 0;
	bool fw = true;                 // SeedPos
	uint32_t offidx = 0, rdoff = 0, seedlen = 0;
	bool operator<(const SatPos& o) const {
		if(size != o.size) return size < o.size;
		if(topf != o.topf) return topf < o.topf;
		if(offidx != o.offidx) return offidx < o.offidx;
		if(rdoff != o.rdoff) return rdoff < o.rdoff;
		if(seedlen != o.seedlen) return seedlen < o.seedlen;
		return fw && !o.fw;
	}
};

struct ExtendRange { size_t off, len, sz; };

// RowSampler (aligner_sw_driver.h:176-267), lensq = szsq = true
struct RowSampler {
	double mass = 0;
	std::vector<double> masses;
	std::vector<bool> elim;
	void init(const std::vector<SatPos>& sl, size_t sai, size_t saf) {
		elim.assign(saf - sai, false);
		mass = 0.0f;
		masses.assign(saf - sai, 0.0);
		for(size_t i = sai; i < saf; i++) {
			double num = (double)(sl[i].nlex + 1);
			num *= num;
			double den = (double)sl[i].size;
			den *= den;
			masses[i - sai] = num / den;
			mass += masses[i - sai];
		}
	}
	void finishedRange(size_t i) { elim[i] = true; mass -= masses[i]; }
	size_t next(Rng& rnd) {
		const double rd = rnd.nextFloat() * mass;
		double sofar = 0.0f;
		size_t last = std::numeric_limits<size_t>::max();
		for(size_t i = 0; i < masses.size(); i++) {
			if(!elim[i]) {
				last = i;
				sofar += masses[i];
				if(rd < sofar) return i;
			}
		}
		return last;
	}
};

// The candidate walk of extendSeeds (aligner_sw_driver.cpp:278-631) as a resumable
// iterator: next() runs the loop up to its next DP problem (PROBLEM, the problem's key)
// or to the loop's exit (an EXTEND_* code); failed() applies a DP that found nothing.
// The walk's own state (position, per-range samplers, elements left) is a value and the
// per-read state it advances (RNG, limit metrics, seen diagonals) is bound by pointer,
// so a copy bound to copies of those runs ahead of the real walk on the assumption
// that every DP fails: the lookahead the scheduler batches (DpKey, bt2x_align.hpp).
class ExtendWalk {
public:
	static constexpr int PROBLEM = 0;
	ExtendWalk(const Params& P, const std::vector<SatPos>& sat, const std::vector<uint32_t>& rand_ns,
	           const std::vector<size_t>& firstRow, const std::vector<bt2x_resolve_out>& res, size_t nelt,
	           size_t rdlen)
		: P_(&P), sat_(&sat), firstRow_(&firstRow), res_(&res), neltLeft_(nelt), rdlen_(rdlen) {
		rands_.resize(sat.size());
		for(size_t i = 0; i < sat.size(); i++) rands_[i].init((uint16_t)rand_ns[i], false);
	}
	void bind(Rng* rnd, Prm* prm, SeenDiags* seen) { rnd_ = rnd; prm_ = prm; seen_ = seen; }
	int next(int64_t minsc, DpKey& k) {
		const Params& P = *P_;
		const size_t n = (uint16_t)sat_->size();                // gws_size is a uint16_t
		for(;;) {
			if(!inPass_) {                                       // while(neltLeft > 0)
				if(neltLeft_ == 0) return EXTEND_EXHAUSTED_CANDIDATES;
				if(minsc == 0) return EXTEND_PERFECT_SCORE;
				inPass_ = true; i_ = 0; first_ = true;
			}
			if(i_ >= n) { inPass_ = false; continue; }
			const SatPos& sp = (*sat_)[i_];
			const bool is_small = sp.size < kNsm;
			if(rands_[i_].done() || !(first_ || is_small)) { i_++; first_ = true; continue; }
			if(minsc == 0) return EXTEND_PERFECT_SCORE;
			if(prm_->nExDps >= P.mxDp || prm_->nMateDps >= P.mxDp) return EXTEND_EXCEEDED_HARD_LIMIT;
			if(prm_->nExUgs >= P.mxUg || prm_->nMateUgs >= P.mxUg) return EXTEND_EXCEEDED_HARD_LIMIT;
			if(prm_->nExIters >= P.mxIter) return EXTEND_EXCEEDED_HARD_LIMIT;
			prm_->nExIters++;
			first_ = false;
			const bool fw = sp.fw;
			uint32_t rdoff = sp.rdoff;
			if(!fw) rdoff = (uint32_t)(rdlen_ - rdoff - sp.seedlen);
			const uint16_t elt = rands_[i_].next(*rnd_);
			const bt2x_resolve_out& wr = (*res_)[(*firstRow_)[i_] + elt];
			neltLeft_--;
			const int64_t tidx = wr.tidx == BT2X_NO_TIDX ? 0 : (int64_t)wr.tidx;
			const int64_t toff = (int64_t)wr.toff, tlen = (int64_t)wr.tlen;
			const int64_t refoff = toff - (int64_t)rdoff;
			const Coord refcoord(tidx, refoff, fw);
			if(seen_->locusPresent(refcoord)) { prm_->nRedundants++; continue; }
			// DynProgFramer::frameSeedExtensionRect, trimToRef (dp_framer.cpp:81-129)
			const int readGaps = P.maxReadGaps(minsc), refGaps = P.maxRefGaps(minsc);
			const size_t maxgap = std::min((size_t)std::max(readGaps, refGaps), P.maxhalf);
			const int64_t refl_pre = refoff - 2 * (int64_t)maxgap;
			const int64_t refr_pre = refoff + ((int64_t)rdlen_ - 1) + 2 * (int64_t)maxgap;
			size_t triml = 0, trimr = 0;
			if(refr_pre >= tlen) trimr = (size_t)(refr_pre - (tlen - 1));
			if(refl_pre < 0) triml = (size_t)(-refl_pre);
			const int64_t refl = refl_pre + (int64_t)triml, refr = refr_pre - (int64_t)trimr;
			const size_t corel = maxgap, corer = corel + 2 * maxgap;
			seen_->add(Interval(refcoord, 1));
			if(refr < refl) continue;                            // entirely trimmed
			// SwAligner::initRef (aligner_sw.cpp:117-229)
			const size_t ncol = (size_t)(refr - refl + 1);
			if(ncol + 1 > BT2X_MAX_COLS) {
				prm_->nExDpFails++; prm_->nDpFail++;
				return EXTEND_EXCEEDED_HARD_LIMIT;
			}
			seen_->add(Interval(Coord(tidx, refl_pre + (int64_t)corel, fw), (int64_t)(corer - corel + 1)));
			k.tidx = tidx; k.refl = refl; k.minsc = minsc; k.ncol = (uint32_t)ncol;
			k.triml = (uint32_t)triml; k.corel = (uint32_t)corel; k.corer = (uint32_t)corer; k.fw = fw;
			return PROBLEM;
		}
	}
	// the DP of the last next() found no alignment; false: the fail streak ends the walk
	bool failed() {
		prm_->nExDps++; prm_->nExDpFails++; prm_->nDpFail++;
		return prm_->nDpFail < P_->streak;
	}
private:
	static constexpr uint64_t kNsm = 5;                          // prioritizeSATups' nsm
	const Params* P_;
	const std::vector<SatPos>* sat_;
	const std::vector<size_t>* firstRow_;
	const std::vector<bt2x_resolve_out>* res_;
	size_t neltLeft_, rdlen_;
	std::vector<Random1toN> rands_;
	size_t i_ = 0;
	bool first_ = true, inPass_ = false;
	Rng* rnd_ = nullptr;
	Prm* prm_ = nullptr;
	SeenDiags* seen_ = nullptr;
};

// SwAligner::initRef's problem for key k (window = BitPairReference::getStretch).
void pose_dp(std::vector<DpWork>& dps, const RefInfo& ref, const DpKey& k, size_t rdlen, int nceil) {
	dps.emplace_back();
	DpWork& d = dps.back();
	d.key = k;
	std::memset(&d.in, 0, sizeof(d.in));
	d.in.refl = k.refl;
	d.in.rdlen = (uint16_t)rdlen;
	d.in.ncol = (uint16_t)k.ncol;
	d.in.minsc = (int16_t)std::max<int64_t>(k.minsc, -254);
	d.in.nceil = (int16_t)nceil;
	d.in.triml = (uint16_t)k.triml; d.in.corel = (uint16_t)k.corel; d.in.corer = (uint16_t)k.corer;
	d.in.fw = k.fw ? 1 : 0;
	d.window.resize(k.ncol);
	ref.stretch((uint32_t)k.tidx, k.refl, k.ncol, d.window.data());
}

} // namespace

// ---------------------------------------------------------------- SAM header

std::string Aligner::header() const {
	std::string o = "@HD\tVN:1.5\tSO:unsorted\tGO:query\n";
	for(size_t i = 0; i < ref_.nrefs(); i++) {
		o += "@SQ\tSN:";
		append_refname(o, ref_.name(i));
		o += "\tLN:" + std::to_string(ref_.len(i)) + "\n";
	}
	return o;
}

// ------------------------------------------------------------- one read

ReadTask Aligner::align_read(ReadCtx* c) {
	const Params& P = p_;
	Read& rd = c->rd;
	const size_t rdlen = rd.length();
	// P0, bt2_search.cpp:2467-2553
	int64_t minsc = P.scoreMin.f<int64_t>((double)rdlen);
	if(minsc > 0) minsc = 0;
	else if(minsc < -254) minsc = -254;
	Rng rnd;
	rnd.init(rd.seed);
	const int interval = std::max(P.msIval.f<int>((double)rdlen), 1);
	const int nceil = std::min(P.nCeil.f<int>((double)rdlen), (int)rdlen);
	const int swNceil = P.nCeil.f<int>((double)rdlen);      // SwAligner::initRead's nceil
	Sink sink;
	sink.mhits = P.mhits;
	SeenDiags seenDiags;
	RedundantAlns redAnchor;
	redAnchor.init(rdlen);
	std::vector<uint32_t> edbuf;         // SwDriver::resGap_.alres.ned_ storage
	std::unordered_map<DpKey, DpResult, DpKeyHash> memo;   // this read's DP results (lookahead)
	std::vector<ExtendRange> exRange[2];
	Prm prm;
	const uint32_t nrounds = (uint32_t)std::min<int>(P.nSeedRounds, interval);
	const uint32_t L = (uint32_t)std::min<size_t>((size_t)P.multiseedLen, rdlen);
	// reads the u8 DP cannot hold never align (initRead, aligner_sw.cpp:59)
	const bool dpOk = rdlen >= 1 && rdlen <= BT2X_MAX_ROWS;
	for(uint32_t roundi = 0; roundi < nrounds && dpOk; roundi++) {
		const uint32_t offset = (uint32_t)((interval * roundi) / nrounds);
		if(offset > 0 && (size_t)P.multiseedLen + offset > rdlen) break;
		// instantiateSeeds (aligner_seed.cpp:411-447): fw seed i at depth, rc seed at rdlen-depth-L
		const uint32_t nseeds = (rdlen - offset > L) ? 1 + (uint32_t)((rdlen - offset - L) / interval) : 1;
		c->seed.in.clear();
		std::vector<std::pair<uint8_t, uint32_t>> seedIds;          // (fw, idx) of each searched seed
		for(int fwi = 0; fwi < 2; fwi++) {
			const bool fw = fwi == 0;
			if((fw && P.nofw) || (!fw && P.norc)) continue;
			const std::vector<uint8_t>& s = fw ? rd.fw : rd.rc;
			for(uint32_t i = 0; i < nseeds; i++) {
				const uint32_t depth = i * interval + offset;
				const uint32_t st = fw ? depth : (uint32_t)(rdlen - depth - L);
				bool ok = true;
				for(uint32_t k = 0; k < L; k++) if(s[st + k] > 3) { ok = false; break; }
				if(!ok) continue;
				bt2x_seed_in si;
				std::memset(&si, 0, sizeof(si));
				si.read_off = fw ? 0 : rdlen;
				si.seed_off = (uint8_t)st;
				si.seed_len = (uint8_t)L;
				c->seed.in.push_back(si);
				seedIds.push_back({(uint8_t)fw, i});
			}
		}
		if(!c->seed.in.empty()) co_await Awaiter{c, REQ_SEED};
		// searchAllSeedsFinalize + SeedResults::add (aligner_seed.cpp:508-540)
		SeedHitsHip hits;
		hits.reset(nseeds);
		std::vector<std::pair<uint64_t, uint8_t>> cacheNlex;        // AlignmentCache: key -> nlex of the first add
		for(size_t k = 0; k < seedIds.size(); k++) {
			const bt2x_seed_out& d = c->seed.out[k];
			if(!d.need_reporting) continue;
			hits.add(seedIds[k].second, seedIds[k].first != 0, d);
			bool have = false;
			for(auto& e : cacheNlex) if(e.first == d.topf) { have = true; break; }
			if(!have) cacheNlex.push_back({d.topf, d.nlex});
		}
		if(hits.nonzeroOffsets() == 0) break;                        // no seed hits: done
		hits.rankSeedHits(rnd, false);

		// ---------------------------------------------- prioritizeSATups (:61-260)
		std::vector<SatPos> satpos2, satpos;
		std::vector<uint32_t> rand_ns;
		satpos2.reserve(hits.nonzeroOffsets());
		satpos.reserve(std::min<size_t>(P.mxIter, 64));
		rand_ns.reserve(std::min<size_t>(P.mxIter, 64));
		size_t nrange = 0, nelt = 0, nsmall = 0, nsmall_elts = 0;
		const size_t nsm = 5, maxelt = P.mxIter;
		for(size_t r = 0; r < hits.nonzeroOffsets(); r++) {
			uint32_t offidx = 0; bool fw = true;
			const SeedHitsHip::Hit& h = hits.hitsByRank(r, offidx, fw);
			const uint32_t rdoff = offidx * interval + offset;           // idx2off
			const uint32_t seedlen = L;
			SatPos sp;
			sp.topf = h.topf; sp.size = h.numElts(); sp.key = h.topf;
			for(auto& e : cacheNlex) if(e.first == h.topf) { sp.nlex = e.second; break; }
			if(sp.size == 0) continue;
			nrange++; nelt += sp.size;
			bool skip = false;
			for(const ExtendRange& er : exRange[fw ? 0 : 1]) {
				if(er.off <= rdoff && er.off + er.len >= rdoff + seedlen && sp.size <= er.sz) { skip = true; break; }
			}
			if(!skip) for(const SatPos& q : satpos2) skip |= (q.key == sp.key);
			if(skip) { nrange--; nelt -= sp.size; continue; }
			sp.origSz = sp.size;
			sp.fw = fw; sp.offidx = offidx; sp.rdoff = rdoff; sp.seedlen = seedlen;
			satpos2.push_back(sp);
			if(sp.size <= nsm) { nsmall++; nsmall_elts += sp.size; }
			if(sp.nlex > 0) {
				const size_t p5 = rdoff - (fw ? sp.nlex : 0);
				exRange[fw ? 0 : 1].push_back({p5, (size_t)seedlen + sp.nlex, sp.size});
			}
		}
		std::stable_sort(satpos2.begin(), satpos2.end());
		size_t nelt_added = 0;
		for(size_t j = 0; j < nsmall && nelt_added < maxelt; j++) {
			satpos.push_back(satpos2[j]);
			rand_ns.push_back((uint32_t)satpos2[j].size);
			nelt_added += satpos2[j].size;
		}
		if(!(nelt_added >= maxelt || nsmall == satpos2.size())) {
			RowSampler rows;
			rows.init(satpos2, nsmall, satpos2.size());
			std::vector<Random1toN> rands(satpos2.size());
			while(nelt_added < maxelt && nelt_added < nelt) {
				const size_t ri = rows.next(rnd) + nsmall;
				if(!rands[ri].inited()) rands[ri].init((uint16_t)satpos2[ri].size, false);
				const size_t rr = rands[ri].next(rnd);
				if(rands[ri].done()) rows.finishedRange(ri - nsmall);
				SatPos sp = satpos2[ri];
				sp.topf = satpos2[ri].topf + rr;
				sp.size = 1;
				sp.nlex = 0;
				satpos.push_back(sp);
				rand_ns.push_back(1);
				nelt_added++;
			}
		}
		const size_t nelt_ = nelt_added;

		// ----------------------- SA resolution of every element extendSeeds may visit
		c->resolve.in.clear();
		std::vector<size_t> firstRow(satpos.size());
		for(size_t i = 0; i < satpos.size(); i++) {
			firstRow[i] = c->resolve.in.size();
			for(uint32_t e = 0; e < rand_ns[i]; e++) {
				bt2x_resolve_in ri;
				std::memset(&ri, 0, sizeof(ri));
				ri.row = satpos[i].topf + e;
				ri.qlen = satpos[i].seedlen;
				c->resolve.in.push_back(ri);
			}
		}
		if(!c->resolve.in.empty()) co_await Awaiter{c, REQ_RESOLVE};

		// -------------------------------------------------- extendSeeds (:278-631)
		int ret;
		{
			prm.nDpFail = 0;
			const int64_t perfectScore = 0;
			ExtendWalk walk(P, satpos, rand_ns, firstRow, c->resolve.out, nelt_, rdlen);
			walk.bind(&rnd, &prm, &seenDiags);
			for(;;) {
				DpKey key;
				ret = walk.next(minsc, key);
				if(ret != ExtendWalk::PROBLEM) break;
				auto hit = memo.find(key);
				if(hit == memo.end()) {
					// pose this problem and the ones the walk reaches next if each of them
					// fails (a copy of the walk over copies of the state it advances)
					c->dps.clear();
					pose_dp(c->dps, ref_, key, rdlen, swNceil);
					if(P.lookahead > 1) {
						Rng rnd2 = rnd;
						Prm prm2 = prm;
						SeenDiags seen2 = seenDiags;
						ExtendWalk ahead = walk;
						ahead.bind(&rnd2, &prm2, &seen2);
						while(c->dps.size() < P.lookahead && ahead.failed()) {
							DpKey k2;
							if(ahead.next(minsc, k2) != ExtendWalk::PROBLEM) break;
							const auto m = memo.find(k2);
							if(m != memo.end()) {
								if(m->second.out.status != 0) break;    // a known success: stop guessing
								continue;
							}
							bool dup = false;
							for(const DpWork& d : c->dps) dup = dup || d.key == k2;
							if(!dup) pose_dp(c->dps, ref_, k2, rdlen, swNceil);
						}
					}
					co_await Awaiter{c, REQ_DP};
					for(DpWork& d : c->dps) memo.emplace(d.key, std::move(d.res));
					c->dps.clear();
					hit = memo.find(key);
				}
				c->ndp_used++;
				const DpResult& d = hit->second;
				if(d.out.status == 0) {
					if(!walk.failed()) { ret = EXTEND_EXCEEDED_SOFT_LIMIT; break; }
					continue;
				}
				prm.nExDps++;
				prm.nExDpSuccs++;
				if(prm.nDpFail > prm.nDpFailStreak) prm.nDpFailStreak = prm.nDpFail;
				prm.nDpFail = 0;
				bool fulfilled = false;
				const int64_t minsc_posed = minsc;
				for(uint32_t k = 0; k < d.out.nrec; k++) {            // while(!swa.done()) nextAlignment
					const bt2x_aln_rec& rec = d.recs[k];
					// -M tightening below raises minsc between the calls of this problem, but the
					// record sequence needs no re-filtering: nextAlignment's score filter compares
					// the candidate's raw u8 cell value (DpBtCandidate::score = lr in 0..255,
					// aligner_swsse_ee_u8.cpp:519) with minsc <= 0 (aligner_sw.cpp:274), so it
					// never fires and the calls proceed exactly as posed (tests/test_e2e.py,
					// tandem-repeat fixture).
					if(minsc != minsc_posed) c->ntight++;
					replay_backtrace_draws(rnd, rec.ntries);
					// the call's writes to the read's edit buffer (bt2x.h)
					if(edbuf.size() < rec.nbuf) edbuf.resize(rec.nbuf);
					std::copy(d.edits.begin() + rec.edit_off, d.edits.begin() + rec.edit_off + rec.nbuf, edbuf.begin());
					if(!rec.ok) break;
					AlnRes res;
					res.score = rec.score;
					res.bases_aligned = rec.bases_aligned;
					res.refid = key.tidx;
					res.refoff = rec.refoff;
					res.fw = key.fw;
					res.rdlen = rdlen;
					res.refns = rec.refns;
					res.ned.assign(d.edits.begin() + rec.edit_off, d.edits.begin() + rec.edit_off + rec.nedit);
					// (the alignment lies inside [0, tlen): the rectangle is trimmed to the reference)
					if(redAnchor.overlap(res)) continue;
					redAnchor.add(res);
					if(sink.report(res)) { fulfilled = true; break; }
					if(P.tighten > 0 && sink.hasSecondBest()) {
						if(P.tighten == 1) {
							if(sink.best >= minsc) {
								minsc = sink.best;
								if(minsc < perfectScore && sink.best == sink.best2) minsc++;
							}
						} else if(P.tighten == 2) {
							if(sink.best2 >= minsc) { minsc = sink.best2; if(minsc < perfectScore) minsc++; }
						} else {
							const int64_t diff = sink.best - sink.best2;
							const int64_t bot = sink.best2 + ((diff * 3) / 4);
							if(bot >= minsc) { minsc = bot; if(minsc < perfectScore) minsc++; }
						}
					}
				}
				if(fulfilled) { ret = EXTEND_POLICY_FULFILLED; break; }
			}
		}
		if(ret == EXTEND_EXHAUSTED_CANDIDATES || ret == EXTEND_EXCEEDED_SOFT_LIMIT || ret == EXTEND_POLICY_FULFILLED) {
			if(hits.numElts() / hits.nonzeroOffsets() < P.seedBoostThresh) break;   // averageHitsPerSeed
			if(sink.done()) break;                                                  // doneWithMate
		} else {
			break;
		}
	}
	(void)nceil;
	c->sam = finish_read(P, ref_, rd, sink, rnd, edbuf, &c->aligned, &c->repetitive);
	c->req = REQ_NONE;
	co_return;
}

// ------------------------------------------------------------- scheduler

namespace {
double now_s() {
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}

// One scheduler iteration: run the GPU launch for every request kind some read is
// waiting on, then resume those reads (in parallel) until each waits again or finishes.
// Returns false when no read is waiting.
bool Aligner::step(std::vector<ReadCtx*>& act, RunStats& st, int threads) {
	std::vector<ReadCtx*> ws, wr, wd;
	for(ReadCtx* c : act) {
		if(c->req == REQ_SEED) ws.push_back(c);
		else if(c->req == REQ_RESOLVE) wr.push_back(c);
		else if(c->req == REQ_DP) wd.push_back(c);
	}
	if(ws.empty() && wr.empty() && wd.empty()) return false;
	static const bool trace = std::getenv("BT2X_TRACE") != nullptr;
	if(trace) {
		long rss = 0;
		if(std::FILE* f = std::fopen("/proc/self/statm", "r")) { long a = 0; if(std::fscanf(f, "%ld %ld", &a, &rss) != 2) rss = 0; std::fclose(f); }
		std::fprintf(stderr, "BT2X_TRACE active=%zu seed=%zu resolve=%zu dp=%zu rss_mb=%ld\n", act.size(), ws.size(),
		             wr.size(), wd.size(), rss * 4096 / (1 << 20));
	}
	const long nws = (long)ws.size(), nwr = (long)wr.size(), nwd = (long)wd.size();
	if(nws) {
		// one launch for every waiting read's seeds: patFw+patRc of each read, then its
		// seeds with read_off rebased (gather/scatter in parallel over reads)
		double t0 = now_s();
		std::vector<uint64_t> rb(nws + 1, 0), sb(nws + 1, 0);
		for(long i = 0; i < nws; i++) {
			rb[i + 1] = rb[i] + 2 * ws[i]->rd.length();
			sb[i + 1] = sb[i] + ws[i]->seed.in.size();
		}
		std::vector<uint8_t> reads(rb[nws]);
		std::vector<bt2x_seed_in> in(sb[nws]);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nws; i++) {
			const ReadCtx* c = ws[i];
			const size_t L = c->rd.length();
			std::copy(c->rd.fw.begin(), c->rd.fw.end(), reads.begin() + (long)rb[i]);
			std::copy(c->rd.rc.begin(), c->rd.rc.end(), reads.begin() + (long)(rb[i] + L));
			for(size_t k = 0; k < c->seed.in.size(); k++) {
				bt2x_seed_in s = c->seed.in[k];
				s.read_off += rb[i];
				in[sb[i] + k] = s;
			}
		}
		std::vector<bt2x_seed_out> out;
		be_.seed_search(reads, in, out);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nws; i++)
			ws[i]->seed.out.assign(out.begin() + (long)sb[i], out.begin() + (long)sb[i + 1]);
		st.seed_launches++; st.seeds += in.size(); st.t_seed += now_s() - t0;
	}
	if(nwr) {
		double t0 = now_s();
		std::vector<uint64_t> ib(nwr + 1, 0);
		for(long i = 0; i < nwr; i++) ib[i + 1] = ib[i] + wr[i]->resolve.in.size();
		std::vector<bt2x_resolve_in> in(ib[nwr]);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nwr; i++)
			std::copy(wr[i]->resolve.in.begin(), wr[i]->resolve.in.end(), in.begin() + (long)ib[i]);
		std::vector<bt2x_resolve_out> out;
		be_.resolve(in, out);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nwr; i++)
			wr[i]->resolve.out.assign(out.begin() + (long)ib[i], out.begin() + (long)ib[i + 1]);
		st.resolve_launches++; st.resolves += in.size(); st.t_resolve += now_s() - t0;
	}
	if(nwd) {
		double t0 = now_s();
		// every waiting read's posed problems in one launch: the read's two orientations
		// (codes and qualities) once per read, one reference window per problem
		std::vector<uint64_t> qb(nwd + 1, 0), pb(nwd + 1, 0);
		for(long i = 0; i < nwd; i++) {
			qb[i + 1] = qb[i] + 2 * wd[i]->rd.length();
			pb[i + 1] = pb[i] + wd[i]->dps.size();
		}
		const uint64_t np = pb[nwd];
		std::vector<uint64_t> fb(np + 1, 0);
		for(long i = 0; i < nwd; i++)
			for(size_t j = 0; j < wd[i]->dps.size(); j++)
				fb[pb[i] + j + 1] = fb[pb[i] + j] + wd[i]->dps[j].window.size();
		std::vector<uint8_t> reads(qb[nwd]), quals(qb[nwd]), refs(fb[np]);
		std::vector<bt2x_dp_in> in(np);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nwd; i++) {
			const ReadCtx* c = wd[i];
			const size_t L = c->rd.length();
			std::copy(c->rd.fw.begin(), c->rd.fw.end(), reads.begin() + (long)qb[i]);
			std::copy(c->rd.rc.begin(), c->rd.rc.end(), reads.begin() + (long)(qb[i] + L));
			std::copy(c->rd.qual.begin(), c->rd.qual.end(), quals.begin() + (long)qb[i]);
			std::copy(c->rd.qualRev.begin(), c->rd.qualRev.end(), quals.begin() + (long)(qb[i] + L));
			for(size_t j = 0; j < c->dps.size(); j++) {
				const DpWork& d = c->dps[j];
				const uint64_t k = pb[i] + j;
				bt2x_dp_in p = d.in;
				p.read_off = p.qual_off = qb[i] + (d.key.fw ? 0 : L);
				p.ref_off = fb[k];
				std::copy(d.window.begin(), d.window.end(), refs.begin() + (long)fb[k]);
				in[k] = p;
			}
		}
		std::vector<bt2x_dp_out> out;
		std::vector<bt2x_aln_rec> recs;
		std::vector<uint32_t> edits;
		be_.dp_align(reads, quals, refs, in, out, recs, edits);
#pragma omp parallel for schedule(static, 256) num_threads(threads)
		for(long i = 0; i < nwd; i++) {
			for(size_t j = 0; j < wd[i]->dps.size(); j++) {
				const uint64_t k = pb[i] + j;
				DpResult& r = wd[i]->dps[j].res;
				r.out = out[k];
				r.recs.assign(recs.begin() + out[k].rec_off, recs.begin() + out[k].rec_off + out[k].nrec);
				// gather each record's edit-buffer image (arena offsets are allocated by the
				// kernel's atomics, so one problem's images are not contiguous)
				r.edits.clear();
				for(bt2x_aln_rec& a : r.recs) {
					const uint32_t o = (uint32_t)r.edits.size();
					r.edits.insert(r.edits.end(), edits.begin() + a.edit_off, edits.begin() + a.edit_off + a.nbuf);
					a.edit_off = o;
				}
			}
		}
		st.dp_launches++; st.dps += np; st.t_dp += now_s() - t0;
	}
	// resume the reads whose requests were served
	std::vector<ReadCtx*> run;
	run.reserve(ws.size() + wr.size() + wd.size());
	run.insert(run.end(), ws.begin(), ws.end());
	run.insert(run.end(), wr.begin(), wr.end());
	run.insert(run.end(), wd.begin(), wd.end());
	double t0 = now_s();
	const long nrun = (long)run.size();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
	for(long i = 0; i < nrun; i++) {
		run[i]->req = REQ_NONE;
		run[i]->task.h.resume();
	}
	st.t_host += now_s() - t0;
	return true;
}

RunStats Aligner::run(FastqReader& fq, std::FILE* out, size_t slots, int threads) {
	RunStats st;
	const std::string hdr = header();
	std::fwrite(hdr.data(), 1, hdr.size(), out);
	uint64_t rdid = 0;
	bool eof = false;
	std::vector<std::unique_ptr<ReadCtx>> window;   // reads in input order, not yet written
	size_t head = 0;                                // first unwritten read in `window`
	std::vector<ReadCtx*> act;
	while(true) {
		// refill the pool
		double t0 = now_s();
		std::vector<ReadCtx*> fresh;
		std::vector<FastqReader::Raw> raw;
		if(!eof && act.size() < slots) {
			const size_t want = slots - act.size();
			if(fq.take(want, raw) < want) eof = true;
		}
		st.t_io += now_s() - t0;
		const long nf = (long)raw.size();
		if(nf) {
			t0 = now_s();
			fresh.resize((size_t)nf);
			for(long i = 0; i < nf; i++) {
				window.emplace_back(new ReadCtx());
				fresh[(size_t)i] = window.back().get();
			}
			// decode + run each new read up to its first request, in parallel
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
			for(long i = 0; i < nf; i++) {
				ReadCtx* c = fresh[(size_t)i];
				FastqReader::decode(raw[(size_t)i], c->rd, rdid + (uint64_t)i, p_.randSeed);
				c->task = align_read(c);
				c->task.h.resume();
			}
			rdid += (uint64_t)nf;
			st.t_host += now_s() - t0;
			act.insert(act.end(), fresh.begin(), fresh.end());
		}
		if(act.empty()) break;
		step(act, st, threads);
		// retire finished reads; write records in input order
		std::vector<ReadCtx*> still;
		still.reserve(act.size());
		for(ReadCtx* c : act) {
			if(c->task.h.done()) {
				c->task.h.destroy();
				c->task.h = nullptr;
			} else {
				still.push_back(c);
			}
		}
		act.swap(still);
		t0 = now_s();
		while(head < window.size() && window[head] && !window[head]->task.h) {
			ReadCtx* c = window[head].get();
			std::fwrite(c->sam.data(), 1, c->sam.size(), out);
			st.reads++;
			if(c->aligned) st.aligned++; else st.unaligned++;
			if(c->repetitive) st.rep++;
			st.dps_used += c->ndp_used;
			st.tight_recs += c->ntight;
			window[head].reset();
			head++;
		}
		if(head > (1u << 16) && head * 2 > window.size()) {
			window.erase(window.begin(), window.begin() + (long)head);
			head = 0;
		}
		st.t_io += now_s() - t0;
	}
	return st;
}

std::string Aligner::align_all(std::vector<Read>& reads, size_t slots, int threads, RunStats* stp) {
	RunStats st;
	std::vector<std::unique_ptr<ReadCtx>> ctx(reads.size());
	std::string out;
	size_t next = 0, head = 0;
	std::vector<ReadCtx*> act;
	while(true) {
		std::vector<ReadCtx*> fresh;
		while(next < reads.size() && act.size() + fresh.size() < slots) {
			ctx[next].reset(new ReadCtx());
			ctx[next]->rd = reads[next];
			ctx[next]->task = align_read(ctx[next].get());
			fresh.push_back(ctx[next].get());
			next++;
		}
		const long nf = (long)fresh.size();
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
		for(long i = 0; i < nf; i++) fresh[i]->task.h.resume();
		act.insert(act.end(), fresh.begin(), fresh.end());
		if(act.empty()) break;
		step(act, st, threads);
		std::vector<ReadCtx*> still;
		for(ReadCtx* c : act) {
			if(c->task.h.done()) { c->task.h.destroy(); c->task.h = nullptr; }
			else still.push_back(c);
		}
		act.swap(still);
		while(head < next && !ctx[head]->task.h) {
			out += ctx[head]->sam;
			st.reads++;
			if(ctx[head]->aligned) st.aligned++; else st.unaligned++;
			st.dps_used += ctx[head]->ndp_used;
			st.tight_recs += ctx[head]->ntight;
			ctx[head].reset();
			head++;
		}
	}
	if(stp) *stp = st;
	return out;
}

} // namespace host
} // namespace bt2x
