// bt2x_align.hpp — end-to-end host driver of the MI355X aligner: FASTQ in, SAM out,
// with every seed search, SA resolution and DP fill/backtrace on the GPU (through a
// Backend; the product backend is the bt2x C-ABI, include/bt2x.h).
//
// The reference runs one read per OpenMP slot through the phase loop of
// multiseedSearchWorker (bt2_search.cpp:2297-2888).  Here each read is a C++20
// coroutine (align_read) that keeps the reference's per-read control flow verbatim and
// suspends wherever the reference would call a hot-path kernel:
//
//   co_await SeedReq      MultiSeedAligner::searchAllSeedsDoAll   (aligner_seed.cpp:674)
//   co_await ResolveReq   GroupWalk2S::advanceElement + joinedToTextOff (group_walk.h:969,
//                         bt2_idx.cpp:54) for every element prioritizeSATups may visit
//   co_await DpReq        SwAligner::align + the nextAlignment sequence (aligner_sw.cpp:235,252)
//
// The Scheduler keeps a pool of reads in flight (a much larger -p), resumes the runnable
// ones in parallel on the host cores, and turns all requests of one kind into one GPU
// launch.  Per-read state (RNG, seen diagonals, redundancy sets, -M tightening, limits)
// never crosses reads, so batching preserves the reference's results read by read.
//
// Host semantics restated here (file:line of the reference):
//   RandomSource            random_source.h:34-140
//   Random1toN              random_util.h:32-230
//   RowSampler              aligner_sw_driver.h:176-267
//   EIvalMergeList(Binned)  ival_list.h (Coord/Interval ref_coord.h)
//   RedundantAlns           aligner_result.cpp:821-914
//   prioritizeSATups        aligner_sw_driver.cpp:61-260
//   extendSeeds             aligner_sw_driver.cpp:278-631
//   frameSeedExtensionRect  dp_framer.cpp:81-129
//   ReportingState / AlnSinkWrap::report / finishRead / selectByScore
//                           aln_sink.cpp:33-210, 643-1384, 1395-1640
//   BowtieMapq2             unique.h:171-380
//   StackedAln (CIGAR, MD)  aligner_result.cpp:448-770
//   SAM record              aln_sink.cpp:1889-2090, sam.cpp:121-730
//   FASTQ parse, genRandSeed pat.cpp:45-88, 1124-1220
#pragma once
#include <algorithm>
#include <cctype>
#include <cmath>
#include <coroutine>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "bt2x.h"
#include "bt2x_shims.hpp"

namespace bt2x {
namespace host {

// ------------------------------------------------------------------ RNG & sampling

// RandomSource, LCG variant (random_source.h:34-140; MERSENNE_TWISTER is off).
struct Rng {
	uint32_t last = 0;
	int lastOff = 30;
	void init(uint32_t s) { last = s; lastOff = 30; }
	uint32_t nextU32() {
		last = 1664525u * last + 1013904223u;
		uint32_t r = last >> 16;
		last = 1664525u * last + 1013904223u;
		r ^= last;
		lastOff = 0;
		return r;
	}
	uint64_t nextU64() { uint64_t a = nextU32(); a <<= 32; return a | nextU32(); }
	size_t nextSizeT() { return (size_t)nextU64(); }
	bool nextBool() {
		if(lastOff > 31) nextU32();
		const uint32_t r = (last >> lastOff) & 1;
		lastOff++;
		return r != 0;
	}
	float nextFloat() { return (float)nextU32() / (float)0xffffffff; }
};

// Random1toN: sampling without replacement, uint16_t domain (random_util.h:32-230).
class Random1toN {
public:
	void init(uint16_t n, bool withoutReplacement) {
		sz_ = n_ = n;
		converted_ = false;
		swaplist_ = n < 128 || withoutReplacement;
		cur_ = 0;
		list_.clear();
		seen_.clear();
		thresh_ = std::max<uint16_t>(16, (uint16_t)(0.10f * n));
	}
	void reset() {
		sz_ = n_ = cur_ = 0; swaplist_ = converted_ = false;
		list_.clear(); seen_.clear(); thresh_ = 0;
	}
	uint16_t next(Rng& rnd) {
		if(cur_ == 0 && !converted_) {
			if(n_ == 1) { cur_ = 1; return 0; }
			if(swaplist_) {
				list_.resize(n_);
				for(uint16_t i = 0; i < n_; i++) list_[i] = i;
			}
		}
		if(swaplist_) {
			const uint16_t r = (uint16_t)(cur_ + (rnd.nextU32() % (uint32_t)(n_ - cur_)));
			if(r != cur_) std::swap(list_[cur_], list_[r]);
			return list_[cur_++];
		}
		bool again = true;
		uint16_t rn = 0;
		const uint16_t seenSz = (uint16_t)seen_.size();
		while(again) {
			rn = (uint16_t)(rnd.nextU32() % (uint32_t)n_);
			again = false;
			for(uint16_t i = 0; i < seenSz; i++) if(seen_[i] == rn) { again = true; break; }
		}
		seen_.push_back(rn);
		cur_++;
		if(seen_.size() >= thresh_ && cur_ < n_) {
			std::sort(seen_.begin(), seen_.end());
			list_.resize(n_ - cur_);
			uint16_t prev = 0, cur = 0;
			for(uint16_t i = 0; i <= seenSz; i++) {
				for(uint16_t j = prev; j < seen_[i]; j++) list_[cur++] = j;
				prev = (uint16_t)(seen_[i] + 1);
			}
			for(uint16_t j = prev; j < n_; j++) list_[cur++] = j;
			seen_.clear();
			cur_ = 0;
			n_ = (uint16_t)list_.size();
			converted_ = true;
			swaplist_ = true;
		}
		return rn;
	}
	bool inited() const { return n_ > 0; }
	bool done() const { return inited() && cur_ >= n_; }
private:
	uint16_t sz_ = 0, n_ = 0, cur_ = 0, thresh_ = 0;
	bool swaplist_ = false, converted_ = false;
	std::vector<uint16_t> list_, seen_;
};

// ------------------------------------------------------------ coordinates & intervals

struct Coord {                      // ref_coord.h Coord: order (ref, orient, off)
	int64_t ref = std::numeric_limits<int64_t>::max();
	int64_t off = std::numeric_limits<int64_t>::max();
	int orient = -1;
	Coord() = default;
	Coord(int64_t r, int64_t o, bool fw) : ref(r), off(o), orient(fw ? 1 : 0) {}
	bool operator<(const Coord& o) const {
		if(ref != o.ref) return ref < o.ref;
		if(orient != o.orient) return orient < o.orient;
		return off < o.off;
	}
	bool operator>(const Coord& o) const { return o < *this; }
	bool operator>=(const Coord& o) const { return !(*this < o); }
};

struct Interval {                   // ref_coord.h Interval
	Coord up;
	int64_t len = 0;
	Interval() = default;
	Interval(const Coord& u, int64_t l) : up(u), len(l) {}
	bool operator<(const Interval& o) const {
		if(up < o.up) return true;
		if(up > o.up) return false;
		return len < o.len;
	}
	Coord downstream() const { Coord c = up; c.off += len; return c; }
	bool contains(const Coord& c) const {
		return c.ref == up.ref && c.orient == up.orient && c.off >= up.off && c.off < up.off + len;
	}
};

// EIvalMergeList (ival_list.h): 16 unsorted intervals, then sort + merge on flush.
class IvalMergeList {
public:
	void add(const Interval& i) {
		if(unsorted_.size() < 16) unsorted_.push_back(i);
		if(unsorted_.size() == 16) flush();
	}
	bool locusPresent(const Coord& loc) const {
		for(const Interval& iv : unsorted_) if(iv.contains(loc)) return true;
		if(sorted_.empty()) return false;
		const size_t beg = (size_t)(std::lower_bound(lhs_.begin(), lhs_.end(), loc) - lhs_.begin());
		if(beg == lhs_.size() || lhs_[beg] > loc) {
			if(beg == 0) return false;
			return sorted_[beg - 1].contains(loc);
		}
		return true;
	}
private:
	void flush() {
		for(const Interval& iv : unsorted_) sorted_.push_back(iv);
		std::stable_sort(sorted_.begin(), sorted_.end());
		size_t nmerged = 0;
		for(size_t i = 1; i < sorted_.size(); i++) {
			if(sorted_[i - 1].downstream() >= sorted_[i].up) {
				nmerged++;
				const Coord up = std::min(sorted_[i - 1].up, sorted_[i].up);
				const Coord dn = std::max(sorted_[i - 1].downstream(), sorted_[i].downstream());
				sorted_[i].up = up;
				sorted_[i].len = dn.off - up.off;
				sorted_[i - 1] = Interval();
			}
		}
		std::stable_sort(sorted_.begin(), sorted_.end());
		sorted_.resize(sorted_.size() - nmerged);
		lhs_.clear();
		for(const Interval& iv : sorted_) lhs_.push_back(iv.up);
		unsorted_.clear();
	}
	std::vector<Interval> sorted_, unsorted_;
	std::vector<Coord> lhs_;
};

// EIvalMergeListBinned: 128 bins by reference id; bins are created on first use.
class SeenDiags {
public:
	void clear() { bins_.clear(); }
	void add(const Interval& i) { bin((uint32_t)(i.up.ref & 127), true)->add(i); }
	bool locusPresent(const Coord& c) const {
		const IvalMergeList* b = const_cast<SeenDiags*>(this)->bin((uint32_t)(c.ref & 127), false);
		return b != nullptr && b->locusPresent(c);
	}
private:
	IvalMergeList* bin(uint32_t k, bool create) {
		for(auto& p : bins_) if(p.first == k) return &p.second;
		if(!create) return nullptr;
		bins_.emplace_back(k, IvalMergeList());
		return &bins_.back().second;
	}
	std::vector<std::pair<uint32_t, IvalMergeList>> bins_;
};

// ----------------------------------------------------------------------- alignments

enum { ET_READ_GAP = 1, ET_REF_GAP = 2, ET_MM = 3 };
inline uint32_t e_pos(uint32_t e) { return BT2X_EDIT_POS(e); }
inline uint32_t e_type(uint32_t e) { return BT2X_EDIT_TYPE(e); }
inline char e_chr(uint32_t e) { return BT2X_EDIT_CHR(e); }
inline uint32_t e_setpos(uint32_t e, uint32_t p) { return (e & ~0x3ffu) | (p & 0x3ffu); }

// Edit::invertPoss(edits, sz, sort=false) (edit.cpp:50-80): reverse, then mirror pos.
inline std::vector<uint32_t> invert_poss(const std::vector<uint32_t>& ed, size_t sz) {
	std::vector<uint32_t> out(ed.rbegin(), ed.rend());
	for(uint32_t& e : out) {
		const uint32_t p = e_pos(e);
		e = e_setpos(e, (uint32_t)(sz - p - (e_type(e) == ET_READ_GAP ? 0 : 1)));
	}
	return out;
}

// AlnScore: only the score orders alignments (aligner_result.h:57-255).
struct AlnRes {                     // the AlnRes fields the unpaired SAM path reads
	int64_t score = 0;
	int bases_aligned = 0;
	int64_t refid = 0, refoff = 0;
	bool fw = true;
	size_t rdlen = 0;               // rdexrows_ (end-to-end: the whole read)
	size_t refns = 0;
	std::vector<uint32_t> ned;      // edits in ned() order (5'-relative after invertEdits)
};

// RedundantAlns (aligner_result.cpp:821-914): DP cells already used by an alignment.
// The reference keeps one ESet per read row; here one open-addressing set of
// (ref, strand, column, row) cells, empty (and never walked) until the first add.
class RedundantAlns {
public:
	void init(size_t) { slots_.clear(); n_ = 0; }
	void add(const AlnRes& r) { walk(r, true); }
	bool overlap(const AlnRes& r) { return n_ != 0 && walk(r, false); }
private:
	// one cell in 16 bytes: reference offset, and (ref id, row, strand) packed; kEmpty marks a
	// free slot (ref ids < 2^40, rows < 2^11)
	struct Cell { int64_t rfoff = 0; uint64_t tag = kEmpty; };
	static constexpr uint64_t kEmpty = ~0ULL;
	static uint64_t tag_of(int64_t rfid, bool fw, uint32_t row) {
		return ((uint64_t)rfid << 12) | ((uint64_t)row << 1) | (fw ? 1u : 0u);
	}
	static uint64_t hash(int64_t rfoff, uint64_t tag) {
		uint64_t z = (uint64_t)rfoff * 0x9e3779b97f4a7c15ULL ^ tag;
		z ^= z >> 29; z *= 0xbf58476d1ce4e5b9ULL; z ^= z >> 32;
		return z;
	}
	bool find_or_insert(int64_t rfid, bool fw, int64_t rfoff, uint32_t row, bool insert) {
		return probe(rfoff, tag_of(rfid, fw, row), insert);
	}
	bool probe(int64_t rfoff, uint64_t tag, bool insert) {
		if(slots_.empty()) { if(!insert) return false; slots_.resize(256); }
		else if(insert && (n_ + 1) * 2 > slots_.size()) {
			std::vector<Cell> old;
			old.swap(slots_);
			slots_.resize(old.size() * 2);
			n_ = 0;
			for(const Cell& c : old) if(c.tag != kEmpty) probe(c.rfoff, c.tag, true);
		}
		const size_t mask = slots_.size() - 1;
		for(size_t h = hash(rfoff, tag) & mask;; h = (h + 1) & mask) {
			Cell& c = slots_[h];
			if(c.tag == kEmpty) {
				if(insert) { c.rfoff = rfoff; c.tag = tag; n_++; }
				return false;
			}
			if(c.tag == tag && c.rfoff == rfoff) return true;
		}
	}
	bool walk(const AlnRes& r, bool insert) {
		int64_t left = r.refoff, right;
		const size_t len = r.rdlen;
		std::vector<uint32_t> inv;
		if(!r.fw) inv = invert_poss(r.ned, r.rdlen);
		const std::vector<uint32_t>& ned = r.fw ? r.ned : inv;
		size_t ni = 0;
		for(size_t i = 0; i < len; i++) {
			size_t diff = 1;
			right = left + 1;
			while(ni < ned.size() && e_pos(ned[ni]) == i) {
				if(e_type(ned[ni]) == ET_REF_GAP) diff = 0;
				ni++;
			}
			if(i < len - 1) {
				size_t nn = ni;
				while(nn < ned.size() && e_pos(ned[nn]) == i + 1) {
					if(e_type(ned[nn]) == ET_READ_GAP) right++;
					nn++;
				}
			}
			for(int64_t j = left; j < right; j++) {
				const bool found = find_or_insert(r.refid, r.fw, j, (uint32_t)i, insert);
				if(!insert && found) return true;
			}
			left = right + diff - 1;
		}
		return false;
	}
	std::vector<Cell> slots_;
	size_t n_ = 0;
};

// ------------------------------------------------------------------------ parameters

struct SimpleFunc {                 // simple_func.h:40-112 (LINEAR / SQRT)
	int type = 1;                   // 1 = const, 2 = linear, 3 = sqrt, 4 = log
	double I = -std::numeric_limits<double>::max(), X = std::numeric_limits<double>::max(), C = 0, L = 0;
	double raw(double x) const {
		double v = type == 1 ? 0.0 : type == 2 ? x : type == 3 ? std::sqrt(x) : std::log(x);
		return std::max(I, std::min(X, C + L * v));
	}
	template<typename T> T f(double x) const {
		const double r = raw(x);
		if(r == std::numeric_limits<double>::max()) return std::numeric_limits<T>::max();
		if(r == std::numeric_limits<double>::min()) return std::numeric_limits<T>::min();
		return (T)r;
	}
};

struct Params {
	// scoring (scoring.h defaults; the DP kernel holds the per-quality tables)
	bt2x_scoring sc;
	SimpleFunc scoreMin, nCeil, msIval;
	int multiseedLen = 22;          // -L
	int nSeedRounds = 2;            // -R
	size_t maxhalf = 15;            // --dpad
	size_t mxIter = 400, mxDp = 300, mxUg = 300, streak = 15;   // -D (maxDpStreak)
	uint64_t seedBoostThresh = 300;
	int64_t mhits = 50;             // -M (msample)
	int tighten = 3;
	uint32_t randSeed = 0;          // --seed
	bool nofw = false, norc = false;
	size_t lookahead = 16;          // DP problems posed per request (not a reference option;
	                                // results do not depend on it)
	Params() {
		bt2x_scoring_default(&sc);
		scoreMin.type = 2; scoreMin.C = (double)-0.6f; scoreMin.L = (double)-0.6f;       // L,-0.6,-0.6
		nCeil.type = 2; nCeil.I = 0.0; nCeil.C = (double)0.0f; nCeil.L = (double)0.15f;   // L,0,0.15
		msIval.type = 3; msIval.I = (double)1.0f; msIval.C = 1.0; msIval.L = 1.15;       // S,1,1.15
	}
	int readGapOpen() const { return sc.rdg_const + sc.rdg_linear; }
	int readGapExtend() const { return sc.rdg_linear; }
	int refGapOpen() const { return sc.rfg_const + sc.rfg_linear; }
	int refGapExtend() const { return sc.rfg_linear; }
	// Scoring::maxReadGaps / maxRefGaps (scoring.cpp:42-98); match bonus 0 end-to-end
	int maxReadGaps(int64_t minsc) const {
		int64_t s = 0; bool first = true; int num = 0;
		while(s >= minsc) { s -= first ? readGapOpen() : readGapExtend(); first = false; num++; }
		return num - 1;
	}
	int maxRefGaps(int64_t minsc) const {
		int64_t s = 0; bool first = true; int num = 0;
		while(s >= minsc) { s -= first ? refGapOpen() : refGapExtend(); first = false; num++; }
		return num - 1;
	}
};

// The bowtie2-align-l options that change the hot path's results (bt2_search.cpp:446-643;
// presets expand to -D/-R/-L/-i, SeedAlignmentPolicy).  Returns the number of argv
// entries consumed at argv[i] (0: not one of these).  bt2x_scoring_init() must follow.
inline int parse_align_option(Params& p, int argc, char** argv, int i) {
	const std::string a = argv[i];
	const bool has = i + 1 < argc;
	auto pair = [&](int& x, int& y) { std::sscanf(argv[i + 1], "%d,%d", &x, &y); };
	if(!has) return 0;
	if(a == "--dpad") { p.maxhalf = (size_t)std::atol(argv[i + 1]); return 2; }
	if(a == "-D") { p.streak = (size_t)std::atol(argv[i + 1]); return 2; }
	if(a == "-R") { p.nSeedRounds = std::atoi(argv[i + 1]); return 2; }
	if(a == "-L") { p.multiseedLen = std::atoi(argv[i + 1]); return 2; }
	if(a == "--seed") { p.randSeed = (uint32_t)std::atol(argv[i + 1]); return 2; }
	if(a == "--mp") { int mx = p.sc.mm_max, mn = p.sc.mm_min; pair(mx, mn); p.sc.mm_max = mx; p.sc.mm_min = mn; return 2; }
	if(a == "--np") { p.sc.n_pen = std::atoi(argv[i + 1]); return 2; }
	if(a == "--rdg") { pair(p.sc.rdg_const, p.sc.rdg_linear); return 2; }
	if(a == "--rfg") { pair(p.sc.rfg_const, p.sc.rfg_linear); return 2; }
	if(a == "--gbar") { p.sc.gapbar = std::atoi(argv[i + 1]); return 2; }
	if(a == "--lookahead") { p.lookahead = (size_t)std::max(1L, std::atol(argv[i + 1])); return 2; }
	return 0;
}

// ----------------------------------------------------------------------- reads

extern const uint8_t kAsc2Dna[256];

struct Read {
	uint64_t rdid = 0;
	std::string name;               // whole header line after '@'
	std::vector<uint8_t> fw, rc;    // patFw / patRc codes 0..4
	std::string qual, qualRev;      // Phred+33
	uint32_t seed = 0;
	size_t length() const { return fw.size(); }
};

// genRandSeed (pat.cpp:45-88)
inline uint32_t gen_rand_seed(const Read& r, uint32_t seed) {
	uint32_t rseed = (seed + 101) * 59 * 61 * 67 * 71 * 73 * 79 * 83;
	for(size_t i = 0; i < r.fw.size(); i++) rseed ^= ((uint32_t)r.fw[i] << ((i & 15) << 1));
	for(size_t i = 0; i < r.fw.size(); i++) rseed ^= (uint32_t)((int)(signed char)r.qual[i] << ((i & 3) << 3));
	for(size_t i = 0; i < r.name.size(); i++) {
		const int p = (int)(signed char)r.name[i];
		if(p == '/') break;
		rseed ^= (uint32_t)(p << ((i & 3) << 3));
	}
	return rseed;
}

// FASTQ input (FastqPatternSource light parse + parse, pat.cpp:1124-1220), Phred+33
// only; '.' is N, non-alphabetic sequence characters are skipped.  The file is mapped:
// take() finds record boundaries (four lines each) serially with memchr, decode() builds
// the Read (codes, reverse complement, genRandSeed) and runs in parallel over records.
class FastqReader {
public:
	struct Raw { const char* l[4]; size_t n[4]; };
	explicit FastqReader(const char* path);
	~FastqReader();
	FastqReader(const FastqReader&) = delete;
	FastqReader& operator=(const FastqReader&) = delete;
	// up to `max` more records appended to `out`; returns how many
	size_t take(size_t max, std::vector<Raw>& out) {
		size_t k = 0;
		while(k < max) {
			Raw r;
			const char* s;
			size_t n;
			do { if(!line(s, n)) return k; } while(n == 0);
			r.l[0] = s; r.n[0] = n;
			for(int j = 1; j < 4; j++) { if(!line(s, n)) { s = map_ + len_; n = 0; } r.l[j] = s; r.n[j] = n; }
			out.push_back(r);
			k++;
		}
		return k;
	}
	static void decode(const Raw& raw, Read& r, uint64_t rdid, uint32_t randSeed) {
		if(raw.l[0][0] != '@') throw std::runtime_error("FASTQ record does not start with '@'");
		r = Read();
		r.rdid = rdid;
		r.name.assign(raw.l[0] + 1, raw.n[0] - 1);
		r.fw.reserve(raw.n[1]);
		for(size_t i = 0; i < raw.n[1]; i++) {
			const unsigned char c = (unsigned char)(raw.l[1][i] == '.' ? 'N' : raw.l[1][i]);
			if(std::isalpha(c)) r.fw.push_back(kAsc2Dna[c]);
		}
		if(raw.n[1] || raw.n[3]) r.qual.assign(raw.l[3], raw.n[3]);
		if(r.qual.size() != r.fw.size())
			throw std::runtime_error("read " + r.name + ": qualities and sequence differ in length");
		if(r.name.empty()) r.name = std::to_string(rdid);
		const size_t L = r.fw.size();
		r.rc.resize(L);
		for(size_t i = 0; i < L; i++) {
			const uint8_t c = r.fw[L - 1 - i];
			r.rc[i] = c < 4 ? (uint8_t)(3 - c) : (uint8_t)4;
		}
		r.qualRev.assign(r.qual.rbegin(), r.qual.rend());
		r.seed = gen_rand_seed(r, randSeed);
	}
private:
	bool line(const char*& s, size_t& n) {
		if(pos_ >= len_) return false;
		s = map_ + pos_;
		const char* nl = (const char*)std::memchr(s, '\n', len_ - pos_);
		n = nl ? (size_t)(nl - s) : len_ - pos_;
		pos_ += n + (nl ? 1 : 0);
		while(n > 0 && s[n - 1] == '\r') n--;
		return true;
	}
	const char* map_ = nullptr;
	size_t len_ = 0, pos_ = 0;
	int fd_ = -1;
};

// ------------------------------------------------------------------- reference

// What the driver needs of the index besides the device copy: reference names and
// lengths (SAM header, plen), and BitPairReference::getStretch over the joined 2-bit
// text (fragment records rstarts: joined offset, text id, text offset).
class RefInfo {
public:
	void init(const bt2x_index_desc& d, const std::string& base);
	size_t nrefs() const { return names_.size(); }
	const std::string& name(size_t i) const { return names_[i]; }
	uint64_t len(size_t i) const { return plen_[i]; }
	// codes of reference tidx over [off, off+n); positions outside a fragment are N
	void stretch(uint32_t tidx, int64_t off, size_t n, uint8_t* out) const;
private:
	struct Frag { int64_t toff; uint64_t len; uint64_t joff; };
	std::vector<std::string> names_;
	std::vector<uint64_t> plen_;
	std::vector<std::vector<Frag>> frags_;
	const uint8_t* text_ = nullptr;
};

// -------------------------------------------------------------- GPU requests

struct SeedWork {                   // one seed round of one read
	std::vector<bt2x_seed_in> in;   // read_off: 0 = patFw, rdlen = patRc
	std::vector<bt2x_seed_out> out;
};
struct ResolveWork {
	std::vector<bt2x_resolve_in> in;
	std::vector<bt2x_resolve_out> out;
};
// A DP problem of one read is fixed by its rectangle and floor: the read, its
// qualities and the N ceiling do not change within the read, and the kernel draws no
// random numbers (it reports how many the reference's backtrace draws, bt2x.h).  So a
// read's results can be memoised by this key and posed ahead of need (lookahead).
struct DpKey {
	int64_t tidx = 0, refl = 0, minsc = 0;
	uint32_t ncol = 0, triml = 0, corel = 0, corer = 0;
	bool fw = true;
	bool operator==(const DpKey& o) const {
		return tidx == o.tidx && refl == o.refl && minsc == o.minsc && ncol == o.ncol && triml == o.triml &&
		       corel == o.corel && corer == o.corer && fw == o.fw;
	}
};
struct DpKeyHash {
	size_t operator()(const DpKey& k) const {
		uint64_t z = (uint64_t)k.refl * 0x9e3779b97f4a7c15ULL ^ ((uint64_t)k.tidx << 32) ^ ((uint64_t)k.minsc << 16) ^
		             ((uint64_t)k.ncol << 1) ^ (k.fw ? 1u : 0u) ^ ((uint64_t)k.triml << 40) ^ ((uint64_t)k.corel << 48);
		z ^= z >> 29; z *= 0xbf58476d1ce4e5b9ULL; z ^= z >> 32;
		return (size_t)z;
	}
};
struct DpResult {                   // SwAligner::align + its nextAlignment sequence
	bt2x_dp_out out;
	std::vector<bt2x_aln_rec> recs; // edit_off relative to `edits`
	std::vector<uint32_t> edits;    // each record's edit-buffer image (nbuf entries)
};
struct DpWork {                     // one posed problem
	DpKey key;
	bt2x_dp_in in;                  // read_off / qual_off / ref_off are set by the scheduler
	std::vector<uint8_t> window;
	DpResult res;
};

enum ReqKind { REQ_NONE = 0, REQ_SEED = 1, REQ_RESOLVE = 2, REQ_DP = 3 };

struct ReadTask {
	struct promise_type {
		ReadTask get_return_object() { return ReadTask{std::coroutine_handle<promise_type>::from_promise(*this)}; }
		std::suspend_always initial_suspend() noexcept { return {}; }
		std::suspend_always final_suspend() noexcept { return {}; }
		void return_void() {}
		void unhandled_exception() { throw; }
	};
	std::coroutine_handle<promise_type> h;
};

struct ReadCtx;
struct Awaiter {
	ReadCtx* c;
	int kind;
	bool await_ready() const noexcept { return false; }
	void await_suspend(std::coroutine_handle<>) noexcept;
	void await_resume() const noexcept {}
};

// Per-read metrics used by the limits (PerReadMetrics, read.h:339)
struct Prm {
	uint64_t nExIters = 0, nExDps = 0, nExUgs = 0, nMateDps = 0, nMateUgs = 0;
	uint64_t nDpFail = 0, nExDpFails = 0, nExDpSuccs = 0, nDpFailStreak = 0, nRedundants = 0;
	int64_t bestLtMinscMate1 = std::numeric_limits<int64_t>::min();
};

struct ReadCtx {
	Read rd;
	int req = REQ_NONE;
	SeedWork seed;
	ResolveWork resolve;
	std::vector<DpWork> dps;        // the problems posed by the current DP request
	std::string sam;                // the finished record(s)
	ReadTask task;
	// statistics for the run summary
	bool aligned = false, repetitive = false;
	uint64_t ndp_used = 0;          // DP results the walk consumed (the rest were lookahead)
	uint64_t ntight = 0;            // nextAlignment records consumed after -M tightened minsc
	                                // within the same DP problem
};

inline void Awaiter::await_suspend(std::coroutine_handle<>) noexcept { c->req = kind; }

// ------------------------------------------------------------------ backend

class Backend {
public:
	virtual ~Backend() {}
	// reads: concatenated oriented reads; in[i].read_off indexes it
	virtual void seed_search(const std::vector<uint8_t>& reads, const std::vector<bt2x_seed_in>& in,
	                         std::vector<bt2x_seed_out>& out) = 0;
	virtual void resolve(const std::vector<bt2x_resolve_in>& in, std::vector<bt2x_resolve_out>& out) = 0;
	virtual void dp_align(const std::vector<uint8_t>& reads, const std::vector<uint8_t>& quals,
	                      const std::vector<uint8_t>& refs, const std::vector<bt2x_dp_in>& in,
	                      std::vector<bt2x_dp_out>& out, std::vector<bt2x_aln_rec>& recs,
	                      std::vector<uint32_t>& edits) = 0;
};

// -------------------------------------------------------------------- driver

struct RunStats {
	uint64_t reads = 0, aligned = 0, unaligned = 0, rep = 0;
	uint64_t seed_launches = 0, resolve_launches = 0, dp_launches = 0;
	uint64_t seeds = 0, resolves = 0, dps = 0, dps_used = 0, tight_recs = 0;
	double t_seed = 0, t_resolve = 0, t_dp = 0, t_host = 0, t_io = 0;
};

class Aligner {
public:
	Aligner(const Params& p, const RefInfo& ref, Backend& be) : p_(p), ref_(ref), be_(be) {}
	// SAM header (@HD, @SQ; sam.cpp:47-80)
	std::string header() const;
	// Align every read of `fq`, writing SAM records in input order to `out`.
	RunStats run(FastqReader& fq, std::FILE* out, size_t slots, int threads);
	// Align a vector of reads (tests); records in input order.
	std::string align_all(std::vector<Read>& reads, size_t slots, int threads, RunStats* st = nullptr);
private:
	ReadTask align_read(ReadCtx* c);
	bool step(std::vector<ReadCtx*>& active, RunStats& st, int threads);
	const Params& p_;
	const RefInfo& ref_;
	Backend& be_;
};

} // namespace host
} // namespace bt2x
