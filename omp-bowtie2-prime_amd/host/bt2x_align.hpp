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
// Host throughput: a read's state lives in a pooled ReadCtx whose buffers keep their
// capacity from one read to the next (the coroutine frame too, ReadCtx::frame_), so the
// steady state allocates almost nothing per read; DP results sit in per-read arenas.
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
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <utility>
#include <functional>
#include <vector>

#include "bt2x.h"
#include "bt2x_shims.hpp"
#include "work_pool.hpp"

namespace bt2x { namespace host {

// Host buffers that cross PCIe (the launch buffers handed to a Backend) come from a
// hook, so the GPU backend can supply page-locked memory that the DMA engines read and
// write directly (pageable copies stage through the driver at a fraction of the link's
// rate).  Resizing such a buffer default-initialises, so a launch does not zero what
// the gather or the GPU overwrites anyway.
void set_host_allocator(void* (*alloc)(size_t), void (*release)(void*));
void* host_alloc(size_t bytes);               // remembers which hook allocated it
void host_free(void* p) noexcept;

template<class T> struct HostAlloc {
	using value_type = T;
	HostAlloc() = default;
	template<class U> HostAlloc(const HostAlloc<U>&) noexcept {}
	T* allocate(size_t n) { return static_cast<T*>(host_alloc(n * sizeof(T))); }
	void deallocate(T* p, size_t) noexcept { host_free(p); }
	template<class U> void construct(U* p) noexcept { ::new((void*)p) U; }
	template<class U, class... A> void construct(U* p, A&&... a) { ::new((void*)p) U(std::forward<A>(a)...); }
	template<class U> bool operator==(const HostAlloc<U>&) const noexcept { return true; }
	template<class U> bool operator!=(const HostAlloc<U>&) const noexcept { return false; }
};
template<class T> using HostVec = std::vector<T, HostAlloc<T>>;

}} // namespace bt2x::host

namespace bt2x {
namespace host {

// glibc malloc for the driver's allocation pattern (set once at start-up, before any
// thread exists): never trim the heap back to the kernel and keep vectors of up to
// 32 MiB off mmap.  With the defaults, buffers that keep growing and shrinking across
// launches go back and forth to the kernel, and on a many-core host the page faults and
// unmaps serialise on the address-space lock: measured on the MI355X box (16 threads,
// 1 M reads), kernel time in the alignment window drops from 16.9 s to 1.3 s and the
// host resumes from 2.06 s to 1.05 s.
void tune_malloc();

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
		if(!swaplist_) seenBits_.assign(((size_t)n + 63) / 64, 0);
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
		// seen-list mode: redraw until unseen (membership by bitset; the reference scans
		// the list, same answers)
		uint16_t rn = 0;
		const uint16_t seenSz = (uint16_t)seen_.size();
		do {
			rn = (uint16_t)(rnd.nextU32() % (uint32_t)n_);
		} while((seenBits_[rn >> 6] >> (rn & 63)) & 1);
		seenBits_[rn >> 6] |= 1ULL << (rn & 63);
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
	std::vector<uint64_t> seenBits_;
};

// Random1toN over the ranges extendSeeds walks.  prioritizeSATups keeps whole only the
// ranges of at most nsm = 5 elements and samples larger ones element by element
// (aligner_sw_driver.cpp:176-257), so every range the walk draws from has <= 5 elements:
// swap-list mode (n < 128) with inline storage, trivially copyable (the DP lookahead
// copies the walk).
struct SmallRandom1toN {
	static constexpr uint32_t kMax = 8;
	uint8_t n = 0, cur = 0;
	uint8_t list[kMax] = {};
	void init(uint32_t nn) {
		if(nn > kMax) throw std::logic_error("SmallRandom1toN: range larger than prioritizeSATups keeps whole");
		n = (uint8_t)nn; cur = 0;
	}
	uint16_t next(Rng& rnd) {
		if(cur == 0) {
			if(n == 1) { cur = 1; return 0; }
			for(uint8_t i = 0; i < n; i++) list[i] = i;
		}
		const uint32_t r = cur + rnd.nextU32() % (uint32_t)(n - cur);
		if(r != cur) std::swap(list[cur], list[r]);
		return list[cur++];
	}
	bool done() const { return n > 0 && cur >= n; }
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
	bool contains(const Coord& c) const {
		return c.ref == up.ref && c.orient == up.orient && c.off >= up.off && c.off < up.off + len;
	}
};

// SwDriver::seenDiags1_ (EIvalMergeListBinned over EIvalMergeList, ival_list.h).  The
// driver only ever asks locusPresent(), i.e. membership in the union of the intervals
// added so far: the reference's sort + merge of every 16 unsorted adds (and its 128 bins
// by reference id) keep exactly that union.  One flat list does the same: an unsorted
// tail of up to 16 intervals, then a sorted run of disjoint merged intervals searched by
// bisection.  Two vectors of PODs, so the DP lookahead's copy reuses capacity.
class SeenDiags {
public:
	// clear; with `base`, this set is an overlay: it answers for base's intervals plus its
	// own (the DP lookahead's walk adds to an overlay over the read's real set)
	void clear(const SeenDiags* base = nullptr) { sorted_.clear(); tail_.clear(); base_ = base; }
	void add(const Interval& i) {
		tail_.push_back(i);
		if(tail_.size() == 16) flush();
	}
	void prefetch() const { __builtin_prefetch(sorted_.data()); __builtin_prefetch(tail_.data(), 1); }
	bool locusPresent(const Coord& c) const {
		if(base_ && base_->locusPresent(c)) return true;
		for(const Interval& iv : tail_) if(iv.contains(c)) return true;
		if(sorted_.empty()) return false;
		// last interval whose start is <= c
		size_t lo = 0, hi = sorted_.size();
		while(lo < hi) {
			const size_t mid = (lo + hi) >> 1;
			if(c < sorted_[mid].up) hi = mid; else lo = mid + 1;
		}
		return lo > 0 && sorted_[lo - 1].contains(c);
	}
private:
	// sort the tail, merge it into the sorted run and coalesce overlapping or touching
	// intervals (same union)
	void flush() {
		auto byUp = [](const Interval& a, const Interval& b) { return a.up < b.up; };
		std::sort(tail_.begin(), tail_.end(), byUp);
		merged_.resize(sorted_.size() + tail_.size());
		std::merge(sorted_.begin(), sorted_.end(), tail_.begin(), tail_.end(), merged_.begin(), byUp);
		tail_.clear();
		size_t w = 0;
		for(size_t i = 0; i < merged_.size(); i++) {
			const Interval& iv = merged_[i];
			if(w > 0) {
				Interval& p = merged_[w - 1];
				if(p.up.ref == iv.up.ref && p.up.orient == iv.up.orient && iv.up.off <= p.up.off + p.len) {
					p.len = std::max(p.up.off + p.len, iv.up.off + iv.len) - p.up.off;
					continue;
				}
			}
			merged_[w++] = iv;
		}
		merged_.resize(w);
		sorted_.swap(merged_);
	}
	std::vector<Interval> sorted_, tail_, merged_;
	const SeenDiags* base_ = nullptr;
};

// ----------------------------------------------------------------------- alignments

enum { ET_READ_GAP = 1, ET_REF_GAP = 2, ET_MM = 3 };
inline uint32_t e_pos(uint32_t e) { return BT2X_EDIT_POS(e); }
inline uint32_t e_type(uint32_t e) { return BT2X_EDIT_TYPE(e); }
inline char e_chr(uint32_t e) { return BT2X_EDIT_CHR(e); }
inline uint32_t e_setpos(uint32_t e, uint32_t p) { return (e & ~0x3ffu) | (p & 0x3ffu); }

// Edit::invertPoss(edits, sz, sort=false) (edit.cpp:50-80): reverse, then mirror pos.
inline void invert_poss(const uint32_t* ed, size_t n, size_t sz, std::vector<uint32_t>& out) {
	out.assign(ed, ed + n);
	std::reverse(out.begin(), out.end());
	for(uint32_t& e : out) {
		const uint32_t p = e_pos(e);
		e = e_setpos(e, (uint32_t)(sz - p - (e_type(e) == ET_READ_GAP ? 0 : 1)));
	}
}

// A reported alignment as the sink keeps it: AlnScore orders by score only
// (aligner_result.h:57-255); its edits are printed from the read's shared edit buffer
// (SURVEY F11), so only their count is kept.
struct AlnRes {
	int64_t score = 0;
	int64_t refid = 0, refoff = 0;
	bool fw = true;
	uint32_t nedit = 0;
	uint32_t refns = 0;
};

// RedundantAlns (aligner_result.cpp:821-914): DP cells (ref, strand, row, ref offset)
// already used by a reported alignment.  A reported alignment's cells in row i are the
// contiguous reference run [left_i, right_i), so it is kept as one run per row; a new
// alignment overlaps iff on some row its run intersects the run of an earlier one on
// the same reference and strand.
class RedundantAlns {
public:
	void init(size_t rdlen) { rdlen_ = rdlen; alns_.clear(); runs_.clear(); eds_.clear(); }
	// ned: the alignment's own edits in ned() order (5'-relative for rc)
	bool overlap(const AlnRes& r, const uint32_t* ned, size_t n) {
		if(alns_.empty()) return false;
		// the runs of each row lie inside the alignment's reference span [lo, hi): spans that
		// do not meet rule a pair out without the per-row scan (a repetitive read reports
		// many alignments at distinct loci; the scan over all of them was quadratic)
		int64_t lo, hi;
		span(r, ned, n, lo, hi);
		bool have_rows = false;
		for(Aln& a : alns_) {
			if(a.refid != r.refid || a.fw != r.fw || a.hi <= lo || hi <= a.lo) continue;
			if(!have_rows) { rows(r, ned, n, tmp_); have_rows = true; }
			if(a.run0 < 0) {                               // its rows, kept from now on
				AlnRes ar;
				ar.refid = a.refid; ar.fw = a.fw; ar.refoff = a.refoff;
				rows(ar, eds_.data() + a.e0, a.ne, tmp2_);
				a.run0 = (int64_t)runs_.size();
				runs_.insert(runs_.end(), tmp2_.begin(), tmp2_.end());
			}
			const int64_t* o = runs_.data() + a.run0;
			for(size_t i = 0; i < rdlen_; i++) {
				const int64_t l = std::max(o[2 * i], tmp_[2 * i]), rr = std::min(o[2 * i + 1], tmp_[2 * i + 1]);
				if(l < rr) return true;
			}
		}
		return false;
	}
	// Most reads report one alignment, which no other is ever compared with: an added
	// alignment keeps its span and edits, and its per-row runs are built the first time a
	// later alignment's span meets it.
	void add(const AlnRes& r, const uint32_t* ned, size_t n) {
		int64_t lo, hi;
		span(r, ned, n, lo, hi);
		alns_.push_back({r.refid, r.fw, r.refoff, (uint32_t)eds_.size(), (uint32_t)n, -1, lo, hi});
		eds_.insert(eds_.end(), ned, ned + n);
	}
private:
	struct Aln { int64_t refid; bool fw; int64_t refoff; uint32_t e0, ne; int64_t run0; int64_t lo, hi; };
	// rows' runs move right monotonically (left_{i+1} >= left_i): the first row's left and
	// the last row's right bound every run.  From rows() below: left_0 = refoff,
	// left_{i+1} = left_i + 1 + [read gaps at pos i+1] - [ref gap at pos i], and the last
	// row's right = its left + 1, so the span is [refoff, refoff + rdlen + read gaps at
	// pos 1..rdlen-1 - ref gaps at pos 0..rdlen-2) of the (inverted, for rc) edits: O(edits)
	// instead of the O(rdlen) row pass (it runs for every reported alignment).
	void span(const AlnRes& r, const uint32_t* ned, size_t n, int64_t& lo, int64_t& hi) const {
		lo = rdlen_ ? r.refoff : 0;
		if(!rdlen_) { hi = 0; return; }
		int64_t d = 0;
		const int64_t L = (int64_t)rdlen_;
		for(size_t k = 0; k < n; k++) {
			const uint32_t t = e_type(ned[k]);
			int64_t p = (int64_t)e_pos(ned[k]);
			if(!r.fw) p = L - p - (t == ET_READ_GAP ? 0 : 1);         // invert_poss
			if(t == ET_READ_GAP && p >= 1 && p <= L - 1) d++;
			else if(t == ET_REF_GAP && p >= 0 && p <= L - 2) d--;
		}
		hi = r.refoff + L + d;
	}
	void rows(const AlnRes& r, const uint32_t* ned0, size_t n, std::vector<int64_t>& out) {
		const uint32_t* ned = ned0;
		if(!r.fw) { invert_poss(ned0, n, rdlen_, inv_); ned = inv_.data(); }
		out.resize(2 * rdlen_);
		int64_t left = r.refoff, right;
		size_t ni = 0;
		for(size_t i = 0; i < rdlen_; i++) {
			size_t diff = 1;
			right = left + 1;
			while(ni < n && e_pos(ned[ni]) == i) {
				if(e_type(ned[ni]) == ET_REF_GAP) diff = 0;
				ni++;
			}
			if(i < rdlen_ - 1) {
				size_t nn = ni;
				while(nn < n && e_pos(ned[nn]) == i + 1) {
					if(e_type(ned[nn]) == ET_READ_GAP) right++;
					nn++;
				}
			}
			out[2 * i] = left; out[2 * i + 1] = right;
			left = right + (int64_t)diff - 1;
		}
	}
	size_t rdlen_ = 0;
	std::vector<Aln> alns_;
	std::vector<int64_t> runs_, tmp_, tmp2_;
	std::vector<uint32_t> eds_, inv_;
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
	bool quiet = false;             // --quiet: no per-read warnings (gQuiet)
	// DP kernel choice (aligner_sw.cpp:77-83, bt2_search.cpp:1350-1356, 2484-2492): the stock
	// build runs u8 only, minsc clamped to -254; a -DENABLE_I16 build (i16build) keeps minsc
	// and runs the i16 kernel unless enable8 && minsc >= -254.  --no-sse8 implies i16build
	// (the stock build ignores it with a warning).
	bool enable8 = true, i16build = false;
	size_t lookahead = 8;           // DP problems posed per request (not a reference option;
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
	// SwAligner::initRef's enable8_ (aligner_sw.cpp:77-83)
	bool dpI16(int64_t minsc) const { return dp_uses_i16(i16build, enable8, minsc); }
};

// SeedAlignmentPolicy's PARSE_FUNC (aligner_seed_policy.cpp:47-75) over an existing
// function: type, constant, coefficient, minimum -- and a fifth token sets the minimum
// too, as there.  false on a bad type letter.
inline bool parse_func_tokens(SimpleFunc& f, const std::string& s) {
	std::vector<std::string> t;
	size_t b = 0;
	for(;;) {
		const size_t e = s.find(',', b);
		t.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
		if(e == std::string::npos) break;
		b = e + 1;
	}
	if(t.size() >= 1) {
		const std::string& y = t[0];
		if(y == "C" || y == "Constant") f.type = 1;
		else if(y == "L" || y == "Linear") f.type = 2;
		else if(y == "S" || y == "Sqrt") f.type = 3;
		else if(y == "G" || y == "Log") f.type = 4;
		else return false;
	}
	if(t.size() >= 2) f.C = std::strtod(t[1].c_str(), nullptr);
	if(t.size() >= 3) f.L = std::strtod(t[2].c_str(), nullptr);
	if(t.size() >= 4) f.I = std::strtod(t[3].c_str(), nullptr);
	if(t.size() >= 5) f.I = std::strtod(t[4].c_str(), nullptr);
	return true;
}

// The bowtie2-align-l options that change the hot path's results (bt2_search.cpp:446-643;
// presets expand to -D/-R/-L/-i, SeedAlignmentPolicy).  Returns the number of argv
// entries consumed at argv[i] (0: not one of these).  bt2x_scoring_init() must follow.
inline int parse_align_option(Params& p, int argc, char** argv, int i) {
	const std::string a = argv[i];
	const bool has = i + 1 < argc;
	auto pair = [&](int& x, int& y) { std::sscanf(argv[i + 1], "%d,%d", &x, &y); };
	if(a == "--sse8") { p.enable8 = true; return 1; }
	if(a == "--no-sse8") { p.enable8 = false; p.i16build = true; return 1; }
	if(a == "--i16-build") { p.i16build = true; return 1; }    // (not a reference option)
	if(a == "--quiet") { p.quiet = true; return 1; }
	if(!has) return 0;
	// --score-min / --n-ceil / -i: the policy strings of bt2_search.cpp:1436-1541, parsed
	// by PARSE_FUNC; a malformed function is reported as an unconsumed option
	if(a == "--score-min" || a == "--min-score") return parse_func_tokens(p.scoreMin, argv[i + 1]) ? 2 : 0;
	if(a == "-i") return parse_func_tokens(p.msIval, argv[i + 1]) ? 2 : 0;
	if(a == "--n-ceil") {
		const std::string v = argv[i + 1];
		const size_t ncomma = (size_t)std::count(v.begin(), v.end(), ',');
		return parse_func_tokens(p.nCeil, ncomma == 2 ? v : "L," + v) ? 2 : 0;
	}
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
	uint32_t nN = 1;                // Ns in the read (decode counts them; 1 = not counted: scan)
	size_t length() const { return fw.size(); }
};

// genRandSeed (pat.cpp:45-88).  The xors are order-free, so the code and quality terms are
// folded 16 / 4 positions at a time (the shifts repeat with that period).
inline uint32_t gen_rand_seed(const Read& r, uint32_t seed) {
	uint32_t rseed = (seed + 101) * 59 * 61 * 67 * 71 * 73 * 79 * 83;
	const size_t n = r.fw.size();
	const uint8_t* fw = r.fw.data();
	const signed char* qu = reinterpret_cast<const signed char*>(r.qual.data());
	size_t i = 0;
	for(; i + 16 <= n; i += 16) {
		uint32_t x = 0;
		for(int k = 0; k < 16; k++) x ^= (uint32_t)fw[i + k] << (2 * k);
		rseed ^= x;
	}
	for(; i < n; i++) rseed ^= ((uint32_t)fw[i] << ((i & 15) << 1));
	for(i = 0; i + 4 <= n; i += 4) {
		uint32_t x = 0;
		for(int k = 0; k < 4; k++) x ^= (uint32_t)((int)qu[i + k] << (8 * k));
		rseed ^= x;
	}
	for(; i < n; i++) rseed ^= (uint32_t)((int)qu[i] << ((i & 3) << 3));
	for(size_t i = 0; i < r.name.size(); i++) {
		const int p = (int)(signed char)r.name[i];
		if(p == '/') break;
		rseed ^= (uint32_t)(p << ((i & 3) << 3));
	}
	return rseed;
}

// FASTQ input (FastqPatternSource light parse + parse, pat.cpp:1124-1220), Phred+33
// only; '.' is N, non-alphabetic sequence characters are skipped.  The files are mapped
// and form one read stream, as bowtie2's comma-separated -U list does; take() finds
// record boundaries (four lines each) serially with memchr, decode() builds the Read
// (codes, reverse complement, genRandSeed) and runs in parallel over records.
//
// Shards (multi-GPU, one process per GPU): shard i of n reads the records that start in
// bytes [i*T/n, (i+1)*T/n) of the concatenated files (T = their total size), each bound
// moved to the next record start (a line beginning '@' whose third line begins '+'), so
// the shards partition the stream in order.  Records are numbered globally
// (first_rdid(): rdid_base plus the records before the shard, counted as take() finds
// them): a read without a name is named by that number, as the reference does.
// rdid_base numbers a stream that continues an earlier one (bt2x-align --warmup-files:
// the timed files follow the warmup files in the -U list).
class FastqReader {
public:
	struct Raw { const char* l[4]; size_t n[4]; };
	explicit FastqReader(const char* path) : FastqReader(std::vector<std::string>{path}) {}
	explicit FastqReader(const std::vector<std::string>& paths, int shard = 0, int nshards = 1, uint64_t rdid_base = 0);
	// records of a whole file, as take() counts them
	static uint64_t count_file_records(const std::string& path);
	~FastqReader();
	FastqReader(const FastqReader&) = delete;
	FastqReader& operator=(const FastqReader&) = delete;
	// up to `max` more records appended to `out`; returns how many
	size_t take(size_t max, std::vector<Raw>& out) {
		size_t k = 0;
		while(k < max) {
			if(cur_ >= f_.size()) break;
			if(pos_ >= pop_end_) populate_ahead();
			Raw r;
			const char* s;
			size_t n;
			bool got = false;
			while(line(s, n)) { if(n) { got = true; break; } }
			if(!got) {                           // this file's part is done: next file
				file_done();
				continue;
			}
			r.l[0] = s; r.n[0] = n;
			const File& F = f_[cur_];
			for(int j = 1; j < 4; j++) { if(!line(s, n)) { s = F.map + F.end; n = 0; } r.l[j] = s; r.n[j] = n; }
			out.push_back(r);
			k++;
			taken_++;
		}
		return k;
	}
	// global number of the shard's first record
	uint64_t first_rdid() const { return first_rdid_; }
	size_t nfiles() const { return f_.size(); }
	// records of this shard up to the end of file f (f < files_done())
	size_t files_done() const { return ends_.size(); }
	uint64_t file_end(size_t f) const { return ends_[f]; }
	// decodes into r, reusing its buffers; name_id numbers an unnamed read
	static void decode(const Raw& raw, Read& r, uint64_t rdid, uint32_t randSeed, uint64_t name_id) {
		if(raw.l[0][0] != '@') throw std::runtime_error("FASTQ record does not start with '@'");
		r.rdid = rdid;
		r.name.assign(raw.l[0] + 1, raw.n[0] - 1);
		// sequence: '.' is N, non-alphabetic characters are skipped (isalpha, "C" locale);
		// written through a pointer into the resized buffer (no per-character push_back)
		const size_t n1 = raw.n[1];
		r.fw.resize(n1);
		uint8_t* fw = r.fw.data();
		size_t L = 0;
		uint32_t nN = 0;
		const unsigned char* sq = reinterpret_cast<const unsigned char*>(raw.l[1]);
		// a line of letters only (the common case): codes by arithmetic on the ASCII value in
		// a branch-free loop the compiler vectorizes (kAsc2Dna's values: A/C/G/T either case
		// 0-3, every other letter 4); anything else ('.', skipped characters) the general loop
		{
			unsigned bad = 0;
			uint32_t nn = 0;
			for(size_t i = 0; i < n1; i++) {
				const unsigned c = sq[i], u = c & 0xdfu;
				bad |= (unsigned)((u - 'A') > 25u);
				const unsigned t = (c >> 1) & 3u;                 // A 0, C 1, T 2, G 3
				const bool acgt = (u == 'A') | (u == 'C') | (u == 'G') | (u == 'T');
				fw[i] = acgt ? (uint8_t)(t ^ (t >> 1)) : (uint8_t)4;
				nn += acgt ? 0u : 1u;
			}
			if(!bad) { L = n1; nN = nn; }
		}
		if(L != n1 || n1 == 0) {
			L = 0; nN = 0;
			for(size_t i = 0; i < n1; i++) {
				const unsigned char c = sq[i] == '.' ? (unsigned char)'N' : sq[i];
				const uint8_t code = kAsc2Dna[c];
				const unsigned alpha = (unsigned)((c | 32u) - 'a') < 26u;
				fw[L] = code;
				nN += (code > 3) & alpha;
				L += alpha;
			}
		}
		r.fw.resize(L);
		r.nN = nN;
		r.qual.clear();
		if(raw.n[1] || raw.n[3]) r.qual.assign(raw.l[3], raw.n[3]);
		if(r.qual.size() != L)
			throw std::runtime_error("read " + r.name + ": qualities and sequence differ in length");
		if(r.name.empty()) r.name = std::to_string(name_id);
		r.rc.resize(L);
		uint8_t* rc = r.rc.data();
		for(size_t i = 0; i < L; i++) {
			const uint8_t c = fw[L - 1 - i];
			rc[i] = c < 4 ? (uint8_t)(3 - c) : (uint8_t)4;
		}
		r.qualRev.resize(L);
		std::reverse_copy(r.qual.begin(), r.qual.end(), r.qualRev.begin());
		r.seed = gen_rand_seed(r, randSeed);
	}
	static void decode(const Raw& raw, Read& r, uint64_t rdid, uint32_t randSeed) { decode(raw, r, rdid, randSeed, rdid); }
private:
	struct File { const char* map = nullptr; size_t len = 0; int fd = -1; size_t beg = 0, end = 0; };
	// Map the next window of the current file's part into the page table in one call
	// (MADV_POPULATE_READ) instead of one minor fault per 4 KiB page as the scan reaches it
	// (~0.7 M faults per 10 M reads); take() runs on the reader's helper thread, so this
	// stays off the scheduler's path.  A kernel without it just faults as before.
	void populate_ahead();
	size_t pop_end_ = 0;
	bool line(const char*& s, size_t& n) {
		const File& F = f_[cur_];
		if(pos_ >= F.end) return false;
		s = F.map + pos_;
		const char* nl = (const char*)std::memchr(s, '\n', F.end - pos_);
		n = nl ? (size_t)(nl - s) : F.end - pos_;
		pos_ += n + (nl ? 1 : 0);
		while(n > 0 && s[n - 1] == '\r') n--;
		return true;
	}
	void file_done() {
		ends_.push_back(taken_);
		if(++cur_ < f_.size()) pos_ = f_[cur_].beg;
		pop_end_ = 0;
	}
	std::vector<File> f_;
	size_t cur_ = 0, pos_ = 0;
	uint64_t first_rdid_ = 0, taken_ = 0;
	std::vector<uint64_t> ends_;
};

// bowtie2's -U list: comma-separated file names
inline std::vector<std::string> split_list(const std::string& s) {
	std::vector<std::string> out;
	size_t b = 0;
	for(;;) {
		const size_t e = s.find(',', b);
		out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
		if(e == std::string::npos) break;
		b = e + 1;
	}
	return out;
}

// A CPU list as the kernel prints it ("0-15,128-143"); false on a malformed list.
bool parse_cpu_list(const std::string& s, std::vector<int>& out);
// The process's CPU affinity as such a list.
std::string affinity_list();
// --cpus: run on exactly these CPUs (sched_setaffinity before any worker thread starts, so
// the threads inherit the mask and first-touch places their memory on those CPUs' node).
// The sharded launcher (bt2x.dist, bench.py) gives each rank of a node a disjoint set
// inside its GPU's NUMA node.  Throws on a malformed list or one the process may not use.
void apply_cpu_list(const std::string& list);

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
	const uint64_t* lens() const { return plen_.data(); }
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
// One memoised DP result: align()'s outcome and its nextAlignment records, which live in
// the read's arenas (ReadCtx::recs; their edit_off index ReadCtx::edits).
struct DpMemo {
	DpKey key;
	bt2x_dp_out out;
	uint32_t rec0 = 0;
};
struct DpWork {                     // one posed problem (its window is fetched at gather)
	DpKey key;
	bt2x_dp_in in;                  // read_off / qual_off / ref_off are set by the scheduler
};

enum ReqKind { REQ_NONE = 0, REQ_SEED = 1, REQ_RESOLVE = 2, REQ_DP = 3, REQ_ROUND = 4 };

struct ReadCtx;

struct ReadTask {
	struct promise_type {
		ReadTask get_return_object() { return ReadTask{std::coroutine_handle<promise_type>::from_promise(*this)}; }
		std::suspend_always initial_suspend() noexcept { return {}; }
		std::suspend_always final_suspend() noexcept { return {}; }
		void return_void() {}
		void unhandled_exception() { throw; }
		// the frame lives in the read's pooled context (Aligner::align_read(ReadCtx*))
		template<class Self> static void* operator new(std::size_t sz, Self&, ReadCtx* c);
		static void operator delete(void* p, std::size_t sz);
	};
	std::coroutine_handle<promise_type> h;
};

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

// SATupleAndPos (aligner_sw_driver.h:118-180)
struct SatPos {
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

// RowSampler (aligner_sw_driver.h:176-267), lensq = szsq = true.  next() is the
// reference's linear dart walk over the non-eliminated ranges; here the running sums it
// accumulates are kept (same order of double additions, so the same values) and the dart
// is placed by bisection; they are rebuilt when a range is eliminated.
struct RowSampler {
	double mass = 0;
	std::vector<double> masses;
	std::vector<uint32_t> live;     // non-eliminated ranges, in order
	std::vector<double> pre;        // pre[k] = masses[live[0]] + ... + masses[live[k]]
	void init(const std::vector<SatPos>& sl, size_t sai, size_t saf) {
		mass = 0.0f;
		masses.assign(saf - sai, 0.0);
		live.resize(saf - sai);
		for(size_t i = sai; i < saf; i++) {
			double num = (double)(sl[i].nlex + 1);
			num *= num;
			double den = (double)sl[i].size;
			den *= den;
			masses[i - sai] = num / den;
			mass += masses[i - sai];
			live[i - sai] = (uint32_t)(i - sai);
		}
		rebuild();
	}
	void finishedRange(size_t i) {
		mass -= masses[i];
		const auto it = std::lower_bound(live.begin(), live.end(), (uint32_t)i);
		if(it != live.end() && *it == (uint32_t)i) live.erase(it);
		rebuild();
	}
	size_t next(Rng& rnd) {
		const double rd = rnd.nextFloat() * mass;
		if(live.empty()) return std::numeric_limits<size_t>::max();
		const size_t k = (size_t)(std::upper_bound(pre.begin(), pre.end(), rd) - pre.begin());   // rd < pre[k]
		return k < pre.size() ? live[k] : live.back();
	}
private:
	void rebuild() {
		pre.resize(live.size());
		double sofar = 0.0f;
		for(size_t k = 0; k < live.size(); k++) { sofar += masses[live[k]]; pre[k] = sofar; }
	}
};

// The host restatement of a seed round after its seed search, with bt2x_seed_round's
// contract (include/bt2x.h): searchAllSeedsFinalize + SeedResults::add
// (aligner_seed.cpp:508-540), rankSeedHits (aligner_seed.h:1000-1061) and
// prioritizeSATups (aligner_sw_driver.cpp:61-260).  Serves the reads the GPU round hands
// back (BT2X_ROUND_REDO) and the CPU test backend; the SAM tests pin it to the reference.
struct RoundScratch {
	SeedHitsHip hits;
	std::vector<std::pair<uint64_t, uint8_t>> cacheNlex;    // AlignmentCache: key -> nlex of the first add
	std::vector<SatPos> satpos2;
	RowSampler rows;
	std::vector<Random1toN> prioRands;
};
// Appends the read's extension list to sats, its BW rows to rows (qlen = seed length) and
// the exRange entries it adds to exr_out; returns status / nonz / numElts in `out` (the
// offsets fields are left to the caller).
void host_round(const bt2x_round_in& in, const bt2x_seed_in* sin, const bt2x_seed_out* sout, const bt2x_exrange* exr,
                uint32_t maxelt, Rng& rnd, RoundScratch& w, bt2x_round_out& out, std::vector<bt2x_sat>& sats,
                std::vector<bt2x_resolve_in>& rows, std::vector<bt2x_exrange>& exr_out);

// The candidate walk of extendSeeds (aligner_sw_driver.cpp:278-631) as a resumable
// iterator: next() runs the loop up to its next DP problem (PROBLEM, the problem's key)
// or to the loop's exit (an EXTEND_* code); failed() applies a DP that found nothing.
// The walk's own state (position, per-range samplers, elements left) is a value and the
// per-read state it advances (RNG, limit metrics, seen diagonals) is bound by pointer,
// so a copy bound to copies of those runs ahead of the real walk on the assumption
// that every DP fails: the lookahead the scheduler batches (DpKey).
class ExtendWalk {
public:
	static constexpr int PROBLEM = 0;
	// res: the round's elements; plen: reference lengths (plen[tidx] = the element's tlen)
	// sat: the extension list (bt2x_seed_round's order; rand_n = the entry's element count)
	template<class SatVec>
	void reset(const Params& P, const SatVec& sat, const std::vector<uint32_t>& firstRow,
	           const std::vector<bt2x_elt>& res, const uint64_t* plen, size_t nelt, size_t rdlen) {
		P_ = &P; firstRow_ = &firstRow; res_ = &res; plen_ = plen; neltLeft_ = nelt; rdlen_ = rdlen;
		rands_.resize(sat.size());
		for(size_t i = 0; i < sat.size(); i++) rands_[i].init(sat[i].rand_n);
		sat_ = sat.data(); nsat_ = sat.size();
		i_ = 0; first_ = true; inPass_ = false;
	}
	void bind(Rng* rnd, Prm* prm, SeenDiags* seen) { rnd_ = rnd; prm_ = prm; seen_ = seen; }
	void prefetch() const { __builtin_prefetch(rands_.data(), 1); }
	int next(int64_t minsc, DpKey& k);
	// the DP of the last next() found no alignment; false: the fail streak ends the walk
	bool failed() {
		prm_->nExDps++; prm_->nExDpFails++; prm_->nDpFail++;
		return prm_->nDpFail < P_->streak;
	}
private:
	static constexpr uint64_t kNsm = 5;                          // prioritizeSATups' nsm
	const Params* P_ = nullptr;
	const bt2x_sat* sat_ = nullptr;
	size_t nsat_ = 0;
	const std::vector<uint32_t>* firstRow_ = nullptr;
	const std::vector<bt2x_elt>* res_ = nullptr;
	const uint64_t* plen_ = nullptr;
	size_t neltLeft_ = 0, rdlen_ = 0;
	std::vector<SmallRandom1toN> rands_;
	size_t i_ = 0;
	bool first_ = true, inPass_ = false;
	int64_t gapMinsc_ = 1;          // minsc of the cached maxgap (1: none)
	size_t maxgap_ = 0;
	Rng* rnd_ = nullptr;
	Prm* prm_ = nullptr;
	SeenDiags* seen_ = nullptr;
};

// AlnSinkWrap for an unpaired read (aln_sink.cpp:583-643, 1395-1445) with its
// ReportingState (aln_sink.cpp:33-210) under -k 1 -M mhits.
struct Sink {
	static constexpr int64_t kMinScore = std::numeric_limits<int64_t>::min();
	enum { EXIT_DID_NOT_EXIT = 1, EXIT_SHORT_CIRCUIT_k, EXIT_SHORT_CIRCUIT_M, EXIT_SHORT_CIRCUIT_TRUMPED,
	       EXIT_NO_ALIGNMENTS, EXIT_WITH_ALIGNMENTS };
	int64_t mhits = 50;
	std::vector<AlnRes> rs;
	int64_t best = kMinScore, best2 = kMinScore;
	uint64_t n = 0;
	bool doneUnpair = false;
	int exitUnpair = EXIT_DID_NOT_EXIT;
	void reset(int64_t m) {
		mhits = m; rs.clear(); best = best2 = kMinScore; n = 0; doneUnpair = false; exitUnpair = EXIT_DID_NOT_EXIT;
	}
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

// One read in flight: its input, its pending request and every per-read buffer of the
// reference's per-slot objects (SwDriver, SeedResults, AlnSinkWrap, RandomSource).
// Contexts are pooled: buffers keep their capacity from read to read.
struct ReadCtx {
	// what the scheduler's passes read of every read in a cohort first, so that the
	// context's first four cache lines (prefetch_ctx) hold it and the read's buffer headers
	int req = REQ_NONE;
	// the backend's read store (Backend::read_store): this context's slot, whether the
	// current read is in it, and whether the launch being gathered puts it there
	uint32_t slot = 0;
	bool in_store = false, put_now = false;
	bool done = false;                   // finished, record not yet handed to the writer
	std::vector<DpWork> dps;             // the problems posed by the current DP request
	std::vector<bt2x_exrange> exRange, exNew;           // extendSeeds' exRange (both strands)
	bt2x_round_in round_in;              // the GPU round's request
	Read rd;
	// request payloads (gathered / scattered by the scheduler)
	std::vector<bt2x_seed_in> seed_in;   // read_off: 0 = patFw, rdlen = patRc
	std::vector<bt2x_seed_out> seed_out;
	std::vector<bt2x_resolve_in> res_in;
	std::vector<bt2x_elt> elts;      // the round's elements (bt2x_seed_round, or converted resolves)
	// DP results of this read (memo by DpKey; records and edit images in arenas)
	std::vector<DpMemo> memo;
	std::vector<bt2x_aln_rec> recs;
	std::vector<uint32_t> edits;
	// seed round: the GPU round's results (or, for a REDO read, the host's)
	bt2x_round_out round_out;
	std::vector<bt2x_sat> sats;
	RoundScratch rs;
	std::vector<uint32_t> firstRow;
	// extendSeeds state
	SeenDiags seenDiags, seen2;
	ExtendWalk walk, ahead;
	RedundantAlns redAnchor;
	Sink sink;
	std::vector<uint32_t> edbuf;         // SwDriver::resGap_.alres.ned_ storage
	std::string sam;                     // the finished record (sam_gpu: its head; the tail comes
	                                     // from bt2x_sam_tails with the cohort's next launch)
	bool sam_gpu = false;
	bt2x_sam_req sam_req;
	ReadTask task;
	// statistics for the run summary
	bool aligned = false, repetitive = false;
	std::string warn;               // the read's stderr warnings (printEEScoreMsg), written at retire
	int met_kind = 0;               // finishRead's counter: 0 nunp_0, 1 nunp_uni1, 2 nunp_uni2, 3 nunp_rep
	uint64_t ndp_used = 0;          // DP results the walk consumed (the rest were lookahead)
	uint64_t ntight = 0;            // nextAlignment records consumed after -M tightened minsc
	                                // within the same DP problem
	// the coroutine frame (ReadTask::promise_type::operator new)
	static constexpr size_t kFrameBytes = 1536;     // align_read's frame is ~1.25 KiB
	alignas(std::max_align_t) unsigned char frame_[kFrameBytes];
};

template<class Self>
inline void* ReadTask::promise_type::operator new(std::size_t sz, Self&, ReadCtx* c) {
	return sz <= ReadCtx::kFrameBytes ? static_cast<void*>(c->frame_) : ::operator new(sz);
}
inline void ReadTask::promise_type::operator delete(void* p, std::size_t sz) {
	if(sz > ReadCtx::kFrameBytes) ::operator delete(p);
}

inline void Awaiter::await_suspend(std::coroutine_handle<>) noexcept { c->req = kind; }

// ------------------------------------------------------------------ backend

class Backend {
public:
	virtual ~Backend() {}
	// reads: concatenated oriented reads; in[i].read_off indexes it
	virtual void seed_search(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& in,
	                         HostVec<bt2x_seed_out>& out) = 0;
	virtual void resolve(const HostVec<bt2x_resolve_in>& in, HostVec<bt2x_resolve_out>& out) = 0;
	virtual void dp_align(const HostVec<uint8_t>& reads, const HostVec<uint8_t>& quals,
	                      const HostVec<uint8_t>& refs, const HostVec<bt2x_dp_in>& in,
	                      HostVec<bt2x_dp_out>& out, HostVec<bt2x_aln_rec>& recs,
	                      HostVec<uint32_t>& edits) = 0;
	// bt2x_seed_round (include/bt2x.h)
	virtual void seed_round(const HostVec<uint8_t>& reads, const HostVec<bt2x_seed_in>& seeds,
	                        const HostVec<bt2x_round_in>& in, const HostVec<bt2x_exrange>& exr,
	                        uint32_t maxelt, HostVec<bt2x_round_out>& out, HostVec<bt2x_sat>& sats,
	                        HostVec<bt2x_elt>& elts, HostVec<bt2x_exrange>& exr_out) = 0;
	// true: DP problems name their reference window (BT2X_DP_REF_TEXT: ref_off = tidx) and
	// the backend cuts it from the index; false: the driver fills refs (RefInfo::stretch)
	virtual bool ref_from_index() const { return false; }
	// true: the backend keeps the reads in flight in a device-resident store
	// (bt2x_store_reads): store_put uploads a launch's new reads (patFw codes then
	// qualities, packed per in[i]) before its requests, and seed_round / dp_align then get
	// empty reads (and quals) and read_off / qual_off index the store's slots
	virtual bool read_store() const { return false; }
	// true: seed_round gets no seeds (bt2x_seed_round with seeds == NULL: the GPU
	// instantiates them, round_in's seed0 / nseeds / seedflags as the driver set them)
	virtual bool device_seeds() const { return false; }
	virtual void store_put(const HostVec<uint8_t>& packed, const HostVec<bt2x_store_in>& in) { (void)packed; (void)in; }
	// true: sam_tails formats aligned records' tails from the read store (bt2x_sam_tails);
	// text holds text_bytes (every request's text_off + its bound), lens gets the lengths
	virtual bool sam_tails_ok() const { return false; }
	virtual void sam_tails(const HostVec<bt2x_sam_req>& req, HostVec<char>& text, uint64_t text_bytes,
	                       HostVec<uint16_t>& lens) { (void)req; (void)text; (void)text_bytes; (void)lens; }
};

// -------------------------------------------------------------------- driver

// ReportingMetrics (aln_sink.h:44-170), the reference's per-run alignment counters, in its
// field order; the unpaired fields are the ones this fork fills (AlnSinkWrap::finishRead,
// aln_sink.cpp:708-713, 990-1013).  Additive: shards sum them (bt2_search.cpp:2867-2869).
struct ReportingMetrics {
	enum { NREAD, NPAIRED, NUNPAIRED, NCONCORD_UNI, NCONCORD_UNI1, NCONCORD_UNI2, NCONCORD_REP, NCONCORD_0,
	       NDISCORD, NUNP_0_UNI, NUNP_0_UNI1, NUNP_0_UNI2, NUNP_0_REP, NUNP_0_0, NUNP_REP_UNI, NUNP_REP_UNI1,
	       NUNP_REP_UNI2, NUNP_REP_REP, NUNP_REP_0, NUNP_UNI, NUNP_UNI1, NUNP_UNI2, NUNP_REP, NUNP_0,
	       SUM_BEST1, SUM_BEST2, SUM_BEST, N };
	uint64_t v[N] = {};
	void merge(const ReportingMetrics& o) { for(int k = 0; k < N; k++) v[k] += o.v[k]; }
};
// AlnSink::printAlSumm for unpaired reads with a repetitive threshold (-M: canRep),
// aln_sink.cpp:349-527.
void print_alignment_summary(const ReportingMetrics& m, std::FILE* f);

struct RunStats {
	uint64_t reads = 0, aligned = 0, unaligned = 0, rep = 0;
	uint64_t seed_launches = 0, resolve_launches = 0, dp_launches = 0;
	uint64_t seeds = 0, resolves = 0, dps = 0, dps_used = 0, tight_recs = 0;
	uint64_t round_launches = 0, rounds = 0, round_redo = 0;
	uint64_t dp_max_launch = 0;     // problems in the largest DP launch
	uint64_t sam_gpu = 0;           // records whose tail bt2x_sam_tails formatted
	double t_sam = 0;
	ReportingMetrics met;
	std::vector<double> t_files;    // when each input file's last record was written
	double t_seed = 0, t_resolve = 0, t_dp = 0, t_round = 0, t_host = 0, t_io = 0, t_alloc = 0, t_step = 0, t_backend = 0,
	       t_wait = 0, t_gather = 0, t_retire = 0;
};

class Aligner {
public:
	Aligner(const Params& p, const RefInfo& ref, Backend& be) : p_(p), ref_(ref), be_(be) {}
	~Aligner();
	// run(): overlap one cohort's GPU launches with the host work of another (default on)
	void set_pipeline(bool on) { pipeline_ = on; }
	// pipelined: the second cohort's launches on their own backend (a second context with
	// its own GPU stream), so the two cohorts' launches also overlap each other on the GPU
	void set_second_backend(Backend* be) { be2_ = be; }
	// seed rounds through bt2x_seed_round (default on; off: seed search, host ranking and
	// prioritization, SA resolution as three requests)
	void set_gpu_round(bool on) { gpu_round_ = on; }
	// --no-hd: no @HD/@SQ/@PG lines (every shard but the first of a split run)
	void set_header(bool on) { header_on_ = on; }
	// Size both launches' buffers for `reads` reads per launch up front: page-locked
	// buffers cost milliseconds per allocation, so growing them launch by launch is slow.
	void reserve_launch_buffers(size_t reads);
	// The byte sizes reserve_launch_buffers asks for, per launch (to pre-allocate them).
	static std::vector<size_t> launch_buffer_bytes(const Params& p, size_t reads);
	Aligner(const Aligner&) = delete;
	Aligner& operator=(const Aligner&) = delete;
	// SAM header (@HD, @SQ; sam.cpp:47-80)
	std::string header() const;
	// Align every read of `fq`, writing SAM records in input order to `out`.
	// t_run (optional): wall time of the run before its buffers are released
	RunStats run(FastqReader& fq, std::FILE* out, size_t slots, int threads, double* t_run = nullptr);
	// Align a vector of reads (tests); records in input order.
	std::string align_all(std::vector<Read>& reads, size_t slots, int threads, RunStats* st = nullptr);
private:
	// one cohort's requests as one seed, one resolve and one DP launch
	struct Launch {
		std::vector<ReadCtx*> ws, wr, wd, wn, run;      // reads waiting on each kind (wn: rounds)
		std::vector<uint64_t> sr, sk, rk, qb, pb, fb;  // per-read offsets into the buffers
		std::vector<uint64_t> nr, nk, ne;               // rounds: read bytes, seeds, exRange entries
		HostVec<uint8_t> seed_reads, dp_reads, dp_quals, dp_refs;
		HostVec<bt2x_seed_in> seed_in;
		HostVec<bt2x_seed_out> seed_out;
		HostVec<bt2x_resolve_in> res_in;
		HostVec<bt2x_resolve_out> res_out;
		HostVec<bt2x_dp_in> dp_in;
		HostVec<bt2x_dp_out> dp_out;
		HostVec<bt2x_aln_rec> recs;
		HostVec<uint32_t> edits;
		HostVec<uint8_t> round_reads;
		HostVec<bt2x_seed_in> round_seeds;
		HostVec<bt2x_round_in> round_in;
		HostVec<bt2x_exrange> round_exr, round_exr_out;
		HostVec<bt2x_round_out> round_out;
		HostVec<bt2x_sat> round_sats;
		HostVec<bt2x_elt> round_elts;
		uint64_t n_round_seeds = 0;                      // the round's seeds (sent or instantiated on the GPU)
		HostVec<uint8_t> store_packed;                   // the launch's new reads for the read store
		HostVec<bt2x_store_in> store_in;
		// record tails formatted on the GPU (before the launch's store puts reuse the slots):
		// the retired reads' ids, record heads, requests, and the returned text
		std::vector<uint64_t> sam_ids;
		std::vector<std::string> sam_recs;
		HostVec<bt2x_sam_req> sam_req;
		HostVec<char> sam_text;
		HostVec<uint16_t> sam_lens;
		uint64_t sam_text_bytes = 0;
		double t_sam = 0;
		double t_seed = 0, t_resolve = 0, t_dp = 0, t_round = 0, t_gather = 0;
		// gather's per-chunk lists, sizes and bases
		struct Chunk {
			std::vector<ReadCtx*> ws, wr, wd, wn;
			uint64_t sbytes = 0, nseed = 0, nres = 0, dbytes = 0, nprob = 0, rbytes = 0, nbytes = 0, nnseed = 0, nexr = 0;
			uint64_t pbytes = 0, nput = 0;               // read-store puts
			uint64_t ws0 = 0, sb0 = 0, sk0 = 0, wr0 = 0, rk0 = 0, wd0 = 0, db0 = 0, pk0 = 0, rb0 = 0;
			uint64_t wn0 = 0, nb0 = 0, nk0 = 0, ne0 = 0, pb0 = 0, np0 = 0;
		};
		std::vector<Chunk> chunks;
	};
	ReadTask align_read(ReadCtx* c);
	bool step(std::vector<ReadCtx*>& active, RunStats& st);
	void gather(Launch& L, const std::vector<ReadCtx*>& cohort);
	void execute(Launch& L);
	void scatter_resume(Launch& L, RunStats& st);
	Launch launch_[2];
	bool pipeline_ = true, gpu_round_ = true, header_on_ = true;
	bool dseeds_ = false;              // be_.device_seeds(), read when a run starts
	ReadCtx* take_ctx();
	// put(id, record) takes a finished read's SAM record; it is called from the pool's
	// threads, for distinct ids
	// With `defer`, reads whose record tail is formatted on the GPU (sam_gpu) go to that
	// launch's tail requests instead of `put`.
	void retire(std::vector<ReadCtx*>& act, RunStats& st, const std::function<void(uint64_t, std::string&)>& put,
	            Launch* defer = nullptr);
	// the tails of launch L's deferred records (L executed): heads + tails to `put`
	void flush_sam(Launch& L, RunStats& st, const std::function<void(uint64_t, std::string&)>& put);
	bool gpu_sam_ = false;                // record tails on the GPU (pipelined run, backend able)
	// pooled read contexts (kept across runs; released by the destructor)
	std::vector<std::unique_ptr<ReadCtx>> ctxs_;
	std::vector<ReadCtx*> free_;
	std::vector<std::vector<ReadCtx*>> retire_keep_, retire_fin_;   // retire()'s per-chunk lists
	std::vector<std::vector<ReadCtx*>> retire_sam_;                  // and the reads it defers
	std::vector<std::string> sam_ring_;   // the SAM writer's ring of record buffers (kept across runs)
	// host threads for the parallel loops over reads
	std::unique_ptr<WorkPool> pool_;
	WorkPool& pool();
	void use_threads(int threads);
	const Params& p_;
	const RefInfo& ref_;
	Backend& be_;
	Backend* be2_ = nullptr;
};

} // namespace host
} // namespace bt2x
