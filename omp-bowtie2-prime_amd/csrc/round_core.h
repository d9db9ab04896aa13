// round_core.h — one read's seed round after its seed search, as the GPU runs it
// (bt2x_seed_round, include/bt2x.h): searchAllSeedsFinalize + SeedResults::add,
// rankSeedHits and prioritizeSATups, in two parts:
//   prep()    everything up to RowSampler's sampling, and how many elements it will draw;
//   sample()  the sampling loop itself (RowSampler darts + Random1toN draws).
// The kernel (round_kernel.hip) runs prep for every read and sample only for the reads
// that need it, compacted, so the long RNG-sequential sampling loops of repetitive reads
// do not hold whole waves of short reads.  Integer/double code shared with the CPU test
// that checks it against the host driver's restatement (tests/cpp/test_round.cpp).
//
// Reference (file:line):
//   searchAllSeedsFinalize / SeedResults::add   aligner_seed.cpp:508-540, aligner_seed.h:603-641
//   AlignmentCache::addOnTheFly (nlex of the first add per BW range)   aligner_cache.h:558
//   SeedResults::rankSeedHits                    aligner_seed.h:1000-1061
//   SwDriver::prioritizeSATups                   aligner_sw_driver.cpp:61-260
//   RowSampler                                   aligner_sw_driver.h:176-267
//   Random1toN                                   random_util.h:32-230
//   RandomSource (LCG)                           random_source.h:34-140
// Floating point: RowSampler's masses and darts are IEEE double/float with no
// contraction (the TU is built with -ffp-contract=off), as on the reference's x86-64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/bt2x.h"

namespace bt2x_round {

constexpr int kMaxOffs = 64;                  // seed offsets per strand
constexpr int kMaxRanges = 2 * kMaxOffs;      // satpos2 entries
constexpr int kArena = 4096;                  // uint16 list storage (swap lists)
constexpr int kHash = 1024;                   // seen-set slots: (range << 16 | element) + 1
constexpr uint32_t kNsm = 5;                  // prioritizeSATups' nsm

struct Rnd {                                  // RandomSource, LCG variant
	uint32_t last;
	int32_t lastOff;
	__host__ __device__ uint32_t nextU32() {
		last = 1664525u * last + 1013904223u;
		uint32_t r = last >> 16;
		last = 1664525u * last + 1013904223u;
		r ^= last;
		lastOff = 0;
		return r;
	}
	__host__ __device__ bool nextBool() {
		if(lastOff > 31) nextU32();
		const uint32_t r = (last >> lastOff) & 1u;
		lastOff++;
		return r != 0;
	}
	__host__ __device__ float nextFloat() { return (float)nextU32() / (float)0xffffffffu; }
};

struct Range {                                // a satpos2 entry (SATupleAndPos)
	uint64_t topf, size;
	uint32_t rdoff;
	uint16_t offidx;
	uint8_t nlex, fw;
};

struct alignas(4) R1N {                       // Random1toN state; lists live in the arena
	uint16_t n, cur, thresh, list;            // list: arena offset of list_
	uint8_t inited, swaplist, converted, pad;
};

// prep()'s per-lane workspace
struct PrepWs {
	uint64_t htopf[2][kMaxOffs], hn[2][kMaxOffs];  // valid where prep()'s strand mask has the bit
	uint8_t hnlex[2][kMaxOffs];               // the cache's nlex for the offset's range
	uint16_t rankIdx[kMaxRanges];
	uint8_t rankFw[kMaxRanges];
	uint64_t cacheTop[kMaxRanges];
	uint8_t cacheNlex[kMaxRanges];
	Range r2[kMaxRanges];                     // prioritizeSATups' ranges, sorted
	bt2x_exrange exnew[kMaxRanges];
};

// sample()'s workspace (one per job; the kernel keeps it in LDS)
struct SampleWs {
	Range big[kMaxRanges];                    // the job's ranges
	double masses[kMaxRanges], pre[kMaxRanges], mlive[kMaxRanges];   // mlive: masses in live order
	uint16_t live[kMaxRanges];
	R1N r1n[kMaxRanges];
	uint16_t arena[kArena];
	uint32_t hash[kHash];
	uint32_t bkey[128], bmlo[128], bmhi[128]; // a batch's keys and the lanes that drew them (wave kernel)
};

// How sample() spreads its list work over the lanes that run one job together.  All
// lanes run the RNG-sequential loop in lockstep on the same values (wave-uniform); the
// list fills, seen-set clears and the seen-to-swap conversion scan are lane-strided.
// The RowSampler's live list and running sums are behind rs_* so the wave version can keep
// them in registers (lane l holds entries l and l+64) and find the dart with two ballots.
struct SerialCoop {                           // one thread (host test, host builds)
	__host__ __device__ uint32_t lane() const { return 0; }
	__host__ __device__ uint32_t width() const { return 1; }
	__host__ __device__ void sync() const {}
	__host__ __device__ uint64_t ballot(bool p) const { return p ? 1u : 0u; }
	__host__ __device__ bool leader() const { return true; }
	// live = 0 .. nb-1 (w.masses filled)
	__host__ __device__ void rs_init(SampleWs& w, uint32_t nb) { for(uint32_t i = 0; i < nb; i++) w.live[i] = (uint16_t)i; }
	// pre[k] = masses[live[0]] + ... + masses[live[k]], summed in that order; entries
	// below `from` are unchanged since the last rebuild
	__host__ __device__ void rs_rebuild(SampleWs& w, uint32_t nlive, uint32_t from) {
		double sofar = from ? w.pre[from - 1] : 0.0f;
		for(uint32_t k = from; k < nlive; k++) { sofar += w.masses[w.live[k]]; w.pre[k] = sofar; }
	}
	// the first live range whose running mass exceeds rd (else the last live one)
	__host__ __device__ uint32_t rs_dart(const SampleWs& w, double rd, uint32_t nlive) const {
		uint32_t lo = 0, hi = nlive;
		while(lo < hi) { const uint32_t mid = (lo + hi) >> 1; if(rd < w.pre[mid]) hi = mid; else lo = mid + 1; }
		return w.live[lo < nlive ? lo : nlive - 1];
	}
	// drop range bi from the live list (order kept); returns its position
	__host__ __device__ uint32_t rs_remove(SampleWs& w, uint32_t bi, uint32_t nlive) {
		uint32_t q = 0;
		while(q < nlive && w.live[q] != bi) q++;
		const uint32_t pos = q;
		for(; q + 1 < nlive; q++) w.live[q] = w.live[q + 1];
		return pos;
	}
	// per-range Random1toN state and range fields (the wave keeps them in registers)
	__host__ __device__ void r1n_reset(SampleWs& w, uint32_t nb) {
		for(uint32_t i = 0; i < nb; i++) { R1N& r = w.r1n[i]; r.inited = 0; r.n = 0; r.cur = 0; r.converted = 0; r.swaplist = 0; }
	}
	__host__ __device__ R1N r1n_get(const SampleWs& w, uint32_t bi) const { return w.r1n[bi]; }
	__host__ __device__ void r1n_set(SampleWs& w, uint32_t bi, const R1N& r) { w.r1n[bi] = r; }
	__host__ __device__ void big_load(const SampleWs&, uint32_t) {}
	__host__ __device__ Range big_get(const SampleWs& w, uint32_t bi) const { return w.big[bi]; }
	// seen-set membership of key, adding it when absent; full: the set had no room
	__host__ __device__ bool seen_test_add(SampleWs& w, uint32_t key, bool& full) const;
};

struct Prep {
	uint32_t status, nonz, nexnew;
	uint32_t n2;                              // ranges in r2
	uint32_t nsmall;                          // ranges of <= nsm elements (r2[0 .. nsmall))
	uint32_t nsmallSat;                       // of those, taken whole (maxelt may stop early)
	uint64_t smallElts;                       // their elements
	uint64_t nsamples;                        // elements sample() draws from r2[nsmall .. n2)
	uint64_t numElts;
};

// prioritizeSATups' "ranges" order (SATupleAndPos::operator<, aligner_sw_driver.h:140-171)
__host__ __device__ inline bool range_less(const Range& a, const Range& b) {
	if(a.size != b.size) return a.size < b.size;
	if(a.topf != b.topf) return a.topf < b.topf;
	if(a.offidx != b.offidx) return a.offidx < b.offidx;
	if(a.rdoff != b.rdoff) return a.rdoff < b.rdoff;
	return a.fw && !b.fw;                     // seedlen is the same for all seeds of a round
}

__host__ __device__ inline bool exr_covers(const bt2x_exrange& er, int fw, uint32_t rdoff, uint32_t L, uint64_t size) {
	return er.fw == fw && er.off <= rdoff && (uint64_t)er.off + er.len >= (uint64_t)rdoff + L && size <= er.sz;
}

// The first q < n with at(q) true, else n.  The kernel runs one read per lane at about one
// wave per SIMD, so it is bound by the latency of its workspace loads: these scans load four
// entries before testing any (at() must be safe to call up to n rounded up to 4).  The host
// build (host_round's twin, tests/cpp/test_round) scans exactly [0, n), so no entry past n
// is read there and sanitizer / valgrind runs of the CPU build stay clean.
template<class F>
__host__ __device__ inline uint32_t find_first4(uint32_t n, const F& at) {
#if !defined(__HIP_DEVICE_COMPILE__)
	for(uint32_t q = 0; q < n; q++)
		if(at(q)) return q;
	return n;
#endif
	for(uint32_t q = 0; q < n; q += 4) {
		const bool t0 = at(q), t1 = at(q + 1), t2 = at(q + 2), t3 = at(q + 3);
		if(t0) return q;
		if(t1) return q + 1 < n ? q + 1 : n;
		if(t2) return q + 2 < n ? q + 2 : n;
		if(t3) return q + 3 < n ? q + 3 : n;
	}
	return n;
}

// Finalize, rank and prioritize up to the sampling decision.
// hn32: the ranking's copy of the range sizes, entry (s, i) at hn32[(s * kMaxOffs + i) *
// hstride], clamped to 0xffffffff (a size the ranking never picks); the kernel keeps it in
// LDS, one column per lane.
__host__ __device__ inline Prep prep(const bt2x_round_in& in, const bt2x_seed_in* sin, const bt2x_seed_out* sout,
                                     const bt2x_exrange* exr, uint32_t maxelt, Rnd& rnd, PrepWs& w,
                                     uint32_t* hn32, uint32_t hstride) {
	Prep res = {};
	res.status = BT2X_ROUND_OK;
	const uint32_t numOffs = in.num_offs, L = in.seedlen, interval = in.interval, offset = in.offset;
	if(numOffs > (uint32_t)kMaxOffs) { res.status = BT2X_ROUND_REDO; return res; }
	// per strand, one bit per seed offset: a hit was added (and not yet ranked) with a
	// non-empty range.  Registers instead of the reference's per-offset flags, so the
	// ranking below loads only the sizes of the offsets still in the running.
	uint64_t live[2] = {0, 0};
	// ---- searchAllSeedsFinalize: SeedResults::add + the per-read cache's first nlex
	uint32_t ncache = 0;
	bt2x_seed_out dn = in.nseeds ? sout[0] : bt2x_seed_out{};
	bt2x_seed_in sn = in.nseeds ? sin[0] : bt2x_seed_in{};
	for(uint32_t k = 0; k < in.nseeds; k++) {
		const bt2x_seed_out d = dn;                // the next seed's loads go out first
		const bt2x_seed_in si = sn;
		if(k + 1 < in.nseeds) { dn = sout[k + 1]; sn = sin[k + 1]; }
		if(!d.need_reporting) continue;
		const bool fw = si.read_off == in.read_off;
		const uint32_t depth = fw ? si.seed_off : (uint32_t)in.rdlen - si.seed_off - L;
		const uint32_t idx = (depth - offset) / interval;
		if(idx < numOffs) {                    // SeedResults::add ignores other offsets
			const int s = fw ? 0 : 1;
			w.htopf[s][idx] = d.topf; w.hn[s][idx] = d.botf - d.topf;
			const uint64_t n = d.botf - d.topf;
			hn32[((uint32_t)s * kMaxOffs + idx) * hstride] = n < 0xffffffffull ? (uint32_t)n : 0xffffffffu;
			if(d.botf > d.topf) live[s] |= 1ull << idx; else live[s] &= ~(1ull << idx);
			res.numElts += d.botf - d.topf;
			res.nonz++;
		}
		uint8_t cnlex = d.nlex;
		const uint32_t qh = find_first4(ncache, [&](uint32_t q) { return w.cacheTop[q] == d.topf; });
		const bool have = qh < ncache;
		if(have) cnlex = w.cacheNlex[qh];
		else {
			if(ncache >= (uint32_t)kMaxRanges) { res.status = BT2X_ROUND_REDO; return res; }
			w.cacheTop[ncache] = d.topf; w.cacheNlex[ncache] = d.nlex; ncache++;
		}
		// the first add of a range fixes its nlex, so the offset's value is final here
		if(idx < numOffs) w.hnlex[fw ? 0 : 1][idx] = cnlex;
	}
	if(res.nonz == 0) { res.status = BT2X_ROUND_NO_HITS; return res; }
	// ---- rankSeedHits (random strand order and start, smallest range first)
	for(uint32_t r = 0; r < res.nonz; r++) {
		uint32_t minsz = 0xffffffffu;
		uint32_t minidx = 0;
		int minfw = 1;
		const bool rb = rnd.nextBool();
		for(int fwi = 0; fwi <= 1; fwi++) {
			const int fw = (fwi == (rb ? 1 : 0)) ? 1 : 0;
			const int s = fw ? 0 : 1;
			const uint32_t i = rnd.nextU32() % numOffs;
			// the offsets in scan order i, i+1, ..., numOffs-1, 0, ..., i-1 (first minimum wins)
			const uint64_t lo = (1ull << i) - 1;
			for(int part = 0; part < 2; part++) {
				uint64_t m = part ? live[s] & lo : live[s] & ~lo;
				while(m) {                     // four offsets a pass (repeats of b0 pad it)
					const uint32_t b0 = (uint32_t)__builtin_ctzll(m);
					m &= m - 1;
					const uint32_t b1 = m ? (uint32_t)__builtin_ctzll(m) : b0;
					m &= m - 1;
					const uint32_t b2 = m ? (uint32_t)__builtin_ctzll(m) : b0;
					m &= m - 1;
					const uint32_t b3 = m ? (uint32_t)__builtin_ctzll(m) : b0;
					m &= m - 1;
					const uint32_t* h = hn32 + (uint32_t)s * kMaxOffs * hstride;
					const uint32_t n0 = h[b0 * hstride], n1 = h[b1 * hstride], n2 = h[b2 * hstride], n3 = h[b3 * hstride];
					if(n0 < minsz) { minsz = n0; minidx = b0; minfw = fw; }
					if(n1 < minsz) { minsz = n1; minidx = b1; minfw = fw; }
					if(n2 < minsz) { minsz = n2; minidx = b2; minfw = fw; }
					if(n3 < minsz) { minsz = n3; minidx = b3; minfw = fw; }
				}
			}
		}
		if(minsz == 0xffffffffu) { res.status = BT2X_ROUND_REDO; return res; }
		live[minfw ? 0 : 1] &= ~(1ull << minidx);
		w.rankIdx[r] = (uint16_t)minidx;
		w.rankFw[r] = (uint8_t)minfw;
	}
	// ---- prioritizeSATups: ranges by rank, minus those an extended range covers
	uint32_t n2 = 0, nsmall = 0;
	uint64_t nelt = 0;
	for(uint32_t r = 0; r < res.nonz; r++) {
		const uint32_t offidx = w.rankIdx[r];
		const int fw = w.rankFw[r];
		const int s = fw ? 0 : 1;
		Range sp;
		sp.topf = w.htopf[s][offidx];
		sp.size = w.hn[s][offidx];
		sp.rdoff = offidx * interval + offset;
		sp.offidx = (uint16_t)offidx;
		sp.fw = (uint8_t)fw;
		sp.nlex = w.hnlex[s][offidx];
		if(sp.size == 0) continue;
		bool skip = false;
		for(uint32_t q = 0; q < in.nexr && !skip; q++) skip = exr_covers(exr[q], fw, sp.rdoff, L, sp.size);
		for(uint32_t q = 0; q < res.nexnew && !skip; q++) skip = exr_covers(w.exnew[q], fw, sp.rdoff, L, sp.size);
		if(!skip) skip = find_first4(n2, [&](uint32_t q) { return w.r2[q].topf == sp.topf; }) < n2;
		if(skip) continue;
		nelt += sp.size;
		w.r2[n2++] = sp;
		if(sp.size <= kNsm) nsmall++;
		if(sp.nlex > 0) {
			bt2x_exrange& e = w.exnew[res.nexnew++];
			e.off = sp.rdoff - (fw ? sp.nlex : 0);
			e.len = (uint16_t)(L + sp.nlex);
			e.sz = sp.size;
			e.fw = (uint8_t)fw;
			e.pad = 0;
		}
	}
	// stable insertion sort (std::stable_sort by SATupleAndPos order)
	for(uint32_t i = 1; i < n2; i++) {
		const Range x = w.r2[i];
		uint32_t j = i;
		while(j > 0 && range_less(x, w.r2[j - 1])) { w.r2[j] = w.r2[j - 1]; j--; }
		w.r2[j] = x;
	}
	// small ranges whole, then (if needed) one draw per element up to maxelt
	uint64_t added = 0;
	uint32_t nsat = 0;
	for(uint32_t j = 0; j < nsmall && added < maxelt; j++) { nsat++; added += w.r2[j].size; }
	res.n2 = n2; res.nsmall = nsmall; res.nsmallSat = nsat; res.smallElts = added;
	res.nsamples = 0;
	if(!(added >= maxelt || nsmall == n2)) {
		const uint64_t top = (uint64_t)maxelt < nelt ? (uint64_t)maxelt : nelt;
		res.nsamples = top > added ? top - added : 0;
	}
	return res;
}

// host callers (tests/cpp/test_round.cpp): the ranking copy on the stack
inline Prep prep(const bt2x_round_in& in, const bt2x_seed_in* sin, const bt2x_seed_out* sout,
                 const bt2x_exrange* exr, uint32_t maxelt, Rnd& rnd, PrepWs& w) {
	uint32_t hn32[2 * kMaxOffs];
	return prep(in, sin, sout, exr, maxelt, rnd, w, hn32, 1);
}

__host__ __device__ inline bool seen_has(const SampleWs& w, uint32_t key) {       // key != 0
	uint32_t h = (key * 2654435761u) >> 22;                                      // 10 bits
	for(int probe = 0; probe < kHash; probe++, h = (h + 1) & (kHash - 1)) {
		const uint32_t v = w.hash[h];
		if(v == key) return true;
		if(v == 0) return false;
	}
	return false;
}

// false when the set is full
__host__ __device__ inline bool seen_add(SampleWs& w, uint32_t key) {
	uint32_t h = (key * 2654435761u) >> 22;
	for(int probe = 0; probe < kHash; probe++, h = (h + 1) & (kHash - 1))
		if(w.hash[h] == 0 || w.hash[h] == key) { w.hash[h] = key; return true; }
	return false;
}

__host__ __device__ inline bool SerialCoop::seen_test_add(SampleWs& w, uint32_t key, bool& full) const {
	if(seen_has(w, key)) return true;
	if(!seen_add(w, key)) full = true;
	return false;
}

__host__ __device__ inline uint32_t popc64(uint64_t m) {
#ifdef __HIP_DEVICE_COMPILE__
	return (uint32_t)__popcll(m);
#else
	return (uint32_t)__builtin_popcountll(m);
#endif
}

// Random1toN::next over range ri; false on workspace overflow.
template<class C>
__host__ __device__ inline bool r1n_next(SampleWs& w, R1N& s, int ri, Rnd& rnd, uint32_t& arenaTop, uint16_t& out,
                                         const C& co) {
	if(s.cur == 0 && !s.converted) {
		if(s.n == 1) { s.cur = 1; out = 0; return true; }
		if(s.swaplist) {
			if(arenaTop + s.n > (uint32_t)kArena) return false;
			const uint32_t list = arenaTop;
			for(uint32_t i = co.lane(); i < s.n; i += co.width()) w.arena[list + i] = (uint16_t)i;
			co.sync();
			s.list = (uint16_t)list;
			arenaTop += s.n;
		}
	}
	if(s.swaplist) {
		const uint32_t r = s.cur + rnd.nextU32() % (uint32_t)(s.n - s.cur);
		const uint16_t a = w.arena[s.list + s.cur], b = w.arena[s.list + r];
		w.arena[s.list + r] = a;                  // r == cur leaves it as it was
		w.arena[s.list + s.cur] = b;
		out = b;
		s.cur++;
		return true;
	}
	// seen-list mode: redraw until unseen (the unseen draw joins the set)
	uint16_t rn;
	bool full = false;
	do {
		rn = (uint16_t)(rnd.nextU32() % (uint32_t)s.n);
	} while(co.seen_test_add(w, ((uint32_t)ri << 16 | rn) + 1u, full));
	if(full) return false;
	s.cur++;                                  // = seen_.size()
	if(s.cur >= s.thresh && s.cur < s.n) {
		// convert to a swap list of the unseen elements, ascending
		const uint32_t nl = (uint32_t)s.n - s.cur;
		if(arenaTop + nl > (uint32_t)kArena) return false;
		const uint32_t base = arenaTop;
		uint32_t k = 0;
		for(uint32_t j0 = 0; j0 < s.n; j0 += co.width()) {
			const uint32_t j = j0 + co.lane();
			const bool un = j < s.n && !seen_has(w, ((uint32_t)ri << 16 | j) + 1u);
			const uint64_t m = co.ballot(un);
			if(un) w.arena[base + k + popc64(m & ((1ull << co.lane()) - 1ull))] = (uint16_t)j;
			k += popc64(m);
		}
		co.sync();
		arenaTop += nl;
		s.list = (uint16_t)base;
		s.cur = 0;
		s.n = (uint16_t)nl;
		s.converted = 1;
		s.swaplist = 1;
	}
	out = rn;
	return true;
}

// sample()'s loop state between draws
struct SampleState {
	double mass;                              // RowSampler's total live mass
	uint32_t nlive;                           // live ranges
	uint32_t arenaTop;                        // swap-list storage used
};

// RowSampler::init over w.big[0 .. nb) (lensq = szsq = true) and a fresh Random1toN per
// range; false if there are more ranges than the workspace holds.
template<class C>
__host__ __device__ inline bool sample_setup(uint32_t nb, SampleWs& w, C& co, SampleState& st) {
	if(nb > (uint32_t)kMaxRanges) return false;
	for(uint32_t k = co.lane(); k < (uint32_t)kHash; k += co.width()) w.hash[k] = 0;
	for(uint32_t i = co.lane(); i < nb; i += co.width()) {
		double num = (double)(w.big[i].nlex + 1);
		num *= num;
		double den = (double)w.big[i].size;
		den *= den;
		w.masses[i] = num / den;
	}
	co.sync();
	co.r1n_reset(w, nb);
	co.big_load(w, nb);
	double mass = 0.0f;
	for(uint32_t i = 0; i < nb; i++) mass += w.masses[i];
	st.mass = mass;
	st.nlive = nb;
	st.arenaTop = 0;
	co.rs_init(w, nb);
	co.rs_rebuild(w, st.nlive, 0);
	return true;
}

// Draw k: one RowSampler dart and one Random1toN::next; emit(k, range, element) on the
// leader lane.  False on workspace overflow.
template<class C, class Emit>
__host__ __device__ inline bool sample_step(uint64_t k, Rnd& rnd, SampleWs& w, C& co, SampleState& st, Emit&& emit) {
	const double rd = rnd.nextFloat() * st.mass;
	// the dart: first live range whose running mass exceeds it (else the last live one)
	if(st.nlive == 0) return false;
	const uint32_t bi = co.rs_dart(w, rd, st.nlive);
	R1N s = co.r1n_get(w, bi);
	const Range rg = co.big_get(w, bi);
	if(!s.inited) {
		const uint16_t n = (uint16_t)rg.size;                              // uint16_t element type
		if(n == 0) return false;
		s.inited = 1; s.n = n; s.cur = 0; s.converted = 0; s.swaplist = n < 128 ? 1 : 0;
		const uint16_t t = (uint16_t)(0.10f * (float)n);
		s.thresh = t > 16 ? t : 16;
	}
	uint16_t rr;
	if(!r1n_next(w, s, (int)bi, rnd, st.arenaTop, rr, co)) return false;
	co.r1n_set(w, bi, s);
	if(s.n > 0 && s.cur >= s.n) {                                          // done(): finishedRange
		st.mass -= w.masses[bi];
		const uint32_t q = co.rs_remove(w, bi, st.nlive);
		st.nlive--;
		co.rs_rebuild(w, st.nlive, q);
	}
	if(co.leader()) emit(k, rg, rr);
	return true;
}

// RowSampler over w.big[0 .. nb) and one Random1toN per range: emit(k, range, element)
// for each of the nsamples draws (on the leader lane).  The caller fills w.big; false on
// workspace overflow.
template<class C, class Emit>
__host__ __device__ inline bool sample(uint32_t nb, uint64_t nsamples, Rnd& rnd, SampleWs& w, C& co,
                                       Emit&& emit) {
	SampleState st;
	if(!sample_setup(nb, w, co, st)) return false;
	for(uint64_t k = 0; k < nsamples; k++)
		if(!sample_step(k, rnd, w, co, st, emit)) return false;
	return true;
}

} // namespace bt2x_round
