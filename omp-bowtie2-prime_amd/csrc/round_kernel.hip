// round_kernel.hip — the per-read part of a seed round on gfx950 (bt2x_seed_round):
// after the seed kernel,
//   round_prep_kernel    one lane per read: searchAllSeedsFinalize, rankSeedHits and
//                        prioritizeSATups up to the sampling decision (round_core.h
//                        prep()).  It reserves the read's whole extension list and row
//                        range with atomics, writes the ranges it keeps whole, and queues
//                        a sampling job (the larger ranges + RNG state) for reads that
//                        draw elements;
//   round_sample_kernel  one wave per queued job, workspace in LDS: RowSampler +
//                        Random1toN draws (sample()), written into the reserved slots;
// then sa_resolve_kernel_dn places every row.
//
// RNG-sequential, branchy integer work of a few hundred operations per read, latency
// bound.  Splitting the sampling off matters: in one kernel, the ~10 % of reads that draw
// up to maxelt elements held their whole wave for every read the wave processed; queued,
// the sampling lanes of a wave carry similar loads.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"
#include "round_core.h"

namespace {

using namespace bt2x_round;

struct Job {                 // one read's sampling work
	uint32_t read;           // index into in/out
	uint32_t nb;             // larger ranges, ranges[range0 .. +nb)
	uint32_t range0;
	uint32_t sat_base, elt_base;
	uint32_t rnd_last;
	int32_t rnd_lastoff;
	uint32_t nsamples;
	uint32_t seedlen;
	uint32_t pad;
};

// This lane's base in a block of the counter reserved for the whole wave (one atomic per
// wave instead of one per lane: the prep kernel's counters are shared by every wave of the
// launch, so per-lane atomics serialised at them).  Every lane of the wave must call it.
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* ctr, uint32_t v) {
	const uint32_t lane = threadIdx.x & 63u;
	uint32_t x = v;                                            // inclusive scan
	for(int d = 1; d < 64; d <<= 1) {
		const uint32_t y = (uint32_t)__shfl_up((int)x, d);
		if(lane >= (uint32_t)d) x += y;
	}
	const uint32_t tot = (uint32_t)__shfl((int)x, 63);
	uint32_t base = 0;
	if(lane == 0 && tot) base = atomicAdd(ctr, tot);
	base = (uint32_t)__shfl((int)base, 0);
	return base + x - v;
}

__global__ void __launch_bounds__(64)
round_prep_kernel(RoundLaunch a) {
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	PrepWs& w = *reinterpret_cast<PrepWs*>(a.ws + (size_t)lane * sizeof(PrepWs));
	Job* jobs = reinterpret_cast<Job*>(a.jobs);
	Range* ranges = reinterpret_cast<Range*>(a.ranges);
	const uint32_t stride = gridDim.x * blockDim.x;
	// prep()'s ranking reads the range sizes once per offset still in the running and rank:
	// in LDS, one column per lane (conflict-free), not in the lane's HBM workspace
	__shared__ uint32_t hn32[2 * kMaxOffs * 64];
	// the wave walks the reads together (inactive lanes past the end), so the counters can
	// be reserved per wave
	for(uint32_t r0 = blockIdx.x * blockDim.x; r0 < a.n; r0 += stride) {
		const uint32_t r = r0 + threadIdx.x;
		const bool act = r < a.n;
		Prep p{};
		bt2x_round_in in{};
		Rnd rnd{0, 0};
		bt2x_round_out o;
		if(act) {
			in = a.in[r];
			rnd = Rnd{in.rnd_last, in.rnd_lastoff};
			p = prep(in, a.seeds + in.seed0, a.seed_out + in.seed0, a.exr + in.exr0, a.maxelt, rnd, w, hn32 + threadIdx.x, 64);
		}
		o.rnd_last = rnd.last; o.rnd_lastoff = rnd.lastOff;
		o.num_elts = p.numElts; o.nonz = p.nonz; o.status = p.status;
		o.sat0 = o.nsat = o.elt0 = o.nelt = o.exr0 = o.nexr = 0;
		const bool ok0 = act && p.status == BT2X_ROUND_OK;
		const uint32_t L = in.seedlen;
		const uint32_t nsat = p.nsmallSat + (uint32_t)p.nsamples, nelt = (uint32_t)(p.smallElts + p.nsamples);
		const uint32_t nb = ok0 ? p.n2 - p.nsmall : 0;
		const bool wantjob = ok0 && p.nsamples;
		const uint32_t job = wave_alloc(&a.counters[3], wantjob ? 1u : 0u);
		const uint32_t range0 = wave_alloc(&a.counters[4], wantjob ? nb : 0u);
		if(wantjob && (job >= a.job_cap || range0 + nb > a.range_cap)) {
			p.status = BT2X_ROUND_REDO;                            // hand the read back to the host
			if(job < a.job_cap) {                                   // an empty job keeps the queue dense
				Job j = {};
				j.read = r; j.rnd_last = rnd.last; j.rnd_lastoff = rnd.lastOff;
				jobs[job] = j;
			}
		}
		const bool ok1 = ok0 && p.status == BT2X_ROUND_OK;
		const uint32_t sat0 = wave_alloc(&a.counters[0], ok1 ? nsat : 0u);
		const uint32_t elt0 = wave_alloc(&a.counters[1], ok1 ? nelt : 0u);
		const uint32_t exr0 = wave_alloc(&a.counters[2], ok1 ? p.nexnew : 0u);
		if(ok1) {
			o.nsat = nsat; o.nelt = nelt; o.nexr = p.nexnew;
			o.sat0 = sat0; o.elt0 = elt0; o.exr0 = p.nexnew ? exr0 : 0;
			if(o.sat0 + nsat <= a.sat_cap && o.elt0 + nelt <= a.row_cap) {
				uint32_t e = o.elt0;
				for(uint32_t i = 0; i < p.nsmallSat; i++) {
					const Range& rg = w.r2[i];
					bt2x_sat s;
					s.rdoff = (uint16_t)rg.rdoff; s.rand_n = (uint8_t)rg.size; s.fwlen = BT2X_SAT_FWLEN(rg.fw, L);
					a.sats[o.sat0 + i] = s;
					for(uint32_t k = 0; k < (uint32_t)rg.size; k++) {
						bt2x_resolve_in ri;
						ri.row = rg.topf + k; ri.qlen = L; ri.pad = 0;
						a.rows[e++] = ri;
					}
				}
			}
			if(o.exr0 + p.nexnew <= a.exr_cap)
				for(uint32_t i = 0; i < p.nexnew; i++) a.exr_out[o.exr0 + i] = w.exnew[i];
			if(p.nsamples) {
				for(uint32_t i = 0; i < nb; i++) ranges[range0 + i] = w.r2[p.nsmall + i];
				Job j;
				j.read = r; j.nb = nb; j.range0 = range0;
				j.sat_base = o.sat0 + p.nsmallSat; j.elt_base = (uint32_t)(o.elt0 + p.smallElts);
				j.rnd_last = rnd.last; j.rnd_lastoff = rnd.lastOff;
				j.nsamples = (uint32_t)p.nsamples; j.seedlen = L; j.pad = 0;
				jobs[job] = j;
			}
		} else if(ok0) {
			o.status = p.status;
		}
		if(act) a.out[r] = o;
	}
}

__device__ __forceinline__ double readlane_f64(double v, uint32_t k) {
	const uint64_t u = __builtin_bit_cast(uint64_t, v);
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)k);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)k);
	return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The sampling kernel's workgroup is one wave, so its threads need no workgroup barrier:
// a wave's LDS operations execute in issue order.  The wave barrier alone only orders
// instruction scheduling (LLVM marks it as touching no memory), so wavefront-scope
// release/acquire fences around it tell the compiler that LDS written before it is read
// after it (no reordering or forwarding of those accesses across it).  At wavefront scope
// they emit no s_waitcnt on global stores, which __syncthreads() would (the outputs it
// writes every batch would be waited for each time).
__device__ __forceinline__ void wave_sync() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// BT2X_ROUND_CLOCK builds: per-phase clock64 sums in bt2x_last_round_stats out[8..11]
#ifdef BT2X_ROUND_CLOCK
#define ROUND_CLOCK(i) do { const uint64_t t1_ = clock64(); stats[i] += t1_ - t_; t_ = t1_; } while(0)
#else
#define ROUND_CLOCK(i) do {} while(0)
#endif

struct WaveCoop {                            // a one-wave workgroup runs one job
	// RowSampler state in registers: live range ids, their masses and running sums of
	// list positions l and l + 64
	uint32_t lv0, lv1;
	double m0, m1, p0, p1;
	// range fields of ranges l and l + 64 (topf, size, rdoff | fw << 24)
	uint32_t ga[4], gb[4];
	// Random1toN state in LDS, w.r1n[] read and written as three 32-bit words (n | cur << 16,
	// thresh | list << 16, inited | swaplist << 8 | converted << 16) so the speculative
	// draws can merge their counts with atomicMax on word 0
	__device__ static uint32_t* r1w(const SampleWs& w, uint32_t bi) {
		return reinterpret_cast<uint32_t*>(const_cast<R1N*>(&w.r1n[bi]));
	}
	__device__ void r1n_reset(const SampleWs& w, uint32_t nb) {
		for(uint32_t i = threadIdx.x; i < nb; i += 64) { uint32_t* p = r1w(w, i); p[0] = 0; p[1] = 0; p[2] = 0; }
		wave_sync();
	}
	__device__ static R1N unpack(uint32_t w0, uint32_t w1, uint32_t w2) {
		R1N r;
		r.n = (uint16_t)w0; r.cur = (uint16_t)(w0 >> 16); r.thresh = (uint16_t)w1; r.list = (uint16_t)(w1 >> 16);
		r.inited = (uint8_t)w2; r.swaplist = (uint8_t)(w2 >> 8); r.converted = (uint8_t)(w2 >> 16); r.pad = 0;
		return r;
	}
	__device__ R1N r1n_get(const SampleWs& w, uint32_t bi) const {
		const uint32_t* p = r1w(w, bi);
		return unpack(p[0], p[1], p[2]);
	}
	__device__ void r1n_set(const SampleWs& w, uint32_t bi, const R1N& r) {
		if(threadIdx.x == 0) {
			uint32_t* p = r1w(w, bi);
			p[0] = (uint32_t)r.n | ((uint32_t)r.cur << 16);
			p[1] = (uint32_t)r.thresh | ((uint32_t)r.list << 16);
			p[2] = (uint32_t)r.inited | ((uint32_t)r.swaplist << 8) | ((uint32_t)r.converted << 16);
		}
		wave_sync();
	}
	__device__ void big_load(const SampleWs& w, uint32_t nb) {
		const uint32_t l = threadIdx.x;
		for(int h = 0; h < 2; h++) {
			uint32_t* g = h ? gb : ga;
			const uint32_t i = l + 64 * h;
			if(i < nb) {
				const Range& r = w.big[i];
				g[0] = (uint32_t)r.topf; g[1] = (uint32_t)(r.topf >> 32); g[2] = (uint32_t)r.size;
				g[3] = r.rdoff | ((uint32_t)r.fw << 24);
			} else {
				g[0] = g[1] = g[2] = g[3] = 0;
			}
		}
	}
	__device__ Range big_get(const SampleWs&, uint32_t bi) const {
		const uint32_t l = bi & 63;
		const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ga[0] : gb[0]), (int)l);
		const uint32_t g1 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ga[1] : gb[1]), (int)l);
		const uint32_t g2 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ga[2] : gb[2]), (int)l);
		const uint32_t g3 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ga[3] : gb[3]), (int)l);
		Range r;
		r.topf = ((uint64_t)g1 << 32) | g0; r.size = g2; r.rdoff = g3 & 0xffffffu; r.fw = (uint8_t)(g3 >> 24);
		r.offidx = 0; r.nlex = 0;
		return r;
	}
	// 64 probes of the linear-probing set at once: the first slot holding the key or
	// empty is where the serial probe would stop
	__device__ bool seen_test_add(SampleWs& w, uint32_t key, bool& full) const {
		uint32_t h = (key * 2654435761u) >> 22;
		for(int base = 0; base < kHash; base += 64) {
			const uint32_t slot = (h + (uint32_t)base + threadIdx.x) & (kHash - 1);
			const uint32_t v = w.hash[slot];
			const uint64_t mk = __ballot(v == key), me = __ballot(v == 0);
			const uint64_t m = mk | me;
			if(m) {
				const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;
				if((mk >> f) & 1) return true;
				if(threadIdx.x == f) w.hash[slot] = key;
				return false;
			}
		}
		full = true;
		return false;
	}
	__device__ uint32_t lane() const { return threadIdx.x; }
	__device__ uint32_t width() const { return 64; }
	__device__ void sync() const { wave_sync(); }
	__device__ uint64_t ballot(bool p) const { return __ballot(p); }
	__device__ bool leader() const { return threadIdx.x == 0; }
	__device__ void rs_init(SampleWs& w, uint32_t nb) {
		const uint32_t l = threadIdx.x;
		lv0 = l; lv1 = l + 64;
		m0 = l < nb ? w.masses[l] : 0.0; m1 = l + 64 < nb ? w.masses[l + 64] : 0.0;
		w.mlive[l] = m0; w.mlive[l + 64] = m1;
		wave_sync();
	}
	// the running sums in list order from position `from` (lane 0, the order SerialCoop
	// sums in), then every lane takes its two
	__device__ void rs_rebuild(SampleWs& w, uint32_t nlive, uint32_t from) {
		const uint32_t l = threadIdx.x;
		if(l == 0) {
			double sofar = from ? w.pre[from - 1] : 0.0f;
			uint32_t k = from;
			for(; k + 4 <= nlive; k += 4) {
				const double a0 = w.mlive[k], a1 = w.mlive[k + 1], a2 = w.mlive[k + 2], a3 = w.mlive[k + 3];
				sofar += a0; w.pre[k] = sofar;
				sofar += a1; w.pre[k + 1] = sofar;
				sofar += a2; w.pre[k + 2] = sofar;
				sofar += a3; w.pre[k + 3] = sofar;
			}
			for(; k < nlive; k++) { sofar += w.mlive[k]; w.pre[k] = sofar; }
		}
		wave_sync();
		p0 = w.pre[l]; p1 = w.pre[l + 64];
	}
	// the count of running sums <= rd is the bisection's upper bound
	__device__ uint32_t rs_dart(const SampleWs&, double rd, uint32_t nlive) const {
		const uint32_t l = threadIdx.x;
		const uint32_t lo = (uint32_t)__popcll(__ballot(l < nlive && p0 <= rd)) +
		                    (uint32_t)__popcll(__ballot(l + 64 < nlive && p1 <= rd));
		const uint32_t idx = lo < nlive ? lo : nlive - 1;
		return (uint32_t)__builtin_amdgcn_readlane((int)(idx < 64 ? lv0 : lv1), (int)(idx & 63));
	}
	__device__ uint32_t rs_remove(SampleWs& w, uint32_t bi, uint32_t nlive) {
		const uint32_t l = threadIdx.x;
		const uint64_t b0 = __ballot(l < nlive && lv0 == bi), b1 = __ballot(l + 64 < nlive && lv1 == bi);
		const uint32_t q = b0 ? (uint32_t)__ffsll((unsigned long long)b0) - 1 : 64 + (uint32_t)__ffsll((unsigned long long)b1) - 1;
		// positions >= q take their successor's entry
		const uint32_t nl0 = __shfl(lv0, (int)((l + 1) & 63)), nl1 = __shfl(lv1, (int)((l + 1) & 63));
		const double nm0 = __shfl(m0, (int)((l + 1) & 63)), nm1 = __shfl(m1, (int)((l + 1) & 63));
		const uint32_t h0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)lv1);     // lv1 of lane 0
		const double hm = readlane_f64(m1, 0);
		if(l >= q) { lv0 = l == 63 ? h0 : nl0; m0 = l == 63 ? hm : nm0; }
		if(l + 64 >= q) { lv1 = nl1; m1 = nm1; }
		w.mlive[l] = m0; w.mlive[l + 64] = m1;
		wave_sync();
		return q;
	}
};

constexpr uint32_t kLcgA = 1664525u, kLcgC = 1013904223u;      // Rnd::nextU32's LCG

// Draws k .. k+63 at once, one per lane, on the guess that each earlier draw of the batch
// is a plain draw: two nextU32 (lane l starts 4l LCG steps on, jA/jC), a dart into a range
// whose Random1toN is either in seen-list mode (an element neither seen before nor drawn by
// an earlier lane, and no conversion to a swap list) or a swap list already laid out (and
// not finished by this draw, and not touching a position an earlier draw of the batch
// moved).  The lanes before the first draw that breaks the guess are exactly the serial
// draws, so they commit together (seen-set inserts, swap-list exchanges, the ranges'
// counts); that draw runs through the serial step (sample_step), which handles every case,
// and the next batch starts after it.
// stats: batches, draws committed by batches, serial draws, swap-list draws in batches;
// clock64 cycles in setup, batch draws, serial draws, the rest (exchanges, output stores).
template<class Put>
__device__ bool sample_wave(uint32_t nb, uint64_t nsamples, Rnd& rnd, SampleWs& w, WaveCoop& co, uint32_t jA,
                            uint32_t jC, uint64_t stats[8], Put&& put) {
#ifdef BT2X_ROUND_CLOCK
	uint64_t t_ = clock64();
#endif
	SampleState st;
	if(!sample_setup(nb, w, co, st)) return false;
	const uint32_t lane = threadIdx.x;
	// Lay out the swap lists of the small ranges (2 <= n < 128) now instead of at their
	// first draw: the list is the identity either way and its arena offset is never
	// observed, and a laid-out list's first draw can join a batch.  Marked `converted`
	// (r1n_next then takes the list as laid out; n = 1 keeps its draw-free first draw, so
	// it stays lazy).  Only when the arena holds every list the job could ever build: the
	// small ranges' lists plus, for each seen-list range (n >= 128) whose conversion
	// threshold the job's draws can reach, its swap list of the n - thresh unseen elements
	// (r1n_next).  Then neither the serial path nor this one can overflow, and a job that
	// might overflow keeps the serial (lazy) layout exactly.
	{
		uint32_t tot = 0, need = 0;
		for(uint32_t i = 0; i < nb; i++) {
			const uint32_t n = (uint16_t)w.big[i].size;
			if(n >= 2 && n < 128) tot += n;
			else if(n >= 128) {
				const uint16_t t = (uint16_t)(0.10f * (float)n);
				const uint32_t thresh = t > 16 ? t : 16;
				if(thresh <= nsamples) need += n - thresh;
			}
		}
		if(tot && tot + need <= (uint32_t)kArena) {
			uint32_t base = 0;
			for(uint32_t i = 0; i < nb; i++) {
				const uint32_t n = (uint16_t)w.big[i].size;
				if(n < 2 || n >= 128) continue;
				for(uint32_t e = lane; e < n; e += 64) w.arena[base + e] = (uint16_t)e;
				if(lane == 0) {
					uint32_t* pw = WaveCoop::r1w(w, i);
					const uint16_t t = (uint16_t)(0.10f * (float)n);
					pw[0] = n;                                             // cur 0
					pw[1] = (uint32_t)(t > 16 ? t : 16) | (base << 16);
					pw[2] = 1u | (1u << 8) | (1u << 16);                   // inited, swaplist, converted
				}
				base += n;
			}
			st.arenaTop = base;
			wave_sync();
		}
	}
	uint64_t k = 0;
	ROUND_CLOCK(4);
	while(k < nsamples) {
		if(st.nlive == 0) return false;                            // as sample_step
		const uint32_t act = nsamples - k < 64 ? (uint32_t)(nsamples - k) : 64u;
		const uint32_t x0 = jA * rnd.last + jC;
		const uint32_t x1 = kLcgA * x0 + kLcgC, x2 = kLcgA * x1 + kLcgC;
		const double rd = (double)((float)((x1 >> 16) ^ x2) / (float)0xffffffffu) * st.mass;
		// the dart (rs_dart's count of running sums <= rd, by bisection)
		uint32_t lo = 0, hi = st.nlive;
		while(lo < hi) {
			const uint32_t mid = (lo + hi) >> 1;
			if(rd < w.pre[mid]) hi = mid; else lo = mid + 1;
		}
		const uint32_t idx = lo < st.nlive ? lo : st.nlive - 1;
		const uint32_t l0 = (uint32_t)__shfl((int)co.lv0, (int)(idx & 63)), l1 = (uint32_t)__shfl((int)co.lv1, (int)(idx & 63));
		const uint32_t bi = idx < 64 ? l0 : l1;
		const uint32_t* rw = WaveCoop::r1w(w, bi);
		const R1N s = WaveCoop::unpack(rw[0], rw[1], rw[2]);
		uint32_t n, cur0, thresh;
		bool swap, ready;
		if(s.inited) {
			n = s.n; cur0 = s.cur; thresh = s.thresh; swap = s.swaplist != 0;
			ready = swap && (cur0 > 0 || s.converted);            // the swap list is laid out
		} else {
			n = (uint16_t)w.big[bi].size; cur0 = 0; swap = n < 128; ready = false;
			const uint16_t t = (uint16_t)(0.10f * (float)n);
			thresh = t > 16 ? t : 16;
		}
		const uint32_t x3 = kLcgA * x2 + kLcgC, x4 = kLcgA * x3 + kLcgC;
		const uint32_t u2 = (x3 >> 16) ^ x4;
		const uint32_t rn = n ? u2 % n : 0;
		const uint32_t key = ((bi << 16) | rn) + 1u;
		// the batch's earlier draws from the same range (its count), one pass per distinct range
		uint32_t cnt = 1;
		for(uint64_t rem = __ballot(lane < act); rem;) {
			const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)bi, (int)((uint32_t)__ffsll((unsigned long long)rem) - 1));
			const uint64_t m = __ballot(bi == b) & rem;
			if(bi == b) cnt = (uint32_t)__popcll(m & ((1ull << lane) - 1ull)) + 1;
			rem &= ~m;
		}
		const uint32_t cur1 = cur0 + cnt;                          // the range's count after this draw
		// a swap list's last element may be drawn in the batch (the range then leaves the
		// sampler after the batch, which ends with that draw); a seen list converts first
		bool reg = lane < act && n != 0 && (swap ? cur1 <= n : cur1 < n);
		uint32_t pos = 0;                                          // swap list: the drawn position
		if(swap) {
			reg = reg && ready;
			pos = cur1 - 1 + (reg ? u2 % (n - (cur1 - 1)) : 0);
		} else {
			reg = reg && cur1 < thresh && !seen_has(w, key);       // cur1 >= thresh: conversion
		}
		const bool term = reg && swap && cur1 == n;                // done(): finishedRange after it
		// Inside the batch, from a 128-slot LDS table (key -> mask of the lanes that drew it):
		// a seen-list draw of a key an earlier lane drew is a redraw (the serial step's); a
		// swap-list draw reads what its range's earlier exchanges left.  With A the list at
		// the batch start, lane L moves v_L to its drawn position r_L and takes the element at
		// r_L: v_L = A[c_L] unless an earlier lane drew c_L (then that lane's v), the element
		// = A[r_L] unless an earlier lane drew r_L (then the last such lane's v).  Cursor
		// positions grow and drawn ones are >= them, so no other write reaches either.
		const uint32_t ikey = swap ? ((bi << 16) | pos) + 1u : key;
		w.bkey[lane] = 0; w.bkey[lane + 64] = 0;
		w.bmlo[lane] = 0; w.bmlo[lane + 64] = 0; w.bmhi[lane] = 0; w.bmhi[lane + 64] = 0;
		wave_sync();
		uint32_t bslot = 0;
		if(reg) {
			bslot = (ikey * 2654435761u) >> 25;
			for(;;) {
				const uint32_t old = atomicCAS(&w.bkey[bslot], 0u, ikey);
				if(old == 0u || old == ikey) break;
				bslot = (bslot + 1) & 127;
			}
		}
		wave_sync();
		if(reg) atomicOr(lane < 32 ? &w.bmlo[bslot] : &w.bmhi[bslot], 1u << (lane & 31));
		wave_sync();
		const uint64_t below = (1ull << lane) - 1ull;
		uint64_t mine = 0;                                         // the lanes that drew our key
		int pr = -1, pc = -1;                                      // last earlier lane drawing r_L / c_L
		if(reg) {
			mine = ((uint64_t)w.bmhi[bslot] << 32) | w.bmlo[bslot];
			if(!swap) {
				if(mine & below) reg = false;                      // a redraw
			} else {
				if(mine & below) pr = 63 - __clzll(mine & below);
				const uint32_t ckey = ((bi << 16) | (cur1 - 1)) + 1u;
				for(uint32_t h = (ckey * 2654435761u) >> 25;; h = (h + 1) & 127) {
					const uint32_t v = w.bkey[h];
					if(v == 0u) break;
					if(v == ckey) {
						const uint64_t mc = (((uint64_t)w.bmhi[h] << 32) | w.bmlo[h]) & below;
						if(mc) pc = 63 - __clzll(mc);
						break;
					}
				}
			}
		}
		const uint64_t bad = __ballot(!reg) & (act == 64 ? ~0ull : ((1ull << act) - 1ull));
		uint32_t F = bad ? (uint32_t)__ffsll((unsigned long long)bad) - 1 : act;
		// the batch ends with the first draw that exhausts its range (if before F)
		const uint64_t terms = __ballot(term) & (F == 64 ? ~0ull : ((1ull << F) - 1ull));
		const uint32_t T = terms ? (uint32_t)__ffsll((unsigned long long)terms) - 1 : 64u;
		if(T < F) F = T + 1;
		const uint64_t com = F == 64 ? ~0ull : ((1ull << F) - 1ull);   // the committed lanes
		bool full = false;
		uint32_t out = rn;
		const bool sw = lane < F && swap;
		const uint32_t cpos = s.list + cur1 - 1, rpos = s.list + pos;   // swap lists: arena positions
		uint32_t v = sw ? w.arena[cpos] : 0u, a0r = sw ? w.arena[rpos] : 0u;
		if(lane < F) {
			uint32_t* pw = WaveCoop::r1w(w, bi);
			atomicMax(&pw[0], n | (cur1 << 16));
			if(!swap) {
				uint32_t h = (key * 2654435761u) >> 22;
				full = true;
				for(int probe = 0; probe < kHash; probe++, h = (h + 1) & (kHash - 1))
					if(atomicCAS(&w.hash[h], 0u, key) == 0u) { full = false; break; }
				pw[1] = thresh | ((uint32_t)s.list << 16);
				pw[2] = 1u;                                        // inited, seen-list mode
			}
		}
		ROUND_CLOCK(5);
		const uint64_t swm = __ballot(sw);
		if(swm) {
			// v_L through the chain of earlier lanes that drew c_L (pointer jumping: after
			// round i a lane points 2^i links up; a lane whose link is a root takes its v)
			int p = sw ? pc : -1;
			for(int it = 0; it < 6; it++) {
				const int src = p >= 0 ? p : (int)lane;
				const uint32_t vp = (uint32_t)__shfl((int)v, src);
				const int pp = __shfl(p, src);
				if(p >= 0) { if(pp < 0) { v = vp; p = -1; } else p = pp; }
			}
			const uint32_t vr = (uint32_t)__shfl((int)v, pr >= 0 ? pr : (int)lane);
			if(sw) out = pr >= 0 ? vr : a0r;
			// the exchanges' net effect: each drawn position ends with the last committed
			// drawer's v, then each cursor position with its draw's element (a cursor position
			// may be an earlier drawn one)
			wave_sync();
			if(sw && 63 - __clzll(mine & com) == (int)lane) w.arena[rpos] = (uint16_t)v;
			wave_sync();
			if(sw) w.arena[cpos] = (uint16_t)out;
			wave_sync();
			stats[3] += (uint32_t)__popcll(swm);
		}
		if(lane < F) put(k + lane, w.big[bi], (uint16_t)out);
		if(__ballot(full)) return false;
		stats[0]++;
		if(F) {
			rnd.last = (uint32_t)__builtin_amdgcn_readlane((int)x4, (int)(F - 1));   // 4F steps on
			rnd.lastOff = 0;
			k += F;
			stats[1] += F;
		}
		if(T < 64 && T + 1 == F) {                                 // finishedRange (as sample_step)
			wave_sync();
			const uint32_t tb = (uint32_t)__builtin_amdgcn_readlane((int)bi, (int)T);
			st.mass -= w.masses[tb];
			const uint32_t q = co.rs_remove(w, tb, st.nlive);
			st.nlive--;
			co.rs_rebuild(w, st.nlive, q);
			wave_sync();
			continue;                                              // the next batch
		}
		wave_sync();
		ROUND_CLOCK(7);
		if(F < act) {
			if(!sample_step(k, rnd, w, co, st, [&](uint64_t kk, const Range& rg, uint16_t elt) { put(kk, rg, elt); }))
				return false;
			k++;
			stats[2]++;
			ROUND_CLOCK(6);
		}
	}
	return true;
}

// One wave per job, its workspace in LDS: the sampling loop is a chain of dependent
// list/mass lookups, so it runs at LDS latency instead of HBM latency.  Jobs are taken
// from a queue counter (counters[5]) so long and short jobs balance over the grid.
__global__ void __launch_bounds__(64)
round_sample_kernel(RoundLaunch a) {
	__shared__ SampleWs w;
	__shared__ uint32_t qsh;
	WaveCoop co;
	const Job* jobs = reinterpret_cast<const Job*>(a.jobs);
	const Range* ranges = reinterpret_cast<const Range*>(a.ranges);
	const uint32_t njobs = min(a.counters[3], a.job_cap);
	const bool fits = a.counters[0] <= a.sat_cap && a.counters[1] <= a.row_cap;
	// lane l's draw in a batch starts 4l LCG steps on: x -> jA * x + jC
	uint32_t jA = 1, jC = 0;
	for(uint32_t i = 0; i < 4 * threadIdx.x; i++) { jA *= kLcgA; jC = kLcgA * jC + kLcgC; }
	// the wave's statistics, added to the launch's counters once at the end (per-job
	// atomics on a handful of shared counters serialised across the grid)
	uint64_t stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	uint64_t nsamp = 0;
	uint32_t maxsamp = 0;
	// first job: the workgroup's own index; then from the queue counter (offset by the grid)
	uint32_t q = blockIdx.x;
	for(;;) {
		if(q >= njobs) break;
		const Job j = jobs[q];
		nsamp += j.nsamples;
		maxsamp = max(maxsamp, j.nsamples);
		for(uint32_t i = threadIdx.x; i < j.nb && i < (uint32_t)kMaxRanges; i += 64) w.big[i] = ranges[j.range0 + i];
		wave_sync();
		Rnd rnd{j.rnd_last, j.rnd_lastoff};
		const bool ok = sample_wave(j.nb, j.nsamples, rnd, w, co, jA, jC, stats, [&](uint64_t k, const Range& rg, uint16_t elt) {
			if(!fits) return;
			bt2x_sat s;
			s.rdoff = (uint16_t)rg.rdoff; s.rand_n = 1; s.fwlen = BT2X_SAT_FWLEN(rg.fw, j.seedlen);
			a.sats[j.sat_base + k] = s;
			bt2x_resolve_in ri;
			ri.row = rg.topf + elt; ri.qlen = j.seedlen; ri.pad = 0;
			a.rows[j.elt_base + k] = ri;
		});
		if(threadIdx.x == 0) {
			bt2x_round_out& o = a.out[j.read];
			o.rnd_last = rnd.last; o.rnd_lastoff = rnd.lastOff;
			if(!ok) o.status = BT2X_ROUND_REDO;
			qsh = gridDim.x + atomicAdd(&a.counters[5], 1u);       // the next job
		}
		wave_sync();
		q = qsh;
		wave_sync();
	}
	if(threadIdx.x == 0) {
		atomicAdd(&a.counters[6], (uint32_t)nsamp);
		atomicMax(&a.counters[7], maxsamp);
		for(int i = 0; i < 4; i++) atomicAdd(&a.counters[8 + i], (uint32_t)stats[i]);
		for(int i = 4; i < 8; i++) atomicAdd(&a.counters[8 + i], (uint32_t)(stats[i] >> 10));
	}
}

} // namespace

size_t bt2x_round_ws_bytes() { return sizeof(PrepWs); }
size_t bt2x_round_job_bytes() { return sizeof(Job); }
size_t bt2x_round_range_bytes() { return sizeof(Range); }

// 4 one-wave workgroups per CU: small work per read, workspaces in HBM
uint32_t bt2x_round_lanes(int ncu) { return (uint32_t)(ncu > 0 ? ncu : 256) * 4u * 64u; }

int bt2x_launch_round(const RoundLaunch& a, void* stream) {
	if(a.n == 0) return 0;
	uint32_t blocks = a.nlanes / 64;
	if(blocks > (a.n + 63) / 64) blocks = (a.n + 63) / 64;
	hipLaunchKernelGGL(round_prep_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
	// persistent: 6 one-wave groups per CU (LDS: ~20 KiB each), jobs from the queue
	uint32_t sblocks = a.nlanes / 64 / 4 * 6;
	if(sblocks > a.job_cap) sblocks = a.job_cap;
	if(sblocks < 1) sblocks = 1;
	hipLaunchKernelGGL(round_sample_kernel, dim3(sblocks), dim3(64), 0, (hipStream_t)stream, a);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
