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

__global__ void __launch_bounds__(64)
round_prep_kernel(RoundLaunch a) {
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	PrepWs& w = *reinterpret_cast<PrepWs*>(a.ws + (size_t)lane * sizeof(PrepWs));
	Job* jobs = reinterpret_cast<Job*>(a.jobs);
	Range* ranges = reinterpret_cast<Range*>(a.ranges);
	for(uint32_t r = lane; r < a.n; r += gridDim.x * blockDim.x) {
		const bt2x_round_in in = a.in[r];
		Rnd rnd{in.rnd_last, in.rnd_lastoff};
		Prep p = prep(in, a.seeds + in.seed0, a.seed_out + in.seed0, a.exr + in.exr0, a.maxelt, rnd, w);
		bt2x_round_out o;
		o.rnd_last = rnd.last; o.rnd_lastoff = rnd.lastOff;
		o.num_elts = p.numElts; o.nonz = p.nonz; o.status = p.status;
		o.sat0 = o.nsat = o.elt0 = o.nelt = o.exr0 = o.nexr = 0;
		if(p.status == BT2X_ROUND_OK) {
			const uint32_t L = in.seedlen;
			const uint32_t nsat = p.nsmallSat + (uint32_t)p.nsamples, nelt = (uint32_t)(p.smallElts + p.nsamples);
			uint32_t job = 0xffffffffu, range0 = 0;
			const uint32_t nb = p.n2 - p.nsmall;
			if(p.nsamples) {
				job = atomicAdd(&a.counters[3], 1u);
				range0 = atomicAdd(&a.counters[4], nb);
				if(job >= a.job_cap || range0 + nb > a.range_cap) {
					p.status = BT2X_ROUND_REDO;                  // hand the read back to the host
					if(job < a.job_cap) {                         // an empty job keeps the queue dense
						Job j = {};
						j.read = r; j.rnd_last = rnd.last; j.rnd_lastoff = rnd.lastOff;
						jobs[job] = j;
					}
				}
			}
			if(p.status == BT2X_ROUND_OK) {
				o.nsat = nsat; o.nelt = nelt; o.nexr = p.nexnew;
				o.sat0 = atomicAdd(&a.counters[0], nsat);
				o.elt0 = atomicAdd(&a.counters[1], nelt);
				o.exr0 = p.nexnew ? atomicAdd(&a.counters[2], p.nexnew) : 0;
				if(o.sat0 + nsat <= a.sat_cap && o.elt0 + nelt <= a.row_cap) {
					uint32_t e = o.elt0;
					for(uint32_t i = 0; i < p.nsmallSat; i++) {
						const Range& rg = w.r2[i];
						bt2x_sat s;
						s.rdoff = rg.rdoff; s.rand_n = (uint16_t)rg.size; s.fw = rg.fw; s.seedlen = (uint8_t)L;
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
			} else {
				o.status = p.status;
			}
		}
		a.out[r] = o;
	}
}

__device__ __forceinline__ double readlane_f64(double v, uint32_t k) {
	const uint64_t u = __builtin_bit_cast(uint64_t, v);
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)k);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)k);
	return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

struct WaveCoop {                            // a one-wave workgroup runs one job
	// RowSampler state in registers: live range ids, their masses and running sums of
	// list positions l and l + 64
	uint32_t lv0, lv1;
	double m0, m1, p0, p1;
	// Random1toN state of ranges l and l + 64 (n | cur << 16, thresh | list << 16, flags)
	// and their fields (topf, size, rdoff | fw << 24)
	uint32_t ra[3], rb[3];
	uint32_t ga[4], gb[4];
	__device__ void r1n_reset(const SampleWs&, uint32_t) {
		for(int i = 0; i < 3; i++) { ra[i] = 0; rb[i] = 0; }
	}
	__device__ R1N r1n_get(const SampleWs&, uint32_t bi) const {
		const uint32_t l = bi & 63;
		const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ra[0] : rb[0]), (int)l);
		const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ra[1] : rb[1]), (int)l);
		const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)(bi < 64 ? ra[2] : rb[2]), (int)l);
		R1N r;
		r.n = (uint16_t)w0; r.cur = (uint16_t)(w0 >> 16); r.thresh = (uint16_t)w1; r.list = (uint16_t)(w1 >> 16);
		r.inited = (uint8_t)w2; r.swaplist = (uint8_t)(w2 >> 8); r.converted = (uint8_t)(w2 >> 16); r.pad = 0;
		return r;
	}
	__device__ void r1n_set(const SampleWs&, uint32_t bi, const R1N& r) {
		const uint32_t w0 = (uint32_t)r.n | ((uint32_t)r.cur << 16), w1 = (uint32_t)r.thresh | ((uint32_t)r.list << 16);
		const uint32_t w2 = (uint32_t)r.inited | ((uint32_t)r.swaplist << 8) | ((uint32_t)r.converted << 16);
		if(threadIdx.x == (bi & 63)) {
			if(bi < 64) { ra[0] = w0; ra[1] = w1; ra[2] = w2; } else { rb[0] = w0; rb[1] = w1; rb[2] = w2; }
		}
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
	__device__ void sync() const { __syncthreads(); }
	__device__ uint64_t ballot(bool p) const { return __ballot(p); }
	__device__ bool leader() const { return threadIdx.x == 0; }
	__device__ void rs_init(SampleWs& w, uint32_t nb) {
		const uint32_t l = threadIdx.x;
		lv0 = l; lv1 = l + 64;
		m0 = l < nb ? w.masses[l] : 0.0; m1 = l + 64 < nb ? w.masses[l + 64] : 0.0;
		w.mlive[l] = m0; w.mlive[l + 64] = m1;
		__syncthreads();
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
		__syncthreads();
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
		__syncthreads();
		return q;
	}
};

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
	for(;;) {
		if(threadIdx.x == 0) qsh = atomicAdd(&a.counters[5], 1u);
		__syncthreads();
		const uint32_t q = qsh;
		__syncthreads();
		if(q >= njobs) break;
		const Job j = jobs[q];
		if(threadIdx.x == 0) { atomicAdd(&a.counters[6], j.nsamples); atomicMax(&a.counters[7], j.nsamples); }
		for(uint32_t i = threadIdx.x; i < j.nb && i < (uint32_t)kMaxRanges; i += 64) w.big[i] = ranges[j.range0 + i];
		__syncthreads();
		Rnd rnd{j.rnd_last, j.rnd_lastoff};
		const bool ok = sample(j.nb, j.nsamples, rnd, w, co, [&](uint64_t k, const Range& rg, uint16_t elt) {
			if(!fits) return;
			bt2x_sat s;
			s.rdoff = rg.rdoff; s.rand_n = 1; s.fw = rg.fw; s.seedlen = (uint8_t)j.seedlen;
			a.sats[j.sat_base + k] = s;
			bt2x_resolve_in ri;
			ri.row = rg.topf + elt; ri.qlen = j.seedlen; ri.pad = 0;
			a.rows[j.elt_base + k] = ri;
		});
		if(threadIdx.x == 0) {
			bt2x_round_out& o = a.out[j.read];
			o.rnd_last = rnd.last; o.rnd_lastoff = rnd.lastOff;
			if(!ok) o.status = BT2X_ROUND_REDO;
		}
		__syncthreads();
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
