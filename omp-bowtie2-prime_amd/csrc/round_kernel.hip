// round_kernel.hip — the per-read part of a seed round on gfx950 (bt2x_seed_round):
// after the seed kernel, one lane per read runs searchAllSeedsFinalize, rankSeedHits and
// prioritizeSATups (round_core.h) and appends the read's extension list and the BW rows
// to resolve to arenas allocated with atomics; sa_resolve_kernel_dn then places the rows.
//
// This is RNG-sequential, branchy integer work with a few hundred operations per read
// (a few thousand for repetitive reads that sample up to maxelt elements): latency, not
// bandwidth.  A persistent grid of lanes, each with a private workspace in HBM, walks the
// reads; the kernel's value is that the host never touches these phases and the rows
// never cross PCIe.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"
#include "round_core.h"

namespace {

using namespace bt2x_round;

__global__ void __launch_bounds__(64)
round_kernel(RoundLaunch a) {
	const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
	Ws& w = *reinterpret_cast<Ws*>(a.ws + (size_t)lane * sizeof(Ws));
	for(uint32_t r = lane; r < a.n; r += gridDim.x * blockDim.x) {
		const bt2x_round_in in = a.in[r];
		Rnd rnd{in.rnd_last, in.rnd_lastoff};
		const Result res = run(in, a.seeds + in.seed0, a.seed_out + in.seed0, a.exr + in.exr0, a.maxelt, rnd, w);
		bt2x_round_out o;
		o.rnd_last = rnd.last; o.rnd_lastoff = rnd.lastOff;
		o.num_elts = res.numElts; o.nonz = res.nonz; o.status = res.status;
		o.sat0 = o.nsat = o.elt0 = o.nelt = o.exr0 = o.nexr = 0;
		if(res.status == BT2X_ROUND_OK) {
			o.nsat = res.nsat; o.nelt = res.nelt; o.nexr = res.nexnew;
			o.sat0 = atomicAdd(&a.counters[0], res.nsat);
			o.elt0 = atomicAdd(&a.counters[1], res.nelt);
			o.exr0 = res.nexnew ? atomicAdd(&a.counters[2], res.nexnew) : 0;
			const uint32_t L = in.seedlen;
			if(o.sat0 + res.nsat <= a.sat_cap && o.elt0 + res.nelt <= a.row_cap) {
				uint32_t e = o.elt0;
				for(uint32_t i = 0; i < res.nsat; i++) {
					const Range& rg = w.r2[w.satRange[i]];
					bt2x_sat s;
					s.rdoff = rg.rdoff; s.rand_n = w.satN[i]; s.fw = rg.fw; s.seedlen = (uint8_t)L;
					a.sats[o.sat0 + i] = s;
					for(uint32_t k = 0; k < w.satN[i]; k++) {
						bt2x_resolve_in ri;
						ri.row = rg.topf + w.satElt[i] + k;
						ri.qlen = L;
						ri.pad = 0;
						a.rows[e++] = ri;
					}
				}
			}
			if(o.exr0 + res.nexnew <= a.exr_cap)
				for(uint32_t i = 0; i < res.nexnew; i++) a.exr_out[o.exr0 + i] = w.exnew[i];
		}
		a.out[r] = o;
	}
}

} // namespace

size_t bt2x_round_ws_bytes() { return sizeof(Ws); }

// 2 one-wave workgroups per CU: the work per read is small, the workspace is not
uint32_t bt2x_round_lanes(int ncu) { return (uint32_t)(ncu > 0 ? ncu : 256) * 2u * 64u; }

int bt2x_launch_round(const RoundLaunch& a, void* stream) {
	if(a.n == 0) return 0;
	uint32_t blocks = a.nlanes / 64;
	if(blocks > (a.n + 63) / 64) blocks = (a.n + 63) / 64;
	hipLaunchKernelGGL(round_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
