// window_kernel.hip — DP reference windows cut from the resident index (gfx950).
//
// SwAligner::initRef fetches each rectangle's reference characters with
// BitPairReference::getStretch (aligner_sw.cpp:117-229, reference.cpp:484-611): the
// window [refl, refl + ncol) of text tidx, N (4) outside the text and in its N runs.
// A problem flagged BT2X_DP_REF_TEXT names (tidx = ref_off, refl, ncol) instead of
// carrying the bytes; this kernel cuts the window from the joined text the context keeps
// in HBM (16 bases per u32, LSB-first) through the fragment table (rstarts: joined
// offset, text id, text offset per maximal non-N stretch, in joined order), so the host
// never touches the 0.8 GB packed text and the windows never cross PCIe.
//
// One wave per problem, one output byte per lane and step; every problem's window goes to
// its slot of kWinSlot bytes in `win`, and its dp_in to `out` with ref_off = the
// slot (unflagged problems are copied from `refs`), so the DP kernels run unchanged.
// HBM-bound: per problem ~ncol/4 bytes of packed text read, ncol bytes written.
#include <hip/hip_runtime.h>

#include "bt2x_device.h"

namespace {

// last fragment k in [lo, hi) with toff_k <= off (lo - 1 if none); fragments of one text
// are in text order
__device__ __forceinline__ int64_t frag_at(const uint64_t* rs, int64_t lo, int64_t hi, int64_t off) {
	int64_t a = lo, b = hi;                     // answer in [lo - 1, hi)
	while(a < b) {
		const int64_t m = (a + b) >> 1;
		if((int64_t)rs[3 * m + 2] <= off) a = m + 1; else b = m;
	}
	return a - 1;
}

// first fragment k with tidx_k >= t
__device__ __forceinline__ int64_t frag_text_lb(const uint64_t* rs, int64_t nfrag, uint64_t t) {
	int64_t a = 0, b = nfrag;
	while(a < b) {
		const int64_t m = (a + b) >> 1;
		if(rs[3 * m + 1] < t) a = m + 1; else b = m;
	}
	return a;
}

__global__ void __launch_bounds__(256) window_kernel(DevIndex ix, const bt2x_dp_in* __restrict__ in, uint32_t n,
                                                     const uint8_t* __restrict__ refs, bt2x_dp_in* __restrict__ out,
                                                     uint8_t* __restrict__ win) {
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6);
	if(i >= n) return;
	bt2x_dp_in p = in[i];
	uint8_t* w = win + (size_t)i * kWinSlot;
	const uint32_t ncol = p.ncol;
	const bool named = (p.flags & BT2X_DP_REF_TEXT) != 0;
	if(named && (!ix.text || !ix.rstarts || p.ref_off >= ix.npat)) {
		// a window the context cannot cut (a launch without BT2X_DPL_REF_TEXT on a context
		// with no resident text, or a text id out of range): N columns, and the DP kernels
		// refuse the problem
		for(uint32_t c = lane; c < ncol; c += 64u) w[c] = 4;
		p.flags |= kDpBadWindow;
	} else if(named) {
		const uint64_t t = p.ref_off;
		const int64_t nfrag = (int64_t)ix.nfrag;
		// text t's fragment range: from the per-text table (one load), else two searches
		const bool tab = ix.tfirst != nullptr;             // t < npat (checked above)
		const int64_t lo = tab ? (int64_t)ix.tfirst[t] : frag_text_lb(ix.rstarts, nfrag, t);
		const int64_t hi = tab ? (int64_t)ix.tfirst[t + 1] : frag_text_lb(ix.rstarts, nfrag, t + 1);
		// one search per problem (every lane the same addresses: broadcast loads), then each
		// column moves forward from the window start's fragment; a window rarely crosses one
		// (per-column binary searches made this kernel a chain of dependent loads per column)
		const int64_t k0 = frag_at(ix.rstarts, lo, hi, p.refl);
		for(uint32_t c = lane; c < ncol; c += 64u) {
			const int64_t off = p.refl + (int64_t)c;
			uint8_t code = 4;
			int64_t kc = k0 < lo ? lo - 1 : k0;
			while(kc + 1 < hi && (int64_t)ix.rstarts[3 * (kc + 1) + 2] <= off) kc++;
			// the last non-empty fragment starting at or before off (RefInfo::stretch's rule)
			for(int64_t k = kc; k >= lo; k--) {
				const uint64_t joff = ix.rstarts[3 * k], toff = ix.rstarts[3 * k + 2];
				const uint64_t jend = k + 1 < nfrag ? ix.rstarts[3 * (k + 1)] : ix.len;
				if(jend == joff) continue;
				const uint64_t j = joff + (uint64_t)(off - (int64_t)toff);
				if(j < jend) code = (uint8_t)((ix.text[j >> 4] >> ((j & 15u) << 1)) & 3u);
				break;
			}
			w[c] = code;
		}
	} else {
		for(uint32_t c = lane; c < ncol; c += 64u) w[c] = refs[p.ref_off + c];
	}
	if(lane == 0) {
		p.ref_off = (uint64_t)i * kWinSlot;
		p.flags &= (uint8_t)~BT2X_DP_REF_TEXT;
		out[i] = p;
	}
}

// Read store (bt2x_store_reads): one wave per read; lane k takes bytes k, k + 64, ... of
// the read: patFw and the qualities as sent, patRc (complement, N stays N) and the
// reversed qualities mirrored (Read::constructRevComps / constructReverses, read.h).
__global__ void __launch_bounds__(256) store_kernel(const uint8_t* __restrict__ packed,
                                                   const bt2x_store_in* __restrict__ in, uint32_t n,
                                                   uint8_t* __restrict__ store) {
	const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
	if(i >= n) return;
	const bt2x_store_in q = in[i];
	const uint32_t len = q.len;
	const uint8_t* src = packed + q.off;
	uint8_t* dst = store + (size_t)q.slot * BT2X_STORE_SLOT_BYTES;
	for(uint32_t k = lane; k < len; k += 64u) {
		const uint8_t c = src[k], ql = src[len + k];
		dst[k] = c;
		dst[2 * len - 1 - k] = c < 4 ? (uint8_t)(3 - c) : c;
		dst[2 * len + k] = ql;
		dst[4 * len - 1 - k] = ql;
	}
}

} // namespace

int bt2x_launch_store(const uint8_t* d_packed, const bt2x_store_in* d_in, uint32_t n, uint8_t* d_store,
                      void* stream) {
	if(n == 0) return BT2X_OK;
	hipLaunchKernelGGL(store_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, d_packed, d_in, n, d_store);
	return hipGetLastError() == hipSuccess ? BT2X_OK : BT2X_E_NODEVICE;
}

int bt2x_launch_windows(const DevIndex& ix, const bt2x_dp_in* d_in, uint32_t n, const uint8_t* d_refs,
                        bt2x_dp_in* d_out, uint8_t* d_win, void* stream) {
	if(n == 0) return BT2X_OK;
	hipLaunchKernelGGL(window_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, ix, d_in, n, d_refs, d_out,
	                   d_win);
	return hipGetLastError() == hipSuccess ? BT2X_OK : BT2X_E_NODEVICE;
}
