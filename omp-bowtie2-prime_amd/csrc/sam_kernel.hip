// sam_kernel.hip -- SAM record tails from the read store (bt2x_sam_tails, include/bt2x.h).
//
// The text an aligned read's record carries after its MAPQ field when the printed edits are
// mismatches only (AlnSinkSam::appendMate, aln_sink.cpp:1889-2090; the tags of
// SamConfig::printAlignedOptFlags, sam.cpp:121-730; CIGAR and MD:Z of StackedAln over
// mismatch-only edits, aligner_result.cpp:448-770): the host keeps the record's head (name,
// flags, reference, position, MAPQ) and every other record; this kernel writes the bulk of
// the bytes (SEQ, QUAL) straight from the read's store slot, so the host never touches the
// read's sequence or qualities to print it.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"

namespace {

constexpr int kTailMax = 2 * BT2X_STORE_MAX_LEN + 200 + 4 * BT2X_SAM_MAX_MM;

__device__ __forceinline__ int put_uint(char* b, int k, uint32_t v) {
	char t[10];
	int n = 0;
	do { t[n++] = (char)('0' + v % 10u); v /= 10u; } while(v);
	while(n) b[k++] = t[--n];
	return k;
}
__device__ __forceinline__ int put_int(char* b, int k, int32_t v) {
	if(v < 0) { b[k++] = '-'; return put_uint(b, k, (uint32_t)(-(int64_t)v)); }
	return put_uint(b, k, (uint32_t)v);
}
__device__ __forceinline__ int put_str(char* b, int k, const char* s) {
	while(*s) b[k++] = *s++;
	return k;
}

// One wave per request (64-thread workgroups, so __syncthreads is the wave's barrier): lane
// 0 writes CIGAR and the tags into the wave's LDS buffer, every lane the sequence and the
// qualities, then the wave copies the tail out.
__global__ void __launch_bounds__(64) sam_tail_kernel(const bt2x_sam_req* __restrict__ req, uint32_t n,
                                                      const uint8_t* __restrict__ store, char* __restrict__ text,
                                                      uint16_t* __restrict__ lens) {
	__shared__ char b[kTailMax];
	const int lane = (int)threadIdx.x;
	for(uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
		const bt2x_sam_req q = req[i];
		const int R = q.rdlen;
		const uint8_t* slot = store + (size_t)q.slot * BT2X_STORE_SLOT_BYTES;
		const uint8_t* codes = slot + (q.fw ? 0 : R);                 // patFw / patRc
		const uint8_t* quals = slot + (q.fw ? 2 * R : 3 * R);         // qualities / reversed
		const int h = (R >= 100 ? 3 : R >= 10 ? 2 : 1) + 1 + 7;       // "<R>M\t*\t0\t0\t"
		for(int k = lane; k < R; k += 64) {
			const uint8_t c = codes[k];
			b[h + k] = "ACGTN"[c > 4 ? 4 : c];
			b[h + R + 1 + k] = (char)quals[k];
		}
		int len = 0;
		if(lane == 0) {
			int k = put_uint(b, 0, (uint32_t)R);
			b[k++] = 'M';
			put_str(b, k, "\t*\t0\t0\t");
			b[h + R] = '\t';
			k = h + 2 * R + 1;
			k = put_str(b, k, "\tAS:i:");
			k = put_int(b, k, q.as);
			if(q.has_xs) { k = put_str(b, k, "\tXS:i:"); k = put_int(b, k, q.xs); }
			k = put_str(b, k, "\tXN:i:");
			k = put_uint(b, k, q.xn);
			k = put_str(b, k, "\tXM:i:");
			k = put_uint(b, k, q.nmm);
			k = put_str(b, k, "\tXO:i:0\tXG:i:0\tNM:i:");
			k = put_uint(b, k, q.nmm);
			k = put_str(b, k, "\tMD:Z:");
			// buildMdz + writeMdz over match runs and mismatches
			int prev = 0;
			bool mm_last = false, first = true;
			for(int e = 0; e < (int)q.nmm; e++) {
				const int p = q.mm_pos[e];
				if(p > prev) { k = put_uint(b, k, (uint32_t)(p - prev)); mm_last = false; first = false; }
				if(mm_last || first) b[k++] = '0';
				b[k++] = (char)q.mm_chr[e];
				mm_last = true; first = false;
				prev = p + 1;
			}
			if(R > prev) k = put_uint(b, k, (uint32_t)(R - prev));
			else if(mm_last) b[k++] = '0';
			k = put_str(b, k, "\tYT:Z:UU\tYF:Z:LN\n");
			len = k;
		}
		len = __builtin_amdgcn_readfirstlane(len);
		__syncthreads();
		char* dst = text + q.text_off;
		for(int k = lane; k < len; k += 64) dst[k] = b[k];
		if(lane == 0) lens[i] = (uint16_t)len;
		__syncthreads();                                               // b is reused
	}
}

} // namespace

int bt2x_launch_sam_tails(const bt2x_sam_req* d_req, uint32_t n, const uint8_t* d_store, char* d_text,
                          uint16_t* d_lens, int ncu, void* stream) {
	if(n == 0) return BT2X_OK;
	uint32_t grid = (uint32_t)ncu * 16u;
	if(grid > n) grid = n;
	hipLaunchKernelGGL(sam_tail_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, d_req, n, d_store, d_text, d_lens);
	return hipGetLastError() == hipSuccess ? BT2X_OK : BT2X_E_NODEVICE;
}
