// seed_kernel.hip — batched exact seed search + left extension on gfx950.
//
// Replaces MultiSeedAligner::searchAllSeedsDoAll(doExtend) (aligner_seed.cpp:674-725):
// searchSeedBi<8> (:820-957, startSearchSeedBi :757-811) then MultiSeedAligner::extend
// (:603-672) for every reported seed.  The reference interleaves 8 seeds per CPU thread
// to overlap cache misses; here every lane owns one seed and thousands of waves keep
// HBM busy, so the dependent LF chain of one seed is hidden by the others.
//
// Per LF step a lane reads the 128-byte side (one L2 line; 8 x dwordx4) that holds the
// row, counts bit-pairs below the row with 64-bit popcounts and adds the side's occ[]
// word and fchr[] (Ebwt::countBt2Side / countBt2SideEx, bt2_idx.h:1811-1972).
// Algorithmic bytes per launch = 128*(2*n_mapBiLFEx + n_mapLF1) + 16*n_ftab.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"

#define OFF_MASK 0xffffffffffffffffULL

namespace {

struct Side {
	uint64_t w[12];          // 12 words of packed BWT (384 chars); constant indices only
	uint64_t o0, o1, o2, o3; // occ[A,C,G,T] at the side start (named: selected, not indexed)
	uint64_t byte_off;       // side byte offset in ebwt
	int charoff;             // row % 384
};

__device__ __forceinline__ void load_side(const DevIndex& ix, uint64_t row, Side& s) {
	const uint64_t side = row / BT2X_SIDE_CHARS;
	s.charoff = (int)(row - side * BT2X_SIDE_CHARS);
	s.byte_off = side * BT2X_SIDE_BYTES;
	const uint4* p = reinterpret_cast<const uint4*>(ix.ebwt + s.byte_off);
#pragma unroll
	for(int k = 0; k < 6; k++) {
		uint4 v = p[k];
		s.w[2 * k] = ((uint64_t)v.y << 32) | v.x;
		s.w[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
	}
	const uint4 v6 = p[6], v7 = p[7];
	s.o0 = ((uint64_t)v6.y << 32) | v6.x;
	s.o1 = ((uint64_t)v6.w << 32) | v6.z;
	s.o2 = ((uint64_t)v7.y << 32) | v7.x;
	s.o3 = ((uint64_t)v7.w << 32) | v7.z;
}

// Bit-pair matches of character c in word w, on the low bit of each pair (countInU64,
// bt2_idx.h:519-537).
__device__ __forceinline__ uint64_t match_c(uint64_t w, int c) {
	const uint64_t ct = c == 0 ? 0xffffffffffffffffULL : c == 1 ? 0xaaaaaaaaaaaaaaaaULL
	                  : c == 2 ? 0x5555555555555555ULL : 0ULL;
	const uint64_t x0 = w ^ ct;
	return x0 & (x0 >> 1) & 0x5555555555555555ULL;
}

__device__ __forceinline__ uint64_t prefix_mask(int charoff, int k) {
	int m = charoff - 32 * k;
	m = m < 0 ? 0 : (m > 32 ? 32 : m);
	return m >= 32 ? 0xffffffffffffffffULL : ((1ULL << (2 * m)) - 1ULL);
}

__device__ __forceinline__ bool dollar_before(const DevIndex& ix, const Side& s) {
	const uint64_t here = s.byte_off + (uint64_t)(s.charoff >> 2);
	if(s.byte_off <= ix.zbyte && here >= ix.zbyte)
		return here > ix.zbyte || (here == ix.zbyte && (s.charoff & 3) > ix.zbp);
	return false;
}

// Ebwt::countBt2Side (bt2_idx.h:1811-1846)
__device__ __forceinline__ uint64_t count_one(const DevIndex& ix, const Side& s, int c) {
	uint64_t cnt = 0;
#pragma unroll
	for(int k = 0; k < 12; k++) cnt += __popcll(match_c(s.w[k], c) & prefix_mask(s.charoff, k));
	if(c == 0 && dollar_before(ix, s)) cnt--;
	// mask-select (a ?: chain gets folded into an indexed, i.e. scratch, load)
	const uint64_t m0 = 0ULL - (uint64_t)(c == 0), m1 = 0ULL - (uint64_t)(c == 1);
	const uint64_t m2 = 0ULL - (uint64_t)(c == 2), m3 = 0ULL - (uint64_t)(c == 3);
	const uint64_t occ = (s.o0 & m0) | (s.o1 & m1) | (s.o2 & m2) | (s.o3 & m3);
	const uint64_t fc = (ix.fchr[0] & m0) | (ix.fchr[1] & m1) | (ix.fchr[2] & m2) | (ix.fchr[3] & m3);
	return occ + cnt + fc;
}

// Ebwt::countBt2SideEx (bt2_idx.h:1940-1972)
__device__ __forceinline__ void count_all(const DevIndex& ix, const Side& s, uint64_t o[4]) {
	uint64_t a = 0, cc = 0, g = 0, t = 0;
#pragma unroll
	for(int k = 0; k < 12; k++) {
		const uint64_t m = prefix_mask(s.charoff, k), w = s.w[k];
		a += __popcll(match_c(w, 0) & m);
		cc += __popcll(match_c(w, 1) & m);
		g += __popcll(match_c(w, 2) & m);
		t += __popcll(match_c(w, 3) & m);
	}
	if(dollar_before(ix, s)) a--;
	o[0] = s.o0 + a + ix.fchr[0];
	o[1] = s.o1 + cc + ix.fchr[1];
	o[2] = s.o2 + g + ix.fchr[2];
	o[3] = s.o3 + t + ix.fchr[3];
}

__device__ __forceinline__ int row_l(const Side& s) {
	// select the word without a dynamic register index (that would spill Side to scratch)
	const int k = s.charoff >> 5, sh = 2 * (s.charoff & 31);
	int c = 0;
#pragma unroll
	for(int q = 0; q < 12; q++) {
		const int cq = (int)((s.w[q] >> sh) & 3);   // computed per word, then selected
		c = (q == k) ? cq : c;
	}
	return c;
}

__device__ __forceinline__ uint64_t ftab_hi(const DevIndex& ix, uint64_t i) {
	const uint64_t v = ix.ftab[i];
	return v <= ix.len ? v : ix.eftab[(v ^ OFF_MASK) * 2 + 1];
}
__device__ __forceinline__ uint64_t ftab_lo(const DevIndex& ix, uint64_t i) {
	const uint64_t v = ix.ftab[i];
	return v <= ix.len ? v : ix.eftab[(v ^ OFF_MASK) * 2];
}

__global__ void __launch_bounds__(256)
seed_kernel(DevIndex ix, const uint8_t* __restrict__ reads, const bt2x_seed_in* __restrict__ in,
            uint32_t n, int do_extend, bt2x_seed_out* __restrict__ out,
            unsigned long long* __restrict__ ctr) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t n_bilf = 0, n_lf1 = 0, n_ftab = 0;
	if(i < n) {
		const bt2x_seed_in p = in[i];
		const uint8_t* rd = reads + p.read_off;
		const uint8_t* seq = rd + p.seed_off;
		const int nsteps = p.seed_len;
		uint64_t top = 0, bot = 0;
		int step = 0;
		bool done = false, report = false;
		const int off = nsteps - 1;
		const int fc = ix.ftab_chars;
		// startSearchSeedBi: ftab jump over the rightmost ftabChars characters
		if(fc > 1 && fc <= nsteps) {
			uint64_t fi = 0;
			for(int k = 0; k < fc; k++) fi = (fi << 2) | (uint64_t)(seq[off - fc + 1 + k] & 3);
			top = ftab_hi(ix, fi);
			bot = ftab_lo(ix, fi + 1);
			n_ftab++;
			if(bot == top) done = true; else step += fc;
		} else {
			const int c = seq[off];
			top = ix.fchr[c]; bot = ix.fchr[c + 1];
			if(bot == top) done = true; else step++;
		}
		if(!done && step == nsteps) { done = true; report = true; }
		Side st, sb;
		while(!done) {
			const int soff = nsteps - step - 1;
			step++;
			const int c = seq[soff];
			uint64_t tc, bc;
			if(bot - top > 1) {       // mapBiLFEx: both ends of the range
				n_bilf++;
				load_side(ix, top, st);
				load_side(ix, bot, sb);
				if(c == 4) break;
				tc = count_one(ix, st, c);
				bc = count_one(ix, sb, c);
			} else {                  // mapLF1(row, l, c)
				if(c == 4) break;
				n_lf1++;
				load_side(ix, top, st);
				if(row_l(st) != c || top == ix.zoff) break;
				tc = count_one(ix, st, c);
				bc = tc + 1;
			}
			if(bc == tc) break;
			top = tc; bot = bc;
			if(step == nsteps) { report = true; break; }
		}
		int nlex = 0;
		if(report && do_extend) {
			// extend() works on copies; the seed's own range is reported unchanged
			uint64_t etop = top, ebot = bot;
			// MultiSeedAligner::extend: walk left over read[seed_off-1 .. 0]
			const int lim = p.seed_off;
			for(int ii = 0; ii < lim; ii++) {
				const int rdc = seq[-1 - ii];
				if(ebot - etop > 1) {
					n_bilf++;
					uint64_t t[4], b[4];
					load_side(ix, etop, st);
					load_side(ix, ebot, sb);
					count_all(ix, st, t);
					count_all(ix, sb, b);
					int nonz = -1; bool abort_ = false;
					const uint64_t orig = ebot - etop;
#pragma unroll
					for(int j = 0; j < 4; j++) {
						if(!abort_ && b[j] > t[j]) {
							if(nonz >= 0) abort_ = true;
							else { nonz = j; etop = t[j]; ebot = b[j]; }
						}
					}
					if(abort_ || (nonz != rdc && rdc <= 3) || ebot - etop < orig) break;
				} else {
					n_lf1++;
					int c = -1;
					if(etop != ix.zoff) {
						load_side(ix, etop, st);
						c = row_l(st);
						etop = count_one(ix, st, c);
					}
					if(c != rdc && rdc <= 3) break;
					ebot = etop + 1;
				}
				if(++nlex == 255) break;
			}
		}
		bt2x_seed_out o;
		o.topf = top; o.botf = bot; o.nlex = (uint8_t)nlex; o.need_reporting = report ? 1 : 0;
#pragma unroll
		for(int k = 0; k < 6; k++) o.pad[k] = 0;
		out[i] = o;
	}
	if(ctr) {
		// wave-level reduction, one atomic per wave per counter
		for(int d = 32; d > 0; d >>= 1) {
			n_bilf += __shfl_xor(n_bilf, d);
			n_lf1 += __shfl_xor(n_lf1, d);
			n_ftab += __shfl_xor(n_ftab, d);
		}
		if((threadIdx.x & 63) == 0) {
			atomicAdd(&ctr[0], (unsigned long long)n_bilf);
			atomicAdd(&ctr[1], (unsigned long long)n_lf1);
			atomicAdd(&ctr[2], (unsigned long long)n_ftab);
		}
	}
}

} // namespace

int bt2x_launch_seed(const DevIndex& ix, const uint8_t* d_reads, const bt2x_seed_in* d_in,
                     uint32_t n, int do_extend, bt2x_seed_out* d_out,
                     unsigned long long* d_ctr, void* stream) {
	if(n == 0) return 0;
	const uint32_t blocks = (n + 255) / 256;
	hipLaunchKernelGGL(seed_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
	                   ix, d_reads, d_in, n, do_extend, d_out, d_ctr);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
