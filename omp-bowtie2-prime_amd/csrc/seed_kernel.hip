// seed_kernel.hip — batched exact seed search + left extension on gfx950.
//
// Replaces MultiSeedAligner::searchAllSeedsDoAll(doExtend) (aligner_seed.cpp:674-725):
// searchSeedBi<8> (:820-957, startSearchSeedBi :757-811) then MultiSeedAligner::extend
// (:603-672) for every reported seed.
//
// MI355X design: a persistent grid whose lanes are independent work loops.  Each lane
// owns one seed at a time and advances it by ONE LF step per loop iteration, whether the
// seed is in its exact search or its left extension; a lane whose seed finishes writes
// the result and takes the next seed (grid-stride) at once.  So a wave's cost is the
// mean per-seed LF chain of its 64 lanes' streams, not the maximum, and search and
// extension share one instruction stream (no divergence between the two phases).
//
// Every LF step is the same computation for a range step (mapBiLFEx, bt2_idx.h:2474)
// and a single-row step (mapLF1, :2511-2542): the occurrence counts of ONE character c
// at the range's two ends.  For a one-row range [top, top+1) the second count comes from
// the same side (the match bit at top), and a step that empties the range is exactly the
// reference's `rowL != c || row == zOff` failure.  Only extension steps over a read N
// (rdc = 4) need all four characters; they take a rare slow path.
//
// A side is 128 B (one L2 line; 96 B of 2-bit BWT + 4 x u64 occ).  The count of c in
// [0, charOff) of a side (Ebwt::countBt2Side, bt2_idx.h:1811-1846) is computed over its
// 24 dwords with bit-pair matches + v_bcnt, predicated by dword index, no scratch.
// Algorithmic bytes per launch = 128*(2*n_mapBiLFEx + n_mapLF1) + 16*n_ftab.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"

#define OFF_MASK 0xffffffffffffffffULL

namespace {

struct Side {
	uint32_t w[24];          // 96 B of packed BWT, constant indices only
	uint64_t occ[4];         // occ[A,C,G,T] at the side start
};

__device__ __forceinline__ void load_side(const DevIndex& ix, uint64_t side, Side& s) {
	const uint4* p = reinterpret_cast<const uint4*>(ix.ebwt + side * BT2X_SIDE_BYTES);
#pragma unroll
	for(int k = 0; k < 6; k++) {
		const uint4 v = p[k];
		s.w[4 * k] = v.x; s.w[4 * k + 1] = v.y; s.w[4 * k + 2] = v.z; s.w[4 * k + 3] = v.w;
	}
	const uint4 v6 = p[6], v7 = p[7];
	s.occ[0] = ((uint64_t)v6.y << 32) | v6.x;
	s.occ[1] = ((uint64_t)v6.w << 32) | v6.z;
	s.occ[2] = ((uint64_t)v7.y << 32) | v7.x;
	s.occ[3] = ((uint64_t)v7.w << 32) | v7.z;
}

// Bit-pair matches of character c in a dword, on the low bit of each pair
// (countInU64, bt2_idx.h:519-537): pairs equal to c become 00 after xor with c*0x5555.
__device__ __forceinline__ uint32_t match_c(uint32_t w, uint32_t pat) {
	const uint32_t x = w ^ pat;
	return ~(x | (x >> 1)) & 0x55555555u;
}

__device__ __forceinline__ uint64_t sel4(const uint64_t v[4], int c) {
	const uint64_t lo = (c & 1) ? v[1] : v[0];
	const uint64_t hi = (c & 1) ? v[3] : v[2];
	return (c & 2) ? hi : lo;
}

// Counts of c in [0, offa) and [0, offb) of one side (offb <= 384; offb = offa + 1 gives
// the one-row step).  Per dword: prefix length s = clamp(2*off - 32*d, 0, 31) bits, and
// v_bfe(m, 0, s) keeps the matches below the offset (match bits sit on even positions,
// so 31 bits cover a full dword).  No lane-mask compares, hence no SGPR pressure.
__device__ __forceinline__ void count_side(const Side& s, uint32_t c, int offa, int offb,
                                           uint32_t& ca, uint32_t& cb) {
	const uint32_t pat = c * 0x55555555u;
	ca = 0; cb = 0;
#pragma unroll
	for(int d = 0; d < 24; d++) {
		const uint32_t m = match_c(s.w[d], pat);
		const uint32_t wa = (uint32_t)min(max(2 * offa - 32 * d, 0), 31);
		const uint32_t wb = (uint32_t)min(max(2 * offb - 32 * d, 0), 31);
		ca += __popc(__builtin_amdgcn_ubfe(m, 0u, wa));
		cb += __popc(__builtin_amdgcn_ubfe(m, 0u, wb));
	}
}

// ---- device block layout: 64 B per 192 rows, one HBM burst per LF step ---------------
// A block is half a .bt2l side with the side's occ[] advanced to its own start, stored
// as u32 (texts < 2^32 rows), so an LF step counts at most 11 dwords instead of 23 and
// reads 64 bytes instead of 128.  Counts are identical to countBt2Side's.
struct Blk {
	uint32_t occ[4];
	uint32_t w[12];
};

__device__ __forceinline__ void load_blk(const DevIndex& ix, uint64_t b, Blk& k) {
	const uint4* p = reinterpret_cast<const uint4*>(ix.blk + b * BT2X_BLK_BYTES);
	const uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
	k.occ[0] = v0.x; k.occ[1] = v0.y; k.occ[2] = v0.z; k.occ[3] = v0.w;
	k.w[0] = v1.x; k.w[1] = v1.y; k.w[2] = v1.z; k.w[3] = v1.w;
	k.w[4] = v2.x; k.w[5] = v2.y; k.w[6] = v2.z; k.w[7] = v2.w;
	k.w[8] = v3.x; k.w[9] = v3.y; k.w[10] = v3.z; k.w[11] = v3.w;
}

__device__ __forceinline__ void count_blk(const Blk& k, uint32_t c, int offa, int offb,
                                          uint32_t& ca, uint32_t& cb) {
	const uint32_t pat = c * 0x55555555u;
	ca = 0; cb = 0;
#pragma unroll
	for(int d = 0; d < 12; d++) {
		const uint32_t m = match_c(k.w[d], pat);
		const uint32_t wa = (uint32_t)min(max(2 * offa - 32 * d, 0), 31);
		const uint32_t wb = (uint32_t)min(max(2 * offb - 32 * d, 0), 31);
		ca += __popc(__builtin_amdgcn_ubfe(m, 0u, wa));
		cb += __popc(__builtin_amdgcn_ubfe(m, 0u, wb));
	}
}

__device__ __forceinline__ uint32_t sel4u(const uint32_t v[4], int c) {
	const uint32_t lo = (c & 1) ? v[1] : v[0];
	const uint32_t hi = (c & 1) ? v[3] : v[2];
	return (c & 2) ? hi : lo;
}

__device__ __forceinline__ uint64_t ftab_hi(const DevIndex& ix, uint64_t i) {
	const uint64_t v = ix.ftab[i];
	return v <= ix.len ? v : ix.eftab[(v ^ OFF_MASK) * 2 + 1];
}
__device__ __forceinline__ uint64_t ftab_lo(const DevIndex& ix, uint64_t i) {
	const uint64_t v = ix.ftab[i];
	return v <= ix.len ? v : ix.eftab[(v ^ OFF_MASK) * 2];
}

__device__ __forceinline__ uint64_t fchr_sel(const DevIndex& ix, int c) {
	return c == 0 ? ix.fchr[0] : c == 1 ? ix.fchr[1] : c == 2 ? ix.fchr[2] : c == 3 ? ix.fchr[3] : ix.fchr[4];
}

enum { PH_START = 0, PH_SEARCH = 1, PH_EXTEND = 2, PH_EXIT = 3 };

// One LF step of character c (0..3) over the range [ra, rb) (rb = ra + 1 for a single
// row): the new range [na, nb).  '$' (row zOff, stored as A) is never counted.
__device__ __forceinline__ void lf_step(const DevIndex& ix, uint64_t ra, uint64_t rb, uint32_t c,
                                        bool one_row, uint64_t& na, uint64_t& nb) {
	const uint64_t sa = ra / BT2X_SIDE_CHARS, sb = rb / BT2X_SIDE_CHARS;
	const int offa = (int)(ra - sa * BT2X_SIDE_CHARS);
	const bool same = one_row || sb == sa;
	// a one-row range counts [0, offa+1) of the same side (offa+1 may be 384)
	const int offb = same ? (int)(rb - sa * BT2X_SIDE_CHARS) : (int)(rb - sb * BT2X_SIDE_CHARS);
	const uint64_t zs = ix.zoff / BT2X_SIDE_CHARS;
	const int zo = (int)(ix.zoff - zs * BT2X_SIDE_CHARS);
	const uint64_t fc = fchr_sel(ix, (int)c);
	Side s;
	load_side(ix, sa, s);
	uint32_t ka, kb;
	count_side(s, c, offa, same ? offb : offa, ka, kb);
	// A-count adjustment for '$' (row zOff, stored as A) before the offset in this side
	// (countBt2Side, bt2_idx.h:1824-1833)
	const uint32_t dla = (c == 0 && sa == zs && zo < offa) ? 1u : 0u;
	const uint64_t base = sel4(s.occ, (int)c) + fc;
	na = base + (ka - dla);
	if(same) {
		const uint32_t dlb = (c == 0 && sa == zs && zo < offb) ? 1u : 0u;
		nb = base + (kb - dlb);
	} else {
		Side t;
		load_side(ix, sb, t);
		uint32_t kt, kt2;
		count_side(t, c, offb, offb, kt, kt2);
		const uint32_t dlb = (c == 0 && sb == zs && zo < offb) ? 1u : 0u;
		nb = sel4(t.occ, (int)c) + fc + (kt - dlb);
	}
}

// LF step over the block layout, 32-bit rows (texts < 2^32 rows; same contract as lf_step).
__device__ __forceinline__ void lf_step_blk32(const DevIndex& ix, uint32_t ra, uint32_t rb, uint32_t c,
                                              bool one_row, uint32_t& na, uint32_t& nb) {
	const uint32_t ba = ra / BT2X_BLK_ROWS, bb = rb / BT2X_BLK_ROWS;
	const int offa = (int)(ra - ba * BT2X_BLK_ROWS);
	const bool same = one_row || bb == ba;
	const int offb = same ? (int)(rb - ba * BT2X_BLK_ROWS) : (int)(rb - bb * BT2X_BLK_ROWS);
	const uint32_t zoff = (uint32_t)ix.zoff;
	const uint32_t zb = zoff / BT2X_BLK_ROWS;
	const int zo = (int)(zoff - zb * BT2X_BLK_ROWS);
	const uint32_t fc = (uint32_t)fchr_sel(ix, (int)c);
	Blk k;
	load_blk(ix, ba, k);
	uint32_t ka, kb;
	count_blk(k, c, offa, same ? offb : offa, ka, kb);
	const uint32_t dla = (c == 0 && ba == zb && zo < offa) ? 1u : 0u;
	const uint32_t base = sel4u(k.occ, (int)c) + fc;
	na = base + ka - dla;
	if(same) {
		const uint32_t dlb = (c == 0 && ba == zb && zo < offb) ? 1u : 0u;
		nb = base + kb - dlb;
	} else {
		Blk t;
		load_blk(ix, bb, t);
		uint32_t kt, kt2;
		count_blk(t, c, offb, offb, kt, kt2);
		const uint32_t dlb = (c == 0 && bb == zb && zo < offb) ? 1u : 0u;
		nb = sel4u(t.occ, (int)c) + fc + kt - dlb;
	}
}

// LF step over the block layout (same contract as lf_step).
__device__ __forceinline__ void lf_step_blk(const DevIndex& ix, uint64_t ra, uint64_t rb, uint32_t c,
                                            bool one_row, uint64_t& na, uint64_t& nb) {
	const uint64_t ba = ra / BT2X_BLK_ROWS, bb = rb / BT2X_BLK_ROWS;
	const int offa = (int)(ra - ba * BT2X_BLK_ROWS);
	const bool same = one_row || bb == ba;
	const int offb = same ? (int)(rb - ba * BT2X_BLK_ROWS) : (int)(rb - bb * BT2X_BLK_ROWS);
	const uint64_t zb = ix.zoff / BT2X_BLK_ROWS;
	const int zo = (int)(ix.zoff - zb * BT2X_BLK_ROWS);
	const uint64_t fc = fchr_sel(ix, (int)c);
	Blk k;
	load_blk(ix, ba, k);
	uint32_t ka, kb;
	count_blk(k, c, offa, same ? offb : offa, ka, kb);
	const uint32_t dla = (c == 0 && ba == zb && zo < offa) ? 1u : 0u;
	const uint64_t base = (uint64_t)sel4u(k.occ, (int)c) + fc;
	na = base + (ka - dla);
	if(same) {
		const uint32_t dlb = (c == 0 && ba == zb && zo < offb) ? 1u : 0u;
		nb = base + (kb - dlb);
	} else {
		Blk t;
		load_blk(ix, bb, t);
		uint32_t kt, kt2;
		count_blk(t, c, offb, offb, kt, kt2);
		const uint32_t dlb = (c == 0 && bb == zb && zo < offb) ? 1u : 0u;
		nb = (uint64_t)sel4u(t.occ, (int)c) + fc + (kt - dlb);
	}
}

template<bool kBlk>
__global__ void __launch_bounds__(256, 4)
seed_kernel(DevIndex ix, const uint8_t* __restrict__ reads, const bt2x_seed_in* __restrict__ in,
            uint32_t n, int do_extend, bt2x_seed_out* __restrict__ out,
            unsigned long long* __restrict__ ctr) {
	const uint32_t stride = gridDim.x * blockDim.x;
	uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t n_bilf = 0, n_lf1 = 0, n_ftab = 0;
	int phase = PH_START;
	const uint8_t* seq = nullptr;
	int nsteps = 0, step = 0, lim = 0, ii = 0, nlex = 0;
	uint64_t top = 0, bot = 0, etop = 0, ebot = 0, ntop = 0, nbot = 0;
	int kk = 0, nz = 0;
	bool report = false;
	const int fc = ix.ftab_chars;
	while(true) {
		bool fin = false;
		if(phase == PH_START) {
			if(idx >= n) {
				phase = PH_EXIT;
			} else {
				const bt2x_seed_in p = in[idx];
				seq = reads + p.read_off + p.seed_off;
				nsteps = p.seed_len;
				lim = do_extend ? p.seed_off : 0;
				ii = 0; nlex = 0; report = false;
				const int off = nsteps - 1;
				// startSearchSeedBi: ftab jump over the rightmost ftabChars characters
				if(fc > 1 && fc <= nsteps) {
					uint64_t fi = 0;
					for(int k = 0; k < fc; k++) fi = (fi << 2) | (uint64_t)(seq[off - fc + 1 + k] & 3);
					top = ftab_hi(ix, fi);
					bot = ftab_lo(ix, fi + 1);
					n_ftab++;
					step = fc;
				} else {
					const int c = seq[off];
					top = fchr_sel(ix, c); bot = fchr_sel(ix, c + 1);
					step = 1;
				}
				if(bot == top) fin = true;
				else if(step == nsteps) { report = true; fin = lim == 0; phase = PH_EXTEND; etop = top; ebot = bot; }
				else phase = PH_SEARCH;
			}
		} else if(phase != PH_EXIT) {
			const bool ext = phase == PH_EXTEND;
			const uint64_t ra = ext ? etop : top, rb = ext ? ebot : bot;
			const bool one = rb - ra == 1;
			const int c = ext ? seq[-1 - ii] : seq[nsteps - step - 1];
			if(kk == 0) { if(one) n_lf1 += (!ext && c == 4) ? 0u : 1u; else n_bilf++; }
			if(!ext && c == 4) {
				fin = true;                       // N in the seed: searchSeedBi drops it
			} else {
				// extension over a read N visits the four characters in four iterations
				const bool nslow = c == 4;
				uint64_t na, nb;
				if(kBlk) lf_step_blk(ix, ra, rb, nslow ? (uint32_t)kk : (uint32_t)c, one, na, nb);
				else lf_step(ix, ra, rb, nslow ? (uint32_t)kk : (uint32_t)c, one, na, nb);
				if(!ext) {
					// searchSeedBi: an empty range ends the search unreported
					if(nb == na) fin = true;
					else {
						top = na; bot = nb; step++;
						if(step == nsteps) { report = true; etop = top; ebot = bot; phase = PH_EXTEND; fin = lim == 0; }
					}
				} else if(!nslow) {
					// extend(): the step survives iff the range keeps its size under rdc
					if(nb - na != rb - ra) fin = true;
					else { etop = na; ebot = nb; ii++; nlex++; fin = (nlex == 255) || (ii == lim); }
				} else {
					// read N: the unique non-empty character continues, a one-row range
					// follows rowL and zOff keeps its row (aligner_seed.cpp:636-660)
					if(nb > na) { nz++; if(nz == 1) { ntop = na; nbot = nb; } }
					if(++kk == 4) {
						if(nz == 0) { ntop = ra; nbot = one ? ra + 1 : rb; }
						else if(one) nbot = ntop + 1;
						if(nz > 1 || (!one && nbot - ntop < rb - ra)) fin = true;
						else { etop = ntop; ebot = nbot; ii++; nlex++; fin = (nlex == 255) || (ii == lim); }
						kk = 0; nz = 0;
					}
				}
			}
		}
		if(fin) {
			bt2x_seed_out o;
			o.topf = top; o.botf = bot; o.nlex = (uint8_t)nlex;
			o.need_reporting = report ? 1 : 0;
#pragma unroll
			for(int k = 0; k < 6; k++) o.pad[k] = 0;
			out[idx] = o;
			idx += stride;
			phase = PH_START;
		}
		if(__all(phase == PH_EXIT)) break;
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

// startSearchSeedBi for every seed (aligner_seed.cpp:757-811): the ftab jump over the
// rightmost ftabChars characters (or the fchr range of one character), in a pre-pass so
// its dependent read -> ftab -> eftab loads overlap across all seeds instead of stalling
// the LF loop.  State per seed in out[]: topf/botf = range, nlex = steps consumed,
// pad[0] = 0 continue, 1 empty (done, unreported), 2 matched (report, then extend).
__global__ void __launch_bounds__(256)
seed_init_kernel(DevIndex ix, const uint8_t* __restrict__ reads, const bt2x_seed_in* __restrict__ in,
                 uint32_t n, bt2x_seed_out* __restrict__ out, unsigned long long* __restrict__ ctr) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t n_ftab = 0;
	if(i < n) {
		const bt2x_seed_in p = in[i];
		const uint8_t* seq = reads + p.read_off + p.seed_off;
		const int nsteps = p.seed_len, off = nsteps - 1, fc = ix.ftab_chars;
		uint64_t top, bot;
		int step;
		if(fc > 1 && fc <= nsteps) {
			uint64_t fi = 0;
			for(int k = 0; k < fc; k++) fi = (fi << 2) | (uint64_t)(seq[off - fc + 1 + k] & 3);
			top = ftab_hi(ix, fi);
			bot = ftab_lo(ix, fi + 1);
			n_ftab = 1;
			step = fc;
		} else {
			const int c = seq[off];
			top = fchr_sel(ix, c); bot = fchr_sel(ix, c + 1);
			step = 1;
		}
		bt2x_seed_out o;
		o.topf = top; o.botf = bot; o.nlex = (uint8_t)step; o.need_reporting = 0;
#pragma unroll
		for(int k = 0; k < 6; k++) o.pad[k] = 0;
		o.pad[0] = bot == top ? 1 : (step == nsteps ? 2 : 0);
		out[i] = o;
	}
	if(ctr) {
		for(int d = 32; d > 0; d >>= 1) n_ftab += __shfl_xor(n_ftab, d);
		if((threadIdx.x & 63) == 0) atomicAdd(&ctr[2], (unsigned long long)n_ftab);
	}
}

// The LF loop over the block layout with 32-bit rows.  kInit: the ftab start was done
// by seed_init_kernel (state in out[]); otherwise the START phase does it inline.
template<bool kInit>
__global__ void __launch_bounds__(256, 4)
seed_kernel_blk(DevIndex ix, const uint8_t* __restrict__ reads, const bt2x_seed_in* __restrict__ in,
                uint32_t n, int do_extend, bt2x_seed_out* __restrict__ out,
                unsigned long long* __restrict__ ctr) {
	const uint32_t stride = gridDim.x * blockDim.x;
	uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t n_bilf = 0, n_lf1 = 0, n_ftab = 0;
	int phase = PH_START;
	const uint8_t* seq = nullptr;
	int nsteps = 0, step = 0, lim = 0, ii = 0, nlex = 0;
	uint32_t top = 0, bot = 0, etop = 0, ebot = 0, ntop = 0, nbot = 0, tp = 0;
	int kk = 0, nz = 0;
	bool report = false, tmode = false;
	while(true) {
		bool fin = false;
		if(phase == PH_START) {
			if(idx >= n) {
				phase = PH_EXIT;
			} else {
				const bt2x_seed_in p = in[idx];
				seq = reads + p.read_off + p.seed_off;
				nsteps = p.seed_len;
				lim = do_extend ? p.seed_off : 0;
				ii = 0; nlex = 0;
				int st0;
				if(kInit) {
					const bt2x_seed_out s0 = out[idx];
					top = (uint32_t)s0.topf; bot = (uint32_t)s0.botf; step = s0.nlex; st0 = s0.pad[0];
				} else {
					// startSearchSeedBi: ftab jump over the rightmost ftabChars characters
					const int off = nsteps - 1, fc = ix.ftab_chars;
					if(fc > 1 && fc <= nsteps) {
						uint64_t fi = 0;
						for(int k = 0; k < fc; k++) fi = (fi << 2) | (uint64_t)(seq[off - fc + 1 + k] & 3);
						top = (uint32_t)ftab_hi(ix, fi);
						bot = (uint32_t)ftab_lo(ix, fi + 1);
						n_ftab++;
						step = fc;
					} else {
						const int c = seq[off];
						top = (uint32_t)fchr_sel(ix, c); bot = (uint32_t)fchr_sel(ix, c + 1);
						step = 1;
					}
					st0 = bot == top ? 1 : (step == nsteps ? 2 : 0);
				}
				report = st0 == 2;
				tmode = false;
				if(st0 == 1) fin = true;
				else if(report) { etop = top; ebot = bot; phase = PH_EXTEND; fin = lim == 0; }
				else phase = PH_SEARCH;
				if(phase == PH_EXTEND && !fin && ix.sa && ebot - etop == 1) { tmode = true; tp = ix.sa[etop]; }
			}
		} else if(phase == PH_EXTEND && tmode) {
			// extend() over a one-row range in text terms: row etop is the suffix at text
			// position tp, its LF step reads text[tp-1]; up to 16 steps per iteration.
			// Same outcomes as the LF1 walk: a read N matches anything, text position 0
			// (row zOff) keeps its row and only read Ns pass it (aligner_seed.cpp:655-664).
			const int cap = min(lim, 255);
			const uint32_t hi = tp > 0 ? (tp - 1) >> 4 : 0;
			const uint32_t whi = tp > 0 ? ix.text[hi] : 0u, wlo = hi > 0 ? ix.text[hi - 1] : 0u;
			bool stop = false;
#pragma unroll
			for(int j = 0; j < 16; j++) {
				if(!stop && ii < cap) {
					const int rdc = seq[-1 - ii];
					n_lf1++;
					if(tp == 0) {
						if(rdc <= 3) stop = true; else { ii++; nlex++; }
					} else {
						const uint32_t pos = tp - 1;
						const uint32_t w = (pos >> 4) == hi ? whi : wlo;
						const int t = (int)((w >> (2 * (pos & 15))) & 3u);
						if(rdc <= 3 && t != rdc) stop = true; else { tp--; ii++; nlex++; }
					}
				}
			}
			fin = stop || ii == lim || nlex == 255;
		} else if(phase != PH_EXIT) {
			const bool ext = phase == PH_EXTEND;
			const uint32_t ra = ext ? etop : top, rb = ext ? ebot : bot;
			const bool one = rb - ra == 1;
			const int c = ext ? seq[-1 - ii] : seq[nsteps - step - 1];
			if(kk == 0) { if(one) n_lf1 += (!ext && c == 4) ? 0u : 1u; else n_bilf++; }
			if(!ext && c == 4) {
				fin = true;                       // N in the seed: searchSeedBi drops it
			} else {
				const bool nslow = c == 4;
				uint32_t na, nb;
				lf_step_blk32(ix, ra, rb, nslow ? (uint32_t)kk : (uint32_t)c, one, na, nb);
				if(!ext) {
					if(nb == na) fin = true;
					else {
						top = na; bot = nb; step++;
						if(step == nsteps) {
							report = true; etop = top; ebot = bot; phase = PH_EXTEND; fin = lim == 0;
							if(!fin && ix.sa && ebot - etop == 1) { tmode = true; tp = ix.sa[etop]; }
						}
					}
				} else if(!nslow) {
					if(nb - na != rb - ra) fin = true;
					else { etop = na; ebot = nb; ii++; nlex++; fin = (nlex == 255) || (ii == lim); }
				} else {
					if(nb > na) { nz++; if(nz == 1) { ntop = na; nbot = nb; } }
					if(++kk == 4) {
						if(nz == 0) { ntop = ra; nbot = one ? ra + 1 : rb; }
						else if(one) nbot = ntop + 1;
						if(nz > 1 || (!one && nbot - ntop < rb - ra)) fin = true;
						else { etop = ntop; ebot = nbot; ii++; nlex++; fin = (nlex == 255) || (ii == lim); }
						kk = 0; nz = 0;
					}
				}
			}
		}
		if(fin) {
			bt2x_seed_out o;
			o.topf = top; o.botf = bot; o.nlex = (uint8_t)nlex;
			o.need_reporting = report ? 1 : 0;
#pragma unroll
			for(int k = 0; k < 6; k++) o.pad[k] = 0;
			out[idx] = o;
			idx += stride;
			phase = PH_START;
		}
		if(__all(phase == PH_EXIT)) break;
	}
	if(ctr) {
		for(int d = 32; d > 0; d >>= 1) {
			n_bilf += __shfl_xor(n_bilf, d);
			n_lf1 += __shfl_xor(n_lf1, d);
			n_ftab += __shfl_xor(n_ftab, d);
		}
		if((threadIdx.x & 63) == 0) {
			atomicAdd(&ctr[0], (unsigned long long)n_bilf);
			atomicAdd(&ctr[1], (unsigned long long)n_lf1);
			if(!kInit) atomicAdd(&ctr[2], (unsigned long long)n_ftab);
		}
	}
}

// BWT character of row r (the block's 2-bit code; row zOff holds '$' stored as A).
__device__ __forceinline__ uint32_t row_l_blk32(const DevIndex& ix, uint32_t r) {
	const uint32_t b = r / BT2X_BLK_ROWS, off = r - b * BT2X_BLK_ROWS;
	Blk k;
	load_blk(ix, b, k);
	const uint32_t q = off >> 4;
	uint32_t w = 0;
#pragma unroll
	for(int d = 0; d < 12; d++) w = ((uint32_t)d == q) ? k.w[d] : w;
	return (w >> (2 * (off & 15))) & 3u;
}

// Full suffix array from the SA sample (Ebwt::_offs, rows r with r % 2^offRate == 0):
// from each sampled row walk LF (text position - 1 per step) until the next sampled row;
// the LF cycle visits every row once, so every row is written exactly once.  LF of zOff
// (text position 0) wraps to the '$' row len (position len).
__global__ void __launch_bounds__(256)
sa_fill_kernel(DevIndex ix, const uint64_t* __restrict__ offs, uint64_t noffs, uint32_t* __restrict__ sa) {
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= noffs) return;
	const uint32_t len = (uint32_t)ix.len, zoff = (uint32_t)ix.zoff;
	const uint32_t mask = (1u << ix.off_rate) - 1u;
	uint32_t r = (uint32_t)(i << ix.off_rate);
	if(r > len) return;
	uint32_t p = (uint32_t)offs[i];
	for(uint32_t guard = 0; guard <= len; guard++) {
		sa[r] = p;
		uint32_t rn;
		if(r == zoff) { rn = len; p = len; }
		else {
			const uint32_t c = row_l_blk32(ix, r);
			uint32_t na, nb;
			lf_step_blk32(ix, r, r + 1, c, true, na, nb);
			rn = na; p = p - 1;
		}
		if((rn & mask) == 0) break;                // sampled: written by its own thread
		r = rn;
	}
}

// Block b = half h of side s = b/2: its 48 BWT bytes, and occ[] at its start = the side's
// occ[] plus (for h = 1) the counts over the side's first 192 rows, '$' excluded.
__global__ void __launch_bounds__(256)
build_blocks_kernel(DevIndex ix, uint64_t nsides, uint8_t* __restrict__ blk) {
	const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if(b >= 2 * nsides) return;
	const uint64_t side = b >> 1;
	const int h = (int)(b & 1);
	Side s;
	load_side(ix, side, s);
	uint32_t occ[4];
#pragma unroll
	for(int c = 0; c < 4; c++) {
		uint32_t n = 0;
		if(h) {
#pragma unroll
			for(int d = 0; d < 12; d++) n += __popc(match_c(s.w[d], (uint32_t)c * 0x55555555u));
		}
		occ[c] = (uint32_t)s.occ[c] + n;
	}
	const uint64_t zs = ix.zoff / BT2X_SIDE_CHARS;
	const uint64_t zc = ix.zoff - zs * BT2X_SIDE_CHARS;
	if(h && zs == side && zc < BT2X_BLK_ROWS) occ[0]--;      // '$' is stored as A
	uint4* o = reinterpret_cast<uint4*>(blk + b * BT2X_BLK_BYTES);
	o[0] = make_uint4(occ[0], occ[1], occ[2], occ[3]);
	uint32_t w[12];
#pragma unroll
	for(int d = 0; d < 12; d++) w[d] = h ? s.w[12 + d] : s.w[d];
	o[1] = make_uint4(w[0], w[1], w[2], w[3]);
	o[2] = make_uint4(w[4], w[5], w[6], w[7]);
	o[3] = make_uint4(w[8], w[9], w[10], w[11]);
}

// ---- SA resolution (GroupWalk2S::advanceElement + Ebwt::joinedToTextOff) ----------

// BWT character of row r over the 64-bit block / side layouts.
__device__ __forceinline__ uint32_t row_l_any(const DevIndex& ix, uint64_t r) {
	if(ix.blk) {
		const uint64_t b = r / BT2X_BLK_ROWS, off = r - b * BT2X_BLK_ROWS;
		const uint8_t by = ix.blk[b * BT2X_BLK_BYTES + 16 + (off >> 2)];
		return (by >> (2 * (off & 3))) & 3u;
	}
	const uint64_t s = r / BT2X_SIDE_CHARS, off = r - s * BT2X_SIDE_CHARS;
	const uint8_t by = ix.ebwt[s * BT2X_SIDE_BYTES + (off >> 2)];
	return (by >> (2 * (off & 3))) & 3u;
}

// Ebwt::getOffset (bt2_idx.cpp:150-174), the value GWState's walk produces
// (group_walk.h:425-432): the resident SA when there is one, else LF to the sample.
__device__ __forceinline__ uint64_t sa_offset(const DevIndex& ix, uint64_t row, uint32_t& steps) {
	steps = 0;
	if(ix.sa) return ix.sa[row];
	const uint64_t mask = (1ULL << ix.off_rate) - 1ULL;
	uint64_t jumps = 0;
	for(int guard = 0; guard < (1 << 16); guard++) {
		if(row == ix.zoff) return jumps;
		if((row & mask) == 0) return jumps + ix.offs[row >> ix.off_rate];
		const uint32_t c = row_l_any(ix, row);
		uint64_t na, nb;
		if(ix.blk) lf_step_blk(ix, row, row + 1, c, true, na, nb);
		else lf_step(ix, row, row + 1, c, true, na, nb);
		row = na; jumps++; steps++;
	}
	return OFF_MASK;
}

// One element: Ebwt::getOffset + joinedToTextOff.
__device__ __forceinline__ bt2x_resolve_out resolve_one(const DevIndex& ix, const bt2x_resolve_in e, int reject,
                                                       uint32_t& steps) {
		bt2x_resolve_out o;
		o.joff = e.row <= ix.len ? sa_offset(ix, e.row, steps) : OFF_MASK;
		o.toff = 0; o.tlen = 0; o.tidx = BT2X_NO_TIDX; o.straddled = 0;
		// joinedToTextOff's binary search over rstarts (bt2_idx.cpp:62-121), same probe
		// order; bounded so an offset in no fragment ('$' suffix) ends with BT2X_NO_TIDX
		const uint64_t off = o.joff;
		uint64_t top = 0, bot = ix.nfrag;
		for(int it = 0; it < 70 && off < ix.len && ix.nfrag > 0; it++) {
			const uint64_t elt = top + ((bot - top) >> 1);
			const uint64_t lower = ix.rstarts[elt * 3];
			const uint64_t upper = elt == ix.nfrag - 1 ? ix.len : ix.rstarts[(elt + 1) * 3];
			if(lower <= off) {
				if(upper > off) {
					const bool st = off + e.qlen > upper;
					o.straddled = st ? 1u : 0u;
					if(!(st && reject)) {
						o.tidx = (uint32_t)ix.rstarts[elt * 3 + 1];
						o.toff = off - lower + ix.rstarts[elt * 3 + 2];   // fw index: no flip
						o.tlen = ix.plen[o.tidx];
					}
					break;
				}
				top = elt;
			} else {
				bot = elt;
			}
		}
		return o;
}

__global__ void __launch_bounds__(256)
sa_resolve_kernel(DevIndex ix, const bt2x_resolve_in* __restrict__ in, uint32_t n, int reject,
                  bt2x_resolve_out* __restrict__ out, unsigned long long* __restrict__ ctr) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t steps = 0;
	if(i < n) out[i] = resolve_one(ix, in[i], reject, steps);
	if(ctr) {
		// LF steps of this wave, one atomic per wave
		uint64_t s = steps;
		for(int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k);
		if((threadIdx.x & 63) == 0 && s) atomicAdd(&ctr[1], (unsigned long long)s);
	}
}

// The same over a count that lives in HBM (written by the kernel that produced the
// elements), grid-stride; at most cap elements.  Out: bt2x_resolve_out, or the seed
// round's 8-byte bt2x_elt.
__device__ __forceinline__ void put_elt(bt2x_resolve_out* out, uint32_t i, const bt2x_resolve_out& o) { out[i] = o; }
__device__ __forceinline__ void put_elt(bt2x_elt* out, uint32_t i, const bt2x_resolve_out& o) {
	// bt2x_elt_pack's layout (bt2x.h): toff bits 0-38, straddled bit 39, tidx bits 40-63
	const uint64_t t = o.tidx == BT2X_NO_TIDX ? BT2X_ELT_TIDX_NONE : (o.tidx & BT2X_ELT_TIDX_NONE);
	bt2x_elt e;
	e.v = (o.toff & ((1ull << 39) - 1)) | ((uint64_t)(o.straddled & 1u) << 39) | (t << 40);
	out[i] = e;
}

template<class Out>
__global__ void __launch_bounds__(256)
sa_resolve_kernel_dn(DevIndex ix, const bt2x_resolve_in* __restrict__ in, const uint32_t* __restrict__ d_n,
                     uint32_t cap, int reject, Out* __restrict__ out, unsigned long long* __restrict__ ctr) {
	const uint32_t n = min(*d_n, cap);
	uint32_t steps = 0;
	for(uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
		put_elt(out, i, resolve_one(ix, in[i], reject, steps));
	if(ctr) {
		uint64_t s = steps;
		for(int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k);
		if((threadIdx.x & 63) == 0 && s) atomicAdd(&ctr[1], (unsigned long long)s);
	}
}

} // namespace

int bt2x_build_sa(const DevIndex& ix, const uint64_t* d_offs, uint64_t noffs, uint32_t* d_sa, void* stream) {
	if(noffs == 0 || !ix.blk) return BT2X_E_ARG;
	hipLaunchKernelGGL(sa_fill_kernel, dim3((unsigned)((noffs + 255) / 256)), dim3(256), 0,
	                   (hipStream_t)stream, ix, d_offs, noffs, d_sa);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}

int bt2x_build_blocks(const DevIndex& ix, uint64_t nsides, uint8_t* d_blk, void* stream) {
	const uint64_t nb = 2 * nsides;
	if(nb == 0) return 0;
	hipLaunchKernelGGL(build_blocks_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
	                   (hipStream_t)stream, ix, nsides, d_blk);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}

// Resident 256-thread blocks per CU for the persistent seed grid.
static int seed_blocks_per_cu(bool blk) {
	static int nb[2] = {0, 0};
	if(nb[blk] == 0) {
		int v = 0;
		const void* fn = blk ? (const void*)seed_kernel_blk<false> : (const void*)seed_kernel<false>;
		if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, fn, 256, 0) != hipSuccess || v < 1) v = 2;
		nb[blk] = v;
	}
	return nb[blk];
}

namespace {
// MultiSeedResults::instantiateSeeds (aligner_seed.cpp:411-447) as the host driver runs it
// (bt2x_align.cpp align_read): per strand (patFw, then patRc) the seeds at depth
// i * interval + offset, i < num_offs -- a patRc seed at rdlen - depth - L -- skipping a
// seed over an N.  One lane per read; never past the read's nseeds slots.  The caller's
// nseeds is checked, not trusted: a read whose instantiated count differs bumps *bad (the
// entry point then refuses the round), and every slot of [seed0, seed0 + nseeds) it leaves
// unwritten gets an in-bounds stand-in (the read's first patFw seed position), so the seed
// search never reads a stale or uninitialised entry.
__global__ void __launch_bounds__(256) seed_gen_kernel(const uint8_t* __restrict__ reads,
                                                       const bt2x_round_in* __restrict__ in, uint32_t n,
                                                       bt2x_seed_in* __restrict__ seeds, uint32_t cap,
                                                       uint32_t* __restrict__ bad) {
	const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	if(r >= n) return;
	const bt2x_round_in q = in[r];
	const uint32_t L = q.seedlen, len = q.rdlen;
	uint64_t k = q.seed0;
	const uint64_t end = min((uint64_t)cap, q.seed0 + q.nseeds);
	uint32_t made = 0;
	for(int s = 0; s < 2; s++) {
		if(q.seedflags & (1u << s)) continue;
		const uint64_t ro = q.read_off + (s ? len : 0);
		for(uint32_t i = 0; i < q.num_offs; i++) {
			const uint32_t depth = i * q.interval + q.offset;
			const uint32_t st = s ? len - depth - L : depth;
			bool ok = true;
			for(uint32_t j = 0; j < L; j++) ok &= reads[ro + st + j] <= 3;
			if(!ok) continue;
			made++;
			if(k >= end) continue;
			bt2x_seed_in si;
			si.read_off = ro; si.seed_off = (uint8_t)st; si.seed_len = (uint8_t)L;
			for(int b = 0; b < 6; b++) si.pad[b] = 0;
			seeds[k++] = si;
		}
	}
	if(made != q.nseeds) atomicAdd(bad, 1u);
	for(; k < end; k++) {
		bt2x_seed_in si;
		si.read_off = q.read_off; si.seed_off = 0; si.seed_len = (uint8_t)L;
		for(int b = 0; b < 6; b++) si.pad[b] = 0;
		seeds[k] = si;
	}
}
} // namespace

int bt2x_launch_seed_gen(const uint8_t* d_reads, const bt2x_round_in* d_in, uint32_t nreads, bt2x_seed_in* d_seeds,
                         uint32_t nseeds, uint32_t* d_bad, void* stream) {
	if(nreads == 0) return 0;
	hipLaunchKernelGGL(seed_gen_kernel, dim3((nreads + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_reads, d_in, nreads,
	                   d_seeds, nseeds, d_bad);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}

int bt2x_launch_seed(const DevIndex& ix, const uint8_t* d_reads, const bt2x_seed_in* d_in,
                     uint32_t n, int do_extend, bt2x_seed_out* d_out,
                     unsigned long long* d_ctr, int ncu, void* stream) {
	if(n == 0) return 0;
	const bool blk = ix.blk != nullptr;
	uint32_t blocks = (uint32_t)(ncu > 0 ? ncu : 256) * (uint32_t)seed_blocks_per_cu(blk);
	const uint32_t need = (n + 255) / 256;
	if(blocks > need) blocks = need;
	if(blk) {
		static int init_pass = -1;
		if(init_pass < 0) { const char* e = getenv("BT2X_SEED_INIT_PASS"); init_pass = (e && e[0] == '1') ? 1 : 0; }
		if(init_pass) {
			hipLaunchKernelGGL(seed_init_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
			                   ix, d_reads, d_in, n, d_out, d_ctr);
			hipLaunchKernelGGL(seed_kernel_blk<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
			                   ix, d_reads, d_in, n, do_extend, d_out, d_ctr);
		} else {
			hipLaunchKernelGGL(seed_kernel_blk<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
			                   ix, d_reads, d_in, n, do_extend, d_out, d_ctr);
		}
	}
	else
		hipLaunchKernelGGL(seed_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
		                   ix, d_reads, d_in, n, do_extend, d_out, d_ctr);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}

namespace {
template<class Out>
int launch_resolve_dn(const DevIndex& ix, const bt2x_resolve_in* d_in, const uint32_t* d_n, uint32_t cap,
                      int reject, Out* d_out, unsigned long long* d_ctr, int ncu, void* stream) {
	if(cap == 0) return 0;
	if(!ix.sa && !ix.offs) return BT2X_E_ARG;
	uint32_t blocks = (uint32_t)(ncu > 0 ? ncu : 256) * 8u;
	if(blocks > (cap + 255) / 256) blocks = (cap + 255) / 256;
	hipLaunchKernelGGL(sa_resolve_kernel_dn<Out>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
	                   ix, d_in, d_n, cap, reject, d_out, d_ctr);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
}

int bt2x_launch_resolve_dn(const DevIndex& ix, const bt2x_resolve_in* d_in, const uint32_t* d_n, uint32_t cap,
                           int reject, bt2x_resolve_out* d_out, unsigned long long* d_ctr, int ncu, void* stream) {
	return launch_resolve_dn(ix, d_in, d_n, cap, reject, d_out, d_ctr, ncu, stream);
}

int bt2x_launch_resolve_dn(const DevIndex& ix, const bt2x_resolve_in* d_in, const uint32_t* d_n, uint32_t cap,
                           int reject, bt2x_elt* d_out, unsigned long long* d_ctr, int ncu, void* stream) {
	return launch_resolve_dn(ix, d_in, d_n, cap, reject, d_out, d_ctr, ncu, stream);
}

int bt2x_launch_resolve(const DevIndex& ix, const bt2x_resolve_in* d_in, uint32_t n, int reject,
                        bt2x_resolve_out* d_out, unsigned long long* d_ctr, void* stream) {
	if(n == 0) return 0;
	if(!ix.sa && !ix.offs) return BT2X_E_ARG;
	hipLaunchKernelGGL(sa_resolve_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
	                   ix, d_in, n, reject, d_out, d_ctr);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
