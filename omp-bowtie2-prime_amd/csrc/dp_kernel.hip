// dp_kernel.hip — end-to-end u8 DP fill + candidate extraction + full backtrace
// enumeration on gfx950, one DP problem per lane.
//
// Replaces SwAligner::align -> alignEnd2EndSseU8 (aligner_swsse_ee_u8.cpp:542-671:
// EEU8_alignOne / EEU8_lazyF / EEU8_alignNucleotides :249-536) and the loop of
// SwAligner::nextAlignment calls (aligner_sw.cpp:252-375) with
// backtraceNucleotidesEnd2EndSseU8 (u8.cpp:746-1352).
//
// Design (MI355X-first, not a Farrar port):
//  * One problem per lane, 64 problems per wave; the lane computes the exact saturating
//    u8 recurrence (no striping, no lazy-F loop: every value equals the striped kernel's,
//    SURVEY F9).
//  * The fill sweeps TWO columns at once, skewed by one row: step s computes cell
//    (s, j) in the low 16-bit half and cell (s-1, j+1) in the high half of every packed
//    operand, so each v_pk_{sub(clamp),max,min,mul}_u16 does two cells.  The high half's
//    inputs are the low half's outputs of the previous step (no extra state), and its
//    outputs replace row s-1 of the per-row state, which the low half has consumed.
//  * Per-row state (H and E of the previous column, 4 rows per dword) and a row-info
//    byte (read code, gap-barrier flag, quality mismatch penalty) live in VGPRs.
//  * Instead of materialising E/F/H (3 B/cell in the reference) the fill writes one
//    traceback byte per cell holding four "not equal" flags (d!=h, f!=h, hu_o!=f,
//    hl_o!=e): exactly what backtraceNucleotidesEnd2EndSseU8's fixed priority
//    (diag > H-up > F-up > H-left > E-left, E/F prefer the open; u8.cpp:843-990) needs
//    at a cell of value >= 1, and a backtrace only visits such cells, each at most once
//    (a revisit hits reportedThrough = bit 7 and fails).  Two steps' bytes of both
//    columns form one dword; each wave store is 256 contiguous bytes.
//  * Candidates (last-row cells with score >= minsc) are enumerated in DpBtCandidate
//    order (score desc, col desc; aligner_sw_nuc.h:149) and backtraced in-kernel; only
//    the final edit lists leave the GPU.
// Algorithmic bytes per problem = R*C (traceback bytes written) + C (reference window)
// + 2*R (read codes + qualities) — SURVEY §8(d)'s 3*R*C for the reference's matrix.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"

namespace {

// Development ablations of the u8 lane fills (variant libraries only, BT2X_LIB; outputs
// invalid): -DBT2X_PROF_NOSTORE drops the traceback stores, -DBT2X_PROF_NOWINDOW the
// reference-window loads (which also changes every cell's value and so the candidates:
// its gain is mostly a shorter candidate ordering, not the loads' waits -- an LDS-DMA
// window ring that removed those waits measured neutral).
#ifdef BT2X_PROF_NOSTORE
constexpr bool kProfStores = false;
#else
constexpr bool kProfStores = true;
#endif
// cache-policy bits of the fill's traceback stores (buffer instruction aux: sc0 1, nt 2, sc1 16)
#ifndef BT2X_TB_STORE_AUX
#define BT2X_TB_STORE_AUX 0
#endif
constexpr int kTbStoreAux = BT2X_TB_STORE_AUX;
#ifdef BT2X_PROF_NOWINDOW
constexpr bool kProfWindow = false;
#else
constexpr bool kProfWindow = true;
#endif

constexpr int kRows = BT2X_MAX_ROWS;          // 160
constexpr int kRowWords = kRows / 4;          // state dwords (4 rows each)
constexpr int kCols = BT2X_MAX_COLS;          // 200
constexpr int kSteps = kRows + 1;             // steps per column pair (rows 0..R-1, skew 1)
constexpr int kPairWords = (kSteps + 1) / 2;  // traceback dwords per column pair (2 steps each)
constexpr uint32_t kDirBytesLane = (kCols / 2) * kPairWords * 4;   // 32400
constexpr uint32_t kLastRowBytesLane = 512;                        // u16 per column (i16 kernel)
constexpr uint32_t kCandBytesLane = kCols;                         // sorted candidate columns
constexpr uint32_t kEditStage = 400;                               // >= R + C + 2
constexpr uint32_t kRecStage = kCols + 8;                          // >= ncand + 1
constexpr int kMoveLogWords = (kRows + kCols + 15) / 16;           // an attempt's moves, 2 bits each
#ifndef BT2X_WALK_BATCH
#define BT2X_WALK_BATCH 32
#endif
constexpr int kWalkBatch = BT2X_WALK_BATCH;                        // walk bytes fetched per round trip (8, 16 or 32)
// Group region: the fill's output for 64 problems (all regions lane-interleaved).
constexpr size_t kDirOff = 0;
constexpr size_t kLastRowOff = kDirOff + (size_t)kDirBytesLane * 64;
constexpr size_t kCandOff = kLastRowOff + (size_t)kLastRowBytesLane * 64;
constexpr size_t kGroupBytes = kCandOff + (size_t)kCandBytesLane * 64;
// Walk slot: staging of one resident walk wave (lane-interleaved).
constexpr size_t kEditOff = 0;
constexpr size_t kRecOff = kEditOff + (size_t)kEditStage * 4 * 64;
constexpr size_t kWalkSlotBytes = kRecOff + (size_t)kRecStage * sizeof(bt2x_aln_rec) * 64;

// Byte address (within a group's lane-interleaved traceback region) of cell (row, col)
// of lane `lane`: column pair p = col/2; even columns sit at step row, odd columns at
// step row + 1; one dword holds two steps of both columns of a pair.  Lane-interleaved
// dwords keep the fill's stores coalesced (256 B per wave store) and let the 64 lanes'
// walks, which follow nearly the same diagonal (every rectangle is framed around its
// seed diagonal), share cache lines.
__device__ __forceinline__ size_t tb_addr(int row, int col, int lane) {
	const int st = row + (col & 1);
	return ((((size_t)(col >> 1) * kPairWords + (st >> 1)) * 64 + lane) << 2) + ((st & 1) << 1) + (col & 1);
}

// Byte offsets of diagonal moves in that layout: (r, 2p+1) -> (r-1, 2p) is -257 (same
// pair, one step pair up, high column -> low), (r, 2p) -> (r-1, 2p-1) is kDiag1Even (one
// column pair left); two diagonal moves are always kDiag2.
constexpr int kDiag1Even = -(kPairWords * 256) + 1;
constexpr int kDiag2 = -257 + kDiag1Even;
__device__ __forceinline__ uint32_t tb_load(__amdgpu_buffer_rsrc_t src, uint32_t off) {
	return __builtin_amdgcn_raw_buffer_load_b8(src, (int)off, 0, 0);   // out of range: 0
}
// s_waitcnt vmcnt(0), expcnt and lgkmcnt left alone (gfx9 encoding: vmcnt bits 3:0 and
// 15:14, expcnt 6:4, lgkmcnt 11:8)
constexpr int kWaitVm0 = 0x0f70;
// The byte at off in the low 8 bits of an (unaligned) dword load, the bits above it the
// following bytes: for loop-carried registers, which the compiler would otherwise keep as
// 8-bit values and re-extend with copies that wait for the loads.  Users test low bits only.
__device__ __forceinline__ uint32_t tb_load4(__amdgpu_buffer_rsrc_t src, uint32_t off) {
	return __builtin_amdgcn_raw_buffer_load_b32(src, (int)off, 0, 0);
}

// 1 in the lowest active lane, else 0 (summed over lanes: wave iterations)
__device__ __forceinline__ unsigned first_active(int lane) {
	const uint64_t e = __builtin_amdgcn_read_exec();
	return (e & (~e + 1)) == (1ull << lane) ? 1u : 0u;
}
// a value every active lane holds alike, as such (scalar registers, SALU arithmetic)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// true when no active lane has `c` set (a wave-uniform value)
__device__ __forceinline__ bool wave_none(bool c) { return __builtin_amdgcn_ballot_w64(c) == 0; }

// traceback flag bits (1 = the equality does NOT hold); TB_MM: read and reference
// bases differ or either is N (the diagonal move records an edit)
enum { TB_DNE = 1, TB_FNE = 2, TB_FONE = 4, TB_EONE = 8, TB_MM = 0x10, TB_MARK = 0x80 };

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as1(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t psubs(uint32_t a, uint32_t b) { return as1(__builtin_elementwise_sub_sat(as2(a), as2(b))); }
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) { return as1(__builtin_elementwise_max(as2(a), as2(b))); }
// v_pk_min_u16.  A constant 0x00010001 bound would be lowered to compares, so callers
// pass it in a register the optimizer cannot see through (`one2`, made opaque once).
// No inline asm here: asm blocks get conservative hazard padding (an s_nop after each).
__device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b) { return as1(__builtin_elementwise_min(as2(a), as2(b))); }
__device__ __forceinline__ uint32_t pmul(uint32_t a, uint32_t b) { return as1(as2(a) * as2(b)); }
__device__ __forceinline__ uint32_t pmul_lo(uint32_t a, uint32_t b) {
	uint32_t r; asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ __forceinline__ uint32_t pshr(uint32_t a, uint32_t sh) { return as1(as2(a) >> (u16x2){(unsigned short)sh, (unsigned short)sh}); }
// per-half "not equal" flag, 0 or 1 (one2 = 0x00010001 in a register)
__device__ __forceinline__ uint32_t pne(uint32_t a, uint32_t b, uint32_t one2) { return pmin(a ^ b, one2); }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
__device__ __forceinline__ uint32_t opaque(uint32_t v) { asm volatile("" : "+v"(v)); return v; }

// ---------------------------------------------- candidate order (DpBtCandidate)
// A lane's last row as byte keys in LDS (lds[q * 64 + lane], 4 columns a dword, q < nw;
// byte 0 = below the threshold) is put in DpBtCandidate order (score desc, col desc,
// aligner_swsse_ee_u8.cpp:519-536 + the sort of btncand_): key = score << 8 | col, 16 bits,
// two keys per packed op; keys of non-qualifying columns (score 0) are below every
// qualifying one and are never reached within ncand.
//
// keys_below: the largest key below cur (cur2 = cur in both halves) among dword q's four
// columns, per half (0 if none).
__device__ __forceinline__ uint32_t keys_below(uint32_t w4, uint32_t q, uint32_t cur2, uint32_t one2) {
	const uint32_t cq = q * 0x40004u + 0x10000u;                   // cols 4q, 4q+1
	const uint32_t ka = perm(cq, w4, 0x01060004u);                 // [4q, s0, 4q+1, s1]
	const uint32_t kb = perm(cq + 0x20002u, w4, 0x03060204u);      // [4q+2, s2, 4q+3, s3]
	return pmax(pmul_lo(pmin(psubs(cur2, ka), one2), ka), pmul_lo(pmin(psubs(cur2, kb), one2), kb));
}

// The ncand sorted keys, emit(k, key) each.  Round 6: per 16-column group the largest key
// not yet emitted is kept (13 groups, two a register); the next candidate is the largest of
// those, and only its group is scanned again for its next key below (every larger key of
// the group is already out) -- ~80 instructions a candidate instead of a max-below-key scan
// of the whole row (~11 per dword, ~500 at 181 columns).  A wave whose lanes have at most
// two candidates keeps the plain scans (the groups' setup costs one).
template<class Emit>
__device__ __forceinline__ void order_candidates(const uint32_t* lds, int lane, int nw, int ncand, uint32_t one2,
                                                 Emit&& emit) {
	constexpr int kGroups = (kCols + 15) / 16;                     // 13
	if(__builtin_amdgcn_ballot_w64(ncand > 2) == 0) {
		int cur_key = 0xffff;
		for(int k = 0; k < ncand; k++) {
			const uint32_t cur2 = (uint32_t)cur_key * 0x10001u;
			uint32_t best2 = 0;
#pragma unroll 2
			for(int q = 0; q < nw; q++) best2 = pmax(best2, keys_below(lds[q * 64 + lane], (uint32_t)q, cur2, one2));
			cur_key = (int)max(best2 & 0xffffu, best2 >> 16);
			emit(k, cur_key);
		}
		return;
	}
	uint32_t gm[(kGroups + 1) / 2];                                // group 2i: low half, 2i+1: high half
#pragma unroll
	for(int i = 0; i < (kGroups + 1) / 2; i++) gm[i] = 0;
#pragma unroll
	for(int g = 0; g < kGroups; g++) {
		if(4 * g >= nw) break;                                     // (wave-uniform)
		uint32_t m2 = 0;
#pragma unroll
		for(int i = 0; i < 4; i++) {
			const int q = 4 * g + i;
			if(q < nw) m2 = pmax(m2, keys_below(lds[q * 64 + lane], (uint32_t)q, 0xffffffffu, one2));
		}
		const uint32_t gmax = max(m2 & 0xffffu, m2 >> 16);
		gm[g >> 1] |= gmax << (16 * (g & 1));
	}
	for(int k = 0; k < ncand; k++) {
		uint32_t m2 = gm[0];
#pragma unroll
		for(int i = 1; i < (kGroups + 1) / 2; i++) m2 = pmax(m2, gm[i]);
		const uint32_t key = max(m2 & 0xffffu, m2 >> 16);
		emit(k, (int)key);
		const int g = (int)(key & 0xffu) >> 4;                     // the key's column -> its group
		const uint32_t cur2 = key * 0x10001u;
		uint32_t b2 = 0;
#pragma unroll
		for(int i = 0; i < 4; i++) {
			const int q = 4 * g + i;
			if(q < nw) b2 = pmax(b2, keys_below(lds[q * 64 + lane], (uint32_t)q, cur2, one2));
		}
		const uint32_t nb = max(b2 & 0xffffu, b2 >> 16);
#pragma unroll
		for(int i = 0; i < (kGroups + 1) / 2; i++) {
			const uint32_t hi = (gm[i] & 0xffffu) | (nb << 16), lo = (gm[i] & 0xffff0000u) | nb;
			gm[i] = (g >> 1) == i ? ((g & 1) ? hi : lo) : gm[i];
		}
	}
}

enum { H_NONE = 0, H_DIAG = 1, H_REF_OPEN = 2, H_RFGAP_EXT = 3, H_READ_OPEN = 4, H_RDGAP_EXT = 5 };
enum { EDIT_READ_GAP = 1, EDIT_REF_GAP = 2, EDIT_MM = 3 };

__device__ __forceinline__ int sat(int v) { return v < 0 ? 0 : v; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t pack_edit(uint32_t pos, int type, int chr, int qchr) {
	return (pos & 0x3ffu) | ((uint32_t)type << 12) | ((uint32_t)(uint8_t)chr << 16) |
	       ((uint32_t)(uint8_t)qchr << 24);
}

// "ACGTN"[c] without a branch tree (c in 0..4)
__device__ __forceinline__ char acgtn(int c) { return (char)((0x4e54474341ULL >> (8 * c)) & 0xffu); }
// mask2dna of a single-base mask 1<<c (c = 4 -> mask 16 -> 'N'), alphabet.cpp:71
__device__ __forceinline__ char mask_chr(int c) { return acgtn(c); }

__device__ __forceinline__ uint64_t cell_digest(uint32_t row, uint32_t col, uint32_t mat, uint32_t val) {
	uint64_t z = ((uint64_t)row << 40) ^ ((uint64_t)col << 20) ^ ((uint64_t)mat << 16) ^ (uint64_t)val;
	z += 0x9e3779b97f4a7c15ULL;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
	return z ^ (z >> 31);
}

__device__ __forceinline__ int wave_max(int v) {
	for(int d = 32; d > 0; d >>= 1) { const int o = __shfl_xor(v, d); v = v > o ? v : o; }
	return v;
}

// Per-row info byte kept in VGPRs during the fill: read code (3 bits; a read N is 7,
// which matches no reference code, with mm = the N penalty), gap-barrier flag (bit 3),
// mismatch penalty for the row's quality (bits 4-7; penalties <= 15, checked at open).
__device__ __forceinline__ uint32_t row_info(int rdc, bool gbar, int mm) {
	return (uint32_t)rdc | (gbar ? 8u : 0u) | ((uint32_t)mm << 4);
}

// A byte string s[0, n) read as dwords: bytes4(k) = s[4k .. 4k+3] (byte r of the result is
// s[4k+r]; bytes at positions >= n are unspecified).  Loads are dword-aligned and clamped
// to the dword holding s[n-1], so they never touch a dword that holds no byte of the
// string (nor a page the string does not reach); unaligned strings are shifted into place
// with v_alignbyte.  n >= 1.
struct ByteStr {
	const uint32_t* base;         // the dword holding s[0]
	uint32_t sh;                  // s[0]'s byte within it
	int lastw;                    // index (from base) of the dword holding s[n-1]
};
__device__ __forceinline__ ByteStr byte_str(const uint8_t* s, int n) {
	ByteStr b;
	b.sh = (uint32_t)((uintptr_t)s & 3u);
	b.base = reinterpret_cast<const uint32_t*>(s - b.sh);      // (pointer arithmetic: stays a global pointer)
	b.lastw = (int)((b.sh + (uint32_t)n - 1u) >> 2);
	return b;
}
__device__ __forceinline__ uint32_t bs_word(const ByteStr& b, int w) { return b.base[w < b.lastw ? w : b.lastw]; }
__device__ __forceinline__ uint32_t bs_bytes4(const ByteStr& b, int k) {
	return __builtin_amdgcn_alignbyte(bs_word(b, k + 1), bs_word(b, k), b.sh);
}

// An edit whose characters are not looked up yet (the walk records row, type and
// reference column only): pos | type << 12 | kEditPending | col << 16.
constexpr uint32_t kEditPending = 0x8000u;
__device__ __forceinline__ uint32_t pend_edit(int pos, int type, int col) {
	return ((uint32_t)pos & 0x3ffu) | ((uint32_t)type << 12) | kEditPending | ((uint32_t)col << 16);
}
// the read row an edit refers to (a read gap is recorded at row + 1, aligner_sw's convention)
__device__ __forceinline__ int pending_row(uint32_t e) {
	return (int)(e & 0x3ffu) - ((((e >> 12) & 7u) == EDIT_READ_GAP) ? 1 : 0);
}
__device__ __forceinline__ uint32_t pending_chars_of(uint32_t e, int rdc, int refc) {
	const int type = (int)((e >> 12) & 7u);
	const uint32_t pos = e & 0x3ffu;
	return type == EDIT_MM ? pack_edit(pos, EDIT_MM, mask_chr(refc), acgtn(rdc))
	     : type == EDIT_REF_GAP ? pack_edit(pos, EDIT_REF_GAP, '-', acgtn(rdc))
	                            : pack_edit(pos, EDIT_READ_GAP, mask_chr(refc), '-');
}
__device__ __forceinline__ uint32_t pending_chars(uint32_t e, const uint8_t* rd, const uint8_t* rf) {
	return pending_chars_of(e, rd[pending_row(e)], rf[(e >> 16) & 0xffu]);
}
// Resolve the pending entries [0, ne) of a finished backtrace in place: characters, and
// for mismatches the penalty (N: npen, else the quality's) and the N count the reference
// accumulates as it walks (u8.cpp backtrace).  Eight entries per batch, loads together.
__device__ __forceinline__ void resolve_edits(const DevScoring& sc, const uint8_t* mmpen, uint32_t* stage_ed, int lane,
                                              int ne, const uint8_t* rd, const uint8_t* rf, const uint8_t* qu,
                                              int* bscore, int* ns) {
	for(int k0 = 0; k0 < ne; k0 += 8) {
		uint32_t v[8];
#pragma unroll
		for(int u = 0; u < 8; u++) v[u] = stage_ed[(size_t)min(k0 + u, ne - 1) * 64 + lane];
		int rdc[8], refc[8], q[8];
#pragma unroll
		for(int u = 0; u < 8; u++) {
			const int r = pending_row(v[u]);
			rdc[u] = rd[r]; refc[u] = rf[(v[u] >> 16) & 0xffu]; q[u] = qu[r];
		}
		int pen[8];
#pragma unroll
		for(int u = 0; u < 8; u++) {
			const int q0 = q[u] - 33;
			pen[u] = mmpen[q0 < 0 ? 0 : (q0 > 255 ? 255 : q0)];
		}
#pragma unroll
		for(int u = 0; u < 8; u++) {
			if(k0 + u >= ne) break;
			const uint32_t e = v[u];
			if(!(e & kEditPending)) continue;                  // resolved already (gap-barrier rows)
			if(((e >> 12) & 7u) == EDIT_MM) {
				const bool amb = rdc[u] > 3 || refc[u] > 3;
				*bscore -= amb ? sc.npen : pen[u];
				*ns += amb ? 1 : 0;
			}
			stage_ed[(size_t)(k0 + u) * 64 + lane] = pending_chars_of(e, rdc[u], refc[u]);
		}
	}
}

// Copy the edit-buffer entries [0, hi) written by one nextAlignment call to the edits
// arena; returns their offset (0 when nothing was written).  A successful call's own
// entries [0, ns) are still in walk order: they are published in ned() order -- reversed
// (fw), or with positions mirrored over `extent` (the reverse-complement strand's
// invertEdits, edit.cpp:50-78) -- which is exactly what the reference's buffer holds
// after the call.  Eight entries per batch: the loads go out together instead of one
// dependent round trip per entry.
__device__ __forceinline__ uint32_t publish_edbuf(const DpLaunch& a, const uint32_t* stage_ed, int lane, int hi,
                                                  const uint8_t* rd, const uint8_t* rf,
                                                  int ns = 0, bool fw = true, int extent = 0) {
	if(hi <= 0) return 0;
	const uint32_t eo = atomicAdd(&a.counters[1], (uint32_t)hi);
	if(eo + (uint32_t)hi <= a.edit_cap) {
		for(int k0 = 0; k0 < hi; k0 += 8) {
			uint32_t v[8];
#pragma unroll
			for(int u = 0; u < 8; u++) {
				const int k = min(k0 + u, hi - 1);
				const int src = (k < ns && fw) ? ns - 1 - k : k;
				v[u] = stage_ed[(size_t)src * 64 + lane];
			}
#pragma unroll
			for(int u = 0; u < 8; u++) {
				const int k = k0 + u;
				if(k >= hi) break;
				uint32_t e = v[u];
				if(e & kEditPending) e = pending_chars(e, rd, rf);
				if(k < ns && !fw) {
					const uint32_t pos = (uint32_t)extent - (e & 0x3ffu) - (((e >> 12) & 7u) == 1u /*read gap*/ ? 0u : 1u);
					e = (e & ~0x3ffu) | (pos & 0x3ffu);
				}
				a.edits[eo + k] = e;
			}
		}
	}
	return eo;
}

// Byte address of cell (row, col) in a traceback layout of G problems per group and PW
// dwords per column pair (tb_addr is G = 64, PW = kPairWords): problem slot tbl.
template<int G, int PW>
__device__ __forceinline__ size_t tb_addr_g(int row, int col, int tbl) {
	const int st = row + (col & 1);
	return ((((size_t)(col >> 1) * PW + (st >> 1)) * G + tbl) << 2) + ((st & 1) << 1) + (col & 1);
}
// The same in 32 bits (a traceback region is far below 4 GiB): the walk's hot path, where
// a 64-bit multiply-add's register pair can alias a ring register and wait for its load.
template<int G, int PW>
__device__ __forceinline__ uint32_t tb_off_g(int row, int col, int tbl) {
	const uint32_t st = (uint32_t)(row + (col & 1));
	// (the multiply in asm: the compiler would form the multiply-add as v_mad_u64_u32,
	// whose 64-bit addend pair can take a ring register and so wait for its load)
	uint32_t pr;
	asm("v_mul_u32_u24 %0, %1, %2" : "=v"(pr) : "v"((uint32_t)(col >> 1)), "v"((uint32_t)PW));
	return ((pr + (st >> 1)) * G + (uint32_t)tbl) * 4u + ((st & 1u) << 1) + ((uint32_t)col & 1u);
}

// SwAligner::nextAlignment until done() for problem pi: its candidates in order (cands,
// [k * 64 + lane]), each not already reportedThrough backtraced over the fill's traceback
// bytes (layout tb_addr_g<G, PW>, problem slot tbl, from dirbase); records and edits
// staged per lane.
template<int G, int PW>
__device__ __forceinline__ void walk_problem(const DevScoring& sc, const uint8_t* mmpen, const DpLaunch& a, uint32_t pi,
                                             int lane, int tbl, const uint8_t* dirbase, uint32_t dirbytes,
                                             const uint8_t* cands, uint32_t* stage_ed,
                                             bt2x_aln_rec* stage_rec, unsigned long long& st_bt, bool refN,
                                             uint32_t* mlog, bool prof, unsigned long long& pw_steps, unsigned long long& pw_iters) {
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe;
	const uint32_t gl = (uint32_t)lane;
	// the layout's move offsets (see kDiag1Even): one step pair up is -4G bytes
	constexpr int kD1E = -(PW * 4 * G) + 1;        // (r, 2p) -> (r-1, 2p-1)
	constexpr int kD1O = -(4 * G + 1);             // (r, 2p+1) -> (r-1, 2p)
	constexpr int kD2 = kD1O + kD1E;               // two diagonal moves
	const __amdgpu_buffer_rsrc_t dirsrc =
		__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(dirbase), 0, (int)dirbytes, 0x00020000);
	bt2x_dp_out o = a.out[pi];
	if(o.status > 0 && o.ncand > 0 && a.ablate != 1) {
		const bt2x_dp_in p = a.in[pi];
		const int R = p.rdlen;
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int ncand = o.ncand;
		const int row0 = R - 1;
		int ndone = 0, nrec = 0;
		// Step budget (a.heavy; 0: none).  A walk runs one chain of HBM round trips per
		// step, and at cohort launch sizes (about one group per wave) its wave, and so
		// the launch, waits for its longest lane: a problem past the budget (a repeat
		// walked attempt after attempt) is dropped here -- nothing of it is kept but
		// edit-arena space -- and redone by the wave kernel with its traceback in LDS.
		const int budget = (a.heavy_list && a.heavy) ? (int)a.heavy : 0x7fffffff;
		int steps = 0;
		bool aborted = false;
		// Candidate starts are fetched ahead: the next candidate's column two attempts early,
		// and the bytes of its first eight cells down its diagonal (its start cell first) one
		// attempt early -- the walk's ring (below) for that attempt, so a short attempt (most
		// are: they run into an earlier path's marks within a few cells) waits on nothing.
		// Bytes fetched before the attempt in between reflect every earlier attempt's marks;
		// that attempt's own marks on those cells are recorded in `cmask` (bit i: the cell i
		// rows up the diagonal) and applied when the ring is taken.
		int c_next = cands[gl];
		uint32_t n0, n1, n2, n3, n4, n5, n6, n7;
#define BT2X_RING_LOAD(A0, A1, A2, A3, A4, A5, A6, A7, BO, COL)                                          \
		{                                                                                         \
			const uint32_t bo_ = (BO);                                                            \
			const int d1_ = ((COL) & 1) ? kD1O : kD1E;                                      \
			A0 = tb_load4(dirsrc, bo_);                      A1 = tb_load4(dirsrc, bo_ + d1_);      \
			A2 = tb_load4(dirsrc, bo_ + kD2);             A3 = tb_load4(dirsrc, bo_ + kD2 + d1_); \
			A4 = tb_load4(dirsrc, bo_ + 2 * kD2);         A5 = tb_load4(dirsrc, bo_ + 2 * kD2 + d1_); \
			A6 = tb_load4(dirsrc, bo_ + 3 * kD2);         A7 = tb_load4(dirsrc, bo_ + 3 * kD2 + d1_); \
		}
		BT2X_RING_LOAD(n0, n1, n2, n3, n4, n5, n6, n7, ((uint32_t)tb_addr_g<G, PW>(row0, c_next, tbl)), c_next)
		int c_next2 = ncand > 1 ? cands[64 + gl] : 0;
		uint32_t cmask = 0;                                    // last attempt's marks on the next ring
		// stage_ed doubles as the reference's per-read edit buffer (SwResult::alres.ned_,
		// bt2x.h "edit-buffer image"): attempts write it from index 0, a success leaves its
		// final list there; hi = entries written during the current call.
		while(ndone < ncand) {
			int ntries = 0, hi = 0;
			bool found = false;
			while(ndone < ncand) {
				if(prof) pw_iters += first_active(lane);    // development counters (BT2X_DP_PROF)
				// Drain the last attempt's stores (its marks and edits) before this one's loads:
				// with stores and loads both pending, the compiler treats vmcnt as out of order
				// and would wait for vmcnt(0) at every step of the walk's ring below
				__builtin_amdgcn_s_waitcnt(kWaitVm0);
				const int col0 = c_next;
				const uint32_t M = TB_MARK;
				uint32_t q0 = n0 | ((cmask & 1u) ? M : 0u), q1 = n1 | ((cmask & 2u) ? M : 0u);
				uint32_t q2 = n2 | ((cmask & 4u) ? M : 0u), q3 = n3 | ((cmask & 8u) ? M : 0u);
				uint32_t q4 = n4 | ((cmask & 16u) ? M : 0u), q5 = n5 | ((cmask & 32u) ? M : 0u);
				uint32_t q6 = n6 | ((cmask & 64u) ? M : 0u), q7 = n7 | ((cmask & 128u) ? M : 0u);
				const uint32_t tb = q0;
				ndone++;
				int dnx = -(1 << 20);                              // the next candidate's diagonal
				if(ndone < ncand) {
					c_next = c_next2;
					dnx = c_next - row0;
					BT2X_RING_LOAD(n0, n1, n2, n3, n4, n5, n6, n7, ((uint32_t)tb_addr_g<G, PW>(row0, c_next, tbl)), c_next)
					if(ndone + 1 < ncand) c_next2 = cands[(size_t)(ndone + 1) * 64 + gl];
				}
				cmask = 0;
				// candidate start cell already traversed -> skipped, no RNG draw
				if(tb & TB_MARK) continue;
				ntries++;
				if(a.ablate == 2) continue;          // profiling: no backtrace walks
				// ------------- backtraceNucleotidesEnd2EndSseU8 -------------
				int row = row0, col = col0, ct = 2 /*H*/, bscore = 0, ns = 0, gaps = 0, ne = 0;
				bool over_core = false, ok = true;
				uint32_t tb_end = 0;
				// The walk reads one byte per step, each depending on the move decided from the
				// last: a chain of cache-missing loads (the fill's bytes left L2 long ago).  Most
				// moves are diagonal (all of them in the bottom gap-barrier rows, which hold no E
				// or F), so the bytes of the next seven cells down the current diagonal are kept
				// in flight: a ring of registers (q0..q7, rotated by unrolling the step, never
				// moved -- a move would wait for the load) refilled one cell per diagonal step,
				// and reloaded from the new cell after a gap move.  The loads are dwords (the byte
				// in bits 0-7): 8-bit values carried around the loop get re-extended by copies
				// that wait for them.  The current attempt never revisits its own cells and
				// earlier attempts' marks were stored before these loads (or are patched in from
				// cmask), so a ring byte is the byte the reference reads.
				uint32_t bo = tb_off_g<G, PW>(row, col, tbl);
				uint32_t fin = 0, okw = 1, abw = 0;               // 0/1 (see BT2X_WALK_STEP)
				// The step loop issues loads only.  Its moves go to a log in LDS (2 bits each:
				// diagonal, diagonal mismatch, up = reference gap, left = read gap; mlog[w * 64 +
				// lane] holds moves 16w .. 16w + 15) and the attempt's marks (setReportedThrough)
				// and edits are written from it after the attempt: vmcnt counts loads and stores
				// in issue order, so a store in the chain made every later step wait for the
				// store's completion, not only for its own load.
				uint32_t macc = 0;                                 // the log's current word
				int nvis = 0;                                      // cells checked (stats)
				// Per diagonal, not per cell: a diagonal move keeps col - row, so whether the path
				// is over the core diagonals and whether it runs down the next candidate's
				// diagonal (cmask) change only with a gap move.
				uint32_t on_next = col0 - row0 == dnx ? 1u : 0u;
				uint32_t ocw = (col0 - row0 + (int)p.triml >= 0) & (col0 - row0 + (int)p.triml >= (int)p.corel) &
				               (col0 - row0 + (int)p.triml <= (int)p.corer);
				int nm = 0;                                        // moves logged
				uint32_t end0 = 0;                                 // the path reached row 0
// The step in integer arithmetic on 0/1 values (0u - b: a mask): as booleans the
// conditions live in lane masks, and their nested ifs cost more scalar mask bookkeeping
// than the work they guard.  Only the gap move, rare across a wave, is a branch.  The log
// word is stored every step (unchanged when the lane did not move), so the last partial
// word needs no flush.
#define BT2X_WALK_STEP(T0, T1, T2, T3, T4, T5, T6, T7)                                                        \
				{                                                                                     \
					const uint32_t c = T0;                        /* the cell's byte in bits 0-7 */   \
					const uint32_t go = 1u - fin;                                                     \
					const uint32_t over = go & ((uint32_t)(budget - 1 - steps) >> 31); /* ++steps > budget */ \
					steps += (int)go;                                                                 \
					const uint32_t chk = go & (over ^ 1u);                                            \
					nvis += (int)chk;                                                                 \
					const uint32_t live = chk & (((c >> 7) & 1u) ^ 1u);  /* not reportedThrough */   \
					const uint32_t mk = chk ^ live;                                                   \
					const uint32_t z = (uint32_t)(row - 1) >> 31;  /* row == 0 */                     \
					const uint32_t up = (uint32_t)(row0 - row);                                       \
					cmask |= (live & on_next & ((up - 8u) >> 31)) << (up & 31u);                      \
					const uint32_t at0 = live & z;                                                    \
					tb_end |= c & (0u - at0);                                                         \
					end0 |= at0;                                                                      \
					const uint32_t mvg = live & (z ^ 1u);                                             \
					/* the reference's fixed priority over the cell's flags (u8.cpp:843-990): H: \
					   diag > F (H-up / F-up) > E (H-left / E-left); E/F prefer the open */       \
					const uint32_t inH = (uint32_t)ct >> 1, inF = (uint32_t)ct & 1u;                  \
					const uint32_t dne = c & 1u, fne = (c >> 1) & 1u;                                 \
					const uint32_t isD = inH & (dne ^ 1u);                                            \
					const uint32_t isF = inF | (inH & dne & (fne ^ 1u));                              \
					const uint32_t isE = 1u - isD - isF;                                              \
					const uint32_t nct = (2u & (0u - isD)) | ((2u - ((c >> 2) & 1u)) & (0u - isF)) | ((2u - 2u * ((c >> 3) & 1u)) & (0u - isE)); \
					const uint32_t ccol = (uint32_t)col;                                              \
					row -= (int)(mvg & (isD | isF));                                                  \
					col -= (int)(mvg & (isD | isE));                                                  \
					ct = (int)(((uint32_t)ct & ~(0u - mvg)) | (nct & (0u - mvg)));                    \
					/* the move, logged (its edit and mark are written after the attempt) */      \
					const uint32_t code = (((c >> 4) & 1u) & (0u - isD)) | (2u & (0u - isF)) | (3u & (0u - isE)); \
					macc |= (code & (0u - mvg)) << (2u * ((uint32_t)nm & 15u));                        \
					mlog[(size_t)(nm >> 4) * 64 + lane] = macc;                                       \
					macc &= 0u - (1u - (mvg & (((uint32_t)nm & 15u) == 15u ? 1u : 0u)));             \
					nm += (int)mvg;                                                                   \
					const uint32_t gp = mvg & (isD ^ 1u);                                             \
					{                                                                                 \
						const uint32_t om = 0u - (nct >> 1), fm = 0u - isF;   /* open, F: masks */    \
						const uint32_t pf = ((uint32_t)rfo & om) | ((uint32_t)rfe & ~om);              \
						const uint32_t pe = ((uint32_t)rdo & om) | ((uint32_t)rde & ~om);              \
						bscore -= (int)(((pf & fm) | (pe & ~fm)) & (0u - gp));                        \
					}                                                                                 \
					gaps += (int)gp;                                                                  \
					okw &= (over | mk) ^ 1u;                                                          \
					abw |= over;                                                                      \
					fin |= over | mk | at0;                                                           \
					uint32_t nbo = bo + 4 * kD2;  /* the next ring load; finished lanes: harmless */ \
					/* a diagonal move: the ring's next cell */                                   \
					bo += (uint32_t)((ccol & 1u) ? kD1O : kD1E) & (0u - (mvg & isD));                 \
					if(gp) {                                                                          \
						bo = tb_off_g<G, PW>(row, col, tbl);                                          \
						const int d1 = (col & 1) ? kD1O : kD1E;                                       \
						const int dg = col - row + (int)p.triml;                                      \
						ocw |= (dg >= 0) & (dg >= (int)p.corel) & (dg <= (int)p.corer);               \
						on_next = (col - row == dnx) ? 1u : 0u;                                       \
						T1 = tb_load4(dirsrc, bo);                  T2 = tb_load4(dirsrc, bo + d1);    \
						T3 = tb_load4(dirsrc, bo + kD2);         T4 = tb_load4(dirsrc, bo + kD2 + d1); \
						T5 = tb_load4(dirsrc, bo + 2 * kD2);     T6 = tb_load4(dirsrc, bo + 2 * kD2 + d1); \
						T7 = tb_load4(dirsrc, bo + 3 * kD2);     T0 = tb_load4(dirsrc, bo + 3 * kD2 + d1); \
					} else {                                                                          \
						T0 = tb_load4(dirsrc, nbo);                                                   \
					}                                                                                 \
				}
				// lanes that finish idle to the end of the wave's step: the exits are wave-uniform
				// (no divergent loop exits, whose joins would copy -- and so wait for -- the
				// ring registers).  Sixteen steps per pass: the compiler waits for every load at
				// the top of the loop (it does not carry the ring's order across the back edge).
				while(true) {
					if(prof) pw_steps += first_active(lane);
					BT2X_WALK_STEP(q0, q1, q2, q3, q4, q5, q6, q7) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q1, q2, q3, q4, q5, q6, q7, q0) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q2, q3, q4, q5, q6, q7, q0, q1) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q3, q4, q5, q6, q7, q0, q1, q2) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q4, q5, q6, q7, q0, q1, q2, q3) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q5, q6, q7, q0, q1, q2, q3, q4) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q6, q7, q0, q1, q2, q3, q4, q5) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q7, q0, q1, q2, q3, q4, q5, q6) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q0, q1, q2, q3, q4, q5, q6, q7) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q1, q2, q3, q4, q5, q6, q7, q0) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q2, q3, q4, q5, q6, q7, q0, q1) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q3, q4, q5, q6, q7, q0, q1, q2) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q4, q5, q6, q7, q0, q1, q2, q3) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q5, q6, q7, q0, q1, q2, q3, q4) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q6, q7, q0, q1, q2, q3, q4, q5) if(wave_none(!fin)) break;
					BT2X_WALK_STEP(q7, q0, q1, q2, q3, q4, q5, q6) if(wave_none(!fin)) break;
				}
#undef BT2X_WALK_STEP
#undef BT2X_RING_LOAD
				st_bt += (unsigned long long)nvis;
				ok = okw != 0; aborted = aborted || abw != 0; over_core = ocw != 0;
if(aborted) break;
// the attempt's marks and edits, from its move log (the reference's order: an
// edit per move that records one, in walk order)
{
	int r = row0, c = col0;
	uint32_t b = (uint32_t)tb_addr_g<G, PW>(r, c, tbl), w = 0;
	for(int k = 0; k < nm; k++) {
		if((k & 15) == 0) w = mlog[(size_t)(k >> 4) * 64 + lane];
		const uint32_t mv = (w >> (2 * (k & 15))) & 3u;
		__builtin_amdgcn_raw_buffer_store_b8((uint8_t)TB_MARK, dirsrc, (int)b, 0, 0);   // setReportedThrough
		if(mv != 0) {
			stage_ed[(size_t)ne * 64 + lane] = mv == 1 ? pend_edit(r, EDIT_MM, c)
			                                 : mv == 2 ? pend_edit(r, EDIT_REF_GAP, c)
			                                           : pend_edit(r + 1, EDIT_READ_GAP, c);
			ne++;
		}
		if(mv <= 1) { b += (c & 1) ? kD1O : kD1E; r--; c--; }
		else if(mv == 2) { b += ((r + (c & 1)) & 1) ? -2 : -(4 * G - 2); r--; }
		else { b += (c & 1) ? ((r & 1) ? -(4 * G - 1) : -3) : ((r & 1) ? kD1E + 4 * G - 2 : kD1E + 2); c--; }
	}
	if(end0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)TB_MARK, dirsrc, (int)b, 0, 0);
}
				if(!ok || !over_core) { hi = max(hi, ne); continue; }
				if(tb_end & TB_MM) {                     // the final (row 0) cell
					stage_ed[(size_t)ne * 64 + lane] = pend_edit(row, EDIT_MM, col);
					ne++;
				}
				resolve_edits(sc, mmpen, stage_ed, lane, ne, rd, rf, qu, &bscore, &ns);
				if(ns > p.nceil) { hi = max(hi, ne); continue; }
				// reference Ns under the alignment: only windows holding an N (flagged by the
				// fill) scan their columns
				int refns = 0;
				if(refN)
					for(int k = col; k <= col0; k++) refns += (rf[k] > 3);
				// trimBeg = 0; ned() order (reverse(), and for the reverse-complement strand
				// invertEdits(), edit.cpp:50-78) is applied as the entries are published
				const int extent = R - (R - row0 - 1);
				hi = max(hi, ne);
				found = true;
				bt2x_aln_rec r;
				r.ntries = (uint16_t)ntries; r.ok = 1; r.pad0 = 0;
				r.score = (int16_t)bscore; r.ns = (uint16_t)ns; r.gaps = (uint16_t)gaps;
				r.nedit = (uint16_t)ne; r.bases_aligned = (uint16_t)(extent - ne);
				r.refns = (uint16_t)refns; r.refoff = (int64_t)col + p.refl;
				r.edit_off = publish_edbuf(a, stage_ed, lane, hi, rd, rf, ne, p.fw != 0, extent); r.nbuf = (uint32_t)hi;
				stage_rec[(size_t)nrec * 64 + lane] = r;
				break;
			}
			if(aborted) break;
			if(!found) {
				bt2x_aln_rec r;
				r.ntries = (uint16_t)ntries; r.ok = 0; r.pad0 = 0; r.score = 0; r.ns = 0; r.gaps = 0;
				r.nedit = 0; r.bases_aligned = 0; r.refns = 0; r.refoff = 0;
				r.edit_off = publish_edbuf(a, stage_ed, lane, hi, rd, rf); r.nbuf = (uint32_t)hi;
				stage_rec[(size_t)nrec * 64 + lane] = r;
				nrec++;
				break;
			}
			nrec++;
		}
		if(aborted) {                                 // the wave kernel redoes the whole call
			a.heavy_list[1 + atomicAdd(&a.heavy_list[0], 1u)] = pi;
			return;
		}
		const uint32_t ro = atomicAdd(&a.counters[0], (uint32_t)nrec);
		if(ro + (uint32_t)nrec <= a.rec_cap)
			for(int k = 0; k < nrec; k++) a.recs[ro + k] = stage_rec[(size_t)k * 64 + lane];
		o.nrec = (uint16_t)nrec; o.rec_off = ro;
		a.out[pi] = o;
	}
}

// ------------------------------------------------------- wave-per-problem mode
// The aligner's DP rounds end in a tail of small launches (the few reads that need many
// rounds): there one lane per problem leaves the chip idle and a launch still costs the
// R x C serial cell updates of one lane, ~1.5-6 ms.  This mode gives each problem a whole
// wave.  Lane l owns rows rpl*l .. rpl*l + rpl - 1 (rpl = 1..4 rows a lane, the fewest
// that fit; 4 until round 6) and the wave sweeps anti-diagonals: at time t lane l computes
// column t - l, taking the H and F of the row above from lane l-1 (one DPP wave_shr), so a
// problem takes C + R/rpl - 1 steps of rpl cells.  Values and flags are the lane kernel's
// (same recurrence and traceback byte); the traceback bytes stay in LDS, column-major with
// a lane's rows in one dword (or banded, below), and the walk reads and marks them at LDS
// latency.
// Cells are plain u32 here, so one body serves both value domains: u8 (top 0xff) and
// i16 (the int16 range shifted to [0, 0xffff]: top 0xffff = score 0, floor 0 = -65535);
// barred gap terms subtract 0x10000, which floors either domain.
constexpr int kWaveTbWords = kCols * kRows / 4;              // 8000 dwords = 31.25 KiB
constexpr size_t kWaveRecStageBytes = (size_t)kRecStage * sizeof(bt2x_aln_rec);
// Banded traceback in LDS (round 6).  Every walk stays inside the diagonal band of
// dp_fill_kernel (a path scoring >= minsc pays for at most G gap positions), so the wave
// kernel keeps only the band's bytes: lane l's rows over its window of columns
// [ws(l), ws(l) + P) with ws(l) = max(0, rpl*l - dl), P dwords a lane (lane-major).  The
// values are still the whole rectangle's (every cell is computed), only the bytes no walk
// can reach are not stored.  19 KiB holds the 150 bp / --dpad 12 band at 3 rows a lane
// (50 lanes x 97 dwords) and whole short-read rectangles (lanes x ncol <= 4864); the
// kernel's LDS then fits 7 waves per CU instead of 4.  A problem whose window does not fit
// goes to the full-rectangle pass (dp_wave_kernel<2>).
constexpr int kWaveBandWords = 4864;                          // 19 KiB

// Traceback byte offsets in LDS: full rectangle (column-major, S bytes a column, a lane's 4
// rows in one dword) or the banded layout above (P4 = 4P bytes a lane).
template<bool kBand> struct TbMap;
// Lane l holds rows [rpl*l, rpl*l + rpl) (row / rpl by a multiply: mul = ceil(2^16 / rpl),
// exact for rows < 192).
template<> struct TbMap<false> {
	int S, rpl, mul;
	__device__ __forceinline__ int operator()(int row, int col) const {
		const int l = (row * mul) >> 16;
		return col * S + 4 * l + (row - l * rpl);
	}
};
template<> struct TbMap<true> {
	int P4, dl, rpl, mul;
	__device__ __forceinline__ int operator()(int row, int col) const {
		const int l = (row * mul) >> 16;
		const int ws = rpl * l - dl > 0 ? rpl * l - dl : 0;
		return l * P4 + ((col - ws) << 2) + (row - l * rpl);
	}
};

__device__ __forceinline__ uint32_t subs(uint32_t a, uint32_t b) { return a > b ? a - b : 0u; }

// align()'s verdict from the last row's maximum lrmax (top-relative value) and the
// number of candidates: alignEnd2EndSseU8 (aligner_swsse_ee_u8.cpp:637-668) and
// alignEnd2EndSseI16 (aligner_swsse_ee_i16.cpp:642-673; its "score" subtracts 0xff from
// the int16 value, so it is lrmax - 0x8000 - 0xff here).
__device__ __forceinline__ void dp_verdict(bool i16, int lrmax, int minsc, int ncand, int& status, int& best) {
	const int score = lrmax - (i16 ? 0x80ff : 0xff);
	if(score < minsc) { status = 0; best = score; }
	else if(lrmax == 0) { status = 0; best = INT32_MIN; }       // saturated (MIN_U8 / MIN_I16)
	else { status = ncand > 0 ? 1 : 0; best = score; }
}

// ------------------------------------------------ the nextAlignment sequence, wave-parallel
// SwAligner::nextAlignment until done() (aligner_sw.cpp:252-375) over a problem whose
// traceback bytes are in LDS (tbb: column-major, S bytes per column), with all 64 lanes.
// A backtrace (u8.cpp:746-1352) is a chain of dependent steps: the serial walk costs one
// LDS round trip per step, and a repeat's candidates, walked one after another, reach
// tens of thousands of steps.  Here:
//  * Free paths, kParBatch candidates at a time, one per lane: the moves depend only on
//    the cells' flags (never on marks), so each candidate's path from its start cell is
//    walked independently, up to row 0 or to a cell marked by an attempt already
//    validated (none of this batch marks anything).  Cells are kept as (row, col) u16.
//  * Validation in DpBtCandidate order, all lanes on one attempt, 64 cells per round: the
//    reference's attempt k walks its path until the first cell some earlier attempt
//    marked (reportedThrough; a marked start cell: skipped, no RNG draw) or to row 0.  A
//    ballot over the chunk's marks finds that cell; the walked cells are marked, their
//    edits (the move to the path's next cell: diagonal with TB_MM, F up = ref gap, E left
//    = read gap; open/extend from the cell's own E/F flag) are staged by prefix count,
//    and score, N count, gaps and the core-diagonal test are lane sums.
// Every mark, record, edit-buffer image and ntries equals the serial walk's: the same
// attempts walk the same cells in the same order; only the order of marking within one
// attempt differs, and no attempt reads its own cells.
constexpr int kParBatch = 56;
constexpr int kPathStride = 362;      // u16 cells per path (>= kRows + kCols - 1); 181 dwords: odd
constexpr size_t kParPathBytes = (size_t)kParBatch * kPathStride * 2;

__device__ __forceinline__ int wave_sum(int v) {
	for(int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
	return v;
}

template<class TbM>
__device__ __forceinline__ void walk_wave_par(const DevScoring& sc, const DpLaunch& a, const bt2x_dp_in& p,
                                              bt2x_dp_out& o, int lane, uint8_t* tbb, const TbM& tm, const uint8_t* cands,
                                              const uint8_t* rdw, const uint16_t* penw, const uint8_t* refw,
                                              uint32_t* stage_ed, bt2x_aln_rec* stage_rec, uint16_t* path,
                                              uint16_t* plen, unsigned long long& st_bt) {
	const int R = p.rdlen, row0 = R - 1, ncand = o.ncand;
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;
	const uint64_t lt = (1ull << lane) - 1ull;
	int ndone = 0, nrec = 0, b0 = 0, bn = 0;
	while(ndone < ncand) {
		int ntries = 0, hi = 0;
		bool found = false;
		while(ndone < ncand) {
			const int k = ndone++;
			if(k >= b0 + bn) {
				// ---- free paths of candidates [k, k + nb)
				const int nb = min(kParBatch, ncand - k);
				if(lane < nb) {
					int row = row0, col = cands[k + lane], ct = 2, n = 0;
					uint16_t* pp = path + lane * kPathStride;
					while(true) {
						const uint32_t tb = tbb[tm(row, col)];
						pp[n++] = (uint16_t)(row | (col << 8));
						if((tb & TB_MARK) || row == 0) break;
						const uint32_t dne = tb & TB_DNE, fne = (tb >> 1) & 1u;
						const uint32_t fext = (tb >> 2) & 1u, eext = (tb >> 3) & 1u;
						const bool inH = ct == 2;
						const bool isD = inH && !dne;
						const bool isF = (ct == 1) || (inH && dne && !fne);
						ct = isD ? 2 : isF ? (fext ? 1 : 2) : (eext ? 0 : 2);
						row -= (isD || isF) ? 1 : 0;
						col -= isF ? 0 : 1;
					}
					plen[lane] = (uint16_t)n;
				}
				b0 = k; bn = nb;
				__syncthreads();
			}
			const int len = (int)uni(plen[k - b0]);
			const uint16_t* pk = path + (k - b0) * kPathStride;
			if(a.ablate == 2) {                                   // profiling: no backtrace walks
				if(!(uni(tbb[tm(pk[0] & 0xff, pk[0] >> 8)]) & TB_MARK)) ntries++;
				continue;
			}
			// ---- validation: attempt k over its path, 64 cells per round
			int ne = 0, walked = 0;
			bool stopped = false, skip = false, termMM = false;
			bool over = false;
			int pen_l = 0, ns_l = 0, gaps_l = 0;
			for(int c0 = 0; c0 < len; c0 += 64) {
				const int idx = c0 + lane;
				const bool v = idx < len;
				const uint32_t cell = v ? pk[idx] : 0u;
				const int row = (int)(cell & 0xffu), col = (int)(cell >> 8);
				const int off = v ? tm(row, col) : 0;
				const uint32_t tb = v ? tbb[off] : 0u;
				const uint64_t mk = __builtin_amdgcn_ballot_w64(v && (tb & TB_MARK));
				if(c0 == 0 && (mk & 1ull)) { skip = true; break; }      // start cell reportedThrough
				const int nwk = mk ? (int)__builtin_ctzll(mk) : min(64, len - c0);
				const bool w = lane < nwk;
				const uint32_t ncell = (w && idx + 1 < len) ? pk[idx + 1] : cell;
				const int nrow = (int)(ncell & 0xffu), ncl = (int)(ncell >> 8);
				const bool term = w && row == 0;                       // a completed path's last cell
				const bool isD = nrow != row && ncl != col, isF = nrow != row && ncl == col;
				const bool mmE = w && !term && isD && (tb & TB_MM);
				const bool gapE = w && !term && !isD;
				const uint64_t eb = __builtin_amdgcn_ballot_w64(mmE || gapE);
				if(mmE || gapE) {
					const int pos = ne + (int)__builtin_popcountll(eb & lt);
					stage_ed[pos] = mmE ? pack_edit((uint32_t)row, EDIT_MM, mask_chr(refw[col]), acgtn(rdw[row]))
					              : isF ? pack_edit((uint32_t)row, EDIT_REF_GAP, '-', acgtn(rdw[row]))
					                    : pack_edit((uint32_t)row + 1, EDIT_READ_GAP, mask_chr(refw[col]), '-');
				}
				ne += (int)__builtin_popcountll(eb);
				if(w) {
					const int diag = col - row + (int)p.triml;
					over |= (diag >= 0) & (diag >= (int)p.corel) & (diag <= (int)p.corer);
					if(mmE) {
						const bool amb = rdw[row] > 3 || refw[col] > 3;
						pen_l += amb ? npen : (int)penw[row];
						ns_l += amb ? 1 : 0;
					}
					if(gapE) {
						const bool open = isF ? !(tb & TB_FONE) : !(tb & TB_EONE);
						pen_l += isF ? (open ? rfo : rfe) : (open ? rdo : rde);
						gaps_l++;
					}
					if(term) termMM = (tb & TB_MM) != 0;
					tbb[off] = (uint8_t)TB_MARK;                           // setReportedThrough
				}
				walked += nwk;
				if(mk) { stopped = true; break; }
			}
			__syncthreads();                                          // the marks, for the next attempt
			if(skip) continue;
			ntries++;
			st_bt += (unsigned long long)(walked + (stopped ? 1 : 0));
			if(stopped) { hi = max(hi, ne); continue; }
			if(__builtin_amdgcn_ballot_w64(over) == 0) { hi = max(hi, ne); continue; }
			// the final (row 0) cell's mismatch
			const uint32_t tcell = uni(pk[len - 1]);
			const int tcol = (int)(tcell >> 8);
			termMM = __builtin_amdgcn_ballot_w64(termMM) != 0;
			int bscore = -wave_sum(pen_l), ns = wave_sum(ns_l);
			const int gaps = wave_sum(gaps_l);
			if(termMM) {
				const int rdc = (int)uni(rdw[0]), refc = (int)uni(refw[tcol]);
				const bool amb = rdc > 3 || refc > 3;
				if(lane == 0) stage_ed[ne] = pack_edit(0u, EDIT_MM, mask_chr(refc), acgtn(rdc));
				ne++;
				bscore -= amb ? npen : (int)uni(penw[0]);
				ns += amb ? 1 : 0;
			}
			if(ns > p.nceil) { hi = max(hi, ne); __syncthreads(); continue; }
			// reference Ns under the alignment: columns [tcol, col0]
			const int col0 = (int)(uni(pk[0]) >> 8);
			int refns = 0;
			for(int c = tcol + lane; c <= col0; c += 64) refns += refw[c] > 3 ? 1 : 0;
			refns = wave_sum(refns);
			const int extent = R;
			hi = max(hi, ne);
			found = true;
			__syncthreads();
			// ned() order of the alignment's own entries [0, ne), in place: reverse (fw) or
			// mirror positions (rc, invertEdits, edit.cpp:50-78)
			uint32_t ev[(kEditStage + 63) / 64];
#pragma unroll
			for(int q = 0; q < (kEditStage + 63) / 64; q++) {
				const int i = q * 64 + lane;
				ev[q] = 0;
				if(i < ne) {
					uint32_t e = stage_ed[p.fw ? ne - 1 - i : i];
					if(!p.fw) {
						const uint32_t pos = (uint32_t)extent - (e & 0x3ffu) - (((e >> 12) & 7u) == EDIT_READ_GAP ? 0u : 1u);
						e = (e & ~0x3ffu) | (pos & 0x3ffu);
					}
					ev[q] = e;
				}
			}
			__syncthreads();
#pragma unroll
			for(int q = 0; q < (kEditStage + 63) / 64; q++) {
				const int i = q * 64 + lane;
				if(i < ne) stage_ed[i] = ev[q];
			}
			__syncthreads();
			uint32_t eo = 0;
			if(hi > 0) {
				if(lane == 0) eo = atomicAdd(&a.counters[1], (uint32_t)hi);
				eo = uni(eo);
				if(eo + (uint32_t)hi <= a.edit_cap) for(int i = lane; i < hi; i += 64) a.edits[eo + i] = stage_ed[i];
			}
			if(lane == 0) {
				bt2x_aln_rec r;
				r.ntries = (uint16_t)ntries; r.ok = 1; r.pad0 = 0;
				r.score = (int16_t)bscore; r.ns = (uint16_t)ns; r.gaps = (uint16_t)gaps;
				r.nedit = (uint16_t)ne; r.bases_aligned = (uint16_t)(extent - ne);
				r.refns = (uint16_t)refns; r.refoff = (int64_t)tcol + p.refl;
				r.edit_off = eo; r.nbuf = (uint32_t)hi;
				stage_rec[nrec] = r;
			}
			break;
		}
		if(!found) {
			uint32_t eo = 0;
			if(hi > 0) {
				if(lane == 0) eo = atomicAdd(&a.counters[1], (uint32_t)hi);
				eo = uni(eo);
				if(eo + (uint32_t)hi <= a.edit_cap) for(int i = lane; i < hi; i += 64) a.edits[eo + i] = stage_ed[i];
			}
			if(lane == 0) {
				bt2x_aln_rec r;
				r.ntries = (uint16_t)ntries; r.ok = 0; r.pad0 = 0; r.score = 0; r.ns = 0; r.gaps = 0;
				r.nedit = 0; r.bases_aligned = 0; r.refns = 0; r.refoff = 0;
				r.edit_off = eo; r.nbuf = (uint32_t)hi;
				stage_rec[nrec] = r;
			}
			nrec++;
			break;
		}
		nrec++;
	}
	uint32_t ro = 0;
	if(lane == 0) ro = atomicAdd(&a.counters[0], (uint32_t)nrec);
	ro = uni(ro);
	__syncthreads();                                                  // stage_rec (lane 0's stores)
	if(ro + (uint32_t)nrec <= a.rec_cap) for(int i = lane; i < nrec; i += 64) a.recs[ro + i] = stage_rec[i];
	o.nrec = (uint16_t)nrec; o.rec_off = ro;
}

// kMode 0: every problem of the launch.  kMode 1 (kBestOnly): the exact `best` of the
// problems the banded lane kernel failed (a.fail_list[0 .. a.counters[2])): the whole
// rectangle's last-row maximum, nothing else.  kMode 2: the problems the lane kernel handed
// over after its fill (a.heavy_list): the whole call, their walks at LDS latency.
// kPar: the nextAlignment sequence with every lane (walk_wave_par) instead of lane 0.
// kBandTb (modes 0 and 2): the banded traceback layout; in mode 0 within kWaveBandWords (a
// problem whose window does not fit goes to mode 2), in mode 2 within kWaveTbWords, which
// holds any problem (at worst the whole rectangle, lane-major, 4 rows a lane).  Mode 0 hands
// problems over on a.heavy_list; it must be followed by the mode-2 pass.
template<int kMode, bool kPar = false, bool kBandTb = false>
__global__ void __launch_bounds__(64)
dp_wave_kernel(DevScoring sc, DpLaunch a) {
	constexpr bool kBestOnly = kMode == 1;
	static_assert(!kBandTb || kMode != 1, "banded traceback: modes 0 and 2");
	constexpr int kTbWords = (kBandTb && kMode == 0) ? kWaveBandWords : kWaveTbWords;
	__shared__ uint32_t tbw[kBestOnly ? 1 : kTbWords];
	__shared__ uint16_t pathw[kPar ? kParBatch * kPathStride : 1];
	__shared__ uint16_t plenw[kPar ? kParBatch : 1];
	__shared__ uint8_t refw[kCols], cands[kCols];
	__shared__ uint16_t lastrow[kCols];
	__shared__ uint32_t stage_ed[kBestOnly ? 1 : kEditStage];
	// the walk's read codes and per-row mismatch penalties (quality -> mmpen), at LDS latency
	__shared__ uint8_t rdw[kBestOnly ? 1 : kRows];
	__shared__ uint16_t penw[kBestOnly ? 1 : kRows];
	uint8_t* tbb = reinterpret_cast<uint8_t*>(tbw);
	const int lane = threadIdx.x;
	bt2x_aln_rec* stage_rec = kBestOnly ? nullptr : reinterpret_cast<bt2x_aln_rec*>(a.scratch + (size_t)blockIdx.x * kWaveRecStageBytes);
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0;
	const uint32_t rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;
	const uint32_t nwork = kMode == 1 ? min(a.counters[2], a.n) : kMode == 2 ? min(a.heavy_list[0], a.n) : a.n;
	for(uint32_t k = blockIdx.x; k < nwork; k += gridDim.x) {
		const uint32_t pi = kMode == 1 ? a.fail_list[k] : kMode == 2 ? a.heavy_list[1 + k] : k;
		const bt2x_dp_in p = a.in[pi];
		if(kMode == 0 && (p.flags & kDpBadWindow)) {             // refused (window_kernel)
			if(lane == 0) {
				bt2x_dp_out o;
				o.nrec = 0; o.rec_off = 0; o.status = -1; o.best = 0; o.ncand = 0;
				a.out[pi] = o;
				atomicAdd(&a.counters[3], 1u);
			}
			continue;
		}
		const int R = p.rdlen, C = p.ncol;
		const bool i16 = (p.flags & BT2X_DP_I16) != 0;
		const uint32_t top = i16 ? 0xffffu : 0xffu;
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		// Rows per lane: the fewest that fit 64 lanes (3 at 150 bp, 2 at 100 bp: a problem takes
		// C + R/rpl - 1 steps of rpl cells, so fewer rows per lane shorten its chain) and whose
		// traceback fits the LDS layout; else the next.  Lane l holds rows [rpl*l, rpl*l + rpl),
		// their bytes in the low rpl bytes of its dword.
		int rpl = (R + 63) >> 6;
		rpl = rpl < 1 ? 1 : rpl;
		int P = 0, dlw = 0, dhw = 0;                // banded layout: window P dwords a lane
		if(kBandTb) {
			// dp_fill_kernel's band (diagonals [-dl, dh])
			const int mo = imax(1, (int)(rdo < rfo ? rdo : rfo));
			int me = (int)(rde < rfe ? rde : rfe);
			me = me < mo ? me : mo;
			const int budget = -(int)p.minsc;
			int G = (me <= 0) ? (1 << 16) : (budget < mo ? 0 : 1 + (budget - mo) / me);
			G = G > (1 << 16) ? (1 << 16) : G;
			dhw = (C - R) + G + 2;
			dlw = G + 4;
		}
		for(; rpl <= 4; rpl++) {
			const int Lr = (R + rpl - 1) / rpl;
			if(kBestOnly) break;
			if(!kBandTb) { if(Lr * C <= kWaveTbWords) break; continue; }
			int wc = dhw + dlw + rpl;               // columns of lane l's rows: [rpl*l - dl, rpl*l + rpl - 1 + dh]
			wc = wc < C ? wc : C;
			P = wc + ((wc ^ rpl) & 1);              // P = rpl mod 2: conflict-free fill stores (stride P - 1 - rpl)
			if(Lr * P <= kTbWords) break;
		}
		if(kBandTb && kMode == 0 && rpl > 4) {      // does not fit: the full-rectangle pass
			if(lane == 0) {
				a.heavy_list[1 + atomicAdd(&a.heavy_list[0], 1u)] = pi;
				if(a.stats) { st_cells += (unsigned long long)R * C; st_cols += C; }
			}
			continue;
		}
		const int L = (R + rpl - 1) / rpl;          // lanes holding rows
		const int S = 4 * L;                        // bytes per traceback column (full layout)
		for(int j = lane; j < C; j += 64) refw[j] = rf[j];
		if(!kBestOnly)
			for(int i = lane; i < R; i += 64) {
				const int q0 = (int)qu[i] - 33;
				rdw[i] = rd[i];
				penw[i] = (uint16_t)a.mmpen[q0 < 0 ? 0 : (q0 > 255 ? 255 : q0)];
			}
		// this lane's rows: read code (7 = N), mismatch penalty, gap-barred open/extend
		uint32_t rc[4], mm[4], rdoe[4], rfoe[4], rfee[4];
#pragma unroll
		for(int r = 0; r < 4; r++) {
			const int i = rpl * lane + r;
			uint32_t c = 7, m = npen;
			bool gbar = true;
			if(r < rpl && i < R) {
				int q = (int)qu[i] - 33;
				q = q < 0 ? 0 : (q > 255 ? 255 : q);
				gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
				const int b = rd[i];
				if(b <= 3) { c = (uint32_t)b; m = (uint32_t)a.mmpen[q]; }
			}
			rc[r] = c; mm[r] = m;
			const uint32_t bar = gbar ? 0x10000u : 0u, r0 = (i == 0) ? 0x10000u : 0u;   // row 0 has no F
			rdoe[r] = rdo + bar; rfoe[r] = rfo + bar + r0; rfee[r] = rfe + bar + r0;
		}
		__syncthreads();
		// ---- fill: H/E of the previous column for my rows; H[i][-1] = E = floor, H[-1][*] = top
		uint32_t Hp0 = 0, Hp1 = 0, Hp2 = 0, Hp3 = 0, Ep0 = 0, Ep1 = 0, Ep2 = 0, Ep3 = 0;
		uint32_t hupPrev = lane == 0 ? top : 0u;    // H[rpl*l-1][j-1]
		uint32_t bot = 0;                           // my bottom row's H | F << 16, last column
		const int lastLane = (R - 1) / rpl, lastR = (R - 1) - lastLane * rpl;
		const int wsl = imax(0, rpl * lane - dlw);  // banded layout: my window's first column
		const int T = C + L - 1;
		for(int t = 0; t < T; t++) {
			const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bot, 0x138, 0xf, 0xf, false);
			const int j = t - lane;
			if(lane < L && j >= 0 && j < C) {
				uint32_t hu = lane == 0 ? top : (up & 0xffffu);
				uint32_t fu = lane == 0 ? 0u : (up >> 16);
				uint32_t hdiag = hupPrev;
				hupPrev = hu;
				const uint32_t refc = refw[j];
				const bool refN = refc > 3;
				uint32_t tbv = 0;
#define BT2X_WAVE_CELL(r, HP, EP)                                                               \
				{                                                                               \
					const uint32_t x = rc[r] ^ refc;                                            \
					const uint32_t pen = refN ? npen : (x ? mm[r] : 0u);                        \
					const uint32_t d = subs(hdiag, pen);                                        \
					const uint32_t hl_o = subs(HP, rdoe[r]), e = max(hl_o, subs(EP, rde));      \
					const uint32_t hu_o = subs(hu, rfoe[r]), f = max(hu_o, subs(fu, rfee[r]));  \
					const uint32_t h = max(max(d, e), f);                                       \
					if(!kBestOnly) {                                                            \
						const uint32_t tb = (x ? (uint32_t)TB_MM : 0u) | (hl_o != e ? (uint32_t)TB_EONE : 0u) | \
						                    (hu_o != f ? (uint32_t)TB_FONE : 0u) | (f != h ? (uint32_t)TB_FNE : 0u) | \
						                    (d != h ? (uint32_t)TB_DNE : 0u);                       \
						tbv |= tb << (8 * r);                                                   \
					}                                                                           \
					hdiag = HP; HP = h; EP = e; hu = h; fu = f;                                 \
				}
				// (rpl is wave-uniform: scalar branches)
				BT2X_WAVE_CELL(0, Hp0, Ep0)
				if(rpl > 1) BT2X_WAVE_CELL(1, Hp1, Ep1)
				if(rpl > 2) BT2X_WAVE_CELL(2, Hp2, Ep2)
				if(rpl > 3) BT2X_WAVE_CELL(3, Hp3, Ep3)
#undef BT2X_WAVE_CELL
				if(kBandTb) {
					const int w = j - wsl;
					if((unsigned)w < (unsigned)P) tbw[lane * P + w] = tbv;
				} else if(!kBestOnly) tbw[j * L + lane] = tbv;
				bot = hu | (fu << 16);
				if(lane == lastLane)
					lastrow[j] = (uint16_t)(lastR == 0 ? Hp0 : lastR == 1 ? Hp1 : lastR == 2 ? Hp2 : Hp3);
			}
		}
		__syncthreads();
		// ---- best score, candidates in DpBtCandidate order (score desc, col desc)
		const int thr = (int)p.minsc + (int)top;
		int lrmax = 0, nc = 0;
		for(int j = lane; j < C; j += 64) { const int v = lastrow[j]; lrmax = imax(lrmax, v); nc += v >= thr; }
		lrmax = wave_max(lrmax);
		for(int d = 32; d > 0; d >>= 1) nc += __shfl_xor(nc, d);
		int status = 0, best = 0;
		dp_verdict(i16, lrmax, p.minsc, nc, status, best);
		if(kBestOnly) {
			if(lane == 0) a.out[pi].best = best;
			__syncthreads();
			continue;
		}
		if(kMode == 0) { st_cells += (unsigned long long)R * C; st_cols += C; }   // (mode 2: the lane kernel counted them)
		// banded layout, lane-0 walk: a problem of many candidates (a repeat's: their walks
		// one after another, 2.4 ms for one such launch of 1,025 problems) is redone by
		// dp_wave_kernel<2>, whose walk runs on every lane (0.37 ms; round 6)
		if(kMode == 0 && kBandTb && !kPar && status && a.wave_hand && (uint32_t)nc >= a.wave_hand && a.ablate != 1) {
			if(lane == 0) a.heavy_list[1 + atomicAdd(&a.heavy_list[0], 1u)] = pi;
			__syncthreads();
			continue;
		}
		bt2x_dp_out o;
		o.nrec = 0; o.rec_off = 0;
		o.status = status; o.best = best; o.ncand = status ? (uint16_t)nc : (uint16_t)0;
		if(!status) {
			if(lane == 0) a.out[pi] = o;
			__syncthreads();
			continue;
		}
		for(int j = lane; j < C; j += 64) {
			const int v = lastrow[j];
			if(v < thr) continue;
			const int key = (v << 8) | j;
			int rank = 0;
			for(int k2 = 0; k2 < C; k2++) { const int w = lastrow[k2]; rank += ((w << 8) | k2) > key; }
			cands[rank] = (uint8_t)j;
		}
		__syncthreads();
		TbMap<kBandTb> tm;
		if constexpr(kBandTb) { tm.P4 = 4 * P; tm.dl = dlw; } else { tm.S = S; }
		tm.rpl = rpl; tm.mul = (65536 + rpl - 1) / rpl;
		if(kPar) {
			if(o.status != 0 && o.ncand > 0 && a.ablate != 1)
				walk_wave_par(sc, a, p, o, lane, tbb, tm, cands, rdw, penw, refw, stage_ed, stage_rec, pathw, plenw, st_bt);
			if(lane == 0) a.out[pi] = o;
			__syncthreads();
			continue;
		}
		// ---- SwAligner::nextAlignment until done(), on lane 0 (see walk_problem).  Every
		// value read from LDS is made wave-uniform (readfirstlane), so the walk's arithmetic
		// runs on the scalar unit: one chain of LDS round trips and SALU ops per step.
		if(lane == 0) {
			if(o.status != 0 && o.ncand > 0 && a.ablate != 1) {
				const int rdo_ = sc.rdo, rde_ = sc.rde, rfo_ = sc.rfo, rfe_ = sc.rfe;
				const int ncand = o.ncand, row0 = R - 1;
				int ndone = 0, nrec = 0;
				while(ndone < ncand) {
					int ntries = 0, hi = 0;
					bool found = false;
					while(ndone < ncand) {
						const int col0 = (int)uni(cands[ndone]);
						ndone++;
						if(uni(tbb[tm(row0, col0)]) & TB_MARK) continue;
						ntries++;
						if(a.ablate == 2) continue;
						int row = row0, col = col0, ct = 2, bscore = 0, ns = 0, gaps = 0, ne = 0;
						bool over_core = false, ok = true;
						uint32_t tb_end = 0;
						int bo = tm(row, col);
						uint32_t tb = uni(tbb[bo]);
						while(true) {
							st_bt++;
							if(tb & TB_MARK) { ok = false; break; }
							const int diag = col - row + (int)p.triml;
							over_core |= (diag >= 0) & (diag >= (int)p.corel) & (diag <= (int)p.corer);
							if(row == 0) { tbb[bo] = (uint8_t)TB_MARK; tb_end = tb; break; }
							const uint32_t dne = tb & TB_DNE, fne = (tb >> 1) & 1u;
							const uint32_t fext = (tb >> 2) & 1u, eext = (tb >> 3) & 1u;
							const bool inH = ct == 2;
							const bool isD = inH && !dne;
							const bool isF = (ct == 1) || (inH && dne && !fne);
							const int nct = isD ? 2 : isF ? (fext ? 1 : 2) : (eext ? 0 : 2);
							const int cbo = bo;
							const int crow = row, ccol = col;
							row -= (isD || isF) ? 1 : 0; col -= isF ? 0 : 1; ct = nct;
							bo = tm(row, col);
							const uint32_t ctb = tb;
							tb = uni(tbb[bo]);
							tbb[cbo] = (uint8_t)TB_MARK;               // setReportedThrough
							if(isD) {
								if(ctb & TB_MM) {
									const int rdc = (int)uni(rdw[crow]), refc = (int)uni(refw[ccol]);
									const bool amb = rdc > 3 || refc > 3;
									stage_ed[ne++] = pack_edit((uint32_t)crow, EDIT_MM, mask_chr(refc), acgtn(rdc));
									bscore -= amb ? sc.npen : (int)uni(penw[crow]);
									if(amb) ns++;
								}
							} else {
								const bool open = nct == 2;
								stage_ed[ne++] = isF ? pack_edit((uint32_t)crow, EDIT_REF_GAP, '-', acgtn((int)uni(rdw[crow])))
								                     : pack_edit((uint32_t)crow + 1, EDIT_READ_GAP, mask_chr((int)uni(refw[ccol])), '-');
								bscore -= isF ? (open ? rfo_ : rfe_) : (open ? rdo_ : rde_);
								gaps++;
							}
						}
						if(!ok || !over_core) { hi = max(hi, ne); continue; }
						if(tb_end & TB_MM) {
							const int rdc = (int)uni(rdw[row]), refc = (int)uni(refw[col]);
							const bool amb = rdc > 3 || refc > 3;
							stage_ed[ne++] = pack_edit((uint32_t)row, EDIT_MM, mask_chr(refc), acgtn(rdc));
							bscore -= amb ? sc.npen : (int)uni(penw[row]);
							if(amb) ns++;
						}
						if(ns > p.nceil) { hi = max(hi, ne); continue; }
						int refns = 0;
						for(int k2 = col; k2 <= col0; k2++) refns += (uni(refw[k2]) > 3);
						const int extent = R - (R - row0 - 1);
						if(p.fw) {
							for(int k2 = 0; k2 < ne / 2; k2++) {
								const uint32_t x = stage_ed[k2];
								stage_ed[k2] = stage_ed[ne - 1 - k2];
								stage_ed[ne - 1 - k2] = x;
							}
						} else {
							for(int k2 = 0; k2 < ne; k2++) {
								const uint32_t e = stage_ed[k2];
								const uint32_t pos = (uint32_t)extent - (e & 0x3ffu) - (((e >> 12) & 7u) == EDIT_READ_GAP ? 0u : 1u);
								stage_ed[k2] = (e & ~0x3ffu) | (pos & 0x3ffu);
							}
						}
						hi = max(hi, ne);
						found = true;
						bt2x_aln_rec r;
						r.ntries = (uint16_t)ntries; r.ok = 1; r.pad0 = 0;
						r.score = (int16_t)bscore; r.ns = (uint16_t)ns; r.gaps = (uint16_t)gaps;
						r.nedit = (uint16_t)ne; r.bases_aligned = (uint16_t)(extent - ne);
						r.refns = (uint16_t)refns; r.refoff = (int64_t)col + p.refl;
						uint32_t eo = 0;
						if(hi > 0) {
							eo = atomicAdd(&a.counters[1], (uint32_t)hi);
							if(eo + (uint32_t)hi <= a.edit_cap) for(int k2 = 0; k2 < hi; k2++) a.edits[eo + k2] = stage_ed[k2];
						}
						r.edit_off = eo; r.nbuf = (uint32_t)hi;
						stage_rec[nrec] = r;
						break;
					}
					if(!found) {
						bt2x_aln_rec r;
						r.ntries = (uint16_t)ntries; r.ok = 0; r.pad0 = 0; r.score = 0; r.ns = 0; r.gaps = 0;
						r.nedit = 0; r.bases_aligned = 0; r.refns = 0; r.refoff = 0;
						uint32_t eo = 0;
						if(hi > 0) {
							eo = atomicAdd(&a.counters[1], (uint32_t)hi);
							if(eo + (uint32_t)hi <= a.edit_cap) for(int k2 = 0; k2 < hi; k2++) a.edits[eo + k2] = stage_ed[k2];
						}
						r.edit_off = eo; r.nbuf = (uint32_t)hi;
						stage_rec[nrec] = r;
						nrec++;
						break;
					}
					nrec++;
				}
				const uint32_t ro = atomicAdd(&a.counters[0], (uint32_t)nrec);
				if(ro + (uint32_t)nrec <= a.rec_cap)
					for(int k2 = 0; k2 < nrec; k2++) a.recs[ro + k2] = stage_rec[k2];
				o.nrec = (uint16_t)nrec; o.rec_off = ro;
			}
			a.out[pi] = o;
		}
		__syncthreads();
	}
	if(!kBestOnly && a.stats && lane == 0) {
		if(kMode == 0) {
			atomicAdd(&a.stats[0], st_cells);
			atomicAdd(&a.stats[1], st_cols);
			atomicAdd(&a.stats[3], st_cells);          // whole rectangles
		}
		atomicAdd(&a.stats[2], st_bt);
	}
}

// kFused: the same wave walks its 64 problems right after their fill, while the
// traceback bytes are still in the Infinity Cache; slots are per resident wave.
// kWide: the 16-bit value domain (launches holding BT2X_DP_I16 problems, the reference's
// alignEnd2EndSseI16): the same sweep with 16-bit row state (2 rows per dword, 80 + 80
// VGPRs, so 2 waves/SIMD instead of 3), a per-lane top value (0xff for u8 problems,
// 0xffff for i16 ones: the int16 range shifted by 0x8000), barred gap terms masked to
// the floor, and 16-bit last rows.  Flags, candidates and the walk are unchanged: every
// traceback test is an equality between a cell on a path scoring >= minsc and a
// neighbour term, identical in both domains (aligner_swsse_ee_i16.cpp:746-1352 is the
// u8 backtrace over int16 cells).
template<bool kDebug, bool kFused, bool kWide>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kWide ? 2 : 3)))
dp_fill_kernel(DevScoring sc, DpLaunch a, uint32_t base, uint32_t nprob) {
	// LDS: the row info during the fill, then the last DP row (4 column keys per dword)
	// for candidate ordering.  12.8 KiB per wave.
	__shared__ uint32_t lds[(kCols / 4) * 64];
	// the mismatch penalty by quality (DevScoring::mmpen), looked up per lane and row
	__shared__ uint32_t pen4[64];
	const uint8_t* pen_lds = reinterpret_cast<const uint8_t*>(pen4);
	constexpr int kStateWords = kWide ? kRows / 2 : kRowWords;   // H/E state dwords per lane
	const int lane = threadIdx.x;
	pen4[lane] = reinterpret_cast<const uint32_t*>(a.mmpen)[lane];
	__syncthreads();
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0, st_comp = 0;
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;
	const uint32_t one2 = opaque(0x00010001u);

	unsigned long long pw_steps = 0, pw_iters = 0, t_fill = 0, t_walk = 0, ngrp = 0;     // BT2X_DP_PROF
	unsigned long long mx_fill = 0, mx_walk = 0, mylen_sum = 0, mylen_max = 0;
	unsigned long long t_pro = 0, t_pair = 0, t_cand = 0;
	const unsigned long long t_start = a.prof ? __builtin_amdgcn_s_memtime() : 0;
	for(uint32_t grp = blockIdx.x; (uint64_t)grp * 64 < nprob; grp += gridDim.x) {
		const unsigned long long t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
		uint8_t* gslot = kFused ? a.scratch + (size_t)blockIdx.x * (kGroupBytes + kWalkSlotBytes)
		                        : a.scratch + (size_t)grp * kGroupBytes;
		uint32_t* dir = reinterpret_cast<uint32_t*>(gslot + kDirOff);
		uint8_t* lastrow = gslot + kLastRowOff;
		uint16_t* lastrow16 = reinterpret_cast<uint16_t*>(gslot + kLastRowOff);
		uint8_t* cands = gslot + kCandOff;
		const uint32_t pi = base + grp * 64 + lane;
		const bool active = grp * 64 + lane < nprob;
		bt2x_dp_in p;
		if(active) p = a.in[pi];
		else { p.read_off = p.qual_off = p.ref_off = 0; p.refl = 0; p.rdlen = 0; p.ncol = 0;
		       p.minsc = 0; p.nceil = 0; p.triml = p.corel = p.corer = 0; p.fw = 1; p.flags = 0; }
		const bool i16 = kWide && (p.flags & BT2X_DP_I16);
		// an i16 problem in a u8 launch (bt2x_dp_align_dev without BT2X_DPL_I16), or one whose
		// named window could not be cut (window_kernel): refused
		const bool refused = active && ((!kWide && (p.flags & BT2X_DP_I16)) || (p.flags & kDpBadWindow));
		const int R = p.rdlen, C = p.ncol;
		const int top = i16 ? 0xffff : 0xff;            // score 0 (H of row -1)
		// wave-uniform bounds in SGPRs: every per-step guard below is a scalar branch
		const int Rmax = __builtin_amdgcn_readfirstlane(wave_max(R));
		const int Cmax = __builtin_amdgcn_readfirstlane(wave_max(C));
		// candidate keys fit a byte (value - threshold + 1 <= 255) when every minsc >= -254;
		// decided here, with every lane active (a butterfly reduction needs all lanes)
		const bool byteKeys = !kWide || __builtin_amdgcn_readfirstlane(wave_max(-(int)p.minsc)) <= 254;
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int thr = (int)p.minsc + top;
		// ------------- row info (rows >= R: N, barred) ------------------------------
		// 4 rows per dword, in LDS for the whole fill (constant per problem; the region
		// holds the last row after the fill).  The read's codes and qualities come in 16
		// rows at a time as dwords (a chain of byte loads per row would make this prologue
		// a tenth of the fill), the penalty per quality from the LDS table.
		const uint32_t kNone = row_info(7, true, npen);
		const ByteStr rds = byte_str(rd, R > 0 ? R : 1), qus = byte_str(qu, R > 0 ? R : 1);
#pragma unroll
		for(int c16 = 0; c16 < kRows / 16; c16++) {
			if(c16 * 16 < Rmax) {                                     // wave-uniform
				uint32_t rw[4], qw[4];
#pragma unroll
				for(int k = 0; k < 4; k++) { rw[k] = bs_bytes4(rds, 4 * c16 + k); qw[k] = bs_bytes4(qus, 4 * c16 + k); }
#pragma unroll
				for(int k = 0; k < 4; k++) {
					uint32_t w = 0;
#pragma unroll
					for(int r = 0; r < 4; r++) {
						const int i = 16 * c16 + 4 * k + r;
						uint32_t b = kNone;
						if(i < R) {
							int q = (int)((qw[k] >> (8 * r)) & 0xffu) - 33;
							q = q < 0 ? 0 : q;
							const bool gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
							const int rc = (int)((rw[k] >> (8 * r)) & 0xffu);
							b = rc > 3 ? row_info(7, gbar, npen) : row_info(rc, gbar, pen_lds[q]);
						}
						w |= b << (8 * r);
					}
					lds[(4 * c16 + k) * 64 + lane] = w;
				}
			} else {
#pragma unroll
				for(int k = 0; k < 4; k++) lds[(4 * c16 + k) * 64 + lane] = kNone * 0x01010101u;
			}
		}
		const unsigned long long tA = a.prof ? __builtin_amdgcn_s_memtime() : 0;
		// ------------- fill: two columns per sweep, per-row state in VGPRs ------------
		// H and E of the previous column: u8 4 rows per dword (40 + 40 dwords for 160
		// rows), wide 2 rows per dword (80 + 80).
		uint32_t Hs[kStateWords], Es[kStateWords];
#pragma unroll
		for(int b = 0; b < kStateWords; b++) { Hs[b] = 0; Es[b] = 0; }
		uint64_t dg0 = 0, dg1 = 0, dg2 = 0;
		int lrmax = 0, ncand = 0;
		const int Rmin = __builtin_amdgcn_readfirstlane(-wave_max(-R));
		const uint32_t rdo2 = (uint32_t)rdo * 0x10001u, rde2 = (uint32_t)rde * 0x10001u;
		const uint32_t rfo2 = (uint32_t)rfo * 0x10001u, rfe2 = (uint32_t)rfe * 0x10001u;
		const uint32_t npen2 = (uint32_t)npen * 0x10001u;
		const uint32_t topLo = (uint32_t)top, topHi = (uint32_t)top << 16;
		// digests hash the reference's stored value: the u8 byte, or the int16 bit pattern
		const uint32_t dgx = i16 ? 0x8000u : 0u;
		// Diagonal band (exact).  A path from row 0 to row R-1 scoring >= minsc
		// pays for at most G gap positions (every gap position costs >= the cheapest extension,
		// the first of a run >= the cheapest open), so it stays inside diagonals [-G, C-R+G]:
		// it starts on a diagonal >= 0 (row 0, col >= 0), ends on one <= C-R, and each gap
		// moves it by one.  Only cells of such paths reach a candidate's score, flags and
		// backtrace (a cell whose every optimal prefix leaves the band is on no candidate's
		// path), so the fill computes each column's rows [j-(C-R+G)-M, j+G+M] (M = 2 extra
		// diagonals); cells outside hold "dead" zeros (<= their true values, so no computed
		// value exceeds the reference's).  The wave sweeps the union of its lanes' windows:
		// per column pair, steps [j0 - wdhi, j0 + wdlo], clipped to [0, Rmax]; both ends move
		// down monotonically, so state rows entering at the bottom were never written (zero)
		// and rows above the top are never read again.  Cells below minsc in the last row may
		// then report a lower `best` (status 0 only; BT2X_DPL_EXACT_BEST recomputes those);
		// candidates, records and edits are the full fill's.  kDebug (E/F/H digests) and
		// band = 0 fill the whole rectangle.
		int wdhi = 1 << 20, wdlo = 1 << 20;
		if(!kDebug && a.band) {
			const int mo = imax(1, rdo < rfo ? rdo : rfo);
			int me = rde < rfe ? rde : rfe;
			me = me < mo ? me : mo;
			const int budget = -(int)p.minsc;                     // cost a candidate may pay
			int G = (me <= 0) ? (1 << 16) : (budget < mo ? 0 : 1 + (budget - mo) / me);
			G = G > (1 << 16) ? (1 << 16) : G;
			constexpr int kBandMargin = 2;
			const int dh = active ? (C - R) + G + kBandMargin : -(1 << 20);
			const int dl = active ? G + kBandMargin + 2 : -(1 << 20);
			wdhi = __builtin_amdgcn_readfirstlane(wave_max(dh));
			wdlo = __builtin_amdgcn_readfirstlane(wave_max(dl));
		}
		const int npairs = (Cmax + 1) >> 1;
		const __amdgpu_buffer_rsrc_t dirsrc =
			__builtin_amdgcn_make_buffer_rsrc(dir, 0, (int)(kDirBytesLane * 64u), 0x00020000);
		// The window's codes as dwords, 16 columns per load at every eighth pair: a load per
		// pair made every pair wait for the previous pair's traceback stores (vmcnt counts
		// loads and stores in issue order, and the compiler cannot count the band's
		// stores), now one pair in eight does.  (Loads kept in flight across pairs are worse:
		// the loop's register rotation copies them, and each copy waits.)  Windows sit in
		// BT2X_MAX_COLS-byte slots (the window pass), so the dwords are aligned; loads are
		// clamped to the window's last dword.
		const uint32_t* rfw = reinterpret_cast<const uint32_t*>(rf);
		const int lastw = ((C > 0 ? C : 1) - 1) >> 2;
		uint32_t cw0 = 0, cw1 = 0, cw2 = 0, cw3 = 0;
		uint32_t refN = 0;                              // an N in the window's columns [0, C)
		for(int pp = 0; pp < npairs; pp++) {
			const int j0 = 2 * pp;
			// opaque per pair: keeps the per-step guards and last-row compares from being
			// hoisted out of the pair loop as 2 x 161 precomputed lane masks (SGPR spills)
			int rmax = Rmax, rmin = Rmin, rl = R;
			int slo = j0 - wdhi, shi = j0 + wdlo;           // this pair's step window (band)
			slo = slo < 0 ? 0 : (slo & ~3);
			shi = (shi > rmax ? rmax : shi) | 3;            // whole blocks (steps past Rmax: unused rows)
			shi = shi > kSteps - 1 ? kSteps - 1 : shi;
			// cells this lane's sweep computes for the pair (two per step)
			if(active && shi >= slo) st_comp += 2u * (unsigned)(shi - slo + 1);
			asm volatile("" : "+s"(rmax), "+s"(rmin), "+v"(rl), "+s"(slo), "+s"(shi));
			// row-info loads stay inside the pair (hoisted out of it they would hold all 40
			// words in VGPRs)
			asm volatile("" ::: "memory");
			if(kProfWindow && (pp & 7) == 0) {            // wave-uniform: the next 16 columns
				const int w0 = pp >> 1;
				cw0 = rfw[min(w0, lastw)]; cw1 = rfw[min(w0 + 1, lastw)];
				cw2 = rfw[min(w0 + 2, lastw)]; cw3 = rfw[min(w0 + 3, lastw)];
				// consumed here, so the wait for them stays inside this branch (at the join it
				// would run at every pair)
				asm volatile("" : "+v"(cw0), "+v"(cw1), "+v"(cw2), "+v"(cw3));
			}
			const uint32_t wsel = (pp & 4) ? ((pp & 2) ? cw3 : cw2) : ((pp & 2) ? cw1 : cw0);
			const uint32_t wsh = (uint32_t)(pp & 1) * 16u;
			const int ca = (j0 < C) ? (int)((wsel >> wsh) & 0xffu) : 4;
			const int cb = (j0 + 1 < C) ? (int)((wsel >> (wsh + 8u)) & 0xffu) : 4;
			const uint32_t refc2 = (uint32_t)ca | ((uint32_t)cb << 16);
			// N reference columns: every row pays the N penalty
			const uint32_t coln = (ca > 3 ? 0x0000ffffu : 0u) | (cb > 3 ? 0xffff0000u : 0u);
			refN |= ((ca > 3) & (j0 < C)) | ((cb > 3) & (j0 + 1 < C));
			// traceback stores through a buffer resource: lane offset in a VGPR, the step
			// offset in an SGPR (no per-store 64-bit address arithmetic)
			const uint32_t pbase = (uint32_t)pp * kPairWords * 256u;
			uint32_t hp = 0, fp = 0, ep = 0, hlp = 0;      // previous step's packed H, F, E, hl
			uint32_t tbacc = 0;
			int lra = 0, lrb = 0;                           // H[R-1][j0], H[R-1][j0+1]
			// Row info of the current block (iw) and of the one above (iv); the next block's is
			// read a block ahead, so no step waits on LDS (the executed blocks are contiguous:
			// the band window [slo, shi]).
			uint32_t cur_iw, cur_iv;
			{
				const int b0 = slo >> 2;
				cur_iw = lds[(b0 < kRowWords ? b0 : kRowWords - 1) * 64 + lane];
				cur_iv = lds[(b0 > 0 ? b0 - 1 : 0) * 64 + lane];
			}
			// the window is widened to whole 4-step blocks: a skipped block costs one scalar
			// branch and a computed one none (the extra rows are outside every lane's band, or
			// past its read: any values do)
#pragma unroll
			for(int b4 = 0; b4 < kSteps; b4 += 4) {
			if(b4 >= slo && b4 <= shi) {                                 // wave-uniform
			const int nb = (b4 >> 2) + 1;
			const uint32_t nxt_iw = lds[(nb < kRowWords ? nb : kRowWords - 1) * 64 + lane];
#pragma unroll
			for(int st = b4; st < b4 + 4 && st < kSteps; st++) {
				{
				const int blk = st >> 2, r = st & 3;
				// --- operands: low half = (row st, col j0), high half = (row st-1, col j0+1)
				const uint32_t iw = cur_iw, iv = cur_iv;
				uint32_t info = (st == 0) ? perm(0, iw, 0x0c0c0c00u)
				              : (st == kRows) ? (perm(iw, 0, 0x0c070c0cu) | (kNone & 0xffu))
				              : (r == 0) ? perm(iv, iw, 0x0c070c00u)
				                         : perm(0, iw, 0x0c000c00u | ((uint32_t)(r - 1) << 16) | (uint32_t)r);
				uint32_t hl, el, hdiag;
				if(!kWide) {
					const uint32_t hsw = st < kRows ? Hs[blk] : 0u, esw = st < kRows ? Es[blk] : 0u;
					// hl: H[st][j0-1] | H[st-1][j0] (row -1 of any column is 0xff: start anywhere)
					hl = (st == 0) ? perm(0, hsw, 0x0c0c0c00u) | 0x00ff0000u
					               : perm(hp, hsw, 0x0c040c00u | (uint32_t)r);
					el = (st == 0) ? perm(0, esw, 0x0c0c0c00u)
					               : perm(ep, esw, 0x0c040c00u | (uint32_t)r);
					hdiag = (st == 0) ? 0x000000ffu : hlp;
				} else {
					const int hw = st >> 1, hr = st & 1;
					const uint32_t hsw = st < kRows ? Hs[hw < kStateWords ? hw : kStateWords - 1] : 0u;
					const uint32_t esw = st < kRows ? Es[hw < kStateWords ? hw : kStateWords - 1] : 0u;
					const uint32_t hsel = hr ? 0x05040302u : 0x05040100u;
					hl = (st == 0) ? ((hsw & 0xffffu) | topHi) : perm(hp, hsw, hsel);
					el = (st == 0) ? (esw & 0xffffu) : perm(ep, esw, hsel);
					hdiag = (st == 0) ? topLo : hlp;
				}
				// penalty: 0 on a match, mm on a mismatch, npen if either base is N
				// (x & 7) << 8 is >= 256 in a half whose codes differ: min(mm, that) = mm or 0
				// (x != 0 also for N bases: a read N is 7 and a reference N is 4)
				const uint32_t xrc = (info ^ refc2) & 0x00070007u;
				uint32_t pen = pmin(pshr(info, 4), xrc << 8);
				pen = (pen & ~coln) | (npen2 & coln);
				const uint32_t gbm = info & 0x00080008u;
				const uint32_t d = psubs(hdiag, pen);
				uint32_t hl_o, el_e, hu_o, fu_e;
				if(!kWide) {
					// gap barrier rows: open/extend penalties >= 256 saturate the term to 0;
					// row 0 has no F (low half at st 0, high half at st 1)
					const uint32_t r0 = (st == 0) ? 0x00000100u : (st == 1) ? 0x01000000u : 0u;
					const uint32_t rdoe = (gbm << 5) + rdo2, rfoe = (gbm << 5) + (rfo2 + r0), rfee = (gbm << 5) + (rfe2 + r0);
					hl_o = psubs(hl, rdoe); el_e = psubs(el, rde2);
					hu_o = psubs(hp, rfoe); fu_e = psubs(fp, rfee);
				} else {
					// 16-bit halves: barred terms are masked to the floor (0x8000 added twice in
					// the reference, aligner_swsse_ee_i16.cpp:112 and :400-420)
					const uint32_t r0 = (st == 0) ? 0x0000ffffu : (st == 1) ? 0xffff0000u : 0u;
					const uint32_t bm = (gbm >> 3) * 0xffffu;
					const uint32_t fm = ~(bm | r0);
					hl_o = psubs(hl, rdo2) & ~bm; el_e = psubs(el, rde2);
					hu_o = psubs(hp, rfo2) & fm; fu_e = psubs(fp, rfe2) & fm;
				}
				const uint32_t e = pmax(hl_o, el_e);
				const uint32_t f = pmax(hu_o, fu_e);
				const uint32_t h = pmax(pmax(d, e), f);
				// traceback flags
				uint32_t tb = pmin(xrc, one2);                        // TB_MM
				tb = (tb << 1) | pne(hl_o, e, one2);                   // TB_EONE
				tb = (tb << 1) | pne(hu_o, f, one2);                   // TB_FONE
				tb = (tb << 1) | pne(f, h, one2);                      // TB_FNE
				tb = (tb << 1) | pne(d, h, one2);                      // TB_DNE
				if(kDebug && a.digests) {
					if(st < R && j0 < C) {
						dg0 += cell_digest(st, j0, 0, (e & 0xffffu) ^ dgx);
						dg1 += cell_digest(st, j0, 1, (f & 0xffffu) ^ dgx);
						dg2 += cell_digest(st, j0, 2, (h & 0xffffu) ^ dgx);
					}
					if(st >= 1 && st - 1 < R && j0 + 1 < C) {
						dg0 += cell_digest(st - 1, j0 + 1, 0, (e >> 16) ^ dgx);
						dg1 += cell_digest(st - 1, j0 + 1, 1, (f >> 16) ^ dgx);
						dg2 += cell_digest(st - 1, j0 + 1, 2, (h >> 16) ^ dgx);
					}
				}
				// last row of each column (per-lane R; only in the wave's R range)
				// wave-uniform; cold (a few steps per column pair): the common path falls
				// through, a taken branch per step would stall the wave's instruction fetch
				if(__builtin_expect(st + 1 >= rmin, 0)) {
					lra = (st == rl - 1) ? (int)(h & (kWide ? 0xffffu : 0xffu)) : lra;
					lrb = (st == rl) ? (int)((h >> 16) & (kWide ? 0xffffu : 0xffu)) : lrb;
				}
				// the high half's outputs (row st-1 of column j0+1) replace row st-1 state
				if(st >= 1) {
					if(!kWide) {
						const int pb = (st - 1) >> 2, pr = (st - 1) & 3;
						const uint32_t selh = (0x03020100u & ~(0xffu << (8 * pr))) | (6u << (8 * pr));
						Hs[pb] = perm(h, Hs[pb], selh);
						Es[pb] = perm(e, Es[pb], selh);
					} else {
						const int pb = (st - 1) >> 1;
						const uint32_t selh = ((st - 1) & 1) ? 0x07060100u : 0x03020706u;
						if(pb < kStateWords) {
							Hs[pb] = perm(h, Hs[pb], selh);
							Es[pb] = perm(e, Es[pb], selh);
						}
					}
				}
				// two steps' flags of both columns per traceback dword
				if(kProfStores && (st & 1)) {
					__builtin_amdgcn_raw_buffer_store_b32(perm(tb, tbacc, 0x06040200u), dirsrc, lane * 4,
					                                      (int)(pbase + (uint32_t)(st >> 1) * 256u), kTbStoreAux);
				} else {
					tbacc = tb;
					if(__builtin_expect(st == shi, 0))
						__builtin_amdgcn_raw_buffer_store_b32(perm(0, tbacc, 0x0c0c0200u), dirsrc, lane * 4,
						                                      (int)(pbase + (uint32_t)(st >> 1) * 256u), kTbStoreAux);
				}
				hlp = hl; hp = h; fp = f; ep = e;
				}
			}
			cur_iv = cur_iw; cur_iw = nxt_iw;
			}
			}
			if(j0 < C) {
				if(kWide) lastrow16[(size_t)j0 * 64 + lane] = (uint16_t)lra;
				else lastrow[(size_t)j0 * 64 + lane] = (uint8_t)lra;
				lrmax = imax(lrmax, lra);
				ncand += (lra >= thr);
			}
			if(j0 + 1 < C) {
				if(kWide) lastrow16[(size_t)(j0 + 1) * 64 + lane] = (uint16_t)lrb;
				else lastrow[(size_t)(j0 + 1) * 64 + lane] = (uint8_t)lrb;
				lrmax = imax(lrmax, lrb);
				ncand += (lrb >= thr);
			}
		}
		const unsigned long long tB = a.prof ? __builtin_amdgcn_s_memtime() : 0;
		if(a.prof) { t_pro += tA - t0; t_pair += tB - tA; }
		if(!active) continue;
		st_cells += (unsigned long long)R * C;
		st_cols += C;
		if(kDebug && a.digests) {
			a.digests[3 * (size_t)pi + 0] = dg0;
			a.digests[3 * (size_t)pi + 1] = dg1;
			a.digests[3 * (size_t)pi + 2] = dg2;
		}
		bt2x_dp_out o;
		o.nrec = 0; o.rec_off = 0;
		int status = 0, best = 0;
		dp_verdict(i16, lrmax, p.minsc, ncand, status, best);
		if(refused) { status = -1; best = 0; atomicAdd(&a.counters[3], 1u); }
		o.status = status; o.best = best; o.ncand = status > 0 ? (uint16_t)ncand : (uint16_t)0;
		if(status <= 0) {
			a.out[pi] = o;
			// the banded fill's best of a failed problem is a lower bound: queue it for the
			// exact pass (dp_wave_kernel<true>)
			if(status == 0 && a.fail_list && a.band && !kDebug) a.fail_list[atomicAdd(&a.counters[2], 1u)] = pi;
			if(kDebug && a.cands)
				for(int k = 0; k < kCols; k++) a.cands[(size_t)pi * kCols + k] = 0xffffffffu;
			continue;
		}
		// ------------- candidate order (DpBtCandidate: score desc, col desc) --------
		// the last row moves into LDS as one key byte per column (u8: the cell value, 0
		// below the threshold never being reached; wide: value - threshold + 1 when it
		// qualifies, else 0 -- a byte when -minsc <= 254, which holds for every u8
		// problem and every i16 problem of default scoring); repeated max-below-key scans
		// emit the sorted candidate columns for the walk (up to the wave's widest problem:
		// columns >= C read as key 0)
		const int nw = (Cmax + 3) >> 2;                  // wave-uniform (Cmax: all lanes)
		a.out[pi] = o;
		const int row0 = R - 1;
		if(byteKeys) {
			for(int q = 0; q < nw; q++) {
				uint32_t w4 = 0;
				for(int r = 0; r < 4; r++) {
					const int j = q * 4 + r;
					if(j < C) {
						uint32_t kv;
						if(!kWide) kv = lastrow[(size_t)j * 64 + lane];
						else { const int v = lastrow16[(size_t)j * 64 + lane]; kv = v >= thr ? (uint32_t)(v - thr + 1) : 0u; }
						w4 |= kv << (8 * r);
					}
				}
				lds[q * 64 + lane] = w4;
			}
			order_candidates(lds, lane, nw, ncand, one2, [&](int k, int bk) {
				cands[(size_t)k * 64 + lane] = (uint8_t)(bk & 0xff);
				if(kDebug && a.cands) {
					const int score = kWide ? (bk >> 8) - 1 + thr : (bk >> 8);
					a.cands[(size_t)pi * kCols + k] = i16 ? BT2X_CAND_PACK16(bk & 0xff, score - 0x8000)
					                                      : BT2X_CAND_PACK(row0, bk & 0xff, score);
				}
			});
		} else {
			// an i16 problem with minsc < -254 in the wave: 32-bit keys (value << 8 | col)
			// straight from the last row (rare: non-default --score-min)
			int cur_key = 0x7fffffff;
			for(int k = 0; k < ncand; k++) {
				int bk = -1;
				for(int j = 0; j < Cmax; j++) {
					const int v = j < C ? (int)lastrow16[(size_t)j * 64 + lane] : -1;
					const int key = v >= thr ? ((v << 8) | j) : -1;
					bk = (key < cur_key && key > bk) ? key : bk;
				}
				cur_key = bk;
				cands[(size_t)k * 64 + lane] = (uint8_t)(bk & 0xff);
				if(kDebug && a.cands)
					a.cands[(size_t)pi * kCols + k] = i16 ? BT2X_CAND_PACK16(bk & 0xff, (bk >> 8) - 0x8000)
					                                      : BT2X_CAND_PACK(row0, bk & 0xff, bk >> 8);
			}
		}
		if(kDebug && a.cands)
			for(int k = ncand; k < kCols; k++) a.cands[(size_t)pi * kCols + k] = 0xffffffffu;
		if(kFused) {
			uint8_t* wslot = gslot + kGroupBytes;
			const unsigned long long t1 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
			if(a.prof) t_cand += t1 - tB;
			const unsigned long long bt0 = st_bt;
			walk_problem<64, kPairWords>(sc, pen_lds, a, pi, lane, lane, gslot + kDirOff, kDirBytesLane * 64u, gslot + kCandOff,
			                             reinterpret_cast<uint32_t*>(wslot + kEditOff), reinterpret_cast<bt2x_aln_rec*>(wslot + kRecOff),
			                             st_bt, refN != 0, lds, a.prof != 0, pw_steps, pw_iters);
			if(a.prof) {
				const unsigned long long t2 = __builtin_amdgcn_s_memtime();
				t_fill += t1 - t0; t_walk += t2 - t1; ngrp++;
				mx_fill = max(mx_fill, t1 - t0); mx_walk = max(mx_walk, t2 - t1);
				// this lane's serial work (walk steps + candidates) and the wave's maximum of it
				mylen_sum += st_bt - bt0 + (unsigned long long)ncand;
				mylen_max = max(mylen_max, st_bt - bt0 + (unsigned long long)ncand);
			}
		}
	}
	if(a.prof) {
		unsigned long long w0 = pw_steps, w1 = pw_iters, ls = mylen_sum, lm = mylen_max;
		for(int d = 32; d > 0; d >>= 1) {
			w0 += __shfl_xor(w0, d); w1 += __shfl_xor(w1, d); ls += __shfl_xor(ls, d);
			const unsigned long long o = __shfl_xor(lm, d); lm = lm > o ? lm : o;
		}
		if(lane == 0) {
			atomicAdd(&a.prof[0], t_fill); atomicAdd(&a.prof[1], t_walk);
			atomicAdd(&a.prof[2], w0); atomicAdd(&a.prof[3], w1); atomicAdd(&a.prof[4], ngrp);
			atomicMax(&a.prof[5], __builtin_amdgcn_s_memtime() - t_start);
			atomicMax(&a.prof[6], mx_fill); atomicMax(&a.prof[7], mx_walk);
			atomicAdd(&a.prof[8], ls); atomicAdd(&a.prof[9], lm); atomicMax(&a.prof[10], lm);
			atomicAdd(&a.prof[11], t_pro); atomicAdd(&a.prof[12], t_pair); atomicAdd(&a.prof[13], t_cand);
		}
	}
	if(a.stats) {
		for(int d = 32; d > 0; d >>= 1) {
			st_cells += __shfl_xor(st_cells, d);
			st_cols += __shfl_xor(st_cols, d);
			st_bt += __shfl_xor(st_bt, d);
			st_comp += __shfl_xor(st_comp, d);
		}
		if(lane == 0) {
			atomicAdd(&a.stats[0], st_cells);
			atomicAdd(&a.stats[1], st_cols);
			if(kFused) atomicAdd(&a.stats[2], st_bt);
			atomicAdd(&a.stats[3], st_comp);
		}
	}
}

// ------------------------------------------------------------- duo fill (two lanes per problem)
// At cohort launch sizes a launch holds about one 64-problem group per SIMD, so the lane
// kernel's launch lasts one lane's dependent chain: ~the band's rows (~94 at 150 bp,
// --dpad 12) of steps per column pair.  Here each problem has two lanes (even lane A, odd
// lane B; 32 problems per wave) that split the band along a diagonal, so a wave sweeps
// about half the steps per column pair and a launch has twice the waves (two per SIMD,
// whose VALU streams interleave).
//  * Column pair p's band rows [s0, e] (s0 = max(2p - wdh, 0)) split at b = s0 + K: A
//    computes rows [s0, b] of pair p (its step b: the high half, row b-1 of column 2p+1,
//    is exact; the low half is not, and B overwrites that byte), B rows [b, e] one
//    iteration later (iteration i: A pair i, B pair i-1).  K (a multiple of 4, ~half the
//    band) is B's slot offset: B keeps row r in register / LDS slot r - K, so both lanes'
//    windows are the same ~K slots and the wave's step code (fully unrolled by slot, as in
//    dp_fill_kernel) serves both.
//  * The split moves down 2 rows per pair, so the halves depend on each other every pair:
//    T1 (A -> B): B's first step needs the step before it, A's outputs (packed H, F, E and
//      hl) at slot (s0 & ~3) + K - 1, the last step of a block; B starts at the block-aligned
//      slot, recomputing up to 2 of A's rows exactly from them.
//    T2 (B -> A): A's rows b, b+1 of the next pair need their left neighbours (H, E of
//      column 2p+1) from B, computed at B's second and third steps: B's state dword after
//      them goes to A (DPP), which splices it in before it reads them.
//    Both are wave-uniform events at blocks known per iteration (one scalar test per
//    block).  A's garbage cells below b (and its garbage low half at b) are overwritten by
//    B's later stores of the same bytes; B's stores of rows it recomputes are exact; cells
//    outside the band obey dp_fill_kernel's rule (computed values <= true values).
//  * Traceback: tb_addr_g<32, kDuoPW> with one spare pair in front (B's pair -1 in the
//    first iteration) and kDuoPW >= (161 + K) / 2 dword rows per pair (B's slots past its
//    window write rows below the matrix, never above another pair).
//  * Last rows, candidates and the walk run on the A lanes (walk_problem<32, kDuoPW>);
//    the owner of row R-1 of each pair (A if R-1 < b, else B) supplies its last-row bytes.
constexpr int kDuoG = 32;                                   // problems per wave
constexpr int kDuoKMax = 80;                                // largest slot offset of B
constexpr int kDuoPW = (kSteps + kDuoKMax + 1) / 2;       // dword rows per column pair
constexpr int kDuoPairs = kCols / 2 + 2;                    // pairs -1 .. kCols / 2
constexpr uint32_t kDuoPairBytes = (uint32_t)kDuoPW * kDuoG * 4;
constexpr uint32_t kDuoDirBytes = (uint32_t)kDuoPairs * kDuoPairBytes;
constexpr size_t kDuoLastRowOff = kDuoDirBytes;                        // [col * 64 + lane]
constexpr size_t kDuoCandOff = kDuoLastRowOff + (size_t)kCols * 64;    // [k * 64 + lane]
constexpr size_t kDuoGroupBytes = kDuoCandOff + (size_t)kCandBytesLane * 64;
static_assert(kDuoGroupBytes <= kGroupBytes, "the duo layout fits a fused slot");

// quad_perm DPP within lane pairs: odd lane l gets lane l-1's value, even lane l gets l+1's
__device__ __forceinline__ uint32_t from_even(uint32_t v) {
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t from_odd(uint32_t v) {
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xf, 0xf, false);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
dp_duo_kernel(DevScoring sc, DpLaunch a, uint32_t nprob) {
	__shared__ uint32_t lds[(kCols / 4) * 64];        // row info during the fill, then candidate keys
	__shared__ uint32_t pen4[64];
	const uint8_t* pen_lds = reinterpret_cast<const uint8_t*>(pen4);
	const int lane = threadIdx.x;
	const bool isB = (lane & 1) != 0;
	const int q = lane >> 1;                           // problem slot in the group
	pen4[lane] = reinterpret_cast<const uint32_t*>(a.mmpen)[lane];
	__syncthreads();
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0, st_comp = 0;
	unsigned long long st_dummy0 = 0, st_dummy1 = 0;                 // walk_problem's profiling counters (unused)
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;
	const uint32_t one2 = opaque(0x00010001u);
	unsigned long long t_fill = 0, t_walk = 0, ngrp = 0, mx_fill = 0, mx_walk = 0;     // BT2X_DP_PROF
	const unsigned long long t_start = a.prof ? __builtin_amdgcn_s_memtime() : 0;
	for(uint32_t grp = blockIdx.x; (uint64_t)grp * kDuoG < nprob; grp += gridDim.x) {
		const unsigned long long t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
		uint8_t* gslot = a.scratch + (size_t)blockIdx.x * (kGroupBytes + kWalkSlotBytes);
		uint8_t* lastrow = gslot + kDuoLastRowOff;
		uint8_t* cands = gslot + kDuoCandOff;
		const uint32_t pi = grp * kDuoG + (uint32_t)q;
		const bool active = pi < nprob;
		bt2x_dp_in p;
		if(active) p = a.in[pi];
		else { p.read_off = p.qual_off = p.ref_off = 0; p.refl = 0; p.rdlen = 0; p.ncol = 0;
		       p.minsc = 0; p.nceil = 0; p.triml = p.corel = p.corer = 0; p.fw = 1; p.flags = 0; }
		const bool refused = active && ((p.flags & BT2X_DP_I16) || (p.flags & kDpBadWindow));
		const int R = p.rdlen, C = p.ncol;
		constexpr int top = 0xff;
		const int Rmax = __builtin_amdgcn_readfirstlane(wave_max(R));
		const int Cmax = __builtin_amdgcn_readfirstlane(wave_max(C));
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int thr = (int)p.minsc + top;
		// the exact band (dp_fill_kernel): pair j0's rows [j0 - wdhi, j0 + wdlo]
		int wdhi, wdlo;
		{
			const int mo = imax(1, rdo < rfo ? rdo : rfo);
			int me = rde < rfe ? rde : rfe;
			me = me < mo ? me : mo;
			const int budget = -(int)p.minsc;
			int G = (me <= 0) ? (1 << 16) : (budget < mo ? 0 : 1 + (budget - mo) / me);
			G = G > (1 << 16) ? (1 << 16) : G;
			constexpr int kBandMargin = 2;
			const int dh = active ? (C - R) + G + kBandMargin : -(1 << 20);
			const int dl = active ? G + kBandMargin + 2 : -(1 << 20);
			wdhi = __builtin_amdgcn_readfirstlane(wave_max(dh));
			wdlo = __builtin_amdgcn_readfirstlane(wave_max(dl));
			wdhi = wdhi > 4 * kRows ? 4 * kRows : wdhi;
			wdlo = wdlo > 4 * kRows ? 4 * kRows : wdlo;
		}
		const int wdh = wdhi + (wdhi & 1);             // even: every window start 2p - wdh is even
		int K = ((wdh + wdlo - 2) / 2 + 2) & ~3;       // balances A's K + 1 rows and B's
		K = K < 8 ? 8 : (K > kDuoKMax ? kDuoKMax : K);
		K = __builtin_amdgcn_readfirstlane(K);
		const int rowoff = isB ? K : 0;                // this lane's slot s holds row s + rowoff
		// ------------- row info per slot (rows >= R: N, barred), as dp_fill_kernel
		const uint32_t kNone = row_info(7, true, npen);
		auto rinfo = [&](int i, uint32_t rb, uint32_t qb) -> uint32_t {
			if(i >= R) return kNone;
			int qq = (int)qb - 33;
			qq = qq < 0 ? 0 : qq;
			const bool gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
			return rb > 3 ? row_info(7, gbar, npen) : row_info((int)rb, gbar, pen_lds[qq]);
		};
		const ByteStr rds = byte_str(rd, R > 0 ? R : 1), qus = byte_str(qu, R > 0 ? R : 1);
		const int w4off = rowoff >> 2;
#pragma unroll
		for(int c16 = 0; c16 < kRows / 16; c16++) {
			if(c16 * 16 < Rmax) {                                     // wave-uniform
				uint32_t rw[4], qw[4];
#pragma unroll
				for(int k = 0; k < 4; k++) {
					rw[k] = bs_bytes4(rds, 4 * c16 + k + w4off); qw[k] = bs_bytes4(qus, 4 * c16 + k + w4off);
				}
#pragma unroll
				for(int k = 0; k < 4; k++) {
					uint32_t w = 0;
#pragma unroll
					for(int r = 0; r < 4; r++) {
						const int i = 16 * c16 + 4 * k + r + rowoff;
						w |= rinfo(i, (rw[k] >> (8 * r)) & 0xffu, (qw[k] >> (8 * r)) & 0xffu) << (8 * r);
					}
					lds[(4 * c16 + k) * 64 + lane] = w;
				}
			} else {
#pragma unroll
				for(int k = 0; k < 4; k++) lds[(4 * c16 + k) * 64 + lane] = kNone * 0x01010101u;
			}
		}
		// B's first step at slot 0 (early pairs) computes row K-1 of the high column: its info
		const uint32_t info_m1 = (isB && K - 1 < R) ? rinfo(K - 1, rd[K - 1], qu[K - 1]) : 0u;
		// ------------- fill
		uint32_t Hs[kRowWords], Es[kRowWords];
#pragma unroll
		for(int b = 0; b < kRowWords; b++) { Hs[b] = 0; Es[b] = 0; }
		int lrmax = 0, ncand = 0;
		const int rl0 = active ? R - rowoff : (1 << 20);            // slot of row R (row R-1 at rl - 1)
		const int Rmin = __builtin_amdgcn_readfirstlane(-wave_max(-rl0));
		const uint32_t rdo2 = (uint32_t)rdo * 0x10001u, rde2 = (uint32_t)rde * 0x10001u;
		const uint32_t rfo2 = (uint32_t)rfo * 0x10001u, rfe2 = (uint32_t)rfe * 0x10001u;
		const uint32_t npen2 = (uint32_t)npen * 0x10001u;
		const int npairs = (Cmax + 1) >> 1;
		const __amdgpu_buffer_rsrc_t dirsrc = __builtin_amdgcn_make_buffer_rsrc(gslot, 0, (int)kDuoDirBytes, 0x00020000);
		// pair p is stored at (p + 1) pair strides; the per-step scalar offset carries pair
		// pp - 1 (B's) and the step's dword row, the lane offset A's extra pair or B's K / 2 rows
		const uint32_t voff = (uint32_t)q * 4u + (isB ? (uint32_t)(K / 2) * (kDuoG * 4u) : kDuoPairBytes);
		const uint32_t* rfw = reinterpret_cast<const uint32_t*>(rf);
		const int lastw = ((C > 0 ? C : 1) - 1) >> 2;
		uint32_t cw0 = 0, cw1 = 0, cw2 = 0, cw3 = 0;
		uint32_t refN = 0;
		uint32_t t1h = 0, t1f = 0, t1e = 0, t1hl = 0;                 // T1 (B lanes after the DPP)
		uint32_t t2h = 0, t2e = 0;                                     // T2 (A lanes)
		for(int pp = 0; pp <= npairs; pp++) {
			const int pl = pp - (isB ? 1 : 0);                        // this lane's pair
			const int j0 = 2 * pl;
			// wave-uniform windows: A's pair pp rows [s0A, s0A + K], B's pair pp-1 slots [s0B, endB]
			const bool hasA = pp < npairs, hasB = pp > 0;
			const int s0A = imax(2 * pp - wdh, 0), s0B = imax(2 * pp - 2 - wdh, 0);
			const int endA = hasA ? min(s0A + K, Rmax) : -1;
			const int endB = hasB ? min(2 * pp - 2 + wdlo, Rmax) - K : -1;
			int slo = (hasB ? s0B : s0A) & ~3;
			int shi = imax(endA, endB) | 3;
			shi = shi > kSteps - 1 ? kSteps - 1 : shi;
			const int kT1 = hasA ? ((s0A & ~3) + K) / 4 - 1 : -1;     // A's step before B's next start
			const int kT2 = hasB ? (s0B + 2) >> 2 : -1;                 // B's rows b, b+1 done
			const int kP = hasB ? ((s0B + K) >> 2) - 1 : -1;            // patch A's rows b, b+1 after it
			uint64_t ev = 0;
			if(kT1 >= 0 && kT1 < 64) ev |= 1ull << kT1;
			if(kT2 >= 0 && kT2 < 64) ev |= 1ull << kT2;
			if(kP >= 0 && kP < 64) ev |= 1ull << kP;
			const uint32_t t2sel = (s0B & 2) ? 0xffff0000u : 0x0000ffffu;   // the patched half
			if(active && hasA && !isB) st_comp += 2u * (unsigned)imax(0, endA - s0A);
			if(active && hasB && isB) st_comp += 2u * (unsigned)imax(0, endB - s0B + 1);
			int rmin = Rmin, rl = rl0;
			// opaque per pair (dp_fill_kernel): keeps the per-step guards and last-row compares from
			// being hoisted out of the pair loop as precomputed lane masks (SGPR spills)
			asm volatile("" : "+s"(rmin), "+s"(slo), "+s"(shi), "+s"(ev), "+v"(rl));
			asm volatile("" ::: "memory");
			// this lane's reference columns: 16 per load at every eighth pair of its own
			if((pl & 7) == 0) {
				const int w0 = pl >> 1;
				cw0 = rfw[min(w0, lastw)]; cw1 = rfw[min(w0 + 1, lastw)];
				cw2 = rfw[min(w0 + 2, lastw)]; cw3 = rfw[min(w0 + 3, lastw)];
				asm volatile("" : "+v"(cw0), "+v"(cw1), "+v"(cw2), "+v"(cw3));
			}
			const uint32_t wsel = (pl & 4) ? ((pl & 2) ? cw3 : cw2) : ((pl & 2) ? cw1 : cw0);
			const uint32_t wsh = (uint32_t)(pl & 1) * 16u;
			const int ca = (j0 >= 0 && j0 < C) ? (int)((wsel >> wsh) & 0xffu) : 4;
			const int cb = (j0 >= 0 && j0 + 1 < C) ? (int)((wsel >> (wsh + 8u)) & 0xffu) : 4;
			const uint32_t refc2 = (uint32_t)ca | ((uint32_t)cb << 16);
			const uint32_t coln = (ca > 3 ? 0x0000ffffu : 0u) | (cb > 3 ? 0xffff0000u : 0u);
			refN |= ((ca > 3) & (j0 >= 0) & (j0 < C)) | ((cb > 3) & (j0 >= 0) & (j0 + 1 < C));
			const uint32_t sbase = (uint32_t)pp * kDuoPairBytes;
			// the step before the window: dead above for A, T1 for B
			uint32_t hp = isB ? t1h : 0u, fp = isB ? t1f : 0u, ep = isB ? t1e : 0u, hlp = isB ? t1hl : 0u;
			uint32_t tbacc = 0;
			int lra = 0, lrb = 0;
			uint32_t cur_iw, cur_iv;
			{
				const int b0 = slo >> 2;
				cur_iw = lds[(b0 < kRowWords ? b0 : kRowWords - 1) * 64 + lane];
				cur_iv = lds[(b0 > 0 ? b0 - 1 : 0) * 64 + lane];
			}
#pragma unroll
			for(int b4 = 0; b4 < kSteps; b4 += 4) {
			if(b4 >= slo && b4 <= shi) {                                 // wave-uniform
			const int nb = (b4 >> 2) + 1;
			const uint32_t nxt_iw = lds[(nb < kRowWords ? nb : kRowWords - 1) * 64 + lane];
#pragma unroll
			for(int st = b4; st < b4 + 4 && st < kSteps; st++) {
				{
				const int blk = st >> 2, r = st & 3;
				const uint32_t iw = cur_iw, iv = cur_iv;
				// slot 0 is row 0 for A, row K for B (whose high half is row K - 1)
				uint32_t info = (st == 0) ? (perm(0, iw, 0x0c0c0c00u) | (info_m1 << 16))
				              : (st == kRows) ? (perm(iw, 0, 0x0c070c0cu) | (kNone & 0xffu))
				              : (r == 0) ? perm(iv, iw, 0x0c070c00u)
				                         : perm(0, iw, 0x0c000c00u | ((uint32_t)(r - 1) << 16) | (uint32_t)r);
				const uint32_t hsw = st < kRows ? Hs[blk] : 0u, esw = st < kRows ? Es[blk] : 0u;
				uint32_t hl = perm(hp, hsw, 0x0c040c00u | (uint32_t)r);
				uint32_t el = perm(ep, esw, 0x0c040c00u | (uint32_t)r);
				uint32_t hdiag = hlp;
				if(st == 0 && !isB) {                   // A's row 0: row -1 is the top (start anywhere)
					hl = perm(0, hsw, 0x0c0c0c00u) | 0x00ff0000u;
					el = perm(0, esw, 0x0c0c0c00u);
					hdiag = 0x000000ffu;
				}
				const uint32_t xrc = (info ^ refc2) & 0x00070007u;
				uint32_t pen = pmin(pshr(info, 4), xrc << 8);
				pen = (pen & ~coln) | (npen2 & coln);
				const uint32_t gbm = info & 0x00080008u;
				const uint32_t d = psubs(hdiag, pen);
				// row 0 has no F (A only: low half at slot 0, high half at slot 1)
				const uint32_t r0 = (st == 0 && !isB) ? 0x00000100u : (st == 1 && !isB) ? 0x01000000u : 0u;
				const uint32_t rdoe = (gbm << 5) + rdo2, rfoe = (gbm << 5) + (rfo2 + r0), rfee = (gbm << 5) + (rfe2 + r0);
				const uint32_t hl_o = psubs(hl, rdoe), el_e = psubs(el, rde2);
				const uint32_t hu_o = psubs(hp, rfoe), fu_e = psubs(fp, rfee);
				const uint32_t e = pmax(hl_o, el_e);
				const uint32_t f = pmax(hu_o, fu_e);
				const uint32_t h = pmax(pmax(d, e), f);
				uint32_t tb = pmin(xrc, one2);                        // TB_MM
				tb = (tb << 1) | pne(hl_o, e, one2);                   // TB_EONE
				tb = (tb << 1) | pne(hu_o, f, one2);                   // TB_FONE
				tb = (tb << 1) | pne(f, h, one2);                      // TB_FNE
				tb = (tb << 1) | pne(d, h, one2);                      // TB_DNE
				// wave-uniform; cold (a few steps per column pair): the common path falls
				// through, a taken branch per step would stall the wave's instruction fetch
				if(__builtin_expect(st + 1 >= rmin, 0)) {
					lra = (st == rl - 1) ? (int)(h & 0xffu) : lra;
					lrb = (st == rl) ? (int)((h >> 16) & 0xffu) : lrb;
				}
				if(st >= 1) {
					const int pb = (st - 1) >> 2, pr = (st - 1) & 3;
					const uint32_t selh = (0x03020100u & ~(0xffu << (8 * pr))) | (6u << (8 * pr));
					Hs[pb] = perm(h, Hs[pb], selh);
					Es[pb] = perm(e, Es[pb], selh);
				}
				if(st & 1) {
					__builtin_amdgcn_raw_buffer_store_b32(perm(tb, tbacc, 0x06040200u), dirsrc, (int)voff,
					                                      (int)(sbase + (uint32_t)(st >> 1) * (kDuoG * 4u)), 0);
				} else {
					tbacc = tb;
					if(__builtin_expect(st == shi, 0))
						__builtin_amdgcn_raw_buffer_store_b32(perm(0, tbacc, 0x0c0c0200u), dirsrc, (int)voff,
						                                      (int)(sbase + (uint32_t)(st >> 1) * (kDuoG * 4u)), 0);
				}
				hlp = hl; hp = h; fp = f; ep = e;
				}
			}
			cur_iv = cur_iw; cur_iw = nxt_iw;
			// the halves' hand-offs at this block (wave-uniform)
			const int bk = b4 >> 2;
			if(__builtin_expect((ev >> bk) & 1ull, 0)) {
				if(bk == kT1) { t1h = hp; t1f = fp; t1e = ep; t1hl = hlp; }   // its last step's outputs
				if(bk == kT2) {                     // B's dword of slots s0B, s0B + 1 (rows b, b+1)
					const bool prev = (s0B & 2) != 0 && bk >= 1;
					const uint32_t xh = prev ? Hs[bk >= 1 ? bk - 1 : 0] : Hs[bk];
					const uint32_t xe = prev ? Es[bk >= 1 ? bk - 1 : 0] : Es[bk];
					t2h = from_odd(xh); t2e = from_odd(xe);
				}
				if(bk == kP && bk + 1 < kRowWords) {   // A: rows b, b+1 of column 2pp-1 from B
					const uint32_t mh = (Hs[bk + 1] & ~t2sel) | (t2h & t2sel);
					const uint32_t me = (Es[bk + 1] & ~t2sel) | (t2e & t2sel);
					Hs[bk + 1] = isB ? Hs[bk + 1] : mh;
					Es[bk + 1] = isB ? Es[bk + 1] : me;
				}
			}
			}
			}
			// T1 to the B lanes for their next window
			t1h = from_even(t1h); t1f = from_even(t1f); t1e = from_even(t1e); t1hl = from_even(t1hl);
			// last rows: the owner of row R-1 of a pair supplies both of its columns (A if
			// R-1 < b, else B; B's come over to its A lane)
			const bool ownA = !isB && hasA && (R - 1 < s0A + K);
			const bool ownB = isB && hasB && (R - 1 >= s0B + K);
			const int xa = (int)from_odd((uint32_t)lra), xb = (int)from_odd((uint32_t)lrb);
			const bool xown = from_odd(ownB ? 1u : 0u) != 0;
			if(!isB && active) {
				const int jA = 2 * pp, jB = 2 * pp - 2;
				if(ownA) {
					if(jA < C) { lastrow[(size_t)jA * 64 + lane] = (uint8_t)lra; lrmax = imax(lrmax, lra); ncand += (lra >= thr); }
					if(jA + 1 < C) { lastrow[(size_t)(jA + 1) * 64 + lane] = (uint8_t)lrb; lrmax = imax(lrmax, lrb); ncand += (lrb >= thr); }
				}
				if(xown) {
					if(jB >= 0 && jB < C) { lastrow[(size_t)jB * 64 + lane] = (uint8_t)xa; lrmax = imax(lrmax, xa); ncand += (xa >= thr); }
					if(jB >= 0 && jB + 1 < C) { lastrow[(size_t)(jB + 1) * 64 + lane] = (uint8_t)xb; lrmax = imax(lrmax, xb); ncand += (xb >= thr); }
				}
			}
		}
		const unsigned long long t1 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
		if(a.prof) { t_fill += t1 - t0; mx_fill = max(mx_fill, t1 - t0); ngrp++; }
		if(!active || isB) continue;                   // A lanes: the verdict, candidates, the walk
		st_cells += (unsigned long long)R * C;
		st_cols += C;
		bt2x_dp_out o;
		o.nrec = 0; o.rec_off = 0;
		int status = 0, best = 0;
		dp_verdict(false, lrmax, p.minsc, ncand, status, best);
		if(refused) { status = -1; best = 0; atomicAdd(&a.counters[3], 1u); }
		o.status = status; o.best = best; o.ncand = status > 0 ? (uint16_t)ncand : (uint16_t)0;
		if(status <= 0) {
			a.out[pi] = o;
			if(status == 0 && a.fail_list) a.fail_list[atomicAdd(&a.counters[2], 1u)] = pi;
			continue;
		}
		// candidate order (DpBtCandidate: score desc, col desc), as dp_fill_kernel's u8 path
		const int nw = (Cmax + 3) >> 2;
		a.out[pi] = o;
		for(int qw = 0; qw < nw; qw++) {
			uint32_t w4 = 0;
			for(int r = 0; r < 4; r++) {
				const int j = qw * 4 + r;
				if(j < C) w4 |= (uint32_t)lastrow[(size_t)j * 64 + lane] << (8 * r);
			}
			lds[qw * 64 + lane] = w4;
		}
		order_candidates(lds, lane, nw, ncand, one2, [&](int k, int bk) { cands[(size_t)k * 64 + lane] = (uint8_t)(bk & 0xff); });
		uint8_t* wslot = gslot + kGroupBytes;
		walk_problem<kDuoG, kDuoPW>(sc, pen_lds, a, pi, lane, q, gslot + kDuoPairBytes, kDuoDirBytes - kDuoPairBytes,
		                                cands, reinterpret_cast<uint32_t*>(wslot + kEditOff),
		                                reinterpret_cast<bt2x_aln_rec*>(wslot + kRecOff), st_bt, refN != 0, lds, false, st_dummy0, st_dummy1);
		if(a.prof) { const unsigned long long t2 = __builtin_amdgcn_s_memtime(); t_walk += t2 - t1; mx_walk = max(mx_walk, t2 - t1); }
	}
	if(a.prof && lane == 0) {
		atomicAdd(&a.prof[0], t_fill); atomicAdd(&a.prof[1], t_walk); atomicAdd(&a.prof[4], ngrp);
		atomicMax(&a.prof[5], __builtin_amdgcn_s_memtime() - t_start);
		atomicMax(&a.prof[6], mx_fill); atomicMax(&a.prof[7], mx_walk);
	}
	if(a.stats) {
		for(int d = 32; d > 0; d >>= 1) {
			st_cells += __shfl_xor(st_cells, d);
			st_cols += __shfl_xor(st_cols, d);
			st_bt += __shfl_xor(st_bt, d);
			st_comp += __shfl_xor(st_comp, d);
		}
		if(lane == 0) {
			atomicAdd(&a.stats[0], st_cells);
			atomicAdd(&a.stats[1], st_cols);
			atomicAdd(&a.stats[2], st_bt);
			atomicAdd(&a.stats[3], st_comp);
		}
	}
}

// ------------------------------------------------------------ split fill (two waves per group)
// At the timed run's cohort launch sizes a launch holds about one 64-problem group per SIMD,
// and a group's fill is one wave's serial sweep of the band: the launch lasts that wave's
// dependent chain, whatever the chip's idle VALU.  Here a group has two waves (two of a
// 256-thread workgroup's four, see kSplitG); both own all 64 problems (lane l = problem l) and split every column pair's
// band window [slo, shi] at a block-aligned row b that moves down with the band:
//  * wave A computes steps [slo, b] and owns rows < b (both columns); its step b is an
//    extra step whose high half (row b-1 of the odd column) it needs for its own next pair
//    (the low half, row b, is not its own and is discarded);
//  * wave B computes steps [b, shi] and owns rows >= b.  Its first step needs the step
//    before it -- A's packed H, F, E and hl after step b-1 of the same pair (T1) -- so B
//    runs one pair behind A;
//  * when b moves down (by 4 rows, every other pair), rows [b, b+4) change owner: A takes
//    B's H/E state dword of that block after B's pair (T2) before it reaches that block.
// So each wave sweeps about half the band per pair and the two halves overlap in time; no
// cell is computed differently from dp_fill_kernel (the same step code, the same band, the
// same dead zeros), and each traceback dword is stored once, by the owner of its two steps.
// T1 and T2 go through two-slot LDS rings with workgroup-scope flags (a pair of waves of one
// CU, on two SIMDs; the waits are short: A needs T2 only at the end of its pair, B waits
// for A's pair).
// After the fill both waves combine their last-row maxima and candidate counts, and each
// orders candidates and walks half of the group's problems (lanes 32w .. 32w+31).
constexpr int kSplitW = 2;                                   // waves per group
// Groups per workgroup.  A workgroup's waves are spread over the CU's SIMDs only when it
// has four of them (measured, tools/micro/valu_chain.hip: two 2-wave workgroups' waves
// pair up on one SIMD), so a workgroup holds two groups: waves 0 and 1 split one, 2 and 3
// the other, and each pair synchronises through its own LDS counters, not s_barrier.
constexpr int kSplitG = 2;
__device__ __forceinline__ void flag_wait(const int* f, int target) {
	while(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void flag_set(int* f, int v, int lane) {
	// every lane's LDS writes before it are complete (release at workgroup scope); one store
	if(lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ void __launch_bounds__(64 * kSplitW * kSplitG) __attribute__((amdgpu_waves_per_eu(3)))
dp_split_kernel(DevScoring sc, DpLaunch a, uint32_t nprob) {
	__shared__ uint32_t lds_g[kSplitG][(kCols / 4) * 64];   // row info during the fill, then keys / move logs   // row info + window rings during the fill, then keys / move logs
	__shared__ uint32_t pen4[64];
	__shared__ uint32_t t1_g[kSplitG][2][4][64];             // A -> B: h, f, e, hl after A's step b-1
	__shared__ uint32_t t2_g[kSplitG][2][2][64];             // B -> A: H, E state dword of block b/4
	__shared__ int xlr_g[kSplitG][2][64], xnc_g[kSplitG][2][64];   // per wave: last-row max, candidate count
	__shared__ int flags_g[kSplitG][8];                      // t1_ready, t1_used, t2_ready; [4] the pair barrier
	const uint8_t* pen_lds = reinterpret_cast<const uint8_t*>(pen4);
	const int lane = threadIdx.x & 63;
	const int wv = __builtin_amdgcn_readfirstlane((int)((threadIdx.x >> 6) & 1));   // 0 = A, 1 = B
	const int sg = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 7));          // the workgroup's group
	const bool isA = wv == 0;
	uint32_t* lds = lds_g[sg];
	uint32_t (&t1buf)[2][4][64] = t1_g[sg];
	uint32_t (&t2buf)[2][2][64] = t2_g[sg];
	int (&xlr)[2][64] = xlr_g[sg];
	int (&xnc)[2][64] = xnc_g[sg];
	int* flags = flags_g[sg];
	if(threadIdx.x < 64) pen4[lane] = reinterpret_cast<const uint32_t*>(a.mmpen)[lane];
	if(threadIdx.x < kSplitG * 8) flags_g[threadIdx.x >> 3][threadIdx.x & 7] = 0;
	__syncthreads();                                   // (the only workgroup barrier)
	// the two waves of a group meet here (an LDS counter; the other group's waves run on)
	int bphase = 0;
	auto pair_bar = [&]() {
		bphase += 2;
		__threadfence_block();
		if(lane == 0) __hip_atomic_fetch_add(&flags[4], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
		flag_wait(&flags[4], bphase);
	};
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0, st_comp = 0, st_d0 = 0, st_d1 = 0;
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;
	const uint32_t one2 = opaque(0x00010001u);
	for(uint32_t grp = blockIdx.x * kSplitG + (uint32_t)sg; (uint64_t)grp * 64 < nprob; grp += gridDim.x * kSplitG) {
		pair_bar();                                    // the last group's walks are done with lds
		if(isA && lane < 4) flags[lane] = 0;
		uint8_t* gslot = a.scratch + ((size_t)blockIdx.x * kSplitG + (size_t)sg) * (kGroupBytes + kWalkSlotBytes);
		uint32_t* dir = reinterpret_cast<uint32_t*>(gslot + kDirOff);
		uint8_t* lastrow = gslot + kLastRowOff;
		const uint32_t pi = grp * 64 + lane;
		const bool active = grp * 64 + lane < nprob;
		bt2x_dp_in p;
		if(active) p = a.in[pi];
		else { p.read_off = p.qual_off = p.ref_off = 0; p.refl = 0; p.rdlen = 0; p.ncol = 0;
		       p.minsc = 0; p.nceil = 0; p.triml = p.corel = p.corer = 0; p.fw = 1; p.flags = 0; }
		const bool refused = active && ((p.flags & BT2X_DP_I16) || (p.flags & kDpBadWindow));
		const int R = p.rdlen, C = p.ncol;
		constexpr int top = 0xff;
		const int Rmax = __builtin_amdgcn_readfirstlane(wave_max(R));
		const int Cmax = __builtin_amdgcn_readfirstlane(wave_max(C));
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int thr = (int)p.minsc + top;
		// ------------- row info, as dp_fill_kernel: the two waves build alternate 16-row blocks
		const uint32_t kNone = row_info(7, true, npen);
		const ByteStr rds = byte_str(rd, R > 0 ? R : 1), qus = byte_str(qu, R > 0 ? R : 1);
		pair_bar();                                    // the flags are reset
#pragma unroll
		for(int c16 = 0; c16 < kRows / 16; c16++) {
			if((c16 & 1) != wv) continue;               // wave-uniform
			if(c16 * 16 < Rmax) {
				uint32_t rw[4], qw[4];
#pragma unroll
				for(int k = 0; k < 4; k++) { rw[k] = bs_bytes4(rds, 4 * c16 + k); qw[k] = bs_bytes4(qus, 4 * c16 + k); }
#pragma unroll
				for(int k = 0; k < 4; k++) {
					uint32_t w = 0;
#pragma unroll
					for(int r = 0; r < 4; r++) {
						const int i = 16 * c16 + 4 * k + r;
						uint32_t bb = kNone;
						if(i < R) {
							int q = (int)((qw[k] >> (8 * r)) & 0xffu) - 33;
							q = q < 0 ? 0 : q;
							const bool gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
							const int rc = (int)((rw[k] >> (8 * r)) & 0xffu);
							bb = rc > 3 ? row_info(7, gbar, npen) : row_info(rc, gbar, pen_lds[q]);
						}
						w |= bb << (8 * r);
					}
					lds[(4 * c16 + k) * 64 + lane] = w;
				}
			} else {
#pragma unroll
				for(int k = 0; k < 4; k++) lds[(4 * c16 + k) * 64 + lane] = kNone * 0x01010101u;
			}
		}
		pair_bar();
		// ------------- fill
		uint32_t Hs[kRowWords], Es[kRowWords];
#pragma unroll
		for(int bb = 0; bb < kRowWords; bb++) { Hs[bb] = 0; Es[bb] = 0; }
		int lrmax = 0, ncand = 0;
		const int Rmin = __builtin_amdgcn_readfirstlane(-wave_max(-R));
		const uint32_t rdo2 = (uint32_t)rdo * 0x10001u, rde2 = (uint32_t)rde * 0x10001u;
		const uint32_t rfo2 = (uint32_t)rfo * 0x10001u, rfe2 = (uint32_t)rfe * 0x10001u;
		const uint32_t npen2 = (uint32_t)npen * 0x10001u;
		// the exact band (dp_fill_kernel): pair p's steps [2p - wdhi, 2p + wdlo]
		int wdhi = 1 << 20, wdlo = 1 << 20;
		if(a.band) {
			const int mo = imax(1, rdo < rfo ? rdo : rfo);
			int me = rde < rfe ? rde : rfe;
			me = me < mo ? me : mo;
			const int budget = -(int)p.minsc;
			int G = (me <= 0) ? (1 << 16) : (budget < mo ? 0 : 1 + (budget - mo) / me);
			G = G > (1 << 16) ? (1 << 16) : G;
			constexpr int kBandMargin = 2;
			const int dh = active ? (C - R) + G + kBandMargin : -(1 << 20);
			const int dl = active ? G + kBandMargin + 2 : -(1 << 20);
			wdhi = __builtin_amdgcn_readfirstlane(wave_max(dh));
			wdlo = __builtin_amdgcn_readfirstlane(wave_max(dl));
		}
		// the split row at pair p: the middle of the band (block-aligned), kept inside the
		// pair's window; both ends and the middle move down by at most 4 per pair
		const int mid = (int)(((long)wdlo - (long)wdhi) / 2);
		auto window = [&](int pp, int& slo, int& shi, int& b) {
			const int j0 = 2 * pp;
			slo = j0 - wdhi; shi = j0 + wdlo;
			slo = slo < 0 ? 0 : (slo & ~3);
			shi = (shi > Rmax ? Rmax : shi) | 3;
			shi = shi > kSteps - 1 ? kSteps - 1 : shi;
			const int bhi = (shi + 1) & ~3;
			int m = j0 + mid;
			m = m < 0 ? 0 : (m & ~3);
			b = m < slo ? slo : (m > bhi ? bhi : m);
		};
		const int npairs = (Cmax + 1) >> 1;
		const __amdgpu_buffer_rsrc_t dirsrc =
			__builtin_amdgcn_make_buffer_rsrc(dir, 0, (int)(kDirBytesLane * 64u), 0x00020000);
		const uint32_t* rfw = reinterpret_cast<const uint32_t*>(rf);
		const int lastw = ((C > 0 ? C : 1) - 1) >> 2;
		uint32_t cw0 = 0, cw1 = 0, cw2 = 0, cw3 = 0;
		uint32_t refN = 0;
		int bprev = 0, bexec_prev = 0;                    // the last pair's split; whether B ran it
		for(int pp = 0; pp < npairs; pp++) {
			const int j0 = 2 * pp;
			int slo, shi, b;
			window(pp, slo, shi, b);
			const bool execA = b > slo, execB = b <= shi;
			// this wave's steps: A [slo, b] (b: the extra step, not stored), B [b, shi]
			int lo = isA ? slo : b, hi = isA ? (b <= shi ? b : shi) : shi;
			const bool exec = isA ? execA : execB;
			// T2: A takes rows [bprev, bprev + 4) from B when the split moved down past them
			const int t2blk = (isA && exec && pp > 0 && b > bprev && bexec_prev) ? (bprev >> 2) : -1;
			// B publishes its state dword of block b/4 for A's next pair, after the step that
			// completes it (b + 4) or after its last step when that comes first
			int nslo, nshi, nb;
			window(pp + 1, nslo, nshi, nb);
			const bool pub = !isA && execB && pp + 1 < npairs && nb > b;
			const int pubblk = pub ? ((shi >= b + 4) ? (b >> 2) + 1 : (b >> 2)) : -1;
			const int pubsrc = b >> 2;
			if(active && exec) st_comp += 2u * (unsigned)(isA ? (b - slo) : (shi - b + 1));
			int rmin = Rmin, rl = R;
			asm volatile("" : "+s"(rmin), "+s"(lo), "+s"(hi), "+v"(rl));
			asm volatile("" ::: "memory");
			if(kProfWindow && (pp & 7) == 0) {
				const int w0 = pp >> 1;
				cw0 = rfw[min(w0, lastw)]; cw1 = rfw[min(w0 + 1, lastw)];
				cw2 = rfw[min(w0 + 2, lastw)]; cw3 = rfw[min(w0 + 3, lastw)];
				asm volatile("" : "+v"(cw0), "+v"(cw1), "+v"(cw2), "+v"(cw3));
			}
			const uint32_t wsel = (pp & 4) ? ((pp & 2) ? cw3 : cw2) : ((pp & 2) ? cw1 : cw0);
			const uint32_t wsh = (uint32_t)(pp & 1) * 16u;
			const int ca = (j0 < C) ? (int)((wsel >> wsh) & 0xffu) : 4;
			const int cb = (j0 + 1 < C) ? (int)((wsel >> (wsh + 8u)) & 0xffu) : 4;
			const uint32_t refc2 = (uint32_t)ca | ((uint32_t)cb << 16);
			const uint32_t coln = (ca > 3 ? 0x0000ffffu : 0u) | (cb > 3 ? 0xffff0000u : 0u);
			refN |= ((ca > 3) & (j0 < C)) | ((cb > 3) & (j0 + 1 < C));
			const uint32_t pbase = (uint32_t)pp * kPairWords * 256u;
			uint32_t hp = 0, fp = 0, ep = 0, hlp = 0;
			if(!isA) {                                  // T1: A's outputs after step b-1
				flag_wait(&flags[0], pp + 1);
				if(execA) {
					hp = t1buf[pp & 1][0][lane]; fp = t1buf[pp & 1][1][lane];
					ep = t1buf[pp & 1][2][lane]; hlp = t1buf[pp & 1][3][lane];
				}
				flag_set(&flags[1], pp + 1, lane);
			}
			uint32_t t1h = 0, t1f = 0, t1e = 0, t1hl = 0;
			uint32_t tbacc = 0;
			int lra = 0, lrb = 0;
			if(exec) {
			uint32_t cur_iw, cur_iv;
			{
				const int b0 = lo >> 2;
				cur_iw = lds[(b0 < kRowWords ? b0 : kRowWords - 1) * 64 + lane];
				cur_iv = lds[(b0 > 0 ? b0 - 1 : 0) * 64 + lane];
			}
#pragma unroll
			for(int b4 = 0; b4 < kSteps; b4 += 4) {
			if(b4 >= (lo & ~3) && b4 <= hi) {                            // wave-uniform
			const int nbk = (b4 >> 2) + 1;
			const uint32_t nxt_iw = lds[(nbk < kRowWords ? nbk : kRowWords - 1) * 64 + lane];
			if(__builtin_expect((b4 >> 2) == t2blk, 0)) {                // A: rows [bprev, bprev+4) from B
				flag_wait(&flags[2], pp);
				Hs[b4 >> 2 < kRowWords ? b4 >> 2 : kRowWords - 1] = t2buf[(pp - 1) & 1][0][lane];
				Es[b4 >> 2 < kRowWords ? b4 >> 2 : kRowWords - 1] = t2buf[(pp - 1) & 1][1][lane];
			}
			const bool lastA = isA && execB && b4 == b;                 // A's extra step only
#pragma unroll
			for(int st = b4; st < b4 + 4 && st < kSteps; st++) {
				if(st == b4 || !lastA) {
				const int blk = st >> 2, r = st & 3;
				const uint32_t iw = cur_iw, iv = cur_iv;
				const uint32_t info = (st == 0) ? perm(0, iw, 0x0c0c0c00u)
				                    : (st == kRows) ? (perm(iw, 0, 0x0c070c0cu) | (kNone & 0xffu))
				                    : (r == 0) ? perm(iv, iw, 0x0c070c00u)
				                               : perm(0, iw, 0x0c000c00u | ((uint32_t)(r - 1) << 16) | (uint32_t)r);
				const uint32_t hsw = st < kRows ? Hs[blk] : 0u, esw = st < kRows ? Es[blk] : 0u;
				const uint32_t hl = (st == 0) ? perm(0, hsw, 0x0c0c0c00u) | 0x00ff0000u
				                              : perm(hp, hsw, 0x0c040c00u | (uint32_t)r);
				const uint32_t el = (st == 0) ? perm(0, esw, 0x0c0c0c00u)
				                              : perm(ep, esw, 0x0c040c00u | (uint32_t)r);
				const uint32_t hdiag = (st == 0) ? 0x000000ffu : hlp;
				const uint32_t xrc = (info ^ refc2) & 0x00070007u;
				uint32_t pen = pmin(pshr(info, 4), xrc << 8);
				pen = (pen & ~coln) | (npen2 & coln);
				const uint32_t gbm = info & 0x00080008u;
				const uint32_t d = psubs(hdiag, pen);
				const uint32_t r0 = (st == 0) ? 0x00000100u : (st == 1) ? 0x01000000u : 0u;
				const uint32_t rdoe = (gbm << 5) + rdo2, rfoe = (gbm << 5) + (rfo2 + r0), rfee = (gbm << 5) + (rfe2 + r0);
				const uint32_t hl_o = psubs(hl, rdoe), el_e = psubs(el, rde2);
				const uint32_t hu_o = psubs(hp, rfoe), fu_e = psubs(fp, rfee);
				const uint32_t e = pmax(hl_o, el_e);
				const uint32_t f = pmax(hu_o, fu_e);
				const uint32_t h = pmax(pmax(d, e), f);
				uint32_t tb = pmin(xrc, one2);                        // TB_MM
				tb = (tb << 1) | pne(hl_o, e, one2);                   // TB_EONE
				tb = (tb << 1) | pne(hu_o, f, one2);                   // TB_FONE
				tb = (tb << 1) | pne(f, h, one2);                      // TB_FNE
				tb = (tb << 1) | pne(d, h, one2);                      // TB_DNE
				if(__builtin_expect(st + 1 >= rmin, 0)) {
					lra = (st == rl - 1) ? (int)(h & 0xffu) : lra;
					lrb = (st == rl) ? (int)((h >> 16) & 0xffu) : lrb;
				}
				if(st >= 1) {
					const int pb = (st - 1) >> 2, pr = (st - 1) & 3;
					const uint32_t selh = (0x03020100u & ~(0xffu << (8 * pr))) | (6u << (8 * pr));
					Hs[pb] = perm(h, Hs[pb], selh);
					Es[pb] = perm(e, Es[pb], selh);
				}
				// stores: the owner's steps only (A's extra step b is B's first)
				if(!lastA) {
					if(kProfStores && (st & 1)) {
						__builtin_amdgcn_raw_buffer_store_b32(perm(tb, tbacc, 0x06040200u), dirsrc, lane * 4,
						                                      (int)(pbase + (uint32_t)(st >> 1) * 256u), kTbStoreAux);
					} else {
						tbacc = tb;
						if(__builtin_expect(st == shi, 0))
							__builtin_amdgcn_raw_buffer_store_b32(perm(0, tbacc, 0x0c0c0200u), dirsrc, lane * 4,
							                                      (int)(pbase + (uint32_t)(st >> 1) * 256u), kTbStoreAux);
					}
				}
				hlp = hl; hp = h; fp = f; ep = e;
				}
			}
			cur_iv = cur_iw; cur_iw = nxt_iw;
			// A: T1 is its outputs after step b-1, the last step of the block before b
			if(isA && b4 + 4 == b) { t1h = hp; t1f = fp; t1e = ep; t1hl = hlp; }
			// B: its state dword of block b/4 for A's next pair
			if(__builtin_expect((b4 >> 2) == pubblk, 0)) {
				const int sb = pubsrc < kRowWords ? pubsrc : kRowWords - 1;
				// (compile-time index: pubsrc is b4/4 or b4/4 - 1)
				const uint32_t xh = ((b4 >> 2) == pubsrc) ? Hs[b4 >> 2 < kRowWords ? b4 >> 2 : kRowWords - 1]
				                                            : Hs[(b4 >> 2) >= 1 ? (b4 >> 2) - 1 : 0];
				const uint32_t xe = ((b4 >> 2) == pubsrc) ? Es[b4 >> 2 < kRowWords ? b4 >> 2 : kRowWords - 1]
				                                            : Es[(b4 >> 2) >= 1 ? (b4 >> 2) - 1 : 0];
				(void)sb;
				t2buf[pp & 1][0][lane] = xh;
				t2buf[pp & 1][1][lane] = xe;
				flag_set(&flags[2], pp + 1, lane);
			}
			}
			}
			}
			if(isA) {                                   // T1 for B (zeros: A computed nothing)
				if(pp >= 2) flag_wait(&flags[1], pp - 1);
				t1buf[pp & 1][0][lane] = t1h; t1buf[pp & 1][1][lane] = t1f;
				t1buf[pp & 1][2][lane] = t1e; t1buf[pp & 1][3][lane] = t1hl;
				flag_set(&flags[0], pp + 1, lane);
			}
			// last rows: the owner of row R-1 at this pair supplies both of its columns
			const bool own = isA ? (R - 1 < b) : (R - 1 >= b);
			if(own && active) {
				if(j0 < C) {
					lastrow[(size_t)j0 * 64 + lane] = (uint8_t)lra;
					lrmax = imax(lrmax, lra);
					ncand += (lra >= thr);
				}
				if(j0 + 1 < C) {
					lastrow[(size_t)(j0 + 1) * 64 + lane] = (uint8_t)lrb;
					lrmax = imax(lrmax, lrb);
					ncand += (lrb >= thr);
				}
			}
			bprev = b; bexec_prev = execB ? 1 : 0;
		}
		xlr[wv][lane] = lrmax;
		xnc[wv][lane] = ncand;
		pair_bar();
		// ------------- verdict, candidate order and walk: wave w takes lanes 32w .. 32w+31
		const bool mine = (lane >> 5) == wv;
		lrmax = imax(xlr[0][lane], xlr[1][lane]);
		ncand = xnc[0][lane] + xnc[1][lane];
		if(active && mine) {
			st_cells += (unsigned long long)R * C;
			st_cols += C;
			bt2x_dp_out o;
			o.nrec = 0; o.rec_off = 0;
			int status = 0, best = 0;
			dp_verdict(false, lrmax, p.minsc, ncand, status, best);
			if(refused) { status = -1; best = 0; atomicAdd(&a.counters[3], 1u); }
			o.status = status; o.best = best; o.ncand = status > 0 ? (uint16_t)ncand : (uint16_t)0;
			a.out[pi] = o;
			if(status == 0 && a.fail_list && a.band) a.fail_list[atomicAdd(&a.counters[2], 1u)] = pi;
			if(status > 0) {
				// candidate order (DpBtCandidate: score desc, col desc), as dp_fill_kernel's u8 path
				const int nw = (Cmax + 3) >> 2;
				for(int q = 0; q < nw; q++) {
					uint32_t w4 = 0;
					for(int r = 0; r < 4; r++) {
						const int j = q * 4 + r;
						if(j < C) w4 |= (uint32_t)lastrow[(size_t)j * 64 + lane] << (8 * r);
					}
					lds[q * 64 + lane] = w4;
				}
				uint8_t* cands = gslot + kCandOff;
				order_candidates(lds, lane, nw, ncand, one2, [&](int k, int bk) { cands[(size_t)k * 64 + lane] = (uint8_t)(bk & 0xff); });
				uint8_t* wslot = gslot + kGroupBytes;
				walk_problem<64, kPairWords>(sc, pen_lds, a, pi, lane, lane, gslot + kDirOff, kDirBytesLane * 64u, cands,
				                             reinterpret_cast<uint32_t*>(wslot + kEditOff), reinterpret_cast<bt2x_aln_rec*>(wslot + kRecOff),
				                             st_bt, refN != 0, lds, false, st_d0, st_d1);
			}
		}
	}
	if(a.stats) {
		for(int d = 32; d > 0; d >>= 1) {
			st_cells += __shfl_xor(st_cells, d);
			st_cols += __shfl_xor(st_cols, d);
			st_bt += __shfl_xor(st_bt, d);
			st_comp += __shfl_xor(st_comp, d);
		}
		if(lane == 0) {
			atomicAdd(&a.stats[0], st_cells);
			atomicAdd(&a.stats[1], st_cols);
			atomicAdd(&a.stats[2], st_bt);
			atomicAdd(&a.stats[3], st_comp);
		}
	}
}

// ------------------------------------------------------------------ walk kernel
// SwAligner::nextAlignment until done(): per problem, its candidates in order, each
// not already reportedThrough backtraced over the fill's traceback bytes.  Low VGPR use
// keeps many waves resident to hide the walk's dependent load chain.
__global__ void __launch_bounds__(64)
dp_walk_kernel(DevScoring sc, DpLaunch a, uint32_t base, uint32_t nprob) {
	__shared__ uint32_t mlog[kMoveLogWords * 64];             // walk_problem's move logs
	const int lane = threadIdx.x;
	uint8_t* wslot = a.walk_scratch + (size_t)blockIdx.x * kWalkSlotBytes;
	uint32_t* stage_ed = reinterpret_cast<uint32_t*>(wslot + kEditOff);
	bt2x_aln_rec* stage_rec = reinterpret_cast<bt2x_aln_rec*>(wslot + kRecOff);
	unsigned long long st_bt = 0;
	unsigned long long st_dummy0 = 0, st_dummy1 = 0;
	// one wave per 64-problem group, lane = problem: the lanes' main walks follow nearly
	// the same diagonal, so their loads of the lane-interleaved bytes share lines
	for(uint32_t grp = blockIdx.x; (uint64_t)grp * 64 < nprob; grp += gridDim.x) {
		const uint32_t q = grp * 64 + lane;
		if(q < nprob) {
			const uint32_t pi = base + q;
			uint8_t* gs = a.scratch + (size_t)grp * kGroupBytes;
			walk_problem<64, kPairWords>(sc, a.mmpen, a, pi, lane, lane, gs + kDirOff, kDirBytesLane * 64u, gs + kCandOff,
			                             stage_ed, stage_rec, st_bt, true, mlog, false, st_dummy0, st_dummy1);
		}
	}
	if(a.stats) {
		for(int d = 32; d > 0; d >>= 1) st_bt += __shfl_xor(st_bt, d);
		if(lane == 0) atomicAdd(&a.stats[2], st_bt);
	}
}

} // namespace

static int blocks_per_cu(const void* fn, int threads = 64) {
	int nb = 0;
	if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, 0) != hipSuccess || nb < 1) nb = 2;
	return nb;
}

// Resident workgroups per CU of every DP kernel variant, measured once (thread-safe
// static initialisation).
namespace {
struct DpOccupancy {
	int fused[2][2];                // [debug][wide]
	int fill[2][2];                 // split-mode fill kernels
	int walk, wave, duo, split;
	int wave_band[2];               // dp_wave_kernel<0, kPar, true>, [kPar]
	DpOccupancy() {
		wave_band[0] = blocks_per_cu((const void*)dp_wave_kernel<0, false, true>);
		wave_band[1] = blocks_per_cu((const void*)dp_wave_kernel<0, true, true>);
		fused[0][0] = blocks_per_cu((const void*)dp_fill_kernel<false, true, false>);
		fused[1][0] = blocks_per_cu((const void*)dp_fill_kernel<true, true, false>);
		fused[0][1] = blocks_per_cu((const void*)dp_fill_kernel<false, true, true>);
		fused[1][1] = blocks_per_cu((const void*)dp_fill_kernel<true, true, true>);
		fill[0][0] = blocks_per_cu((const void*)dp_fill_kernel<false, false, false>);
		fill[1][0] = blocks_per_cu((const void*)dp_fill_kernel<true, false, false>);
		fill[0][1] = blocks_per_cu((const void*)dp_fill_kernel<false, false, true>);
		fill[1][1] = blocks_per_cu((const void*)dp_fill_kernel<true, false, true>);
		walk = blocks_per_cu((const void*)dp_walk_kernel);
		wave = blocks_per_cu((const void*)dp_wave_kernel<1>);
		duo = blocks_per_cu((const void*)dp_duo_kernel);
		split = blocks_per_cu((const void*)dp_split_kernel, 64 * kSplitW * kSplitG);
	}
};
const DpOccupancy& occupancy() { static const DpOccupancy o; return o; }

// DP modes: fused (default): one persistent kernel fills and walks each group (the walk
// reads bytes written moments ago); split (BT2X_DP_MODE=split, experiments): fill
// kernel over a chunk, then a walk kernel.  Read per launch.
bool dp_split_mode() {
	const char* e = getenv("BT2X_DP_MODE");
	return e && e[0] == 's';
}

// Largest launch run one wave per problem (BT2X_DP_WAVE=0: never, =1: always; else
// BT2X_DP_WAVE_MAX problems, default 32768: below that a lane-per-problem launch does not
// fill the chip and costs its serial R x C fill anyway).
// The nextAlignment sequence of the wave kernel on every lane (walk_wave_par): the walks the
// lane kernel hands over (default on; BT2X_DP_PARWALK=0: lane 0 as before) and, with
// BT2X_DP_PARWALK=2, the small launches too.  Read per launch (tests switch it).
int dp_parwalk() {
	const char* e = getenv("BT2X_DP_PARWALK");
	return e ? (e[0] - '0') : 1;
}

// The two-lanes-per-problem fill (dp_duo_kernel) for banded u8 launches of at most
// BT2X_DP_DUO_MAX problems (default 65536: about one 64-problem group per SIMD, where one
// lane's chain is the launch's latency; larger launches fill the SIMDs with dp_fill_kernel's
// waves, and the duo kernel's extra steps would cost throughput).  BT2X_DP_DUO=0: never,
// =1: always.  Read per launch (tests switch it).
bool dp_duo(uint32_t n) {
	const char* e = getenv("BT2X_DP_DUO");
	if(e && e[0] == '0') return false;
	if(e && e[0] == '1') return true;
	const char* x = getenv("BT2X_DP_DUO_MAX");
	return n <= (x ? (uint32_t)atoll(x) : 65536u);
}

// The two-wave split fill (dp_split_kernel): off by default (BT2X_DP_SPLIT=1: every banded
// u8 launch of at most BT2X_DP_SPLIT_MAX problems, default 131072; it then takes precedence
// over the duo fill).  Measured at the timed run's cohort shapes (round 6):
// halving each wave's sweep leaves the fill within 3 % (77.6 vs 80.0 ms of fill-only
// replay) -- the fill there is bound by its traceback stores' memory path, not by one
// wave's dependent chain -- and the whole DP 5 % slower.  Read per launch (tests switch it).
bool dp_split(uint32_t n) {
	const char* e = getenv("BT2X_DP_SPLIT");
	if(!(e && e[0] == '1')) return false;
	const char* x = getenv("BT2X_DP_SPLIT_MAX");
	return n <= (x ? (uint32_t)atoll(x) : 131072u);
}

// The banded traceback layout of the wave kernels (default on; in the small-launch mode it
// needs the hand-over list, i.e. BT2X_DP_HEAVY != 0; BT2X_DP_WAVE_BAND=0: whole rectangles
// in LDS, column-major, 4 rows a lane, as up to round 5).
// Read per launch (tests switch it).
bool dp_wave_band() {
	const char* e = getenv("BT2X_DP_WAVE_BAND");
	return !(e && e[0] == '0');
}

uint32_t dp_wave_max() {                        // read per launch (tests switch modes)
	const char* w = getenv("BT2X_DP_WAVE");
	const char* x = getenv("BT2X_DP_WAVE_MAX");
	return (w && w[0] == '0') ? 0u : (w && w[0] == '1') ? 0xffffffffu : (x ? (uint32_t)atoll(x) : 32768u);
}

template<bool kDebug, bool kFused>
void launch_fill(bool wide, uint32_t grid, hipStream_t s, const DevScoring& sc, const DpLaunch& a, uint32_t base,
                 uint32_t np) {
	if(wide) hipLaunchKernelGGL((dp_fill_kernel<kDebug, kFused, true>), dim3(grid), dim3(64), 0, s, sc, a, base, np);
	else hipLaunchKernelGGL((dp_fill_kernel<kDebug, kFused, false>), dim3(grid), dim3(64), 0, s, sc, a, base, np);
}
} // namespace

// Scratch: split = `chunk_groups` fill group regions + one staging slot per resident walk
// wave; fused = one group region + staging slot per resident fill wave (the wave-per-
// problem mode uses the same region as per-wave record staging).
size_t bt2x_dp_scratch_bytes(int ncu, uint32_t chunk_groups) {
	const DpOccupancy& o = occupancy();
	if(!dp_split_mode()) {
		int nb = 0;
		for(int d = 0; d < 2; d++) for(int w = 0; w < 2; w++) nb = max(nb, o.fused[d][w]);
		nb = max(nb, max(o.duo, o.split * kSplitG));
		return (size_t)ncu * nb * (kGroupBytes + kWalkSlotBytes);
	}
	return (size_t)chunk_groups * kGroupBytes + (size_t)ncu * o.walk * kWalkSlotBytes;
}

int bt2x_launch_dp(const DevScoring& sc, const DpLaunch& a0, void* stream) {
	if(a0.n == 0) return 0;
	hipStream_t s = (hipStream_t)stream;
	const DpOccupancy& occ = occupancy();
	const bool dbg = a0.digests || a0.cands;
	const bool wide = a0.wide != 0;
	DpLaunch a = a0;
	const uint32_t groups_all = (a0.n + 63) / 64;
	if(!dbg && a0.n <= dp_wave_max()) {
		// small launch: one wave per problem (persistent; 4 waves per CU with whole
		// rectangles in LDS, 8 with the banded layout); it fills whole rectangles, so every
		// best is exact
		const bool band = a0.heavy_list != nullptr && dp_wave_band();
		const bool par = dp_parwalk() >= 2;
		const size_t slots = bt2x_dp_scratch_bytes(a0.ncu, a0.chunk_groups) / kWaveRecStageBytes;
		uint32_t wb = (uint32_t)a0.ncu * (band ? (uint32_t)occ.wave_band[par ? 1 : 0] : 4u);
		if(wb > slots) wb = (uint32_t)slots;
		if(wb > a0.n) wb = a0.n;
		if(band) {
			if(par) hipLaunchKernelGGL((dp_wave_kernel<0, true, true>), dim3(wb), dim3(64), 0, s, sc, a);
			else hipLaunchKernelGGL((dp_wave_kernel<0, false, true>), dim3(wb), dim3(64), 0, s, sc, a);
			// the problems handed over: band window too wide, or many candidates
			uint32_t wb2 = (uint32_t)a0.ncu * 4u;
			if(wb2 > slots) wb2 = (uint32_t)slots;
			if(wb2 > a0.n) wb2 = a0.n;
			if(dp_parwalk() >= 1) hipLaunchKernelGGL((dp_wave_kernel<2, true, true>), dim3(wb2), dim3(64), 0, s, sc, a);
			else hipLaunchKernelGGL((dp_wave_kernel<2, false, true>), dim3(wb2), dim3(64), 0, s, sc, a);
		} else if(par) hipLaunchKernelGGL((dp_wave_kernel<0, true>), dim3(wb), dim3(64), 0, s, sc, a);
		else hipLaunchKernelGGL((dp_wave_kernel<0, false>), dim3(wb), dim3(64), 0, s, sc, a);
		return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
	}
	if(!dbg && !wide && a0.band && !dp_split_mode() && dp_split(a0.n)) {
		uint32_t fb = (uint32_t)a0.ncu * (uint32_t)occ.split;
		if(fb > (groups_all + kSplitG - 1) / kSplitG) fb = (groups_all + kSplitG - 1) / kSplitG;
		hipLaunchKernelGGL(dp_split_kernel, dim3(fb), dim3(64 * kSplitW * kSplitG), 0, s, sc, a, a0.n);
	} else if(!dbg && !wide && a0.band && !dp_split_mode() && dp_duo(a0.n)) {
		const uint32_t groups = (a0.n + kDuoG - 1) / kDuoG;
		uint32_t fb = (uint32_t)a0.ncu * (uint32_t)occ.duo;
		if(fb > groups) fb = groups;
		hipLaunchKernelGGL(dp_duo_kernel, dim3(fb), dim3(64), 0, s, sc, a, a0.n);
	} else if(!dp_split_mode()) {
		uint32_t fb = (uint32_t)a0.ncu * (uint32_t)occ.fused[dbg ? 1 : 0][wide ? 1 : 0];
		if(fb > groups_all) fb = groups_all;
		if(dbg) launch_fill<true, true>(wide, fb, s, sc, a, 0u, a0.n);
		else launch_fill<false, true>(wide, fb, s, sc, a, 0u, a0.n);
	} else {
		a.walk_scratch = a0.scratch + (size_t)a0.chunk_groups * kGroupBytes;
		a.heavy_list = nullptr;                  // no redo pass here: the walk kernel walks everything
		const uint32_t chunk = a0.chunk_groups * 64;
		for(uint32_t base = 0; base < a0.n; base += chunk) {
			const uint32_t np = (a0.n - base < chunk) ? a0.n - base : chunk;
			const uint32_t groups = (np + 63) / 64;
			uint32_t fb = (uint32_t)a0.ncu * (uint32_t)occ.fill[dbg ? 1 : 0][wide ? 1 : 0];
			if(fb > groups) fb = groups;
			if(dbg) launch_fill<true, false>(wide, fb, s, sc, a, base, np);
			else launch_fill<false, false>(wide, fb, s, sc, a, base, np);
			if(a0.ablate == 1) continue;
			uint32_t wb = (uint32_t)a0.ncu * (uint32_t)occ.walk;
			if(wb > groups) wb = groups;
			hipLaunchKernelGGL(dp_walk_kernel, dim3(wb), dim3(64), 0, s, sc, a, base, np);
		}
	}
	// exact best of the problems the banded fill failed (queued in a.fail_list)
	if(a0.fail_list && a0.band && !dbg) {
		const uint32_t wb = (uint32_t)a0.ncu * (uint32_t)occ.wave;
		hipLaunchKernelGGL(dp_wave_kernel<1>, dim3(wb), dim3(64), 0, s, sc, a);
	}
	// the walks the lane kernel handed over (a.heavy_list): one wave per problem
	if(a0.heavy_list && !dbg && !dp_split_mode()) {
		uint32_t wb = (uint32_t)a0.ncu * 4u;
		const size_t slots = bt2x_dp_scratch_bytes(a0.ncu, a0.chunk_groups) / kWaveRecStageBytes;
		if(wb > slots) wb = (uint32_t)slots;
		const bool band = dp_wave_band();
		if(dp_parwalk() >= 1) {
			if(band) hipLaunchKernelGGL((dp_wave_kernel<2, true, true>), dim3(wb), dim3(64), 0, s, sc, a);
			else hipLaunchKernelGGL((dp_wave_kernel<2, true>), dim3(wb), dim3(64), 0, s, sc, a);
		} else {
			if(band) hipLaunchKernelGGL((dp_wave_kernel<2, false, true>), dim3(wb), dim3(64), 0, s, sc, a);
			else hipLaunchKernelGGL((dp_wave_kernel<2, false>), dim3(wb), dim3(64), 0, s, sc, a);
		}
	}
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
