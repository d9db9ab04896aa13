// dp_kernel.hip — end-to-end u8 DP fill + candidate extraction + full backtrace
// enumeration on gfx950, one DP problem per lane.
//
// Replaces SwAligner::align -> alignEnd2EndSseU8 (aligner_swsse_ee_u8.cpp:542-671:
// EEU8_alignOne / EEU8_lazyF / EEU8_alignNucleotides :249-536) and the loop of
// SwAligner::nextAlignment calls (aligner_sw.cpp:252-375) with
// backtraceNucleotidesEnd2EndSseU8 (u8.cpp:746-1352).
//
// Design (MI355X-first, not a Farrar port):
//  * One problem per lane, 64 problems per wave; the lane sweeps its matrix column by
//    column and computes the exact saturating-u8 recurrence (no striping, no lazy-F
//    loop: every stored value equals the striped kernel's).
//  * Per-row state (H and E of the previous column, the read code and its quality's
//    mismatch penalty) lives in LDS, one dword per row per lane, lane-interleaved so a
//    wave's access to a row is 64 consecutive dwords (conflict-free).
//  * Instead of materialising E/F/H (3 B/cell in the reference) the fill writes ONE
//    traceback byte per cell: the predecessor the reference's backtrace would pick for
//    the H, E and F cell (its fixed priority diag > H-up > F-up > H-left > E-left,
//    u8.cpp:968-990 and :843-916), plus bit 7 = reportedThrough.  The backtrace only ever
//    consults a cell on its first visit (a second visit hits reportedThrough and fails),
//    so this byte is all it needs.  Four rows are packed per dword; each wave store is
//    256 contiguous bytes.
//  * Candidates (last-row cells with score >= minsc) are enumerated in DpBtCandidate
//    order (score desc, col desc; aligner_sw_nuc.h:149) and backtraced in-kernel; only
//    the final edit lists leave the GPU.
// Algorithmic bytes per problem = R*C (traceback bytes written) + C (reference window)
// + 2*R (read codes + qualities) — SURVEY §8(d)'s 3*R*C for the reference's matrix.
#include <hip/hip_runtime.h>
#include "bt2x_device.h"

namespace {

constexpr int kRows = BT2X_MAX_ROWS;          // 160
constexpr int kRowWords = kRows / 4;          // traceback dwords per column
constexpr int kCols = BT2X_MAX_COLS;          // 200
constexpr uint32_t kDirBytesLane = kCols * kRowWords * 4;       // 32000
constexpr uint32_t kLastRowBytesLane = 256;
constexpr uint32_t kEditStage = 400;                               // >= R + C + 2
constexpr uint32_t kRecStage = 200;                                // >= ncand
// scratch layout of one wave slot (all regions lane-interleaved)
constexpr size_t kDirOff = 0;
constexpr size_t kLastRowOff = kDirOff + (size_t)kDirBytesLane * 64;
constexpr size_t kEditOff = kLastRowOff + (size_t)kLastRowBytesLane * 64;
constexpr size_t kRecOff = kEditOff + (size_t)kEditStage * 4 * 64;
constexpr size_t kSlotBytes = kRecOff + (size_t)kRecStage * sizeof(bt2x_aln_rec) * 64;
static_assert(kSlotBytes <= (size_t)BT2X_DP_SCRATCH_PER_LANE * 64, "scratch slot too small");

enum { H_NONE = 0, H_DIAG = 1, H_REF_OPEN = 2, H_RFGAP_EXT = 3, H_READ_OPEN = 4, H_RDGAP_EXT = 5 };
enum { EDIT_READ_GAP = 1, EDIT_REF_GAP = 2, EDIT_MM = 3 };

__device__ __forceinline__ int sat(int v) { return v < 0 ? 0 : v; }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t pack_edit(uint32_t pos, int type, int chr, int qchr) {
	return (pos & 0x3ffu) | ((uint32_t)type << 12) | ((uint32_t)(uint8_t)chr << 16) |
	       ((uint32_t)(uint8_t)qchr << 24);
}

__device__ __forceinline__ char acgtn(int c) { return c == 0 ? 'A' : c == 1 ? 'C' : c == 2 ? 'G' : c == 3 ? 'T' : 'N'; }
// mask2dna of a single-base mask 1<<c (c = 4 -> mask 16 -> 'N'), alphabet.cpp:71
__device__ __forceinline__ char mask_chr(int c) { return acgtn(c); }

__device__ __forceinline__ uint64_t cell_digest(uint32_t row, uint32_t col, uint32_t mat, uint32_t val) {
	uint64_t z = ((uint64_t)row << 40) ^ ((uint64_t)col << 20) ^ ((uint64_t)mat << 16) ^ (uint64_t)val;
	z += 0x9e3779b97f4a7c15ULL;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
	return z ^ (z >> 31);
}

struct BtResult {
	int score, ns, gaps, nedit, bases, refns, off;
};

__device__ __forceinline__ int wave_max(int v) {
	for(int d = 32; d > 0; d >>= 1) { const int o = __shfl_xor(v, d); v = v > o ? v : o; }
	return v;
}

// Per-row info byte kept in LDS during the fill: read code (3 bits), gap-barrier flag
// (bit 3), mismatch penalty for the row's quality (bits 4-7; Scoring::mmpens <= 15).
__device__ __forceinline__ uint32_t row_info(int rdc, bool gbar, int mm) {
	return (uint32_t)rdc | (gbar ? 8u : 0u) | ((uint32_t)mm << 4);
}

template<bool kDebug>
__global__ void __launch_bounds__(64)
dp_kernel(DevScoring sc, DpLaunch a) {
	// LDS, reused: during the fill the row-info bytes (4 rows per dword), afterwards the
	// last DP row (4 columns per dword) for candidate enumeration.  12.8 KiB per wave.
	__shared__ uint32_t lds[(kCols / 4) * 64];
	const int lane = threadIdx.x;
	uint8_t* slot = a.scratch + (size_t)blockIdx.x * kSlotBytes;
	uint32_t* dir = reinterpret_cast<uint32_t*>(slot + kDirOff);
	uint8_t* lastrow = slot + kLastRowOff;
	uint32_t* stage_ed = reinterpret_cast<uint32_t*>(slot + kEditOff);
	bt2x_aln_rec* stage_rec = reinterpret_cast<bt2x_aln_rec*>(slot + kRecOff);
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0;
	const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe, npen = sc.npen;

	for(uint32_t chunk = blockIdx.x; (uint64_t)chunk * 64 < a.n; chunk += gridDim.x) {
		const uint32_t pi = chunk * 64 + lane;
		const bool active = pi < a.n;
		bt2x_dp_in p;
		if(active) p = a.in[pi];
		else { p.read_off = p.qual_off = p.ref_off = 0; p.refl = 0; p.rdlen = 0; p.ncol = 0;
		       p.minsc = 0; p.nceil = 0; p.triml = p.corel = p.corer = 0; p.fw = 1; p.pad = 0; }
		const int R = p.rdlen, C = p.ncol;
		const int Rmax = wave_max(R), Cmax = wave_max(C);
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int thr = (int)p.minsc + 0xff;
		// ------------- row info (rows >= R: N, barred, no penalty) ----------------
		// 4 rows per dword, held in VGPRs for the whole fill (constant per problem)
		uint32_t Info[kRowWords];
#pragma unroll
		for(int blk = 0; blk < kRowWords; blk++) {
			uint32_t w = row_info(4, true, 0) * 0x01010101u;
			if(blk * 4 < Rmax) {
				w = 0;
#pragma unroll
				for(int r = 0; r < 4; r++) {
					const int i = blk * 4 + r;
					uint32_t b = row_info(4, true, 0);
					if(i < R) {
						int q = (int)qu[i] - 33;
						q = q < 0 ? 0 : (q > 255 ? 255 : q);
						const bool gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
						b = row_info(rd[i], gbar, sc.mmpen[q]);
					}
					w |= b << (8 * r);
				}
			}
			Info[blk] = w;
		}
		// ------------- fill: column-major, per-row state in VGPRs --------------
		// H and E of the previous column, 4 rows per dword (40 dwords each for 160 rows).
		uint32_t Hs[kRowWords], Es[kRowWords];
#pragma unroll
		for(int b = 0; b < kRowWords; b++) { Hs[b] = 0; Es[b] = 0; }
		uint64_t dg0 = 0, dg1 = 0, dg2 = 0;
		int lrmax = 0, ncand = 0;
		const int lastblk = (R - 1) >> 2, lastsh = 8 * ((R - 1) & 3);
		int refn = (C > 0) ? rf[0] : 4;
		for(int j = 0; j < Cmax; j++) {
			const int refc = refn;
			if(j + 1 < C) refn = rf[j + 1];            // prefetch next column's base
			const bool colok = j < C;
			const bool refamb = refc > 3;
			int hdiag = 0xff, hup = 0, fup = 0;        // H[-1][j-1] = 0xff: start anywhere
			uint32_t lrw = 0;
#pragma unroll
			for(int blk = 0; blk < kRowWords; blk++) {
				if(blk * 4 < Rmax) {                     // wave-uniform
				uint32_t info = Info[blk];
				asm volatile("" : "+v"(info));      // keep the per-row fields from being hoisted (VGPR blow-up)
				const uint32_t hw = Hs[blk], ew = Es[blk];
				uint32_t nh = 0, ne = 0, tbw = 0;
#pragma unroll
				for(int r = 0; r < 4; r++) {
					const int i = blk * 4 + r;
					const int hl = (int)((hw >> (8 * r)) & 0xffu);
					const int el = (int)((ew >> (8 * r)) & 0xffu);
					const uint32_t inf = (info >> (8 * r)) & 0xffu;
					const int rdc = (int)(inf & 7u);
					const bool gb = (inf & 8u) != 0;
					const int mm = (int)(inf >> 4);
					const int pen = (refamb || rdc > 3) ? npen : (rdc == refc ? 0 : mm);
					// E[i][j] = max(E[i][j-1] - rde, H[i][j-1] - rdo (barred rows: none)), >= 0
					const int hl_o = hl - rdo, el_e = el - rde;
					const int e = imax(imax(el_e, gb ? 0 : hl_o), 0);
					// F[i][j] = max(F[i-1][j] - rfe, H[i-1][j] - rfo), barred rows 0, row 0 = 0
					const int hu_o = hup - rfo, fu_e = fup - rfe;
					const int f = (i == 0 || gb) ? 0 : imax(imax(hu_o, fu_e), 0);
					const int d = ((i == 0) ? 0xff : hdiag) - pen;
					const int h = imax(imax(d, e), f);
					uint32_t tb = 0;
					if(i > 0) {
						// Traceback choice of backtraceNucleotidesEnd2EndSseU8 for each cell type.
						// Exact for every cell a backtrace can reach (value >= 1).
						// branch-free: 0/1 flags combined arithmetically
						const uint32_t f_open = hu_o == f, f_ext = (fu_e == f) & !f_open;
						const uint32_t e_open = hl_o == e, e_ext = (el_e == e) & !e_open;
						const uint32_t fd = f_open | (f_ext << 1), ed = e_open | (e_ext << 1);
						const uint32_t isd = d == h;
						const uint32_t isf = (f == h) & !isd;
						const uint32_t ise = (e == h) & !isd & !isf;
						const uint32_t hd = isd | (isf * (fd + 1)) | (ise * (ed + 3));
						tb = hd | (ed << 3) | (fd << 5);
					}
					if(kDebug && a.digests && colok && i < R) {
						dg0 += cell_digest(i, j, 0, e);
						dg1 += cell_digest(i, j, 1, f);
						dg2 += cell_digest(i, j, 2, h);
					}
					nh |= (uint32_t)h << (8 * r);
					ne |= (uint32_t)e << (8 * r);
					tbw |= tb << (8 * r);
					hdiag = hl; hup = h; fup = f;
				}
				Hs[blk] = nh; Es[blk] = ne;
				lrw = (blk == lastblk) ? nh : lrw;
				if(colok) dir[((size_t)j * kRowWords + blk) * 64 + lane] = tbw;
				}
			}
			if(colok) {
				const int lr = (int)((lrw >> lastsh) & 0xffu);
				lastrow[(size_t)j * 64 + lane] = (uint8_t)lr;
				lrmax = imax(lrmax, lr);
				ncand += (lr >= thr);
			}
		}
		if(!active || a.ablate) continue;
		st_cells += (unsigned long long)R * C;
		st_cols += C;
		if(kDebug && a.digests) {
			a.digests[3 * (size_t)pi + 0] = dg0;
			a.digests[3 * (size_t)pi + 1] = dg1;
			a.digests[3 * (size_t)pi + 2] = dg2;
		}
		bt2x_dp_out o;
		o.nrec = 0; o.rec_off = 0;
		const int score = lrmax - 0xff;
		if(score < p.minsc) {
			o.status = 0; o.best = score; o.ncand = 0;
			a.out[pi] = o;
			if(kDebug && a.cands)
				for(int k = 0; k < kCols; k++) a.cands[(size_t)pi * kCols + k] = 0xffffffffu;
			continue;
		}
		o.status = ncand > 0 ? 1 : 0; o.best = score; o.ncand = (uint16_t)ncand;
		// ------------- nextAlignment() sequence until done() -----------------
		// move the last row into LDS (the row state is no longer needed)
		for(int q = 0; q < (C + 3) >> 2; q++) {
			uint32_t w4 = 0;
			for(int r = 0; r < 4; r++) {
				const int j = q * 4 + r;
				if(j < C) w4 |= (uint32_t)lastrow[(size_t)j * 64 + lane] << (8 * r);
			}
			lds[q * 64 + lane] = w4;
		}
		int cur_key = 0x7fffffff, ndone = 0, nrec = 0;
		const int row0 = R - 1;
		while(ndone < ncand) {
			int ntries = 0;
			bool found = false;
			BtResult res;
			res.nedit = 0;
			while(ndone < ncand) {
				// next candidate in DpBtCandidate order: largest key = score*256+col below cur_key
				// (4 columns per LDS dword; columns >= C hold 0 and never qualify)
				int best = -1;
				const int nw = (C + 3) >> 2;
#pragma unroll 2
				for(int q = 0; q < nw; q++) {
					const uint32_t w4 = lds[q * 64 + lane];
#pragma unroll
					for(int r = 0; r < 4; r++) {
						const int s = (int)((w4 >> (8 * r)) & 0xffu);
						const int key = s * 256 + q * 4 + r;
						best = (s >= thr && key < cur_key && key > best) ? key : best;
					}
				}
				if(best < 0) { ndone = ncand; break; }   // unreachable: ncand counted above
				cur_key = best;
				const int col0 = best & 0xff;
				if(kDebug && a.cands)
					a.cands[(size_t)pi * kCols + ndone] = BT2X_CAND_PACK(row0, col0, best >> 8);
				ndone++;
				// candidate start cell already traversed -> skipped, no RNG draw
				{
					const uint32_t w = dir[((size_t)col0 * kRowWords + (row0 >> 2)) * 64 + lane];
					if((w >> (8 * (row0 & 3) + 7)) & 1) continue;
				}
				ntries++;
				// ------------- backtraceNucleotidesEnd2EndSseU8 -------------
				int row = row0, col = col0, ct = 2 /*H*/, bscore = 0, ns = 0, gaps = 0, ne = 0;
				bool over_core = false, ok = true;
				int trimBeg = 0;
				// One dependent load round trip per step: the next cell's traceback byte and
				// its read/ref/quality bytes are issued before this cell's stores (the mark
				// byte and the staged edit), so the in-order vmcnt never waits on a store.
				const uint8_t* dir8 = reinterpret_cast<const uint8_t*>(dir);
				uint8_t* dirw8 = reinterpret_cast<uint8_t*>(dir);
				size_t bi = (((size_t)col * kRowWords + (row >> 2)) * 64 + lane) * 4 + (row & 3);
				uint32_t tb = dir8[bi];
				int rdc = rd[row], refc = rf[col], qch = qu[row];
				while(true) {
					st_bt++;
					if(tb & 0x80u) { ok = false; break; }          // reportedThrough
					int move = H_NONE;
					bool empty = false;
					if(row > 0) {
						if(ct == 2) move = (int)(tb & 7u);
						else if(ct == 0) { const int ed = (int)((tb >> 3) & 3u); move = ed == 1 ? H_READ_OPEN : ed == 2 ? H_RDGAP_EXT : H_NONE; }
						else { const int fd = (int)((tb >> 5) & 3u); move = fd == 1 ? H_REF_OPEN : fd == 2 ? H_RFGAP_EXT : H_NONE; }
						empty = (move == H_NONE);
					}
					const int diag = col - row + (int)p.triml;
					if(diag >= 0 && diag >= (int)p.corel && diag <= (int)p.corer) over_core = true;
					const size_t cur_bi = bi;
					const uint32_t cur_tb = tb;
					if(empty || row == 0) {
						dirw8[cur_bi] = (uint8_t)(cur_tb | 0x80u);  // setReportedThrough
						trimBeg = row;
						break;
					}
					const int crow = row, ccol = col, crdc = rdc, crefc = refc, cq = qch;
					// next cell
					if(move == H_DIAG) { row--; col--; ct = 2; }
					else if(move == H_REF_OPEN || move == H_RFGAP_EXT) { row--; ct = (move == H_REF_OPEN) ? 2 : 1; }
					else { col--; ct = (move == H_READ_OPEN) ? 2 : 0; }
					bi = (((size_t)col * kRowWords + (row >> 2)) * 64 + lane) * 4 + (row & 3);
					tb = dir8[bi];
					rdc = rd[row]; refc = rf[col]; qch = qu[row];
					// stores for the cell just left
					dirw8[cur_bi] = (uint8_t)(cur_tb | 0x80u);      // setReportedThrough
					if(move == H_DIAG) {
						const bool amb = crdc > 3 || crefc > 3;
						if(amb || crdc != crefc) {
							const int q0 = cq - 33;
							const int q = q0 < 0 ? 0 : (q0 > 255 ? 255 : q0);
							stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)crow, EDIT_MM, mask_chr(crefc), acgtn(crdc));
							ne++;
							bscore -= amb ? sc.npen : (int)sc.mmpen[q];
						}
						if(amb) ns++;
					} else if(move == H_REF_OPEN || move == H_RFGAP_EXT) {
						stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)crow, EDIT_REF_GAP, '-', acgtn(crdc));
						ne++;
						bscore -= (move == H_REF_OPEN) ? rfo : rfe;
						gaps++;
					} else {
						stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)crow + 1, EDIT_READ_GAP, mask_chr(crefc), '-');
						ne++;
						bscore -= (move == H_READ_OPEN) ? rdo : rde;
						gaps++;
					}
					(void)ccol;
				}
				if(!ok || !over_core) continue;
				{
					const bool amb = rdc > 3 || refc > 3;
					if(amb || rdc != refc) {
						const int q0 = qch - 33;
						const int q = q0 < 0 ? 0 : (q0 > 255 ? 255 : q0);
						stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)row, EDIT_MM, mask_chr(refc), acgtn(rdc));
						ne++;
						bscore -= amb ? sc.npen : (int)sc.mmpen[q];
					}
					if(amb) ns++;
				}
				if(ns > p.nceil) continue;
				int refns = 0;
				for(int k = col; k <= col0; k++) refns += (rf[k] > 3);
				const int extent = R - trimBeg - (R - row0 - 1);
				res.score = bscore; res.ns = ns; res.gaps = gaps; res.nedit = ne;
				res.bases = extent - ne; res.refns = refns; res.off = col;
				// publish the edit list in ned() order: reverse(), pos -= trimBeg, and for
				// the reverse-complement strand invertEdits() (edit.cpp:50-78)
				const uint32_t eo = atomicAdd(&a.counters[1], (uint32_t)ne);
				if(eo + (uint32_t)ne <= a.edit_cap) {
					for(int k = 0; k < ne; k++) {
						const uint32_t e = stage_ed[(size_t)(p.fw ? ne - 1 - k : k) * 64 + lane];
						uint32_t pos = (e & 0x3ffu) - (uint32_t)trimBeg;
						if(!p.fw) pos = (uint32_t)extent - pos - (((e >> 12) & 7u) == EDIT_READ_GAP ? 0u : 1u);
						a.edits[eo + k] = (e & ~0x3ffu) | (pos & 0x3ffu);
					}
				}
				found = true;
				{
					bt2x_aln_rec r;
					r.ntries = (uint16_t)ntries; r.ok = 1; r.pad0 = 0;
					r.score = (int16_t)res.score; r.ns = (uint16_t)res.ns; r.gaps = (uint16_t)res.gaps;
					r.nedit = (uint16_t)res.nedit; r.bases_aligned = (uint16_t)res.bases;
					r.refns = (uint16_t)res.refns; r.refoff = (int64_t)res.off + p.refl;
					r.edit_off = eo; r.pad1 = 0;
					stage_rec[(size_t)nrec * 64 + lane] = r;
				}
				break;
			}
			if(!found) {
				bt2x_aln_rec r;
				r.ntries = (uint16_t)ntries; r.ok = 0; r.pad0 = 0; r.score = 0; r.ns = 0; r.gaps = 0;
				r.nedit = 0; r.bases_aligned = 0; r.refns = 0; r.refoff = 0; r.edit_off = 0; r.pad1 = 0;
				stage_rec[(size_t)nrec * 64 + lane] = r;
				nrec++;
				break;
			}
			nrec++;
		}
		const uint32_t ro = atomicAdd(&a.counters[0], (uint32_t)nrec);
		if(ro + (uint32_t)nrec <= a.rec_cap)
			for(int k = 0; k < nrec; k++) a.recs[ro + k] = stage_rec[(size_t)k * 64 + lane];
		o.nrec = (uint16_t)nrec; o.rec_off = ro;
		a.out[pi] = o;
		if(kDebug && a.cands)
			for(int k = ncand; k < kCols; k++) a.cands[(size_t)pi * kCols + k] = 0xffffffffu;
	}
	if(a.stats) {
		for(int d = 32; d > 0; d >>= 1) {
			st_cells += __shfl_xor(st_cells, d);
			st_cols += __shfl_xor(st_cols, d);
			st_bt += __shfl_xor(st_bt, d);
		}
		if(lane == 0) {
			atomicAdd(&a.stats[0], st_cells);
			atomicAdd(&a.stats[1], st_cols);
			atomicAdd(&a.stats[2], st_bt);
		}
	}
}

} // namespace

size_t bt2x_dp_slot_bytes() { return kSlotBytes; }

// Resident 64-lane workgroups per CU for the DP kernel (VGPR/LDS-limited), so the
// persistent grid fills the chip exactly once.
int bt2x_dp_blocks_per_cu() {
	int nb = 0;
	if(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dp_kernel<false>, 64, 0) != hipSuccess || nb < 1) nb = 4;
	return nb;
}

int bt2x_launch_dp(const DevScoring& sc, const DpLaunch& a, void* stream) {
	if(a.n == 0) return 0;
	uint32_t waves = (a.n + 63) / 64;
	if(waves > a.nslots) waves = a.nslots;
	if(a.digests || a.cands)
		hipLaunchKernelGGL(dp_kernel<true>, dim3(waves), dim3(64), 0, (hipStream_t)stream, sc, a);
	else
		hipLaunchKernelGGL(dp_kernel<false>, dim3(waves), dim3(64), 0, (hipStream_t)stream, sc, a);
	return hipGetLastError() == hipSuccess ? 0 : BT2X_E_NODEVICE;
}
