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

template<bool kDebug>
__global__ void __launch_bounds__(64)
dp_kernel(DevScoring sc, DpLaunch a) {
	__shared__ uint32_t rowst[kRows * 64];       // per row: H | E<<8 | rdc<<16 | mmpen<<24
	const int lane = threadIdx.x;
	uint8_t* slot = a.scratch + (size_t)blockIdx.x * kSlotBytes;
	uint32_t* dir = reinterpret_cast<uint32_t*>(slot + kDirOff);
	uint8_t* lastrow = slot + kLastRowOff;
	uint32_t* stage_ed = reinterpret_cast<uint32_t*>(slot + kEditOff);
	bt2x_aln_rec* stage_rec = reinterpret_cast<bt2x_aln_rec*>(slot + kRecOff);
	unsigned long long st_cells = 0, st_cols = 0, st_bt = 0;

	for(uint32_t chunk = blockIdx.x; (uint64_t)chunk * 64 < a.n; chunk += gridDim.x) {
		const uint32_t pi = chunk * 64 + lane;
		if(pi >= a.n) continue;
		const bt2x_dp_in p = a.in[pi];
		const int R = p.rdlen, C = p.ncol;
		const uint8_t* rd = a.reads + p.read_off;
		const uint8_t* qu = a.quals + p.qual_off;
		const uint8_t* rf = a.refs + p.ref_off;
		const int thr = (int)p.minsc + 0xff;
		for(int i = 0; i < R; i++) {
			const int rdc = rd[i];
			int q = (int)qu[i] - 33;
			q = q < 0 ? 0 : (q > 255 ? 255 : q);
			rowst[i * 64 + lane] = ((uint32_t)rdc << 16) | ((uint32_t)sc.mmpen[q] << 24);
		}
		uint64_t dg0 = 0, dg1 = 0, dg2 = 0;
		int lrmax = 0, ncand = 0;
		// ---------------- fill: column-major exact recurrence ----------------
		for(int j = 0; j < C; j++) {
			const int refc = rf[j];
			int hdiag = 0xff;           // H[-1][j-1] = 0xff: alignment may start anywhere
			int hup = 0, fup = 0, h = 0;
			uint32_t dword = 0;
			for(int i = 0; i < R; i++) {
				const uint32_t w = rowst[i * 64 + lane];
				const int hl = (int)(w & 0xff), el = (int)((w >> 8) & 0xff);
				const int rdc = (int)((w >> 16) & 0xff), mm = (int)(w >> 24);
				const bool gbar = (i < sc.gapbar) || (R - 1 - i < sc.gapbar);
				const int e = imax(sat(el - sc.rde), gbar ? 0 : sat(hl - sc.rdo));
				const int f = (i == 0 || gbar) ? 0 : imax(sat(fup - sc.rfe), sat(hup - sc.rfo));
				const int pen = (rdc > 3 || refc > 3) ? sc.npen : (rdc == refc ? 0 : mm);
				const int d = (i == 0) ? 0xff : hdiag;
				h = imax(sat(d - pen), imax(e, f));
				uint32_t tb = 0;
				if(i > 0) {
					const bool ga = !gbar;
					int hd = H_NONE;
					if(j > 0 && hdiag - pen == h) hd = H_DIAG;
					else if(ga && hup - sc.rfo == h) hd = H_REF_OPEN;
					else if(ga && fup - sc.rfe == h) hd = H_RFGAP_EXT;
					else if(ga && j > 0 && hl - sc.rdo == h) hd = H_READ_OPEN;
					else if(ga && j > 0 && el - sc.rde == h) hd = H_RDGAP_EXT;
					int ed = 0;
					if(j > 0) ed = (hl - sc.rdo == e) ? 1 : ((el - sc.rde == e) ? 2 : 0);
					const int fd = (hup - sc.rfo == f) ? 1 : ((fup - sc.rfe == f) ? 2 : 0);
					tb = (uint32_t)hd | ((uint32_t)ed << 3) | ((uint32_t)fd << 5);
				}
				dword |= tb << (8 * (i & 3));
				if((i & 3) == 3 || i == R - 1) {
					dir[((size_t)j * kRowWords + (i >> 2)) * 64 + lane] = dword;
					dword = 0;
				}
				if(kDebug && a.digests) {
					dg0 += cell_digest(i, j, 0, e);
					dg1 += cell_digest(i, j, 1, f);
					dg2 += cell_digest(i, j, 2, h);
				}
				rowst[i * 64 + lane] = (w & 0xffff0000u) | (uint32_t)h | ((uint32_t)e << 8);
				hdiag = hl;
				hup = h; fup = f;
			}
			lastrow[(size_t)j * 64 + lane] = (uint8_t)h;
			lrmax = imax(lrmax, h);
			ncand += (h >= thr);
		}
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
		uint8_t* lr8 = reinterpret_cast<uint8_t*>(rowst);
		for(int j = 0; j < C; j++) lr8[(j >> 2) * 256 + lane * 4 + (j & 3)] = lastrow[(size_t)j * 64 + lane];
		int cur_key = 0x7fffffff, ndone = 0, nrec = 0;
		const int row0 = R - 1;
		const int rdo = sc.rdo, rde = sc.rde, rfo = sc.rfo, rfe = sc.rfe;
		while(ndone < ncand) {
			int ntries = 0;
			bool found = false;
			BtResult res;
			res.nedit = 0;
			while(ndone < ncand) {
				// next candidate in DpBtCandidate order: largest key = score*256+col below cur_key
				int best = -1;
				for(int j = 0; j < C; j++) {
					const int s = lr8[(j >> 2) * 256 + lane * 4 + (j & 3)];
					const int key = s * 256 + j;
					if(s >= thr && key < cur_key && key > best) best = key;
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
				while(true) {
					st_bt++;
					const size_t wi = ((size_t)col * kRowWords + (row >> 2)) * 64 + lane;
					uint32_t w = dir[wi];
					const int sh = 8 * (row & 3);
					const uint32_t tb = (w >> sh) & 0xffu;
					if(tb & 0x80u) { ok = false; break; }          // reportedThrough
					int move = H_NONE;
					bool empty = false;
					if(row > 0) {
						if(ct == 2) move = (int)(tb & 7u);
						else if(ct == 0) { const int ed = (int)((tb >> 3) & 3u); move = ed == 1 ? H_READ_OPEN : ed == 2 ? H_RDGAP_EXT : H_NONE; }
						else { const int fd = (int)((tb >> 5) & 3u); move = fd == 1 ? H_REF_OPEN : fd == 2 ? H_RFGAP_EXT : H_NONE; }
						empty = (move == H_NONE);
					}
					dir[wi] = w | (0x80u << sh);                   // setReportedThrough
					const int diag = col - row + (int)p.triml;
					if(diag >= 0 && diag >= (int)p.corel && diag <= (int)p.corer) over_core = true;
					if(empty || row == 0) { trimBeg = row; break; }
					const int rdc = rd[row];
					if(move == H_DIAG) {
						const int refc = rf[col];
						const bool amb = rdc > 3 || refc > 3;
						if(amb || rdc != refc) {
							const int q0 = (int)qu[row] - 33;
							const int q = q0 < 0 ? 0 : (q0 > 255 ? 255 : q0);
							stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)row, EDIT_MM, mask_chr(refc), acgtn(rdc));
							ne++;
							bscore -= amb ? sc.npen : (int)sc.mmpen[q];
						}
						if(amb) ns++;
						row--; col--; ct = 2;
					} else if(move == H_REF_OPEN || move == H_RFGAP_EXT) {
						stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)row, EDIT_REF_GAP, '-', acgtn(rdc));
						ne++;
						bscore -= (move == H_REF_OPEN) ? rfo : rfe;
						ct = (move == H_REF_OPEN) ? 2 : 1;
						row--; gaps++;
					} else {
						stage_ed[(size_t)ne * 64 + lane] = pack_edit((uint32_t)row + 1, EDIT_READ_GAP, mask_chr(rf[col]), '-');
						ne++;
						bscore -= (move == H_READ_OPEN) ? rdo : rde;
						ct = (move == H_READ_OPEN) ? 2 : 0;
						col--; gaps++;
					}
				}
				if(!ok || !over_core) continue;
				{
					const int rdc = rd[row], refc = rf[col];
					const bool amb = rdc > 3 || refc > 3;
					if(amb || rdc != refc) {
						const int q0 = (int)qu[row] - 33;
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
