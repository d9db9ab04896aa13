/*
 * oracle/bt2x_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of sfiligoi/omp-bowtie2-prime's hot path, written from the
 * reference's algorithm (citations are /root/reference file:line):
 *
 *   index load      Ebwt::readIntoMemory            bt2_io.cpp:39-560
 *   occ / LF        SideLocus::initFromRow          bt2_idx.h:370-398
 *                   Ebwt::countBt2Side(Ex)          bt2_idx.h:1811-1846, 1940-1972
 *                   Ebwt::rowL / mapLF1             bt2_idx.h:2306, 2511-2564
 *                   Ebwt::ftabSeqToInt / ftabLoHi   bt2_idx.h:1384, 1447-1600
 *   seed search     startSearchSeedBi / searchSeedBi<8>  aligner_seed.cpp:757-957
 *   extension       MultiSeedAligner::extend        aligner_seed.cpp:603-672
 *   DP fill         EEU8_alignOne/lazyF/alignNucleotides aligner_swsse_ee_u8.cpp:249-536,
 *                   restated as the exact saturating-u8 recurrence (lane width does
 *                   not change any stored value).
 *   candidates      alignEnd2EndSseU8 + DpBtCandidate ordering  u8.cpp:542-671,
 *                   aligner_sw_nuc.h:149-157
 *   backtrace       backtraceNucleotidesEnd2EndSseU8  u8.cpp:746-1352
 *   call sequence   SwAligner::nextAlignment          aligner_sw.cpp:252-375
 *   scoring         Scoring::initPens/score/mm        scoring.h:94-132, 232-288
 *   SA resolution   Ebwt::getOffset                   bt2_idx.cpp:150-174 (the value
 *                   GroupWalk2S::advanceElement yields, group_walk.h:425-432, 969-1005)
 *                   Ebwt::joinedToTextOff             bt2_idx.cpp:54-121
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#include "bt2x_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define OFF_MASK 0xffffffffffffffffULL

/* ------------------------------------------------------------------ index */

typedef struct { uint64_t* blocks[8]; int n; } owner_t;

static int read_exact(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

int bt2o_index_load(const char* base, int load_offs, bt2x_index_desc* o) {
	char path[4096];
	memset(o, 0, sizeof(*o));
	snprintf(path, sizeof path, "%s.1.bt2l", base);
	FILE* f = fopen(path, "rb");
	if(!f) return BT2X_E_IO;
	uint32_t one; uint64_t len; int32_t lineRate, lps, offRate, ftabChars, flags;
	int rc = 0;
	rc |= read_exact(f, &one, 4); rc |= read_exact(f, &len, 8);
	rc |= read_exact(f, &lineRate, 4); rc |= read_exact(f, &lps, 4);
	rc |= read_exact(f, &offRate, 4); rc |= read_exact(f, &ftabChars, 4);
	rc |= read_exact(f, &flags, 4);
	if(rc || one != 1 || lineRate != 7) { fclose(f); return BT2X_E_IO; }
	owner_t* own = (owner_t*)calloc(1, sizeof(owner_t));
	uint64_t npat; read_exact(f, &npat, 8);
	uint64_t* plen = (uint64_t*)malloc(8 * (npat ? npat : 1));
	rc |= read_exact(f, plen, 8 * npat);
	uint64_t nfrag; rc |= read_exact(f, &nfrag, 8);
	uint64_t* rstarts = (uint64_t*)malloc(24 * (nfrag ? nfrag : 1));
	rc |= read_exact(f, rstarts, 24 * nfrag);
	/* EbwtParams::init, bt2_idx.h:134-165 */
	uint64_t sideSz = 1ULL << lineRate, sideBwtSz = sideSz - 32;
	uint64_t bwtSz = len / 4 + 1;
	uint64_t numSides = (bwtSz + sideBwtSz - 1) / sideBwtSz;
	uint64_t ebwtTot = numSides * sideSz;
	uint8_t* ebwt = (uint8_t*)malloc(ebwtTot);
	rc |= read_exact(f, ebwt, ebwtTot);
	uint64_t zoff; rc |= read_exact(f, &zoff, 8);
	rc |= read_exact(f, o->fchr, 40);
	uint64_t ftabLen = (1ULL << (2 * ftabChars)) + 1;
	uint64_t* ftab = (uint64_t*)malloc(8 * ftabLen);
	rc |= read_exact(f, ftab, 8 * ftabLen);
	uint64_t eftabLen = 2 * (uint64_t)ftabChars;
	uint64_t* eftab = (uint64_t*)malloc(8 * eftabLen);
	rc |= read_exact(f, eftab, 8 * eftabLen);
	fclose(f);
	own->blocks[own->n++] = plen; own->blocks[own->n++] = rstarts;
	own->blocks[own->n++] = (uint64_t*)ebwt; own->blocks[own->n++] = ftab;
	own->blocks[own->n++] = eftab;
	o->len = len; o->zoff = zoff; o->ftab_chars = ftabChars; o->off_rate = offRate;
	o->line_rate = lineRate; o->flags = flags;
	o->ebwt = ebwt; o->ebwt_bytes = ebwtTot; o->ftab = ftab; o->ftab_len = ftabLen;
	o->eftab = eftab; o->eftab_len = eftabLen; o->plen = plen; o->npat = npat;
	o->rstarts = rstarts; o->nfrag = nfrag; o->owner = own;
	if(rc) { bt2o_index_free(o); return BT2X_E_IO; }
	if(load_offs) {
		snprintf(path, sizeof path, "%s.2.bt2l", base);
		f = fopen(path, "rb");
		if(!f) { bt2o_index_free(o); return BT2X_E_IO; }
		uint64_t offsLen = (len + 1 + (1ULL << offRate) - 1) >> offRate;
		uint64_t* offs = (uint64_t*)malloc(8 * offsLen);
		rc |= read_exact(f, &one, 4);
		rc |= read_exact(f, offs, 8 * offsLen);
		fclose(f);
		own->blocks[own->n++] = offs;
		o->offs = offs; o->offs_len = offsLen;
		if(rc) { bt2o_index_free(o); return BT2X_E_IO; }
	}
	return BT2X_OK;
}

void bt2o_index_free(bt2x_index_desc* o) {
	owner_t* own = (owner_t*)o->owner;
	if(own) { for(int i = 0; i < own->n; i++) free(own->blocks[i]); free(own); }
	memset(o, 0, sizeof(*o));
}

/* ---------------------------------------------------------------- scoring */

void bt2o_scoring_default(bt2x_scoring* sc) {
	memset(sc, 0, sizeof(*sc));
	sc->mm_max = 6; sc->mm_min = 2; sc->n_pen = 1;        /* scoring.h:38-50 */
	sc->rdg_const = 5; sc->rdg_linear = 3;                /* scoring.h:70-79 */
	sc->rfg_const = 5; sc->rfg_linear = 3;
	sc->gapbar = 4;                                       /* bt2_search.cpp:374 */
	bt2o_scoring_init(sc);
}

void bt2o_scoring_init(bt2x_scoring* sc) {
	/* Scoring::initPens, COST_MODEL_QUAL for mismatches, constant for Ns (scoring.h:94-132) */
	for(int i = 0; i < 256; i++) {
		int ii = i < 40 ? i : 40;
		float frac = (float)ii / 40.0f;
		sc->mmpens[i] = sc->mm_min + (int)(frac * (float)(sc->mm_max - sc->mm_min));
		sc->npens[i] = sc->n_pen;
	}
}

/* ----------------------------------------------------------- occ counting */

typedef struct { uint64_t side_byte_off; int by, bp; } locus_t;

static inline void locus_from_row(uint64_t row, locus_t* l) {
	/* SideLocus::initFromRow: 384 chars per 128-byte side (bt2_idx.h:370-398) */
	uint64_t side = row / BT2X_SIDE_CHARS;
	uint32_t charOff = (uint32_t)(row % BT2X_SIDE_CHARS);
	l->side_byte_off = side * BT2X_SIDE_BYTES;
	l->by = (int)(charOff >> 2);
	l->bp = (int)(charOff & 3);
}

/* # of bit-pairs equal to c in bytes [0,by) plus the first bp pairs of byte by. */
static inline uint64_t count_upto(const uint8_t* side, int by, int bp, int c) {
	static const uint64_t ctab[4] = { 0xffffffffffffffffULL, 0xaaaaaaaaaaaaaaaaULL,
	                                  0x5555555555555555ULL, 0ULL };
	uint64_t cnt = 0;
	int i = 0;
	for(; i + 7 < by; i += 8) {       /* countInU64, bt2_idx.h:519-537 */
		uint64_t dw; memcpy(&dw, side + i, 8);
		uint64_t x0 = dw ^ ctab[c];
		uint64_t x3 = x0 & ((x0 >> 1) & 0x5555555555555555ULL);
		cnt += (uint64_t)__builtin_popcountll(x3);
	}
	for(; i < by; i++)
		for(int k = 0; k < 4; k++) cnt += (((side[i] >> (2 * k)) & 3) == c);
	for(int k = 0; k < bp; k++) cnt += (((side[by] >> (2 * k)) & 3) == c);
	return cnt;
}

static inline int dollar_before(const bt2x_index_desc* idx, const locus_t* l) {
	/* '$' is stored as an 'A' at zOff; discount it when it lies before the locus
	 * inside this side (bt2_idx.h:1819-1826, 1943-1952, postReadInit :1684-1694). */
	uint64_t zs = idx->zoff / BT2X_SIDE_CHARS, zc = idx->zoff % BT2X_SIDE_CHARS;
	uint64_t zbyte = zs * BT2X_SIDE_BYTES + (zc >> 2);
	int zbp = (int)(zc & 3);
	uint64_t here = l->side_byte_off + (uint64_t)l->by;
	if(l->side_byte_off <= zbyte && here >= zbyte)
		if(here > zbyte || (here == zbyte && l->bp > zbp)) return 1;
	return 0;
}

static inline uint64_t side_occ(const uint8_t* side, int c) {
	uint64_t v; memcpy(&v, side + 96 + 8 * c, 8); return v;
}

uint64_t bt2o_count_side(const bt2x_index_desc* idx, uint64_t row, int c) {
	locus_t l; locus_from_row(row, &l);
	const uint8_t* side = idx->ebwt + l.side_byte_off;
	uint64_t cnt = count_upto(side, l.by, l.bp, c);
	if(c == 0 && dollar_before(idx, &l)) cnt--;
	return side_occ(side, c) + cnt + idx->fchr[c];
}

void bt2o_count_side_ex(const bt2x_index_desc* idx, uint64_t row, uint64_t out[4]) {
	locus_t l; locus_from_row(row, &l);
	const uint8_t* side = idx->ebwt + l.side_byte_off;
	for(int c = 0; c < 4; c++) out[c] = count_upto(side, l.by, l.bp, c);
	if(dollar_before(idx, &l)) out[0]--;
	for(int c = 0; c < 4; c++) out[c] += side_occ(side, c) + idx->fchr[c];
}

int bt2o_row_l(const bt2x_index_desc* idx, uint64_t row) {
	locus_t l; locus_from_row(row, &l);
	return (idx->ebwt[l.side_byte_off + (uint64_t)l.by] >> (2 * l.bp)) & 3;
}

/* mapLF1(row, l, c) (bt2_idx.h:2511-2535) */
static inline uint64_t map_lf1_c(const bt2x_index_desc* idx, uint64_t row, int c) {
	if(bt2o_row_l(idx, row) != c || row == idx->zoff) return OFF_MASK;
	return bt2o_count_side(idx, row, c);
}

/* mapLF1(row&, l) (bt2_idx.h:2542-2564): returns L char or -1 at '$'. */
static inline int map_lf1(const bt2x_index_desc* idx, uint64_t* row) {
	if(*row == idx->zoff) return -1;
	int c = bt2o_row_l(idx, *row);
	*row = bt2o_count_side(idx, *row, c);
	return c;
}

static inline uint64_t ftab_hi(const bt2x_index_desc* idx, uint64_t i) {
	uint64_t v = idx->ftab[i];
	if(v <= idx->len) return v;
	return idx->eftab[(v ^ OFF_MASK) * 2 + 1];
}
static inline uint64_t ftab_lo(const bt2x_index_desc* idx, uint64_t i) {
	uint64_t v = idx->ftab[i];
	if(v <= idx->len) return v;
	return idx->eftab[(v ^ OFF_MASK) * 2];
}

/* ------------------------------------------------------------ seed search */

static void search_one(const bt2x_index_desc* idx, const uint8_t* seq, int nsteps,
                       bt2x_seed_out* o, bt2x_counters* ctr) {
	uint64_t top = 0, bot = 0;
	int step = 0, done = 0, report = 0;
	const int off = nsteps - 1;
	const int fc = idx->ftab_chars;
	/* startSearchSeedBi (aligner_seed.cpp:757-811) */
	if(fc > 1 && fc <= nsteps) {
		uint64_t fi = 0;
		for(int i = 0; i < fc; i++) fi = (fi << 2) | (uint64_t)(seq[off - fc + 1 + i] & 3);
		top = ftab_hi(idx, fi); bot = ftab_lo(idx, fi + 1);
		if(ctr) ctr->n_ftab++;
		if(bot - top == 0) done = 1;
		else step += fc;
	} else {
		int c = seq[off];
		top = idx->fchr[c]; bot = idx->fchr[c + 1];
		if(bot - top == 0) done = 1;
		else step++;
	}
	if(!done && step == nsteps) { done = 1; report = 1; }
	/* searchSeedBi<8> step loop (aligner_seed.cpp:870-954) */
	while(!done) {
		int soff = nsteps - step - 1;          /* SeedAlignerSearchWorkState(off) */
		step++;
		uint64_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
		int big = (bot - top) > 1;             /* bloc.valid() */
		if(big) {
			bt2o_count_side_ex(idx, top, t);
			bt2o_count_side_ex(idx, bot, b);
			if(ctr) ctr->n_bilf++;
		}
		int c = seq[soff];
		if(c == 4) { done = 1; break; }
		if(!big) {
			if(ctr) ctr->n_lf1++;
			t[c] = map_lf1_c(idx, top, c);
			if(t[c] == OFF_MASK) { done = 1; break; }
			b[c] = t[c] + 1;
		}
		if(b[c] == t[c]) { done = 1; break; }
		top = t[c]; bot = b[c];
		if(step == nsteps) { report = 1; done = 1; break; }
	}
	o->topf = top; o->botf = bot; o->need_reporting = (uint8_t)report; o->nlex = 0;
}

/* MultiSeedAligner::extend (aligner_seed.cpp:603-672).  left points at the read char
 * immediately left of the seed; lim chars are available. */
static int extend_one(const bt2x_index_desc* idx, uint64_t top, uint64_t bot,
                      const uint8_t* left, int lim, bt2x_counters* ctr) {
	int nlex = 0;
	for(int ii = 0; ii < lim; ii++) {
		int rdc = left[-ii];
		if(bot - top > 1) {
			if(ctr) ctr->n_bilf++;
			uint64_t t[4], b[4];
			bt2o_count_side_ex(idx, top, t);
			bt2o_count_side_ex(idx, bot, b);
			int nonz = -1, abort_ = 0;
			uint64_t origSz = bot - top;
			for(int j = 0; j < 4; j++) {
				if(b[j] > t[j]) {
					if(nonz >= 0) { abort_ = 1; break; }
					nonz = j; top = t[j]; bot = b[j];
				}
			}
			if(abort_ || (nonz != rdc && rdc <= 3) || bot - top < origSz) break;
		} else {
			if(ctr) ctr->n_lf1++;
			int c = map_lf1(idx, &top);
			if(c != rdc && rdc <= 3) break;
			bot = top + 1;
		}
		if(++nlex == 255) break;
	}
	return nlex;
}

int bt2o_seed_search(const bt2x_index_desc* idx, const uint8_t* reads,
                     const bt2x_seed_in* in, uint32_t n, int do_extend,
                     bt2x_seed_out* out, bt2x_counters* ctr) {
	if(ctr) memset(ctr, 0, sizeof(*ctr));
	for(uint32_t i = 0; i < n; i++) {
		const uint8_t* rd = reads + in[i].read_off;
		const uint8_t* seq = rd + in[i].seed_off;
		if(in[i].seed_len < 1 || in[i].seed_len > 32) return BT2X_E_ARG;
		search_one(idx, seq, in[i].seed_len, &out[i], ctr);
		if(do_extend && out[i].need_reporting && in[i].seed_off > 0)
			out[i].nlex = (uint8_t)extend_one(idx, out[i].topf, out[i].botf, seq - 1,
			                                  in[i].seed_off, ctr);
	}
	if(ctr) {
		ctr->n_problems = n;
		ctr->alg_bytes = 128 * (2 * ctr->n_bilf + ctr->n_lf1) + 16 * ctr->n_ftab;
	}
	return BT2X_OK;
}

/* --------------------------------------------------------------------- DP */

enum { MAT_E = 0, MAT_F = 1, MAT_H = 2 };  /* SSEMatrixConsts (aligner_swsse.h:104-113) */
enum { BT_DIAG = 1, BT_REF_OPEN, BT_RFGAP_EXT, BT_READ_OPEN, BT_RDGAP_EXT };
enum { EDIT_READ_GAP = 1, EDIT_REF_GAP = 2, EDIT_MM = 3 };   /* edit.h:36-39 */

static const char MASK2DNA[17] = { '?','A','C','M','G','R','S','V','T','W','Y','H','K','D','B','N','N' };

static inline int sat(int v) { return v < 0 ? 0 : v; }

/* Scoring::score(rdc, refm, q) (scoring.h:241-251); match bonus 0 in end-to-end. */
static inline int sc_score(const bt2x_scoring* sc, int rdc, int refm, int q) {
	if(rdc > 3 || refm > 15) return -sc->npens[q];
	if(refm & (1 << rdc)) return 0;
	return -sc->mmpens[q];
}
/* Scoring::mm(rdc, refm, q) (scoring.h:232-235), used by QUAL2 (aligner_sw.h:86) */
static inline int sc_mm(const bt2x_scoring* sc, int rdc, int refm, int q) {
	return (rdc > 3 || refm > 15) ? sc->npens[q] : sc->mmpens[q];
}
static inline int matches_ex(int i, int j) {           /* mask.h:37-43 */
	if(j >= 16 || i > 3) return -1;
	return ((1 << i) & j) != 0 ? 1 : 0;
}

/* Cell values: u8 problems in [0, 0xff] (0xff = score 0, aligner_swsse_ee_u8.cpp:58-61);
 * i16 problems (BT2X_DP_I16, aligner_swsse_ee_i16.cpp:58-63) hold the int16 value + 0x8000,
 * i.e. [0, 0xffff] with 0xffff = score 0: saturating adds of non-positive scores in the
 * signed domain are saturating subtractions of penalties here, floor 0 = 0x8000. */
typedef struct {
	int R, C;
	uint16_t E[BT2X_MAX_ROWS][BT2X_MAX_COLS];
	uint16_t F[BT2X_MAX_ROWS][BT2X_MAX_COLS];
	uint16_t H[BT2X_MAX_ROWS][BT2X_MAX_COLS];
	uint8_t rt[BT2X_MAX_ROWS][BT2X_MAX_COLS];   /* reportedThrough bit */
} dpmat_t;

typedef struct { int row, col, score; } cand_t;

static int cand_cmp(const void* a, const void* b) {
	/* DpBtCandidate::operator< : score desc, row desc, col desc */
	const cand_t* x = (const cand_t*)a; const cand_t* y = (const cand_t*)b;
	if(x->score != y->score) return x->score > y->score ? -1 : 1;
	if(x->row != y->row) return x->row > y->row ? -1 : 1;
	if(x->col != y->col) return x->col > y->col ? -1 : 1;
	return 0;
}

typedef struct {
	int ok;
	int score, ns, gaps, nedit, bases_aligned, refns, off;
	int nraw;                       /* edit-buffer entries written by the last attempt */
	uint32_t edits[BT2X_MAX_ROWS + BT2X_MAX_COLS + 8];
} btres_t;

static inline uint32_t pack_edit(uint32_t pos, int type, int chr, int qchr) {
	return (pos & 0x3ffu) | ((uint32_t)type << 12) | ((uint32_t)(uint8_t)chr << 16) |
	       ((uint32_t)(uint8_t)qchr << 24);
}

/* backtraceNucleotidesEnd2EndSseU8 (aligner_swsse_ee_u8.cpp:746-1352).  Only the
 * '#if 1' (deterministic) branches exist.  Every visited cell is marked
 * reportedThrough; meeting a marked cell fails the backtrace (branch frames point at
 * cells that are themselves marked, so unwinding the stack can never resume). */
static int backtrace(const bt2x_scoring* sc, dpmat_t* m, const uint8_t* rd, const uint8_t* qu,
                     const uint8_t* rf, const bt2x_dp_in* p, int row, int col, btres_t* res,
                     uint64_t* btcells, uint32_t* raw) {
	const int R = m->R;
	const int rdo = sc->rdg_const + sc->rdg_linear, rde = sc->rdg_linear;
	const int rfo = sc->rfg_const + sc->rfg_linear, rfe = sc->rfg_linear;
	int ct = MAT_H, score = 0, ns = 0, gaps = 0;
	int nedit = 0, trimBeg = 0;
	const int trimEnd = R - row - 1, origCol = col;
	/* raw: the caller's persistent edit buffer (SwResult::alres.ned_ storage), written
	 * in backtrace order from index 0; res->nraw = entries written by this attempt */
	int over_core = 0;
	res->nraw = 0;
	while(row >= 0) {
		(*btcells)++;
		const int rdc = rd[row], refm = 1 << rf[col], q = qu[row] - 33;
		int empty = 0, canMoveThru = 1, cur = 0;
		if(m->rt[row][col]) {
			canMoveThru = 0;
		} else if(row > 0) {
			const int gapsAllowed = !(row < sc->gapbar || R - row - 1 < sc->gapbar);
			if(ct == MAT_E) {
				int cur_sc = m->E[row][col], mask = 0;
				if(col > 0 && (int)m->H[row][col - 1] - rdo == cur_sc) mask |= 1;
				if(col > 0 && (int)m->E[row][col - 1] - rde == cur_sc) mask |= 2;
				if(mask == 3 || mask == 1) cur = BT_READ_OPEN;
				else if(mask == 2) cur = BT_RDGAP_EXT;
				else { empty = 1; canMoveThru = 1; }
			} else if(ct == MAT_F) {
				int cur_sc = m->F[row][col], mask = 0;
				if((int)m->H[row - 1][col] - rfo == cur_sc) mask |= 1;
				if((int)m->F[row - 1][col] - rfe == cur_sc) mask |= 2;
				if(mask == 3 || mask == 1) cur = BT_REF_OPEN;
				else if(mask == 2) cur = BT_RFGAP_EXT;
				else { empty = 1; canMoveThru = 1; }
			} else {
				int cur_sc = m->H[row][col], mask = 0;
				if(gapsAllowed) {
					if((int)m->H[row - 1][col] - rfo == cur_sc) mask |= 1;
					if(col > 0 && (int)m->H[row][col - 1] - rdo == cur_sc) mask |= 2;
					if((int)m->F[row - 1][col] - rfe == cur_sc) mask |= 4;
					if(col > 0 && (int)m->E[row][col - 1] - rde == cur_sc) mask |= 8;
				}
				if(col > 0 && (int)m->H[row - 1][col - 1] + sc_score(sc, rdc, refm, q) == cur_sc)
					mask |= 16;
				/* single option or fixed priority diag > H-up > F-up > H-left > E-left
				 * (u8.cpp:968-990) */
				if(mask & 16) cur = BT_DIAG;
				else if(mask & 1) cur = BT_REF_OPEN;
				else if(mask & 4) cur = BT_RFGAP_EXT;
				else if(mask & 2) cur = BT_READ_OPEN;
				else if(mask & 8) cur = BT_RDGAP_EXT;
				else { empty = 1; canMoveThru = 1; }
			}
		}
		m->rt[row][col] = 1;
		if(!canMoveThru) { res->nraw = nedit; return 0; }
		{
			long long diag = (long long)col - row + p->triml;   /* core diagonal check */
			if(diag >= 0 && (uint64_t)diag >= p->corel && (uint64_t)diag <= p->corer) over_core = 1;
		}
		if(empty || row == 0) { trimBeg = row; break; }
		switch(cur) {
		case BT_DIAG: {
			int mt = matches_ex(rdc, refm);
			ct = MAT_H;
			if(mt != 1) {
				raw[nedit++] = pack_edit((uint32_t)row, EDIT_MM, MASK2DNA[refm], "ACGTN"[rdc]);
				score -= sc_mm(sc, rdc, refm, q);
			}
			if(mt == -1) ns++;
			row--; col--;
			break;
		}
		case BT_REF_OPEN: case BT_RFGAP_EXT:
			raw[nedit++] = pack_edit((uint32_t)row, EDIT_REF_GAP, '-', "ACGTN"[rdc]);
			score -= (cur == BT_REF_OPEN) ? rfo : rfe;
			ct = (cur == BT_REF_OPEN) ? MAT_H : MAT_F;
			row--; gaps++;
			break;
		case BT_READ_OPEN: case BT_RDGAP_EXT:
			raw[nedit++] = pack_edit((uint32_t)row + 1, EDIT_READ_GAP, MASK2DNA[refm], '-');
			score -= (cur == BT_READ_OPEN) ? rdo : rde;
			ct = (cur == BT_READ_OPEN) ? MAT_H : MAT_E;
			col--; gaps++;
			break;
		default:
			res->nraw = nedit;
			return 0;
		}
	}
	if(!over_core) { res->nraw = nedit; return 0; }
	{
		const int rdc = rd[row], refm = 1 << rf[col], q = qu[row] - 33;
		int mt = matches_ex(rdc, refm);
		if(mt != 1) {
			raw[nedit++] = pack_edit((uint32_t)row, EDIT_MM, MASK2DNA[refm], "ACGTN"[rdc]);
			score -= sc_mm(sc, rdc, refm, q);
		}
		if(mt == -1) ns++;
	}
	if(ns > p->nceil) { res->nraw = nedit; return 0; }
	/* res.reverse(); setShape (pos -= trimBeg); for rc invertEdits (aligner_result.h:852,
	 * edit.cpp:50-78): reverse again and pos = extent - pos - (readgap ? 0 : 1). */
	const int extent = R - trimBeg - trimEnd;
	for(int k = 0; k < nedit; k++) {
		uint32_t e = p->fw ? raw[nedit - 1 - k] : raw[k];
		uint32_t pos = BT2X_EDIT_POS(e) - (uint32_t)trimBeg;
		if(!p->fw) pos = (uint32_t)extent - pos - (BT2X_EDIT_TYPE(e) == EDIT_READ_GAP ? 0u : 1u);
		res->edits[k] = (e & ~0x3ffu) | (pos & 0x3ffu);
	}
	int refns = 0;
	for(int i = col; i <= origCol; i++) refns += (rf[i] > 3);
	/* the reference reverses / inverts ned_ in place: the buffer now holds the final list */
	for(int k = 0; k < nedit; k++) raw[k] = res->edits[k];
	res->nraw = nedit;
	res->ok = 1; res->score = score; res->ns = ns; res->gaps = gaps; res->nedit = nedit;
	res->bases_aligned = extent - nedit; res->refns = refns; res->off = col;
	return 1;
}

int bt2o_dp_align(const bt2x_scoring* sc,
                  const uint8_t* reads, const uint8_t* quals, const uint8_t* refs,
                  const bt2x_dp_in* in, uint32_t n, bt2x_dp_out* out,
                  bt2x_aln_rec* recs, uint32_t rec_cap, uint32_t* nrec_used,
                  uint32_t* edits, uint32_t edit_cap, uint32_t* nedit_used,
                  bt2x_dp_debug* debug, bt2x_counters* ctr) {
	dpmat_t* m = (dpmat_t*)malloc(sizeof(dpmat_t));
	btres_t* res = (btres_t*)malloc(sizeof(btres_t));
	cand_t cands[BT2X_MAX_COLS];
	uint32_t nrec = 0, nedit = 0;
	int overflow = 0;
	const int rdo = sc->rdg_const + sc->rdg_linear, rde = sc->rdg_linear;
	const int rfo = sc->rfg_const + sc->rfg_linear, rfe = sc->rfg_linear;
	if(ctr) memset(ctr, 0, sizeof(*ctr));
	for(uint32_t pi = 0; pi < n; pi++) {
		const bt2x_dp_in* p = &in[pi];
		const int R = p->rdlen, C = p->ncol;
		if(R < 1 || R > BT2X_MAX_ROWS || C < 1 || C + 1 > BT2X_MAX_COLS) { free(m); free(res); return BT2X_E_ARG; }
		const int i16 = (p->flags & BT2X_DP_I16) != 0;
		if(p->minsc > 0 || p->minsc < (i16 ? -32767 : -254)) { free(m); free(res); return BT2X_E_ARG; }
		const uint8_t* rd = reads + p->read_off;
		const uint8_t* qu = quals + p->qual_off;
		const uint8_t* rf = refs + p->ref_off;
		/* top: H of row -1 = score 0 (u8: 0xff; i16: 0x7fff + 0x8000) */
		const int top = i16 ? 0xffff : 0xff;
		m->R = R; m->C = C;
		/* Fill: the exact saturating recurrence the striped kernels compute (u8.cpp:249-536,
		 * i16.cpp:253-541): H[-1][*] = top, H[*][-1] = floor, E[*][0] = floor, F[0][*] = floor;
		 * the gap barrier subtracts top (u8: 0xff once; i16: 0x8000 added twice). */
		int lrmax = 0, ncand = 0;
		for(int j = 0; j < C; j++) {
			int refm = 1 << rf[j];
			for(int i = 0; i < R; i++) {
				int gbar = (i < sc->gapbar || R - i - 1 < sc->gapbar) ? top : 0;
				int e = 0, f = 0;
				if(j > 0) {
					int e1 = sat(m->E[i][j - 1] - rde);
					int e2 = sat(sat(m->H[i][j - 1] - rdo) - gbar);
					e = e1 > e2 ? e1 : e2;
				}
				if(i > 0) {
					int f1 = sat(m->F[i - 1][j] - rfe);
					int f2 = sat(m->H[i - 1][j] - rfo);
					f = sat((f1 > f2 ? f1 : f2) - gbar);
				}
				int diag = (i == 0) ? top : (j == 0 ? 0 : m->H[i - 1][j - 1]);
				int pen = -sc_score(sc, rd[i], refm, qu[i] - 33);
				int h = sat(diag - pen);
				if(e > h) h = e;
				if(f > h) h = f;
				m->E[i][j] = (uint16_t)e; m->F[i][j] = (uint16_t)f; m->H[i][j] = (uint16_t)h;
				m->rt[i][j] = 0;
			}
			int lr = m->H[R - 1][j];
			if(lr > lrmax) lrmax = lr;
			/* candidate: lr - 0xff / lr_i16 - 0x7fff >= minsc; DpBtCandidate::score = the raw
			 * cell value (u8.cpp:518-521, i16.cpp:526-529) */
			if(lr - top >= p->minsc) {
				cands[ncand].row = R - 1; cands[ncand].col = j; cands[ncand].score = i16 ? lr - 0x8000 : lr; ncand++;
			}
		}
		if(ctr) { ctr->dp_cells += (uint64_t)R * C; ctr->dp_cols += C; }
		if(debug && debug->digests) {
			uint64_t d[3] = {0, 0, 0};
			for(int i = 0; i < R; i++) for(int j = 0; j < C; j++) {
				/* the stored value: the u8 byte, or the int16 bit pattern */
				const uint32_t x = i16 ? 0x8000u : 0u;
				d[0] += bt2x_cell_digest(i, j, MAT_E, m->E[i][j] ^ x);
				d[1] += bt2x_cell_digest(i, j, MAT_F, m->F[i][j] ^ x);
				d[2] += bt2x_cell_digest(i, j, MAT_H, m->H[i][j] ^ x);
			}
			memcpy(debug->digests + 3 * (size_t)pi, d, sizeof d);
		}
		bt2x_dp_out* o = &out[pi];
		o->nrec = 0; o->rec_off = nrec; o->ncand = 0;
		/* alignEnd2EndSseU8 / alignEnd2EndSseI16: score = lrmax - 0xff of the stored value
		 * (u8.cpp:637-668; i16.cpp:642-673, where 0xff is subtracted from the int16) */
		int score = (i16 ? lrmax - 0x8000 : lrmax) - 0xff;
		if(score < p->minsc) { o->status = 0; o->best = score; ncand = 0; }
		else if(lrmax == 0) { o->status = 0; o->best = INT32_MIN; ncand = 0; }
		else {
			qsort(cands, (size_t)ncand, sizeof(cand_t), cand_cmp);
			o->status = ncand > 0; o->best = score;
		}
		o->ncand = (uint16_t)ncand;
		if(debug && debug->cands) {
			uint32_t* dc = debug->cands + (size_t)pi * BT2X_MAX_COLS;
			for(int k = 0; k < BT2X_MAX_COLS; k++)
				dc[k] = k >= ncand ? 0xffffffffu
				      : i16 ? BT2X_CAND_PACK16(cands[k].col, cands[k].score)
				            : BT2X_CAND_PACK(cands[k].row, cands[k].col, cands[k].score);
		}
		if(!o->status) continue;
		/* nextAlignment() until done() (aligner_sw.cpp:252-375) */
		int cural = 0;
		/* SwResult::alres.ned_ storage: every backtrace attempt writes its edits from index
		 * 0 (failed attempts leave them behind), successes leave the final list in place.
		 * Each record publishes the entries written during its call (BT2X_REC_NBUF). */
		uint32_t edbuf[BT2X_MAX_ROWS + BT2X_MAX_COLS + 8];
		while(cural < ncand) {
			int ntries = 0, found = 0, hi = 0;
			while(cural < ncand) {
				const cand_t* cd = &cands[cural];
				if(cd->score < p->minsc) { cural++; continue; }
				if(m->rt[cd->row][cd->col]) { cural++; continue; }
				ntries++;
				uint64_t btc = 0;
				int ok = backtrace(sc, m, rd, qu, rf, p, cd->row, cd->col, res, &btc, edbuf);
				if(res->nraw > hi) hi = res->nraw;
				if(ctr) ctr->bt_cells += btc;
				if(ok) { found = 1; break; }
				cural++;
			}
			if(nrec < rec_cap) {
				bt2x_aln_rec* r = &recs[nrec];
				memset(r, 0, sizeof(*r));
				r->ntries = (uint16_t)ntries;
				r->ok = (uint8_t)found;
				if(found) {
					r->score = (int16_t)res->score; r->ns = (uint16_t)res->ns;
					r->gaps = (uint16_t)res->gaps; r->nedit = (uint16_t)res->nedit;
					r->bases_aligned = (uint16_t)res->bases_aligned; r->refns = (uint16_t)res->refns;
					r->refoff = (int64_t)res->off + p->refl;
				}
				r->nbuf = (uint32_t)hi;
				r->edit_off = hi > 0 ? nedit : 0;
				if(nedit + (uint32_t)hi <= edit_cap)
					memcpy(edits + nedit, edbuf, sizeof(uint32_t) * (size_t)hi);
				else overflow = 1;
			} else overflow = 1;
			nedit += (uint32_t)hi;
			nrec++; o->nrec++;
			if(!found) break;
			cural++;
		}
	}
	if(ctr) {
		ctr->n_problems = n;
		/* SURVEY §8(d) B_dp: 3 B/cell materialised + C ref bytes + profile */
		ctr->alg_bytes = 3 * ctr->dp_cells + ctr->dp_cols;
	}
	free(m); free(res);
	if(nrec_used) *nrec_used = nrec;
	if(nedit_used) *nedit_used = nedit;
	return overflow ? BT2X_E_OVERFLOW : BT2X_OK;
}

/* ---------------------------------------------------------- SA resolution */

/* Ebwt::getOffset(row) (bt2_idx.cpp:150-174): LF-walk left until row zOff (offset =
 * jumps) or a sampled row (offs[row >> offRate] + jumps). */
static uint64_t get_offset(const bt2x_index_desc* idx, uint64_t row, uint64_t* steps) {
	const uint64_t mask = ((uint64_t)1 << idx->off_rate) - 1;
	uint64_t jumps = 0;
	for(;;) {
		if(row == idx->zoff) return jumps;
		if((row & mask) == 0) return jumps + idx->offs[row >> idx->off_rate];
		map_lf1(idx, &row);
		jumps++;
		if(steps) (*steps)++;
	}
}

/* Ebwt::joinedToTextOff (bt2_idx.cpp:54-121) for the forward index (fw_ = true), with
 * the outputs a zero-initialised caller sees (aligner_sw_driver.cpp:392-402).  The
 * reference's search never ends for an offset in no fragment; here that gives
 * BT2X_NO_TIDX (only the '$' suffix row reaches it). */
static void joined_to_text_off(const bt2x_index_desc* idx, uint64_t qlen, uint64_t off, int reject,
                               bt2x_resolve_out* o) {
	uint64_t top = 0, bot = idx->nfrag;
	o->tidx = BT2X_NO_TIDX; o->toff = 0; o->tlen = 0; o->straddled = 0;
	if(off >= idx->len || idx->nfrag == 0) return;
	for(;;) {
		const uint64_t elt = top + ((bot - top) >> 1);
		const uint64_t lower = idx->rstarts[elt * 3];
		const uint64_t upper = elt == idx->nfrag - 1 ? idx->len : idx->rstarts[(elt + 1) * 3];
		if(lower <= off) {
			if(upper > off) {
				if(off + qlen > upper) {
					o->straddled = 1;
					if(reject) return;
				}
				o->tidx = (uint32_t)idx->rstarts[elt * 3 + 1];
				o->toff = off - lower + idx->rstarts[elt * 3 + 2];
				o->tlen = idx->plen[o->tidx];
				return;
			}
			top = elt;
		} else {
			bot = elt;
		}
	}
}

int bt2o_resolve(const bt2x_index_desc* idx, const bt2x_resolve_in* in, uint32_t n, int reject_straddle,
                 bt2x_resolve_out* out, bt2x_counters* ctr) {
	uint64_t steps = 0;
	if(!idx->offs) return BT2X_E_ARG;
	for(uint32_t i = 0; i < n; i++) {
		if(in[i].row > idx->len) return BT2X_E_ARG;
		const uint64_t off = get_offset(idx, in[i].row, &steps);
		joined_to_text_off(idx, in[i].qlen, off, reject_straddle, &out[i]);
		out[i].joff = off;
	}
	if(ctr) {
		memset(ctr, 0, sizeof(*ctr));
		ctr->n_lf1 = steps;
		ctr->n_problems = n;
	}
	return BT2X_OK;
}

/* ------------------------------------------------------------------- RNG */
void bt2o_rng_init(bt2o_rng* r, uint32_t seed) { r->last = seed; r->last_off = 30; }
uint32_t bt2o_rng_next_u32(bt2o_rng* r) {          /* random_source.h:52-61 */
	uint32_t ret;
	r->last = 1664525u * r->last + 1013904223u;
	ret = r->last >> 16;
	r->last = 1664525u * r->last + 1013904223u;
	ret ^= r->last;
	r->last_off = 0;
	return ret;
}
