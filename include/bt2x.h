/*
 * bt2x.h — C-ABI of the MI355X-native Bowtie 2 hot path (seed search + DP).
 *
 * This is the drop-in boundary for sfiligoi/omp-bowtie2-prime's two data-parallel
 * hot loops.  Plain pointers and sizes only; no C++ or torch
 * types cross it.  Every entry point cites the reference interface it replaces.
 *
 *   bt2x_index_load / bt2x_index_free   Ebwt::readIntoMemory (bt2_io.cpp:39-560): parse a
 *                                       forward .1/.2.bt2l pair into host arrays.
 *   bt2x_open / bt2x_close              one context per GPU; uploads the index arrays
 *                                       (Ebwt::_ebwt/_ftab/_eftab/_fchr, bt2_idx.h:2617-2639).
 *   bt2x_open_shared                    a further context (own stream) over the same index.
 *   bt2x_seed_search                    MultiSeedAligner::searchAllSeedsDoAll(doExtend)
 *                                       (aligner_seed.cpp:674-725): exact backward search of
 *                                       every seed (searchSeedBi<8>, :820-957) and the
 *                                       left extension (MultiSeedAligner::extend, :603-672).
 *   bt2x_dp_align                       SwAligner::align (aligner_sw.cpp:235 ->
 *                                       alignEnd2EndSseU8, aligner_swsse_ee_u8.cpp:542) followed
 *                                       by every SwAligner::nextAlignment call until done()
 *                                       (aligner_sw.cpp:252-375, backtrace u8.cpp:746-1352).
 *
 * Conventions: return 0 on success, negative BT2X_E_* on error, never
 * throw.  Host buffers are caller-owned, device buffers are context-owned.  Calls on one
 * context are serialised.  The *_dev variants take device pointers (inputs already resident
 * in HBM) and a hipStream_t passed as void*; they are asynchronous on that stream.
 * The product path has no CPU fallback: without a usable GPU bt2x_open fails with
 * BT2X_E_NODEVICE.
 */
#ifndef BT2X_H_
#define BT2X_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: bt2x_elt 8 B, bt2x_sat 4 B, bt2x_last_round_stats 4 words, bt2x_seed_round_dev's
 * d_used 4 words.  4: bt2x_sam_tails[_dev] and bt2x_sam_req.  bt2x_abi_version() returns
 * the library's value: a binding compares it with the header it was written against
 * before any other call. */
#define BT2X_ABI_VERSION 4

enum {
	BT2X_OK = 0,
	BT2X_E_ARG = -1,        /* bad argument / shape outside the reference's limits */
	BT2X_E_IO = -2,         /* index file missing or malformed */
	BT2X_E_NODEVICE = -3,   /* no HIP device / HIP call failed */
	BT2X_E_OVERFLOW = -4,   /* result arena too small; required sizes reported */
	BT2X_E_NOMEM = -5
};

/* Reference limits that are part of the observable behaviour. */
#define BT2X_MAX_ROWS 160      /* ALN_MAX_ROWS, aligner_result.h:42 */
#define BT2X_MAX_COLS 200      /* ALN_MAX_COLS, aligner_result.h:43 (rflen+1 <= 200) */
#define BT2X_SIDE_BYTES 128    /* .bt2l side: 96 B of BWT + 4 x u64 occ (bt2_idx.h:134-165) */
#define BT2X_SIDE_CHARS 384    /* 48 * OFF_SIZE (bt2_idx.h:377) */

/* ------------------------------------------------------------------ index */

/* In-memory forward index, the arrays Ebwt holds after loadIntoMemory(). */
typedef struct {
	uint64_t len;            /* _eh._len: length of the joined text              */
	uint64_t zoff;           /* _zOff: BWT row whose L char is '$'                */
	uint64_t fchr[5];        /* _fchr                                             */
	int32_t  ftab_chars;     /* _eh._ftabChars (10)                               */
	int32_t  off_rate;       /* _eh._offRate (4)                                  */
	int32_t  line_rate;      /* _eh._lineRate (7 => 128-byte sides)               */
	int32_t  flags;
	const uint8_t*  ebwt;    uint64_t ebwt_bytes;  /* _ebwt, numSides * 128       */
	const uint64_t* ftab;    uint64_t ftab_len;    /* _ftab, 4^ftabChars + 1      */
	const uint64_t* eftab;   uint64_t eftab_len;   /* _eftab, 2 * ftabChars       */
	const uint64_t* offs;    uint64_t offs_len;    /* _offs (SA sample, .2.bt2l)  */
	const uint64_t* plen;    uint64_t npat;        /* _plen: reference lengths    */
	const uint64_t* rstarts; uint64_t nfrag;       /* _rstarts: 3 words/fragment  */
	const uint8_t*  text2;   uint64_t text2_bytes; /* joined text, 2 bits/base LSB-first
	                                                  (.4.bt2l, BitPairReference)      */
	void* owner;             /* loader-owned storage (bt2x_index_free) */
} bt2x_index_desc;

/* Parse <base>.1.bt2l like Ebwt::readIntoMemory; with load_offs also <base>.2.bt2l (SA
 * sample) and <base>.4.bt2l (packed joined text).  Given both, bt2x_open rebuilds the
 * full suffix array in HBM (an MI355X-first choice: 4 B/row resident, so SA lookups
 * and unique-range seed extension need no LF walks).  The arrays are read-only views of
 * the files mapped into memory (no copies): processes of one node that load the same
 * index share one host copy through the page cache, and the desc stays valid until
 * bt2x_index_free. */
int  bt2x_index_load(const char* basename, int load_offs, bt2x_index_desc* out);
void bt2x_index_free(bt2x_index_desc* idx);

/* Build <outbase>.{1,2,3,4}.bt2l from a FASTA file, byte-identical to the reference's
 * bowtie2-build-l (bt2_build.cpp / Ebwt::buildToDisk, bt2_idx.h:2922) for lineRate 7.
 * Host-only (SA-IS suffix sorting); used to index synthetic genomes on the GPU box. */
int  bt2x_build_index(const char* fasta, const char* outbase, int off_rate, int ftab_chars);

/* Same, with the suffix array of the joined text supplied by the caller (n = joined
 * length + 1, '$' row last: sa[n-1] == n-1), e.g. sorted on the GPU for genome-scale
 * synthetic indexes.  Optional per-row gathers computed alongside it (NULL = derive
 * from the text): bwt[i] = text[sa[i]-1] (any value where sa[i] == 0) and keys[i] =
 * the ftab_chars-mer at sa[i], 2 bits/char MSB-first (any value for suffixes shorter
 * than ftab_chars).  Cheap consistency checks only; BT2X_E_ARG if they fail. */
int  bt2x_build_index_sa(const char* fasta, const char* outbase, int off_rate, int ftab_chars,
                         const uint64_t* sa, uint64_t n, const uint8_t* bwt, const uint32_t* keys);

/* ---------------------------------------------------------------- scoring */

/* Scoring scheme (scoring.h:28-132).  Defaults: bt2x_scoring_default(). */
typedef struct {
	int32_t mm_max, mm_min;          /* --mp MX,MN  (6,2), COST_MODEL_QUAL          */
	int32_t n_pen;                   /* --np (1), COST_MODEL_CONSTANT               */
	int32_t rdg_const, rdg_linear;   /* --rdg (5,3): open = const+linear, ext = lin  */
	int32_t rfg_const, rfg_linear;   /* --rfg (5,3)                                  */
	int32_t gapbar;                  /* --gbar (4)                                   */
	int32_t mmpens[256];             /* filled by bt2x_scoring_init (initPens)       */
	int32_t npens[256];
} bt2x_scoring;

void bt2x_scoring_default(bt2x_scoring* sc);
/* Recompute the per-quality tables from the scalar fields (Scoring::initPens). */
void bt2x_scoring_init(bt2x_scoring* sc);

/* ---------------------------------------------------------------- context */

typedef struct bt2x_ctx bt2x_ctx;

/* sc = NULL: defaults.  Penalties above 15 (--mp MX > 15 or --np > 15) are rejected
 * with BT2X_E_ARG: the u8 DP kernel packs a row's penalty into 4 bits. */
int  bt2x_open(int hip_device, const bt2x_index_desc* idx, const bt2x_scoring* sc, bt2x_ctx** out);
/* A second context on base's GPU that shares base's device index and scoring (nothing is
 * uploaded) but has its own stream and buffers, so calls on the two contexts run
 * concurrently on the device (the reference's worker threads each own their aligner
 * objects over one shared Ebwt, bt2_search.cpp:2297-2888).  base must outlive it. */
int  bt2x_open_shared(const bt2x_ctx* base, bt2x_ctx** out);
void bt2x_close(bt2x_ctx* ctx);
/* NUMA node of the host socket the GPU hangs off (sysfs numa_node of its PCI device), or
 * -1 if unknown: a host driver keeps its threads and memory there (bt2x-align does). */
int  bt2x_device_numa_node(int hip_device);
/* Last kernel's duration in ms (HIP events on the launching stream), by kernel id. */
enum { BT2X_K_SEED = 0, BT2X_K_DP = 1, BT2X_K_RESOLVE = 2, BT2X_K_ROUND = 3, BT2X_K_COUNT = 4 };
double bt2x_last_kernel_ms(const bt2x_ctx* ctx, int kernel);
/* Algorithmic bytes / counters of the last call, by kernel id. */
typedef struct {
	uint64_t n_bilf;      /* mapBiLFEx calls (2 sides each)   */
	uint64_t n_lf1;       /* mapLF1 calls (1 side)            */
	uint64_t n_ftab;      /* ftab lookups (16 B)              */
	uint64_t dp_cells;    /* R*C summed over DP problems      */
	uint64_t dp_cols;     /* C summed                         */
	uint64_t bt_cells;    /* backtrace cells visited          */
	uint64_t n_problems;
	uint64_t alg_bytes;   /* algorithmic HBM bytes of the launch: for the DP, the
	                         traceback bytes the kernel writes (dp_cells_computed) plus
	                         the reference windows; SURVEY §8(d)'s reference-equivalent
	                         figure is 3*dp_cells + dp_cols + profile bytes */
	uint64_t dp_cells_computed; /* DP cells the fill computed (the diagonal band, or the
	                         whole rectangle when unbanded), <= dp_cells */
} bt2x_counters;
int bt2x_last_counters(const bt2x_ctx* ctx, int kernel, bt2x_counters* out);
/* The last seed round's sampling work (bt2x_seed_round[_dev]): out[0] reads, out[1] reads
 * that sampled (RowSampler jobs), out[2] elements drawn, out[3] most elements one read drew.
 * Writes exactly these 4 words (the abi-1 contract). */
int bt2x_last_round_stats(const bt2x_ctx* ctx, uint32_t out[4]);
/* The same words followed by how the sampling kernel drew them: out[4] 64-draw batches,
 * out[5] draws committed by a batch, out[6] draws taken one at a time, out[7] of out[5] from
 * swap lists; out[8..11] the kernel's clock in units of 1024 cycles summed over jobs
 * (BT2X_ROUND_CLOCK builds; else 0): setup, batch draws, serial draws, the rest.  Writes
 * min(n, BT2X_ROUND_STATS_N) words; returns that count (or a negative BT2X_E_*). */
#define BT2X_ROUND_STATS_N 12
int bt2x_last_round_stats_ex(const bt2x_ctx* ctx, uint32_t* out, uint32_t n);

/* ------------------------------------------------------------ seed search */

/* One exact seed (SeedAlignerSearchParams, aligner_seed.cpp:81-171).  The oriented read
 * (patFw for fw seeds, patRc for rc seeds; codes 0-3, 4 = N) starts at reads[read_off].
 * The seed is read[seed_off .. seed_off+seed_len); extension walks left over
 * read[seed_off-1] .. read[0] (SeedResults::get_rel_offs, aligner_seed.h:1155). */
typedef struct {
	uint64_t read_off;
	uint8_t  seed_off;       /* < 256 (uint8_t in the reference)          */
	uint8_t  seed_len;       /* n_seed_steps, 1..32                       */
	uint8_t  pad[6];
} bt2x_seed_in;

/* SeedAlignerSearchData (aligner_seed.cpp:173-202). */
typedef struct {
	uint64_t topf, botf;     /* last BW range set (valid when need_reporting) */
	uint8_t  nlex;           /* left-extension length, <= 255                */
	uint8_t  need_reporting; /* 1 = seed matched exactly over all its steps  */
	uint8_t  pad[6];
} bt2x_seed_out;

int bt2x_seed_search(bt2x_ctx* ctx, const uint8_t* reads, uint64_t reads_bytes,
                     const bt2x_seed_in* in, uint32_t n, int do_extend, bt2x_seed_out* out);
int bt2x_seed_search_dev(bt2x_ctx* ctx, const uint8_t* d_reads, const bt2x_seed_in* d_in,
                         uint32_t n, int do_extend, bt2x_seed_out* d_out, void* stream);

/* -------------------------------------------------------------------- DP */

/* One end-to-end DP problem, i.e. SwAligner state after initRead + initRef
 * (aligner_sw.cpp:35-229): oriented read codes/qualities (rd_/qu_), reference window
 * codes (0-4; rf_ before the 1<<c mask step) of ncol columns, DPRect fields.
 *
 * flags & BT2X_DP_I16 selects the signed 16-bit kernel, i.e. SwAligner::initRef's
 * enable8_ == false in a -DENABLE_I16 build (aligner_sw.cpp:77-83: enable8 && minsc >=
 * -254): alignEnd2EndSseI16 (aligner_swsse_ee_i16.cpp:548-676) instead of the u8 one.
 * Scores then live in [0x8000, 0x7fff] (0x7fff = score 0, no saturation before -65535),
 * minsc is not clamped (it must be >= -32767, the field's range), align()'s best is the
 * reference's lrmax - 0xff of the i16 value (aligner_swsse_ee_i16.cpp:645), and every
 * attempted candidate consumes {reseed = rnd.nextU32()+1; rnd.init(reseed);} instead of
 * the u8 path's rnd.init(reseed+1) (aligner_sw.cpp:336-348; bt2x_aln_rec.ntries). */
typedef struct {
	uint64_t read_off;       /* reads[read_off .. +rdlen): codes 0-4            */
	uint64_t qual_off;       /* quals[qual_off .. +rdlen): Phred+33 characters  */
	uint64_t ref_off;        /* refs[ref_off .. +ncol): codes 0-4               */
	int64_t  refl;           /* rect.refl; reported offset = col + refl         */
	uint16_t rdlen;          /* rows, 1..BT2X_MAX_ROWS                          */
	uint16_t ncol;           /* rflen_, ncol + 1 <= BT2X_MAX_COLS               */
	int16_t  minsc;          /* clamped to >= -254 (aligner_sw.cpp:77-83)       */
	int16_t  nceil;          /* max Ns in the reference portion                 */
	uint16_t triml, corel, corer;
	uint8_t  fw;             /* orientation: rc results get invertEdits()       */
	uint8_t  flags;          /* BT2X_DP_I16, BT2X_DP_REF_TEXT                      */
} bt2x_dp_in;
#define BT2X_DP_I16 1u
/* The window comes from the index instead of refs[]: ref_off holds the text id (tidx) and
 * the window is text tidx's [refl, refl + ncol), N (4) outside the text and in its N runs
 * -- BitPairReference::getStretch as SwAligner::initRef calls it (aligner_sw.cpp:117-229).
 * The context cuts it from the joined text it keeps in HBM (BT2X_CAP_REF_TEXT). */
#define BT2X_DP_REF_TEXT 2u

/* Result of align() for one problem.  Its nextAlignment() call sequence is
 * recs[rec_off .. rec_off + nrec). */
typedef struct {
	int32_t  status;         /* align() return value                            */
	int32_t  best;           /* best score out of align() (u8: lrmax - 0xff; i16: the
	                          * reference's lrmax - 0xff of the int16 value);
	                          * INT32_MIN if saturated.  Exact whenever status != 0,
	                          * and for failed problems too with BT2X_OPT_EXACT_BEST
	                          * (the default).  Without it a failed problem of a
	                          * launch the banded lane kernel runs may report a lower
	                          * best (still < minsc): the fill skips cells no path
	                          * scoring >= minsc can use.  The reference copies a failed
	                          * problem's best into prm.bestLtMinscMate1
	                          * (aligner_sw_driver.cpp:515-517), printed by ZT:Z under
	                          * --mapq-extra (sam.cpp:519-544). */
	uint16_t ncand;          /* btncand_.size()                                  */
	uint16_t nrec;
	uint32_t rec_off;
} bt2x_dp_out;

/* One nextAlignment(res, minsc, rnd) call.  ntries = candidates backtraced during the
 * call; the caller replays the RNG as ntries x {reseed = rnd.nextU32()+1;
 * rnd.init(reseed+1);} (aligner_sw.cpp:324-336). */
typedef struct {
	uint16_t ntries;
	uint8_t  ok;             /* 1: an alignment was returned; 0: call returned false */
	uint8_t  pad0;
	int16_t  score;          /* AlnScore::score_                                 */
	uint16_t ns;             /* AlnScore::ns_                                    */
	uint16_t gaps;           /* AlnScore::gaps_                                  */
	uint16_t nedit;          /* edits_ = ned().size()                             */
	uint16_t bases_aligned;  /* basesAligned_                                    */
	uint16_t refns;          /* AlnRes::refns_                                   */
	int64_t  refoff;         /* refcoord_.off() = col + rect.refl                */
	uint32_t edit_off;       /* edits[edit_off .. +nedit), final order of ned()  */
	uint32_t nbuf;           /* edit-buffer image, see below                     */
} bt2x_aln_rec;

/* Edit-buffer image.  The reference keeps the edits of every nextAlignment() attempt in
 * one per-read buffer (SwDriver::resGap_.alres.ned_, a DList whose storage is inline) and
 * the alignments it reports copy only the pointer to that storage (DList's implicit copy,
 * ds.h:979-1040).  The SAM record printed at the end of the read therefore shows the
 * buffer's final contents, not the reported edits.  To reproduce that, each
 * record carries edits[edit_off .. edit_off + nbuf): the buffer entries written during
 * the call, as they stand when it returns (a failed backtrace leaves the edits it pushed
 * in backtrace order; a success leaves its final list, which is also the first nedit
 * entries).  A caller replays the images of the calls it consumed, in order, over one
 * buffer per read. */

/* Packed Edit (edit.h:58-310): pos in bits 0-9, type (EDIT_TYPE_*) 12-14,
 * chr 16-23, qchr 24-31 (ASCII, as in Edit::chr/qchr). */
#define BT2X_EDIT_POS(e)  ((uint32_t)(e) & 0x3ffu)
#define BT2X_EDIT_TYPE(e) (((uint32_t)(e) >> 12) & 7u)
#define BT2X_EDIT_CHR(e)  ((char)(((uint32_t)(e) >> 16) & 0xffu))
#define BT2X_EDIT_QCHR(e) ((char)(((uint32_t)(e) >> 24) & 0xffu))

/* Optional debug outputs (may be NULL): per-problem order-independent digests of the
 * filled E, F, H matrices (bt2x_cell_digest of each cell's value as the reference
 * stores it: the u8 byte, or the int16 bit pattern) and the sorted candidate list
 * (DpBtCandidate order, aligner_sw_nuc.h:149), BT2X_MAX_COLS entries per problem
 * (0xffffffff past ncand).  u8 entries are BT2X_CAND_PACK(row, col, score); i16
 * entries BT2X_CAND_PACK16(col, score) (the row is always rdlen - 1,
 * aligner_swsse_ee_i16.cpp:529); score = DpBtCandidate::score, the raw cell value. */
#define BT2X_CAND_PACK(row, col, score) (((uint32_t)(col) << 16) | ((uint32_t)(row) << 8) | (uint32_t)(score))
#define BT2X_CAND_PACK16(col, score) (((uint32_t)(col) << 16) | ((uint32_t)(score) & 0xffffu))
typedef struct {
	uint64_t* digests;       /* 3 per problem: E, F, H                       */
	uint32_t* cands;         /* BT2X_MAX_COLS per problem                    */
} bt2x_dp_debug;

/* Arena capacities are caller-given; on BT2X_E_OVERFLOW *nrec_used / *nedit_used hold
 * the required sizes and the call may be repeated with larger arenas.  reads == quals ==
 * NULL: read_off and qual_off index the read store (bt2x_store_reads, below). */
int bt2x_dp_align(bt2x_ctx* ctx,
                  const uint8_t* reads, uint64_t reads_bytes,
                  const uint8_t* quals, uint64_t quals_bytes,
                  const uint8_t* refs, uint64_t refs_bytes,
                  const bt2x_dp_in* in, uint32_t n,
                  bt2x_dp_out* out,
                  bt2x_aln_rec* recs, uint32_t rec_cap, uint32_t* nrec_used,
                  uint32_t* edits, uint32_t edit_cap, uint32_t* nedit_used,
                  bt2x_dp_debug* debug);

/* Device-pointer variant: all buffers in HBM; counters (4 x u32: recs used, edits used,
 * then kernel scratch) in HBM.  "Edits used" is the arena's high-water mark and may exceed
 * the entries the records reference: a problem whose backtrace walk the lane kernel hands
 * over to the wave kernel (the step budget, BT2X_DP_HEAVY) has already published the edit
 * images of its earlier nextAlignment calls, and the wave kernel publishes the whole call
 * sequence again; the dead ranges are never referenced, and since a retry with the
 * reported size repeats the same hand-overs, that size is what the launch needs.
 * The context's per-launch device buffers (heavy list, failed list, GPU-cut windows) are
 * shared by all calls: calls on one context must be serialised, whatever their streams
 * (like every other entry point; use one context per concurrent stream).
 * launch_flags: BT2X_DPL_I16 when any problem carries
 * BT2X_DP_I16 (the 16-bit kernels run the launch; an i16 problem in a launch without
 * it is reported BT2X_E_ARG by the host variant, and comes back with status -1 here),
 * BT2X_DPL_EXACT_BEST for exact best of failed problems (bt2x_dp_out.best),
 * BT2X_DPL_REF_TEXT when any problem carries BT2X_DP_REF_TEXT (its window is cut from the
 * index first, inside the BT2X_K_DP events).  The host variant derives all three (the
 * second from BT2X_OPT_EXACT_BEST). */
#define BT2X_DPL_I16 1u
#define BT2X_DPL_EXACT_BEST 2u
#define BT2X_DPL_REF_TEXT 4u     /* some problem is BT2X_DP_REF_TEXT */
int bt2x_dp_align_dev(bt2x_ctx* ctx, const uint8_t* d_reads, const uint8_t* d_quals,
                      const uint8_t* d_refs, const bt2x_dp_in* d_in, uint32_t n,
                      bt2x_dp_out* d_out, bt2x_aln_rec* d_recs, uint32_t rec_cap,
                      uint32_t* d_edits, uint32_t edit_cap, uint32_t* d_counters,
                      bt2x_dp_debug* d_debug, uint32_t launch_flags, void* stream);

/* ------------------------------------------------------------- read store */

/* A device-resident copy of the reads in flight: a read's codes and qualities cross PCIe
 * once instead of with every seed round and DP request that needs them (the reference
 * hands SwAligner::initRead the same Read object for every DP, aligner_sw.cpp:59).  The
 * store is BT2X_STORE_SLOT_BYTES per slot; slot s holds, from byte s * SLOT_BYTES on, the
 * read's patFw codes (0-4), its patRc codes, its Phred+33 qualities and the reversed
 * qualities, rdlen bytes each and in that order.  bt2x_store_reads writes n reads into
 * their slots: read i's patFw codes at packed[in[i].off], its qualities right after them
 * (2 * len bytes); the GPU derives patRc and the reversed qualities.  bt2x_seed_round and
 * bt2x_dp_align called with reads == NULL (and quals == NULL) then take read_off and
 * qual_off as offsets into the store.  The store grows to the largest slot written and
 * keeps its contents; calls on the context's stream stay in order.  Requests are checked
 * against the written extent ((highest slot put + 1) * SLOT_BYTES), not the allocation;
 * a slot below it that was never put reads as N codes (4).  A slot's layout is tied to
 * the len it was put with: offsets into it must use that rdlen. */
#define BT2X_STORE_SLOT_BYTES 1024u
#define BT2X_STORE_MAX_LEN 256u
typedef struct {
	uint64_t off;            /* packed[off .. +len): patFw codes; [off+len .. +len): quals */
	uint32_t slot;
	uint16_t len;            /* 1..BT2X_STORE_MAX_LEN */
	uint16_t pad;
} bt2x_store_in;
int bt2x_store_reads(bt2x_ctx* ctx, const uint8_t* packed, uint64_t packed_bytes, const bt2x_store_in* in,
                     uint32_t n);

/* SAM record tails from the read store (ABI 4, round 6).  Replaces the text the reference's
 * AlnSinkSam::appendMate writes after an aligned read's MAPQ field (aln_sink.cpp:1889-2090,
 * SamConfig::printAlignedOptFlags sam.cpp:121-730) for the common record whose printed
 * edits are mismatches only (the CIGAR is one <rdlen>M run; StackedAln over such edits,
 * aligner_result.cpp:448-770).  Per request: "CIGAR\t*\t0\t0\tSEQ\tQUAL\tAS:i:as
 * [\tXS:i:xs]\tXN:i:xn\tXM:i:nmm\tXO:i:0\tXG:i:0\tNM:i:nmm\tMD:Z:md\tYT:Z:UU\tYF:Z:LN\n"
 * (the leading tab before CIGAR is the caller's).  SEQ/QUAL are the store slot's patFw and
 * qualities (fw) or patRc and reversed qualities, codes printed as ACGTN.  mm_pos are the
 * mismatches' positions in the printed read (0-based, increasing, < rdlen), mm_chr their
 * reference characters.  The text goes to text[text_off ..) and is at most
 * BT2X_SAM_TAIL_MAX(rdlen, nmm) bytes; lens[i] receives its length.  The slot must hold the
 * read the request names (put with the same rdlen). */
#define BT2X_SAM_MAX_MM 16
#define BT2X_SAM_TAIL_MAX(rdlen, nmm) (2u * (rdlen) + 200u + 4u * (nmm))
typedef struct {
	uint32_t slot;
	uint16_t rdlen;          /* 1..BT2X_STORE_MAX_LEN */
	uint8_t fw;              /* 1: patFw + qualities; 0: patRc + reversed qualities */
	uint8_t nmm;             /* 0..BT2X_SAM_MAX_MM */
	int32_t as;              /* AS:i */
	int32_t xs;              /* XS:i, printed when has_xs */
	uint32_t xn;             /* XN:i */
	uint32_t has_xs;
	uint64_t text_off;
	uint16_t mm_pos[BT2X_SAM_MAX_MM];
	uint8_t mm_chr[BT2X_SAM_MAX_MM];
} bt2x_sam_req;
/* host buffers: text holds text_bytes bytes (every request's text_off + its bound) */
int bt2x_sam_tails(bt2x_ctx* ctx, const bt2x_sam_req* req, uint32_t n, char* text, uint64_t text_bytes,
                   uint16_t* lens);
/* HBM buffers, async on `stream` (NULL: the context's stream) */
int bt2x_sam_tails_dev(bt2x_ctx* ctx, const bt2x_sam_req* d_req, uint32_t n, char* d_text, uint16_t* d_lens,
                       void* stream);

/* Context options.  BT2X_OPT_EXACT_BEST (default 1): bt2x_dp_align reports the exact
 * best of failed problems (one extra unbanded pass over them); 0 when the caller never
 * reads it (bowtie2 prints it only under --mapq-extra). */
enum { BT2X_OPT_EXACT_BEST = 1 };
int bt2x_set_option(bt2x_ctx* ctx, int option, int64_t value);

/* What the context can do: BT2X_CAP_REF_TEXT -- DP problems may name their window
 * (BT2X_DP_REF_TEXT); needs the joined text resident, i.e. an index loaded with
 * load_offs and a text of < 2^32 rows. */
#define BT2X_CAP_REF_TEXT 1u
int bt2x_capabilities(const bt2x_ctx* ctx, uint32_t* caps);

/* Order-independent digest of one matrix cell (shared by oracle, kernel and harness). */
static inline uint64_t bt2x_cell_digest(uint32_t row, uint32_t col, uint32_t mat, uint32_t val) {
	uint64_t z = ((uint64_t)row << 40) ^ ((uint64_t)col << 20) ^ ((uint64_t)mat << 16) ^ (uint64_t)val;
	z += 0x9e3779b97f4a7c15ULL;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
	return z ^ (z >> 31);
}

/* Rows [first, first+n) of the device-resident full suffix array (BT2X_E_ARG if the
 * context has none: no SA sample/text loaded, or a text of 2^32 rows or more). */
int bt2x_suffix_array(bt2x_ctx* ctx, uint64_t first, uint64_t n, uint32_t* out);

/* --------------------------------------------------------- SA resolution */

/* One BW element of a seed hit to place on the reference.  Replaces, per element,
 * GroupWalk2S::advanceElement (group_walk.h:969; GWState::init/advance :402/:687,
 * Ebwt::tryOffset bt2_idx.h:1621), whose WalkResult::toff is the joined-text offset
 * of the row (== Ebwt::getOffset(row), bt2_idx.cpp:150, asserted at group_walk.h:430),
 * followed by Ebwt::joinedToTextOff(qlen, toff, ...) (bt2_idx.cpp:54) as
 * SwDriver::extendSeeds calls it (aligner_sw_driver.cpp:388-402; qlen = wr.elt.len,
 * the seed key length). */
typedef struct {
	uint64_t row;            /* BWT row, <= len                                         */
	uint32_t qlen;           /* hit length                                              */
	uint32_t pad;
} bt2x_resolve_in;

typedef struct {
	uint64_t joff;           /* offset into the joined text (WalkResult::toff)           */
	uint64_t toff;           /* textoff: offset into reference tidx                      */
	uint64_t tlen;           /* plen[tidx]                                               */
	uint32_t tidx;           /* reference index; BT2X_NO_TIDX when reject_straddle
	                            rejected the hit (toff = tlen = 0 then, the caller's
	                            zero-initialised values at aligner_sw_driver.cpp:392) or
	                            joff lies in no fragment (only row len, the '$' suffix) */
	uint32_t straddled;      /* 1 if joff + qlen runs past the fragment's end            */
} bt2x_resolve_out;
#define BT2X_NO_TIDX 0xffffffffu

/* One element of a seed round (bt2x_seed_round): the reference coordinate of
 * bt2x_resolve_out without the joined offset and the text length (the caller's
 * plen[tidx]), packed into 8 bytes across PCIe instead of 32:
 *   bits  0..38  textoff (offset into reference tidx)
 *   bit  39      straddled (the hit runs past its fragment's end)
 *   bits 40..63  tidx; 0xffffff = BT2X_NO_TIDX (toff = 0): the row lies in no fragment
 * so a seed round needs fewer than 2^24 - 1 references (BT2X_E_ARG otherwise) and texts
 * shorter than 2^39.  Read them with bt2x_elt_toff / _tidx / _straddled. */
typedef struct {
	uint64_t v;
} bt2x_elt;
#define BT2X_ELT_TIDX_NONE 0xffffffu
static inline uint64_t bt2x_elt_toff(bt2x_elt e) { return e.v & ((1ull << 39) - 1); }
static inline uint32_t bt2x_elt_straddled(bt2x_elt e) { return (uint32_t)(e.v >> 39) & 1u; }
static inline uint32_t bt2x_elt_tidx(bt2x_elt e) {
	const uint32_t t = (uint32_t)(e.v >> 40);
	return t == BT2X_ELT_TIDX_NONE ? BT2X_NO_TIDX : t;
}
static inline bt2x_elt bt2x_elt_pack(uint64_t toff, uint32_t tidx, uint32_t straddled) {
	bt2x_elt e;
	e.v = (toff & ((1ull << 39) - 1)) | ((uint64_t)(straddled & 1u) << 39) |
	      ((uint64_t)(tidx == BT2X_NO_TIDX ? BT2X_ELT_TIDX_NONE : tidx & BT2X_ELT_TIDX_NONE) << 40);
	return e;
}

/* With the resident full suffix array this is one 4-byte lookup per element; without
 * it (texts of 2^32 rows or more, BT2X_FULL_SA=0) the kernel walks LF to the SA sample
 * exactly like GWState (<= 2^offRate - 1 steps).  Needs an index loaded with
 * load_offs (BT2X_E_ARG otherwise).  Rows > len give BT2X_E_ARG (host variant). */
int bt2x_resolve(bt2x_ctx* ctx, const bt2x_resolve_in* in, uint32_t n, int reject_straddle,
                 bt2x_resolve_out* out);
int bt2x_resolve_dev(bt2x_ctx* ctx, const bt2x_resolve_in* d_in, uint32_t n, int reject_straddle,
                     bt2x_resolve_out* d_out, void* stream);

/* ------------------------------------------------------------- seed round */

/* One read's seed round: its seeds (searched as bt2x_seed_search does), then the rest of
 * the round up to the first DP, per read on the GPU:
 *   SeedAligner::searchAllSeedsFinalize + SeedResults::add  aligner_seed.cpp:508-540,
 *                                                            aligner_seed.h:603-641
 *   SeedResults::rankSeedHits                               aligner_seed.h:1000-1061
 *   SwDriver::prioritizeSATups                               aligner_sw_driver.cpp:61-260
 *     (RowSampler aligner_sw_driver.h:176-267, Random1toN random_util.h:32-230)
 *   GroupWalk2S::advanceElement + joinedToTextOff for every   group_walk.h:969,
 *     element extendSeeds may visit (as bt2x_resolve)        bt2_idx.cpp:54
 * The read's RandomSource is carried in and out (rnd_last / rnd_lastoff = the LCG state
 * and bit offset, random_source.h:34-140).  Seeds: in[r].nseeds entries of `seeds`
 * starting at in[r].seed0, patFw seeds (read_off == in[r].read_off) and patRc seeds
 * (read_off == in[r].read_off + rdlen) instantiated at depth i*interval + offset as in
 * MultiSeedResults::instantiateSeeds (aligner_seed.cpp:411-447). */
typedef struct {
	uint64_t read_off;       /* patFw at reads[read_off], patRc right after it           */
	uint64_t seed0;          /* first seed of the read in `seeds`                         */
	uint32_t rnd_last;       /* RandomSource state before rankSeedHits                    */
	int32_t  rnd_lastoff;
	uint32_t exr0;           /* exRange entries of earlier rounds: exr[exr0 .. +nexr)     */
	uint16_t nexr;
	uint16_t nseeds;         /* seeds searched for the read                               */
	uint16_t num_offs;       /* SeedResults::numOffs(): seed offsets per strand            */
	uint16_t rdlen;
	uint16_t interval;       /* msIval(rdlen)                                             */
	uint16_t offset;         /* this round's offset: interval * round / nrounds           */
	uint16_t seedlen;        /* multiseedLen clipped to rdlen                              */
	uint16_t seedflags;      /* seeds == NULL (below): 1 = no patFw seeds (--nofw), 2 = no
	                            patRc seeds (--norc)                                        */
	uint16_t pad[2];
} bt2x_round_in;

/* extendSeeds' exRange entry: a read span [off, off+len) of strand fw already covered by
 * a unique-extended range of sz elements (aligner_sw_driver.cpp:97-144). */
typedef struct {
	uint64_t sz;
	uint32_t off;
	uint16_t len;
	uint8_t  fw;
	uint8_t  pad;
} bt2x_exrange;

/* One SATupleAndPos of the read's extension list, in prioritizeSATups order: rand_n BW
 * elements (the whole range when it has <= 5 elements, else one sampled element), seed
 * of length seedlen at read offset rdoff of strand fw.  4 bytes: fw and seedlen share a
 * byte (BT2X_SAT_FW / BT2X_SAT_LEN, BT2X_SAT_FWLEN to build it). */
typedef struct {
	uint16_t rdoff;
	uint8_t  rand_n;
	uint8_t  fwlen;          /* bit 7: fw; bits 0-6: seedlen */
} bt2x_sat;
#define BT2X_SAT_FW(s) ((uint32_t)(s).fwlen >> 7)
#define BT2X_SAT_LEN(s) ((uint32_t)(s).fwlen & 0x7fu)
#define BT2X_SAT_FWLEN(fw, len) ((uint8_t)(((fw) ? 0x80u : 0u) | ((uint32_t)(len) & 0x7fu)))

enum { BT2X_ROUND_OK = 0, BT2X_ROUND_NO_HITS = 1, BT2X_ROUND_REDO = 2 };

typedef struct {
	uint32_t rnd_last;       /* RandomSource state after ranking and sampling             */
	int32_t  rnd_lastoff;
	uint64_t num_elts;       /* SeedResults::numElts()                                    */
	uint32_t nonz;           /* SeedResults::nonzeroOffsets()                             */
	uint32_t status;         /* BT2X_ROUND_OK; NO_HITS (no seed hit: the read's seed rounds
	                            end); REDO: the read exceeded the kernel's per-read workspace
	                            (more than 64 seed offsets per strand or very repetitive
	                            sampling) -- the caller runs this round with
	                            bt2x_seed_search + its own prioritization + bt2x_resolve    */
	uint32_t sat0, nsat;     /* sats[sat0 .. +nsat)                                       */
	uint32_t elt0, nelt;     /* elts[elt0 .. +nelt): the sats' elements in order           */
	uint32_t exr0, nexr;     /* exRange entries this round added: exr_out[exr0 .. +nexr)   */
} bt2x_round_out;

/* maxelt: -D ... maxIters (prioritizeSATups' maxelt, 400 by default).  Output arenas are
 * caller-sized; BT2X_E_OVERFLOW reports the required sizes in used[0..2] (sats, elts,
 * exr_out) and the call may be repeated.  reads == NULL: read_off (of in[] and seeds[])
 * indexes the read store (bt2x_store_reads).  seeds == NULL: the GPU instantiates every
 * read's seeds itself, as listed above (patFw seeds, then patRc seeds, each strand at
 * depths i * interval + offset for i < num_offs, a seed over an N skipped, a strand off
 * per seedflags), into seeds[seed0 .. +nseeds) of a context-owned array of nseeds entries:
 * in[r].nseeds must be the count that gives (and the reads' seeds must not overlap).  The
 * library checks it on the GPU: when any read's count differs the call returns BT2X_E_ARG
 * (its slots were filled with in-bounds stand-ins, so nothing stale was searched). */
int bt2x_seed_round(bt2x_ctx* ctx, const uint8_t* reads, uint64_t reads_bytes,
                    const bt2x_seed_in* seeds, uint32_t nseeds,
                    const bt2x_round_in* in, uint32_t nreads,
                    const bt2x_exrange* exr, uint32_t nexr, uint32_t maxelt,
                    bt2x_round_out* out,
                    bt2x_sat* sats, uint32_t sat_cap,
                    bt2x_elt* elts, uint32_t elt_cap,
                    bt2x_exrange* exr_out, uint32_t exr_cap,
                    uint32_t used[3]);
/* Device-pointer variant (inputs resident in HBM; d_used: 4 x u32 in HBM, [0..2] as used[]
 * above and [3] the number of reads whose GPU-instantiated seed count differed from
 * in[r].nseeds -- nonzero means the round's outputs are not to be used).  Events:
 * BT2X_K_SEED brackets the seed kernel, BT2X_K_RESOLVE the ranking + resolution,
 * BT2X_K_ROUND the whole round. */
int bt2x_seed_round_dev(bt2x_ctx* ctx, const uint8_t* d_reads, const bt2x_seed_in* d_seeds, uint32_t nseeds,
                        const bt2x_round_in* d_in, uint32_t nreads, const bt2x_exrange* d_exr, uint32_t maxelt,
                        bt2x_round_out* d_out, bt2x_sat* d_sats, uint32_t sat_cap,
                        bt2x_elt* d_elts, uint32_t elt_cap, bt2x_exrange* d_exr_out, uint32_t exr_cap,
                        uint32_t* d_used, void* stream);

/* Page-locked host memory for the buffers a caller hands to the host-pointer entry points
 * (their copies then run as DMA at the link's rate instead of staging through pageable
 * memory).  NULL on failure; bt2x_host_free(NULL) is a no-op.  Not needed for
 * correctness: every entry point accepts ordinary memory. */
void* bt2x_host_alloc(size_t bytes);
void  bt2x_host_free(void* p);

const char* bt2x_version(void);
int bt2x_abi_version(void);      /* BT2X_ABI_VERSION the library was built with */
/* sizeof of the ABI structs (seed_in, seed_out, dp_in, dp_out, aln_rec, scoring,
 * index_desc, counters, resolve_in, resolve_out, round_in, round_out, sat, exrange, elt,
 * store_in), for binding self-checks; returns the count. */
int bt2x_abi_sizes(uint32_t* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* BT2X_H_ */
