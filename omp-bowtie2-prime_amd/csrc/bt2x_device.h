// bt2x_device.h — device-side types shared by the gfx950 kernels and the host API.
//
// MI355X layout of the FM index (SURVEY §3.4, bt2_idx.h:2617-2639): the .bt2l side
// array is uploaded verbatim (128-byte sides, 128-byte aligned in HBM, so one side is
// exactly one L2 line), ftab/eftab/fchr as-is.  Nothing is re-packed: the reference's
// own layout is already one cache line per LF step.
#pragma once
#include <stdint.h>
#include "../../include/bt2x.h"

struct DevIndex {
	const uint8_t* ebwt;      // numSides * 128 bytes (.bt2l sides, as uploaded)
	const uint8_t* blk;       // device re-layout (bt2x_build_blocks): 64-byte blocks of 192
	                          // rows = 4 x u32 occ at the block start + 48 B of BWT; NULL if
	                          // the text is too long for u32 counts (then sides are used)
	const uint64_t* ftab;     // 4^ftabChars + 1
	const uint64_t* eftab;    // 2 * ftabChars
	uint64_t len;             // joined text length
	uint64_t zoff;            // '$' row
	uint64_t zbyte;           // byte offset of '$' in ebwt (Ebwt::postReadInit, bt2_idx.h:1684)
	uint64_t fchr[5];
	int32_t zbp;              // bit-pair of '$' within zbyte
	int32_t ftab_chars;
	int32_t off_rate;
	const uint32_t* sa;       // full suffix array (rows 0..len), rebuilt in HBM at open; or NULL
	const uint32_t* text;     // joined text, 16 bases per u32 (LSB-first); with sa
	const uint64_t* offs;     // SA sample (.2.bt2l), kept only when there is no full sa
	const uint64_t* rstarts;  // 3 words per fragment (joined off, tidx, text off)
	const uint64_t* plen;     // reference lengths
	uint64_t nfrag;
	const uint32_t* tfirst;   // text t's fragments are rstarts[tfirst[t] .. tfirst[t+1]) (npat+1
	                          // entries; fragments are in joined = text order); or NULL
	uint64_t npat;            // number of texts (tfirst has npat + 1 entries)
};

// Internal dp_in flag (never set by callers; bt2x.h uses bits 0-1): the window kernel
// could not cut the problem's BT2X_DP_REF_TEXT window (no resident text, or a text id out
// of range), so the DP kernels refuse it (status -1, counters[3]) instead of reading it.
constexpr uint8_t kDpBadWindow = 0x80u;
// DP windows (window_kernel): one slot per problem, BT2X_MAX_COLS bytes rounded up to 16
// so the fill's 16-byte LDS-DMA chunks are aligned; the buffer has a 64-byte tail.
constexpr uint32_t kWinSlot = (BT2X_MAX_COLS + 15) & ~15u;

struct DevScoring {
	int32_t rdo, rde, rfo, rfe;   // read/ref gap open (const+linear) and extend (linear)
	int32_t gapbar;
	int32_t npen;                 // constant N penalty (COST_MODEL_CONSTANT)
	uint8_t mmpen[256];           // mismatch penalty by (qual-33), COST_MODEL_QUAL
};

// Launch helpers implemented in the kernel translation units.
#define BT2X_BLK_ROWS 192
#define BT2X_BLK_BYTES 64
int bt2x_build_blocks(const DevIndex& ix, uint64_t nsides, uint8_t* d_blk, void* stream);
int bt2x_build_sa(const DevIndex& ix, const uint64_t* d_offs, uint64_t noffs, uint32_t* d_sa, void* stream);
int bt2x_launch_seed(const DevIndex& ix, const uint8_t* d_reads, const bt2x_seed_in* d_in,
                     uint32_t n, int do_extend, bt2x_seed_out* d_out,
                     unsigned long long* d_ctr, int ncu, void* stream);
// a seed round's seeds instantiated on the GPU (bt2x_seed_round with seeds == NULL)
int bt2x_launch_seed_gen(const uint8_t* d_reads, const bt2x_round_in* d_in, uint32_t nreads, bt2x_seed_in* d_seeds,
                         uint32_t nseeds, uint32_t* d_bad, void* stream);

int bt2x_launch_resolve(const DevIndex& ix, const bt2x_resolve_in* d_in, uint32_t n, int reject,
                        bt2x_resolve_out* d_out, unsigned long long* d_ctr, void* stream);
// element count in HBM (*d_n, at most cap): persistent grid-stride launch
int bt2x_launch_resolve_dn(const DevIndex& ix, const bt2x_resolve_in* d_in, const uint32_t* d_n, uint32_t cap,
                           int reject, bt2x_resolve_out* d_out, unsigned long long* d_ctr, int ncu, void* stream);
int bt2x_launch_resolve_dn(const DevIndex& ix, const bt2x_resolve_in* d_in, const uint32_t* d_n, uint32_t cap,
                           int reject, bt2x_elt* d_out, unsigned long long* d_ctr, int ncu, void* stream);

// DP windows cut from the resident text (window_kernel.hip): every problem's window to
// win[i * BT2X_MAX_COLS ..), its dp_in to out[i] with ref_off rebased and the flag cleared.
int bt2x_launch_windows(const DevIndex& ix, const bt2x_dp_in* d_in, uint32_t n, const uint8_t* d_refs,
                        bt2x_dp_in* d_out, uint8_t* d_win, void* stream);

// Seed round (round_kernel.hip): per read, finalize + rank + prioritize after its seed
// search; sats/rows/exr_out allocated by atomics on counters[0..2].
struct RoundLaunch {
	const bt2x_seed_in* seeds; const bt2x_seed_out* seed_out;
	const bt2x_round_in* in; uint32_t n;
	const bt2x_exrange* exr;
	uint32_t maxelt;
	bt2x_round_out* out;
	bt2x_sat* sats; uint32_t sat_cap;
	bt2x_resolve_in* rows; uint32_t row_cap;
	bt2x_exrange* exr_out; uint32_t exr_cap;
	uint32_t* counters;            // [0] sats, [1] rows, [2] exr_out, [3] sampling jobs, [4] their ranges
	                               // (used, may exceed caps)
	uint8_t* jobs; uint32_t job_cap;
	uint8_t* ranges; uint32_t range_cap;
	uint8_t* ws; uint32_t nlanes;  // per-lane workspace of the prep kernel
};
size_t bt2x_round_ws_bytes();
size_t bt2x_round_job_bytes();
size_t bt2x_round_range_bytes();
uint32_t bt2x_round_lanes(int ncu);
int bt2x_launch_round(const RoundLaunch& a, void* stream);
// read store (bt2x_store_reads): n packed reads into their BT2X_STORE_SLOT_BYTES slots
// SAM record tails (bt2x_sam_tails): one wave per request
int bt2x_launch_sam_tails(const bt2x_sam_req* d_req, uint32_t n, const uint8_t* d_store, char* d_text,
                          uint16_t* d_lens, int ncu, void* stream);
int bt2x_launch_store(const uint8_t* d_packed, const bt2x_store_in* d_in, uint32_t n, uint8_t* d_store,
                      void* stream);

struct DpLaunch {
	const uint8_t* reads; const uint8_t* quals; const uint8_t* refs;
	const bt2x_dp_in* in; uint32_t n;
	bt2x_dp_out* out;
	bt2x_aln_rec* recs; uint32_t rec_cap;
	uint32_t* edits; uint32_t edit_cap;
	uint32_t* counters;            // [0] recs used, [1] edits used, [2] fail_list entries, [3] refused
	                               // (i16 problems in a u8 launch)
	unsigned long long* stats;     // dp_cells, dp_cols, bt_cells, dp_cells_computed
	uint64_t* digests;             // optional, 3 per problem
	uint32_t* cands;               // optional, BT2X_MAX_COLS per problem
	uint8_t* scratch;              // chunk_groups fill regions, then the walk staging slots
	uint8_t* walk_scratch;         // set by bt2x_launch_dp
	uint32_t chunk_groups;         // 64-problem groups per fill/walk chunk
	int ncu;                       // compute units (persistent grid sizing)
	uint32_t* queue;               // walk-kernel problem queue counter (device)
	uint32_t ablate;               // profiling only: 1 = stop after the fill, 2 = no backtrace walks (outputs invalid)
	uint32_t band;                 // 1: lane-kernel fill restricted to the exact diagonal band (dp_kernel.hip)
	uint32_t wide;                 // 1: the 16-bit lane kernels (some problem is BT2X_DP_I16)
	uint32_t* fail_list;           // n entries, or NULL: queue the banded fill's failed problems for
	                               // the exact-best pass (BT2X_DPL_EXACT_BEST)
	uint32_t* heavy_list;          // [0]: count, then problem indices: problems whose walk the lane
	                               // kernel hands to the wave kernel (more than `heavy` candidates)
	uint32_t heavy;
	uint32_t wave_hand;            // small-launch wave kernel (banded layout): a problem with at least
	                               // this many candidates goes to heavy_list for the wave-parallel
	                               // walk of dp_wave_kernel<2> (0: never)
	unsigned long long* prof;      // development (BT2X_DP_PROF=1): lane-kernel fill cycles, walk
	                               // cycles, walk wave-steps, candidate wave-iterations, groups
	const uint8_t* mmpen;          // DevScoring::mmpen in HBM (256 B): the kernels index it per lane,
	                               // which a kernel-argument array would turn into SGPR spills
};
size_t bt2x_dp_scratch_bytes(int ncu, uint32_t chunk_groups);
int bt2x_launch_dp(const DevScoring& sc, const DpLaunch& a, void* stream);
