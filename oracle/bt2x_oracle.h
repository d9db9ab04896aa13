/*
 * oracle/bt2x_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference hot path, used as the checker for the
 * HIP kernels (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg only).
 * It takes and returns exactly the structs of include/bt2x.h so a test can feed the
 * same batch to both.  Parity of this restatement is pinned against golden vectors
 * dumped from the reference itself (oracle/refharness.cpp -> tests/golden/).
 */
#ifndef BT2X_ORACLE_H_
#define BT2X_ORACLE_H_
#include "../include/bt2x.h"

#ifdef __cplusplus
extern "C" {
#endif

int  bt2o_index_load(const char* basename, int load_offs, bt2x_index_desc* out);
void bt2o_index_free(bt2x_index_desc* idx);
void bt2o_scoring_default(bt2x_scoring* sc);
void bt2o_scoring_init(bt2x_scoring* sc);

int bt2o_seed_search(const bt2x_index_desc* idx, const uint8_t* reads,
                     const bt2x_seed_in* in, uint32_t n, int do_extend,
                     bt2x_seed_out* out, bt2x_counters* ctr);

int bt2o_dp_align(const bt2x_scoring* sc,
                  const uint8_t* reads, const uint8_t* quals, const uint8_t* refs,
                  const bt2x_dp_in* in, uint32_t n, bt2x_dp_out* out,
                  bt2x_aln_rec* recs, uint32_t rec_cap, uint32_t* nrec_used,
                  uint32_t* edits, uint32_t edit_cap, uint32_t* nedit_used,
                  bt2x_dp_debug* debug, bt2x_counters* ctr);

/* SA resolution of BW elements: getOffset + joinedToTextOff (needs load_offs). */
int bt2o_resolve(const bt2x_index_desc* idx, const bt2x_resolve_in* in, uint32_t n, int reject_straddle,
                 bt2x_resolve_out* out, bt2x_counters* ctr);

/* Helpers exposed for unit tests of the primitives. */
uint64_t bt2o_count_side(const bt2x_index_desc* idx, uint64_t row, int c);
void     bt2o_count_side_ex(const bt2x_index_desc* idx, uint64_t row, uint64_t out[4]);
int      bt2o_row_l(const bt2x_index_desc* idx, uint64_t row);

/* Per-read RNG (random_source.h:34-140) so tests can replay nextAlignment draws. */
typedef struct { uint32_t last; int last_off; } bt2o_rng;
void     bt2o_rng_init(bt2o_rng* r, uint32_t seed);
uint32_t bt2o_rng_next_u32(bt2o_rng* r);

#ifdef __cplusplus
}
#endif
#endif
