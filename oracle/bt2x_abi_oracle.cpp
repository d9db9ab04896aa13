// bt2x_abi_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// The part of the bt2x C-ABI (include/bt2x.h) that include/bt2x_shims.hpp calls --
// index load, context open/close, seed search, DP -- answered by the CPU oracle
// (oracle/bt2x_oracle.c) instead of the GPU.  Linked only into the CPU variant of the
// patched reference aligner (oracle/ref_glue_build.py --cpu), so the drop-in's glue runs
// in the CPU test suite; the product (bt2x-align, libbt2x.so) never links it.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "bt2x_oracle.h"

struct bt2x_ctx {
	const bt2x_index_desc* idx;
	bt2x_scoring sc;
};

extern "C" {

int bt2x_index_load(const char* basename, int load_offs, bt2x_index_desc* out) {
	return bt2o_index_load(basename, load_offs, out);
}
void bt2x_index_free(bt2x_index_desc* idx) { bt2o_index_free(idx); }
void bt2x_scoring_default(bt2x_scoring* sc) { bt2o_scoring_default(sc); }
void bt2x_scoring_init(bt2x_scoring* sc) { bt2o_scoring_init(sc); }

int bt2x_open(int /*hip_device*/, const bt2x_index_desc* idx, const bt2x_scoring* sc, bt2x_ctx** out) {
	if(!idx || !out) return BT2X_E_ARG;
	bt2x_ctx* c = new bt2x_ctx;
	c->idx = idx;
	if(sc) c->sc = *sc; else bt2o_scoring_default(&c->sc);
	*out = c;
	return BT2X_OK;
}
void bt2x_close(bt2x_ctx* c) { delete c; }

int bt2x_seed_search(bt2x_ctx* c, const uint8_t* reads, uint64_t /*reads_bytes*/, const bt2x_seed_in* in, uint32_t n,
                     int do_extend, bt2x_seed_out* out) {
	if(!c) return BT2X_E_ARG;
	return bt2o_seed_search(c->idx, reads, in, n, do_extend, out, nullptr) ? BT2X_E_ARG : BT2X_OK;
}

int bt2x_dp_align(bt2x_ctx* c, const uint8_t* reads, uint64_t, const uint8_t* quals, uint64_t, const uint8_t* refs,
                  uint64_t, const bt2x_dp_in* in, uint32_t n, bt2x_dp_out* out, bt2x_aln_rec* recs, uint32_t rec_cap,
                  uint32_t* nrec_used, uint32_t* edits, uint32_t edit_cap, uint32_t* nedit_used, bt2x_dp_debug* debug) {
	if(!c) return BT2X_E_ARG;
	uint32_t nrec = 0, ned = 0;
	const int rc = bt2o_dp_align(&c->sc, reads, quals, refs, in, n, out, recs, rec_cap, &nrec, edits, edit_cap, &ned,
	                             debug, nullptr);
	if(std::getenv("BT2X_GLUE_TRACE"))
		for(uint32_t i = 0; i < n && !rc; i++) {
			const bt2x_dp_in& p = in[i];
			std::fprintf(stderr, "ABI dp rd=%llu q=%llu ref=%llu refl=%lld rdlen=%u ncol=%u minsc=%d nceil=%d trim=%u core=[%u,%u] "
			             "fw=%u flags=%u -> status=%d best=%d nrec=%u\n", (unsigned long long)p.read_off,
			             (unsigned long long)p.qual_off, (unsigned long long)p.ref_off, (long long)p.refl, p.rdlen, p.ncol,
			             p.minsc, p.nceil, p.triml, p.corel, p.corer, p.fw, p.flags, out[i].status, out[i].best, out[i].nrec);
			for(uint32_t k = 0; k < out[i].nrec && out[i].rec_off + k < rec_cap; k++) {
				const bt2x_aln_rec& r = recs[out[i].rec_off + k];
				std::fprintf(stderr, "ABI   rec ok=%d score=%d refoff=%lld ntries=%u nedit=%u nbuf=%u\n", (int)r.ok, r.score,
				             (long long)r.refoff, (unsigned)r.ntries, (unsigned)r.nedit, (unsigned)r.nbuf);
			}
		}
	if(nrec_used) *nrec_used = nrec;
	if(nedit_used) *nedit_used = ned;
	if(rc) return rc;
	return (nrec > rec_cap || ned > edit_cap) ? BT2X_E_OVERFLOW : BT2X_OK;
}

}  // extern "C"
