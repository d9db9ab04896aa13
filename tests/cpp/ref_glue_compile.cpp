// Compile-only check (tests/test_integration.py, needs /root/reference): the INTEGRATION.md
// patches -- include/bt2x_shims.hpp and include/bt2x_ref_glue.hpp -- instantiated with
// the reference's own types (BTDnaString, BTString, Scoring, BitPairReference, DPRect,
// RandomSource, SwResult/AlnRes, SeedAlignerSearchParams/Data).  Built with the
// reference's compile definitions (oracle/Makefile REFDEFS); never linked or run.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>
#include <omp.h>
#define private public                  // the patched member bodies use MultiSeedAligner's members
#include "bowtie2-align.cpp"            // the reference's single TU, in its own include order
#undef private
#include "bt2x_ref_glue.hpp"

// aligner_seed.cpp:674, patched (INTEGRATION.md "Seed search"): the member's new body.
void patched_searchAllSeedsDoAll(MultiSeedAligner& self, bt2x::Device& dev, bool doExtend) {
	bt2x::MultiSeedAlignerHip gpu(dev);
	if(!bt2x::glue::search_all_seeds(gpu, self._paramVec, self._dataVec, self._bufVec_filled, doExtend)) throw 1;
}

// aligner_sw_driver.cpp:481-538, patched (INTEGRATION.md "DP"): SwAligner swapped for the
// shim, each result translated into the driver's SwResult.
size_t patched_extend(bt2x::Device& dev, const Read& rd, const Scoring& sc, bool fw, TRefId tidx, const DPRect& rect,
                      const BitPairReference& ref, TRefOff tlen, TAlScore minsc, bool enable8, size_t nwindow,
                      RandomSource& rnd, SwResult& res) {
	bt2x::SwAlignerHip swa(dev);
	const size_t rdlen = rd.length();
	size_t nsInLeftShift = 0;
	if(!swa.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, rdlen, sc)) return 0;
	if(!swa.initRef(fw, (size_t)tidx, rect, ref, (int64_t)tlen, (int64_t)minsc, enable8, true, nwindow, nsInLeftShift))
		return 0;
	int64_t best = 0;
	size_t n = 0;
	if(swa.align(best)) {
		bt2x::AlnView v;
		while(!swa.done()) {
			res.reset();
			const bool ok = swa.nextAlignment(v, (int64_t)minsc, rnd);
			bt2x::glue::to_swresult(v, ok, res, (size_t)tidx, (int64_t)tlen, rdlen);
			if(!ok) break;
			n++;
		}
	}
	return n;
}
