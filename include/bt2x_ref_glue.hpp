// bt2x_ref_glue.hpp — the two patches INTEGRATION.md applies to the reference, as
// templates over its own types, so the patched members are one-line calls:
//
//   MultiSeedAligner::searchAllSeedsDoAll (aligner_seed.cpp:674-725)
//       -> bt2x::glue::search_all_seeds(gpu, _paramVec, _dataVec, _bufVec_filled, doExtend)
//   SwAligner results in SwDriver::extendSeeds (aligner_sw_driver.cpp:481-538)
//       -> bt2x::glue::to_swresult(view, res, tidx, tlen, rdlen)
//
// Params/Data are SeedAlignerSearchParams / SeedAlignerSearchData (aligner_seed.cpp:81-202);
// Res is SwResult (aligner_sw_common.h) whose alres is an AlnRes (aligner_result.h).
// tests/cpp/ref_glue_compile.cpp instantiates both with the reference's types
// (tests/test_integration.py, when /root/reference is present).
#pragma once
#include <cstdint>
#include <type_traits>
#include <vector>

#include "bt2x_shims.hpp"

namespace bt2x {
namespace glue {

// The seed batch of MultiSeedAligner as one GPU call.  The reference's extension walks
// seq[-ii] over the `lim` read characters left of the seed (SeedResults::get_rel_offs,
// aligner_seed.h:1155), and the seed itself is read[lim .. lim+len) of the same oriented
// read (SeedAligner::instantiateSeq, aligner_seed.cpp:301-314), so the kernel gets that
// read's prefix in place: seeds of one read orientation share one pointer, which
// MultiSeedAlignerHip::add copies once.  Returns false on a device error (the caller's
// `throw 1`).
template<class Params, class Data>
bool search_all_seeds(MultiSeedAlignerHip& gpu, const Params* paramVec, Data* dataVec, size_t n, bool doExtend) {
	gpu.clear();
	for(size_t i = 0; i < n; i++) {
		const Params& p = paramVec[i];
		const char* left = nullptr;
		uint8_t lim = 0;
		p.sr->get_rel_offs(p.fw, (uint8_t)p.sr->idx2off(p.seedoffidx), left, lim);
		const char* read = lim ? left - (lim - 1) : left;          // the oriented read's first character
		if(read + lim != p.cs.seq) return false;                   // not the layout above
		gpu.add(reinterpret_cast<const uint8_t*>(read), (size_t)lim + p.cs.seq_len, /*seed_off*/ lim,
		        /*seed_len*/ (size_t)p.cs.n_seed_steps);
	}
	if(!gpu.searchAllSeedsDoAll(doExtend)) return false;
	for(size_t i = 0; i < n; i++) {
		const bt2x_seed_out& o = gpu.data((uint32_t)i);
		Data& d = dataVec[i];
		// searchSeedBi's per-seed reset (aligner_seed.cpp:849): the seed key (SAKey) the
		// caller's seed cache is keyed on is set here, not by the search itself
		d.resetData(paramVec[i].cs.seq, paramVec[i].cs.seq_len);
		d.bwt.topf = o.topf;                 // BwtTopBotFw (valid when need_reporting)
		d.bwt.botf = o.botf;
		d.nlex = o.nlex;
		d.need_reporting = o.need_reporting != 0;
	}
	return true;
}

// One nextAlignment() result into the caller's SwResult, as the reference's backtrace
// leaves it (aligner_swsse_ee_u8.cpp:1284-1301, aligner_sw.cpp:361-375): AlnScore (score,
// basesAligned, edits = ned().size(), ns, gaps), ned() holding the call's edit-buffer image
// trimmed to the alignment's edits (the storage the reported copies alias),
// shape and refns.  Call it after every nextAlignment(), also one that returned false
// (then only the edit buffer is written, as the reference's failed backtrace does).
template<class Res>
void to_swresult(const AlnView& v, bool ok, Res& res, size_t tidx, int64_t tlen, size_t rdlen) {
	auto& a = res.alres;
	using EditT = typename std::remove_reference<decltype(a.ned()[0])>::type;
	using ScoreT = typename std::remove_cv<typename std::remove_reference<decltype(a.score())>::type>::type;
	a.ned().clear();
	for(uint32_t e : v.image)
		a.ned().push_back(EditT(BT2X_EDIT_POS(e), BT2X_EDIT_CHR(e), BT2X_EDIT_QCHR(e), (int)BT2X_EDIT_TYPE(e)));
	if(!ok) return;
	a.ned().resize(v.edits.size());          // DList::resize = trim (ds.h:1026)
	a.setScore(ScoreT(v.score, v.bases_aligned, (int)v.edits.size(), v.ns, v.gaps));
	a.setShape(tidx, v.refoff, tlen, v.fw, rdlen, true /*pretrimSoft*/, 0, 0, true, 0, 0);
	a.setRefNs(v.refns);
}

} // namespace glue
} // namespace bt2x
