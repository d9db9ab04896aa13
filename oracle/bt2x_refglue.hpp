// bt2x_refglue.hpp — TEST INFRASTRUCTURE ONLY (oracle/ref_glue_build.py).
//
// The state INTEGRATION.md's patches need inside the reference aligner, included ahead of
// its single translation unit (bowtie2-align.cpp): one bt2x context per process, opened on
// first use with the reference's own index prefix and scoring scheme, calls serialised
// across the reference's OpenMP threads, and a SwAlignerHip per SwAligner object.  The
// patched member bodies (aligner_seed.cpp:674 searchAllSeedsDoAll; aligner_sw.cpp's
// SwAligner::initRead/initRef/align/nextAlignment and aligner_sw.h's done()) call these.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <unordered_map>

#include "bt2x_shims.hpp"
#include "bt2x_ref_glue.hpp"

namespace bt2x_refglue {

// defined after the reference's TU (they read its globals bt2index and multiseed_sc)
bt2x::Device& device();

// BT2X_GLUE_TRACE=1: one stderr line per patched call (debugging the drop-in)
inline bool trace() {
	static const bool t = std::getenv("BT2X_GLUE_TRACE") != nullptr;
	return t;
}

inline std::mutex& gpu_mutex() {
	static std::mutex m;
	return m;
}

// the GPU side of one SwAligner (keyed by its address; SwAligners live per thread)
struct Sw {
	explicit Sw(bt2x::Device& d) : swa(d) {}
	bt2x::SwAlignerHip swa;
	size_t refidx = 0;
	int64_t reflen = 0;
};
inline Sw& sw(const void* owner) {
	thread_local std::unordered_map<const void*, std::unique_ptr<Sw>> m;
	std::unique_ptr<Sw>& p = m[owner];
	if(!p) p.reset(new Sw(device()));
	return *p;
}

// The reference's Scoring as the C-ABI's (tables copied, not recomputed).
template<class Sc>
bt2x_scoring scoring_of(const Sc& sc) {
	bt2x_scoring s;
	bt2x_scoring_default(&s);
	s.mm_max = sc.mmpMax; s.mm_min = sc.mmpMin; s.n_pen = sc.npen;
	s.rdg_const = sc.rdGapConst; s.rdg_linear = sc.rdGapLinear;
	s.rfg_const = sc.rfGapConst; s.rfg_linear = sc.rfGapLinear;
	s.gapbar = sc.gapbar;
	for(int i = 0; i < 256; i++) { s.mmpens[i] = sc.mmpens[i]; s.npens[i] = sc.npens[i]; }
	return s;
}

} // namespace bt2x_refglue
