// oracle/refharness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the GPU box).
//
// Golden-vector dumper.  Compiles the reference aligner's own translation units
// in place (-I/root/reference, the same list bowtie2-align.cpp:1-38 includes,
// minus bowtie_main.cpp) and drives its hot-path classes directly:
//
//   seeds : MultiSeedResults::prepareOneSeed / instantiateSeeds
//           (aligner_seed.cpp:411), MultiSeedAligner::searchAllSeedsDoAll(true)
//           (aligner_seed.cpp:674) -> per-seed (topf, botf, need_reporting, nlex)
//   dp    : DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81),
//           SwAligner::initRead/initRef/align/nextAlignment (aligner_sw.cpp:35-375)
//           -> rectangle, reference window, E/F/H digests, sorted candidates and
//           the full sequence of nextAlignment() results with RNG state.
//   resolve : the seeds' reported BW ranges through GroupWalk2S::init/advanceElement
//           (group_walk.h:917-1005) and Ebwt::joinedToTextOff (bt2_idx.cpp:54) as
//           SwDriver::extendSeeds calls them (aligner_sw_driver.cpp:383-402), plus
//           joinedToTextOff at every fragment boundary (straddle / reject cases).
//   rank    : SeedAligner::searchAllSeedsFinalize (aligner_seed.cpp:508-540) ->
//           SeedResults::add (aligner_seed.h:603) and rankSeedHits(rnd, all)
//           (aligner_seed.h:1000-1061) with a per-(read, round) RNG seed -> rank order,
//           hit counters and the RNG state afterwards.
//
// Options (scoring, seed length, --dpad, ...) are parsed by the reference's own
// parseOptions() (bt2_search.cpp:1578) so every default is the reference's.
// Private members are opened with a preprocessor switch purely to read results.
#include <algorithm>
#include <atomic>
#include <cassert>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
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
#include <unordered_map>
#include <utility>
#include <vector>
#include <getopt.h>
#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>
#include <omp.h>
#include "../include/bt2x.h"

#define private public
#define protected public
#include "edit.cpp"
#include "ds.cpp"
#include "ccnt_lut.cpp"
#include "ref_read.cpp"
#include "alphabet.cpp"
#include "shmem.cpp"
#include "bt2_locks.cpp"
#include "bt2_idx.cpp"
#include "bt2_io.cpp"
#include "bt2_util.cpp"
#include "reference.cpp"
#include "multikey_qsort.cpp"
#include "random_source.cpp"
#include "qual.cpp"
#include "pat.cpp"
#include "sam.cpp"
#include "read_qseq.cpp"
#include "aligner_seed_policy.cpp"
#include "aligner_cache.cpp"
#include "aligner_result.cpp"
#include "ref_coord.cpp"
#include "mask.cpp"
#include "pe.cpp"
#include "aln_sink.cpp"
#include "dp_framer.cpp"
#include "scoring.cpp"
#include "presets.cpp"
#include "unique.cpp"
#include "simple_func.cpp"
#include "outq.cpp"
#ifdef ENABLE_I16
#include "aligner_swsse_ee_i16.cpp"     // the -DENABLE_I16 build (bowtie2-align.cpp:31-33)
#endif
#include "aligner_swsse_ee_u8.cpp"
#include "aligner_sw.cpp"
#include "aligner_sw_driver.cpp"
#include "aligner_seed.cpp"
#include "bt2_search.cpp"
#undef private
#undef protected

namespace harness {

struct Fq { std::string name, seq, qual; };

static bool readFq(std::istream& in, Fq& r) {
	std::string plus;
	if(!std::getline(in, r.name)) return false;
	if(!std::getline(in, r.seq)) return false;
	if(!std::getline(in, plus)) return false;
	if(!std::getline(in, r.qual)) return false;
	if(!r.name.empty() && r.name[0] == '@') r.name = r.name.substr(1);
	return true;
}

static void parseRefOptions(const std::string& idx, const std::string& reads,
                            int nextra, char** extra) {
	std::vector<const char*> av;
	av.push_back("bowtie2-align-l");
	av.push_back("-x"); av.push_back(idx.c_str());
	av.push_back("-U"); av.push_back(reads.c_str());
	for(int i = 0; i < nextra; i++) av.push_back(extra[i]);
	resetOptions();
	parseOptions((int)av.size(), av.data());
}

static Ebwt* loadEbwt(const std::string& idx) {
	Ebwt* e = new Ebwt(idx, 0, -1, true, -1, 0, false, false, false,
	                   true, true, true, true, false, false, false, false);
	e->loadIntoMemory(0, -1, true, true, true, true, false);
	return e;
}

static const char* DNA = "ACGTN";

// -------------------------------------------------------------------- seeds
static int cmdSeeds(int argc, char** argv) {
	if(argc < 4) { fprintf(stderr, "seeds <idx> <reads.fq> <out> [bt2 opts]\n"); return 2; }
	std::string idx = argv[1], fq = argv[2], out = argv[3];
	parseRefOptions(idx, fq, argc - 4, argv + 4);
	Ebwt* ebwt = loadEbwt(idx);
	FILE* fo = fopen(out.c_str(), "w");
	fprintf(fo, "# seeds idx=%s reads=%s seedlen=%d rounds=%d\n", idx.c_str(), fq.c_str(),
	        (int)multiseedLen, (int)nSeedRounds);
	MultiSeedResults srs(1, multiseedLen, gNofw, gNorc);
	MultiSeedAligner als(ebwt, srs);
	std::ifstream in(fq);
	Fq r; size_t ridx = 0, nseeds = 0;
	while(readFq(in, r)) {
		Read rd(r.name.c_str(), r.seq.c_str(), r.qual.c_str());
		const size_t rdlen = rd.length();
		size_t myidx = ridx++;
		if(rdlen >= 256 || rdlen < 1) continue;      // bt2_search.cpp:2495 (rdlen<256)
		const int interval = std::max((int)msIval.f<int>((double)rdlen), 1);
		const uint32_t nrounds = std::min<uint16_t>(nSeedRounds, interval);
		for(uint32_t roundi = 0; roundi < nrounds; roundi++) {
			const uint32_t offset = (interval * roundi) / nrounds;
			if(offset > 0 && multiseedLen + offset > rdlen) break;   // bt2_search.cpp:2575
			srs.clearSeeds();
			srs.prepareOneSeed(0, offset, interval, &rd);
			Read* rds[1] = { &rd };
			srs.instantiateSeeds(rds);
			als.reserveBuffers();
			als.prepareSearchAllSeedsOne(0);
			als.searchAllSeedsDoAll(true);
			for(size_t k = 0; k < als._bufVec_filled; k++) {
				const SeedAlignerSearchParams& p = als._paramVec[k];
				const SeedAlignerSearchData& d = als._dataVec[k];
				const char* base = p.fw ? rd.patFw.buf() : rd.patRc.buf();
				long seqoff = (long)(p.cs.seq - base);
				fprintf(fo, "S %zu %u %d %d %ld %d %llu %llu %d %d\n", myidx, roundi,
				        (int)p.fw, (int)p.seedoffidx, seqoff, (int)p.cs.n_seed_steps,
				        (unsigned long long)d.bwt.topf, (unsigned long long)d.bwt.botf,
				        (int)d.need_reporting, (int)d.nlex);
				nseeds++;
			}
		}
	}
	fclose(fo);
	fprintf(stderr, "seeds: %zu reads, %zu seed searches\n", ridx, nseeds);
	return 0;
}

// ----------------------------------------------------------------------- dp
// Order-independent digest of one matrix: sum of bt2x_cell_digest over cells of the
// stored value (u8: the byte; i16: the int16 bit pattern).
template<bool kI16>
static uint64_t digestMat(const SSEMatrix<kI16, ALN_MAX_ROWS, ALN_MAX_COLS>& m,
                          size_t nrow, size_t ncol, int mat) {
	uint64_t h = 0;
	for(size_t i = 0; i < nrow; i++)
		for(size_t j = 0; j < ncol; j++)
			h += bt2x_cell_digest((uint32_t)i, (uint32_t)j, (uint32_t)mat,
			                      (uint32_t)(m.elt(i, j, mat) & (kI16 ? 0xffff : 0xff)));
	return h;
}

// Read names of simulated reads: "<anything>:<refidx>:<off>:<fw>"; off = leftmost
// reference offset of the read's true alignment, fw = 1 if forward strand.
static bool parseOrigin(const std::string& nm, long& tidx, long& off, int& fw) {
	std::vector<std::string> f; std::string cur;
	for(char c : nm) { if(c == ':' || c == ' ') { f.push_back(cur); cur.clear(); } else cur += c; }
	f.push_back(cur);
	if(f.size() < 4) return false;
	tidx = atol(f[f.size()-3].c_str()); off = atol(f[f.size()-2].c_str()); fw = atoi(f.back().c_str());
	return true;
}

static int cmdDp(int argc, char** argv) {
	if(argc < 5) { fprintf(stderr, "dp <idx> <reads.fq> <out> <seed> [bt2 opts]\n"); return 2; }
	std::string idx = argv[1], fq = argv[2], out = argv[3];
	uint32_t seed = (uint32_t)atol(argv[4]);
	parseRefOptions(idx, fq, argc - 5, argv + 5);
	Ebwt* ebwt = loadEbwt(idx);
	BitPairReference ref(idx, false, false, NULL, NULL, false, false, false, false, false, false);
	if(!ref.loaded()) { fprintf(stderr, "reference not loaded\n"); return 1; }
	Scoring sc(bonusMatch, penMmcType, penMmcMax, penMmcMin, scoreMin, nCeil, penNType, penN,
	           penNCatPair, penRdGapConst, penRfGapConst, penRdGapLinear, penRfGapLinear, gGapBarrier);
	FILE* fo = fopen(out.c_str(), "w");
	fprintf(fo, "# dp idx=%s reads=%s maxhalf=%zu gapbar=%d mmp=%d,%d np=%d rdg=%d,%d rfg=%d,%d sse8=%d\n",
	        idx.c_str(), fq.c_str(), (size_t)maxhalf, (int)gGapBarrier, (int)penMmcMax, (int)penMmcMin,
	        (int)penN, (int)penRdGapConst, (int)penRdGapLinear, (int)penRfGapConst, (int)penRfGapLinear,
	        (int)enable8);
	SwAligner* swap = new SwAligner();
	SwAligner& swa = *swap;
	RandomSource jrnd; jrnd.init(seed);
	std::ifstream in(fq);
	Fq r; size_t ridx = 0, nprob = 0;
	DynProgFramer dpframe(!gReportOverhangs);
	while(readFq(in, r)) {
		size_t myidx = ridx++;
		long tidx, off; int fwTrue;
		if(!parseOrigin(r.name, tidx, off, fwTrue)) continue;
		Read rd(r.name.c_str(), r.seq.c_str(), r.qual.c_str());
		const size_t rdlen = rd.length();
		if(rdlen >= 256 || rdlen < 2) continue;
		TAlScore minsc = scoreMin.f<TAlScore>((double)rdlen);
		if(minsc > 0) minsc = 0;
#ifndef ENABLE_I16
		if(minsc < -254) minsc = -254;             // bt2_search.cpp:2484-2492
#endif
		int nceil = std::min((int)nCeil.f<int>((double)rdlen), (int)rdlen);
		swa.reset();
		if(!swa.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, rdlen, sc)) {
			fprintf(fo, "R %zu initRead-fail %zu\n", myidx, rdlen);
			continue;
		}
		const int64_t tlen = (int64_t)ebwt->plen()[tidx];
		// Diagonals: the true one, small shifts, band-edge shifts and one on the
		// opposite strand, the way distinct seed hits reach extendSeeds.
		std::vector<std::pair<long,int> > probs;
		probs.push_back(std::make_pair(off, fwTrue));
		probs.push_back(std::make_pair(off + 1 + (long)(jrnd.nextU32() % 4), fwTrue));
		probs.push_back(std::make_pair(off - 1 - (long)(jrnd.nextU32() % 16), fwTrue));
		if(jrnd.nextU32() % 4 == 0) probs.push_back(std::make_pair(off, 1 - fwTrue));
		for(size_t pi = 0; pi < probs.size(); pi++) {
			int64_t refoff = probs[pi].first;
			bool fw = probs[pi].second != 0;
			int readGaps = sc.maxReadGaps(minsc, rdlen);
			int refGaps  = sc.maxRefGaps(minsc, rdlen);
			DPRect rect;
			bool found = dpframe.frameSeedExtensionRect(refoff, rdlen, tlen, readGaps, refGaps,
			                                            (size_t)nceil, maxhalf, rect);
			if(!found) { fprintf(fo, "F %zu %ld %d frame-trimmed\n", myidx, (long)refoff, (int)fw); continue; }
			size_t nwindow = 0;
			if(refoff >= rect.refl) nwindow = (size_t)(refoff - rect.refl);
			size_t nsInLeftShift = 0;
			swa.reset();
			swa.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, rdlen, sc);
			bool okRef = swa.initRef(fw, (TRefId)tidx, rect, ref, tlen, minsc, enable8, true,
			                         nwindow, nsInLeftShift);
			if(!okRef) { fprintf(fo, "F %zu %ld %d initRef-fail\n", myidx, (long)refoff, (int)fw); continue; }
			std::string win;
			for(size_t i = 0; i < swa.rflen_; i++) win += DNA[firsts5[(int)swa.rf_[i]]];
			uint32_t rseed = jrnd.nextU32();
			// the P line's last field: 1 when the problem runs the i16 kernel (enable8_ false)
#ifdef ENABLE_I16
			const bool useI16 = !swa.enable8_;
#else
			const bool useI16 = false;
#endif
			fprintf(fo, "P %zu %zu %d %s %s %s %lld %lld %zu %zu %zu %lld %d %u %lld %ld %lld %d\n", nprob, myidx, (int)fw,
			        r.seq.c_str(), r.qual.c_str(), win.c_str(), (long long)rect.refl, (long long)rect.refr,
			        (size_t)rect.triml, (size_t)rect.corel, (size_t)rect.corer, (long long)minsc, nceil, rseed,
			        (long long)refoff, tidx, (long long)tlen, (int)useI16);
			nprob++;
			TAlScore best = std::numeric_limits<TAlScore>::min();
			bool ok = swa.align(best);
			uint64_t dg[3];
			for(int mat = 0; mat < 3; mat++) {
#ifdef ENABLE_I16
				if(useI16) { dg[mat] = digestMat((fw ? swa.sseI16fw_ : swa.sseI16rc_).mat_, rdlen, swa.rflen_, mat); continue; }
#endif
				dg[mat] = digestMat((fw ? swa.sseU8fw_ : swa.sseU8rc_).mat_, rdlen, swa.rflen_, mat);
			}
			fprintf(fo, "A %d %lld %zu %016llx %016llx %016llx\n", (int)ok, (long long)best,
			        (size_t)swa.btncand_.size(), (unsigned long long)dg[SSEMatrixConsts::E],
			        (unsigned long long)dg[SSEMatrixConsts::F], (unsigned long long)dg[SSEMatrixConsts::H]);
			fprintf(fo, "C");
			for(size_t c = 0; c < swa.btncand_.size(); c++)
				fprintf(fo, " %zu,%zu,%lld", swa.btncand_[c].row, swa.btncand_[c].col,
				        (long long)swa.btncand_[c].score);
			fprintf(fo, "\n");
			if(ok) {
				RandomSource rnd; rnd.init(rseed);
				SwResult res;
				while(!swa.done()) {
					res.reset();
					swa.nextAlignment(res, minsc, rnd);
					if(res.empty()) { fprintf(fo, "N 0 %u\n", rnd.last); break; }
					AlnRes& a = res.alres;
					fprintf(fo, "N 1 %u %lld %lld %lld %d %d %lld %zu %zu", rnd.last,
					        (long long)a.score_.score_, (long long)a.score_.ns_, (long long)a.score_.gaps_,
					        a.score_.edits_, a.score_.basesAligned_, (long long)a.refcoord_.off(),
					        (size_t)a.refns_, (size_t)a.ned_.size());
					for(size_t e = 0; e < a.ned_.size(); e++) {
						const Edit& ed = a.ned_[e];
						fprintf(fo, " %u,%d,%c,%c", ed.pos, (int)ed.type, (char)ed.chr, (char)ed.qchr);
					}
					fprintf(fo, "\n");
				}
			}
			fprintf(fo, "E\n");
		}
	}
	fclose(fo);
	fprintf(stderr, "dp: %zu reads, %zu problems\n", ridx, nprob);
	delete swap;
	return 0;
}


// ------------------------------------------------------------------ resolve
static void printJ(FILE* fo, const Ebwt* ebwt, TIndexOffU qlen, TIndexOffU off) {
	for(int rej = 0; rej < 2; rej++) {
		TIndexOffU tidx = 0, toff = 0, tlen = 0;      // zero-initialised like the caller
		bool straddled = false;
		ebwt->joinedToTextOff(qlen, off, tidx, toff, tlen, rej != 0, straddled);
		fprintf(fo, " %lld %llu %llu %d", tidx == OFF_MASK ? -1LL : (long long)tidx,
		        (unsigned long long)toff, (unsigned long long)tlen, (int)straddled);
	}
}

static int cmdResolve(int argc, char** argv) {
	if(argc < 4) { fprintf(stderr, "resolve <idx> <reads.fq> <out> [bt2 opts]\n"); return 2; }
	std::string idx = argv[1], fq = argv[2], out = argv[3];
	parseRefOptions(idx, fq, argc - 4, argv + 4);
	Ebwt* ebwt = loadEbwt(idx);
	BitPairReference ref(idx, false, false, NULL, NULL, false, false, false, false, false, false);
	if(!ref.loaded()) { fprintf(stderr, "reference not loaded\n"); return 1; }
	FILE* fo = fopen(out.c_str(), "w");
	if(getenv("HARNESS_UNBUF")) setvbuf(fo, NULL, _IONBF, 0);
	fprintf(fo, "# resolve idx=%s reads=%s len=%llu nfrag=%llu offrate=%d\n", idx.c_str(), fq.c_str(),
	        (unsigned long long)ebwt->_eh._len, (unsigned long long)ebwt->_nFrag, (int)ebwt->_eh._offRate);
	// fragment boundaries: J off qlen  {tidx toff tlen straddled} x {keep, reject}
	const TIndexOffU nf = ebwt->_nFrag, len = ebwt->_eh._len;
	size_t nj = 0;
	for(TIndexOffU f = 0; f < nf && f < 400; f++) {
		const TIndexOffU lower = ebwt->rstarts()[f * 3];
		const TIndexOffU upper = f + 1 == nf ? len : ebwt->rstarts()[(f + 1) * 3];
		const TIndexOffU qls[3] = {1, (TIndexOffU)multiseedLen, 100};
		for(int q = 0; q < 3; q++) {
			const TIndexOffU ql = qls[q];
			std::set<TIndexOffU> offs;
			offs.insert(lower); offs.insert(lower + 1); offs.insert(upper - 1);
			if(upper >= ql) { offs.insert(upper - ql); offs.insert(upper - ql + 1); }
			if(upper >= ql + 1) offs.insert(upper - ql - 1);
			for(TIndexOffU o : offs) {
				if(o < lower || o >= upper) continue;
				fprintf(fo, "J %llu %llu", (unsigned long long)o, (unsigned long long)ql);
				printJ(fo, ebwt, ql, o);
				fprintf(fo, "\n");
				nj++;
			}
		}
	}
	// seed ranges through GroupWalk2S
	MultiSeedResults srs(1, multiseedLen, gNofw, gNorc);
	MultiSeedAligner als(ebwt, srs);
	GroupWalkState gwstate(GW_CAT);
	PerReadMetrics prm;
	RandomSource rnd; rnd.init(7);
	std::ifstream in(fq);
	Fq r; size_t ridx = 0, nw = 0;
	while(readFq(in, r)) {
		Read rd(r.name.c_str(), r.seq.c_str(), r.qual.c_str());
		const size_t rdlen = rd.length();
		size_t myidx = ridx++;
		if(rdlen >= 256 || rdlen < 1) continue;
		const int interval = std::max((int)msIval.f<int>((double)rdlen), 1);
		const uint32_t nrounds = std::min<uint16_t>(nSeedRounds, interval);
		for(uint32_t roundi = 0; roundi < nrounds; roundi++) {
			const uint32_t offset = (interval * roundi) / nrounds;
			if(offset > 0 && multiseedLen + offset > rdlen) break;
			srs.clearSeeds();
			srs.prepareOneSeed(0, offset, interval, &rd);
			Read* rds[1] = { &rd };
			srs.instantiateSeeds(rds);
			als.reserveBuffers();
			als.prepareSearchAllSeedsOne(0);
			als.searchAllSeedsDoAll(true);
			for(size_t k = 0; k < als._bufVec_filled; k++) {
				const SeedAlignerSearchParams& p = als._paramVec[k];
				const SeedAlignerSearchData& d = als._dataVec[k];
				if(!d.need_reporting) continue;
				const TIndexOffU topf = d.bwt.topf, sz = d.bwt.botf - d.bwt.topf;
				if(sz == 0) continue;
				const size_t klen = (size_t)p.cs.n_seed_steps;
				fprintf(fo, "G %zu %u %d %d %llu %llu %zu\n", myidx, roundi, (int)p.fw, (int)p.seedoffidx,
				        (unsigned long long)topf, (unsigned long long)d.bwt.botf, klen);
				if(sz <= (TIndexOffU)TStateVSize) {
					// GroupWalk2S keeps its walk states in a fixed DList of TStateVSize (6)
					// (group_walk.h:92, :900); a range of n elements creates at most n
					// states, so ranges of <= 6 elements walk safely.  Larger ranges can
					// overflow it (st.expand(), group_walk.h:762, writes past the DList
					// into hit_) -- for them the W record is Ebwt::getOffset(row), the
					// value group_walk.h:425-432 asserts the walk produces.
					// A cache slice pair as AlignmentCache::queryQval makes (aligner_cache.h:636-644)
					EList<TIndexOffU> salist;
					salist.resize(2 * sz);
					TSlice offs(salist, 0, sz), fmap(salist, sz, sz);
					offs.fill(OFF_MASK); fmap.fill(OFF_MASK);
					SARangeWithOffs<TSlice> sa(topf, klen, offs, fmap);
					GroupWalk2S<TSlice> gw;
					gw.init(*ebwt, ref, sa, rnd);
					for(TIndexOffU e = 0; e < sz; e++) {
						WalkResult wr;
						gw.advanceElement(e, *ebwt, ref, sa, gwstate, wr, prm);
						fprintf(fo, "W %llu %llu %llu %llu", (unsigned long long)wr.elt.elt,
						        (unsigned long long)wr.bwrow, (unsigned long long)wr.toff,
						        (unsigned long long)wr.elt.len);
						printJ(fo, ebwt, wr.elt.len, wr.toff);
						fprintf(fo, "\n");
						nw++;
					}
				} else {
					const TIndexOffU step = sz <= 8 ? 1 : sz / 8;
					for(TIndexOffU e = 0; e < sz; e += step) {
						const TIndexOffU row = topf + e, toff = ebwt->getOffset(row);
						fprintf(fo, "V %llu %llu %llu %llu", (unsigned long long)e, (unsigned long long)row,
						        (unsigned long long)toff, (unsigned long long)klen);
						printJ(fo, ebwt, klen, toff);
						fprintf(fo, "\n");
						nw++;
					}
				}
			}
		}
	}
	fclose(fo);
	fprintf(stderr, "resolve: %zu reads, %zu walk results, %zu boundary probes\n", ridx, nw, nj);
	return 0;
}

// --------------------------------------------------------------------- rank
static void printRank(FILE* fo, const char* tag, size_t ridx, uint32_t roundi, uint32_t seed,
                      const SeedResults& sr, const RandomSource& rnd) {
	fprintf(fo, "%s %zu %u %u %u %zu %zu %zu %zu %zu %zu %zu %zu %u", tag, ridx, roundi, seed,
	        (unsigned)sr.numOffs_, (size_t)sr.nonzTot_, (size_t)sr.nonzFw_, (size_t)sr.nonzRc_, (size_t)sr.numElts_,
	        (size_t)sr.numEltsFw_, (size_t)sr.numEltsRc_, (size_t)sr.uniTot_, (size_t)sr.repTot_,
	        rnd.last);
	for(size_t r = 0; r < sr.rankOffs_.size(); r++) {
		uint32_t offidx = 0, off = 0, seedlen = 0; bool fw = true;
		const QVal& qv = sr.hitsByRank(r, offidx, off, fw, seedlen);
		fprintf(fo, " %u,%d,%llu", offidx, (int)fw, (unsigned long long)qv.numElts());
	}
	fprintf(fo, "\n");
}

static int cmdRank(int argc, char** argv) {
	if(argc < 4) { fprintf(stderr, "rank <idx> <reads.fq> <out> [bt2 opts]\n"); return 2; }
	std::string idx = argv[1], fq = argv[2], out = argv[3];
	parseRefOptions(idx, fq, argc - 4, argv + 4);
	Ebwt* ebwt = loadEbwt(idx);
	FILE* fo = fopen(out.c_str(), "w");
	fprintf(fo, "# rank idx=%s reads=%s seedlen=%d rounds=%d\n", idx.c_str(), fq.c_str(),
	        (int)multiseedLen, (int)nSeedRounds);
	MultiSeedResults srs(1, multiseedLen, gNofw, gNorc);
	MultiSeedAligner als(ebwt, srs);
	std::ifstream in(fq);
	Fq r; size_t ridx = 0, nk = 0;
	while(readFq(in, r)) {
		Read rd(r.name.c_str(), r.seq.c_str(), r.qual.c_str());
		const size_t rdlen = rd.length();
		size_t myidx = ridx++;
		if(rdlen >= 256 || rdlen < 1) continue;
		const int interval = std::max((int)msIval.f<int>((double)rdlen), 1);
		const uint32_t nrounds = std::min<uint16_t>(nSeedRounds, interval);
		for(uint32_t roundi = 0; roundi < nrounds; roundi++) {
			const uint32_t offset = (interval * roundi) / nrounds;
			if(offset > 0 && multiseedLen + offset > rdlen) break;
			srs.clearSeeds();
			srs.prepareOneSeed(0, offset, interval, &rd);
			Read* rds[1] = { &rd };
			srs.instantiateSeeds(rds);
			als.reserveBuffers();
			als.prepareSearchAllSeedsOne(0);
			als.searchAllSeedsDoAll(true);
			SeedResults& sr = srs.getSR(0);
			als._als[0].searchAllSeedsFinalize(als.getCache(0), sr);
			if(sr.nonzeroOffsets() == 0) { fprintf(fo, "Z %zu %u\n", myidx, roundi); continue; }
			const uint32_t seed = (uint32_t)(myidx * 2654435761u + roundi * 97u + 1u);
			RandomSource rnd; rnd.init(seed);
			sr.rankSeedHits(rnd, false);
			printRank(fo, "K", myidx, roundi, seed, sr, rnd);
			sr.rankOffs_.clear(); sr.rankFws_.clear();
			sr.rankSeedHits(rnd, true);
			printRank(fo, "A", myidx, roundi, seed, sr, rnd);
			nk++;
		}
	}
	fclose(fo);
	fprintf(stderr, "rank: %zu reads, %zu ranked rounds\n", ridx, nk);
	return 0;
}

// -------------------------------------------------------------------- bench
// CPU baseline for bench.py: the reference's own hot path, OpenMP-parallel the way
// bt2_search.cpp drives it, over a FASTQ sample whose names carry the true origin.
//   seeds: batches of 4096 reads -> prepareOneSeed (round 0) -> instantiateSeeds ->
//          prepareSearchAllSeedsOne -> searchAllSeedsDoAll(extend)   (bt2_search.cpp:2572-2640)
//   dp:    omp parallel over reads, one SwAligner per thread: frameSeedExtensionRect at
//          the true origin, initRead, initRef, align, nextAlignment until done
//          (SwDriver::extendSeeds' per-DP sequence, aligner_sw_driver.cpp:481-538)
// Only the two compute phases are timed.
static double nowSec() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }

static int cmdBench(int argc, char** argv) {
	if(argc < 3) { fprintf(stderr, "bench <idx> <reads.fq> [bt2 opts]\n"); return 2; }
	std::string idx = argv[1], fq = argv[2];
	parseRefOptions(idx, fq, argc - 3, argv + 3);
	Ebwt* ebwt = loadEbwt(idx);
	BitPairReference ref(idx, false, false, NULL, NULL, false, false, false, false, false, false);
	if(!ref.loaded()) { fprintf(stderr, "reference not loaded\n"); return 1; }
	Scoring sc(bonusMatch, penMmcType, penMmcMax, penMmcMin, scoreMin, nCeil, penNType, penN,
	           penNCatPair, penRdGapConst, penRfGapConst, penRdGapLinear, penRfGapLinear, gGapBarrier);
	std::vector<Read*> reads; std::vector<long> tids, offs; std::vector<int> fws;
	{
		std::ifstream in(fq); Fq r;
		while(readFq(in, r)) {
			long tidx, off; int fw;
			if(!parseOrigin(r.name, tidx, off, fw)) continue;
			Read* rd = new Read(r.name.c_str(), r.seq.c_str(), r.qual.c_str());
			if(rd->length() < 2 || rd->length() >= 256) { delete rd; continue; }
			reads.push_back(rd); tids.push_back(tidx); offs.push_back(off); fws.push_back(fw);
		}
	}
	const size_t n = reads.size();
	const int nthr = omp_get_max_threads();
	// ---- seeds
	const uint32_t B = 4096;
	MultiSeedResults srs(B, multiseedLen, gNofw, gNorc);
	MultiSeedAligner als(ebwt, srs);
	std::vector<const Read*> rds(B);
	size_t nseeds = 0;
	double t0 = nowSec();
	for(size_t b0 = 0; b0 < n; b0 += B) {
		const uint32_t m = (uint32_t)std::min<size_t>(B, n - b0);
		srs.clearSeeds();
		for(uint32_t k = 0; k < B; k++) {
			const Read* rd = reads[b0 + std::min<uint32_t>(k, m - 1)];
			rds[k] = rd;
			if(k < m) {
				const int interval = std::max((int)msIval.f<int>((double)rd->length()), 1);
				srs.prepareOneSeed(k, 0, interval, rd);
			}
		}
		srs.instantiateSeeds(rds.data());
		als.reserveBuffers();
#pragma omp parallel for schedule(dynamic, 64)
		for(uint32_t k = 0; k < m; k++) als.prepareSearchAllSeedsOne(k);
		als.searchAllSeedsDoAll(true);
		nseeds += als._bufVec_filled;
	}
	const double tSeed = nowSec() - t0;
	// ---- dp
	size_t nprob = 0, naln = 0;
	t0 = nowSec();
#pragma omp parallel reduction(+:nprob,naln)
	{
		SwAligner* swa = new SwAligner();
		DynProgFramer dpframe(!gReportOverhangs);
#pragma omp for schedule(dynamic, 64)
		for(size_t i = 0; i < n; i++) {
			const Read& rd = *reads[i];
			const size_t rdlen = rd.length();
			TAlScore minsc = scoreMin.f<TAlScore>((double)rdlen);
			if(minsc > 0) minsc = 0;
			if(minsc < -254) minsc = -254;
			const int nceil = std::min((int)nCeil.f<int>((double)rdlen), (int)rdlen);
			const int64_t tlen = (int64_t)ebwt->plen()[tids[i]];
			DPRect rect;
			if(!dpframe.frameSeedExtensionRect(offs[i], rdlen, tlen, sc.maxReadGaps(minsc, rdlen),
			                                   sc.maxRefGaps(minsc, rdlen), (size_t)nceil, maxhalf, rect)) continue;
			const size_t nwindow = offs[i] >= rect.refl ? (size_t)(offs[i] - rect.refl) : 0;
			size_t nsInLeftShift = 0;
			swa->reset();
			if(!swa->initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, rdlen, sc)) continue;
			if(!swa->initRef(fws[i] != 0, (TRefId)tids[i], rect, ref, tlen, minsc, true, true,
			                 nwindow, nsInLeftShift)) continue;
			nprob++;
			TAlScore best = std::numeric_limits<TAlScore>::min();
			if(!swa->align(best)) continue;
			RandomSource rnd; rnd.init((uint32_t)i * 2654435761u + 1);
			SwResult res;
			while(!swa->done()) {
				res.reset();
				swa->nextAlignment(res, minsc, rnd);
				if(res.empty()) break;
				naln++;
			}
		}
		delete swa;
	}
	const double tDp = nowSec() - t0;
	printf("BENCH threads=%d reads=%zu seeds=%zu seed_s=%.6f dp_probs=%zu dp_alns=%zu dp_s=%.6f\n",
	       nthr, n, nseeds, tSeed, nprob, naln, tDp);
	for(Read* r : reads) delete r;
	delete ebwt;
	return 0;
}

} // namespace harness

int main(int argc, char** argv) {
	if(argc < 2) { fprintf(stderr, "usage: refharness seeds|dp ...\n"); return 2; }
	std::string cmd = argv[1];
	try {
		if(cmd == "seeds") return harness::cmdSeeds(argc - 1, argv + 1);
		if(cmd == "dp") return harness::cmdDp(argc - 1, argv + 1);
		if(cmd == "bench") return harness::cmdBench(argc - 1, argv + 1);
		if(cmd == "resolve") return harness::cmdResolve(argc - 1, argv + 1);
		if(cmd == "rank") return harness::cmdRank(argc - 1, argv + 1);
	} catch(int e) {
		fprintf(stderr, "reference threw %d\n", e);
		return 1;
	}
	fprintf(stderr, "unknown command %s\n", cmd.c_str());
	return 2;
}
