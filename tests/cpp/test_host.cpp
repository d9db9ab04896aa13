// test_host.cpp — host-side logic of include/bt2x_shims.hpp that needs no GPU, driven
// with the reference's own recorded inputs and printed in the golden file's format.
//
//   test_host rank <seeds.txt> <rank.txt>
//       seeds.txt = refharness "seeds" records (per-seed kernel outputs: topf, botf,
//       need_reporting, nlex); rank.txt = refharness "rank" records, used only for each
//       round's numOffs and RNG seed.  For every ranked round: SeedHitsHip::add over the
//       round's seeds (searchAllSeedsFinalize order), rankSeedHits(rnd, false) -> "K"
//       line, then rankSeedHits(rnd, true) -> "A" line (same format as the golden).
// tests/test_host_logic.py compares the output with tests/golden/rank_rep.txt.xz.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "bt2x_shims.hpp"

namespace {

struct Rng {                        // RandomSource (random_source.h:34-105)
	uint32_t a = 1664525, c = 1013904223, last = 0;
	int lastOff = 30;
	void init(uint32_t s) { last = s; lastOff = 30; }
	uint32_t nextU32() { last = a * last + c; uint32_t r = last >> 16; last = a * last + c; lastOff = 0; return r ^ last; }
	bool nextBool() {
		if(lastOff > 31) nextU32();
		const uint32_t r = (last >> lastOff) & 1;
		lastOff++;
		return r != 0;
	}
};

struct SeedRec { int fw; uint32_t idx; bt2x_seed_out d; };

void print(const char* tag, size_t ridx, uint32_t round, uint32_t seed, const bt2x::SeedHitsHip& h, const Rng& rnd) {
	printf("%s %zu %u %u %zu %zu %zu %zu %llu %llu %llu %zu %zu %u", tag, ridx, round, seed, h.numOffs(),
	       h.nonzeroOffsets(), h.nonzFw(), h.nonzRc(), (unsigned long long)h.numElts(),
	       (unsigned long long)h.numEltsFw(), (unsigned long long)h.numEltsRc(), h.uniTot(), h.repTot(), rnd.last);
	for(size_t r = 0; r < h.ranked(); r++) {
		uint32_t offidx = 0; bool fw = true;
		const auto& hit = h.hitsByRank(r, offidx, fw);
		printf(" %u,%d,%llu", offidx, (int)fw, (unsigned long long)hit.numElts());
	}
	printf("\n");
}

int rank_mode(const char* seeds_path, const char* rank_path) {
	std::map<std::pair<size_t, uint32_t>, std::vector<SeedRec>> seeds;
	{
		std::ifstream in(seeds_path);
		std::string line;
		while(std::getline(in, line)) {
			if(line.empty() || line[0] != 'S') continue;
			std::istringstream ss(line.substr(2));
			size_t ridx; uint32_t round; int fw; uint32_t idx; long seqoff; int nsteps;
			unsigned long long topf, botf; int rep, nlex;
			if(!(ss >> ridx >> round >> fw >> idx >> seqoff >> nsteps >> topf >> botf >> rep >> nlex)) return 2;
			SeedRec r;
			std::memset(&r.d, 0, sizeof(r.d));
			r.fw = fw; r.idx = idx;
			r.d.topf = topf; r.d.botf = botf; r.d.need_reporting = (uint8_t)rep; r.d.nlex = (uint8_t)nlex;
			seeds[{ridx, round}].push_back(r);
		}
	}
	std::ifstream in(rank_path);
	std::string line;
	bt2x::SeedHitsHip h;
	while(std::getline(in, line)) {
		if(line.empty() || line[0] != 'K') continue;
		std::istringstream ss(line.substr(2));
		size_t ridx; uint32_t round, seed, numOffs;
		if(!(ss >> ridx >> round >> seed >> numOffs)) return 2;
		h.reset(numOffs);
		// searchAllSeedsFinalize: fw seeds first, then rc, each in seed-index order
		for(int fwi = 0; fwi < 2; fwi++)
			for(const SeedRec& r : seeds[{ridx, round}])
				if((r.fw != 0) == (fwi == 0)) h.add(r.idx, r.fw != 0, r.d);
		Rng rnd; rnd.init(seed);
		h.rankSeedHits(rnd, false);
		print("K", ridx, round, seed, h, rnd);
		h.reset(numOffs);
		for(const SeedRec& r : seeds[{ridx, round}]) h.add(r.idx, r.fw != 0, r.d);
		h.rankSeedHits(rnd, true);
		print("A", ridx, round, seed, h, rnd);
	}
	return 0;
}

} // namespace

int main(int argc, char** argv) {
	if(argc >= 4 && std::string(argv[1]) == "rank") return rank_mode(argv[2], argv[3]);
	fprintf(stderr, "usage: test_host rank <seeds.txt> <rank.txt>\n");
	return 2;
}
