// test_shims.cpp — drives include/bt2x_shims.hpp the way the reference's SwDriver drives
// SwAligner, with minimal stand-ins for the reference's types (same member names), and
// prints results in the golden file's own record format (oracle/refharness.cpp "dp"):
//   A ok best ncand / N 1 rnd score ns gaps nedit bases refoff refns nedit edits... / N 0 rnd
// tests/test_gpu_parity.py compares the output with tests/golden/dp_rep*.txt.xz.
//
// usage: test_shims <index basename> <problems.txt> <batch|single> [gapbar mm_max mm_min np rdg_c rdg_l rfg_c rfg_l
//                   [sse8]]
// problems.txt lines: fw seq qual win refl refr triml corel corer minsc nceil rseed tlen
// Built twice: test_shims (the stock build) and test_shims_i16 (-DENABLE_I16: the shims then
// pick the i16 kernel as SwAligner::initRef does, aligner_sw.cpp:77-83; sse8 0 = --no-sse8).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "bt2x_shims.hpp"

namespace {

int code(char c) {
	switch(c) { case 'A': case 'a': return 0; case 'C': case 'c': return 1; case 'G': case 'g': return 2;
	            case 'T': case 't': return 3; default: return 4; }
}

struct DnaStr {                     // BTDnaString stand-in: codes, operator[], length()
	std::vector<uint8_t> v;
	size_t length() const { return v.size(); }
	int operator[](size_t i) const { return v[i]; }
};
struct QualStr {                    // BTString stand-in
	std::string s;
	size_t length() const { return s.size(); }
	char operator[](size_t i) const { return s[i]; }
};
struct SimpleFuncStub { int v; template<class T> T f(double) const { return (T)v; } };
struct ScoringStub { SimpleFuncStub nCeil; };
struct RectStub { int64_t refl, refr; size_t triml, corel, corer; };
struct WindowRefs {                 // BitPairReference stand-in: knows only the DP window
	int64_t refl; std::string win;
	int getBase(size_t, size_t off) const {
		const int64_t k = (int64_t)off - refl;
		return (k >= 0 && k < (int64_t)win.size()) ? code(win[(size_t)k]) : 4;
	}
};
struct Rng {                        // RandomSource (random_source.h:46-61)
	uint32_t a = 1664525, c = 1013904223, last = 0;
	void init(uint32_t s) { last = s; }
	uint32_t nextU32() { last = a * last + c; uint32_t r = last >> 16; last = a * last + c; return r ^ last; }
};

struct Prob {
	int fw; std::string seq, qual, win; int64_t refl, refr; size_t triml, corel, corer;
	int64_t minsc; int nceil; uint32_t rseed; int64_t tlen;
};

void print_result(FILE* fo, bt2x::SwBatch& b, int pid, const Prob& p, Rng& rnd) {
	int64_t best = 0;
	const bool ok = b.align(pid, best);
	fprintf(fo, "A %d %lld %u\n", (int)ok, (long long)best, (unsigned)b.out(pid).ncand);
	if(!ok) return;
	bt2x::AlnView res;
	while(!b.done(pid)) {
		if(!b.nextAlignment(pid, res, rnd)) { fprintf(fo, "N 0 %u\n", rnd.last); break; }
		fprintf(fo, "N 1 %u %d %d %d %d %d %lld %d %zu", rnd.last, res.score, res.ns, res.gaps,
		        (int)res.edits.size(), res.bases_aligned, (long long)res.refoff, res.refns, res.edits.size());
		for(uint32_t e : res.edits)
			fprintf(fo, " %u,%u,%c,%c", BT2X_EDIT_POS(e), BT2X_EDIT_TYPE(e), BT2X_EDIT_CHR(e), BT2X_EDIT_QCHR(e));
		fprintf(fo, "\n");
	}
	(void)p;
}

} // namespace

int main(int argc, char** argv) {
	if(argc < 4) { fprintf(stderr, "usage: test_shims <idx> <problems.txt> batch|single [scoring]\n"); return 2; }
	std::vector<Prob> probs;
	{
		std::ifstream in(argv[2]);
		std::string line;
		while(std::getline(in, line)) {
			std::istringstream ss(line);
			Prob p;
			if(ss >> p.fw >> p.seq >> p.qual >> p.win >> p.refl >> p.refr >> p.triml >> p.corel >> p.corer
			      >> p.minsc >> p.nceil >> p.rseed >> p.tlen) probs.push_back(p);
		}
	}
	bt2x_scoring sc;
	bt2x_scoring_default(&sc);
	if(argc >= 12) {
		sc.gapbar = atoi(argv[4]); sc.mm_max = atoi(argv[5]); sc.mm_min = atoi(argv[6]); sc.n_pen = atoi(argv[7]);
		sc.rdg_const = atoi(argv[8]); sc.rdg_linear = atoi(argv[9]); sc.rfg_const = atoi(argv[10]); sc.rfg_linear = atoi(argv[11]);
		bt2x_scoring_init(&sc);
	}
	const bool enable8 = argc < 13 || atoi(argv[12]) != 0;
	try {
		bt2x::Index idx(argv[1]);
		bt2x::Device dev(0, idx, sc);
		const bool batch = std::string(argv[3]) == "batch";
		// per problem: forward/reverse read strings as the reference's Read holds them
		std::vector<DnaStr> fwd(probs.size()), rev(probs.size());
		std::vector<QualStr> qf(probs.size()), qr(probs.size());
		for(size_t i = 0; i < probs.size(); i++) {
			for(char ch : probs[i].seq) fwd[i].v.push_back((uint8_t)code(ch));
			for(size_t k = fwd[i].v.size(); k > 0; k--) { const uint8_t c = fwd[i].v[k - 1]; rev[i].v.push_back(c > 3 ? 4 : 3 - c); }
			qf[i].s = probs[i].qual;
			qr[i].s.assign(probs[i].qual.rbegin(), probs[i].qual.rend());
		}
		FILE* fo = stdout;
		if(batch) {
			// SwBatch: every problem queued, one launch, results replayed per problem
			bt2x::SwBatch b(dev);
			std::vector<int> pid(probs.size(), -1);
			for(size_t i = 0; i < probs.size(); i++) {
				const Prob& p = probs[i];
				ScoringStub ss{{p.nceil}};
				int slot = -1;
				if(!b.initRead(fwd[i], rev[i], qf[i], qr[i], fwd[i].length(), ss, slot)) continue;
				RectStub rect{p.refl, p.refr, p.triml, p.corel, p.corer};
				WindowRefs refs{p.refl, p.win};
				size_t nsUpto = 0;
				b.initRef(slot, p.fw != 0, 0, rect, refs, p.tlen, p.minsc, 0, nsUpto, pid[i], enable8);
			}
			b.run();
			for(size_t i = 0; i < probs.size(); i++) {
				fprintf(fo, "P %zu\n", i);
				if(pid[i] < 0) { fprintf(fo, "X\n"); continue; }
				Rng rnd; rnd.init(probs[i].rseed);
				print_result(fo, b, pid[i], probs[i], rnd);
			}
		} else {
			// SwAlignerHip: the reference's call sequence verbatim, one problem at a time
			bt2x::SwAlignerHip swa(dev);
			for(size_t i = 0; i < probs.size(); i++) {
				const Prob& p = probs[i];
				fprintf(fo, "P %zu\n", i);
				ScoringStub ss{{p.nceil}};
				RectStub rect{p.refl, p.refr, p.triml, p.corel, p.corer};
				WindowRefs refs{p.refl, p.win};
				size_t nsUpto = 0;
				if(!swa.initRead(fwd[i], rev[i], qf[i], qr[i], fwd[i].length(), ss) ||
				   !swa.initRef(p.fw != 0, 0, rect, refs, p.tlen, p.minsc, enable8, true, 0, nsUpto)) {
					fprintf(fo, "X\n"); continue;
				}
				int64_t best = 0;
				const bool ok = swa.align(best);
				fprintf(fo, "A %d %lld\n", (int)ok, (long long)best);
				if(!ok) continue;
				Rng rnd; rnd.init(p.rseed);
				bt2x::AlnView res;
				while(!swa.done()) {
					if(!swa.nextAlignment(res, p.minsc, rnd)) { fprintf(fo, "N 0 %u\n", rnd.last); break; }
					fprintf(fo, "N 1 %u %d %d %d %d %d %lld %d %zu", rnd.last, res.score, res.ns, res.gaps,
					        (int)res.edits.size(), res.bases_aligned, (long long)res.refoff, res.refns, res.edits.size());
					for(uint32_t e : res.edits)
						fprintf(fo, " %u,%u,%c,%c", BT2X_EDIT_POS(e), BT2X_EDIT_TYPE(e), BT2X_EDIT_CHR(e), BT2X_EDIT_QCHR(e));
					fprintf(fo, "\n");
				}
			}
		}
	} catch(const bt2x::Error& e) {
		fprintf(stderr, "%s\n", e.what());
		return 3;
	}
	return 0;
}
