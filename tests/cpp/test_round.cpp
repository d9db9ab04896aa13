// test_round.cpp — TEST INFRASTRUCTURE: the seed round that bt2x_seed_round runs on the
// GPU (searchAllSeedsFinalize + rankSeedHits + prioritizeSATups + the rows to resolve)
// against the host driver's restatement, host_round (omp-bowtie2-prime_amd/host), which
// tests/test_e2e.py pins to the reference's own SAM output.  Read by read, on seeds the
// CPU oracle searched, for two seed rounds (the second with the first's exRange) and
// several maxelt values (small ones force the sampling paths: RowSampler, Random1toN's
// seen list and its conversion to a swap list).
//
//   test_round <index base> <reads.fq> --core   round_core.h compiled for the host
//   test_round <index base> <reads.fq> --gpu    the product kernel through the C-ABI
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../omp-bowtie2-prime_amd/csrc/round_core.h"
#include "../../omp-bowtie2-prime_amd/host/bt2x_align.hpp"
#include "../../oracle/bt2x_oracle.h"

using namespace bt2x::host;

namespace {

size_t g_converted = 0, g_seenmode = 0;       // Random1toN ranges sampled in seen-list mode / converted

struct Case {
	bt2x_round_in in;
	std::vector<bt2x_seed_in> seeds;
	std::vector<bt2x_seed_out> so;
	std::vector<bt2x_exrange> exr;
	std::vector<uint8_t> read;         // patFw then patRc
};

struct Got {
	bt2x_round_out out;
	std::vector<bt2x_sat> sats;
	std::vector<uint64_t> rows;
	std::vector<bt2x_exrange> exr;
};

bool same(const Got& a, const Got& b, std::string& why) {
	const bt2x_round_out &x = a.out, &y = b.out;
	if(x.status != y.status) { why = "status " + std::to_string(x.status) + " vs " + std::to_string(y.status); return false; }
	if(x.nonz != y.nonz || x.num_elts != y.num_elts) { why = "hit counts"; return false; }
	if(x.rnd_last != y.rnd_last || x.rnd_lastoff != y.rnd_lastoff) { why = "RNG state"; return false; }
	if(x.status != BT2X_ROUND_OK) return true;
	if(a.sats.size() != b.sats.size()) { why = "nsat " + std::to_string(a.sats.size()) + " vs " + std::to_string(b.sats.size()); return false; }
	for(size_t i = 0; i < a.sats.size(); i++)
		if(std::memcmp(&a.sats[i], &b.sats[i], sizeof(bt2x_sat)) != 0) { why = "sat " + std::to_string(i); return false; }
	if(a.rows != b.rows) { why = "rows"; return false; }
	if(a.exr.size() != b.exr.size()) { why = "exRange count"; return false; }
	for(size_t i = 0; i < a.exr.size(); i++)
		if(std::memcmp(&a.exr[i], &b.exr[i], sizeof(bt2x_exrange)) != 0) { why = "exRange " + std::to_string(i); return false; }
	return true;
}

Got run_host(const Case& c, uint32_t maxelt) {
	Got g;
	Rng rnd;
	rnd.last = c.in.rnd_last; rnd.lastOff = c.in.rnd_lastoff;
	RoundScratch w;
	std::vector<bt2x_resolve_in> rows;
	host_round(c.in, c.seeds.data(), c.so.data(), c.exr.data(), maxelt, rnd, w, g.out, g.sats, rows, g.exr);
	for(const bt2x_resolve_in& r : rows) g.rows.push_back(r.row);
	return g;
}

struct CoreWs { bt2x_round::PrepWs p; bt2x_round::SampleWs s; };

// prep() then sample(), composed the way round_kernel.hip lays the read's output out
Got run_core(const Case& c, uint32_t maxelt, CoreWs& w) {
	Got g;
	bt2x_round::Rnd rnd{c.in.rnd_last, c.in.rnd_lastoff};
	const bt2x_round::Prep p = bt2x_round::prep(c.in, c.seeds.data(), c.so.data(), c.exr.data(), maxelt, rnd, w.p);
	std::memset(&g.out, 0, sizeof g.out);
	g.out.status = p.status; g.out.nonz = p.nonz; g.out.num_elts = p.numElts;
	if(p.status == BT2X_ROUND_OK) {
		for(uint32_t i = 0; i < p.nsmallSat; i++) {
			const bt2x_round::Range& rg = w.p.r2[i];
			bt2x_sat s;
			s.rdoff = (uint16_t)rg.rdoff; s.rand_n = (uint8_t)rg.size; s.fwlen = BT2X_SAT_FWLEN(rg.fw, c.in.seedlen);
			g.sats.push_back(s);
			for(uint32_t k = 0; k < (uint32_t)rg.size; k++) g.rows.push_back(rg.topf + k);
		}
		if(p.nsamples) {
			const bt2x_round::Range* big = w.p.r2 + p.nsmall;
			const uint32_t nb = p.n2 - p.nsmall;
			for(uint32_t i = 0; i < nb && i < (uint32_t)bt2x_round::kMaxRanges; i++) w.s.big[i] = big[i];
			bt2x_round::SerialCoop co;
			const size_t s0 = g.sats.size(), e0 = g.rows.size();
			g.sats.resize(s0 + p.nsamples);
			g.rows.resize(e0 + p.nsamples);
			const bool ok = bt2x_round::sample(nb, p.nsamples, rnd, w.s, co, [&](uint64_t k, const bt2x_round::Range& rg, uint16_t elt) {
				bt2x_sat s;
				s.rdoff = (uint16_t)rg.rdoff; s.rand_n = 1; s.fwlen = BT2X_SAT_FWLEN(rg.fw, c.in.seedlen);
				g.sats[s0 + k] = s;
				g.rows[e0 + k] = rg.topf + elt;
			});
			if(!ok) g.out.status = BT2X_ROUND_REDO;
			for(uint32_t i = 0; i < nb; i++) {
				if(w.s.r1n[i].inited && w.s.r1n[i].converted) g_converted++;
				if(w.s.r1n[i].inited && (!w.s.r1n[i].swaplist || w.s.r1n[i].converted)) g_seenmode++;
			}
		}
		g.exr.assign(w.p.exnew, w.p.exnew + p.nexnew);
	}
	g.out.rnd_last = rnd.last; g.out.rnd_lastoff = rnd.lastOff;
	return g;
}

} // namespace

int main(int argc, char** argv) {
	if(argc < 4) { std::fprintf(stderr, "usage: test_round <index> <reads.fq> --core|--gpu\n"); return 2; }
	const bool gpu = std::string(argv[3]) == "--gpu";
	Params P;
	bt2x_scoring_init(&P.sc);
	bt2x::Index index(argv[1], true);
	const bt2x_index_desc& idx = index.desc();
	std::vector<Read> reads;
	{
		FastqReader fq(argv[2]);
		std::vector<FastqReader::Raw> raw;
		fq.take(1u << 30, raw);
		reads.resize(raw.size());
		for(size_t i = 0; i < raw.size(); i++) FastqReader::decode(raw[i], reads[i], i, 0);
	}
	// every read's seed rounds, searched by the CPU oracle
	std::vector<Case> cases;
	for(const Read& rd : reads) {
		const size_t rdlen = rd.length();
		if(rdlen < 1 || rdlen > BT2X_MAX_ROWS) continue;
		const int interval = std::max(P.msIval.f<int>((double)rdlen), 1);
		const uint32_t L = (uint32_t)std::min<size_t>((size_t)P.multiseedLen, rdlen);
		const uint32_t nrounds = (uint32_t)std::min<int>(P.nSeedRounds, interval);
		for(uint32_t roundi = 0; roundi < nrounds; roundi++) {
			const uint32_t offset = (uint32_t)((interval * roundi) / nrounds);
			if(offset > 0 && (size_t)P.multiseedLen + offset > rdlen) break;
			const uint32_t nseeds = (rdlen - offset > L) ? 1 + (uint32_t)((rdlen - offset - L) / interval) : 1;
			Case c;
			c.read.assign(rd.fw.begin(), rd.fw.end());
			c.read.insert(c.read.end(), rd.rc.begin(), rd.rc.end());
			for(int fwi = 0; fwi < 2; fwi++) {
				const std::vector<uint8_t>& s = fwi == 0 ? rd.fw : rd.rc;
				for(uint32_t i = 0; i < nseeds; i++) {
					const uint32_t depth = i * interval + offset;
					const uint32_t st = fwi == 0 ? depth : (uint32_t)(rdlen - depth - L);
					bool ok = true;
					for(uint32_t k = 0; k < L; k++) if(s[st + k] > 3) { ok = false; break; }
					if(!ok) continue;
					bt2x_seed_in si;
					std::memset(&si, 0, sizeof si);
					si.read_off = fwi == 0 ? 0 : rdlen;
					si.seed_off = (uint8_t)st; si.seed_len = (uint8_t)L;
					c.seeds.push_back(si);
				}
			}
			if(c.seeds.empty()) break;
			c.so.resize(c.seeds.size());
			if(bt2o_seed_search(&idx, c.read.data(), c.seeds.data(), (uint32_t)c.seeds.size(), 1, c.so.data(), nullptr) != 0)
				{ std::fprintf(stderr, "oracle seed search failed\n"); return 2; }
			std::memset(&c.in, 0, sizeof c.in);
			c.in.rnd_last = rd.seed ^ (roundi * 0x9e3779b9u); c.in.rnd_lastoff = (int32_t)(rd.seed % 33);
			c.in.nseeds = (uint16_t)c.seeds.size(); c.in.num_offs = (uint16_t)nseeds; c.in.rdlen = (uint16_t)rdlen;
			c.in.interval = (uint16_t)interval; c.in.offset = (uint16_t)offset; c.in.seedlen = (uint16_t)L;
			// round 2 sees round 1's exRange entries (from the host restatement)
			if(roundi > 0 && !cases.empty()) {
				const Got prev = run_host(cases.back(), (uint32_t)P.mxIter);
				c.exr = cases.back().exr;
				c.exr.insert(c.exr.end(), prev.exr.begin(), prev.exr.end());
			}
			c.in.nexr = (uint16_t)c.exr.size();
			cases.push_back(c);
		}
	}
	const uint32_t maxelts[] = {400, 1, 3, 7, 20, 60};
	size_t bad = 0, n = 0, nsampled = 0;
	if(!gpu) {
		std::vector<CoreWs> ws(1);
		for(uint32_t me : maxelts)
			for(const Case& c : cases) {
				const Got a = run_host(c, me), b = run_core(c, me, ws[0]);
				std::string why;
				n++;
				nsampled += a.out.status == BT2X_ROUND_OK && a.sats.size() && a.sats.back().rand_n == 1 && a.out.nelt > 5;
				if(!same(a, b, why)) {
					if(bad < 5) std::fprintf(stderr, "mismatch (maxelt %u, rdlen %u): %s\n", me, c.in.rdlen, why.c_str());
					bad++;
				}
			}
	} else {
		bt2x::Device dev(0, index, P.sc);
		for(uint32_t me : maxelts) {
			// one launch over all cases
			std::vector<uint8_t> rb;
			std::vector<bt2x_seed_in> seeds;
			std::vector<bt2x_round_in> in;
			std::vector<bt2x_exrange> exr;
			for(const Case& c : cases) {
				bt2x_round_in q = c.in;
				q.read_off = rb.size(); q.seed0 = seeds.size(); q.exr0 = (uint32_t)exr.size();
				for(bt2x_seed_in s : c.seeds) { s.read_off += rb.size(); seeds.push_back(s); }
				rb.insert(rb.end(), c.read.begin(), c.read.end());
				exr.insert(exr.end(), c.exr.begin(), c.exr.end());
				in.push_back(q);
			}
			std::vector<bt2x_round_out> out(in.size());
			std::vector<bt2x_sat> sats(in.size() * 420);
			std::vector<bt2x_elt> elts(in.size() * 420);
			std::vector<bt2x_exrange> exro(in.size() * 130);
			uint32_t used[3];
			const int rc = bt2x_seed_round(dev.ctx(), rb.data(), rb.size(), seeds.data(), (uint32_t)seeds.size(), in.data(),
			                               (uint32_t)in.size(), exr.data(), (uint32_t)exr.size(), me, out.data(), sats.data(),
			                               (uint32_t)sats.size(), elts.data(), (uint32_t)elts.size(), exro.data(),
			                               (uint32_t)exro.size(), used);
			if(rc != BT2X_OK) { std::fprintf(stderr, "bt2x_seed_round: %d\n", rc); return 1; }
			std::vector<bt2x_resolve_in> allrows;
			for(size_t r = 0; r < cases.size(); r++) {
				const Got a = run_host(cases[r], me);
				Got b;
				b.out = out[r];
				if(out[r].status == BT2X_ROUND_OK) {
					b.sats.assign(sats.begin() + out[r].sat0, sats.begin() + out[r].sat0 + out[r].nsat);
					b.exr.assign(exro.begin() + out[r].exr0, exro.begin() + out[r].exr0 + out[r].nexr);
					// rows are checked through their resolution: resolve the host's rows on the
					// GPU too and compare the placements
					std::vector<bt2x_resolve_in> hr;
					for(uint64_t row : a.rows) { bt2x_resolve_in x; std::memset(&x, 0, sizeof x); x.row = row; x.qlen = cases[r].in.seedlen; hr.push_back(x); }
					std::vector<bt2x_resolve_out> ho(hr.size());
					if(!hr.empty() && bt2x_resolve(dev.ctx(), hr.data(), (uint32_t)hr.size(), 0, ho.data()) != BT2X_OK) return 1;
					bool eq = ho.size() == out[r].nelt;
					for(size_t k = 0; eq && k < ho.size(); k++)
						eq = ho[k].toff == bt2x_elt_toff(elts[out[r].elt0 + k]) && ho[k].tidx == bt2x_elt_tidx(elts[out[r].elt0 + k]) &&
						     ho[k].straddled == bt2x_elt_straddled(elts[out[r].elt0 + k]);
					b.rows = eq ? a.rows : std::vector<uint64_t>{};
				}
				std::string why;
				n++;
				nsampled += a.out.status == BT2X_ROUND_OK && a.sats.size() && a.sats.back().rand_n == 1 && a.out.nelt > 5;
				if(out[r].status == BT2X_ROUND_REDO) continue;            // handed back to the host by design
				if(!same(a, b, why)) {
					if(bad < 5) std::fprintf(stderr, "GPU mismatch (maxelt %u, read case %zu): %s\n", me, r, why.c_str());
					bad++;
				}
			}
		}
	}
	std::printf("round cases=%zu checks=%zu sampled=%zu seenmode=%zu converted=%zu mismatches=%zu\n", cases.size(), n,
	            nsampled, g_seenmode, g_converted, bad);
	return bad ? 1 : 0;
}
