// bt2x_build.cpp — .bt2l index builder (host C++), byte-identical to the reference's
// bowtie2-build-l at its defaults (lineRate 7, offRate 4, ftabChars 10).
//
// Needed because the GPU box never has the reference: benches and large parity runs
// build their synthetic genomes' indexes there.  Format and semantics follow
//   FASTA -> fragment records   fastaRefReadSize / fastaRefReadSizes (ref_read.cpp:28-330)
//   .3/.4 (packed reference)    BitPairReference::szsFromFasta (reference.cpp:597-678),
//                               RefRecord::write (ref_read.h:94), BitpairOutFileBuf (filebuf.h:558)
//   header, plen, rstarts       Ebwt::writeFromMemory (bt2_io.cpp:801), joinToDisk
//                               (bt2_idx.h:2788), szsToDisk (bt2_io.cpp:933)
//   BWT sides, occ, zOff, fchr, Ebwt::buildToDisk (bt2_idx.h:2922-3267)
//   ftab/eftab, SA sample (.2)
// The suffix array comes from our own SA-IS (not the reference's blockwise DC sort);
// the BWT/SA of a text are unique, so the files are identical.  The reference orders
// '$' after every base (fchr[A] = 0, the '$' row is row len), which is the reverse of
// the suffix order of the complemented text with '$' smallest — that is what we sort.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bt2x.h"

namespace {

// ------------------------------------------------------------------ SA-IS
template<typename I>
void get_buckets(const std::vector<I>& cnt, std::vector<I>& bkt, int K, bool end) {
	I sum = 0;
	for(int c = 0; c < K; c++) { sum += cnt[c]; bkt[c] = end ? sum : sum - cnt[c]; }
}

// Suffix array of T[0..n) where T[n-1] is the unique smallest symbol (0), T in [0,K).
template<typename I, typename C>
void sais(const C* T, I* SA, I n, int K) {
	std::vector<uint8_t> t(n);               // 1 = S-type
	t[n - 1] = 1;
	for(I i = n - 1; i-- > 0;) t[i] = (T[i] < T[i + 1] || (T[i] == T[i + 1] && t[i + 1])) ? 1 : 0;
	auto isLMS = [&](I i) { return i > 0 && t[i] && !t[i - 1]; };
	std::vector<I> cnt(K, 0), bkt(K);
	for(I i = 0; i < n; i++) cnt[T[i]]++;
	auto induce = [&]() {
		get_buckets(cnt, bkt, K, false);
		for(I i = 0; i < n; i++) {
			const I j = SA[i];
			if(j != (I)-1 && j > 0 && !t[j - 1]) SA[bkt[T[j - 1]]++] = j - 1;
		}
		get_buckets(cnt, bkt, K, true);
		for(I i = n; i-- > 0;) {
			const I j = SA[i];
			if(j != (I)-1 && j > 0 && t[j - 1]) SA[--bkt[T[j - 1]]] = j - 1;
		}
	};
	// step 1: sort LMS substrings
	std::fill(SA, SA + n, (I)-1);
	get_buckets(cnt, bkt, K, true);
	for(I i = 1; i < n; i++) if(isLMS(i)) SA[--bkt[T[i]]] = i;
	induce();
	// compact sorted LMS positions into SA[0..n1)
	I n1 = 0;
	for(I i = 0; i < n; i++) if(SA[i] != (I)-1 && isLMS(SA[i])) SA[n1++] = SA[i];
	std::fill(SA + n1, SA + n, (I)-1);
	// name LMS substrings
	I name = 0, prev = (I)-1;
	for(I i = 0; i < n1; i++) {
		const I pos = SA[i];
		bool diff = (prev == (I)-1);
		if(!diff) {
			for(I d = 0;; d++) {
				if(T[pos + d] != T[prev + d] || t[pos + d] != t[prev + d]) { diff = true; break; }
				if(d > 0 && (isLMS(pos + d) || isLMS(prev + d))) {
					diff = !(isLMS(pos + d) && isLMS(prev + d));
					break;
				}
			}
		}
		if(diff) { name++; prev = pos; }
		SA[n1 + pos / 2] = name - 1;
	}
	// gather names in text order into the tail
	I j = n - 1;
	for(I i = n - 1; i + 1 > n1; i--) {
		if(SA[i] != (I)-1) SA[j--] = SA[i];
		if(i == n1) break;
	}
	// step 2: sort the reduced string
	I* s1 = SA + n - n1;
	I* SA1 = SA;
	if(name < n1) {
		sais<I, I>(s1, SA1, n1, (int)name);
	} else {
		for(I i = 0; i < n1; i++) SA1[s1[i]] = i;
	}
	// step 3: induce the final SA from the sorted LMS suffixes
	{
		I k = 0;
		for(I i = 1; i < n; i++) if(isLMS(i)) s1[k++] = i;          // positions of LMS in text order
		for(I i = 0; i < n1; i++) SA1[i] = s1[SA1[i]];
		std::fill(SA + n1, SA + n, (I)-1);
		get_buckets(cnt, bkt, K, true);
		for(I i = n1; i-- > 0;) {
			const I p = SA[i];
			SA[i] = (I)-1;
			SA[--bkt[T[p]]] = p;
		}
		induce();
	}
}

// -------------------------------------------------------------- FASTA
struct RefRecord { uint64_t off, len; bool first; };

uint8_t dnacat(int c) {      // asc2dnacat (alphabet.cpp:36)
	switch(c) {
	case 'A': case 'C': case 'G': case 'T': case 'a': case 'c': case 'g': case 't': return 1;
	case '-': return 3;
	case 'B': case 'D': case 'H': case 'K': case 'M': case 'N': case 'R': case 'S': case 'V':
	case 'W': case 'X': case 'Y': case 'b': case 'd': case 'h': case 'k': case 'm': case 'n':
	case 'r': case 's': case 'v': case 'w': case 'x': case 'y': return 2;
	default: return 0;
	}
}
int dnacode(int c) {
	switch(c) { case 'A': case 'a': return 0; case 'C': case 'c': return 1; case 'G': case 'g': return 2; default: return 3; }
}

struct Parsed {
	std::vector<RefRecord> recs;       // after fastaRefReadSizes' filtering
	std::vector<std::string> names;
	std::vector<uint8_t> text;         // joined unambiguous text, codes 0-3
};

// fastaRefReadSize semantics over a whole file: a record per run of unambiguous
// characters, off = number of gap/ambiguous characters since the previous record (or
// the start of the sequence); trailing gaps give a (off, 0) record; empty sequences
// give a (0, 0, first) record.
bool parse_fasta(const char* path, Parsed& P) {
	FILE* f = fopen(path, "rb");
	if(!f) return false;
	std::vector<char> buf;
	{
		char tmp[1 << 16];
		size_t r;
		while((r = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + r);
		fclose(f);
	}
	size_t i = 0, n = buf.size();
	while(i < n && isspace((unsigned char)buf[i])) i++;
	if(i >= n || buf[i] != '>') return false;
	while(i < n) {
		// header line(s): consecutive '>' lines keep only the last name
		std::string name;
		while(i < n && buf[i] == '>') {
			name.clear();
			i++;
			while(i < n && buf[i] != '\n' && buf[i] != '\r') name.push_back(buf[i++]);
			while(i < n && (buf[i] == '\n' || buf[i] == '\r')) i++;
		}
		P.names.push_back(name);
		// sequence body until next '>' at line start (any '>' ends it, as in the reference)
		bool first = true;
		uint64_t off = 0, len = 0;
		bool inrun = false;
		size_t nrec_before = P.recs.size();
		while(i < n && buf[i] != '>') {
			const int c = (unsigned char)buf[i++];
			const uint8_t cat = dnacat(c);
			if(cat == 1) {
				inrun = true; len++;
				P.text.push_back((uint8_t)dnacode(c));
			} else if(cat >= 2) {
				if(inrun) {
					P.recs.push_back({off, len, first});
					first = false; off = 0; len = 0; inrun = false;
				}
				off++;
			}
		}
		if(inrun) P.recs.push_back({off, len, first});
		else if(off > 0 || first) P.recs.push_back({off, 0, first});
		(void)nrec_before;
	}
	// fastaRefReadSizes drops (0, 0, !first) records
	std::vector<RefRecord> kept;
	for(const auto& r : P.recs) if(!(r.len == 0 && r.off == 0 && !r.first)) kept.push_back(r);
	P.recs.swap(kept);
	return true;
}

template<typename T> void put(std::vector<uint8_t>& o, T v) {
	const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
	o.insert(o.end(), p, p + sizeof(T));
}

bool write_file(const std::string& path, const std::vector<uint8_t>& data) {
	FILE* f = fopen(path.c_str(), "wb");
	if(!f) return false;
	const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
	return fclose(f) == 0 && ok;
}

} // namespace

static int build_impl(const char* fasta, const char* outbase, int off_rate, int ftab_chars,
                      const uint64_t* sa_in, uint64_t sa_n, const uint8_t* bwt_in, const uint32_t* key_in) {
	if(!fasta || !outbase || off_rate < 0 || off_rate > 16 || ftab_chars < 1 || ftab_chars > 16) return BT2X_E_ARG;
	Parsed P;
	if(!parse_fasta(fasta, P)) return BT2X_E_IO;
	const uint64_t len = P.text.size();
	if(len == 0) return BT2X_E_ARG;
	const std::string base(outbase);
	// ---------------- .3 / .4: packed reference (BitPairReference::szsFromFasta)
	{
		std::vector<uint8_t> o3;
		put<int32_t>(o3, 1);
		put<uint64_t>(o3, (uint64_t)P.recs.size());
		for(const auto& r : P.recs) { put<uint64_t>(o3, r.off); put<uint64_t>(o3, r.len); o3.push_back(r.first ? 1 : 0); }
		if(!write_file(base + ".3.bt2l", o3)) return BT2X_E_IO;
		std::vector<uint8_t> o4((len + 3) / 4, 0);
		for(uint64_t k = 0; k < len; k++) o4[k >> 2] |= (uint8_t)(P.text[k] << (2 * (k & 3)));
		if(!write_file(base + ".4.bt2l", o4)) return BT2X_E_IO;
	}
	// ---------------- suffix array (rows 0..len; '$' sorts last)
	const uint64_t n = len + 1;
	if(sa_in) {
		// caller-supplied suffix array (e.g. sorted on the GPU): cheap consistency checks --
		// '$' row last, entries in range, first characters non-decreasing
		if(sa_n != n || sa_in[len] != len) return BT2X_E_ARG;
		if(!bwt_in)
			for(uint64_t k = 0; k + 1 < len; k++)
				if(sa_in[k] >= len || P.text[sa_in[k]] > P.text[sa_in[k + 1]]) return BT2X_E_ARG;
	}
	std::vector<uint64_t> SA(sa_in ? 0 : n);
	if(!sa_in) {
		std::vector<uint8_t> Tc(n);
		for(uint64_t k = 0; k < len; k++) Tc[k] = (uint8_t)(4 - P.text[k]);   // 3-c, shifted by 1
		Tc[len] = 0;                                                          // sentinel
		if(n < 0xffffffffULL) {
			std::vector<uint32_t> sa32(n);
			sais<uint32_t, uint8_t>(Tc.data(), sa32.data(), (uint32_t)n, 5);
			for(uint64_t k = 0; k < n; k++) SA[k] = sa32[n - 1 - k];          // reverse order
		} else {
			std::vector<uint64_t> sa64(n);
			sais<uint64_t, uint8_t>(Tc.data(), sa64.data(), n, 5);
			for(uint64_t k = 0; k < n; k++) SA[k] = sa64[n - 1 - k];
		}
	}
	// ---------------- EbwtParams (bt2_idx.h:134-165), lineRate 7
	const int lineRate = 7;
	const uint64_t sideSz = 1ULL << lineRate, sideBwtSz = sideSz - 32;
	const uint64_t bwtSz = len / 4 + 1;
	const uint64_t numSides = (bwtSz + sideBwtSz - 1) / sideBwtSz;
	const uint64_t ebwtTot = numSides * sideSz;
	const uint64_t ftabLen = (1ULL << (2 * ftab_chars)) + 1, eftabLen = 2ULL * ftab_chars;
	const uint64_t offMask = ~0ULL << off_rate;
	// ---------------- buildToDisk
	std::vector<uint8_t> ebwt(ebwtTot, 0);
	std::vector<uint64_t> ftab(ftabLen, 0), eftab(eftabLen, 0);
	std::vector<uint8_t> absorb(ftabLen, 0);
	std::vector<uint64_t> offs;
	uint64_t fchr[5] = {0, 0, 0, 0, 0}, occ[4] = {0, 0, 0, 0}, occSave[4] = {0, 0, 0, 0};
	uint64_t zOff = ~0ULL, si = 0;
	uint8_t absorbCnt = 0;
	for(uint64_t side = 0; side < ebwtTot; side += sideSz) {
		uint8_t* sp = &ebwt[side];
		for(uint64_t sideCur = 0; sideCur < sideBwtSz; sideCur++) {
			uint8_t byte = 0;
			for(int bpi = 0; bpi < 4; bpi++, si++) {
				int bwtChar = 0;
				bool count = true;
				if(si <= len) {
					const uint64_t saElt = sa_in ? sa_in[si] : SA[si];
					if(saElt == 0) { bwtChar = 0; count = false; zOff = si; }
					else { bwtChar = bwt_in ? bwt_in[si] : P.text[saElt - 1]; fchr[bwtChar]++; }
					if(len - saElt >= (uint64_t)ftab_chars) {
						uint64_t sufInt = 0;
						if(key_in) sufInt = key_in[si];
						else for(int k = 0; k < ftab_chars; k++) sufInt = (sufInt << 2) | P.text[saElt + k];
						ftab[sufInt + 1]++;
						if(absorbCnt > 0) { absorb[sufInt] = absorbCnt; absorbCnt = 0; }
					} else {
						absorbCnt++;
					}
					if((si & offMask) == si) offs.push_back(saElt);
				}
				if(count) occ[bwtChar]++;
				byte |= (uint8_t)(bwtChar << (2 * bpi));
			}
			sp[sideCur] = byte;
		}
		std::memcpy(sp + sideBwtSz, occSave, 32);
		std::memcpy(occSave, occ, 32);
	}
	if(absorbCnt > 0) absorb[ftabLen - 1] = absorbCnt;
	for(int i = 1; i < 4; i++) fchr[i] += fchr[i - 1];
	for(int i = 4; i >= 1; i--) fchr[i] = fchr[i - 1];
	fchr[0] = 0;
	const uint64_t OFF_MASK = ~0ULL;
	auto ftabHi = [&](uint64_t i) -> uint64_t {
		return ftab[i] <= len ? ftab[i] : eftab[(ftab[i] ^ OFF_MASK) * 2 + 1];
	};
	uint64_t eftabCur = 0;
	for(uint64_t i = 1; i < ftabLen; i++) {
		const uint64_t lo = ftab[i] + ftabHi(i - 1);
		if(absorb[i] > 0) {
			const uint64_t hi = lo + absorb[i];
			if(eftabCur * 2 + 1 >= eftabLen) return BT2X_E_ARG;
			eftab[eftabCur * 2] = lo;
			eftab[eftabCur * 2 + 1] = hi;
			ftab[i] = (eftabCur++) ^ OFF_MASK;
		} else {
			ftab[i] = lo;
		}
	}
	// ---------------- .1.bt2l
	{
		std::vector<uint8_t> o1;
		o1.reserve(ebwtTot + 8 * ftabLen + 4096);
		put<int32_t>(o1, 1);
		put<uint64_t>(o1, len);
		put<int32_t>(o1, lineRate);
		put<int32_t>(o1, 2);
		put<int32_t>(o1, off_rate);
		put<int32_t>(o1, ftab_chars);
		put<int32_t>(o1, -1);                            // flags (writeFromMemory: -(1), fw index)
		// joinToDisk: nPat, plen[], nFrag
		uint64_t nPat = 0, nFrag = 0;
		for(const auto& r : P.recs) { if(r.len > 0) nFrag++; if(r.first) nPat++; }
		std::vector<uint64_t> plen;
		for(const auto& r : P.recs) {
			if(r.first) plen.push_back(r.len + r.off);
			else plen.back() += r.len + r.off;
		}
		put<uint64_t>(o1, nPat);
		for(uint64_t v : plen) put<uint64_t>(o1, v);
		put<uint64_t>(o1, nFrag);
		// szsToDisk
		uint64_t seq = 0, off = 0, totlen = 0;
		for(const auto& r : P.recs) {
			if(r.first) off = 0;
			off += r.off;
			if(r.first) seq++;
			if(r.len == 0) continue;
			put<uint64_t>(o1, totlen); put<uint64_t>(o1, seq - 1); put<uint64_t>(o1, off);
			totlen += r.len; off += r.len;
		}
		o1.insert(o1.end(), ebwt.begin(), ebwt.end());
		put<uint64_t>(o1, zOff);
		for(int k = 0; k < 5; k++) put<uint64_t>(o1, fchr[k]);
		for(uint64_t v : ftab) put<uint64_t>(o1, v);
		for(uint64_t v : eftab) put<uint64_t>(o1, v);
		for(size_t k = 0; k < P.names.size(); k++) {
			std::string nm = P.names[k];
			if(nm.empty()) nm = std::to_string(k);
			o1.insert(o1.end(), nm.begin(), nm.end());
			o1.push_back('\n');
		}
		o1.push_back('\0');
		if(!write_file(base + ".1.bt2l", o1)) return BT2X_E_IO;
	}
	// ---------------- .2.bt2l
	{
		std::vector<uint8_t> o2;
		o2.reserve(4 + 8 * offs.size());
		put<int32_t>(o2, 1);
		for(uint64_t v : offs) put<uint64_t>(o2, v);
		if(!write_file(base + ".2.bt2l", o2)) return BT2X_E_IO;
	}
	return BT2X_OK;
}

extern "C" int bt2x_build_index(const char* fasta, const char* outbase, int off_rate, int ftab_chars) {
	return build_impl(fasta, outbase, off_rate, ftab_chars, nullptr, 0, nullptr, nullptr);
}

extern "C" int bt2x_build_index_sa(const char* fasta, const char* outbase, int off_rate, int ftab_chars,
                                   const uint64_t* sa, uint64_t n, const uint8_t* bwt, const uint32_t* keys) {
	if(!sa || (keys && ftab_chars > 16)) return BT2X_E_ARG;
	return build_impl(fasta, outbase, off_rate, ftab_chars, sa, n, bwt, keys);
}
