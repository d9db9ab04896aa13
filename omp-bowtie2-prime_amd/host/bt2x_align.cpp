// bt2x_align.cpp — the host driver of bt2x_align.hpp: per-read coroutine (the
// reference's multiseedSearchWorker phases for one read), the batching scheduler,
// reporting and SAM formatting.  Compiled without -ffast-math and with
// -ffp-contract=off: RowSampler darts and MAPQ thresholds are float/double compares
// that must round exactly like the reference's x86-64 build.
#include "bt2x_align.hpp"

#include <atomic>
#include <cctype>
#include <cerrno>
#include <charconv>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

#include <climits>

#include <fcntl.h>
#include <sched.h>
#include <future>
#include <malloc.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef __AVX2__
#include <immintrin.h>
#endif

#ifdef BT2X_PHASE_PROF
// Development-only phase profiler of the per-read coroutine (-DBT2X_PHASE_PROF): TSC
// cycles per phase summed over threads, printed at the end of run().
#include <mutex>
#include <x86intrin.h>
namespace {
constexpr int kPhases = 16;
const char* kPhaseName[kPhases] = {"init", "seeds", "rank", "prioritize", "resolve_in", "walk", "lookahead",
                                   "records", "finish", "scatter", "g_pass1", "g_bases", "g_pass2", "walk_reset",
                                   "memo", "spare"};
struct PhaseAcc { uint64_t c[kPhases] = {}; uint64_t last = 0; PhaseAcc(); };
std::mutex g_ph_mu;
std::vector<PhaseAcc*> g_ph_all;
PhaseAcc::PhaseAcc() { std::lock_guard<std::mutex> g(g_ph_mu); g_ph_all.push_back(this); }
thread_local PhaseAcc t_ph;
inline void ph_start() { t_ph.last = __rdtsc(); }
inline void ph(int k) { const uint64_t n = __rdtsc(); t_ph.c[k] += n - t_ph.last; t_ph.last = n; }
void ph_print() {
	uint64_t tot[kPhases] = {}, all = 0;
	for(PhaseAcc* a : g_ph_all) for(int k = 0; k < kPhases; k++) tot[k] += a->c[k];
	for(int k = 0; k < kPhases; k++) all += tot[k];
	for(int k = 0; k < kPhases; k++)
		std::fprintf(stderr, "PHASE %-11s %7.3f Gcyc %5.1f%%\n", kPhaseName[k], tot[k] / 1e9, 100.0 * tot[k] / (all ? all : 1));
}
}
#define PH_START() ph_start()
#define PH(k) ph(k)
#else
#define PH_START() ((void)0)
#define PH(k) ((void)0)
#endif

namespace bt2x {
namespace host {

void tune_malloc() {
	mallopt(M_TRIM_THRESHOLD, INT_MAX);
	mallopt(M_TOP_PAD, 64 << 20);
	mallopt(M_MMAP_THRESHOLD, 32 << 20);
}

namespace {
struct HostHooks { void* (*alloc)(size_t); void (*release)(void*); };
void* plain_alloc(size_t n) { return std::malloc(n); }
void plain_free(void* p) { std::free(p); }
std::atomic<const HostHooks*> g_hooks{nullptr};
const HostHooks kPlain{plain_alloc, plain_free};
constexpr size_t kHostHdr = 64;               // keeps the payload 64-byte aligned
}

void set_host_allocator(void* (*alloc)(size_t), void (*release)(void*)) {
	// hooks live for the process; a block is freed by the hook that allocated it
	g_hooks.store(alloc ? new HostHooks{alloc, release} : &kPlain);
}

void* host_alloc(size_t bytes) {
	const HostHooks* h = g_hooks.load();
	if(!h) h = &kPlain;
	uint8_t* p = static_cast<uint8_t*>(h->alloc(bytes + kHostHdr));
	if(!p) throw std::bad_alloc();
	*reinterpret_cast<const HostHooks**>(p) = h;
	return p + kHostHdr;
}

void host_free(void* q) noexcept {
	if(!q) return;
	uint8_t* p = static_cast<uint8_t*>(q) - kHostHdr;
	(*reinterpret_cast<const HostHooks**>(p))->release(p);
}

const uint8_t kAsc2Dna[256] = {   // alphabet.cpp:142 (A/C/G/T, either case; all else N)
#define N4 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4
	N4, N4, N4, N4,
	4, 0, 4, 1, 4, 4, 4, 2, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 0, 4, 1, 4, 4, 4, 2, 4, 4, 4, 4, 4, 4, 4, 4,
	4, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4,
	N4, N4, N4, N4, N4, N4, N4, N4
#undef N4
};

// ------------------------------------------------------------------- summary

void print_alignment_summary(const ReportingMetrics& m, std::FILE* f) {
	using M = ReportingMetrics;
	auto pct = [](uint64_t num, uint64_t den) { return den ? 100.0 * (double)num / (double)den : 0.0; };
	const uint64_t nread = m.v[M::NREAD], nun = m.v[M::NUNPAIRED];
	if(nread > 0) std::fprintf(f, "%llu reads; of these:\n", (unsigned long long)nread);
	else std::fprintf(f, "%llu reads\n", (unsigned long long)nread);
	if(nun > 0) {
		std::fprintf(f, "  %llu (%.2f%%) were unpaired; of these:\n", (unsigned long long)nun, pct(nun, nread));
		std::fprintf(f, "    %llu (%.2f%%) aligned 0 times\n", (unsigned long long)m.v[M::NUNP_0], pct(m.v[M::NUNP_0], nun));
		std::fprintf(f, "    %llu (%.2f%%) aligned exactly 1 time\n", (unsigned long long)m.v[M::NUNP_UNI1],
		             pct(m.v[M::NUNP_UNI1], nun));
		const uint64_t more = m.v[M::NUNP_UNI2] + m.v[M::NUNP_REP];
		std::fprintf(f, "    %llu (%.2f%%) aligned >1 times\n", (unsigned long long)more, pct(more, nun));
	}
	const uint64_t tot_al = m.v[M::NUNP_UNI] + m.v[M::NUNP_REP];
	std::fprintf(f, "%.2f%% overall alignment rate\n", pct(tot_al, nun));
}

// ---------------------------------------------------------------- FastqReader

namespace {
// first record start at or after byte `at` of a FASTQ map: a line beginning '@' whose
// third line begins '+' (quality lines may begin with '@', never with a following
// '+' line two lines later unless they are a header)
size_t next_record(const char* m, size_t len, size_t at) {
	if(at == 0) return 0;
	size_t pos = at;
	// start of the next line at or after `at` (at itself when the previous byte is '\n')
	if(m[pos - 1] != '\n') {
		const char* nl = (const char*)std::memchr(m + pos, '\n', len - pos);
		if(!nl) return len;
		pos = (size_t)(nl - m) + 1;
	}
	auto next_line = [&](size_t q) -> size_t {
		const char* nl = (const char*)std::memchr(m + q, '\n', len - q);
		return nl ? (size_t)(nl - m) + 1 : len;
	};
	while(pos < len) {
		if(m[pos] == '@') {
			const size_t l2 = next_line(pos);
			const size_t l3 = l2 < len ? next_line(l2) : len;
			if(l3 < len && m[l3] == '+') return pos;
		}
		pos = next_line(pos);
	}
	return len;
}

// records in m[0, n) as FastqReader::take() finds them: empty lines (after stripping
// '\r') are skipped, and a record is a non-empty header line plus the next three lines
uint64_t count_records(const char* m, size_t n) {
	uint64_t k = 0;
	size_t pos = 0;
	auto line = [&](size_t& len) -> bool {
		if(pos >= n) return false;
		const char* s = m + pos;
		const char* nl = (const char*)std::memchr(s, '\n', n - pos);
		len = nl ? (size_t)(nl - s) : n - pos;
		pos += len + (nl ? 1 : 0);
		while(len > 0 && s[len - 1] == '\r') len--;
		return true;
	};
	size_t len = 0;
	while(line(len)) {
		if(!len) continue;
		for(int j = 1; j < 4; j++) if(!line(len)) break;
		k++;
	}
	return k;
}
}

uint64_t FastqReader::count_file_records(const std::string& path) {
	FastqReader r(std::vector<std::string>{path});
	return r.f_.empty() || !r.f_[0].len ? 0 : count_records(r.f_[0].map, r.f_[0].len);
}

FastqReader::FastqReader(const std::vector<std::string>& paths, int shard, int nshards, uint64_t rdid_base) {
	if(nshards < 1 || shard < 0 || shard >= nshards) throw std::runtime_error("bad shard " + std::to_string(shard) + "/" + std::to_string(nshards));
	size_t total = 0;
	for(const std::string& path : paths) {
		File F;
		F.fd = ::open(path.c_str(), O_RDONLY);
		if(F.fd < 0) throw std::runtime_error("cannot open reads file " + path);
		f_.push_back(F);
		struct stat sb;
		if(::fstat(F.fd, &sb) != 0) throw std::runtime_error("cannot stat " + path);
		f_.back().len = (size_t)sb.st_size;
		if(f_.back().len) {
			void* m = ::mmap(nullptr, f_.back().len, PROT_READ, MAP_PRIVATE, F.fd, 0);
			if(m == MAP_FAILED) throw std::runtime_error("cannot map " + path);
			::madvise(m, f_.back().len, MADV_SEQUENTIAL);
			f_.back().map = (const char*)m;
		}
		total += f_.back().len;
	}
	// this shard's byte range [lo, hi) of the concatenated stream, both snapped to record
	// starts within their file
	const size_t lo = (size_t)((unsigned __int128)total * (unsigned)shard / (unsigned)nshards);
	const size_t hi = (size_t)((unsigned __int128)total * (unsigned)(shard + 1) / (unsigned)nshards);
	size_t off = 0;
	first_rdid_ = rdid_base;
	for(File& F : f_) {
		const size_t a = std::min(std::max(lo, off) - off, F.len), b = std::min(std::max(hi, off) - off, F.len);
		F.beg = next_record(F.map, F.len, a);
		F.end = shard + 1 == nshards ? F.len : next_record(F.map, F.len, b);
		if(F.end < F.beg) F.end = F.beg;
		// records before the shard in this file, counted as take() reads them (blank lines
		// between records are not records)
		if(F.beg) first_rdid_ += count_records(F.map, F.beg);
		off += F.len;
	}
	if(!f_.empty()) pos_ = f_[0].beg;
}

void FastqReader::populate_ahead() {
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
	constexpr size_t kWindow = 64u << 20;
	const File& F = f_[cur_];
	const size_t page = 4096;
	const size_t a = pos_ & ~(page - 1);
	const size_t b = std::min(F.end, pos_ + kWindow);
	if(b > a && F.map) ::madvise((void*)(F.map + a), b - a, MADV_POPULATE_READ);
	pop_end_ = b >= F.end ? (size_t)-1 : b;
}

FastqReader::~FastqReader() {
	for(File& F : f_) {
		if(F.map) ::munmap((void*)F.map, F.len);
		if(F.fd >= 0) ::close(F.fd);
	}
}

// ------------------------------------------------------------------- CPU sets

bool parse_cpu_list(const std::string& s, std::vector<int>& out) {
	out.clear();
	size_t i = 0;
	while(i < s.size()) {
		size_t j = i;
		while(j < s.size() && std::isdigit((unsigned char)s[j])) j++;
		if(j == i) return false;
		const long a = std::atol(s.substr(i, j - i).c_str());
		long b = a;
		if(j < s.size() && s[j] == '-') {
			size_t k = ++j;
			while(j < s.size() && std::isdigit((unsigned char)s[j])) j++;
			if(j == k) return false;
			b = std::atol(s.substr(k, j - k).c_str());
		}
		if(b < a || b >= CPU_SETSIZE) return false;
		for(long c = a; c <= b; c++) out.push_back((int)c);
		if(j < s.size() && s[j] != ',') return false;
		i = j + 1;
	}
	return !out.empty();
}

std::string affinity_list() {
	cpu_set_t cur;
	if(sched_getaffinity(0, sizeof cur, &cur) != 0) return "";
	std::string out;
	for(int c = 0; c < CPU_SETSIZE; c++) {
		if(!CPU_ISSET(c, &cur)) continue;
		int e = c;
		while(e + 1 < CPU_SETSIZE && CPU_ISSET(e + 1, &cur)) e++;
		if(!out.empty()) out += ',';
		out += std::to_string(c);
		if(e > c) out += '-' + std::to_string(e);
		c = e;
	}
	return out;
}

void apply_cpu_list(const std::string& list) {
	std::vector<int> cpus;
	if(!parse_cpu_list(list, cpus)) throw std::runtime_error("--cpus: malformed CPU list '" + list + "'");
	cpu_set_t want;
	CPU_ZERO(&want);
	for(int c : cpus) CPU_SET(c, &want);
	if(sched_setaffinity(0, sizeof want, &want) != 0)
		throw std::runtime_error("--cpus " + list + ": none of these CPUs may be used by this process");
}

// ------------------------------------------------------------------- RefInfo

void RefInfo::init(const bt2x_index_desc& d, const std::string& base) {
	plen_.assign(d.plen, d.plen + d.npat);
	text_ = d.text2;
	if(!text_) throw std::runtime_error("RefInfo: index loaded without the packed text (.4.bt2l)");
	frags_.assign(d.npat, {});
	// rstarts: (joined offset, text id, text offset) per fragment (Ebwt::_rstarts)
	for(uint64_t k = 0; k < d.nfrag; k++) {
		const uint64_t joff = d.rstarts[3 * k], tidx = d.rstarts[3 * k + 1], toff = d.rstarts[3 * k + 2];
		const uint64_t jend = (k + 1 < d.nfrag) ? d.rstarts[3 * (k + 1)] : d.len;
		if(tidx >= d.npat) throw std::runtime_error("RefInfo: bad fragment record");
		if(jend > joff) frags_[tidx].push_back({(int64_t)toff, jend - joff, joff});
	}
	// reference names: the text after eftab in <base>.1.bt2l, one per line (bt2_io.cpp:499)
	const std::string p1 = base + ".1.bt2l";
	std::FILE* f = std::fopen(p1.c_str(), "rb");
	if(!f) throw std::runtime_error("cannot open " + p1);
	const uint64_t sideSz = 128, sideBwt = 96;
	const uint64_t numSides = (d.len / 4 + 1 + sideBwt - 1) / sideBwt;
	const uint64_t hdr = 4 + 8 + 5 * 4 + 8 + 8 * d.npat + 8 + 24 * d.nfrag;
	const uint64_t off = hdr + numSides * sideSz + 8 + 40 + 8 * d.ftab_len + 8 * d.eftab_len;
	std::fseek(f, (long)off, SEEK_SET);
	std::string cur;
	int ch;
	while((ch = std::fgetc(f)) != EOF) {
		if(ch == '\n') { names_.push_back(cur); cur.clear(); }
		else cur.push_back((char)ch);
	}
	std::fclose(f);
	if(!cur.empty()) names_.push_back(cur);
	while(names_.size() < d.npat) names_.push_back(std::to_string(names_.size()));
	names_.resize(d.npat);
}

namespace {
// byte of the packed text (4 bases, LSB first) -> its 4 codes as bytes
struct Unpack4 {
	uint32_t t[256];
	Unpack4() {
		for(uint32_t b = 0; b < 256; b++)
			t[b] = (b & 3) | (((b >> 2) & 3) << 8) | (((b >> 4) & 3) << 16) | (((b >> 6) & 3) << 24);
	}
};
const Unpack4 kUnpack4;
}

void RefInfo::stretch(uint32_t tidx, int64_t off, size_t n, uint8_t* out) const {
	std::memset(out, 4, n);
	const std::vector<Frag>& fs = frags_[tidx];
	// fragments are in text order: start at the last one beginning at or before `off`
	size_t k = (size_t)(std::upper_bound(fs.begin(), fs.end(), off,
	                                     [](int64_t o, const Frag& f) { return o < f.toff; }) - fs.begin());
	if(k > 0) k--;
	for(; k < fs.size() && fs[k].toff < off + (int64_t)n; k++) {
		const Frag& fr = fs[k];
		const int64_t a = std::max<int64_t>(off, fr.toff);
		const int64_t b = std::min<int64_t>(off + (int64_t)n, fr.toff + (int64_t)fr.len);
		if(a >= b) continue;
		uint8_t* o = out + (a - off);
		uint64_t j = fr.joff + (uint64_t)(a - fr.toff);
		size_t m = (size_t)(b - a);
		while(m && (j & 3)) { *o++ = (text_[j >> 2] >> ((j & 3) << 1)) & 3; j++; m--; }
		const uint8_t* t = text_ + (j >> 2);
		for(; m >= 4; m -= 4, o += 4, j += 4) std::memcpy(o, &kUnpack4.t[*t++], 4);
		while(m) { *o++ = (text_[j >> 2] >> ((j & 3) << 1)) & 3; j++; m--; }
	}
}

// -------------------------------------------------------------- reporting

namespace {

enum { EXTEND_EXHAUSTED_CANDIDATES = 1, EXTEND_POLICY_FULFILLED, EXTEND_PERFECT_SCORE,
       EXTEND_EXCEEDED_SOFT_LIMIT, EXTEND_EXCEEDED_HARD_LIMIT };

template<class T> inline void append_int(std::string& o, T v) {
	char b[24];
	const auto r = std::to_chars(b, b + sizeof b, v);
	o.append(b, (size_t)(r.ptr - b));
}

// StackedAln (aligner_result.cpp:448-770) over the Watson-strand read: CIGAR appended to
// `cig`, MD:Z value to `md`.  ned: the printed edits (ned() order, 5'-relative for rc).
void cigar_md(const Read& rd, bool fw, const uint32_t* ned0, size_t nedn, std::string& cig, std::string& md) {
	thread_local std::vector<uint32_t> inv;
	thread_local std::string ref, rel, rdc;
	const std::vector<uint8_t>& s = fw ? rd.fw : rd.rc;
	const uint32_t* ed = ned0;
	if(!fw) { invert_poss(ned0, nedn, rd.length(), inv); ed = inv.data(); }
	// Fast path: mismatches only, in increasing read order inside the read (no gap to
	// left-align): the CIGAR is one M run and MD interleaves match runs and reference bases
	// exactly as buildMdz/writeMdz do below.
	{
		bool simple = !s.empty();
		for(size_t q = 0; q < nedn && simple; q++)
			simple = e_type(ed[q]) == ET_MM && e_pos(ed[q]) < s.size() && (q == 0 || e_pos(ed[q]) > e_pos(ed[q - 1]));
		if(simple) {
			append_int(cig, s.size());
			cig.push_back('M');
			size_t prev = 0;
			bool mm_last = false, first = true;
			for(size_t q = 0; q < nedn; q++) {
				const size_t p = e_pos(ed[q]);
				if(p > prev) { append_int(md, p - prev); mm_last = false; first = false; }
				if(mm_last || first) md.push_back('0');
				md.push_back(e_chr(ed[q]));
				mm_last = true; first = false;
				prev = p + 1;
			}
			if(s.size() > prev) append_int(md, s.size() - prev);
			else if(mm_last) md.push_back('0');
			return;
		}
	}
	ref.clear(); rel.clear(); rdc.clear();
	size_t rdoff = 0;
	static const char kAcgtn[] = "ACGTN";
	// The printed edits come from the read's shared edit buffer and may step
	// past the read's end; the reference then reads stale bytes of its read buffer, which
	// only ever reach the output through left-alignment of an adjacent gap.  N stands in.
	auto at = [&](size_t i) -> int { return i < s.size() ? s[i] : 4; };
	for(size_t q = 0; q < nedn; q++) {
		const uint32_t e = ed[q];
		const size_t pos = e_pos(e);
		while(rdoff < pos) { const int c = at(rdoff++); ref.push_back(kAcgtn[c]); rel.push_back('='); rdc.push_back(kAcgtn[c]); }
		const uint32_t t = e_type(e);
		if(t == ET_MM) { const int c = at(rdoff++); ref.push_back(e_chr(e)); rel.push_back('X'); rdc.push_back(kAcgtn[c]); }
		else if(t == ET_REF_GAP) { const int c = at(rdoff++); ref.push_back('-'); rel.push_back('I'); rdc.push_back(kAcgtn[c]); }
		else if(t == ET_READ_GAP) { ref.push_back(e_chr(e)); rel.push_back('D'); rdc.push_back('-'); }
	}
	while(rdoff < s.size()) { const int c = s[rdoff++]; ref.push_back(kAcgtn[c]); rel.push_back('='); rdc.push_back(kAcgtn[c]); }
	// leftAlign(pastMms = false)
	const size_t ln = ref.size();
	for(size_t i = 0; i < ln; i++) {
		const char g = rel[i];
		if(g == '=' || g == 'X') continue;
		size_t glen = 1;
		for(size_t j = i + 1; j < ln; j++) { if(rel[j] != g) break; glen++; }
		if(i >= 1) {   // i == 0 would index [-1] in the reference; a gap never opens row 0
			size_t l = i - 1, r2 = l + glen;
			std::string& gp = (g == 'I') ? ref : rdc;
			const std::string& ngp = (g == 'I') ? rdc : ref;
			while(l > 0 && ngp[l] == ngp[r2]) {
				if(rel[l] == 'X') break;
				std::swap(gp[l], gp[r2]);
				std::swap(rel[l], rel[r2]);
				l--; r2--;
			}
		}
		i += glen - 1;
	}
	// CIGAR (xeq = false)
	for(size_t i = 0; i < ln; i++) {
		char op = rel[i] == 'X' || rel[i] == '=' ? 'M' : rel[i];
		size_t run = 1;
		for(; i + run < ln; run++) {
			const char op2 = rel[i + run] == 'X' || rel[i + run] == '=' ? 'M' : rel[i + run];
			if(op2 != op) break;
		}
		i += run - 1;
		append_int(cig, run);
		cig.push_back(op);
	}
	// MD:Z (buildMdz + writeMdz)
	bool mm_last = false, rdgap_last = false, first_print = true;
	for(size_t i = 0; i < ln; i++) {
		const char op = rel[i];
		if(op == '=') {
			size_t run = 1, nins = 0;
			for(; i + run < ln; run++) {
				if(rel[i + run] == '=') {}
				else if(rel[i + run] == 'I') nins++;
				else break;
			}
			i += run - 1;
			if(run - nins > 0) {
				append_int(md, run - nins);
				first_print = false; mm_last = false; rdgap_last = false;
			}
		} else if(op == 'X') {
			if(rdgap_last || mm_last || first_print) md.push_back('0');
			md.push_back(ref[i]);
			first_print = false; mm_last = true; rdgap_last = false;
		} else if(op == 'D') {
			if(mm_last || first_print) md.push_back('0');
			if(!rdgap_last) md.push_back('^');
			md.push_back(ref[i]);
			first_print = false; mm_last = false; rdgap_last = true;
		}
	}
	if(mm_last || rdgap_last) md.push_back('0');
}

// BowtieMapq2::mapq, monotone (end-to-end) branch, unpaired (unique.h:187-330).
int64_t mapq_v2(const Params& p, size_t rdlen, int64_t best, bool hasSecbest, int64_t secbestIn) {
	const int64_t scPer = 0;
	const int64_t scMin = p.scoreMin.f<int64_t>((float)rdlen);
	int64_t secbest = scMin - 1;
	const int64_t diff = std::max<int64_t>(1, scPer - scMin);
	int64_t ret = 0;
	const int64_t bestOver = best - scMin;
	if(!hasSecbest) {
		if     (bestOver >= diff * (double)0.8f) ret = 42;
		else if(bestOver >= diff * (double)0.7f) ret = 40;
		else if(bestOver >= diff * (double)0.6f) ret = 24;
		else if(bestOver >= diff * (double)0.5f) ret = 23;
		else if(bestOver >= diff * (double)0.4f) ret = 8;
		else if(bestOver >= diff * (double)0.3f) ret = 3;
		else                                     ret = 0;
	} else {
		secbest = secbestIn;
		const int64_t bestdiff = std::labs(std::labs((long)best) - std::labs((long)secbest));
		if(bestdiff >= diff * (double)0.9f) ret = bestOver == diff ? 39 : 33;
		else if(bestdiff >= diff * (double)0.8f) ret = bestOver == diff ? 38 : 27;
		else if(bestdiff >= diff * (double)0.7f) ret = bestOver == diff ? 37 : 26;
		else if(bestdiff >= diff * (double)0.6f) ret = bestOver == diff ? 36 : 22;
		else if(bestdiff >= diff * (double)0.5f) {
			if(bestOver == diff) ret = 35;
			else if(bestOver >= diff * (double)0.84f) ret = 25;
			else if(bestOver >= diff * (double)0.68f) ret = 16;
			else ret = 5;
		} else if(bestdiff >= diff * (double)0.4f) {
			if(bestOver == diff) ret = 34;
			else if(bestOver >= diff * (double)0.84f) ret = 21;
			else if(bestOver >= diff * (double)0.68f) ret = 14;
			else ret = 4;
		} else if(bestdiff >= diff * (double)0.3f) {
			if(bestOver == diff) ret = 32;
			else if(bestOver >= diff * (double)0.88f) ret = 18;
			else if(bestOver >= diff * (double)0.67f) ret = 15;
			else ret = 3;
		} else if(bestdiff >= diff * (double)0.2f) {
			if(bestOver == diff) ret = 31;
			else if(bestOver >= diff * (double)0.88f) ret = 17;
			else if(bestOver >= diff * (double)0.67f) ret = 11;
			else ret = 0;
		} else if(bestdiff >= diff * (double)0.1f) {
			if(bestOver == diff) ret = 30;
			else if(bestOver >= diff * (double)0.88f) ret = 12;
			else if(bestOver >= diff * (double)0.67f) ret = 7;
			else ret = 0;
		} else if(bestdiff > 0) {
			ret = bestOver >= diff * (double)0.67f ? 6 : 2;
		} else {
			ret = bestOver >= diff * (double)0.67f ? 1 : 0;
		}
	}
	return ret;
}

// cigar_md's fast path as a bt2x_sam_req: the printed edits (ned() order; mirrored for the
// reverse strand) are mismatches in increasing read order, so the CIGAR is one M run and MD
// interleaves match runs and reference characters; false otherwise (the host formats it).
bool mm_only_tail(size_t rdlen, bool fw, const uint32_t* ned0, size_t nedn, bt2x_sam_req& q) {
	if(rdlen == 0) return false;
	uint32_t prev = 0;
	for(size_t k = 0; k < nedn; k++) {
		// invert_poss for the reverse strand: reversed order, position rdlen - pos - 1
		const uint32_t e = fw ? ned0[k] : ned0[nedn - 1 - k];
		if(e_type(e) != ET_MM) return false;
		const uint32_t p = fw ? e_pos(e) : (uint32_t)(rdlen - e_pos(e) - 1);
		if(p >= rdlen || (k && p <= prev)) return false;
		q.mm_pos[k] = (uint16_t)p;
		q.mm_chr[k] = (uint8_t)e_chr(e);
		prev = p;
	}
	q.nmm = (uint8_t)nedn;
	return true;
}

// isspace in the C locale (the reference's): ' ', \t, \n, \v, \f, \r
inline bool c_space(unsigned char ch) { return ch == ' ' || (ch >= '\t' && ch <= '\r'); }

void append_name(std::string& o, const std::string& name) {   // SamConfig::printReadName
	const size_t n = std::min<size_t>(name.size(), 255);
	size_t k = 0;
	while(k < n && !c_space((unsigned char)name[k])) k++;
	o.append(name.data(), k);
}

void append_refname(std::string& o, const std::string& name) {   // SamConfig::printRefName
	size_t k = 0;
	while(k < name.size() && !c_space((unsigned char)name[k])) k++;
	o.append(name.data(), k);
}

void append_seq(std::string& o, const std::vector<uint8_t>& s) {
	if(s.empty()) { o.push_back('*'); return; }
	const size_t b = o.size(), n = s.size();
	o.resize(b + n);
	char* d = &o[b];
	const uint8_t* c = s.data();
	size_t i = 0;
#ifdef __AVX2__
	// codes 0-4 through a byte shuffle, 32 a step
	const __m256i tab = _mm256_setr_epi8('A', 'C', 'G', 'T', 'N', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
	                                     'A', 'C', 'G', 'T', 'N', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
	for(; i + 32 <= n; i += 32)
		_mm256_storeu_si256(reinterpret_cast<__m256i*>(d + i),
		                    _mm256_shuffle_epi8(tab, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(c + i))));
#endif
	for(; i < n; i++) d[i] = "ACGTN"[c[i]];
}

// AlnSinkWrap::finishRead, unpaired branch (aln_sink.cpp:643-1384) -> one SAM record in
// `o` (AlnSinkSam::appendMate, aln_sink.cpp:1889-2090; tags per sam.cpp:121-730).
// gpu (optional): an aligned record whose printed edits are mismatches only gets its head
// (name through MAPQ) in `o` and its tail as *gpu (bt2x_sam_tails: CIGAR, SEQ, QUAL and
// the tags, from the read store; text_off and slot are the caller's); returns true then.
bool finish_read(const Params& p, const RefInfo& ref, const Read& rd, Sink& sk, Rng& rnd,
                 const std::vector<uint32_t>& edbuf, bool* aligned, bool* rep, std::string& o,
                 bt2x_sam_req* gpu = nullptr) {
	// ReportingState::finish + getReport
	if(!sk.doneUnpair) {
		sk.doneUnpair = true;
		sk.exitUnpair = sk.n > 0 ? Sink::EXIT_WITH_ALIGNMENTS : Sink::EXIT_NO_ALIGNMENTS;
	}
	uint64_t nunpair = 0;
	bool unpairMax = false;
	if(sk.n > 0) {
		if(sk.exitUnpair == Sink::EXIT_SHORT_CIRCUIT_M) { unpairMax = true; nunpair = 1; }
		else if(sk.exitUnpair == Sink::EXIT_WITH_ALIGNMENTS) nunpair = std::min<uint64_t>(sk.n, 1);
	}
	o.clear();
	// one allocation per record at most (name, SEQ, QUAL, CIGAR/MD and the tags)
	o.reserve(rd.name.size() + 2 * rd.length() + 384);
	append_name(o, rd.name);
	if(nunpair == 0) {
		*aligned = false; *rep = unpairMax;
		o += "\t4\t*\t0\t0\t*\t*\t0\t0\t";
		append_seq(o, rd.fw);
		o.push_back('\t');
		if(rd.qual.empty()) o.push_back('*'); else o += rd.qual;
		o += "\tYT:Z:UU\tYF:Z:LN\n";
		return false;
	}
	// selectByScore (aln_sink.cpp:1477-1640): sort by score desc (ties by index desc),
	// shuffle equal-score streaks with the read's RNG
	const size_t sz = sk.rs.size();
	thread_local std::vector<std::pair<int64_t, size_t>> buf;
	buf.resize(sz);
	for(size_t i = 0; i < sz; i++) buf[i] = {sk.rs[i].score, i};
	// descending (score, index): the reverse of the stable ascending sort by score, and the
	// pairs are distinct, so an unstable sort gives it without stable_sort's temporary buffer
	std::sort(buf.begin(), buf.end(), std::greater<std::pair<int64_t, size_t>>());
	auto shuffle = [&](size_t begin, size_t num) {
		if(num < 2) return;
		size_t left = num;
		for(size_t i = begin; i < begin + num - 1; i++) {
			const size_t rndi = rnd.nextSizeT() % left;
			if(rndi > 0) std::swap(buf[i], buf[i + rndi]);
			left--;
		}
	};
	size_t streak = 0;
	for(size_t i = 1; i < buf.size(); i++) {
		if(buf[i].first == buf[i - 1].first) { if(streak == 0) streak = 1; streak++; }
		else { if(streak > 1) shuffle(i - streak, streak); streak = 0; }
	}
	if(streak > 1) shuffle(buf.size() - streak, streak);
	// Every reported AlnRes shares the read's edit buffer (DList copies keep the source's
	// storage pointer, ds.h:979-1040): the record shows its first ned().size() entries as
	// they stand now.
	const AlnRes& r = sk.rs[buf[0].second];
	const uint32_t* ned = edbuf.data();
	const size_t nedn = std::min<size_t>(r.nedit, edbuf.size());
	const int64_t bestU = r.score;
	const bool hasSec = buf.size() > 1;
	const int64_t secU = hasSec ? sk.rs[buf[1].second].score : 0;
	*aligned = true; *rep = unpairMax;
	if(gpu && nedn <= BT2X_SAM_MAX_MM && !rd.qual.empty() && rd.length() <= BT2X_STORE_MAX_LEN &&
	   mm_only_tail(rd.length(), r.fw, ned, nedn, *gpu)) {
		o += r.fw ? "\t0\t" : "\t16\t";
		append_refname(o, ref.name((size_t)r.refid));
		o.push_back('\t');
		append_int(o, r.refoff + 1);
		o.push_back('\t');
		append_int(o, mapq_v2(p, rd.length(), bestU, hasSec, secU));
		o.push_back('\t');
		gpu->rdlen = (uint16_t)rd.length();
		gpu->fw = r.fw ? 1 : 0;
		gpu->as = (int32_t)r.score;
		gpu->has_xs = hasSec ? 1u : 0u;
		gpu->xs = (int32_t)secU;
		gpu->xn = (uint32_t)r.refns;
		return true;
	}
	thread_local std::string cig, md;
	cig.clear(); md.clear();
	cigar_md(rd, r.fw, ned, nedn, cig, md);
	// record
	o += r.fw ? "\t0\t" : "\t16\t";
	append_refname(o, ref.name((size_t)r.refid));
	o.push_back('\t');
	append_int(o, r.refoff + 1);
	o.push_back('\t');
	append_int(o, mapq_v2(p, rd.length(), bestU, hasSec, secU));
	o.push_back('\t');
	o += cig;
	o += "\t*\t0\t0\t";
	append_seq(o, r.fw ? rd.fw : rd.rc);
	o.push_back('\t');
	o += (r.fw ? rd.qual : rd.qualRev);
	o += "\tAS:i:"; append_int(o, r.score);
	if(hasSec) { o += "\tXS:i:"; append_int(o, secU); }
	o += "\tXN:i:"; append_int(o, r.refns);
	size_t num_mm = 0, num_go = 0, num_gx = 0;
	for(size_t i = 0; i < nedn; i++) {
		const uint32_t t = e_type(ned[i]);
		if(t == ET_MM) num_mm++;
		else if(t == ET_READ_GAP) {
			num_go++; num_gx++;
			while(i < nedn - 1 && e_pos(ned[i + 1]) == e_pos(ned[i]) && e_type(ned[i + 1]) == ET_READ_GAP) { i++; num_gx++; }
		} else if(t == ET_REF_GAP) {
			num_go++; num_gx++;
			while(i < nedn - 1 && e_pos(ned[i + 1]) == e_pos(ned[i]) + 1 && e_type(ned[i + 1]) == ET_REF_GAP) { i++; num_gx++; }
		}
	}
	o += "\tXM:i:"; append_int(o, num_mm);
	o += "\tXO:i:"; append_int(o, num_go);
	o += "\tXG:i:"; append_int(o, num_gx);
	o += "\tNM:i:"; append_int(o, nedn);
	o += "\tMD:Z:"; o += md;
	o += "\tYT:Z:UU\tYF:Z:LN\n";
	return false;
}

// SwAligner::initRef's problem for key k (the window, BitPairReference::getStretch, is
// fetched when the scheduler gathers the launch).
void pose_dp(const Params& P, std::vector<DpWork>& dps, const DpKey& k, size_t rdlen, int nceil) {
	dps.emplace_back();
	DpWork& d = dps.back();
	d.key = k;
	std::memset(&d.in, 0, sizeof(d.in));
	d.in.refl = k.refl;
	d.in.rdlen = (uint16_t)rdlen;
	d.in.ncol = (uint16_t)k.ncol;
	const bool i16 = P.dpI16(k.minsc);
	if(i16 && k.minsc < -32767) throw std::runtime_error("minimum score below the i16 kernel's range");
	d.in.minsc = (int16_t)std::max<int64_t>(k.minsc, i16 ? -32767 : -254);
	d.in.flags = i16 ? BT2X_DP_I16 : 0;
	d.in.nceil = (int16_t)nceil;
	d.in.triml = (uint16_t)k.triml; d.in.corel = (uint16_t)k.corel; d.in.corer = (uint16_t)k.corer;
	d.in.fw = k.fw ? 1 : 0;
}

long find_memo(const std::vector<DpMemo>& memo, const DpKey& k) {
	for(size_t i = 0; i < memo.size(); i++) if(memo[i].key == k) return (long)i;
	return -1;
}

} // namespace

int ExtendWalk::next(int64_t minsc, DpKey& k) {
	const Params& P = *P_;
	const size_t n = (uint16_t)nsat_;                       // gws_size is a uint16_t
	for(;;) {
		if(!inPass_) {                                       // while(neltLeft > 0)
			if(neltLeft_ == 0) return EXTEND_EXHAUSTED_CANDIDATES;
			if(minsc == 0) return EXTEND_PERFECT_SCORE;
			inPass_ = true; i_ = 0; first_ = true;
		}
		if(i_ >= n) { inPass_ = false; continue; }
		const bt2x_sat& sp = sat_[i_];
		const bool is_small = sp.rand_n < kNsm;
		if(rands_[i_].done() || !(first_ || is_small)) { i_++; first_ = true; continue; }
		if(minsc == 0) return EXTEND_PERFECT_SCORE;
		if(prm_->nExDps >= P.mxDp || prm_->nMateDps >= P.mxDp) return EXTEND_EXCEEDED_HARD_LIMIT;
		if(prm_->nExUgs >= P.mxUg || prm_->nMateUgs >= P.mxUg) return EXTEND_EXCEEDED_HARD_LIMIT;
		if(prm_->nExIters >= P.mxIter) return EXTEND_EXCEEDED_HARD_LIMIT;
		prm_->nExIters++;
		first_ = false;
		const bool fw = BT2X_SAT_FW(sp) != 0;
		uint32_t rdoff = sp.rdoff;
		if(!fw) rdoff = (uint32_t)(rdlen_ - rdoff - BT2X_SAT_LEN(sp));
		const uint16_t elt = rands_[i_].next(*rnd_);
		const bt2x_elt& wr = (*res_)[(*firstRow_)[i_] + elt];
		neltLeft_--;
		// (no fragment: tidx, toff and tlen stay 0, the caller's initial values,
		// aligner_sw_driver.cpp:392)
		const uint32_t wt = bt2x_elt_tidx(wr);
		const bool none = wt == BT2X_NO_TIDX;
		const int64_t tidx = none ? 0 : (int64_t)wt;
		const int64_t toff = (int64_t)bt2x_elt_toff(wr), tlen = none ? 0 : (int64_t)plen_[wt];
		const int64_t refoff = toff - (int64_t)rdoff;
		const Coord refcoord(tidx, refoff, fw);
		if(seen_->locusPresent(refcoord)) { prm_->nRedundants++; continue; }
		// DynProgFramer::frameSeedExtensionRect, trimToRef (dp_framer.cpp:81-129)
		if(minsc != gapMinsc_) {
			const int readGaps = P.maxReadGaps(minsc), refGaps = P.maxRefGaps(minsc);
			maxgap_ = std::min((size_t)std::max(readGaps, refGaps), P.maxhalf);
			gapMinsc_ = minsc;
		}
		const size_t maxgap = maxgap_;
		const int64_t refl_pre = refoff - 2 * (int64_t)maxgap;
		const int64_t refr_pre = refoff + ((int64_t)rdlen_ - 1) + 2 * (int64_t)maxgap;
		size_t triml = 0, trimr = 0;
		if(refr_pre >= tlen) trimr = (size_t)(refr_pre - (tlen - 1));
		if(refl_pre < 0) triml = (size_t)(-refl_pre);
		const int64_t refl = refl_pre + (int64_t)triml, refr = refr_pre - (int64_t)trimr;
		const size_t corel = maxgap, corer = corel + 2 * maxgap;
		seen_->add(Interval(refcoord, 1));
		if(refr < refl) continue;                            // entirely trimmed
		// SwAligner::initRef (aligner_sw.cpp:117-229)
		const size_t ncol = (size_t)(refr - refl + 1);
		if(ncol + 1 > BT2X_MAX_COLS) {
			prm_->nExDpFails++; prm_->nDpFail++;
			return EXTEND_EXCEEDED_HARD_LIMIT;
		}
		seen_->add(Interval(Coord(tidx, refl_pre + (int64_t)corel, fw), (int64_t)(corer - corel + 1)));
		k.tidx = tidx; k.refl = refl; k.minsc = minsc; k.ncol = (uint32_t)ncol;
		k.triml = (uint32_t)triml; k.corel = (uint32_t)corel; k.corer = (uint32_t)corer; k.fw = fw;
		return PROBLEM;
	}
}

void host_round(const bt2x_round_in& in, const bt2x_seed_in* sin, const bt2x_seed_out* sout, const bt2x_exrange* exr,
                uint32_t maxelt, Rng& rnd, RoundScratch& w, bt2x_round_out& out, std::vector<bt2x_sat>& sats,
                std::vector<bt2x_resolve_in>& rows, std::vector<bt2x_exrange>& exr_out) {
	std::memset(&out, 0, sizeof out);
	const uint32_t numOffs = in.num_offs, interval = in.interval, offset = in.offset, L = in.seedlen;
	const size_t exr0 = exr_out.size();
	// searchAllSeedsFinalize + SeedResults::add (aligner_seed.cpp:508-540)
	SeedHitsHip& hits = w.hits;
	hits.reset(numOffs);
	w.cacheNlex.clear();
	for(uint32_t k = 0; k < in.nseeds; k++) {
		const bt2x_seed_out& d = sout[k];
		if(!d.need_reporting) continue;
		const bool fw = sin[k].read_off == in.read_off;
		const uint32_t depth = fw ? sin[k].seed_off : (uint32_t)(in.rdlen - sin[k].seed_off - L);
		hits.add((depth - offset) / interval, fw, d);
		bool have = false;
		for(auto& e : w.cacheNlex) if(e.first == d.topf) { have = true; break; }
		if(!have) w.cacheNlex.push_back({d.topf, d.nlex});
	}
	out.nonz = (uint32_t)hits.nonzeroOffsets();
	out.num_elts = hits.numElts();
	if(out.nonz == 0) {
		out.status = BT2X_ROUND_NO_HITS;
		out.rnd_last = rnd.last; out.rnd_lastoff = rnd.lastOff;
		return;
	}
	hits.rankSeedHits(rnd, false);
	// prioritizeSATups (aligner_sw_driver.cpp:61-260)
	std::vector<SatPos>& satpos2 = w.satpos2;
	satpos2.clear();
	size_t nelt = 0, nsmall = 0;
	const size_t nsm = 5;
	auto covered = [&](const bt2x_exrange& er, bool fw, uint32_t rdoff, uint64_t size) {
		return (er.fw != 0) == fw && er.off <= rdoff && (uint64_t)er.off + er.len >= (uint64_t)rdoff + L && size <= er.sz;
	};
	for(size_t r = 0; r < hits.nonzeroOffsets(); r++) {
		uint32_t offidx = 0; bool fw = true;
		const SeedHitsHip::Hit& h = hits.hitsByRank(r, offidx, fw);
		const uint32_t rdoff = offidx * interval + offset;           // idx2off
		SatPos sp;
		sp.topf = h.topf; sp.size = h.numElts(); sp.key = h.topf;
		for(auto& e : w.cacheNlex) if(e.first == h.topf) { sp.nlex = e.second; break; }
		if(sp.size == 0) continue;
		bool skip = false;
		for(uint32_t q = 0; q < in.nexr && !skip; q++) skip = covered(exr[q], fw, rdoff, sp.size);
		for(size_t q = exr0; q < exr_out.size() && !skip; q++) skip = covered(exr_out[q], fw, rdoff, sp.size);
		if(!skip) for(const SatPos& o : satpos2) skip |= (o.key == sp.key);
		if(skip) continue;
		nelt += sp.size;
		sp.origSz = sp.size;
		sp.fw = fw; sp.offidx = offidx; sp.rdoff = rdoff; sp.seedlen = L;
		satpos2.push_back(sp);
		if(sp.size <= nsm) nsmall++;
		if(sp.nlex > 0) {
			bt2x_exrange er;
			std::memset(&er, 0, sizeof er);
			er.off = rdoff - (fw ? sp.nlex : 0);
			er.len = (uint16_t)(L + sp.nlex);
			er.sz = sp.size;
			er.fw = fw ? 1 : 0;
			exr_out.push_back(er);
		}
	}
	std::stable_sort(satpos2.begin(), satpos2.end());
	const size_t sat0 = sats.size();
	auto emit = [&](const SatPos& sp, uint64_t first, uint32_t n) {
		bt2x_sat st;
		st.rdoff = (uint16_t)sp.rdoff; st.rand_n = (uint8_t)n; st.fwlen = BT2X_SAT_FWLEN(sp.fw, L);
		sats.push_back(st);
		for(uint32_t e = 0; e < n; e++) {
			bt2x_resolve_in ri;
			std::memset(&ri, 0, sizeof(ri));
			ri.row = first + e;
			ri.qlen = L;
			rows.push_back(ri);
		}
	};
	size_t added = 0;
	for(size_t j = 0; j < nsmall && added < maxelt; j++) {
		emit(satpos2[j], satpos2[j].topf, (uint32_t)satpos2[j].size);
		added += satpos2[j].size;
	}
	if(!(added >= maxelt || nsmall == satpos2.size())) {
		w.rows.init(satpos2, nsmall, satpos2.size());
		std::vector<Random1toN>& rands = w.prioRands;
		if(rands.size() < satpos2.size()) rands.resize(satpos2.size());
		for(size_t q = 0; q < satpos2.size(); q++) rands[q].reset();
		while(added < maxelt && added < nelt) {
			const size_t ri = w.rows.next(rnd) + nsmall;
			if(!rands[ri].inited()) rands[ri].init((uint16_t)satpos2[ri].size, false);
			const size_t rr = rands[ri].next(rnd);
			if(rands[ri].done()) w.rows.finishedRange(ri - nsmall);
			emit(satpos2[ri], satpos2[ri].topf + rr, 1);
			added++;
		}
	}
	out.status = BT2X_ROUND_OK;
	out.nsat = (uint32_t)(sats.size() - sat0);
	out.nelt = (uint32_t)added;
	out.nexr = (uint32_t)(exr_out.size() - exr0);
	out.rnd_last = rnd.last; out.rnd_lastoff = rnd.lastOff;
}

// ---------------------------------------------------------------- SAM header

std::string Aligner::header() const {
	std::string o = "@HD\tVN:1.5\tSO:unsorted\tGO:query\n";
	for(size_t i = 0; i < ref_.nrefs(); i++) {
		o += "@SQ\tSN:";
		append_refname(o, ref_.name(i));
		o += "\tLN:" + std::to_string(ref_.len(i)) + "\n";
	}
	return o;
}

// ------------------------------------------------------------- one read

ReadTask Aligner::align_read(ReadCtx* c) {
	const Params& P = p_;
	Read& rd = c->rd;
	const size_t rdlen = rd.length();
	// P0, bt2_search.cpp:2467-2553
	int64_t minsc = P.scoreMin.f<int64_t>((double)rdlen);
	c->warn.clear();
	// printEEScoreMsg (bt2_search.cpp:1870-1891, 2484-2492): the same "positive number"
	// text for the stock build's -254 clamp
	auto ee_warn = [&] {
		if(!P.quiet)
			c->warn += "Warning: minimum score function gave positive number in --end-to-end mode for read '" + rd.name +
			           "; setting to 0 instead\n";
	};
	if(minsc > 0) { ee_warn(); minsc = 0; }
	else if(minsc < -254 && !P.i16build) { ee_warn(); minsc = -254; }        // stock build only
	PH_START();
	Rng rnd;
	rnd.init(rd.seed);
	const int interval = std::max(P.msIval.f<int>((double)rdlen), 1);
	const int swNceil = P.nCeil.f<int>((double)rdlen);      // SwAligner::initRead's nceil
	Sink& sink = c->sink;
	sink.reset(P.mhits);
	c->seenDiags.clear();
	c->redAnchor.init(rdlen);
	c->edbuf.clear();
	c->memo.clear(); c->recs.clear(); c->edits.clear();
	c->exRange.clear();
	c->ndp_used = c->ntight = 0;
	c->aligned = c->repetitive = false;
	Prm prm;
	const uint32_t nrounds = (uint32_t)std::min<int>(P.nSeedRounds, interval);
	const uint32_t L = (uint32_t)std::min<size_t>((size_t)P.multiseedLen, rdlen);
	// reads the u8 DP cannot hold never align (initRead, aligner_sw.cpp:59)
	const bool dpOk = rdlen >= 1 && rdlen <= BT2X_MAX_ROWS;
	PH(0);
	for(uint32_t roundi = 0; roundi < nrounds && dpOk; roundi++) {
		const uint32_t offset = (uint32_t)((interval * roundi) / nrounds);
		if(offset > 0 && (size_t)P.multiseedLen + offset > rdlen) break;
		// instantiateSeeds (aligner_seed.cpp:411-447): fw seed i at depth, rc seed at rdlen-depth-L
		const uint32_t nseeds = (rdlen - offset > L) ? 1 + (uint32_t)((rdlen - offset - L) / interval) : 1;
		// the seed list; with the seeds instantiated on the GPU (and the round not handed
		// back) only its length: every seed of an N-free read, else the ones clear of an N
		auto instantiate = [&](bool list) {
			c->seed_in.clear();
			uint32_t nvalid = 0;
			for(int fwi = 0; fwi < 2; fwi++) {
				const bool fw = fwi == 0;
				if((fw && P.nofw) || (!fw && P.norc)) continue;
				if(!list && !rd.nN) { nvalid += nseeds; continue; }
				const std::vector<uint8_t>& s = fw ? rd.fw : rd.rc;
				for(uint32_t i = 0; i < nseeds; i++) {
					const uint32_t depth = i * interval + offset;
					const uint32_t st = fw ? depth : (uint32_t)(rdlen - depth - L);
					bool ok = true;
					if(rd.nN) for(uint32_t k = 0; k < L; k++) if(s[st + k] > 3) { ok = false; break; }
					if(!ok) continue;
					nvalid++;
					if(!list) continue;
					bt2x_seed_in si;
					std::memset(&si, 0, sizeof(si));
					si.read_off = fw ? 0 : rdlen;
					si.seed_off = (uint8_t)st;
					si.seed_len = (uint8_t)L;
					c->seed_in.push_back(si);
				}
			}
			return nvalid;
		};
		const bool gpu_seeds = gpu_round_ && dseeds_;
		const uint32_t nvalid = instantiate(!gpu_seeds);
		PH(1);
		if(nvalid == 0) break;                                       // no seed, no hit: done
		// the rest of the round up to extendSeeds: on the GPU (bt2x_seed_round), or for a
		// read it hands back, as seed search + host_round + SA resolution
		bt2x_round_in& q = c->round_in;
		std::memset(&q, 0, sizeof q);
		q.rnd_last = rnd.last; q.rnd_lastoff = rnd.lastOff;
		q.nseeds = (uint16_t)nvalid; q.num_offs = (uint16_t)nseeds; q.rdlen = (uint16_t)rdlen;
		q.interval = (uint16_t)interval; q.offset = (uint16_t)offset; q.seedlen = (uint16_t)L;
		q.seedflags = (uint16_t)((P.nofw ? 1 : 0) | (P.norc ? 2 : 0));
		q.nexr = (uint16_t)c->exRange.size();
		c->sats.clear(); c->exNew.clear();
		bool redo = !gpu_round_;
		if(!redo) {
			co_await Awaiter{c, REQ_ROUND};                          // fills round_out, sats, elts, exNew
			PH_START();
			redo = c->round_out.status == BT2X_ROUND_REDO;
			if(redo) { c->sats.clear(); c->exNew.clear(); }
			else { rnd.last = c->round_out.rnd_last; rnd.lastOff = c->round_out.rnd_lastoff; }
		}
		if(redo) {
			if(gpu_seeds) instantiate(true);                         // the host searches the seeds itself
			co_await Awaiter{c, REQ_SEED};
			PH_START();
			q.read_off = 0;                                          // seeds: patFw at 0, patRc at rdlen
			c->res_in.clear();
			host_round(q, c->seed_in.data(), c->seed_out.data(), c->exRange.data(), (uint32_t)P.mxIter, rnd, c->rs,
			           c->round_out, c->sats, c->res_in, c->exNew);
			if(!c->res_in.empty()) co_await Awaiter{c, REQ_RESOLVE};
			PH_START();
		}
		const bt2x_round_out& ro = c->round_out;
		if(ro.status == BT2X_ROUND_NO_HITS) break;                   // no seed hits: done
		c->exRange.insert(c->exRange.end(), c->exNew.begin(), c->exNew.end());
		// the extension list (SATupleAndPos: the round's bt2x_sat entries) and each entry's
		// first element
		c->firstRow.resize(c->sats.size());
		uint32_t e0 = 0;
		for(size_t k = 0; k < c->sats.size(); k++) { c->firstRow[k] = e0; e0 += c->sats[k].rand_n; }
		const size_t nelt_ = ro.nelt;
		PH(4);

		// -------------------------------------------------- extendSeeds (:278-631)
		int ret;
		{
			prm.nDpFail = 0;
			const int64_t perfectScore = 0;
			c->walk.reset(P, c->sats, c->firstRow, c->elts, ref_.lens(), nelt_, rdlen);
			c->walk.bind(&rnd, &prm, &c->seenDiags);
			PH(13);
			for(;;) {
				DpKey key;
				ret = c->walk.next(minsc, key);
				PH(5);
				if(ret != ExtendWalk::PROBLEM) break;
				long mi = find_memo(c->memo, key);
				PH(14);
				if(mi < 0) {
					// pose this problem and the ones the walk reaches next if each of them
					// fails (a copy of the walk over copies of the state it advances)
					c->dps.clear();
					pose_dp(P, c->dps, key, rdlen, swNceil);
					if(P.lookahead > 1) {
						Rng rnd2 = rnd;
						Prm prm2 = prm;
						c->seen2.clear(&c->seenDiags);
						c->ahead = c->walk;
						c->ahead.bind(&rnd2, &prm2, &c->seen2);
						while(c->dps.size() < P.lookahead && c->ahead.failed()) {
							DpKey k2;
							if(c->ahead.next(minsc, k2) != ExtendWalk::PROBLEM) break;
							const long m = find_memo(c->memo, k2);
							if(m >= 0) {
								if(c->memo[(size_t)m].out.status != 0) break;    // a known success: stop guessing
								continue;
							}
							bool dup = false;
							for(const DpWork& d : c->dps) dup = dup || d.key == k2;
							if(!dup) pose_dp(P, c->dps, k2, rdlen, swNceil);
						}
					}
					PH(6);
					co_await Awaiter{c, REQ_DP};
					PH_START();
					c->dps.clear();
					mi = find_memo(c->memo, key);
				}
				c->ndp_used++;
				const DpMemo d = c->memo[(size_t)mi];
				if(d.out.status == 0) {
					if(!c->walk.failed()) { ret = EXTEND_EXCEEDED_SOFT_LIMIT; break; }
					continue;
				}
				prm.nExDps++;
				prm.nExDpSuccs++;
				if(prm.nDpFail > prm.nDpFailStreak) prm.nDpFailStreak = prm.nDpFail;
				prm.nDpFail = 0;
				bool fulfilled = false;
				const int64_t minsc_posed = minsc;
				for(uint32_t k = 0; k < d.out.nrec; k++) {            // while(!swa.done()) nextAlignment
					const bt2x_aln_rec& rec = c->recs[d.rec0 + k];
					// -M tightening below raises minsc between the calls of this problem, but the
					// record sequence needs no re-filtering: nextAlignment's score filter compares
					// the candidate's raw cell value (DpBtCandidate::score = lr: 0..255 for u8,
					// aligner_swsse_ee_u8.cpp:519; >= 0 for every i16 candidate, i16.cpp:527)
					// with minsc <= 0 (aligner_sw.cpp:274), so it never fires and the calls
					// proceed exactly as posed (tests/test_e2e.py, tandem-repeat fixture).
					if(minsc != minsc_posed) c->ntight++;
					replay_backtrace_draws(rnd, rec.ntries, P.dpI16(key.minsc));
					// the call's writes to the read's edit buffer (bt2x.h)
					if(c->edbuf.size() < rec.nbuf) c->edbuf.resize(rec.nbuf);
					std::copy(c->edits.begin() + rec.edit_off, c->edits.begin() + rec.edit_off + rec.nbuf, c->edbuf.begin());
					if(!rec.ok) break;
					AlnRes res;
					res.score = rec.score;
					res.refid = key.tidx;
					res.refoff = rec.refoff;
					res.fw = key.fw;
					res.nedit = rec.nedit;
					res.refns = rec.refns;
					const uint32_t* ned = c->edits.data() + rec.edit_off;
					// (the alignment lies inside [0, tlen): the rectangle is trimmed to the reference)
					if(c->redAnchor.overlap(res, ned, rec.nedit)) continue;
					c->redAnchor.add(res, ned, rec.nedit);
					if(sink.report(res)) { fulfilled = true; break; }
					if(P.tighten > 0 && sink.hasSecondBest()) {
						if(P.tighten == 1) {
							if(sink.best >= minsc) {
								minsc = sink.best;
								if(minsc < perfectScore && sink.best == sink.best2) minsc++;
							}
						} else if(P.tighten == 2) {
							if(sink.best2 >= minsc) { minsc = sink.best2; if(minsc < perfectScore) minsc++; }
						} else {
							const int64_t diff = sink.best - sink.best2;
							const int64_t bot = sink.best2 + ((diff * 3) / 4);
							if(bot >= minsc) { minsc = bot; if(minsc < perfectScore) minsc++; }
						}
					}
				}
				PH(7);
				if(fulfilled) { ret = EXTEND_POLICY_FULFILLED; break; }
			}
		}
		if(ret == EXTEND_EXHAUSTED_CANDIDATES || ret == EXTEND_EXCEEDED_SOFT_LIMIT || ret == EXTEND_POLICY_FULFILLED) {
			if(c->round_out.num_elts / c->round_out.nonz < P.seedBoostThresh) break;   // averageHitsPerSeed
			if(sink.done()) break;                                                  // doneWithMate
		} else {
			break;
		}
	}
	PH(5);
	c->sam_gpu = finish_read(P, ref_, rd, sink, rnd, c->edbuf, &c->aligned, &c->repetitive, c->sam,
	                         gpu_sam_ && c->in_store ? &c->sam_req : nullptr);
	if(c->sam_gpu) c->sam_req.slot = c->slot;
	// the finishRead counter update (aln_sink.cpp:994-1013): rs1u_ holds every alignment found
	c->met_kind = c->repetitive ? 3 : !c->aligned ? 0 : sink.rs.size() == 1 ? 1 : 2;
	PH(8);
	c->req = REQ_NONE;
	c->done = true;
	co_return;
}

// ------------------------------------------------------------- scheduler

namespace {
double now_s() {
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}

// A cohort's read contexts are cold when a pass over the cohort reaches them (its host
// state is far larger than the caches): the loops below fetch a read's leading lines (and,
// before a resume, its coroutine frame) a few reads ahead.  BT2X_HOST_PREFETCH=0: off.
namespace {
bool host_prefetch() {
	static const bool on = [] { const char* e = std::getenv("BT2X_HOST_PREFETCH"); return !(e && e[0] == '0'); }();
	return on;
}
bool host_prefetch_read() {                     // BT2X_HOST_PREFETCH_READ=0: off
	static const bool on = [] { const char* e = std::getenv("BT2X_HOST_PREFETCH_READ"); return !(e && e[0] == '0'); }();
	return on;
}
// BT2X_HOST_PREFETCH_CTX=0: a resume prefetches only the context's first lines and the
// arenas its results go to; else the whole context ahead and, three reads ahead, the
// walk's per-read state (cold since the read's last resume a cohort ago)
bool host_prefetch_full() {
	static const bool on = [] { const char* e = std::getenv("BT2X_HOST_PREFETCH_CTX"); return !(e && e[0] == '0'); }();
	return on;
}
bool host_prefetch_frame() {                   // BT2X_HOST_PREFETCH_FRAME=0: off
	static const bool on = [] { const char* e = std::getenv("BT2X_HOST_PREFETCH_FRAME"); return !(e && e[0] == '0'); }();
	return on;
}
bool host_prefetch_more() {                    // BT2X_HOST_PREFETCH_MORE=0: off
	static const bool on = [] { const char* e = std::getenv("BT2X_HOST_PREFETCH_MORE"); return !(e && e[0] == '0'); }();
	return on;
}
inline void prefetch_ctx(const ReadCtx* c, bool frame) {
	for(int k = 0; k < 4; k++) __builtin_prefetch(reinterpret_cast<const char*>(c) + 64 * k);
	if(frame)
		for(int k = 0; k < 8; k++) __builtin_prefetch(c->frame_ + 64 * k);
}
// the context's members past the first lines (vector headers, walk and sink state)
inline void prefetch_ctx_rest(const ReadCtx* c) {
	for(size_t k = 256; k < offsetof(ReadCtx, frame_); k += 64) __builtin_prefetch(reinterpret_cast<const char*>(c) + k);
	if(host_prefetch_frame())                  // the frame past the first 512 bytes
		for(size_t k = 512; k < ReadCtx::kFrameBytes; k += 64) __builtin_prefetch(c->frame_ + k);
}
}

// ----- one launch: gather a cohort's waiting requests, run them, scatter the results

// Classify the cohort's reads by pending request and fill the launch's input buffers
// (one seed, one resolve and one DP launch).  Two parallel passes over chunks of the
// cohort: sizes per chunk, then (after a prefix sum over chunks) the copies; the
// waiting lists keep cohort order, so a launch's layout is deterministic.
void Aligner::gather(Launch& L, const std::vector<ReadCtx*>& cohort) {
	const double tg = now_s();
	constexpr long kChunk = 1024;
	const long n = (long)cohort.size();
	const long nch = (n + kChunk - 1) / kChunk;
	if((long)L.chunks.size() < nch) L.chunks.resize((size_t)nch);
	const bool ref_index = be_.ref_from_index();
	const bool store = be_.read_store();
	const bool dseeds = be_.device_seeds();
	PH_START();
	pool().parallel_for(nch, 1, [&](long ch) {
		Launch::Chunk& C = L.chunks[(size_t)ch];
		C.ws.clear(); C.wr.clear(); C.wd.clear(); C.wn.clear();
		C.sbytes = C.nseed = C.nres = C.dbytes = C.nprob = C.rbytes = C.nbytes = C.nnseed = C.nexr = 0;
		C.pbytes = C.nput = 0;
		const long e = std::min(n, (ch + 1) * kChunk);
		const bool pf = host_prefetch();
		for(long i = ch * kChunk; i < e; i++) {
			ReadCtx* c = cohort[(size_t)i];
			if(pf && i + 4 < e) prefetch_ctx(cohort[(size_t)i + 4], false);
			if(c->req == REQ_SEED) {
				C.ws.push_back(c); C.sbytes += 2 * c->rd.length(); C.nseed += c->seed_in.size();
			} else if(c->req == REQ_RESOLVE) {
				C.wr.push_back(c); C.nres += c->res_in.size();
			} else if(c->req == REQ_DP) {
				C.wd.push_back(c); C.nprob += c->dps.size();
				if(!store) C.dbytes += 2 * c->rd.length();
				if(!ref_index) for(const DpWork& d : c->dps) C.rbytes += d.key.ncol;
			} else if(c->req == REQ_ROUND) {
				C.wn.push_back(c); C.nnseed += c->round_in.nseeds;
				if(!store) C.nbytes += 2 * c->rd.length();
				C.nexr += c->exRange.size();
			}
			// a read a round or DP request brings to the store for the first time
			c->put_now = store && !c->in_store && (c->req == REQ_DP || c->req == REQ_ROUND);
			if(c->put_now) { C.pbytes += 2 * c->rd.length(); C.nput++; }
		}
	});
	PH(10);
	// chunk bases
	uint64_t nws = 0, nwr = 0, nwd = 0, sb = 0, sk = 0, rk = 0, db = 0, pk = 0, rb = 0;
	uint64_t nwn = 0, nb = 0, nk = 0, ne = 0, ppb = 0, npt = 0;
	for(long ch = 0; ch < nch; ch++) {
		Launch::Chunk& C = L.chunks[(size_t)ch];
		C.ws0 = nws; C.sb0 = sb; C.sk0 = sk; C.wr0 = nwr; C.rk0 = rk; C.wd0 = nwd; C.db0 = db; C.pk0 = pk; C.rb0 = rb;
		C.wn0 = nwn; C.nb0 = nb; C.nk0 = nk; C.ne0 = ne; C.pb0 = ppb; C.np0 = npt;
		ppb += C.pbytes; npt += C.nput;
		nws += C.ws.size(); sb += C.sbytes; sk += C.nseed;
		nwr += C.wr.size(); rk += C.nres;
		nwd += C.wd.size(); db += C.dbytes; pk += C.nprob; rb += C.rbytes;
		nwn += C.wn.size(); nb += C.nbytes; nk += C.nnseed; ne += C.nexr;
	}
	L.ws.resize(nws); L.wr.resize(nwr); L.wd.resize(nwd); L.wn.resize(nwn);
	L.round_reads.resize(nb); L.round_seeds.resize(dseeds ? 0 : nk); L.round_in.resize(nwn); L.round_exr.resize(ne);
	L.n_round_seeds = nk;
	L.sr.resize(nws + 1); L.sk.resize(nws + 1); L.rk.resize(nwr + 1);
	L.qb.resize(nwd + 1); L.pb.resize(nwd + 1); L.fb.resize(pk + 1);
	L.sr[nws] = sb; L.sk[nws] = sk; L.rk[nwr] = rk; L.qb[nwd] = db; L.pb[nwd] = pk; L.fb[pk] = rb;
	PH(11);
	L.seed_reads.resize(sb); L.seed_in.resize(sk);
	L.res_in.resize(rk);
	L.dp_reads.resize(db); L.dp_quals.resize(db); L.dp_refs.resize(rb); L.dp_in.resize(pk);
	L.store_packed.resize(ppb); L.store_in.resize(npt);
	pool().parallel_for(nch, 1, [&](long ch) {
		const Launch::Chunk& C = L.chunks[(size_t)ch];
		// read-store puts: the read's patFw codes then its qualities (the GPU derives the
		// reverse complement and the reversed qualities); rounds and DP requests run on
		// rdlen <= BT2X_MAX_ROWS reads only, within BT2X_STORE_MAX_LEN
		uint64_t ppo = C.pb0, pno = C.np0;
		auto put = [&](ReadCtx* c) {
			const size_t len = c->rd.length();
			uint8_t* d = L.store_packed.data() + ppo;
			std::memcpy(d, c->rd.fw.data(), len);
			std::memcpy(d + len, c->rd.qual.data(), len);
			bt2x_store_in si;
			si.off = ppo; si.slot = c->slot; si.len = (uint16_t)len; si.pad = 0;
			L.store_in[pno++] = si;
			ppo += 2 * len;
			c->in_store = true;
		};
		// seeds: patFw+patRc of each read, then its seeds with read_off rebased
		uint64_t sbo = C.sb0, sko = C.sk0;
		for(size_t k = 0; k < C.ws.size(); k++) {
			ReadCtx* c = C.ws[k];
			const size_t i = C.ws0 + k, len = c->rd.length();
			L.ws[i] = c; L.sr[i] = sbo; L.sk[i] = sko;
			std::copy(c->rd.fw.begin(), c->rd.fw.end(), L.seed_reads.begin() + (long)sbo);
			std::copy(c->rd.rc.begin(), c->rd.rc.end(), L.seed_reads.begin() + (long)(sbo + len));
			for(const bt2x_seed_in& q0 : c->seed_in) {
				bt2x_seed_in q = q0;
				q.read_off += sbo;
				L.seed_in[sko++] = q;
			}
			sbo += 2 * len;
		}
		// SA elements
		uint64_t rko = C.rk0;
		for(size_t k = 0; k < C.wr.size(); k++) {
			ReadCtx* c = C.wr[k];
			L.wr[C.wr0 + k] = c; L.rk[C.wr0 + k] = rko;
			std::copy(c->res_in.begin(), c->res_in.end(), L.res_in.begin() + (long)rko);
			rko += c->res_in.size();
		}
		// DP: the read's two orientations (codes and qualities) once per read, one
		// reference window per posed problem (BitPairReference::getStretch)
		uint64_t dbo = C.db0, pko = C.pk0, rbo = C.rb0;
		const bool pf = host_prefetch();
		for(size_t k = 0; k < C.wd.size(); k++) {
			ReadCtx* c = C.wd[k];
			if(pf && k + 3 < C.wd.size()) {                   // the read's codes and qualities
				const ReadCtx* c3 = C.wd[k + 3];
				const Read& r3 = c3->rd;
				if(!store) {
					__builtin_prefetch(r3.fw.data()); __builtin_prefetch(r3.rc.data());
					__builtin_prefetch(r3.qual.data()); __builtin_prefetch(r3.qualRev.data());
				} else if(c3->put_now) {
					__builtin_prefetch(r3.fw.data()); __builtin_prefetch(r3.qual.data());
				}
				__builtin_prefetch(c3->dps.data());
			}
			const size_t i = C.wd0 + k, len = c->rd.length();
			L.wd[i] = c; L.qb[i] = dbo; L.pb[i] = pko;
			if(!store) {
				std::copy(c->rd.fw.begin(), c->rd.fw.end(), L.dp_reads.begin() + (long)dbo);
				std::copy(c->rd.rc.begin(), c->rd.rc.end(), L.dp_reads.begin() + (long)(dbo + len));
				// (memcpy: char -> uint8_t through std::copy is a scalar byte loop)
				std::memcpy(L.dp_quals.data() + dbo, c->rd.qual.data(), len);
				std::memcpy(L.dp_quals.data() + dbo + len, c->rd.qualRev.data(), len);
			} else if(c->put_now) {
				put(c);
			}
			const uint64_t sbase = (uint64_t)c->slot * BT2X_STORE_SLOT_BYTES;
			for(const DpWork& d : c->dps) {
				bt2x_dp_in q = d.in;
				if(store) {                              // store slot: patFw, patRc, qual, qualRev
					q.read_off = sbase + (d.key.fw ? 0 : len);
					q.qual_off = sbase + 2 * len + (d.key.fw ? 0 : len);
				} else {
					q.read_off = q.qual_off = dbo + (d.key.fw ? 0 : len);
				}
				L.fb[pko] = rbo;
				if(ref_index) {                          // the backend cuts the window from the index
					q.ref_off = (uint64_t)d.key.tidx;
					q.flags |= BT2X_DP_REF_TEXT;
				} else {
					q.ref_off = rbo;
					ref_.stretch((uint32_t)d.key.tidx, d.key.refl, d.key.ncol, L.dp_refs.data() + rbo);
					rbo += d.key.ncol;
				}
				L.dp_in[pko++] = q;
			}
			if(!store) dbo += 2 * len;
		}
		// seed rounds: the read, its seeds rebased, its round header, its exRange entries
		uint64_t nbo = C.nb0, nko = C.nk0, neo = C.ne0;
		for(size_t k = 0; k < C.wn.size(); k++) {
			ReadCtx* c = C.wn[k];
			if(pf && k + 3 < C.wn.size()) {
				const ReadCtx* c3 = C.wn[k + 3];
				__builtin_prefetch(c3->rd.fw.data());
				if(store) __builtin_prefetch(c3->rd.qual.data()); else __builtin_prefetch(c3->rd.rc.data());
				if(!dseeds) __builtin_prefetch(c3->seed_in.data());
				if(!c3->exRange.empty()) __builtin_prefetch(c3->exRange.data());
			}
			const size_t i = C.wn0 + k, len = c->rd.length();
			L.wn[i] = c;
			uint64_t roff = nbo;
			if(!store) {
				std::copy(c->rd.fw.begin(), c->rd.fw.end(), L.round_reads.begin() + (long)nbo);
				std::copy(c->rd.rc.begin(), c->rd.rc.end(), L.round_reads.begin() + (long)(nbo + len));
				nbo += 2 * len;
			} else {
				if(c->put_now) put(c);
				roff = (uint64_t)c->slot * BT2X_STORE_SLOT_BYTES;
			}
			bt2x_round_in q = c->round_in;
			q.read_off = roff; q.seed0 = nko; q.exr0 = (uint32_t)neo; q.nexr = (uint16_t)c->exRange.size();
			L.round_in[i] = q;
			if(dseeds) {
				nko += c->round_in.nseeds;               // (instantiated on the GPU)
			} else {
				for(const bt2x_seed_in& q0 : c->seed_in) {
					bt2x_seed_in sq = q0;
					sq.read_off += roff;
					L.round_seeds[nko++] = sq;
				}
			}
			std::copy(c->exRange.begin(), c->exRange.end(), L.round_exr.begin() + (long)neo);
			neo += c->exRange.size();
		}
	});
	PH(12);
	L.t_gather = now_s() - tg;
}

// The launch's backend calls (on the GPU thread when pipelined; launch 1 on the second
// backend when there is one).
void Aligner::execute(Launch& L) {
	Backend& be = (be2_ && &L == &launch_[1]) ? *be2_ : be_;
	L.t_seed = L.t_resolve = L.t_dp = L.t_round = L.t_sam = 0;
	if(!L.sam_req.empty()) {                  // retired reads' record tails, before their slots are reused
		const double t0 = now_s();
		be.sam_tails(L.sam_req, L.sam_text, L.sam_text_bytes, L.sam_lens);
		L.t_sam = now_s() - t0;
	}
	if(!L.store_in.empty()) be.store_put(L.store_packed, L.store_in);   // before the requests that read them
	if(!L.wn.empty()) {
		const double t0 = now_s();
		be.seed_round(L.round_reads, L.round_seeds, L.round_in, L.round_exr, (uint32_t)p_.mxIter, L.round_out,
		              L.round_sats, L.round_elts, L.round_exr_out);
		L.t_round = now_s() - t0;
	}
	if(!L.ws.empty()) {
		const double t0 = now_s();
		be.seed_search(L.seed_reads, L.seed_in, L.seed_out);
		L.t_seed = now_s() - t0;
	}
	if(!L.wr.empty()) {
		const double t0 = now_s();
		be.resolve(L.res_in, L.res_out);
		L.t_resolve = now_s() - t0;
	}
	if(!L.wd.empty()) {
		const double t0 = now_s();
		be.dp_align(L.dp_reads, L.dp_quals, L.dp_refs, L.dp_in, L.dp_out, L.recs, L.edits);
		L.t_dp = now_s() - t0;
	}
}

// Hand every served read its results and resume it until it waits again or finishes.
void Aligner::scatter_resume(Launch& L, RunStats& st) {
	const long nws = (long)L.ws.size(), nwr = (long)L.wr.size(), nwd = (long)L.wd.size(), nwn = (long)L.wn.size();
	if(nwn) {
		st.round_launches++; st.rounds += (uint64_t)nwn; st.t_round += L.t_round;
		st.seeds += L.n_round_seeds;
		for(const bt2x_round_out& o : L.round_out) st.resolves += o.nelt;
	}
	if(nws) { st.seed_launches++; st.seeds += L.seed_in.size(); st.t_seed += L.t_seed; }
	if(nwr) { st.resolve_launches++; st.resolves += L.res_in.size(); st.t_resolve += L.t_resolve; }
	if(nwd) {
		st.dp_launches++; st.dps += L.dp_in.size(); st.t_dp += L.t_dp;
		st.dp_max_launch = std::max<uint64_t>(st.dp_max_launch, L.dp_in.size());
	}
	st.t_backend += L.t_seed + L.t_resolve + L.t_dp + L.t_round;
	L.run.clear();
	L.run.insert(L.run.end(), L.wn.begin(), L.wn.end());
	L.run.insert(L.run.end(), L.ws.begin(), L.ws.end());
	L.run.insert(L.run.end(), L.wr.begin(), L.wr.end());
	L.run.insert(L.run.end(), L.wd.begin(), L.wd.end());
	const long nrun = (long)L.run.size();
	const double t0 = now_s();
	st.t_gather += L.t_gather;
	const bool prefetch = host_prefetch(), full = host_prefetch_full(), more = host_prefetch_more();
	static const long chunk = [] { const char* e = std::getenv("BT2X_SCATTER_CHUNK"); return e ? std::max(1L, std::atol(e)) : 64L; }();
	pool().parallel_for(nrun, chunk, [&](long i) {
		ReadCtx* c = L.run[(size_t)i];
		if(prefetch) {
			if(i + 6 < nrun) {
				const ReadCtx* c6 = L.run[(size_t)i + 6];
				prefetch_ctx(c6, true);
				if(full) prefetch_ctx_rest(c6);
			}
			if(i + 3 < nrun) {                                // the arenas the results are copied into
				const ReadCtx* c3 = L.run[(size_t)i + 3];
				if(full) {
					c3->seenDiags.prefetch(); c3->walk.prefetch();
					__builtin_prefetch(c3->firstRow.data()); __builtin_prefetch(c3->memo.data());
					__builtin_prefetch(c3->dps.data()); __builtin_prefetch(c3->sink.rs.data());
					__builtin_prefetch(c3->edbuf.data());
					if(more) {                                  // the lookahead's copies, the other strand
						c3->seen2.prefetch(); c3->ahead.prefetch();
						__builtin_prefetch(c3->exRange.data());
						__builtin_prefetch(c3->rd.rc.data()); __builtin_prefetch(c3->rd.qualRev.data());
					}
				}
				__builtin_prefetch(c3->elts.data(), 1); __builtin_prefetch(c3->sats.data(), 1);
				__builtin_prefetch(c3->recs.data() + c3->recs.size(), 1);
				__builtin_prefetch(c3->edits.data() + c3->edits.size(), 1);
				// the read itself (a resume that finishes the read formats its record)
				if(host_prefetch_read()) {
					__builtin_prefetch(c3->rd.name.data()); __builtin_prefetch(c3->rd.fw.data());
					__builtin_prefetch(c3->rd.qual.data()); __builtin_prefetch(c3->sam.data(), 1);
				}
			}
		}
		if(i < nwn) {
			const bt2x_round_out& o = L.round_out[(size_t)i];
			c->round_out = o;
			if(o.status == BT2X_ROUND_OK) {
				c->sats.assign(L.round_sats.begin() + o.sat0, L.round_sats.begin() + o.sat0 + o.nsat);
				c->elts.assign(L.round_elts.begin() + o.elt0, L.round_elts.begin() + o.elt0 + o.nelt);
				c->exNew.assign(L.round_exr_out.begin() + o.exr0, L.round_exr_out.begin() + o.exr0 + o.nexr);
			}
			c->req = REQ_NONE;
			c->task.h.resume();
			return;
		}
		i -= nwn;
		if(i < nws) {
			c->seed_out.assign(L.seed_out.begin() + (long)L.sk[i], L.seed_out.begin() + (long)L.sk[i + 1]);
		} else if(i < nws + nwr) {
			const long r = i - nws;
			// the three-request path's resolves as round elements
			c->elts.resize((size_t)(L.rk[r + 1] - L.rk[r]));
			for(size_t k = 0; k < c->elts.size(); k++) {
				const bt2x_resolve_out& o = L.res_out[L.rk[r] + k];
				c->elts[k] = bt2x_elt_pack(o.toff, o.tidx, o.straddled);
			}
		} else {
			const long r = i - nws - nwr;
			for(size_t j = 0; j < c->dps.size(); j++) {
				const uint64_t k = L.pb[r] + j;
				const bt2x_dp_out& o = L.dp_out[k];
				DpMemo m;
				m.key = c->dps[j].key;
				m.out = o;
				m.rec0 = (uint32_t)c->recs.size();
				c->memo.push_back(m);
				// each record's edit-buffer image moves to the read's edit arena (arena
				// offsets are allocated by the kernel's atomics, so one problem's images
				// are not contiguous)
				for(uint32_t q = 0; q < o.nrec; q++) {
					bt2x_aln_rec a = L.recs[o.rec_off + q];
					const uint32_t eo = (uint32_t)c->edits.size();
					c->edits.insert(c->edits.end(), L.edits.begin() + a.edit_off, L.edits.begin() + a.edit_off + a.nbuf);
					a.edit_off = eo;
					c->recs.push_back(a);
				}
			}
		}
		c->req = REQ_NONE;
		c->task.h.resume();
	});
	st.t_host += now_s() - t0;
}

// One scheduler iteration over `act`: every pending request in one launch per kind,
// then the served reads resume.  Returns false when no read is waiting.
bool Aligner::step(std::vector<ReadCtx*>& act, RunStats& st) {
	Launch& L = launch_[0];
	gather(L, act);
	if(L.ws.empty() && L.wr.empty() && L.wd.empty() && L.wn.empty()) return false;
	static const bool trace = std::getenv("BT2X_TRACE") != nullptr;
	if(trace) std::fprintf(stderr, "BT2X_TRACE active=%zu seed=%zu resolve=%zu dp=%zu\n", act.size(), L.ws.size(),
	                       L.wr.size(), L.wd.size());
	execute(L);
	scatter_resume(L, st);
	return true;
}

namespace {
// Finished records by read id until they can be written in input order.
class OutRing {
public:
	OutRing() : slot_(1 << 12), ready_(1 << 12, 0) {}
	// make room for ids below `end`
	void reserve(uint64_t end) {
		if(end - base_ <= slot_.size()) return;
		size_t cap = slot_.size();
		while(end - base_ > cap) cap *= 2;
		std::vector<std::string> s(cap);
		std::vector<uint8_t> r(cap, 0);
		for(uint64_t id = base_; id < base_ + slot_.size(); id++) {
			s[id & (cap - 1)].swap(slot_[id & (slot_.size() - 1)]);
			r[id & (cap - 1)] = ready_[id & (slot_.size() - 1)];
		}
		slot_.swap(s); ready_.swap(r);
	}
	// hand over read id's record (the caller gets back an empty buffer with capacity)
	void put(uint64_t id, std::string& rec) {
		const size_t k = id & (slot_.size() - 1);
		slot_[k].swap(rec);
		rec.clear();
		ready_[k] = 1;
	}
	template<class F> void drain(F&& write) {
		for(;;) {
			const size_t k = base_ & (slot_.size() - 1);
			if(!ready_[k]) return;
			write(slot_[k]);
			slot_[k].clear();
			ready_[k] = 0;
			base_++;
		}
	}
private:
	std::vector<std::string> slot_;
	std::vector<uint8_t> ready_;
	uint64_t base_ = 0;
};

// SAM output off the scheduler's thread, in input order: finished records are put into a
// ring by read id (from the pool's threads, for ids the scheduler reserved), and a writer
// thread moves the ready prefix into 4 MiB chunks and fwrites them.  The ring only grows
// in reserve(), on the scheduler's thread, under the lock the writer holds while it
// drains.
class OrderedSamWriter {
public:
	// `store`: the ring's strings, kept by the caller across runs, so the records' buffers
	// are neither allocated again nor freed when the run ends (freeing a ring grown behind a
	// lagging writer cost ~0.3 s at the end of a 10 M-read run)
	OrderedSamWriter(std::FILE* f, std::vector<std::string>& store) : f_(f), store_(store) {
		slot_.swap(store_);
		size_t cap = 1 << 16;
		while(cap < slot_.size()) cap *= 2;
		if(slot_.size() != cap) slot_.resize(cap);
		ready_.reset(new std::atomic<uint8_t>[cap]);
		for(size_t i = 0; i < cap; i++) ready_[i].store(0, std::memory_order_relaxed);
		cap_ = cap;
		std::fflush(f_);                                  // (the header) before the raw writes
		th_ = std::thread([this] { loop(); });
	}
	~OrderedSamWriter() {
		finish();
		for(std::string& r : slot_) r.clear();
		store_.swap(slot_);
	}
	void reserve(uint64_t end) {                       // scheduler thread
		if(end - base_.load(std::memory_order_acquire) <= cap_) return;
		std::lock_guard<std::mutex> g(mu_);
		size_t cap = cap_;
		while(end - base_.load(std::memory_order_relaxed) > cap) cap *= 2;
		if(cap != cap_) grow(cap);
	}
	void put(uint64_t id, std::string& rec) {          // any thread
		const size_t k = id & (cap_ - 1);
		slot_[k].swap(rec);
		rec.clear();
		ready_[k].store(1, std::memory_order_release);
	}
	void kick() {
		{ std::lock_guard<std::mutex> g(mu_); kicked_ = true; }
		cv_.notify_one();
	}
	uint64_t written() const { return base_.load(std::memory_order_acquire); }
	void finish() {
		if(!th_.joinable()) return;
		{ std::lock_guard<std::mutex> g(mu_); stop_ = true; }
		cv_.notify_one();
		th_.join();
	}
private:
	static constexpr size_t kChunk = 4u << 20;
	void grow(size_t cap) {                            // (lock held, or before the thread starts)
		std::vector<std::string> s(cap);
		std::unique_ptr<std::atomic<uint8_t>[]> r(new std::atomic<uint8_t>[cap]);
		for(size_t i = 0; i < cap; i++) r[i].store(0, std::memory_order_relaxed);
		const uint64_t b = base_.load(std::memory_order_relaxed);
		for(uint64_t id = b; cap_ && id < b + cap_; id++) {
			s[id & (cap - 1)].swap(slot_[id & (cap_ - 1)]);
			r[id & (cap - 1)].store(ready_[id & (cap_ - 1)].load(std::memory_order_acquire), std::memory_order_relaxed);
		}
		slot_.swap(s);
		ready_.swap(r);
		cap_ = cap;
	}
	// moves the ready prefix (at most one chunk) into `chunk`; true if it stopped on a full chunk
	bool drain(std::string& chunk) {
		std::lock_guard<std::mutex> g(mu_);
		uint64_t b = base_.load(std::memory_order_relaxed);
		for(;;) {
			const size_t k = b & (cap_ - 1);
			if(!ready_[k].load(std::memory_order_acquire)) break;
			chunk += slot_[k];
			slot_[k].clear();
			ready_[k].store(0, std::memory_order_relaxed);
			base_.store(++b, std::memory_order_release);
			if(chunk.size() >= kChunk) return true;
		}
		return false;
	}
	void loop() {
		std::string chunk;
		chunk.reserve(kChunk + 4096);
		for(;;) {
			bool stop;
			{
				std::unique_lock<std::mutex> g(mu_);
				cv_.wait(g, [&] { return stop_ || kicked_; });
				kicked_ = false;
				stop = stop_;
			}
			bool full;
			do {
				full = drain(chunk);
				if(full || (stop && !chunk.empty())) {
					put_chunk(chunk);
					chunk.clear();
				}
			} while(full);
			if(stop) return;
		}
	}
	// the chunk straight to the file descriptor (the FILE's buffer, flushed when the writer
	// starts, would copy every byte once more); fwrite if the stream has no descriptor
	void put_chunk(const std::string& c) {
		const int fd = ::fileno(f_);
		size_t o = 0;
		while(fd >= 0 && o < c.size()) {
			const ssize_t w = ::write(fd, c.data() + o, c.size() - o);
			if(w < 0 && errno == EINTR) continue;
			if(w <= 0) break;                            // (as an unchecked fwrite: the run's output is short)
			o += (size_t)w;
		}
		if(fd < 0) std::fwrite(c.data(), 1, c.size(), f_);
	}
	std::FILE* f_;
	std::vector<std::string>& store_;
	std::vector<std::string> slot_;
	std::unique_ptr<std::atomic<uint8_t>[]> ready_;
	size_t cap_ = 0;
	std::atomic<uint64_t> base_{0};
	std::mutex mu_;
	std::condition_variable cv_;
	bool kicked_ = false, stop_ = false;
	std::thread th_;
};

// The per-read counters retire() adds up (RunStats' share of them).
struct RetireAcc {
	uint64_t reads = 0, aligned = 0, unaligned = 0, rep = 0, dps_used = 0, tight_recs = 0;
	ReportingMetrics met;
	void count(const ReadCtx* c) {
		reads++;
		if(c->aligned) aligned++; else unaligned++;
		if(c->repetitive) rep++;
		using M = ReportingMetrics;
		met.v[M::NREAD]++;
		met.v[M::NUNPAIRED]++;
		static constexpr int kind_field[4] = {M::NUNP_0, M::NUNP_UNI1, M::NUNP_UNI2, M::NUNP_REP};
		met.v[kind_field[c->met_kind]]++;
		if(c->met_kind == 1 || c->met_kind == 2) met.v[M::NUNP_UNI]++;
		dps_used += c->ndp_used;
		tight_recs += c->ntight;
	}
	void into(RunStats& st) const {
		st.reads += reads; st.aligned += aligned; st.unaligned += unaligned; st.rep += rep;
		st.dps_used += dps_used; st.tight_recs += tight_recs;
		st.met.merge(met);
	}
};
}

WorkPool& Aligner::pool() { return *pool_; }

void Aligner::use_threads(int threads) {
	if(!pool_ || pool_->threads() != std::max(1, threads)) pool_.reset(new WorkPool(threads));
}

ReadCtx* Aligner::take_ctx() {
	if(free_.empty()) {
		ctxs_.emplace_back(new ReadCtx);
		ctxs_.back()->slot = (uint32_t)(ctxs_.size() - 1);
		return ctxs_.back().get();
	}
	ReadCtx* c = free_.back();
	free_.pop_back();
	return c;
}

Aligner::~Aligner() {
	// contexts hold tens of buffers each: release them in parallel
	const long n = (long)ctxs_.size();
	if(pool_) pool().parallel_for(n, 256, [&](long i) { ctxs_[(size_t)i].reset(); });
}

// Retire the finished reads of `act` (their records go to `put`, their contexts back to
// the pool); the others stay in `act`.  Parallel over 1024-read chunks, each with its own
// counters; then a serial compaction.
void Aligner::retire(std::vector<ReadCtx*>& act, RunStats& st, const std::function<void(uint64_t, std::string&)>& put,
                     Launch* defer) {
	const long n = (long)act.size(), nch = (n + 1023) / 1024;
	std::vector<RetireAcc> acc((size_t)nch);
	// each chunk splits its reads into the ones still running and the finished ones (in
	// order), so the serial part only concatenates the chunks' lists: a serial pass over
	// the cohort's cold contexts cost ~2.5 ms per step
	if(retire_keep_.size() < (size_t)nch) {
		retire_keep_.resize((size_t)nch); retire_fin_.resize((size_t)nch); retire_sam_.resize((size_t)nch);
	}
	const bool pf = host_prefetch();
	std::vector<uint64_t> sam_bytes((size_t)nch, 0);
	pool().parallel_for(nch, 1, [&](long ch) {
		RetireAcc& a = acc[(size_t)ch];
		std::vector<ReadCtx*>& keep = retire_keep_[(size_t)ch];
		std::vector<ReadCtx*>& fin = retire_fin_[(size_t)ch];
		std::vector<ReadCtx*>& sam = retire_sam_[(size_t)ch];
		keep.clear(); fin.clear(); sam.clear();
		const long e = std::min(n, (ch + 1) * 1024);
		for(long i = ch * 1024; i < e; i++) {
			ReadCtx* c = act[(size_t)i];
			if(pf && i + 4 < e) __builtin_prefetch(&act[(size_t)i + 4]->done);
			if(!c->done) { keep.push_back(c); continue; }
			c->task.h.destroy();
			c->task.h = nullptr;
			a.count(c);
			if(!c->warn.empty()) std::fputs(c->warn.c_str(), stderr);
			if(defer && c->sam_gpu) {
				sam.push_back(c);
				sam_bytes[(size_t)ch] += BT2X_SAM_TAIL_MAX(c->sam_req.rdlen, c->sam_req.nmm);
			} else {
				put(c->rd.rdid, c->sam);
			}
			c->done = false;
			fin.push_back(c);
		}
	});
	for(const RetireAcc& a : acc) a.into(st);
	act.clear();
	for(long ch = 0; ch < nch; ch++) {
		act.insert(act.end(), retire_keep_[(size_t)ch].begin(), retire_keep_[(size_t)ch].end());
		free_.insert(free_.end(), retire_fin_[(size_t)ch].begin(), retire_fin_[(size_t)ch].end());
	}
	if(!defer) return;
	// the deferred records: heads and requests into the launch, at each chunk's base (the
	// contexts go back to the pool above, but no read takes them before this returns)
	Launch& L = *defer;
	std::vector<uint64_t> base((size_t)nch + 1, 0), tbase((size_t)nch + 1, 0);
	base[0] = L.sam_ids.size();
	tbase[0] = L.sam_text_bytes;
	for(long ch = 0; ch < nch; ch++) {
		base[(size_t)ch + 1] = base[(size_t)ch] + retire_sam_[(size_t)ch].size();
		tbase[(size_t)ch + 1] = tbase[(size_t)ch] + sam_bytes[(size_t)ch];
	}
	const size_t total = base[(size_t)nch];
	if(total == base[0]) return;
	L.sam_ids.resize(total);
	if(L.sam_recs.size() < total) L.sam_recs.resize(total);
	L.sam_req.resize(total);
	L.sam_text_bytes = tbase[(size_t)nch];
	pool().parallel_for(nch, 1, [&](long ch) {
		uint64_t k = base[(size_t)ch], t = tbase[(size_t)ch];
		for(ReadCtx* c : retire_sam_[(size_t)ch]) {
			L.sam_ids[k] = c->rd.rdid;
			L.sam_recs[k].swap(c->sam);              // (the context keeps the old buffer's capacity)
			c->sam.clear();
			bt2x_sam_req& q = L.sam_req[k];
			q = c->sam_req;
			q.text_off = t;
			t += BT2X_SAM_TAIL_MAX(q.rdlen, q.nmm);
			c->sam_gpu = false;
			k++;
		}
	});
}

void Aligner::flush_sam(Launch& L, RunStats& st, const std::function<void(uint64_t, std::string&)>& put) {
	const long n = (long)L.sam_ids.size();
	if(!n) return;
	st.sam_gpu += (uint64_t)n;
	st.t_sam += L.t_sam;
	pool().parallel_for(n, 256, [&](long i) {
		std::string& r = L.sam_recs[(size_t)i];
		r.append(L.sam_text.data() + L.sam_req[(size_t)i].text_off, L.sam_lens[(size_t)i]);
		put(L.sam_ids[(size_t)i], r);
	});
	L.sam_ids.clear();
	L.sam_req.clear();
	L.sam_text_bytes = 0;
}

namespace {
// Element counts of reserve_launch_buffers for a cohort of `reads`, generous for 150 bp
// reads: half of them in a seed round (fw + rc, ~20 seeds, up to 64 elements each), all
// of them in a DP request (3 problems of ~200 columns on average).
struct LaunchSizes {
	size_t nr, nd, np;
	LaunchSizes(const Params& p, size_t reads)
		: nr(reads / 2), nd(reads), np(reads * 3) { (void)p; }
};
}

std::vector<size_t> Aligner::launch_buffer_bytes(const Params& p, size_t reads) {
	const LaunchSizes z(p, reads);
	return {z.nr * 320, z.nr * 24 * sizeof(bt2x_seed_in), z.nr * sizeof(bt2x_round_in), z.nr * 4 * sizeof(bt2x_exrange),
	        z.nr * sizeof(bt2x_round_out), z.nr * 64 * sizeof(bt2x_sat), z.nr * 64 * sizeof(bt2x_elt),
	        z.nr * 4 * sizeof(bt2x_exrange), z.nd * 320, z.nd * 320, z.np * 210, z.np * sizeof(bt2x_dp_in),
	        z.np * sizeof(bt2x_dp_out), (z.np * 4 + 64) * sizeof(bt2x_aln_rec), (z.np * 48 + 256) * sizeof(uint32_t),
	        z.nd * 320, z.nd * sizeof(bt2x_store_in)};
}

void Aligner::reserve_launch_buffers(size_t reads) {
	const LaunchSizes z(p_, reads);
	for(Launch& L : launch_) {
		L.round_reads.reserve(z.nr * 320); L.round_seeds.reserve(z.nr * 24); L.round_in.reserve(z.nr);
		L.round_exr.reserve(z.nr * 4); L.round_out.reserve(z.nr); L.round_sats.reserve(z.nr * 64);
		L.round_elts.reserve(z.nr * 64); L.round_exr_out.reserve(z.nr * 4);
		L.dp_reads.reserve(z.nd * 320); L.dp_quals.reserve(z.nd * 320); L.dp_refs.reserve(z.np * 210);
		L.dp_in.reserve(z.np); L.dp_out.reserve(z.np); L.recs.reserve(z.np * 4 + 64); L.edits.reserve(z.np * 48 + 256);
		L.store_packed.reserve(z.nd * 320); L.store_in.reserve(z.nd);
	}
}

RunStats Aligner::run(FastqReader& fq, std::FILE* out, size_t slots, int threads, double* t_run) {
	RunStats st;
	use_threads(threads);
	dseeds_ = be_.device_seeds();
	// record tails on the GPU: pipelined runs (a launch per cohort to carry the requests)
	// whose backends keep the reads in a store and can format them
	gpu_sam_ = pipeline_ && be_.sam_tails_ok() && (!be2_ || be2_->sam_tails_ok());
	const double t_start = now_s();
	if(header_on_) {
		const std::string hdr = header();
		std::fwrite(hdr.data(), 1, hdr.size(), out);
	}
	uint64_t rdid = 0;
	const uint64_t rdid0 = fq.first_rdid();
	bool eof = false;
	std::vector<FastqReader::Raw> raw;
	std::vector<ReadCtx*> fresh;
	OrderedSamWriter writer(out, sam_ring_);
	const auto put = [&writer](uint64_t id, std::string& rec) { writer.put(id, rec); };
	if(slots < 2) slots = 2;
	reserve_launch_buffers(pipeline_ ? slots / 2 : slots);
	// FASTQ records are taken ahead on a helper thread (the record scan is serial): while
	// fewer than a cohort's worth of taken records wait, one batch of a cohort's size is in
	// flight while the scheduler resumes, retires and gathers; refill decodes straight from
	// the taken records (no copies of the record list).  The reader is touched by one thread
	// at a time (the main thread only after collecting the batch in flight).
	const size_t batch = pipeline_ ? slots / 2 : slots;
	std::vector<FastqReader::Raw> ahead, incoming;
	size_t ahead_pos = 0;
	bool src_eof = false;
	std::future<size_t> ahead_f;
	auto start_ahead = [&] {
		if(src_eof || ahead_f.valid() || ahead.size() - ahead_pos >= batch) return;
		incoming.clear();
		ahead_f = std::async(std::launch::async, [&fq, &incoming, batch] { return fq.take(batch, incoming); });
	};
	std::vector<uint64_t> file_ends;           // the reader's file_end() values, copied while it is idle
	auto note_files = [&] { while(file_ends.size() < fq.files_done()) file_ends.push_back(fq.file_end(file_ends.size())); };
	auto collect = [&] {
		if(!ahead_f.valid()) return;
		if(ahead_f.get() < batch) src_eof = true;
		note_files();
		if(ahead_pos == ahead.size()) { ahead.swap(incoming); ahead_pos = 0; return; }
		ahead.erase(ahead.begin(), ahead.begin() + (long)ahead_pos);      // the remainder: < one batch
		ahead_pos = 0;
		ahead.insert(ahead.end(), incoming.begin(), incoming.end());
	};
	// New reads join cohort `co` (up to `cap` reads in it): decoded and run up to their
	// first request, in parallel.
	auto refill = [&](std::vector<ReadCtx*>& co, size_t cap) {
		double t0 = now_s();
		raw.clear();
		const FastqReader::Raw* src = nullptr;
		long nf = 0;
		if(!eof && co.size() < cap) {
			const size_t want = cap - co.size();
			if(ahead.size() - ahead_pos < want) collect();
			const size_t n = std::min(want, ahead.size() - ahead_pos);
			if(n < want && !src_eof) {
				// (the helper is idle here: collect() joined it) the rest synchronously
				raw.insert(raw.end(), ahead.begin() + (long)ahead_pos, ahead.begin() + (long)(ahead_pos + n));
				ahead_pos += n;
				if(fq.take(want - n, raw) < want - n) src_eof = true;
				note_files();
				src = raw.data();
				nf = (long)raw.size();
			} else {
				src = ahead.data() + ahead_pos;
				nf = (long)n;
				ahead_pos += n;
			}
			if(src_eof && ahead_pos == ahead.size() && !ahead_f.valid()) eof = true;
			// input files whose last record is out
			const uint64_t written = writer.written();
			while(st.t_files.size() < file_ends.size() && file_ends[st.t_files.size()] <= written)
				st.t_files.push_back(now_s() - t_start);
		}
		st.t_io += now_s() - t0;
		if(!nf) { start_ahead(); return; }
		t0 = now_s();
		fresh.resize((size_t)nf);
		for(long i = 0; i < nf; i++) fresh[(size_t)i] = take_ctx();
		writer.reserve(rdid + (uint64_t)nf);
		st.t_alloc += now_s() - t0;
		const bool pf = host_prefetch(), pf_more = host_prefetch_more();
		pool().parallel_for(nf, 64, [&](long i) {
			ReadCtx* c = fresh[(size_t)i];
			if(pf && i + 6 < nf) {
				prefetch_ctx(fresh[(size_t)i + 6], true);
				if(pf_more) prefetch_ctx_rest(fresh[(size_t)i + 6]);
			}
			if(pf && i + 3 < nf) {                             // the buffers decode writes
				const Read& r3 = fresh[(size_t)i + 3]->rd;
				__builtin_prefetch(r3.fw.data(), 1); __builtin_prefetch(r3.rc.data(), 1);
				__builtin_prefetch(r3.qual.data(), 1); __builtin_prefetch(r3.qualRev.data(), 1);
				__builtin_prefetch(r3.name.data(), 1);
			}
			FastqReader::decode(src[i], c->rd, rdid + (uint64_t)i, p_.randSeed, rdid0 + rdid + (uint64_t)i);
			c->in_store = false;
			c->task = align_read(c);
			c->task.h.resume();
		});
		// (the decoded records are consumed: the helper may refill `incoming` from here on)
		start_ahead();
		rdid += (uint64_t)nf;
		st.t_host += now_s() - t0;
		co.insert(co.end(), fresh.begin(), fresh.end());
	};
	auto retire_write = [&](std::vector<ReadCtx*>& co, Launch* defer) {
		const double t0 = now_s();
		retire(co, st, put, defer);
		const double t1 = now_s();
		writer.kick();
		st.t_io += now_s() - t0;
		st.t_retire += t1 - t0;
	};
	if(!pipeline_) {
		std::vector<ReadCtx*> act;
		while(true) {
			refill(act, slots);
			if(act.empty()) break;
			const double t0 = now_s();
			step(act, st);
			st.t_step += now_s() - t0;
			retire_write(act, nullptr);
		}
	} else {
		// Two cohorts of up to slots/2 reads alternate: while the GPU thread runs one
		// cohort's launches, the host threads resume the other with its previous results,
		// retire and refill it, and gather its next launch.  With a second backend each
		// cohort has a GPU thread of its own, and a cohort's next launch starts as soon as it
		// is gathered, alongside the other cohort's launch still on the GPU.
		std::vector<ReadCtx*> co[2];
		const size_t cap = slots / 2;
		auto empty = [](const Launch& L) {
			return L.ws.empty() && L.wr.empty() && L.wd.empty() && L.wn.empty() && L.sam_req.empty();
		};
		// A backend error on a GPU thread is carried over to this one and rethrown after the
		// join; unwinding on either side joins the threads first (a joinable std::thread must
		// not be destroyed).
		std::exception_ptr gpu_err[2];
		std::thread gpu[2];
		struct Joiner { std::thread* t; ~Joiner() { for(int k = 0; k < 2; k++) if(t[k].joinable()) t[k].join(); } } joiner{gpu};
		auto start = [&](int k) {
			gpu[k] = std::thread([this, k, &gpu_err] {
				try { execute(launch_[k]); } catch(...) { gpu_err[k] = std::current_exception(); }
			});
		};
		auto join = [&](int k) {
			if(gpu[k].joinable()) gpu[k].join();
			if(gpu_err[k]) std::rethrow_exception(gpu_err[k]);
		};
		const bool two = be2_ != nullptr;
		int a = 0;
		refill(co[0], cap);
		gather(launch_[0], co[0]);
		start(0);
		refill(co[1], cap);
		gather(launch_[1], co[1]);
		if(two) start(1);
		while(true) {
			// invariant: launch a is on (or through) the GPU; launch b is gathered, and with one
			// backend it starts once launch a is through
			const double t0 = now_s();
			join(a);
			st.t_wait += now_s() - t0;
			const int b = 1 - a;
			if(!two) start(b);
			const double t1 = now_s();
			flush_sam(launch_[a], st, put);              // the tails this launch formatted
			scatter_resume(launch_[a], st);
			retire_write(co[a], gpu_sam_ ? &launch_[a] : nullptr);
			refill(co[a], cap);
			gather(launch_[a], co[a]);
			st.t_step += now_s() - t1;
			if(eof && co[a].empty() && co[b].empty() && empty(launch_[a]) && empty(launch_[b])) break;
			if(two) start(a);
			a = b;
		}
		join(0);
		join(1);
	}
	if(ahead_f.valid()) ahead_f.get();            // (a batch taken past the end: empty)
	writer.finish();
	if(t_run) *t_run = now_s() - t_start;
	while(st.t_files.size() < fq.nfiles()) st.t_files.push_back(now_s() - t_start);
#ifdef BT2X_PHASE_PROF
	ph_print();
#endif
	return st;
}

std::string Aligner::align_all(std::vector<Read>& reads, size_t slots, int threads, RunStats* stp) {
	RunStats st;
	gpu_sam_ = false;                              // (records formatted here, in step())
	use_threads(threads);
	dseeds_ = be_.device_seeds();
	std::vector<ReadCtx*> act, fresh;
	OutRing ring;
	std::string out;
	size_t next = 0;
	if(slots < 1) slots = 1;
	while(true) {
		fresh.clear();
		while(next < reads.size() && act.size() + fresh.size() < slots) {
			ReadCtx* c = take_ctx();
			c->rd = reads[next];
			c->rd.rdid = next;
			fresh.push_back(c);
			next++;
		}
		ring.reserve(next);
		const long nf = (long)fresh.size();
		pool().parallel_for(nf, 64, [&](long i) {
			fresh[i]->in_store = false;
			fresh[i]->task = align_read(fresh[i]);
			fresh[i]->task.h.resume();
		});
		act.insert(act.end(), fresh.begin(), fresh.end());
		if(act.empty()) break;
		step(act, st);
		retire(act, st, [&ring](uint64_t id, std::string& rec) { ring.put(id, rec); });
		ring.drain([&](const std::string& s) { out += s; });
	}
	if(stp) *stp = st;
	return out;
}

} // namespace host
} // namespace bt2x
