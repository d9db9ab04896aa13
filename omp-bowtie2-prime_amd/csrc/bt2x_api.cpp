// bt2x_api.cpp — host side of the C-ABI (include/bt2x.h): index loader, scoring
// tables, per-GPU context, staging and launches.  No CPU compute path exists: every
// seed search and DP goes through the gfx950 kernels, and without a HIP device
// bt2x_open fails with BT2X_E_NODEVICE.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "bt2x_device.h"


#define HIPCHK(x) do { if((x) != hipSuccess) return BT2X_E_NODEVICE; } while(0)

// ----------------------------------------------------------------- index load
// The seed round's device counters (b_rcnt): 0-2 arena use (sats, elts, exRange out),
// 3-7 sampling jobs/ranges/queue/draws, 8-15 sampling statistics, 16 the reads whose
// GPU-instantiated seed count differs from in[r].nseeds (seed_gen_kernel).
constexpr int kRoundCounters = 17;
constexpr int kRoundSeedMismatch = 16;

namespace {
// The host image of an index is the .bt2l files themselves, mapped read-only: the arrays
// bt2x_index_desc points at are views into the mappings (no copies), so ranks of one node
// that load the same index share its pages through the page cache -- one host copy per
// node, not per GPU -- and the pages a run never reads after bt2x_open's upload (the BWT,
// the SA sample; the packed text unless host-cut windows ask for it) stay unread.
struct Mapping {
	const uint8_t* p = nullptr;
	size_t n = 0;
};
struct IndexOwner {
	std::vector<Mapping> maps;
	~IndexOwner() { for(const Mapping& m : maps) if(m.p && m.n) munmap(const_cast<uint8_t*>(m.p), m.n); }
};

// Map a whole file read-only (empty files map to an empty view).
bool map_file(IndexOwner* o, const std::string& path, Mapping& m) {
	const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
	if(fd < 0) return false;
	struct stat st;
	if(fstat(fd, &st) != 0) { close(fd); return false; }
	m.n = (size_t)st.st_size;
	m.p = nullptr;
	if(m.n) {
		void* v = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, fd, 0);
		if(v == MAP_FAILED) { close(fd); return false; }
		m.p = (const uint8_t*)v;
		o->maps.push_back(m);
	}
	close(fd);
	return true;
}

// A bounds-checked cursor over a mapping: scalar fields are copied out, arrays are views.
struct Cursor {
	const Mapping& m;
	size_t at = 0;
	bool ok = true;
	template<typename T> T get() {
		T v{};
		if(!ok || at + sizeof(T) > m.n) { ok = false; return v; }
		std::memcpy(&v, m.p + at, sizeof(T));
		at += sizeof(T);
		return v;
	}
	template<typename T> const T* view(uint64_t count) {
		const uint64_t bytes = count * sizeof(T);
		if(!ok || count > m.n / (sizeof(T) ? sizeof(T) : 1) || at + bytes > m.n) { ok = false; return nullptr; }
		const T* v = reinterpret_cast<const T*>(m.p + at);
		at += bytes;
		return v;
	}
};
}

// Ebwt::readIntoMemory (bt2_io.cpp:39-560) for the 64-bit (.bt2l) forward index.
extern "C" int bt2x_index_load(const char* base, int load_offs, bt2x_index_desc* o) {
	if(!base || !o) return BT2X_E_ARG;
	std::memset(o, 0, sizeof(*o));
	std::unique_ptr<IndexOwner> own(new IndexOwner());
	Mapping m1;
	if(!map_file(own.get(), std::string(base) + ".1.bt2l", m1)) return BT2X_E_IO;
	Cursor c1{m1};
	const uint32_t one = c1.get<uint32_t>();
	const uint64_t len = c1.get<uint64_t>();
	const int32_t lineRate = c1.get<int32_t>(), lps = c1.get<int32_t>(), offRate = c1.get<int32_t>();
	const int32_t ftabChars = c1.get<int32_t>(), flags = c1.get<int32_t>();
	(void)lps;
	// only the fork's build is supported: little-endian, lineRate 7 (128-B sides)
	if(!c1.ok || one != 1 || lineRate != 7 || ftabChars < 1 || ftabChars > 16) return BT2X_E_IO;
	const uint64_t npat = c1.get<uint64_t>();
	const uint64_t* plen = c1.view<uint64_t>(npat);
	const uint64_t nfrag = c1.get<uint64_t>();
	const uint64_t* rstarts = c1.view<uint64_t>(nfrag <= m1.n / 24 ? 3 * nfrag : m1.n);     // (too many: fails)
	const uint64_t sideSz = 1ULL << lineRate, sideBwtSz = sideSz - 32;    // EbwtParams::init
	const uint64_t numSides = (len / 4 + 1 + sideBwtSz - 1) / sideBwtSz;
	const uint64_t ebwtTot = numSides * sideSz;
	const uint8_t* ebwt = c1.view<uint8_t>(ebwtTot);
	const uint64_t zoff = c1.get<uint64_t>();
	if(const uint64_t* fc = c1.view<uint64_t>(5)) std::memcpy(o->fchr, fc, 40);
	const uint64_t ftabLen = (1ULL << (2 * ftabChars)) + 1, eftabLen = 2ULL * ftabChars;
	const uint64_t* ftab = c1.view<uint64_t>(ftabLen);
	const uint64_t* eftab = c1.view<uint64_t>(eftabLen);
	if(!c1.ok) return BT2X_E_IO;
	o->len = len; o->zoff = zoff; o->ftab_chars = ftabChars; o->off_rate = offRate;
	o->line_rate = lineRate; o->flags = flags;
	o->ebwt = ebwt; o->ebwt_bytes = ebwtTot;
	o->ftab = ftab; o->ftab_len = ftabLen; o->eftab = eftab; o->eftab_len = eftabLen;
	o->plen = plen; o->npat = npat; o->rstarts = rstarts; o->nfrag = nfrag;
	if(load_offs) {
		Mapping m2;
		if(!map_file(own.get(), std::string(base) + ".2.bt2l", m2)) return BT2X_E_IO;
		Cursor c2{m2};
		if(offRate < 0 || offRate > 62) return BT2X_E_IO;
		const uint64_t offsLen = (len + 1 + (1ULL << offRate) - 1) >> offRate;
		(void)c2.get<uint32_t>();                             // endianness word
		const uint64_t* offs = c2.view<uint64_t>(offsLen);
		if(!c2.ok) return BT2X_E_IO;
		o->offs = offs; o->offs_len = offsLen;
		// packed joined text (BitPairReference .4: the non-N bases, 4 per byte)
		Mapping m4;
		if(map_file(own.get(), std::string(base) + ".4.bt2l", m4)) {
			Cursor c4{m4};
			const uint64_t tb = (len + 3) / 4;
			const uint8_t* t = c4.view<uint8_t>(tb);
			if(!c4.ok) return BT2X_E_IO;
			o->text2 = t; o->text2_bytes = tb;
		}
	}
	o->owner = own.release();
	return BT2X_OK;
}

extern "C" void bt2x_index_free(bt2x_index_desc* o) {
	if(!o) return;
	delete reinterpret_cast<IndexOwner*>(o->owner);
	std::memset(o, 0, sizeof(*o));
}

// -------------------------------------------------------------------- scoring
extern "C" void bt2x_scoring_init(bt2x_scoring* sc) {
	// Scoring::initPens (scoring.h:94-132): COST_MODEL_QUAL mismatches, constant N
	for(int i = 0; i < 256; i++) {
		const int ii = i < 40 ? i : 40;
		const float frac = (float)ii / 40.0f;
		sc->mmpens[i] = sc->mm_min + (int)(frac * (float)(sc->mm_max - sc->mm_min));
		sc->npens[i] = sc->n_pen;
	}
}

extern "C" void bt2x_scoring_default(bt2x_scoring* sc) {
	std::memset(sc, 0, sizeof(*sc));
	sc->mm_max = 6; sc->mm_min = 2; sc->n_pen = 1;      // scoring.h:38-50
	sc->rdg_const = 5; sc->rdg_linear = 3;              // scoring.h:70-79
	sc->rfg_const = 5; sc->rfg_linear = 3;
	sc->gapbar = 4;                                     // bt2_search.cpp:374
	bt2x_scoring_init(sc);
}

extern "C" void* bt2x_host_alloc(size_t bytes) {
	void* p = nullptr;
	if(hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return nullptr;
	return p;
}

extern "C" void bt2x_host_free(void* p) {
	if(p) (void)hipHostFree(p);
}

extern "C" const char* bt2x_version(void) { return "bt2x 0.4 (gfx950; abi 4)"; }
extern "C" int bt2x_abi_version(void) { return BT2X_ABI_VERSION; }

// -------------------------------------------------------------------- context
struct DevBuf {
	void* p = nullptr; size_t cap = 0;
	int ensure(size_t n) {
		if(n <= cap) return 0;
		if(p) (void)hipFree(p);
		p = nullptr; cap = 0;
		size_t want = n + n / 4 + 4096;
		if(hipMalloc(&p, want) != hipSuccess) return BT2X_E_NOMEM;
		cap = want;
		return 0;
	}
	void release() { if(p) (void)hipFree(p); p = nullptr; cap = 0; }
};

// Every resource the context holds is released by its destructor, so bt2x_open's early
// error returns (through HIPCHK and friends) leak nothing.
struct bt2x_ctx {
	~bt2x_ctx();
	int device = 0;
	hipStream_t stream = nullptr;
	hipEvent_t sync_ev = nullptr;              // blocking-sync event: host waits sleep, not spin
	hipEvent_t ev[BT2X_K_COUNT][2] = {};
	bool ev_valid[BT2X_K_COUNT] = {};
	DevIndex ix{};
	DevScoring sc{};
	void* d_ebwt = nullptr; void* d_ftab = nullptr; void* d_eftab = nullptr; void* d_blk = nullptr;
	void* d_sa = nullptr; void* d_text = nullptr;
	void* d_offs = nullptr; void* d_rstarts = nullptr; void* d_plen = nullptr; void* d_tfirst = nullptr;
	DevBuf b_reads, b_quals, b_refs, b_in, b_out, b_recs, b_edits, b_dbg_dig, b_dbg_cand;
	// seed round: host-variant staging, and the round's own scratch (seed results, rows
	// to resolve, per-lane workspace)
	DevBuf b_rin, b_exr, b_rout, b_sats, b_elts, b_exro, b_used, b_sout, b_rows, b_ws, b_jobs, b_ranges, b_rcnt;
	const uint32_t* d_resolve_n = nullptr;     // element count of the last round's resolve (HBM)
	DevBuf scratch, b_fail, b_heavy, b_in2, b_win;         // + DP windows cut from the text (BT2X_DP_REF_TEXT)
	// the read store (bt2x_store_reads) and its upload staging
	uint8_t* d_store = nullptr;
	uint64_t store_bytes = 0;   // allocated (with growth slack)
	uint64_t store_hw = 0;      // (highest slot written + 1) * BT2X_STORE_SLOT_BYTES: requests are checked against it
	DevBuf b_pack, b_sin, b_gseeds;                         // + seeds instantiated on the GPU
	DevBuf b_sreq, b_stext, b_slens;                        // SAM tails (bt2x_sam_tails)
	uint64_t npat = 0;
	bool exact_best = true;                    // BT2X_OPT_EXACT_BEST
	int ncu = 0;
	uint32_t chunk_groups = 16384;             // DP chunk: 1 Mi problems, ~34 GB of traceback bytes
	uint32_t* d_queue = nullptr;
	unsigned long long* d_stats = nullptr;     // [0..2] seed, [4..6] dp, [8..10] resolve
	uint8_t* d_mmpen = nullptr;                // sc.mmpen in HBM (DpLaunch::mmpen)
	uint32_t* d_counters = nullptr;
	uint64_t n_seed_last = 0, n_dp_last = 0, n_resolve_last = 0;
	uint32_t n_round_last = 0;
	bool shares_index = false;                 // bt2x_open_shared: the index arrays are the base's
};

bt2x_ctx::~bt2x_ctx() {
	(void)hipSetDevice(device);
	if(stream) (void)hipStreamSynchronize(stream);
	for(DevBuf* b : {&b_reads, &b_quals, &b_refs, &b_in, &b_out, &b_recs, &b_edits, &b_dbg_dig, &b_dbg_cand, &scratch, &b_fail, &b_heavy,
	                 &b_in2, &b_win,
	                 &b_rin, &b_exr, &b_rout, &b_sats, &b_elts, &b_exro, &b_used, &b_sout, &b_rows, &b_ws,
	                 &b_jobs, &b_ranges, &b_rcnt, &b_pack, &b_sin, &b_gseeds, &b_sreq, &b_stext, &b_slens})
		b->release();
	if(d_store) (void)hipFree(d_store);
	if(!shares_index)
		for(void* p : {d_ebwt, d_ftab, d_eftab, d_blk, d_sa, d_text, d_offs, d_rstarts, d_plen, d_tfirst})
			if(p) (void)hipFree(p);
	for(void* p : {(void*)d_stats, (void*)d_counters, (void*)d_queue, (void*)d_mmpen})
		if(p) (void)hipFree(p);
	for(int k = 0; k < BT2X_K_COUNT; k++)
		for(int j = 0; j < 2; j++) if(ev[k][j]) (void)hipEventDestroy(ev[k][j]);
	if(sync_ev) (void)hipEventDestroy(sync_ev);
	if(stream) (void)hipStreamDestroy(stream);
}

namespace {
// Wait for the context's stream.  The host-pointer entry points are called from a driver
// thread that shares the CPUs with the host's per-read work: the wait blocks on an event
// (hipEventBlockingSync) instead of spinning in hipStreamSynchronize (BT2X_SPIN_WAIT=1
// restores that).
// BT2X_SPIN_WAIT=2: poll the event, sleeping 20 us between polls (the runtime's blocking
// wait still spins a while before it sleeps).
hipError_t stream_wait(bt2x_ctx* c) {
	static const int spin = [] { const char* e = getenv("BT2X_SPIN_WAIT"); return e ? atoi(e) : 0; }();
	if(spin == 1 || !c->sync_ev) return hipStreamSynchronize(c->stream);
	hipError_t e = hipEventRecord(c->sync_ev, c->stream);
	if(e != hipSuccess || spin != 2) return e != hipSuccess ? e : hipEventSynchronize(c->sync_ev);
	while((e = hipEventQuery(c->sync_ev)) == hipErrorNotReady) usleep(20);
	return e;
}
}

namespace {
// a temporary device allocation freed on every exit path
struct DevTmp {
	void* p = nullptr;
	~DevTmp() { if(p) (void)hipFree(p); }
};
}

namespace {
DevScoring to_dev(const bt2x_scoring& s) {
	DevScoring d{};
	d.rdo = s.rdg_const + s.rdg_linear; d.rde = s.rdg_linear;
	d.rfo = s.rfg_const + s.rfg_linear; d.rfe = s.rfg_linear;
	d.gapbar = s.gapbar; d.npen = s.npens[0];
	for(int i = 0; i < 256; i++) d.mmpen[i] = (uint8_t)(s.mmpens[i] < 0 ? 0 : s.mmpens[i] > 255 ? 255 : s.mmpens[i]);
	return d;
}
}

extern "C" int bt2x_open(int device, const bt2x_index_desc* idx, const bt2x_scoring* sc, bt2x_ctx** out) {
	if(!idx || !out) return BT2X_E_ARG;
	*out = nullptr;
	if(sc) {
		// the u8 DP kernel packs a row's mismatch/N penalty into 4 bits (defaults: <= 6 / 1)
		for(int i = 0; i < 256; i++) if(sc->mmpens[i] < 0 || sc->mmpens[i] > 15) return BT2X_E_ARG;
		if(sc->npens[0] < 0 || sc->npens[0] > 15) return BT2X_E_ARG;
	}
	int ndev = 0;
	if(hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return BT2X_E_NODEVICE;
	std::unique_ptr<bt2x_ctx> c(new bt2x_ctx());
	c->device = device;
	HIPCHK(hipSetDevice(device));
	HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
	HIPCHK(hipEventCreateWithFlags(&c->sync_ev, hipEventBlockingSync | hipEventDisableTiming));
	for(int k = 0; k < BT2X_K_COUNT; k++) {
		HIPCHK(hipEventCreate(&c->ev[k][0]));
		HIPCHK(hipEventCreate(&c->ev[k][1]));
	}
	HIPCHK(hipMalloc(&c->d_ebwt, idx->ebwt_bytes + 256));
	HIPCHK(hipMemcpy(c->d_ebwt, idx->ebwt, idx->ebwt_bytes, hipMemcpyHostToDevice));
	HIPCHK(hipMalloc(&c->d_ftab, 8 * idx->ftab_len));
	HIPCHK(hipMemcpy(c->d_ftab, idx->ftab, 8 * idx->ftab_len, hipMemcpyHostToDevice));
	HIPCHK(hipMalloc(&c->d_eftab, 8 * (idx->eftab_len + 1)));
	HIPCHK(hipMemcpy(c->d_eftab, idx->eftab, 8 * idx->eftab_len, hipMemcpyHostToDevice));
	c->ix.ebwt = (const uint8_t*)c->d_ebwt;
	c->ix.ftab = (const uint64_t*)c->d_ftab;
	c->ix.eftab = (const uint64_t*)c->d_eftab;
	c->ix.len = idx->len;
	c->ix.zoff = idx->zoff;
	const uint64_t zs = idx->zoff / BT2X_SIDE_CHARS, zc = idx->zoff % BT2X_SIDE_CHARS;
	c->ix.zbyte = zs * BT2X_SIDE_BYTES + (zc >> 2);          // Ebwt::postReadInit
	c->ix.zbp = (int32_t)(zc & 3);
	for(int k = 0; k < 5; k++) c->ix.fchr[k] = idx->fchr[k];
	c->ix.ftab_chars = idx->ftab_chars;
	c->ix.blk = nullptr;
	// device re-layout of the BWT into 64-byte blocks (u32 counts: rows < 2^32); the
	// seed kernel then reads one 64 B block per LF step.  BT2X_FM_SIDES=1 keeps the sides.
	{
		const char* e = getenv("BT2X_FM_SIDES");
		const uint64_t nsides = idx->ebwt_bytes / BT2X_SIDE_BYTES;
		if(!(e && e[0] == '1') && idx->len + 1 < 0xffffffffULL && nsides > 0) {
			HIPCHK(hipMalloc(&c->d_blk, 2 * nsides * BT2X_BLK_BYTES + 256));
			if(bt2x_build_blocks(c->ix, nsides, (uint8_t*)c->d_blk, c->stream)) return BT2X_E_NODEVICE;
			HIPCHK(hipStreamSynchronize(c->stream));
			c->ix.blk = (const uint8_t*)c->d_blk;
			HIPCHK(hipFree(c->d_ebwt));
			c->d_ebwt = nullptr;
			c->ix.ebwt = nullptr;
		}
	}
	// full suffix array + packed text in HBM (needs the SA sample and .4 text; load_offs)
	c->ix.off_rate = idx->off_rate;
	c->ix.sa = nullptr; c->ix.text = nullptr;
	{
		const char* e = getenv("BT2X_FULL_SA");
		if(!(e && e[0] == '0') && c->ix.blk && idx->offs && idx->offs_len && idx->text2 &&
		   idx->off_rate >= 0 && idx->off_rate < 16) {
			const size_t tbytes = ((idx->text2_bytes + 3) & ~(size_t)3) + 64;
			HIPCHK(hipMalloc(&c->d_text, tbytes));
			HIPCHK(hipMemset(c->d_text, 0, tbytes));
			HIPCHK(hipMemcpy(c->d_text, idx->text2, idx->text2_bytes, hipMemcpyHostToDevice));
			HIPCHK(hipMalloc(&c->d_sa, (idx->len + 1) * sizeof(uint32_t) + 64));
			DevTmp d_offs;
			HIPCHK(hipMalloc(&d_offs.p, idx->offs_len * sizeof(uint64_t)));
			HIPCHK(hipMemcpy(d_offs.p, idx->offs, idx->offs_len * sizeof(uint64_t), hipMemcpyHostToDevice));
			const int rc = bt2x_build_sa(c->ix, (const uint64_t*)d_offs.p, idx->offs_len, (uint32_t*)c->d_sa, c->stream);
			HIPCHK(hipStreamSynchronize(c->stream));
			if(rc) return rc;
			c->ix.sa = (const uint32_t*)c->d_sa;
			c->ix.text = (const uint32_t*)c->d_text;
		}
	}
	// SA resolution (bt2x_resolve): fragment table always; the SA sample only when no
	// full SA was built (the resolve kernel then walks LF to it, as GroupWalk does)
	c->ix.offs = nullptr; c->ix.rstarts = nullptr; c->ix.plen = nullptr; c->ix.nfrag = idx->nfrag;
	c->npat = idx->npat;
	c->ix.npat = idx->npat;
	if(idx->nfrag && idx->rstarts && idx->plen && idx->npat) {
		HIPCHK(hipMalloc(&c->d_rstarts, 24 * idx->nfrag));
		HIPCHK(hipMemcpy(c->d_rstarts, idx->rstarts, 24 * idx->nfrag, hipMemcpyHostToDevice));
		HIPCHK(hipMalloc(&c->d_plen, 8 * idx->npat));
		HIPCHK(hipMemcpy(c->d_plen, idx->plen, 8 * idx->npat, hipMemcpyHostToDevice));
		c->ix.rstarts = (const uint64_t*)c->d_rstarts;
		c->ix.plen = (const uint64_t*)c->d_plen;
		// each text's first fragment (the window kernel's per-problem search starts there)
		if(idx->nfrag < 0xffffffffULL) {
			std::vector<uint32_t> tf(idx->npat + 1);
			uint64_t k = 0;
			for(uint64_t t = 0; t <= idx->npat; t++) {
				while(k < idx->nfrag && idx->rstarts[3 * k + 1] < t) k++;
				tf[t] = (uint32_t)k;
			}
			HIPCHK(hipMalloc(&c->d_tfirst, 4 * tf.size()));
			HIPCHK(hipMemcpy(c->d_tfirst, tf.data(), 4 * tf.size(), hipMemcpyHostToDevice));
			c->ix.tfirst = (const uint32_t*)c->d_tfirst;
		}
	} else {
		c->ix.nfrag = 0;
	}
	if(!c->ix.sa && idx->offs && idx->offs_len && idx->off_rate >= 0 && idx->off_rate < 32) {
		HIPCHK(hipMalloc(&c->d_offs, 8 * idx->offs_len));
		HIPCHK(hipMemcpy(c->d_offs, idx->offs, 8 * idx->offs_len, hipMemcpyHostToDevice));
		c->ix.offs = (const uint64_t*)c->d_offs;
	}
	bt2x_scoring s;
	if(sc) s = *sc; else bt2x_scoring_default(&s);
	c->sc = to_dev(s);
	HIPCHK(hipMalloc(&c->d_mmpen, sizeof c->sc.mmpen));
	HIPCHK(hipMemcpy(c->d_mmpen, c->sc.mmpen, sizeof c->sc.mmpen, hipMemcpyHostToDevice));
	HIPCHK(hipMalloc((void**)&c->d_stats, 32 * sizeof(unsigned long long)));
	HIPCHK(hipMemset(c->d_stats, 0, 32 * sizeof(unsigned long long)));
	HIPCHK(hipMalloc((void**)&c->d_counters, 16 * sizeof(uint32_t)));
	hipDeviceProp_t prop;
	HIPCHK(hipGetDeviceProperties(&prop, device));
	// one 64-lane wave per workgroup; as many as are co-resident (register-bound)
	c->ncu = prop.multiProcessorCount;
	HIPCHK(hipMalloc((void**)&c->d_queue, 4 * sizeof(uint32_t)));
	if(const char* cg = getenv("BT2X_DP_CHUNK_GROUPS")) { const long v = atol(cg); if(v >= 1 && v <= 65536) c->chunk_groups = (uint32_t)v; }
	*out = c.release();
	return BT2X_OK;
}

extern "C" int bt2x_open_shared(const bt2x_ctx* base, bt2x_ctx** out) {
	if(!base || !out) return BT2X_E_ARG;
	*out = nullptr;
	std::unique_ptr<bt2x_ctx> c(new bt2x_ctx());
	c->device = base->device;
	c->shares_index = true;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
	HIPCHK(hipEventCreateWithFlags(&c->sync_ev, hipEventBlockingSync | hipEventDisableTiming));
	for(int k = 0; k < BT2X_K_COUNT; k++) {
		HIPCHK(hipEventCreate(&c->ev[k][0]));
		HIPCHK(hipEventCreate(&c->ev[k][1]));
	}
	c->ix = base->ix;
	c->sc = base->sc;
	c->d_ebwt = base->d_ebwt; c->d_ftab = base->d_ftab; c->d_eftab = base->d_eftab; c->d_blk = base->d_blk;
	c->d_sa = base->d_sa; c->d_text = base->d_text; c->d_offs = base->d_offs; c->d_rstarts = base->d_rstarts;
	c->d_plen = base->d_plen; c->d_tfirst = base->d_tfirst;
	c->npat = base->npat; c->exact_best = base->exact_best; c->ncu = base->ncu; c->chunk_groups = base->chunk_groups;
	HIPCHK(hipMalloc(&c->d_mmpen, sizeof c->sc.mmpen));
	HIPCHK(hipMemcpy(c->d_mmpen, c->sc.mmpen, sizeof c->sc.mmpen, hipMemcpyHostToDevice));
	HIPCHK(hipMalloc((void**)&c->d_stats, 32 * sizeof(unsigned long long)));
	HIPCHK(hipMemset(c->d_stats, 0, 32 * sizeof(unsigned long long)));
	HIPCHK(hipMalloc((void**)&c->d_counters, 16 * sizeof(uint32_t)));
	HIPCHK(hipMalloc((void**)&c->d_queue, 4 * sizeof(uint32_t)));
	*out = c.release();
	return BT2X_OK;
}

extern "C" int bt2x_device_numa_node(int device) {
	char bus[64] = {0};
	if(hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, device) != hipSuccess) return -1;
	for(char* p = bus; *p; p++) if(*p >= 'A' && *p <= 'F') *p = (char)(*p - 'A' + 'a');
	const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
	FILE* f = std::fopen(path.c_str(), "r");
	if(!f) return -1;
	int node = -1;
	if(std::fscanf(f, "%d", &node) != 1) node = -1;
	std::fclose(f);
	return node;
}

extern "C" void bt2x_close(bt2x_ctx* c) {
	delete c;        // ~bt2x_ctx releases everything
}

extern "C" int bt2x_set_option(bt2x_ctx* c, int option, int64_t value) {
	if(!c) return BT2X_E_ARG;
	if(option == BT2X_OPT_EXACT_BEST) { c->exact_best = value != 0; return BT2X_OK; }
	return BT2X_E_ARG;
}

extern "C" double bt2x_last_kernel_ms(const bt2x_ctx* c, int k) {
	if(!c || k < 0 || k >= BT2X_K_COUNT || !c->ev_valid[k]) return -1.0;
	float ms = -1.0f;
	if(hipEventSynchronize(c->ev[k][1]) != hipSuccess) return -1.0;
	if(hipEventElapsedTime(&ms, c->ev[k][0], c->ev[k][1]) != hipSuccess) return -1.0;
	return (double)ms;
}

extern "C" int bt2x_last_counters(const bt2x_ctx* c, int k, bt2x_counters* out) {
	if(!c || !out || k < 0 || k >= BT2X_K_COUNT) return BT2X_E_ARG;
	unsigned long long st[16];
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipStreamSynchronize(c->stream));
	HIPCHK(hipMemcpy(st, c->d_stats, sizeof st, hipMemcpyDeviceToHost));
	std::memset(out, 0, sizeof(*out));
	if(k == BT2X_K_SEED) {
		out->n_bilf = st[0]; out->n_lf1 = st[1]; out->n_ftab = st[2];
		out->n_problems = c->n_seed_last;
		out->alg_bytes = 128 * (2 * out->n_bilf + out->n_lf1) + 16 * out->n_ftab;
	} else if(k == BT2X_K_RESOLVE) {
		out->n_lf1 = st[9];
		out->n_problems = c->n_resolve_last;
		if(c->d_resolve_n) {
			// the count is written by the round's kernels on the caller's stream
			if(c->ev_valid[BT2X_K_RESOLVE]) HIPCHK(hipEventSynchronize(c->ev[BT2X_K_RESOLVE][1]));
			uint32_t nr = 0;
			HIPCHK(hipMemcpy(&nr, c->d_resolve_n, sizeof nr, hipMemcpyDeviceToHost));
			out->n_problems = nr;
		}
		// per element: 16 B in + 32 B out + one 4 B SA entry, or per LF step one 64 B
		// block (128 B side) and one 8 B sample word at the end of the walk
		const uint64_t step_b = c->ix.blk ? BT2X_BLK_BYTES : BT2X_SIDE_BYTES;
		out->alg_bytes = out->n_problems * (16 + 32) +
		                 (c->ix.sa ? 4 * out->n_problems : step_b * out->n_lf1 + 8 * out->n_problems);
	} else if(k == BT2X_K_ROUND) {
		return BT2X_E_ARG;                     // see BT2X_K_SEED and BT2X_K_RESOLVE
	} else {
		if(c->ev_valid[BT2X_K_DP]) HIPCHK(hipEventSynchronize(c->ev[BT2X_K_DP][1]));
		HIPCHK(hipMemcpy(st, c->d_stats, sizeof st, hipMemcpyDeviceToHost));
		out->dp_cells = st[4]; out->dp_cols = st[5]; out->bt_cells = st[6]; out->dp_cells_computed = st[7];
		out->n_problems = c->n_dp_last;
		// traceback byte per cell the fill computes and writes + reference window
		out->alg_bytes = out->dp_cells_computed + out->dp_cols;
	}
	return BT2X_OK;
}

extern "C" int bt2x_last_round_stats_ex(const bt2x_ctx* c, uint32_t* out, uint32_t n) {
	if(!c || (!out && n)) return BT2X_E_ARG;
	uint32_t all[BT2X_ROUND_STATS_N] = {};
	if(c->b_rcnt.p) {
		uint32_t cnt[16];
		HIPCHK(hipSetDevice(c->device));
		HIPCHK(hipStreamSynchronize(c->stream));
		HIPCHK(hipMemcpy(cnt, c->b_rcnt.p, sizeof cnt, hipMemcpyDeviceToHost));
		all[0] = c->n_round_last; all[1] = cnt[3]; all[2] = cnt[6]; all[3] = cnt[7];
		for(int i = 0; i < 8; i++) all[4 + i] = cnt[8 + i];
	}
	const uint32_t k = n < BT2X_ROUND_STATS_N ? n : BT2X_ROUND_STATS_N;
	for(uint32_t i = 0; i < k; i++) out[i] = all[i];
	return (int)k;
}

extern "C" int bt2x_last_round_stats(const bt2x_ctx* c, uint32_t out[4]) {
	if(!out) return BT2X_E_ARG;
	const int r = bt2x_last_round_stats_ex(c, out, 4);
	return r < 0 ? r : BT2X_OK;
}

// ------------------------------------------------------------- seed search
extern "C" int bt2x_seed_search_dev(bt2x_ctx* c, const uint8_t* d_reads, const bt2x_seed_in* d_in,
                                    uint32_t n, int do_extend, bt2x_seed_out* d_out, void* stream) {
	if(!c) return BT2X_E_ARG;
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipMemsetAsync(c->d_stats, 0, 3 * sizeof(unsigned long long), s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_SEED][0], s));
	int rc = bt2x_launch_seed(c->ix, d_reads, d_in, n, do_extend, d_out, c->d_stats, c->ncu, s);
	HIPCHK(hipEventRecord(c->ev[BT2X_K_SEED][1], s));
	c->ev_valid[BT2X_K_SEED] = true;
	c->n_seed_last = n;
	return rc;
}

extern "C" int bt2x_seed_search(bt2x_ctx* c, const uint8_t* reads, uint64_t reads_bytes,
                                const bt2x_seed_in* in, uint32_t n, int do_extend, bt2x_seed_out* out) {
	if(!c || (n && (!reads || !in || !out))) return BT2X_E_ARG;
	if(n == 0) return BT2X_OK;
	for(uint32_t i = 0; i < n; i++)
		if(in[i].seed_len < 1 || in[i].seed_len > 32 || in[i].read_off + in[i].seed_off + in[i].seed_len > reads_bytes)
			return BT2X_E_ARG;
	HIPCHK(hipSetDevice(c->device));
	int rc;
	if((rc = c->b_reads.ensure(reads_bytes)) || (rc = c->b_in.ensure(sizeof(bt2x_seed_in) * n)) ||
	   (rc = c->b_out.ensure(sizeof(bt2x_seed_out) * n))) return rc;
	HIPCHK(hipMemcpyAsync(c->b_reads.p, reads, reads_bytes, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->b_in.p, in, sizeof(bt2x_seed_in) * n, hipMemcpyHostToDevice, c->stream));
	rc = bt2x_seed_search_dev(c, (const uint8_t*)c->b_reads.p, (const bt2x_seed_in*)c->b_in.p, n,
	                          do_extend, (bt2x_seed_out*)c->b_out.p, c->stream);
	if(rc) return rc;
	HIPCHK(hipMemcpyAsync(out, c->b_out.p, sizeof(bt2x_seed_out) * n, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	return BT2X_OK;
}

// ---------------------------------------------------------------------- DP
// Scratch sized for min(batch, chunk) groups; grows with the largest batch seen.
static int ensure_scratch(bt2x_ctx* c, uint32_t n, uint32_t* groups) {
	uint32_t g = (n + 63) / 64;
	if(g > c->chunk_groups) g = c->chunk_groups;
	if(g < 1) g = 1;
	const size_t need = bt2x_dp_scratch_bytes(c->ncu, g);
	int rc = c->scratch.ensure(need);
	// use every group the buffer holds (a larger earlier batch may have grown it)
	*groups = g;
	return rc;
}

extern "C" int bt2x_dp_align_dev(bt2x_ctx* c, const uint8_t* d_reads, const uint8_t* d_quals,
                                 const uint8_t* d_refs, const bt2x_dp_in* d_in, uint32_t n,
                                 bt2x_dp_out* d_out, bt2x_aln_rec* d_recs, uint32_t rec_cap,
                                 uint32_t* d_edits, uint32_t edit_cap, uint32_t* d_counters,
                                 bt2x_dp_debug* d_debug, uint32_t launch_flags, void* stream) {
	if(!c || !d_counters) return BT2X_E_ARG;
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIPCHK(hipSetDevice(c->device));
	uint32_t groups = 0;
	int rc = ensure_scratch(c, n, &groups);
	if(rc) return rc;
	const bool exact = (launch_flags & BT2X_DPL_EXACT_BEST) != 0;
	if(exact && (rc = c->b_fail.ensure(sizeof(uint32_t) * (size_t)(n ? n : 1)))) return rc;
	HIPCHK(hipMemsetAsync(d_counters, 0, 4 * sizeof(uint32_t), s));
	HIPCHK(hipMemsetAsync(c->d_stats + 4, 0, 4 * sizeof(unsigned long long), s));
	DpLaunch a{};
	a.reads = d_reads; a.quals = d_quals; a.refs = d_refs; a.in = d_in; a.n = n; a.out = d_out;
	a.recs = d_recs; a.rec_cap = rec_cap; a.edits = d_edits; a.edit_cap = edit_cap;
	a.counters = d_counters; a.stats = c->d_stats + 4;
	a.mmpen = c->d_mmpen;
	a.digests = d_debug ? d_debug->digests : nullptr;
	a.cands = d_debug ? d_debug->cands : nullptr;
	a.scratch = (uint8_t*)c->scratch.p; a.chunk_groups = groups; a.ncu = c->ncu; a.queue = c->d_queue;
	{ const char* ab = getenv("BT2X_DP_ABLATE"); a.ablate = (ab && *ab >= '1' && *ab <= '2') ? (uint32_t)(*ab - '0') : 0u; }
	{ const char* bd = getenv("BT2X_DP_BAND"); a.band = (bd && bd[0] == '0') ? 0u : 1u; }
	a.wide = (launch_flags & BT2X_DPL_I16) ? 1u : 0u;
	a.fail_list = exact ? (uint32_t*)c->b_fail.p : nullptr;
	// lane-kernel walks past `heavy` steps are redone by the wave kernel, traceback in LDS
	// (BT2X_DP_HEAVY=0: never); read per launch (tests switch it)
	{
		const char* hv = getenv("BT2X_DP_HEAVY");
		a.heavy = hv ? (uint32_t)atol(hv) : 800u;
		if(a.heavy && !d_debug) {
			if((rc = c->b_heavy.ensure(sizeof(uint32_t) * ((size_t)n + 1)))) return rc;
			a.heavy_list = (uint32_t*)c->b_heavy.p;
			HIPCHK(hipMemsetAsync(a.heavy_list, 0, sizeof(uint32_t), s));
		}
		// the wave kernel's walks of many candidates go to the wave-parallel walk
		// (BT2X_DP_WAVE_HAND candidates, default 16; 0: never); read per launch
		const char* wh = getenv("BT2X_DP_WAVE_HAND");
		a.wave_hand = wh ? (uint32_t)atol(wh) : 16u;
	}
	static const bool prof = [] { const char* e = getenv("BT2X_DP_PROF"); return e && e[0] == '1'; }();
	if(prof) { a.prof = c->d_stats + 16; HIPCHK(hipMemsetAsync(a.prof, 0, 14 * sizeof(unsigned long long), s)); }
	HIPCHK(hipEventRecord(c->ev[BT2X_K_DP][0], s));
	// every problem's window goes to a BT2X_MAX_COLS-byte slot (cut from the index for
	// BT2X_DP_REF_TEXT problems, copied from d_refs for the others): the fill kernel reads
	// its window as aligned dwords, 16 columns per load
	if((launch_flags & BT2X_DPL_REF_TEXT) && (!c->ix.text || !c->ix.rstarts)) return BT2X_E_ARG;
	if((rc = c->b_in2.ensure(sizeof(bt2x_dp_in) * (size_t)(n ? n : 1))) ||
	   (rc = c->b_win.ensure((size_t)kWinSlot * (n ? n : 1) + 64)))
		return rc;
	if((rc = bt2x_launch_windows(c->ix, d_in, n, d_refs, (bt2x_dp_in*)c->b_in2.p, (uint8_t*)c->b_win.p, s))) return rc;
	a.in = (const bt2x_dp_in*)c->b_in2.p;
	a.refs = (const uint8_t*)c->b_win.p;
	rc = bt2x_launch_dp(c->sc, a, s);
	HIPCHK(hipEventRecord(c->ev[BT2X_K_DP][1], s));
	if(prof) {                                   // development: where a lane-kernel wave's time goes
		unsigned long long pv[14];
		HIPCHK(hipStreamSynchronize(s));
		HIPCHK(hipMemcpy(pv, a.prof, sizeof pv, hipMemcpyDeviceToHost));
		float ms = 0;
		hipEventElapsedTime(&ms, c->ev[BT2X_K_DP][0], c->ev[BT2X_K_DP][1]);
		uint32_t nheavy = 0;
		if(a.heavy_list) HIPCHK(hipMemcpy(&nheavy, a.heavy_list, sizeof nheavy, hipMemcpyDeviceToHost));
		std::fprintf(stderr, "BT2X_DP_PROF n=%u ms=%.3f groups=%llu fill_cyc=%llu walk_cyc=%llu walk_steps=%llu cand_iters=%llu "
		             "max_wave_cyc=%llu max_fill_cyc=%llu max_walk_cyc=%llu heavy=%u lane_work_sum=%llu "
		             "wave_lane_max_sum=%llu lane_max=%llu pro_cyc=%llu pair_cyc=%llu cand_cyc=%llu\n",
		             n, ms, pv[4], pv[0], pv[1], pv[2], pv[3], pv[5], pv[6], pv[7], nheavy, pv[8], pv[9], pv[10], pv[11],
		             pv[12], pv[13]);
	}
	c->ev_valid[BT2X_K_DP] = true;
	c->n_dp_last = n;
	return rc;
}

extern "C" int bt2x_capabilities(const bt2x_ctx* c, uint32_t* caps) {
	if(!c || !caps) return BT2X_E_ARG;
	*caps = (c->ix.text && c->ix.rstarts) ? BT2X_CAP_REF_TEXT : 0u;
	return BT2X_OK;
}

extern "C" int bt2x_dp_align(bt2x_ctx* c,
                             const uint8_t* reads, uint64_t reads_bytes,
                             const uint8_t* quals, uint64_t quals_bytes,
                             const uint8_t* refs, uint64_t refs_bytes,
                             const bt2x_dp_in* in, uint32_t n,
                             bt2x_dp_out* out,
                             bt2x_aln_rec* recs, uint32_t rec_cap, uint32_t* nrec_used,
                             uint32_t* edits, uint32_t edit_cap, uint32_t* nedit_used,
                             bt2x_dp_debug* debug) {
	// reads == quals == NULL: read_off / qual_off index the read store (bt2x_store_reads)
	const bool from_store = !reads && !quals;
	if(from_store) reads_bytes = quals_bytes = c ? c->store_hw : 0;
	if(!c || (n && ((!from_store && (!reads || !quals)) || (!refs && refs_bytes) || !in || !out))) return BT2X_E_ARG;
	if(nrec_used) *nrec_used = 0;
	if(nedit_used) *nedit_used = 0;
	if(n == 0) return BT2X_OK;
	// shape checks: the kernel trusts these (reference limits; the u8 kernel's
	// minsc floor, aligner_sw.cpp:77-83)
	uint32_t launch_flags = c->exact_best ? BT2X_DPL_EXACT_BEST : 0u;
	const bool can_text = c->ix.text && c->ix.rstarts;
	for(uint32_t i = 0; i < n; i++) {
		const bt2x_dp_in& p = in[i];
		const bool i16 = (p.flags & BT2X_DP_I16) != 0, text = (p.flags & BT2X_DP_REF_TEXT) != 0;
		if(p.rdlen < 1 || p.rdlen > BT2X_MAX_ROWS || p.ncol < 1 || p.ncol + 1 > BT2X_MAX_COLS ||
		   p.read_off + p.rdlen > reads_bytes || p.qual_off + p.rdlen > quals_bytes ||
		   (text ? (!can_text || p.ref_off >= c->npat) : p.ref_off + p.ncol > refs_bytes) ||
		   p.minsc < (i16 ? -32767 : -254) || p.minsc > 0 || (p.flags & ~(BT2X_DP_I16 | BT2X_DP_REF_TEXT)) != 0)
			return BT2X_E_ARG;
		if(i16) launch_flags |= BT2X_DPL_I16;
		if(text) launch_flags |= BT2X_DPL_REF_TEXT;
	}
	HIPCHK(hipSetDevice(c->device));
	int rc;
	if((!from_store && ((rc = c->b_reads.ensure(reads_bytes)) || (rc = c->b_quals.ensure(quals_bytes)))) ||
	   (rc = c->b_refs.ensure(refs_bytes ? refs_bytes : 1)) || (rc = c->b_in.ensure(sizeof(bt2x_dp_in) * n)) ||
	   (rc = c->b_out.ensure(sizeof(bt2x_dp_out) * n)) ||
	   (rc = c->b_recs.ensure(sizeof(bt2x_aln_rec) * (size_t)(rec_cap ? rec_cap : 1))) ||
	   (rc = c->b_edits.ensure(sizeof(uint32_t) * (size_t)(edit_cap ? edit_cap : 1)))) return rc;
	bt2x_dp_debug dd{nullptr, nullptr};
	if(debug && debug->digests) {
		if((rc = c->b_dbg_dig.ensure(sizeof(uint64_t) * 3 * n))) return rc;
		dd.digests = (uint64_t*)c->b_dbg_dig.p;
	}
	if(debug && debug->cands) {
		if((rc = c->b_dbg_cand.ensure(sizeof(uint32_t) * BT2X_MAX_COLS * n))) return rc;
		dd.cands = (uint32_t*)c->b_dbg_cand.p;
	}
	if(!from_store) {
		HIPCHK(hipMemcpyAsync(c->b_reads.p, reads, reads_bytes, hipMemcpyHostToDevice, c->stream));
		HIPCHK(hipMemcpyAsync(c->b_quals.p, quals, quals_bytes, hipMemcpyHostToDevice, c->stream));
	}
	if(refs_bytes) HIPCHK(hipMemcpyAsync(c->b_refs.p, refs, refs_bytes, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->b_in.p, in, sizeof(bt2x_dp_in) * n, hipMemcpyHostToDevice, c->stream));
	rc = bt2x_dp_align_dev(c, from_store ? c->d_store : (const uint8_t*)c->b_reads.p,
	                       from_store ? c->d_store : (const uint8_t*)c->b_quals.p,
	                       (const uint8_t*)c->b_refs.p, (const bt2x_dp_in*)c->b_in.p, n,
	                       (bt2x_dp_out*)c->b_out.p, (bt2x_aln_rec*)c->b_recs.p, rec_cap,
	                       (uint32_t*)c->b_edits.p, edit_cap, c->d_counters,
	                       (dd.digests || dd.cands) ? &dd : nullptr, launch_flags, c->stream);
	if(rc) return rc;
	uint32_t used[4] = {0, 0, 0, 0};
	HIPCHK(hipMemcpyAsync(used, c->d_counters, sizeof used, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipMemcpyAsync(out, c->b_out.p, sizeof(bt2x_dp_out) * n, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	if(nrec_used) *nrec_used = used[0];
	if(nedit_used) *nedit_used = used[1];
	if(used[3]) return BT2X_E_ARG;                            // cannot happen: launch_flags cover in[]
	if(used[0] > rec_cap || used[1] > edit_cap) return BT2X_E_OVERFLOW;
	if(used[0]) HIPCHK(hipMemcpyAsync(recs, c->b_recs.p, sizeof(bt2x_aln_rec) * used[0], hipMemcpyDeviceToHost, c->stream));
	if(used[1]) HIPCHK(hipMemcpyAsync(edits, c->b_edits.p, sizeof(uint32_t) * used[1], hipMemcpyDeviceToHost, c->stream));
	if(dd.digests) HIPCHK(hipMemcpyAsync(debug->digests, dd.digests, sizeof(uint64_t) * 3 * n, hipMemcpyDeviceToHost, c->stream));
	if(dd.cands) HIPCHK(hipMemcpyAsync(debug->cands, dd.cands, sizeof(uint32_t) * BT2X_MAX_COLS * n, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	return BT2X_OK;
}

// Struct sizes, so bindings can check their mirrors of bt2x.h.
extern "C" int bt2x_abi_sizes(uint32_t* out, int n) {
	const uint32_t s[] = {(uint32_t)sizeof(bt2x_seed_in), (uint32_t)sizeof(bt2x_seed_out),
	                      (uint32_t)sizeof(bt2x_dp_in), (uint32_t)sizeof(bt2x_dp_out),
	                      (uint32_t)sizeof(bt2x_aln_rec), (uint32_t)sizeof(bt2x_scoring),
	                      (uint32_t)sizeof(bt2x_index_desc), (uint32_t)sizeof(bt2x_counters),
	                      (uint32_t)sizeof(bt2x_resolve_in), (uint32_t)sizeof(bt2x_resolve_out),
	                      (uint32_t)sizeof(bt2x_round_in), (uint32_t)sizeof(bt2x_round_out),
	                      (uint32_t)sizeof(bt2x_sat), (uint32_t)sizeof(bt2x_exrange), (uint32_t)sizeof(bt2x_elt),
	                      (uint32_t)sizeof(bt2x_store_in), (uint32_t)sizeof(bt2x_sam_req)};
	const int m = (int)(sizeof s / sizeof s[0]);
	for(int i = 0; i < n && i < m; i++) out[i] = s[i];
	return m;
}

extern "C" int bt2x_suffix_array(bt2x_ctx* c, uint64_t first, uint64_t n, uint32_t* out) {
	if(!c || !out) return BT2X_E_ARG;
	if(!c->ix.sa) return BT2X_E_ARG;
	if(first + n > c->ix.len + 1) return BT2X_E_ARG;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipMemcpy(out, c->ix.sa + first, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
	return BT2X_OK;
}

// ---------------------------------------------------------------- SA resolve
extern "C" int bt2x_resolve_dev(bt2x_ctx* c, const bt2x_resolve_in* d_in, uint32_t n, int reject_straddle,
                                bt2x_resolve_out* d_out, void* stream) {
	if(!c) return BT2X_E_ARG;
	if(!c->ix.sa && !c->ix.offs) return BT2X_E_ARG;       // index loaded without load_offs
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipMemsetAsync(c->d_stats + 8, 0, 3 * sizeof(unsigned long long), s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_RESOLVE][0], s));
	const int rc = bt2x_launch_resolve(c->ix, d_in, n, reject_straddle ? 1 : 0, d_out, c->d_stats + 8, s);
	HIPCHK(hipEventRecord(c->ev[BT2X_K_RESOLVE][1], s));
	c->ev_valid[BT2X_K_RESOLVE] = true;
	c->n_resolve_last = n;
	c->d_resolve_n = nullptr;
	return rc;
}

// ------------------------------------------------------------------- seed round
extern "C" int bt2x_seed_round_dev(bt2x_ctx* c, const uint8_t* d_reads, const bt2x_seed_in* d_seeds, uint32_t nseeds,
                                   const bt2x_round_in* d_in, uint32_t nreads, const bt2x_exrange* d_exr,
                                   uint32_t maxelt, bt2x_round_out* d_out, bt2x_sat* d_sats, uint32_t sat_cap,
                                   bt2x_elt* d_elts, uint32_t elt_cap, bt2x_exrange* d_exr_out,
                                   uint32_t exr_cap, uint32_t* d_used, void* stream) {
	if(!c || !d_used) return BT2X_E_ARG;
	if(!c->ix.sa && !c->ix.offs) return BT2X_E_ARG;        // index loaded without load_offs
	if(c->npat >= BT2X_ELT_TIDX_NONE || c->ix.len >= (1ull << 39)) return BT2X_E_ARG;   // bt2x_elt's fields
	hipStream_t s = stream ? (hipStream_t)stream : c->stream;
	HIPCHK(hipSetDevice(c->device));
	int rc;
	const uint32_t lanes = bt2x_round_lanes(c->ncu);
	// sampling jobs: at most one per read; their ranges: 24 per job on average before a
	// read is handed back (a read has at most 2 x 64 ranges, typically a few)
	const uint32_t job_cap = nreads ? nreads : 1, range_cap = 24 * job_cap;
	if((rc = c->b_sout.ensure(sizeof(bt2x_seed_out) * (size_t)(nseeds ? nseeds : 1))) ||
	   (rc = c->b_rows.ensure(sizeof(bt2x_resolve_in) * (size_t)(elt_cap ? elt_cap : 1))) ||
	   (rc = c->b_ws.ensure(bt2x_round_ws_bytes() * lanes)) ||
	   (rc = c->b_jobs.ensure(bt2x_round_job_bytes() * job_cap)) ||
	   (rc = c->b_ranges.ensure(bt2x_round_range_bytes() * range_cap)) ||
	   (rc = c->b_rcnt.ensure(kRoundCounters * sizeof(uint32_t)))) return rc;
	uint32_t* cnt = (uint32_t*)c->b_rcnt.p;
	HIPCHK(hipEventRecord(c->ev[BT2X_K_ROUND][0], s));
	HIPCHK(hipMemsetAsync(cnt, 0, kRoundCounters * sizeof(uint32_t), s));
	if(!d_seeds && nseeds) {                         // instantiateSeeds on the GPU
		if((rc = c->b_gseeds.ensure(sizeof(bt2x_seed_in) * (size_t)nseeds)) ||
		   (rc = bt2x_launch_seed_gen(d_reads, d_in, nreads, (bt2x_seed_in*)c->b_gseeds.p, nseeds, cnt + kRoundSeedMismatch, s)))
			return rc;
		d_seeds = (const bt2x_seed_in*)c->b_gseeds.p;
	}
	// 1. seed search (searchAllSeedsDoAll)
	HIPCHK(hipMemsetAsync(c->d_stats, 0, 3 * sizeof(unsigned long long), s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_SEED][0], s));
	if((rc = bt2x_launch_seed(c->ix, d_reads, d_seeds, nseeds, 1, (bt2x_seed_out*)c->b_sout.p, c->d_stats, c->ncu, s)))
		return rc;
	HIPCHK(hipEventRecord(c->ev[BT2X_K_SEED][1], s));
	c->ev_valid[BT2X_K_SEED] = true;
	c->n_seed_last = nseeds;
	c->n_round_last = nreads;
	// 2. finalize + rank + prioritize per read, then 3. place every row
	HIPCHK(hipMemsetAsync(c->d_stats + 8, 0, 3 * sizeof(unsigned long long), s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_RESOLVE][0], s));
	RoundLaunch a;
	a.seeds = d_seeds; a.seed_out = (const bt2x_seed_out*)c->b_sout.p;
	a.in = d_in; a.n = nreads; a.exr = d_exr; a.maxelt = maxelt;
	a.out = d_out; a.sats = d_sats; a.sat_cap = sat_cap;
	a.rows = (bt2x_resolve_in*)c->b_rows.p; a.row_cap = elt_cap;
	a.exr_out = d_exr_out; a.exr_cap = exr_cap;
	a.counters = cnt; a.ws = (uint8_t*)c->b_ws.p; a.nlanes = lanes;
	a.jobs = (uint8_t*)c->b_jobs.p; a.job_cap = job_cap; a.ranges = (uint8_t*)c->b_ranges.p; a.range_cap = range_cap;
	if((rc = bt2x_launch_round(a, s))) return rc;
	if((rc = bt2x_launch_resolve_dn(c->ix, a.rows, cnt + 1, elt_cap, 0, d_elts, c->d_stats + 8, c->ncu, s)))
		return rc;
	HIPCHK(hipMemcpyAsync(d_used, cnt, 3 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
	HIPCHK(hipMemcpyAsync(d_used + 3, cnt + kRoundSeedMismatch, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_RESOLVE][1], s));
	HIPCHK(hipEventRecord(c->ev[BT2X_K_ROUND][1], s));
	c->ev_valid[BT2X_K_RESOLVE] = c->ev_valid[BT2X_K_ROUND] = true;
	c->d_resolve_n = cnt + 1;
	return BT2X_OK;
}

extern "C" int bt2x_seed_round(bt2x_ctx* c, const uint8_t* reads, uint64_t reads_bytes,
                               const bt2x_seed_in* seeds, uint32_t nseeds,
                               const bt2x_round_in* in, uint32_t nreads,
                               const bt2x_exrange* exr, uint32_t nexr, uint32_t maxelt,
                               bt2x_round_out* out,
                               bt2x_sat* sats, uint32_t sat_cap,
                               bt2x_elt* elts, uint32_t elt_cap,
                               bt2x_exrange* exr_out, uint32_t exr_cap,
                               uint32_t used[3]) {
	// reads == NULL: read_off indexes the read store (bt2x_store_reads)
	const bool from_store = !reads;
	if(from_store) reads_bytes = c ? c->store_hw : 0;
	if(!c || !used || (nreads && (!in || !out))) return BT2X_E_ARG;
	used[0] = used[1] = used[2] = 0;
	if(nreads == 0) return BT2X_OK;
	for(uint32_t i = 0; i < nseeds && seeds; i++)
		if(seeds[i].seed_len < 1 || seeds[i].seed_len > 32 || seeds[i].read_off + seeds[i].seed_off + seeds[i].seed_len > reads_bytes)
			return BT2X_E_ARG;
	for(uint32_t r = 0; r < nreads; r++) {
		const bt2x_round_in& q = in[r];
		if(q.seed0 + q.nseeds > nseeds || (uint64_t)q.exr0 + q.nexr > nexr || q.interval == 0 || q.seedlen == 0 ||
		   q.read_off + 2ull * q.rdlen > reads_bytes)
			return BT2X_E_ARG;
		// seeds instantiated on the GPU: every one inside the read
		if(!seeds && (q.seedlen > 32 || q.seedlen > q.rdlen || (uint64_t)(q.num_offs ? q.num_offs - 1 : 0) * q.interval + q.offset + q.seedlen > q.rdlen))
			return BT2X_E_ARG;
	}
	HIPCHK(hipSetDevice(c->device));
	int rc;
	if((!from_store && (rc = c->b_reads.ensure(reads_bytes ? reads_bytes : 1))) ||
	   (rc = c->b_in.ensure(sizeof(bt2x_seed_in) * (size_t)(nseeds ? nseeds : 1))) ||
	   (rc = c->b_rin.ensure(sizeof(bt2x_round_in) * nreads)) ||
	   (rc = c->b_exr.ensure(sizeof(bt2x_exrange) * (size_t)(nexr ? nexr : 1))) ||
	   (rc = c->b_rout.ensure(sizeof(bt2x_round_out) * nreads)) ||
	   (rc = c->b_sats.ensure(sizeof(bt2x_sat) * (size_t)(sat_cap ? sat_cap : 1))) ||
	   (rc = c->b_elts.ensure(sizeof(bt2x_elt) * (size_t)(elt_cap ? elt_cap : 1))) ||
	   (rc = c->b_exro.ensure(sizeof(bt2x_exrange) * (size_t)(exr_cap ? exr_cap : 1))) ||
	   (rc = c->b_used.ensure(4 * sizeof(uint32_t)))) return rc;
	if(reads_bytes && !from_store) HIPCHK(hipMemcpyAsync(c->b_reads.p, reads, reads_bytes, hipMemcpyHostToDevice, c->stream));
	if(nseeds && seeds) HIPCHK(hipMemcpyAsync(c->b_in.p, seeds, sizeof(bt2x_seed_in) * nseeds, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->b_rin.p, in, sizeof(bt2x_round_in) * nreads, hipMemcpyHostToDevice, c->stream));
	if(nexr) HIPCHK(hipMemcpyAsync(c->b_exr.p, exr, sizeof(bt2x_exrange) * nexr, hipMemcpyHostToDevice, c->stream));
	rc = bt2x_seed_round_dev(c, from_store ? c->d_store : (const uint8_t*)c->b_reads.p, seeds ? (const bt2x_seed_in*)c->b_in.p : nullptr, nseeds,
	                         (const bt2x_round_in*)c->b_rin.p, nreads, (const bt2x_exrange*)c->b_exr.p, maxelt,
	                         (bt2x_round_out*)c->b_rout.p, (bt2x_sat*)c->b_sats.p, sat_cap,
	                         (bt2x_elt*)c->b_elts.p, elt_cap, (bt2x_exrange*)c->b_exro.p, exr_cap,
	                         (uint32_t*)c->b_used.p, c->stream);
	if(rc) return rc;
	uint32_t u4[4] = {0, 0, 0, 0};
	HIPCHK(hipMemcpyAsync(u4, c->b_used.p, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipMemcpyAsync(out, c->b_rout.p, sizeof(bt2x_round_out) * nreads, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	used[0] = u4[0]; used[1] = u4[1]; used[2] = u4[2];
	if(u4[3]) return BT2X_E_ARG;                       // some in[r].nseeds != the seeds its read gives
	if(used[0] > sat_cap || used[1] > elt_cap || used[2] > exr_cap) return BT2X_E_OVERFLOW;
	if(used[0]) HIPCHK(hipMemcpyAsync(sats, c->b_sats.p, sizeof(bt2x_sat) * used[0], hipMemcpyDeviceToHost, c->stream));
	if(used[1]) HIPCHK(hipMemcpyAsync(elts, c->b_elts.p, sizeof(bt2x_elt) * used[1], hipMemcpyDeviceToHost, c->stream));
	if(used[2]) HIPCHK(hipMemcpyAsync(exr_out, c->b_exro.p, sizeof(bt2x_exrange) * used[2], hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	return BT2X_OK;
}

extern "C" int bt2x_store_reads(bt2x_ctx* c, const uint8_t* packed, uint64_t packed_bytes, const bt2x_store_in* in,
                                uint32_t n) {
	if(!c || (n && (!packed || !in))) return BT2X_E_ARG;
	if(n == 0) return BT2X_OK;
	uint32_t top = 0;
	for(uint32_t i = 0; i < n; i++) {
		if(in[i].len < 1 || in[i].len > BT2X_STORE_MAX_LEN || in[i].off + 2ull * in[i].len > packed_bytes) return BT2X_E_ARG;
		top = std::max(top, in[i].slot);
	}
	HIPCHK(hipSetDevice(c->device));
	const uint64_t need = ((uint64_t)top + 1) * BT2X_STORE_SLOT_BYTES;
	if(need > c->store_bytes) {                      // grow, keeping the slots already written
		const uint64_t want = std::max<uint64_t>(need + need / 4, (uint64_t)1 << 20);
		void* p = nullptr;
		if(hipMalloc(&p, want) != hipSuccess) return BT2X_E_NOMEM;
		// the new region reads as N codes until a read is put there
		HIPCHK(hipMemsetAsync((uint8_t*)p + c->store_bytes, 4, want - c->store_bytes, c->stream));
		if(c->d_store) {
			HIPCHK(hipMemcpyAsync(p, c->d_store, c->store_bytes, hipMemcpyDeviceToDevice, c->stream));
			HIPCHK(hipStreamSynchronize(c->stream));
			(void)hipFree(c->d_store);
		}
		c->d_store = (uint8_t*)p;
		c->store_bytes = want;
	}
	c->store_hw = std::max(c->store_hw, need);
	int rc;
	if((rc = c->b_pack.ensure(packed_bytes)) || (rc = c->b_sin.ensure(sizeof(bt2x_store_in) * n))) return rc;
	HIPCHK(hipMemcpyAsync(c->b_pack.p, packed, packed_bytes, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->b_sin.p, in, sizeof(bt2x_store_in) * n, hipMemcpyHostToDevice, c->stream));
	if((rc = bt2x_launch_store((const uint8_t*)c->b_pack.p, (const bt2x_store_in*)c->b_sin.p, n, c->d_store, c->stream)))
		return rc;
	HIPCHK(stream_wait(c));                          // the caller may reuse `packed` on return
	return BT2X_OK;
}

// ---------------------------------------------------------------- SAM tails
extern "C" int bt2x_sam_tails_dev(bt2x_ctx* c, const bt2x_sam_req* d_req, uint32_t n, char* d_text, uint16_t* d_lens,
                                  void* stream) {
	if(!c || (n && (!d_req || !d_text || !d_lens))) return BT2X_E_ARG;
	if(n == 0) return BT2X_OK;
	if(!c->d_store) return BT2X_E_ARG;
	HIPCHK(hipSetDevice(c->device));
	return bt2x_launch_sam_tails(d_req, n, c->d_store, d_text, d_lens, c->ncu, stream ? stream : (void*)c->stream);
}

extern "C" int bt2x_sam_tails(bt2x_ctx* c, const bt2x_sam_req* req, uint32_t n, char* text, uint64_t text_bytes,
                              uint16_t* lens) {
	if(!c || (n && (!req || !text || !lens))) return BT2X_E_ARG;
	if(n == 0) return BT2X_OK;
	for(uint32_t i = 0; i < n; i++) {                // the kernel trusts these
		const bt2x_sam_req& q = req[i];
		if(q.rdlen < 1 || q.rdlen > BT2X_STORE_MAX_LEN || q.nmm > BT2X_SAM_MAX_MM) return BT2X_E_ARG;
		if((uint64_t)(q.slot + 1) * BT2X_STORE_SLOT_BYTES > c->store_hw) return BT2X_E_ARG;
		if(q.text_off + BT2X_SAM_TAIL_MAX(q.rdlen, q.nmm) > text_bytes) return BT2X_E_ARG;
		for(int e = 0; e < q.nmm; e++)
			if(q.mm_pos[e] >= q.rdlen || (e && q.mm_pos[e] <= q.mm_pos[e - 1])) return BT2X_E_ARG;
	}
	HIPCHK(hipSetDevice(c->device));
	int rc;
	if((rc = c->b_sreq.ensure(sizeof(bt2x_sam_req) * n)) || (rc = c->b_stext.ensure(text_bytes)) ||
	   (rc = c->b_slens.ensure(sizeof(uint16_t) * n)))
		return rc;
	HIPCHK(hipMemcpyAsync(c->b_sreq.p, req, sizeof(bt2x_sam_req) * n, hipMemcpyHostToDevice, c->stream));
	if((rc = bt2x_sam_tails_dev(c, (const bt2x_sam_req*)c->b_sreq.p, n, (char*)c->b_stext.p, (uint16_t*)c->b_slens.p,
	                            c->stream)))
		return rc;
	HIPCHK(hipMemcpyAsync(lens, c->b_slens.p, sizeof(uint16_t) * n, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipMemcpyAsync(text, c->b_stext.p, text_bytes, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	return BT2X_OK;
}

extern "C" int bt2x_resolve(bt2x_ctx* c, const bt2x_resolve_in* in, uint32_t n, int reject_straddle,
                            bt2x_resolve_out* out) {
	if(!c || (n && (!in || !out))) return BT2X_E_ARG;
	if(!c->ix.sa && !c->ix.offs) return BT2X_E_ARG;
	if(n == 0) return BT2X_OK;
	for(uint32_t i = 0; i < n; i++) if(in[i].row > c->ix.len) return BT2X_E_ARG;
	HIPCHK(hipSetDevice(c->device));
	int rc;
	if((rc = c->b_in.ensure(sizeof(bt2x_resolve_in) * n)) || (rc = c->b_out.ensure(sizeof(bt2x_resolve_out) * n)))
		return rc;
	HIPCHK(hipMemcpyAsync(c->b_in.p, in, sizeof(bt2x_resolve_in) * n, hipMemcpyHostToDevice, c->stream));
	rc = bt2x_resolve_dev(c, (const bt2x_resolve_in*)c->b_in.p, n, reject_straddle,
	                      (bt2x_resolve_out*)c->b_out.p, c->stream);
	if(rc) return rc;
	HIPCHK(hipMemcpyAsync(out, c->b_out.p, sizeof(bt2x_resolve_out) * n, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(stream_wait(c));
	return BT2X_OK;
}
