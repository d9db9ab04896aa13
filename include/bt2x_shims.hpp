// bt2x_shims.hpp — C++ host side above the bt2x C-ABI, mirroring the reference's call
// surface for the hot path so bt2_search.cpp's per-read loop can keep
// its shape:
//
//   MultiSeedAlignerHip  ~ MultiSeedAligner::searchAllSeedsDoAll(doExtend)
//                          (aligner_seed.cpp:674-725; params/data = aligner_seed.cpp:81-202)
//   SwAlignerHip         ~ SwAligner::initRead / initRef / align / nextAlignment / done /
//                          reset (aligner_sw.cpp:35, :117, :235, :252; aligner_sw.h:322,342)
//   SwBatch              the same per-problem calls, queued: many initRead/initRef
//                          problems, one GPU launch, then per-problem align()/nextAlignment()
//                          replayed from the results (what a batched extendSeeds uses).
//
// Header-only, duck-typed over the reference's own types so it compiles inside the
// reference's TU without including them here:
//   read strings  S: s[i] -> code 0..4, s.length()      (BTDnaString, sstring.h)
//   quality str   Q: q[i] -> Phred+33 char               (BTString)
//   scoring       Sc: sc.nCeil.template f<int>(double)   (Scoring, scoring.h:449)
//   reference     Refs: refs.getBase(tidx, toff) -> 0..4 (BitPairReference, reference.h:89)
//   rectangle     Rect: refl, refr, triml, corel, corer  (DPRect, dp_framer.h:62-88)
//   RNG           Rnd: nextU32(), init(uint32_t)         (RandomSource, random_source.h:46-52)
// Per-call failures return false exactly where the reference's methods do (rows > 160,
// rflen + 1 > 200, no alignment); device/ABI failures throw bt2x::Error (the reference
// aborts with `throw 1` on fatal errors).  There is no CPU fallback.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "bt2x.h"

namespace bt2x {

struct Error : std::runtime_error {
	int code;
	Error(int rc, const std::string& what) : std::runtime_error(what + ": bt2x error " + std::to_string(rc)), code(rc) {}
};

inline void check(int rc, const char* what) { if(rc != BT2X_OK) throw Error(rc, what); }

// SwAligner::nextAlignment's per-candidate RNG use: u8 kernel (aligner_sw.cpp:324-336)
// reseed = nextU32()+1; init(reseed); backtrace; init(reseed+1); i16 kernel (:338-348)
// reseed = nextU32()+1; backtrace; init(reseed).  The backtraces draw nothing.
template<class Rnd>
inline void replay_backtrace_draws(Rnd& rnd, unsigned ntries, bool i16 = false) {
	for(unsigned t = 0; t < ntries; t++) {
		const uint32_t reseed = rnd.nextU32() + 1;
		rnd.init(reseed);
		if(!i16) rnd.init(reseed + 1);
	}
}

// SwAligner::initRef's kernel choice (aligner_sw.cpp:77-83): a -DENABLE_I16 build runs
// the i16 kernel unless enable8 && minsc >= -254 and leaves minsc as is; the stock build
// always runs u8 with minsc clamped to -254.  The shims follow the build they are
// compiled into (the reference's own ENABLE_I16 macro).
#ifdef ENABLE_I16
constexpr bool kI16Build = true;
#else
constexpr bool kI16Build = false;
#endif
inline bool dp_uses_i16(bool i16build, bool enable8, int64_t minsc) { return i16build && !(enable8 && minsc >= -254); }

// -------------------------------------------------------------- index / device

class Index {
public:
	explicit Index(const char* basename, bool load_offs = false) {
		std::memset(&d_, 0, sizeof(d_));
		check(bt2x_index_load(basename, load_offs ? 1 : 0, &d_), "bt2x_index_load");
	}
	~Index() { bt2x_index_free(&d_); }
	Index(const Index&) = delete;
	Index& operator=(const Index&) = delete;
	const bt2x_index_desc& desc() const { return d_; }
private:
	bt2x_index_desc d_;
};

// One context per GPU (index + scoring uploaded once).
class Device {
public:
	Device(int hip_device, const Index& idx, const bt2x_scoring& sc) : sc_(sc) {
		check(bt2x_open(hip_device, &idx.desc(), &sc, &ctx_), "bt2x_open");
	}
	~Device() { bt2x_close(ctx_); }
	Device(const Device&) = delete;
	Device& operator=(const Device&) = delete;
	bt2x_ctx* ctx() const { return ctx_; }
	const bt2x_scoring& scoring() const { return sc_; }
private:
	bt2x_ctx* ctx_ = nullptr;
	bt2x_scoring sc_;
};

// ---------------------------------------------------------------- seed search

// The flattened seed batch of MultiSeedAligner (_paramVec/_dataVec,
// aligner_seed.cpp:561-581): add() one entry per instantiated seed, then
// searchAllSeedsDoAll() fills data(i) = {topf, botf, nlex, need_reporting}.
class MultiSeedAlignerHip {
public:
	explicit MultiSeedAlignerHip(Device& dev) : dev_(dev) {}
	void clear() { reads_.clear(); in_.clear(); out_.clear(); last_ = nullptr; }
	// seq = the oriented read (patFw for fw seeds, patRc for rc), codes 0..4.
	// The read is copied once per distinct pointer in a row (seeds of one read share it).
	uint32_t add(const uint8_t* seq, size_t read_len, size_t seed_off, size_t seed_len) {
		if(seq != last_ || read_len != last_len_) {
			last_off_ = reads_.size();
			reads_.insert(reads_.end(), seq, seq + read_len);
			last_ = seq; last_len_ = read_len;
		}
		bt2x_seed_in s;
		std::memset(&s, 0, sizeof(s));
		s.read_off = last_off_;
		s.seed_off = (uint8_t)seed_off;
		s.seed_len = (uint8_t)seed_len;
		in_.push_back(s);
		return (uint32_t)(in_.size() - 1);
	}
	template<class S>
	uint32_t add(const S& read, size_t seed_off, size_t seed_len) {
		tmp_.resize(read.length());
		for(size_t i = 0; i < tmp_.size(); i++) tmp_[i] = (uint8_t)read[i];
		last_ = nullptr;
		return add(tmp_.data(), tmp_.size(), seed_off, seed_len);
	}
	// == MultiSeedAligner::searchAllSeedsDoAll(doExtend); false on a device error.
	bool searchAllSeedsDoAll(bool doExtend) {
		out_.resize(in_.size());
		if(in_.empty()) return true;
		return bt2x_seed_search(dev_.ctx(), reads_.data(), reads_.size(), in_.data(),
		                        (uint32_t)in_.size(), doExtend ? 1 : 0, out_.data()) == BT2X_OK;
	}
	size_t size() const { return in_.size(); }
	const bt2x_seed_out& data(uint32_t i) const { return out_[i]; }
private:
	Device& dev_;
	std::vector<uint8_t> reads_, tmp_;
	std::vector<bt2x_seed_in> in_;
	std::vector<bt2x_seed_out> out_;
	const uint8_t* last_ = nullptr;
	size_t last_len_ = 0, last_off_ = 0;
};

// Per-read seed hits after the seed kernel: SeedAligner::searchAllSeedsFinalize
// (aligner_seed.cpp:508-540) feeds every need_reporting seed to SeedResults::add
// (aligner_seed.h:603-641) as a QVal of one BW range with botf - topf elements; then
// rankSeedHits (aligner_seed.h:1000-1061) orders them for extension and hitsByRank
// (:1120-1145) reads the order back.  Rnd: nextBool(), nextU32() (RandomSource).
class SeedHitsHip {
public:
	struct Hit {
		uint64_t topf = 0, botf = 0;
		uint8_t nlex = 0;
		bool valid = false;
		uint64_t numElts() const { return botf - topf; }
	};
	// SeedResults::clearSeeds + reset: numOffs seed offsets per strand.
	void reset(uint32_t numOffs) {
		numOffs_ = numOffs;
		hits_[0].assign(numOffs, Hit()); hits_[1].assign(numOffs, Hit());
		sorted_[0].assign(numOffs, false); sorted_[1].assign(numOffs, false);
		rankOffs_.clear(); rankFws_.clear();
		nonzTot_ = nonzFw_ = nonzRc_ = uniTot_ = repTot_ = 0;
		numElts_ = numEltsFw_ = numEltsRc_ = 0;
	}
	// searchAllSeedsFinalize's per-seed step: seed i of strand fw, kernel output d.
	void add(uint32_t seedIdx, bool fw, const bt2x_seed_out& d) {
		if(!d.need_reporting || seedIdx >= numOffs_) return;
		Hit& h = hits_[fw ? 0 : 1][seedIdx];
		h.topf = d.topf; h.botf = d.botf; h.nlex = d.nlex; h.valid = true;
		const uint64_t n = h.numElts();
		(fw ? numEltsFw_ : numEltsRc_) += n;
		(fw ? nonzFw_ : nonzRc_)++;
		numElts_ += n;
		nonzTot_++;
		if(n == 1) uniTot_++; else repTot_++;
	}
	template<class Rnd>
	void rankSeedHits(Rnd& rnd, bool all) {
		if(all) {
			for(uint32_t i = 1; i < numOffs_; i++)
				for(int fwi = 0; fwi <= 1; fwi++)
					if(hits_[fwi][i].valid && hits_[fwi][i].numElts() > 0) push(i, fwi == 0);
			if(numOffs_ > 0 && hits_[0][0].valid && hits_[0][0].numElts() > 0) push(0, true);
			if(numOffs_ > 0 && hits_[1][0].valid && hits_[1][0].numElts() > 0) push(0, false);
			return;
		}
		while(rankOffs_.size() < nonzTot_) {
			uint64_t minsz = 0xffffffffu;              // MAX_U32 (aligner_seed.h:1024)
			uint32_t minidx = 0;
			bool minfw = true;
			const bool rb = rnd.nextBool();
			for(int fwi = 0; fwi <= 1; fwi++) {
				const bool fw = (fwi == (rb ? 1 : 0));
				const std::vector<Hit>& rrs = hits_[fw ? 0 : 1];
				const std::vector<bool>& sorted = sorted_[fw ? 0 : 1];
				uint32_t i = rnd.nextU32() % numOffs_;
				for(uint32_t ii = 0; ii < numOffs_; ii++) {
					if(rrs[i].valid && rrs[i].numElts() > 0 && !sorted[i] && rrs[i].numElts() < minsz) {
						minsz = rrs[i].numElts(); minidx = i; minfw = fw;
					}
					if(++i == numOffs_) i = 0;
				}
			}
			if(minsz == 0xffffffffu) throw Error(BT2X_E_ARG, "rankSeedHits: no rankable hit");
			sorted_[minfw ? 0 : 1][minidx] = true;
			push(minidx, minfw);
		}
	}
	size_t nonzeroOffsets() const { return nonzTot_; }
	size_t numOffs() const { return numOffs_; }
	size_t ranked() const { return rankOffs_.size(); }
	// hitsByRank(r, offidx, off, fw, seedlen) minus the offset arithmetic
	const Hit& hitsByRank(size_t r, uint32_t& offidx, bool& fw) const {
		offidx = rankOffs_[r]; fw = rankFws_[r];
		return hits_[fw ? 0 : 1][offidx];
	}
	const Hit& hit(bool fw, uint32_t i) const { return hits_[fw ? 0 : 1][i]; }
	size_t nonzFw() const { return nonzFw_; }
	size_t nonzRc() const { return nonzRc_; }
	uint64_t numElts() const { return numElts_; }
	uint64_t numEltsFw() const { return numEltsFw_; }
	uint64_t numEltsRc() const { return numEltsRc_; }
	size_t uniTot() const { return uniTot_; }
	size_t repTot() const { return repTot_; }
private:
	void push(uint32_t i, bool fw) { rankOffs_.push_back(i); rankFws_.push_back(fw); }
	uint32_t numOffs_ = 0;
	std::vector<Hit> hits_[2];
	std::vector<bool> sorted_[2];
	std::vector<uint32_t> rankOffs_;
	std::vector<bool> rankFws_;
	size_t nonzTot_ = 0, nonzFw_ = 0, nonzRc_ = 0, uniTot_ = 0, repTot_ = 0;
	uint64_t numElts_ = 0, numEltsFw_ = 0, numEltsRc_ = 0;
};

// ------------------------------------------------------------------------ DP

// One alignment out of nextAlignment(): the AlnRes fields the caller copies
// (AlnScore score/ns/gaps/basesAligned, refcoord off, refns, ned() edits).
struct AlnView {
	int score = 0, ns = 0, gaps = 0, bases_aligned = 0, refns = 0;
	int64_t refoff = 0;
	bool fw = true;
	std::vector<uint32_t> edits;   // packed, BT2X_EDIT_* accessors, final ned() order
	// The call's writes to the read's edit buffer (bt2x.h "edit-buffer image"),
	// set by every nextAlignment() call, also one that returns false.  A caller that needs
	// the reference's printed CIGAR/MD copies it into its SwResult's ned() storage.
	std::vector<uint32_t> image;
};

class SwBatch {
public:
	explicit SwBatch(Device& dev) : dev_(dev) {}

	// Drop everything (SwAligner::reset + a new read batch).
	void reset() {
		rslots_.clear(); reads_.clear(); quals_.clear();
		clear_problems();
	}
	// Drop the queued problems and results, keep the bound reads.
	void clear_problems() {
		refs_.clear(); in_.clear(); out_.clear(); recs_.clear(); edits_.clear(); cursor_.clear();
		ran_ = false;
	}

	// SwAligner::initRead (aligner_sw.cpp:35): false if rdlen > BT2X_MAX_ROWS.
	// Returns the read slot through `slot`.
	template<class S, class Q, class Sc>
	bool initRead(const S& rdfw, const S& rdrc, const Q& qufw, const Q& qurc, size_t rdlen,
	              const Sc& sc, int& slot) {
		if(rdlen > BT2X_MAX_ROWS || rdlen == 0) return false;
		ReadSlot r;
		r.len = rdlen;
		r.nceil = sc.nCeil.template f<int>((double)rdfw.length());
		r.fw_off = append_codes(rdfw, rdlen);
		r.rc_off = append_codes(rdrc, rdlen);
		r.qfw_off = append_quals(qufw, rdlen);
		r.qrc_off = append_quals(qurc, rdlen);
		rslots_.push_back(r);
		slot = (int)rslots_.size() - 1;
		return true;
	}

	// SwAligner::initRef (aligner_sw.cpp:117-229): fetch rect.refl .. rect.refr + 1 (one
	// extra column), Ns outside [0, reflen); false if that is more than BT2X_MAX_COLS
	// characters.  nsUpto counts Ns among the first `upto` window characters.
	template<class Rect, class Refs>
	bool initRef(int slot, bool fw, size_t refidx, const Rect& rect, const Refs& refs,
	             int64_t reflen, int64_t minsc, size_t upto, size_t& nsUpto, int& prob,
	             bool enable8 = true) {
		const int64_t rfi = rect.refl, rff = rect.refr + 2;
		const size_t rflen = (size_t)(rff - rfi);
		if(rflen > BT2X_MAX_COLS) return false;
		const ReadSlot& r = rslots_.at((size_t)slot);
		const bool i16 = dp_uses_i16(kI16Build, enable8, minsc);
		if(!i16 && minsc < -254) minsc = -254;       // aligner_sw.cpp:77-83
		if(minsc < -32767) throw Error(BT2X_E_ARG, "SwBatch::initRef: minsc below the int16 range");
		bt2x_dp_in p;
		std::memset(&p, 0, sizeof(p));
		p.read_off = fw ? r.fw_off : r.rc_off;
		p.qual_off = fw ? r.qfw_off : r.qrc_off;
		p.ref_off = refs_.size();
		p.refl = rect.refl;
		p.rdlen = (uint16_t)r.len;
		p.ncol = (uint16_t)(rflen - 1);
		p.minsc = (int16_t)minsc;
		p.nceil = (int16_t)r.nceil;
		p.triml = (uint16_t)rect.triml; p.corel = (uint16_t)rect.corel; p.corer = (uint16_t)rect.corer;
		p.fw = fw ? 1 : 0;
		p.flags = i16 ? BT2X_DP_I16 : 0;
		nsUpto = 0;
		for(size_t i = 0; i < rflen; i++) {
			const int64_t off = rfi + (int64_t)i;
			const int c = (off < 0 || off >= reflen) ? 4 : refs.getBase(refidx, (size_t)off);
			if(i < upto && c > 3) nsUpto++;
			if(i + 1 < rflen) refs_.push_back((uint8_t)c);
		}
		in_.push_back(p);
		prob = (int)in_.size() - 1;
		return true;
	}

	// One launch for every queued problem: align() + every nextAlignment() call.
	void run() {
		const uint32_t n = (uint32_t)in_.size();
		out_.resize(n);
		cursor_.assign(n, 0);
		ran_ = true;
		if(n == 0) return;
		uint32_t rec_cap = 4 * n + 64, edit_cap = 48 * n + 256;
		for(int attempt = 0; attempt < 2; attempt++) {
			recs_.resize(rec_cap);
			edits_.resize(edit_cap);
			uint32_t nrec = 0, ned = 0;
			const int rc = bt2x_dp_align(dev_.ctx(), reads_.data(), reads_.size(), quals_.data(), quals_.size(),
			                             refs_.data(), refs_.size(), in_.data(), n, out_.data(),
			                             recs_.data(), rec_cap, &nrec, edits_.data(), edit_cap, &ned, nullptr);
			if(rc == BT2X_E_OVERFLOW && attempt == 0) { rec_cap = nrec; edit_cap = ned; continue; }
			check(rc, "bt2x_dp_align");
			return;
		}
	}

	// SwAligner::align (aligner_sw.cpp:235): the fill's verdict and best score.
	bool align(int prob, int64_t& best) const {
		need_ran();
		const bt2x_dp_out& o = out_.at((size_t)prob);
		best = o.best;
		return o.status != 0;
	}

	// SwAligner::done (aligner_sw.h:322): no more nextAlignment() results.
	bool done(int prob) const {
		need_ran();
		const bt2x_dp_out& o = out_.at((size_t)prob);
		return o.status == 0 || cursor_[(size_t)prob] >= o.nrec;
	}

	// SwAligner::nextAlignment (aligner_sw.cpp:252-375): the next result of this
	// problem's call sequence; the RNG advances exactly as the reference's does.
	template<class Rnd>
	bool nextAlignment(int prob, AlnView& res, Rnd& rnd) {
		need_ran();
		const bt2x_dp_out& o = out_.at((size_t)prob);
		uint32_t& k = cursor_[(size_t)prob];
		if(o.status == 0 || k >= o.nrec) return false;
		const bt2x_aln_rec& r = recs_[o.rec_off + k++];
		replay_backtrace_draws(rnd, r.ntries, (in_[(size_t)prob].flags & BT2X_DP_I16) != 0);
		res.image.assign(edits_.begin() + r.edit_off, edits_.begin() + r.edit_off + r.nbuf);
		if(!r.ok) { cursor_[(size_t)prob] = o.nrec; return false; }
		res.score = r.score; res.ns = r.ns; res.gaps = r.gaps; res.bases_aligned = r.bases_aligned;
		res.refns = r.refns; res.refoff = r.refoff; res.fw = in_[(size_t)prob].fw != 0;
		res.edits.assign(edits_.begin() + r.edit_off, edits_.begin() + r.edit_off + r.nedit);
		return true;
	}

	size_t size() const { return in_.size(); }
	const bt2x_dp_out& out(int prob) const { return out_.at((size_t)prob); }

private:
	struct ReadSlot { size_t len; int nceil; uint64_t fw_off, rc_off, qfw_off, qrc_off; };
	void need_ran() const { if(!ran_) throw Error(BT2X_E_ARG, "SwBatch: run() not called"); }
	template<class S> uint64_t append_codes(const S& s, size_t n) {
		const uint64_t o = reads_.size();
		for(size_t i = 0; i < n; i++) reads_.push_back((uint8_t)s[i]);
		return o;
	}
	template<class Q> uint64_t append_quals(const Q& q, size_t n) {
		const uint64_t o = quals_.size();
		for(size_t i = 0; i < n; i++) quals_.push_back((uint8_t)q[i]);
		return o;
	}

	Device& dev_;
	std::vector<ReadSlot> rslots_;
	std::vector<uint8_t> reads_, quals_, refs_;
	std::vector<bt2x_dp_in> in_;
	std::vector<bt2x_dp_out> out_;
	std::vector<bt2x_aln_rec> recs_;
	std::vector<uint32_t> edits_;
	std::vector<uint32_t> cursor_;
	bool ran_ = false;
};

// The SwAligner call surface one problem at a time (a SwBatch of one): a literal
// drop-in for code that has not been restructured to batch.  Correct, not fast.
class SwAlignerHip {
public:
	explicit SwAlignerHip(Device& dev) : b_(dev) {}
	template<class S, class Q, class Sc>
	bool initRead(const S& rdfw, const S& rdrc, const Q& qufw, const Q& qurc, size_t rdlen, const Sc& sc) {
		b_.reset();
		prob_ = slot_ = -1;
		return b_.initRead(rdfw, rdrc, qufw, qurc, rdlen, sc, slot_);
	}
	template<class Rect, class Refs>
	bool initRef(bool fw, size_t refidx, const Rect& rect, const Refs& refs, int64_t reflen,
	             int64_t minsc, bool enable8, bool /*extend*/, size_t upto, size_t& nsUpto) {
		prob_ = -1;
		if(slot_ < 0) return false;
		b_.clear_problems();
		return b_.initRef(slot_, fw, refidx, rect, refs, reflen, minsc, upto, nsUpto, prob_, enable8);
	}
	bool align(int64_t& best) {
		if(prob_ < 0) return false;
		b_.run();
		return b_.align(prob_, best);
	}
	template<class Rnd>
	bool nextAlignment(AlnView& res, int64_t /*minsc*/, Rnd& rnd) { return b_.nextAlignment(prob_, res, rnd); }
	bool done() const { return prob_ < 0 || b_.done(prob_); }
	void reset() { prob_ = -1; }
private:
	SwBatch b_;
	int slot_ = -1, prob_ = -1;
};

} // namespace bt2x
