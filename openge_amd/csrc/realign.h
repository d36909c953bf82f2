// realign.h -- host side of local realignment (LocalRealignment, algorithms/local_realignment.cpp;
// ConstrainedMateFixingManager, util/gatk/ConstrainedMateFixingManager.cpp).
//
// The reference streams reads through map_func one at a time, cleans each interval's read bin on a
// thread pool and funnels everything through the mate-fixing writer.  Here the same semantics run as
// phases over the whole coordinate-sorted input:
//   A  binning      (map_func :455-553)            sequential, builds the event list
//   B  prepare      (clean :681-700, determineReadsThatNeedCleaning :918-999)  parallel per interval
//   C  offset scan  (findBestOffset :1126-1164 x every (consensus, altRead) pair) -> ScanFn (GPU)
//   D  decide       (clean :713-892: sums, LOD, updateRead, entropy, constize, NM/UQ/MD) parallel
//   E  emit         (emitReadLists :370-376 + ConstrainedMateFixingManager) sequential
// C is the only data-parallel hot loop and is delegated to a ScanFn: the product library binds the
// HIP kernel (realign.hip); nothing here computes offsets itself.
#pragma once
#include <cstdint>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

#include "uvector.h"

namespace oge {

struct CigOp {
    char t;      // 'M','I','D','N','S','H','P','=','X'
    uint32_t n;
    bool operator==(const CigOp &o) const { return t == o.t && n == o.n; }
};

// CIGAR with inline room for 4 operations (nearly every short-read alignment), so decoding millions
// of records does not allocate.
class Cigar {
public:
    Cigar() = default;
    Cigar(const Cigar &o) { assign(o.begin(), o.end()); }
    Cigar(Cigar &&o) noexcept { take(o); }
    ~Cigar() { delete[] heap_; }
    Cigar &operator=(const Cigar &o) {
        if (this != &o) assign(o.begin(), o.end());
        return *this;
    }
    Cigar &operator=(Cigar &&o) noexcept {
        if (this != &o) {
            delete[] heap_;
            heap_ = nullptr;
            take(o);
        }
        return *this;
    }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    CigOp *begin() { return data(); }
    CigOp *end() { return data() + n_; }
    const CigOp *begin() const { return data(); }
    const CigOp *end() const { return data() + n_; }
    CigOp &operator[](size_t i) { return data()[i]; }
    const CigOp &operator[](size_t i) const { return data()[i]; }
    CigOp &back() { return data()[n_ - 1]; }
    void clear() { n_ = 0; }
    void reserve(size_t c) {
        if (c <= cap_) return;
        CigOp *h = new CigOp[c];
        std::memcpy((void *)h, (const void *)data(), n_ * sizeof(CigOp));
        delete[] heap_;
        heap_ = h;
        cap_ = (uint32_t)c;
    }
    void resize(size_t c) {
        reserve(c);
        n_ = (uint32_t)c;
    }
    void push_back(const CigOp &x) {
        if (n_ == cap_) reserve(2 * cap_);
        data()[n_++] = x;
    }
    void insert(CigOp *at, const CigOp *first, const CigOp *last) {  // append form only
        (void)at;
        for (; first != last; ++first) push_back(*first);
    }
    bool operator==(const Cigar &o) const {
        if (n_ != o.n_) return false;
        for (uint32_t i = 0; i < n_; ++i)
            if (!(data()[i] == o.data()[i])) return false;
        return true;
    }
    bool operator!=(const Cigar &o) const { return !(*this == o); }

private:
    CigOp *data() { return heap_ ? heap_ : inl_; }
    const CigOp *data() const { return heap_ ? heap_ : inl_; }
    void assign(const CigOp *f, const CigOp *l) {
        n_ = 0;
        reserve((size_t)(l - f));
        for (; f != l; ++f) data()[n_++] = *f;
    }
    void take(Cigar &o) {
        n_ = o.n_;
        cap_ = o.cap_;
        if (o.heap_) {
            heap_ = o.heap_;
            o.heap_ = nullptr;
        } else {
            std::memcpy((void *)inl_, (const void *)o.inl_, n_ * sizeof(CigOp));
        }
        o.n_ = 0;
        o.cap_ = kInline;
    }
    static constexpr uint32_t kInline = 4;
    CigOp inl_[kInline];
    CigOp *heap_ = nullptr;
    uint32_t n_ = 0, cap_ = kInline;
};

// One BAM record, decoded into mutable fields (the OGERead/BamAlignment state the reference edits).
// Fields the realigner never changes (name, bases, qualities) are views into the input record, which
// outlives the run; tags are viewed until the first edit copies them.
struct RRead {
    int32_t ref = -1, pos = -1, mref = -1, mpos = -1, tlen = 0;
    uint16_t mapq = 0, flag = 0;
    std::string_view name;     // without the NUL
    Cigar cigar;
    uint32_t l_seq = 0;
    std::string_view seq4;     // packed 4-bit bases (BAM layout)
    std::string_view qual;     // raw phred bytes (BAM layout)
    std::string_view tags_in;  // raw tag bytes of the input record
    std::string tags_own;      // edited tag bytes (valid when tags_owned)
    bool tags_owned = false;
    int32_t mq_add = -1;       // MQ:S value appended at encode (the mate fixer's AddTag("MQ")), -1 = none
    uint32_t name_hash = 0;    // FNV-1a of name (mate-table probe)
    bool cleaned = false;      // realigned in the interval being emitted
    uint32_t idx = 0;          // input order (stands in for the reference's heap-address tie-break)

    std::string_view tags() const { return tags_owned ? std::string_view(tags_own) : tags_in; }
    std::string &tags_mut() {
        if (!tags_owned) {
            tags_own.assign(tags_in.data(), tags_in.size());
            tags_owned = true;
        }
        return tags_own;
    }

    bool mapped() const { return !(flag & 0x4); }
    bool paired() const { return flag & 0x1; }
    bool mate_mapped() const { return !(flag & 0x8); }
    bool rev() const { return flag & 0x10; }
    bool dup() const { return flag & 0x400; }
    std::string bases() const;        // BamAlignment::getQueryBases ("=ACMGRSVTWYHKDBN")
    std::string quals_ascii() const;  // getQualities: byte + 33 (char arithmetic)
};

bool rread_decode(const uint8_t *rec, RRead &r, std::string &err);
void rread_encode(const RRead &r, std::vector<uint8_t> &out);  // appends; bin recomputed (W1)
size_t rread_encoded_size(const RRead &r);
void rread_encode_to(const RRead &r, uint8_t *p);  // writes rread_encoded_size(r) bytes

// ---- tags (BamAlignment::AddTag / EditTag / RemoveTag semantics) ----
bool tag_find(std::string_view tags, const char *tag, size_t *at, size_t *len);
bool tag_add_int(std::string &tags, const char *tag, char type, int64_t v, int bytes);  // no-op if present
bool tag_add_string(std::string &tags, const char *tag, const std::string &v);
void tag_remove(std::string &tags, const char *tag);
std::string cigar_to_string(const Cigar &c);

// ---- offset scan batch (phase C) ----
struct ScanPair {
    uint32_t cons;      // consensus index in the batch
    uint32_t read;      // altRead index in the batch
    int32_t orig;       // original alignment start - leftmostIndex
    int32_t max_start;  // consensus length - read cigar length (findBestOffset :1149-1150)
};
struct ScanBatch {
    uvector<uint8_t> cons;           // consensus bytes, back to back
    uvector<uint64_t> cons_off;      // n_cons + 1
    uvector<uint8_t> bases;          // altRead bases (M/I only), back to back
    uvector<uint8_t> quals;          // raw phred bytes aligned with bases
    uvector<uint64_t> read_off;      // n_reads + 1
    uvector<ScanPair> pairs;
};
// Fills best_index / best_score (one per pair).  Returns 0 on success.
typedef std::function<int(const ScanBatch &, std::vector<int32_t> &best_index, std::vector<int32_t> &best_score)> ScanFn;

// ---- consensus generation (phase B) + offset scan (phase C) on the device (r06) ----
// determineReadsThatNeedCleaning (:918-999) per toClean read -- unclipped bases, leftAlignIndel of the
// two-block reads (util/gatk/AlignmentUtils.cpp:632-677), mismatchQualitySumIgnoreCigar, getMismatchCount,
// createAlternateConsensus (:1022-1088) -- and the per-interval consensus set (distinct strings in
// creation order), then the findBestOffset batch, all on the GPU (realign_prep.hip).  The host hands over
// each interval's reference window and its toClean reads (record offsets into the arena it staged) and
// gets back what phase D needs.
struct DevPrepBatch {
    hvector<uint8_t> ref;       // reference windows back to back (ReadBin::getReference: padded, upper-cased)
    hvector<uint64_t> ref_off;  // n_iv + 1
    hvector<uint64_t> rd_off;   // n_iv + 1: interval w's reads are rec[rd_off[w] .. rd_off[w + 1])
    hvector<uint64_t> rec;      // toClean reads in interval order: byte offset of the record in the staged arena
    hvector<int32_t> start;     // read pos - the interval's leftmost (startOnRef)
};
// per toClean read (32 bytes): flags, the left-aligned cigar when the read has one, the sums
enum : uint8_t { DP_SKIP = 1, DP_ALT = 2, DP_CAND = 4, DP_NEWCIG = 8, DP_KEPT = 16, DP_HOST = 32, DP_DUP = 64 };
struct DevPrepRead {
    uint8_t flags;     // DP_*: SKIP = empty cigar (refRead), ALT = mismatch sum > 0 (an altRead), CAND = its
                       // consensus is valid, NEWCIG = newCigar set (ops below), KEPT = its consensus is the first
                       // of its string in the interval, HOST = the device could not handle it (its interval runs
                       // on the host), DUP = FLAG 0x400
    uint8_t n_ops;
    uint16_t ul;       // unclipped length (bases of the M / I operations)
    int32_t raw;       // mismatchQualitySumIgnoreCigar at the original start
    int32_t aligner;   // getMismatchCount's mismatch-quality sum (AlignmentUtils.cpp:58-108)
    uint32_t cig_len;  // getCigarLength of its current cigar (findBestOffset's maxStart)
    uint32_t ops[4];   // newCigar: length << 4 | BAM op code
};
static_assert(sizeof(DevPrepRead) == 32, "DevPrepRead layout");
struct DevPrepOut {
    hvector<DevPrepRead> reads;           // one per DevPrepBatch read
    std::vector<uint8_t> iv_host;         // per interval: 1 = run phase B / C of this interval on the host
    std::vector<int64_t> iv_total_raw;    // per interval: sum of raw over non-duplicate altReads
    std::vector<uint64_t> iv_pair_base;   // per interval: its first pair in best_index / best_score
    hvector<int32_t> best_index, best_score;
    uint64_t pairs = 0, ops = 0;          // scan pairs, algorithmic compare-accumulates
    bool generic = false;                 // the byte-wise scan kernel ran
    double t_upload = 0, t_device = 0, t_download = 0;
};
struct DevPrep {
    // ndev devices (realign sharded by interval ranges): the work intervals are cut into ndev
    // contiguous ranges balanced by toClean reads, and device g runs phase B + C of range g; the host phases
    // (binning, decisions, the mate-fixing writer) run once over the whole input, so the result is the
    // one-device result for any input -- a single contig included -- with no writer state to hand across a cut.
    int ndev = 1;
    // Start copying the record arena [lo, hi) of `recs` to device g (may return before it is done; run
    // waits for it).  Offsets in DevPrepBatch::rec are relative to lo.
    std::function<int(int g, const uint8_t *recs, uint64_t lo, uint64_t hi)> stage;
    std::function<int(int g, const DevPrepBatch &, DevPrepOut &)> run;  // called concurrently for the devices
};

struct RealignParams {
    double lod_threshold = 5.0;          // LOD_THRESHOLD (local_realignment.cpp:1435)
    double mismatch_threshold = 0.15;    // MISMATCH_THRESHOLD (:1438)
    int max_records_in_memory = 150000;  // (:1439)
    int max_isize_for_movement = 3000;   // (:1440)
    int max_pos_move_allowed = 200;      // (:1441)
    int max_reads = 20000;               // (:1444)
    bool no_original_alignment_tags = false;
    int threads = 0;
    bool mate_sequential = false;        // one writer over the whole stream (tests compare the two)
};

struct RealignStats {
    uint64_t intervals = 0, intervals_cleaned = 0, reads_realigned = 0, scan_pairs = 0, scan_ops = 0;
    uint64_t mate_segments = 0;  // writer segments run in parallel (1 = sequential)
    uint64_t tail_waiting = 0;   // reads the writer still held when the stream ended (a run cut at a
                                 // contig boundary is exact unless this reaches maxRecordsInMemory)
    double t_bin = 0, t_prepare = 0, t_scan = 0, t_decide = 0, t_emit = 0, t_run = 0;
    double t_fasta = 0, t_decode = 0, t_mate = 0, t_release = 0;  // parts of t_bin / t_emit; teardown
    double t_scan_build = 0;                                       // part of t_scan: batch assembly
    std::vector<std::pair<std::string, double>> more;              // finer timers (name, seconds), in the stats JSON
};

// Output record bytes: malloc'ed without zero-fill so the parallel encoder's first touch is the only
// pass over fresh pages.
struct ByteBuf {
    ByteBuf() = default;
    ByteBuf(const ByteBuf &) = delete;
    ByteBuf &operator=(const ByteBuf &) = delete;
    // n bytes (uninitialised) + 16 zeroed bytes of slack past them
    bool alloc(size_t n) {
        v_ = bytevec();
        n_ = 0;
        try {
            v_.reserve(n + 16);
            v_.resize(n + 16);
        } catch (const std::bad_alloc &) {
            v_ = bytevec();
            return false;
        }
        memset(v_.data() + n, 0, 16);
        n_ = n;
        return true;
    }
    uint8_t *data() { return v_.data(); }
    const uint8_t *data() const { return v_.data(); }
    size_t size() const { return n_; }
    // hands the storage over (size() + 16 bytes: the slack included, what a ReadBatch holds), no copy
    void take(bytevec &dst) {
        dst = std::move(v_);
        v_ = bytevec();
        n_ = 0;
    }

private:
    bytevec v_;
    size_t n_ = 0;
};

// Runs LocalRealignment over coordinate-sorted records.  `ref_names` = the BAM header's @SQ names
// (sequence dictionary), `fasta` = path of the reference FASTA, `intervals` = path of the target
// interval list ("chr:start-stop", 1-based).  Output records (encoded, in emission order) are
// written to `out`, their offsets (n + 1) to `out_off`.
// dev (optional): phases B and C on the device for every interval it can handle (the others, and all of
// them without dev, on host threads with `scan`) -- the same results either way.
int realign_run(const std::vector<std::string> &ref_names, const uint8_t *recs, const uint64_t *offs, uint64_t n,
                const std::string &fasta, const std::string &intervals, const RealignParams &P, const ScanFn &scan,
                ByteBuf &out, std::vector<uint64_t> &out_off, RealignStats &st, std::string &err, const DevPrep *dev = nullptr);

}  // namespace oge
