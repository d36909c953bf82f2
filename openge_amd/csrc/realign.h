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
#include <string>
#include <vector>

namespace oge {

struct CigOp {
    char t;      // 'M','I','D','N','S','H','P','=','X'
    uint32_t n;
    bool operator==(const CigOp &o) const { return t == o.t && n == o.n; }
};
typedef std::vector<CigOp> Cigar;

// One BAM record, decoded into mutable fields (the OGERead/BamAlignment state the reference edits).
struct RRead {
    int32_t ref = -1, pos = -1, mref = -1, mpos = -1, tlen = 0;
    uint16_t mapq = 0, flag = 0;
    std::string name;          // without the NUL
    Cigar cigar;
    uint32_t l_seq = 0;
    std::string seq4;          // packed 4-bit bases (BAM layout)
    std::string qual;          // raw phred bytes (BAM layout)
    std::string tags;          // raw tag bytes
    uint32_t idx = 0;          // input order (stands in for the reference's heap-address tie-break)

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

// ---- tags (BamAlignment::AddTag / EditTag / RemoveTag semantics) ----
bool tag_find(const std::string &tags, const char *tag, size_t *at, size_t *len);
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
    std::vector<uint8_t> cons;           // consensus bytes, back to back
    std::vector<uint64_t> cons_off;      // n_cons + 1
    std::vector<uint8_t> bases;          // altRead bases (M/I only), back to back
    std::vector<uint8_t> quals;          // raw phred bytes aligned with bases
    std::vector<uint64_t> read_off;      // n_reads + 1
    std::vector<ScanPair> pairs;
};
// Fills best_index / best_score (one per pair).  Returns 0 on success.
typedef std::function<int(const ScanBatch &, std::vector<int32_t> &best_index, std::vector<int32_t> &best_score)> ScanFn;

struct RealignParams {
    double lod_threshold = 5.0;          // LOD_THRESHOLD (local_realignment.cpp:1435)
    double mismatch_threshold = 0.15;    // MISMATCH_THRESHOLD (:1438)
    int max_records_in_memory = 150000;  // (:1439)
    int max_isize_for_movement = 3000;   // (:1440)
    int max_pos_move_allowed = 200;      // (:1441)
    int max_reads = 20000;               // (:1444)
    bool no_original_alignment_tags = false;
    int threads = 0;
};

struct RealignStats {
    uint64_t intervals = 0, intervals_cleaned = 0, reads_realigned = 0, scan_pairs = 0, scan_ops = 0;
    double t_bin = 0, t_prepare = 0, t_scan = 0, t_decide = 0, t_emit = 0;
};

// Runs LocalRealignment over coordinate-sorted records.  `ref_names` = the BAM header's @SQ names
// (sequence dictionary), `fasta` = path of the reference FASTA, `intervals` = path of the target
// interval list ("chr:start-stop", 1-based).  Output records (encoded, in emission order) are
// appended to `out`, their offsets to `out_off`.
int realign_run(const std::vector<std::string> &ref_names, const uint8_t *recs, const uint64_t *offs, uint64_t n,
                const std::string &fasta, const std::string &intervals, const RealignParams &P, const ScanFn &scan,
                std::vector<uint8_t> &out, std::vector<uint64_t> &out_off, RealignStats &st, std::string &err);

}  // namespace oge
