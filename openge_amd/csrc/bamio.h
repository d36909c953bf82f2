// bamio.h -- host-side BAM/BGZF codec and header model for the openge_amd drop-in.
//
// Replaces the reference's L2 codec layer for the hot path:
//   BgzfInputStream  (util/bgzf_input_stream.cpp:65-142,208-240)  -> bgzf_inflate_all()
//   BgzfOutputStream (util/bgzf_output_stream.cpp:59-250)         -> BgzfWriter
//   BamDeserializer::open/read (util/bam_deserializer.h:38-193)   -> bam_parse()
//   BamSerializer::open/write  (util/bam_serializer.h:46-147)     -> bam_write_header()/records
//   BamHeader parse/toString   (util/bam_header.cpp:108-278)      -> BamHeaderModel
// Records stay in their BAM byte layout inside one contiguous arena with a u64 offset per
// record, which is exactly what the device kernels consume.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "uvector.h"

namespace oge {

// ---------------- BGZF ----------------
// Inflate an entire BGZF byte string (any number of blocks) into `out`, in parallel.
// Returns false and fills `err` on a malformed or truncated stream.
// out is sized to the stream (plus `slack` zeroed bytes past it) without a serial zero-fill first
bool bgzf_inflate_all(const uint8_t *src, size_t n, bytevec &out, int threads, std::string &err, size_t slack = 64);
const char *bgzf_codec_name();  // "libdeflate" or "zlib"
// OGE_BGZF_CODEC=zlib|libdeflate: compress on the host even when the records sit on the device.
bool bgzf_host_codec_forced();

// Compress n bytes into BGZF blocks (65280-byte payloads) in memory, no EOF marker.
std::vector<uint8_t> bgzf_compress_host(const uint8_t *src, size_t n, int level);
// The 28-byte empty BGZF block that ends every BAM file.
extern const uint8_t kBgzfEof[28];

class BgzfWriter {
public:
    // level: zlib level 0..9; block payload is 65280 bytes (htslib framing; the reference uses
    // 65536/65472, SURVEY Q17 -- compressed bytes are not part of parity).
    BgzfWriter(FILE *f, int level, int threads);
    ~BgzfWriter();
    void write(const void *data, size_t n);
    // Append n bytes: whole blocks are compressed straight from the caller's bytes, all in parallel,
    // with no staging copy (only a partial tail block is copied).
    void write_span(const uint8_t *data, size_t n);
    // Append already-compressed BGZF blocks (e.g. from oge_bgzf_deflate_dev): the pending partial
    // block is flushed as a block of its own first, so block boundaries stay intact.
    void write_compressed(const uint8_t *z, size_t n);
    void close();  // flush + EOF marker
    // Make the writer inert without touching the FILE (the caller is about to fclose it after a
    // failure): a background write in flight is joined, pending bytes are dropped, no EOF block.
    void abandon();
    // false once any fwrite / pwrite / fflush failed (sticky); the caller turns it into an exit status
    bool ok() const { return !failed_; }
private:
    void put(const uint8_t *p, size_t n);  // fwrite with the sticky error flag
    void flush_blocks(bool final);
    void emit(std::vector<std::vector<uint8_t>> &&blocks);  // ordered, written by a background thread
    void drain();                                          // wait for the background write
    FILE *f_;
    std::thread writer_;
    std::vector<std::vector<uint8_t>> writing_;
    int level_, threads_;
    std::vector<uint8_t> pending_;
    bool closed_;
    std::atomic<bool> failed_{false};
};

// ---------------- header model ----------------
struct SqRecord { std::string name, as, m5, sp, ur; long long length = -1; };
struct RgRecord { std::string id, cn, ds, dt, fo, ks, lb, pg, pi, pl, pu, sm; };
struct PgRecord { std::string id, pn, cl, pp, vn; };

struct BamHeaderModel {
    std::string format_version;
    enum SortOrder { UNKNOWN = 0, UNSORTED = 1, QUERYNAME = 2, COORDINATE = 3 } sort_order = UNKNOWN;
    std::vector<SqRecord> sq;
    std::vector<RgRecord> rg;
    std::vector<PgRecord> pg;
    std::vector<std::string> co;
    bool parse(const std::string &text, std::string &err);
    std::string to_string() const;
    // Library id per read group in the order MarkDuplicates would discover them does not
    // matter; ids here: 1 + index of the distinct LB name, "Unknown Library" last.
};

// FileWriter's @PG line (algorithms/file_writer.cpp:76-89): ID openge, or openge-k when taken,
// VN 0.3-dev (OPENGE_VERSION_STRING), CL = the command line.
void add_program_record(BamHeaderModel &h, const std::string &cl);

// ---------------- BAM ----------------
struct BamFile {
    BamHeaderModel header;
    std::string header_text;              // as stored in the file
    std::vector<std::string> ref_names;   // binary reference list
    std::vector<int32_t> ref_lens;
    bytevec data;                         // decompressed stream (records start at rec_base)
    size_t rec_base = 0;
    std::vector<uint64_t> offsets;        // record offsets relative to data.data() + rec_base
    const uint8_t *recs() const { return data.data() + rec_base; }
    uint64_t rec_bytes() const { return data.size() - rec_base; }
};

bool bam_read_file(const std::string &path, BamFile &out, int threads, std::string &err);
// madvise(MADV_HUGEPAGE) over a large buffer before its first touch
void want_huge_pages(void *p, size_t n);
bool bam_parse(bytevec &&raw, BamFile &out, std::string &err, int threads = 1);
// The whole file (parallel pread for regular files).
bool read_file_bytes(const std::string &path, bytevec &comp, int threads, std::string &err);
// Header text, @SQ / binary reference list of a decompressed stream prefix d[0, n) -> *rec_base.
bool bam_parse_header(const uint8_t *d, size_t n, BamFile &out, std::string &err, size_t *rec_base);
// Serialize header block (magic, text, reference list taken from the header @SQ lines, as
// BamSerializer::open does at util/bam_serializer.h:54-76).
std::vector<uint8_t> bam_encode_header(const BamHeaderModel &h);

} // namespace oge
