// modules.h -- the AlgorithmModule operator API of OpenGE (algorithms/algorithm_module.h:33-107),
// re-designed for MI355X: a chain of modules hands ONE batch of records (the whole input) from
// module to module instead of streaming OGERead* through polled per-module queues.  Records stay in
// HBM between device modules (ReadSorter -> MarkDuplicates is fused into one device pipeline), and
// only the file endpoints touch host memory.  Module names, setters and defaults follow the
// reference; each class cites the module it replaces.
//
// Built on the C ABI only (include/openge_hip.h): this layer is what an OpenGE maintainer would
// link against, and it contains no HIP code of its own.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/openge_hip.h"
#include "bamio.h"

namespace oge {

struct ChainContext;

// Start reading the chain's input file into host memory on helper threads (the CLI calls this before it
// brings up HIP); FileReader takes the bytes when it streams that file to the device.
void prefetch_input(const std::string &path);

// Records of one chain, resident in host memory, HBM, or both.
struct ReadBatch {
    BamHeaderModel header;
    std::vector<std::string> ref_names;
    uint64_t n = 0;
    // host form
    bytevec recs;                     // + 16 bytes of slack
    std::vector<uint64_t> offs;       // n + 1
    bool host_valid = false;
    // device form
    uint8_t *d_recs = nullptr;
    uint64_t *d_offs = nullptr;
    uint64_t d_bytes = 0;
    bool dev_valid = false;
    // dedup output applied by the writer (-r / -R: records carrying 0x400 are not written)
    bool drop_duplicates = false;
    // multi-GPU (--gpus G): the records as G slices in rank order, each in its rank's HBM (owned by
    // the rank's context); when set, the host and device forms above are unused
    struct Slice {
        oge_ctx *ctx;
        uint8_t *d_recs;
        uint64_t *d_offs;  // n + 1 byte offsets from d_recs
        uint64_t n;
    };
    std::vector<Slice> slices;
    // multi-GPU input (--gpus G, one BAM file): the records as G input shards in rank order (contiguous
    // ranges of the file's records, each decoded by its rank from its own byte range of the file,
    // oge_bgzf_decode_shard), owned by the ranks' contexts; run_ranks takes them as they are
    std::vector<Slice> shards;
    // inputs larger than HBM: the output is produced range by range when the writer asks for it
    // (oge_sort_markdup_chunked); each range is handed to `sink` in output order
    using RangeSink = std::function<int(const uint8_t *d_recs, const uint64_t *d_offs, uint64_t n)>;
    std::function<int(ChainContext &, const RangeSink &)> produce;

    uint64_t bytes() const { return host_valid ? offs[n] : d_bytes; }
};

struct ChainContext {
    oge_ctx *ctx = nullptr;
    int device = 0;
    int threads = 0;
    bool verbose = false;
    // --gpus G: rank contexts (rank 0 = ctx, rank g on device (device + g) % devices; ranks share a
    // device when there are fewer devices than ranks) and their communicators
    int gpus = 1;
    std::vector<oge_ctx *> rank_ctx;
    std::vector<oge_comm *> comms;
    int init_ranks();
    void close_ranks();
    int fail(const std::string &where);  // prints oge_last_error, returns -1
    int to_device(ReadBatch &b);
    int to_host(ReadBatch &b);
    void free_device(ReadBatch &b);
};

class AlgorithmModule {
public:
    virtual ~AlgorithmModule() {}
    void addSink(AlgorithmModule *sink) { sink_ = sink; sink->source_ = this; }
    // AlgorithmModule::runChain (algorithm_module.cpp:92-116): run every module of the chain that
    // ends at this one, from its first source.  Returns 0 or the first failing module's status
    // (the reference always returns 0).
    int runChain(ChainContext &cc);
    static void setVerbose(bool v) { verbose_ = v; }
    static bool isVerbose() { return verbose_; }
    const char *name() const { return name_; }
    AlgorithmModule *sink() const { return sink_; }

protected:
    explicit AlgorithmModule(const char *name) : name_(name) {}
    // consume `b` (the previous module's output) in place; sources ignore it and fill it
    virtual int runInternal(ChainContext &cc, ReadBatch &b) = 0;
    AlgorithmModule *source_ = nullptr, *sink_ = nullptr;
    static bool verbose_;
    const char *name_;
    friend class ReadSorter;
};

// FileReader (algorithms/file_reader.cpp:29-63): BAM input(s).  Several inputs are interleaved as
// the reference's MultiReader does (a ByPosition merge of the file heads,
// util/read_stream_reader.h:132-153) unless a ReadSorter follows, which makes the interleaving
// irrelevant; the header is the first file's (a differing dictionary only warns, :116-124).
class FileReader : public AlgorithmModule {
public:
    FileReader() : AlgorithmModule("FileReader") {}
    void addFile(const std::string &f) { files_.push_back(f); }
    void addFiles(const std::vector<std::string> &f) { files_.insert(files_.end(), f.begin(), f.end()); }
    void setLoadStringData(bool) {}  // the record arena always keeps the full record bytes
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    // One BGZF file straight into HBM: inflate + record walk on the GPU (returns 1 when the host
    // reader should take over, e.g. to report a format error with the reference's message).
    int read_device(ChainContext &cc, ReadBatch &b, const std::string &path);
    // --gpus G: every rank reads and decodes its own byte range of the one input file (b.shards)
    int read_sharded(ChainContext &cc, ReadBatch &b, const std::string &path);
    bool sink_takes_shards() const;
    bool sink_sorts() const;
    static int merge_inputs(ReadBatch &b, const std::vector<uint64_t> &file_end, int threads);
    std::vector<std::string> files_;
};

// Filter (algorithms/filter.h:30-70, filter.cpp:185-249): mergesort's -r region / -q mapq, as a
// device compaction (oge_filter_records_dev).  Trimming (setTrimBeginLength/EndLength) edits
// records and is only reachable from the bpipe `filter` command, which is out of scope; its
// length condition (len > trim total) is kept.
class Filter : public AlgorithmModule {
public:
    Filter() : AlgorithmModule("Filter") { oge_filter_opts_init(&opts_); }
    void setRegion(const std::string &region) { region_ = region; has_region_ = true; }
    std::string getRegion() const { return region_; }
    void setCountLimit(int ct) { opts_.count_limit = ct < 0 ? 0 : (uint64_t)ct; }
    size_t getCountLimit() const { return opts_.count_limit; }
    void setQualityLimit(int mapq) { opts_.mapq_min = mapq; }
    int getQualityLimit() const { return opts_.mapq_min; }
    void setMinimumReadLength(int l) { opts_.min_len = l; }
    void setMaximumReadLength(int l) { opts_.max_len = l; }
    bool setReadLengths(const std::string &s);  // "64", "64-72", "-64", "+64" (filter.cpp:150-183)
    uint64_t kept = 0;
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    std::string region_;
    bool has_region_ = false;
    oge_filter_opts opts_;
};

// ReadSorter (algorithms/read_sorter.h:32-105): coordinate sort (oge_sort_coord_dev) or, with
// setSortBy(QUERYNAME), name sort (oge_sort_name_dev) on the GPU, then the permutation gather.  The temp-file knobs are accepted for interface parity; one device sort
// replaces the reference's spilled runs and k-way merge.
class ReadSorter : public AlgorithmModule {
public:
    explicit ReadSorter(const std::string &tmpdir = "/tmp/") : AlgorithmModule("ReadSorter") { (void)tmpdir; }
    void setSortBy(BamHeaderModel::SortOrder o) { order_ = o; }
    void setCompressTempFiles(bool) {}
    void setAlignmentsPerTempfile(int) {}
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    BamHeaderModel::SortOrder order_ = BamHeaderModel::COORDINATE;
public:
    BamHeaderModel::SortOrder sortBy() const { return order_; }
};

// MarkDuplicates (algorithms/mark_duplicates.h:27-68): -v --nosplit semantics on the GPU.
class MarkDuplicates : public AlgorithmModule {
public:
    explicit MarkDuplicates(const std::string &tmpdir = "/tmp/") : AlgorithmModule("MarkDuplicates") { (void)tmpdir; }
    bool removeDuplicates = false;
    bool compatNonverbose = false;  // reproduce the index bug of runs without -v
    int splitChains = 0;            // > 1 = the result of the split-by-chromosome chains
    uint64_t duplicates = 0;
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    friend class ReadSorter;
};

// LocalRealignment (algorithms/local_realignment.h:67-527): oge_localrealign (host phases + the
// GPU offset scan).
class LocalRealignment : public AlgorithmModule {
public:
    LocalRealignment() : AlgorithmModule("LocalRealignment") {}
    bool verbose = false;
    void setReferenceFilename(const std::string &f) { reference_ = f; }
    void setIntervalsFilename(const std::string &f) { intervals_ = f; }
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    std::string reference_, intervals_;
};

// The multi-GPU form of ReadSorter (+ MarkDuplicates) and of a standalone MarkDuplicates: the batch
// is cut into G contiguous input ranges, one per rank, and oge_sort_markdup_dist leaves b.slices.
int run_ranks(ChainContext &cc, ReadBatch &b, bool sort, const oge_markdup_opts *opts, uint64_t *n_dup);

// FileWriter (algorithms/file_writer.cpp:69-196): BAM output, @PG record unless --nopg, BGZF at the
// given level, bin recomputed on every record.
class FileWriter : public AlgorithmModule {
public:
    FileWriter() : AlgorithmModule("FileWriter") {}
    void setFilename(const std::string &f) { filename_ = f; }
    void setCompressionLevel(int l) { level_ = l; }
    int write_device(ChainContext &cc, ReadBatch &b, BgzfWriter &w, double *t_dev, double *t_d2h, double *t_wait);
    int write_slices(ChainContext &cc, ReadBatch &b, BgzfWriter &w);
    int write_ranges(ChainContext &cc, ReadBatch &b, BgzfWriter &w);
    void addProgramLine(const std::string &cl) { program_line_ = cl; }
    int setFormat(const std::string &f);  // only "bam" is supported (SAM/FASTQ out of scope)
protected:
    int runInternal(ChainContext &cc, ReadBatch &b) override;
    std::string filename_ = "stdout", program_line_;
    int level_ = 6;
};

}  // namespace oge
