// pipeline.hip -- the whole `openge mergesort [-M]` chain on a BGZF BAM resident in HBM.
//
// Replaces the module chain FileReader -> ReadSorter -> [MarkDuplicates] -> FileWriter that
// MergeSortCommand::runCommand wires (openge/src/commands/command_mergesort.cpp:68-117): the
// reader's BgzfInputStream + BamDeserializer (util/bgzf_input_stream.cpp:65-142,208-240,
// util/bam_deserializer.h:143-193), the sorter and marker (algorithms/read_sorter.cpp:48-232,
// algorithms/mark_duplicates.cpp:185-475) and the writer's BamSerializer + BgzfOutputStream
// (util/bam_serializer.h:105-147, util/bgzf_output_stream.cpp:59-250, @PG at
// algorithms/file_writer.cpp:76-89).  Every stage runs on the device; the host parses the BAM header
// (a copy of the stream's first bytes) and compresses the output header block.
//
//   index    oge_bgzf_index_ws  (device framing walk)
//   inflate  oge_bgzf_inflate_dev into X, CRC-32 checked
//   records  oge_record_walk (block_size walk; the fill expands the count walk's record slots)
//   sort     oge_sort_markdup_dev (or sort + gather without -M) X -> Y, bins recomputed
//   [-R]     oge_drop_flagged_dev Y -> X
//   write    header block (host) + oge_bgzf_deflate_dev + EOF block into the free buffer
//
// oge_mergesort_bgzf_dist runs the same chain over G ranks (one input file per rank, the sort and
// dedup through oge_sort_markdup_dist, every rank deflating its own output slice);
// oge_mergesort_bgzf_shard does it for ONE input file whose byte ranges the ranks decode (shard.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "bamio.h"
#include "bgzf_dev.h"
#include "oge_ctx.h"

using namespace oge;

namespace {

struct Hold {  // keep every sub-call's stage events for the caller
    oge_ctx *c;
    explicit Hold(oge_ctx *x) : c(x) {
        c->reset_timing();
        c->timing_hold++;
    }
    ~Hold() { c->timing_hold--; }
};

// MarkDuplicates::getLibraryName (algorithms/mark_duplicates.cpp:301-318): the LB of the record's
// @RG, "Unknown Library" when absent or empty; distinct names get distinct ids.
struct LibTable {
    std::string ids;
    std::vector<int16_t> libs;
    oge_markdup_opts o;
    LibTable(const BamHeaderModel &h, int32_t n_ref, const oge_mergesort_opts *mo) {
        std::map<std::string, int16_t> lib_ids;
        int16_t next = 1;
        for (auto &rg : h.rg) {
            const std::string lib = rg.lb.empty() ? std::string("Unknown Library") : rg.lb;
            auto it = lib_ids.find(lib);
            if (it == lib_ids.end()) it = lib_ids.emplace(lib, next++).first;
            libs.push_back(it->second);
            ids += rg.id;
            ids.push_back('\0');
        }
        auto unk = lib_ids.find("Unknown Library");
        libs.push_back(0);
        memset(&o, 0, sizeof o);
        o.n_ref = n_ref;
        o.rg_ids = ids.c_str();
        o.rg_ids_bytes = ids.size();
        o.rg_lib = libs.data();
        o.n_rg = (int32_t)h.rg.size();
        o.unknown_lib = unk != lib_ids.end() ? unk->second : next;
        o.compat_nonverbose_index = mo->compat_nonverbose_index;
        o.split_chains = mo->split_chains;
    }
};

}  // namespace

extern "C" void oge_mergesort_opts_init(oge_mergesort_opts *o) {
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->level = 6;  // FileWriter's default compression level (commands.cpp:129, -c)
}

static int decode_records(oge_ctx *ctx, uint8_t *X, uint64_t total, uint64_t **xoff_o, uint64_t *n_o, BamFile *f);

// The reader half: framing index, inflate into X (ws "pipe_x", *cap bytes), header parse, record walk.
static int decode(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint8_t **Xo, uint64_t *cap_out, uint64_t **xoff_o,
                  uint64_t *n_o, BamFile *f) {
    // ---- framing index (device; host walk of a copy when the chain is not exact)
    OgeStageTimer *tm = ctx->begin_stage("bgzf_index");
    OgeBgzfIndex ix;
    int rc = oge_bgzf_index_ws(ctx, d_z, zbytes, &ix);
    ctx->end_stage(tm);
    if (rc < 0) return rc;
    if (rc == 1) {
        uint64_t nb = 0;
        rc = oge_bgzf_index_dev(ctx, d_z, zbytes, nullptr, nullptr, nullptr, nullptr, 0, &nb);
        if (rc != OGE_OK && rc != OGE_ERR_ARG) return rc;
        uint64_t *a = (uint64_t *)ctx->ws("pipe_ix", (3 * nb + 2) * 8);
        uint32_t *c = (uint32_t *)ctx->ws("pipe_ixc", (nb + 1) * 4);
        if (!a || !c) return OGE_ERR_HIP;
        rc = oge_bgzf_index_dev(ctx, d_z, zbytes, a, a + nb, a + 2 * nb, c, nb, &nb);
        if (rc) return rc;
        ix.d0 = a, ix.d1 = a + nb, ix.uoff = a + 2 * nb, ix.crc = c, ix.nblk = nb;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&ix.total, ix.uoff + nb, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    const uint64_t total = ix.total;
    if (!total) return oge_fail(ctx, OGE_ERR_IO, "empty BAM stream (no BAM magic)");

    // ---- inflate into X (X is also the deflate target later: it must hold the bound)
    const uint64_t cap = std::max<uint64_t>(total, oge_bgzf_bound(total) + (1u << 20)) + 64;
    uint8_t *X = (uint8_t *)ctx->ws("pipe_x", cap);
    if (!X) return OGE_ERR_HIP;
    rc = oge_bgzf_inflate_dev(ctx, d_z, zbytes, ix.d0, ix.d1, ix.uoff, ix.crc, ix.nblk, X);
    if (rc) return rc;

    *Xo = X;
    *cap_out = cap;
    return decode_records(ctx, X, total, xoff_o, n_o, f);
}

// The reader's second half on the decompressed stream X[0, total): header parse (host, a copy of the
// first bytes), record walk.
static int decode_records(oge_ctx *ctx, uint8_t *X, uint64_t total, uint64_t **xoff_o, uint64_t *n_o, BamFile *f) {
    int rc = OGE_OK;
    OgeStageTimer *tm = nullptr;
    // ---- header (host parse of the stream's first bytes)
    std::string err;
    size_t rec_base = 0;
    for (uint64_t pre = std::min<uint64_t>(total, 1 << 20);; pre = std::min<uint64_t>(total, pre * 8)) {
        std::vector<uint8_t> h(pre);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h.data(), X, pre, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        *f = BamFile();
        if (bam_parse_header(h.data(), pre, *f, err, &rec_base)) break;
        if (pre == total) return oge_fail(ctx, OGE_ERR_IO, ("BAM header: " + err).c_str());
    }
    const int32_t n_ref = (int32_t)f->ref_names.size();

    // ---- record boundaries
    tm = ctx->begin_stage("rec_walk");
    // the count walk keeps each chunk's record positions for the fill (in the sorted-records arena when it
    // is already there: sort_stage writes it only later)
    uint64_t n = 0, x = 0;
    const auto y = ctx->bufs.find("pipe_y");
    void *rel = y != ctx->bufs.end() ? y->second.p : nullptr;
    const uint64_t rel_cap = rel ? y->second.cap : 0;
    rc = oge_record_walk(ctx, X, rec_base, total, total, true, n_ref, nullptr, 0, &n, &x, true, rel, rel_cap);
    if (rc) return rc;
    uint64_t *xoff = (uint64_t *)ctx->ws("pipe_xoff", (n + 1) * 8);
    if (!xoff) return OGE_ERR_HIP;
    rc = oge_record_walk(ctx, X, rec_base, total, total, true, n_ref, xoff, n + 1, &n, &x, true);
    if (rc) return rc;
    ctx->end_stage(tm);
    *xoff_o = xoff;
    *n_o = n;
    return OGE_OK;
}

// The writer half: [header block(s)] + device deflate of records [soff[0], soff[m]) of src + [EOF]
// into dst (dst_cap bytes).
static int encode(oge_ctx *ctx, const uint8_t *src, const uint64_t *soff, uint64_t m, const std::vector<uint8_t> *header,
                  bool eof, int level, uint8_t *dst, uint64_t dst_cap, uint64_t *out_bytes) {
    const std::vector<uint8_t> hz = header ? bgzf_compress_host(header->data(), header->size(), level) : std::vector<uint8_t>();
    uint64_t ends[2] = {0, 0};
    if (m) {
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&ends[0], soff, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&ends[1], soff + m, 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t len = ends[1] - ends[0];
    if (hz.size() + oge_bgzf_bound(len) + 28 > dst_cap) return oge_fail(ctx, OGE_ERR_LIMIT, "output buffer too small");
    if (!hz.empty()) OGE_HIP_TRY(ctx, hipMemcpyAsync(dst, hz.data(), hz.size(), hipMemcpyHostToDevice, ctx->stream));
    uint64_t zb = 0;
    if (len) {
        const int rc = oge_bgzf_deflate_dev(ctx, src + ends[0], len, level, dst + hz.size(), dst_cap - hz.size() - 28, &zb);
        if (rc) return rc;
    }
    if (eof) OGE_HIP_TRY(ctx, hipMemcpyAsync(dst + hz.size() + zb, kBgzfEof, 28, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *out_bytes = hz.size() + zb + (eof ? 28 : 0);
    return OGE_OK;
}

static std::vector<uint8_t> out_header(const BamFile &f, const oge_mergesort_opts *mo) {
    BamHeaderModel oh = f.header;
    oh.sort_order = BamHeaderModel::COORDINATE;  // read_sorter.cpp:257-258
    if (mo->program_line) add_program_record(oh, mo->program_line);
    return bam_encode_header(oh);
}

// sort (+ markdup) X -> Y (ws "pipe_y", cap bytes) with bins recomputed and 0x400 applied; with -R the
// kept records go back into X.  *src / *soff / *m: the records to write; *spare: the other buffer.
static int sort_stage(oge_ctx *ctx, uint8_t *X, uint64_t *xoff, uint64_t n, uint64_t cap, const BamFile &f, const oge_mergesort_opts *mo,
                      uint8_t **src, uint64_t **soff, uint64_t *m, uint64_t *nd, uint8_t **spare) {
    const int32_t n_ref = (int32_t)f.ref_names.size();
    uint8_t *Y = (uint8_t *)ctx->ws("pipe_y", cap);
    uint64_t *yoff = (uint64_t *)ctx->ws("pipe_yoff", (n + 1) * 8);
    uint32_t *perm = (uint32_t *)ctx->ws("pipe_perm", (n + 1) * 4);
    if (!Y || !yoff || !perm) return OGE_ERR_HIP;
    *nd = 0;
    LibTable lt(f.header, n_ref, mo);
    int rc;
    if (mo->mark_duplicates) {
        rc = oge_sort_markdup_dev(ctx, X, xoff, n, &lt.o, perm, Y, yoff, nd);
    } else {
        rc = oge_sort_coord_dev(ctx, X, xoff, n, n_ref, perm);
        if (!rc) rc = oge_gather_records_dev(ctx, X, xoff, perm, n, Y, yoff);
    }
    if (rc) return rc;
    *src = Y, *spare = X, *soff = yoff, *m = n;
    if (mo->mark_duplicates && mo->remove_duplicates) {  // -R: MarkDuplicates::runInternal :456-458
        OgeStageTimer *tm = ctx->begin_stage("drop_dups");
        rc = oge_drop_flagged_dev(ctx, Y, yoff, n, 0x400, X, xoff, m);
        ctx->end_stage(tm);
        if (rc) return rc;
        *src = X, *spare = Y, *soff = xoff;
    }
    return OGE_OK;
}

// The chain's two record arenas ("pipe_x", "pipe_y": decompressed stream / output file, sorted records)
// sized for streams of up to `total` decompressed bytes, allocated now: a service that reserves them once
// at start-up never re-acquires tens of GB of HBM inside a call (HBM this process or another freed is
// wiped by the driver before it is handed out again: ~35-45 GB/s, profiles/r05g_alloc.txt).  The arenas
// are free between calls; *x / *y / *cap let the caller stage data in them meanwhile.
extern "C" int oge_mergesort_reserve(oge_ctx *ctx, uint64_t total, void **x, void **y, uint64_t *cap_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    (void)hipSetDevice(ctx->device);
    const uint64_t cap = std::max<uint64_t>(total, oge_bgzf_bound(total) + (1u << 20)) + 64;
    void *a = ctx->ws("pipe_x", cap), *b = ctx->ws("pipe_y", cap);
    if (!a || !b) return OGE_ERR_HIP;
    if (x) *x = a;
    if (y) *y = b;
    if (cap_out) *cap_out = cap;
    return OGE_OK;
}

extern "C" int oge_mergesort_bgzf_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const oge_mergesort_opts *mo,
                                      const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads, uint64_t *n_dup) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!mo || !d_out || !out_bytes || (zbytes && !d_z)) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    if (mo->level < 0 || mo->level > 9) return oge_fail(ctx, OGE_ERR_ARG, "level must be 0..9");
    (void)hipSetDevice(ctx->device);
    Hold hold(ctx);
    *d_out = nullptr;
    *out_bytes = 0;
    uint8_t *X;
    uint64_t cap, *xoff, n;
    BamFile f;
    int rc = decode(ctx, d_z, zbytes, &X, &cap, &xoff, &n, &f);
    if (rc) return rc;
    uint8_t *src, *dst;
    uint64_t *soff, m, nd;
    rc = sort_stage(ctx, X, xoff, n, cap, f, mo, &src, &soff, &m, &nd, &dst);
    if (rc) return rc;

    // ---- output: header block(s) (host zlib/libdeflate, tiny), device deflate of the records, EOF
    const std::vector<uint8_t> hb = out_header(f, mo);
    uint64_t ob = 0;
    rc = encode(ctx, src, soff, m, &hb, true, mo->level, dst, cap, &ob);
    if (rc) return rc;
    *d_out = dst;
    *out_bytes = ob;
    if (n_reads) *n_reads = m;
    if (n_dup) *n_dup = nd;
    return OGE_OK;
}

// The same chain on a BAM file in HOST memory with the PCIe transfers overlapped (the
// reference's reader / writer threads overlap I/O with the modules, util/bgzf_input_stream.cpp:180-206,
// util/bgzf_output_stream.cpp:252-285): the file goes up in G chunks on a copy stream while the host
// indexes its framing (oge_bgzf_index_host_mt) and the blocks of every chunk already up are inflated;
// after the sort, the output is deflated in block-aligned segments into two device buffers whose copies
// down to h_out run (high-priority stream) while the next segment is compressed.  The output bytes equal oge_mergesort_bgzf_dev's
// (segments of whole payloads: the same blocks).  h_z / h_out page-locked for full speed.
static uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *e = getenv(name);
    return e && *e ? strtoull(e, nullptr, 10) : dflt;
}

extern "C" int oge_mergesort_bgzf_host(oge_ctx *ctx, const uint8_t *h_z, uint64_t zbytes, const oge_mergesort_opts *mo, uint8_t *h_out,
                                       uint64_t out_cap, uint64_t *out_bytes, uint64_t *n_reads, uint64_t *n_dup) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!mo || !out_bytes || !h_out || (zbytes && !h_z)) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    if (mo->level < 0 || mo->level > 9) return oge_fail(ctx, OGE_ERR_ARG, "level must be 0..9");
    (void)hipSetDevice(ctx->device);
    Hold hold(ctx);
    *out_bytes = 0;
    // OGE_HOSTPIPE_TRACE: host timestamps of the steps on stderr (where the PCIe-inclusive time goes)
    const bool trace = getenv("OGE_HOSTPIPE_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what, uint64_t k = 0) {
        if (trace)
            fprintf(stderr, "[hostpipe] %8.1f ms %s %llu\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), what,
                    (unsigned long long)k);
    };
    hipStream_t cs = ctx->side_stream(3);
    uint8_t *dz = (uint8_t *)ctx->ws("hostpipe_z", zbytes + 64);
    if (!cs || !dz) return OGE_ERR_HIP;
    // ---- 1. the file up in G chunks on the copy stream (4 KiB-aligned cuts), an event after each
    const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(env_u64("OGE_HOSTPIPE_GROUPS", 8), 64));
    const uint64_t C = ((zbytes + G - 1) / G + 4095) & ~4095ull;
    std::vector<hipEvent_t> up;
    struct Evs {
        std::vector<hipEvent_t> *v;
        ~Evs() {
            for (auto e : *v) (void)hipEventDestroy(e);
        }
    } evs{&up};
    // Every exit, error paths included, waits for the copy stream (uploads reading h_z, downloads writing
    // h_out) and the context stream (the direct mode's emitter writes h_out): a caller may free or reuse
    // its page-locked buffers as soon as this returns.  Declared after `evs`, so it runs first.
    struct Drain {
        hipStream_t a, b;
        ~Drain() {
            (void)hipStreamSynchronize(a);
            (void)hipStreamSynchronize(b);
        }
    } drain{cs, ctx->stream};
    // test hook: OGE_HOSTPIPE_FAIL_SEG=k makes segment k (k >= 1) fail after the earlier segments' copies
    // were queued (tests/test_gpu_pipeline.py::test_host_pipeline_failed_segment_drains)
    const uint64_t fail_seg = env_u64("OGE_HOSTPIPE_FAIL_SEG", 0);
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // dz may still be read by this context's last call
    for (uint64_t o = 0; o < zbytes; o += C) {
        hipEvent_t e;
        OGE_HIP_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        up.push_back(e);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dz + o, h_z + o, std::min(C, zbytes - o), hipMemcpyHostToDevice, cs));
        OGE_HIP_TRY(ctx, hipEventRecord(e, cs));
    }
    mark("upload queued");
    // ---- 2. the framing, on the host meanwhile
    OgeStageTimer *tm = ctx->begin_stage("bgzf_index");
    std::vector<uint64_t> d0, d1, uo;
    std::vector<uint32_t> crc;
    if (!oge_bgzf_index_host_mt(h_z, zbytes, (int)env_u64("OGE_HOSTPIPE_THREADS", 16), d0, d1, uo, crc)) {
        uint64_t nb = 0;  // the sequential walk, for its error messages
        int rc = oge_bgzf_index(h_z, zbytes, nullptr, nullptr, nullptr, nullptr, 0, &nb);
        if (rc != OGE_OK && rc != OGE_ERR_ARG) return oge_fail(ctx, rc, oge_last_error(nullptr));
        d0.resize(nb), d1.resize(nb), uo.resize(nb + 1), crc.resize(nb);
        rc = oge_bgzf_index(h_z, zbytes, d0.data(), d1.data(), uo.data(), crc.data(), nb, &nb);
        if (rc) return oge_fail(ctx, rc, oge_last_error(nullptr));
    }
    const uint64_t nb = d0.size(), total = uo[nb];
    if (!total) return oge_fail(ctx, OGE_ERR_IO, "empty BAM stream (no BAM magic)");
    uint64_t *dix = (uint64_t *)ctx->ws("pipe_ix", (3 * nb + 2) * 8);
    uint32_t *dcrc = (uint32_t *)ctx->ws("pipe_ixc", (nb + 1) * 4);
    if (!dix || !dcrc) return OGE_ERR_HIP;
    if (nb) {
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dix, d0.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dix + nb, d1.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dcrc, crc.data(), nb * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dix + 2 * nb, uo.data(), (nb + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    ctx->end_stage(tm);
    mark("host index done");
    // ---- 3. inflate: the blocks whose bytes are up, chunk after chunk (the X of the device chain)
    const uint64_t cap = std::max<uint64_t>(total, oge_bgzf_bound(total) + (1u << 20)) + 64;
    uint8_t *X = (uint8_t *)ctx->ws("pipe_x", cap);
    if (!X) return OGE_ERR_HIP;
    uint64_t b = 0;
    for (size_t g = 0; g < up.size(); ++g) {
        const uint64_t end = std::min(zbytes, (g + 1) * C);
        uint64_t b1 = b;
        while (b1 < nb && d1[b1] + 8 <= end) ++b1;
        if (g + 1 == up.size()) b1 = nb;
        OGE_HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, up[g], 0));
        if (b1 > b) {
            const int rc = oge_bgzf_inflate_dev(ctx, dz, zbytes, dix + b, dix + nb + b, dix + 2 * nb + b, dcrc + b, b1 - b, X);
            if (rc) return rc;
        }
        b = b1;
    }
    mark("inflate queued");
    // ---- 4. records, sort (+ markdup)
    uint64_t *xoff, n;
    BamFile f;
    int rc = decode_records(ctx, X, total, &xoff, &n, &f);
    if (rc) return rc;
    mark("records walked");
    uint8_t *src, *spare;
    uint64_t *soff, m, nd;
    rc = sort_stage(ctx, X, xoff, n, cap, f, mo, &src, &soff, &m, &nd, &spare);
    if (rc) return rc;
    (void)spare;
    mark("sorted");
    // ---- 5. header block(s), then the records deflated segment by segment, each copied down while the
    //         next one is compressed
    const std::vector<uint8_t> hb = out_header(f, mo);
    const std::vector<uint8_t> hz = bgzf_compress_host(hb.data(), hb.size(), mo->level);
    if (hz.size() + 28 > out_cap) return oge_fail(ctx, OGE_ERR_LIMIT, "output buffer too small");
    memcpy(h_out, hz.data(), hz.size());
    uint64_t ends[2] = {0, 0};
    if (m) {
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&ends[0], soff, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&ends[1], soff + m, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    const uint64_t len = ends[1] - ends[0];
    // OGE_HOSTPIPE_DIRECT=1, h_out page-locked with room for the bound: the emitter writes the blocks
    // straight into it over PCIe.  Off by default: the kernels' stores reach ~42 GB/s over the link
    // (r05n: 1.37 s for the 56.6 GB output) against ~57 GB/s for the copies of the segmented path.
    uint8_t *hdev = nullptr;
    if (len && hz.size() + oge_bgzf_bound(len) + 28 <= out_cap && env_u64("OGE_HOSTPIPE_DIRECT", 0)) {
        hipPointerAttribute_t at;
        void *dp = nullptr;
        if (hipPointerGetAttributes(&at, h_out) == hipSuccess && at.type == hipMemoryTypeHost &&
            hipHostGetDevicePointer(&dp, h_out, 0) == hipSuccess)
            hdev = (uint8_t *)dp;
        (void)hipGetLastError();
    }
    if (hdev) {
        uint64_t got = 0;
        rc = oge_bgzf_deflate_dev(ctx, src + ends[0], len, mo->level, hdev + hz.size(), oge_bgzf_bound(len), &got);
        if (rc) return rc;
        mark("deflated into host memory", got);
        memcpy(h_out + hz.size() + got, kBgzfEof, 28);
        *out_bytes = hz.size() + got + 28;
        if (n_reads) *n_reads = m;
        if (n_dup) *n_dup = nd;
        return OGE_OK;
    }
    const uint64_t SEG = (uint64_t)oge_bgzf::kPay * std::max<uint64_t>(1, env_u64("OGE_HOSTPIPE_SEG_BLOCKS", 32768));
    const uint64_t bnd = oge_bgzf_bound(std::min(len, SEG));
    // each segment is compressed at the same offset mod 256 as its place in h_out: a copy whose source
    // and destination are co-aligned runs at the link's rate (45 GB/s otherwise, profiles/r05k_bench.log)
    uint8_t *zb[2] = {(uint8_t *)ctx->ws("hostpipe_out0", bnd + 256), (uint8_t *)ctx->ws("hostpipe_out1", bnd + 256)};
    if (!zb[0] || !zb[1]) return OGE_ERR_HIP;
    hipEvent_t dn[2];
    OGE_HIP_TRY(ctx, hipEventCreateWithFlags(&dn[0], hipEventDisableTiming));
    up.push_back(dn[0]);
    OGE_HIP_TRY(ctx, hipEventCreateWithFlags(&dn[1], hipEventDisableTiming));
    up.push_back(dn[1]);
    uint64_t pos = hz.size();
    for (uint64_t s0 = 0, k = 0; s0 < len; s0 += SEG, ++k) {
        const uint64_t sl = std::min(SEG, len - s0);
        if (k >= 2) OGE_HIP_TRY(ctx, hipEventSynchronize(dn[k & 1]));  // that buffer's copy is done
        mark("segment buffer free", k);
        uint64_t got = 0;
        const uint64_t sh = ((uintptr_t)(h_out + pos)) & 255;
        if (fail_seg && k == fail_seg) return oge_fail(ctx, OGE_ERR_HIP, "injected segment failure (OGE_HOSTPIPE_FAIL_SEG)");
        rc = oge_bgzf_deflate_dev(ctx, src + ends[0] + s0, sl, mo->level, zb[k & 1] + sh, bnd, &got);  // returns when written
        if (rc) return rc;
        mark("segment deflated", k);
        if (pos + got + 28 > out_cap) return oge_fail(ctx, OGE_ERR_LIMIT, "output buffer too small");
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h_out + pos, zb[k & 1] + sh, got, hipMemcpyDeviceToHost, cs));
        OGE_HIP_TRY(ctx, hipEventRecord(dn[k & 1], cs));
        pos += got;
    }
    OGE_HIP_TRY(ctx, hipStreamSynchronize(cs));
    mark("downloaded", pos);
    memcpy(h_out + pos, kBgzfEof, 28);
    *out_bytes = pos + 28;
    if (n_reads) *n_reads = m;
    if (n_dup) *n_dup = nd;
    return OGE_OK;
}

// The sort + dedup + write half of the multi-rank chains: this rank's decoded records (its input
// shard; a rank whose decode failed passes rc != 0 and still joins the collectives with no records,
// then reports its error) through oge_sort_markdup_dist, then its slice of the one output file: rank 0's
// starts with the header, the last rank's ends with the EOF block, so the slices concatenate.
static int dist_sort_write(oge_comm *comm, int rc, const std::string &why, uint8_t *X, uint64_t *xoff, uint64_t n, const BamFile &f,
                           const oge_mergesort_opts *mo, const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads_total,
                           uint64_t *n_dup_total) {
    oge_ctx *ctx = oge_comm_ctx(comm);
    const int rank = oge_comm_rank(comm), G = oge_comm_size(comm);
    const int32_t n_ref = (int32_t)f.ref_names.size();
    LibTable lt(f.header, n_ref, mo);
    uint8_t *dout = nullptr;
    uint64_t *doff = nullptr, no = 0, nd = 0;
    const int rd = oge_sort_markdup_dist(comm, rc ? nullptr : X, rc ? nullptr : xoff, rc ? 0 : n, n_ref, 1,
                                         mo->mark_duplicates ? &lt.o : nullptr, &dout, &doff, &no, &nd);
    if (rc) return oge_fail(ctx, rc, why.c_str());
    if (rd) return rd;
    const uint8_t *src = dout;
    const uint64_t *soff = doff;
    uint64_t m = no;
    uint8_t *Y = nullptr;
    uint64_t *yoff = (uint64_t *)ctx->ws("pipe_yoff", (no + 1) * 8);
    if (!yoff) return OGE_ERR_HIP;
    if (mo->mark_duplicates && mo->remove_duplicates) {
        uint64_t bytes = 0;
        if (no) {
            OGE_HIP_TRY(ctx, hipMemcpyAsync(&bytes, doff + no, 8, hipMemcpyDeviceToHost, ctx->stream));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        Y = (uint8_t *)ctx->ws("pipe_y", bytes + 64);
        if (!Y) return OGE_ERR_HIP;
        OgeStageTimer *tm = ctx->begin_stage("drop_dups");
        rc = oge_drop_flagged_dev(ctx, dout, doff, no, 0x400, Y, yoff, &m);
        ctx->end_stage(tm);
        if (rc) return rc;
        src = Y, soff = yoff;
    }
    uint64_t len = 0;
    if (m) {
        uint64_t e[2];
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&e[0], soff, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&e[1], soff + m, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        len = e[1] - e[0];
    }
    const std::vector<uint8_t> hb = out_header(f, mo);
    const uint64_t zcap = oge_bgzf_bound(len) + (rank == 0 ? bgzf_compress_host(hb.data(), hb.size(), mo->level).size() : 0) + 64;
    uint8_t *Z = (uint8_t *)ctx->ws("pipe_z", zcap);
    if (!Z) return OGE_ERR_HIP;
    uint64_t ob = 0;
    rc = encode(ctx, src, soff, m, rank == 0 ? &hb : nullptr, rank == G - 1, mo->level, Z, zcap, &ob);
    if (rc) return rc;
    *d_out = Z;
    *out_bytes = ob;
    uint64_t tot = m;  // records written over all ranks
    rc = oge_comm_sum_u64(comm, &tot, 1);
    if (rc) return rc;
    if (n_reads_total) *n_reads_total = tot;
    if (n_dup_total) *n_dup_total = nd;
    return OGE_OK;
}

static int dist_args(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, const oge_mergesort_opts *mo, const uint8_t **d_out,
                     uint64_t *out_bytes) {
    if (!comm) return oge_fail(nullptr, OGE_ERR_ARG, "null communicator");
    oge_ctx *ctx = oge_comm_ctx(comm);
    if (!mo || !d_out || !out_bytes || (zbytes && !d_z)) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    if (mo->level < 0 || mo->level > 9) return oge_fail(ctx, OGE_ERR_ARG, "level must be 0..9");
    (void)hipSetDevice(ctx->device);
    *d_out = nullptr;
    *out_bytes = 0;
    return OGE_OK;
}

// The same chain over G ranks: rank g's input is its own BAM file (mergesort's inputs, one per rank;
// the header of rank 0's file is the output's, as MultiReader takes the first file's).
extern "C" int oge_mergesort_bgzf_dist(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, const oge_mergesort_opts *mo,
                                       const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads_total, uint64_t *n_dup_total) {
    if (const int rc = dist_args(comm, d_z, zbytes, mo, d_out, out_bytes)) return rc;
    oge_ctx *ctx = oge_comm_ctx(comm);
    Hold hold(ctx);
    oge_comm_reset_stats(comm);
    uint8_t *X = nullptr;
    uint64_t cap = 0, *xoff = nullptr, n = 0;
    BamFile f;
    // a rank whose decode fails still joins the collectives (with no records), and reports its error
    const int rc = decode(ctx, d_z, zbytes, &X, &cap, &xoff, &n, &f);
    return dist_sort_write(comm, rc, rc ? ctx->err : std::string(), X, xoff, n, f, mo, d_out, out_bytes, n_reads_total, n_dup_total);
}

// ONE input file over G ranks (config 4): rank g holds the file's bytes from a_g on and decodes the
// blocks that start in its own_bytes (shard.hip), then the same sort + dedup + write half.
extern "C" int oge_mergesort_bgzf_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own_bytes,
                                        const oge_mergesort_opts *mo, const uint8_t **d_out, uint64_t *out_bytes,
                                        uint64_t *n_reads_total, uint64_t *n_dup_total) {
    if (const int rc = dist_args(comm, d_z, zbytes, mo, d_out, out_bytes)) return rc;
    oge_ctx *ctx = oge_comm_ctx(comm);
    Hold hold(ctx);
    oge_comm_reset_stats(comm);
    uint8_t *X = nullptr;
    uint64_t *xoff = nullptr, n = 0;
    std::vector<uint8_t> h;
    int rc = oge_decode_shard(comm, d_z, zbytes, own_bytes, &X, &xoff, &n, &h);
    if (rc) return rc;  // collective: every rank failed together
    BamFile f;
    std::string err;
    size_t rec_base = 0;
    if (!bam_parse_header(h.data(), h.size(), f, err, &rec_base)) return oge_fail(ctx, OGE_ERR_IO, ("BAM header: " + err).c_str());
    return dist_sort_write(comm, OGE_OK, std::string(), X, xoff, n, f, mo, d_out, out_bytes, n_reads_total, n_dup_total);
}
