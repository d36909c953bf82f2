// modules.cpp -- AlgorithmModule chain over the C ABI (see modules.h).
#include "modules.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cerrno>
#include <cstring>
#include <map>
#include <memory>
#include <functional>
#include <atomic>
#include <thread>
#include <unistd.h>
#include <sys/stat.h>
#include <fcntl.h>

#include "bam_layout.h"

// realign.hip (C++): the realignment result's records and offsets moved out without a copy
void oge_realign_result_take(oge_realign_result *r, oge::bytevec &recs, std::vector<uint64_t> &offs);

namespace oge {

bool AlgorithmModule::verbose_ = false;

int ChainContext::fail(const std::string &where) {
    fprintf(stderr, "openge: %s: %s\n", where.c_str(), oge_last_error(ctx));
    return -1;
}

// OGE_WRITE_DEVICE=1: host batches are deflated on the GPU (FileWriter, LocalRealignment's result)
static bool write_device_forced() {
    const char *e = getenv("OGE_WRITE_DEVICE");
    return e && !strcmp(e, "1");
}

int ChainContext::to_device(ReadBatch &b) {
    if (b.dev_valid) return 0;
    const uint64_t bytes = b.offs[b.n];
    void *r = nullptr, *o = nullptr;
    if (oge_dev_alloc(ctx, bytes + 64, &r) || oge_dev_alloc(ctx, (b.n + 1) * 8, &o)) return fail("device allocation");
    if (oge_memcpy(ctx, r, b.recs.data(), bytes, 1) || oge_memcpy(ctx, o, b.offs.data(), (b.n + 1) * 8, 1))
        return fail("host->device copy");
    b.d_recs = (uint8_t *)r;
    b.d_offs = (uint64_t *)o;
    b.d_bytes = bytes;
    b.dev_valid = true;
    return 0;
}

int ChainContext::to_host(ReadBatch &b) {
    if (b.host_valid) return 0;
    b.recs.clear();
    b.recs.reserve(b.d_bytes + 16);
    want_huge_pages(b.recs.data(), b.d_bytes + 16);
    b.recs.resize(b.d_bytes + 16);  // uninitialised: the copy below writes every byte but the slack
    memset(b.recs.data() + b.d_bytes, 0, 16);
    b.offs.resize(b.n + 1);
    if (oge_memcpy(ctx, b.recs.data(), b.d_recs, b.d_bytes, 2) || oge_memcpy(ctx, b.offs.data(), b.d_offs, (b.n + 1) * 8, 2))
        return fail("device->host copy");
    b.host_valid = true;
    return 0;
}

void ChainContext::free_device(ReadBatch &b) {
    if (b.d_recs) oge_dev_free(ctx, b.d_recs);
    if (b.d_offs) oge_dev_free(ctx, b.d_offs);
    b.d_recs = nullptr;
    b.d_offs = nullptr;
    b.dev_valid = false;
}

int ChainContext::init_ranks() {
    if (gpus <= 1 || !comms.empty()) return 0;
    const int ndev = oge_device_count();
    if (ndev < 1) return fail("--gpus");
    rank_ctx.assign(gpus, nullptr);
    rank_ctx[0] = ctx;
    for (int g = 1; g < gpus; ++g) {
        if (oge_ctx_create((device + g) % ndev, &rank_ctx[g])) {
            rank_ctx.resize(g);
            return fail("--gpus: context");
        }
        const char *pool = getenv("OGE_POOL");
        if (!(pool && std::string(pool) == "0")) oge_ctx_set_pool(rank_ctx[g], 1);
    }
    // the multi-process route of bench.py / a torchrun launch, one host thread per rank: one id, every
    // rank joins concurrently (RCCL between distinct GPUs, the host-staged transport when they share one)
    std::vector<uint8_t> id(oge_comm_unique_id_bytes());
    if (oge_comm_unique_id(id.data(), id.size())) return fail("--gpus: communicator id");
    comms.assign(gpus, nullptr);
    std::vector<int> rcs(gpus, 0);
    std::vector<std::string> why(gpus);
    {
        std::vector<std::thread> ts;
        for (int g = 0; g < gpus; ++g)
            ts.emplace_back([&, g]() {
                // every rank is a thread of this process: the shared-segment meeting is node-local by
                // construction, so ranks sharing a device take the host transport
                rcs[g] = oge_comm_init_rank_mode(rank_ctx[g], gpus, g, id.data(), gpus > ndev ? "host" : "node", &comms[g]);
                if (rcs[g]) why[g] = oge_last_error(rank_ctx[g]);
            });
        for (auto &t : ts) t.join();
    }
    for (int g = 0; g < gpus; ++g)
        if (rcs[g]) {
            fprintf(stderr, "openge: --gpus: rank %d communicator: %s\n", g, why[g].c_str());
            for (oge_comm *c : comms)
                if (c) oge_comm_destroy(c);
            comms.clear();
            return -1;
        }
    if (verbose)
        fprintf(stderr, "[openge] %d ranks on %d device(s), transport %s\n", gpus, std::min(gpus, ndev), oge_comm_transport(comms[0]));
    return 0;
}

void ChainContext::close_ranks() {
    for (oge_comm *c : comms) oge_comm_destroy(c);
    comms.clear();
    for (size_t g = 1; g < rank_ctx.size(); ++g) oge_ctx_destroy(rank_ctx[g]);
    rank_ctx.clear();
}

// Cut the batch into G contiguous input ranges and run oge_sort_markdup_dist on every rank (one host
// thread each).  A rank whose own preparation failed still joins the collectives with an empty shard
// so the others finish, and the failure is reported.
int run_ranks(ChainContext &cc, ReadBatch &b, bool sort, const oge_markdup_opts *opts, uint64_t *n_dup) {
    const bool sharded = !b.shards.empty();  // the reader left every rank its own input shard
    if (cc.init_ranks() || (!sharded && cc.to_device(b))) return -1;
    const int G = cc.gpus;
    const uint64_t n = b.n;
    const int32_t n_ref = (int32_t)b.ref_names.size();
    std::vector<uint64_t> cut(G + 1), boff(G + 1);
    for (int g = 0; g <= G && !sharded; ++g) {
        cut[g] = n * (uint64_t)g / (uint64_t)G;
        if (oge_memcpy(cc.ctx, &boff[g], b.d_offs + cut[g], 8, 2)) return cc.fail("device->host copy");
    }
    std::vector<ReadBatch::Slice> sl(G);
    std::vector<int> rcs(G, 0);
    std::vector<uint64_t> nds(G, 0);
    std::vector<std::string> why(G);
    std::vector<std::thread> ts;
    for (int g = 0; g < G; ++g)
        ts.emplace_back([&, g]() {
            oge_ctx *c = cc.rank_ctx[g];
            uint8_t *dout = nullptr;
            uint64_t *doff = nullptr, no = 0, nd = 0;
            if (sharded) {  // the rank's own shard, in its HBM already
                const ReadBatch::Slice &s = b.shards[g];
                rcs[g] = oge_sort_markdup_dist(cc.comms[g], s.d_recs, s.d_offs, s.n, n_ref, sort ? 1 : 0, opts, &dout, &doff, &no, &nd);
                if (rcs[g]) why[g] = oge_last_error(c);
                sl[g] = {c, dout, doff, no};
                nds[g] = nd;
                return;
            }
            const uint64_t lo = cut[g], m = cut[g + 1] - lo, bytes = boff[g + 1] - boff[g];
            void *r = nullptr, *o = nullptr;
            int rc = oge_dev_alloc(c, bytes + 64, &r);
            if (!rc) rc = oge_dev_alloc(c, (m + 1) * 8, &o);
            if (!rc && bytes) rc = oge_memcpy(c, r, b.d_recs + boff[g], bytes, 4);
            if (!rc) rc = oge_memcpy(c, o, b.d_offs + lo, (m + 1) * 8, 4);
            if (rc) why[g] = oge_last_error(c);
            // the offsets stay absolute: the records pointer is shifted back by the range's first one
            const int rd = rc ? oge_sort_markdup_dist(cc.comms[g], nullptr, nullptr, 0, n_ref, sort ? 1 : 0, opts, &dout, &doff, &no, &nd)
                              : oge_sort_markdup_dist(cc.comms[g], (const uint8_t *)r - boff[g], (const uint64_t *)o, m, n_ref,
                                                      sort ? 1 : 0, opts, &dout, &doff, &no, &nd);
            if (!rc && rd) why[g] = oge_last_error(c);
            rcs[g] = rc ? rc : rd;
            if (r) oge_dev_free(c, r);
            if (o) oge_dev_free(c, o);
            sl[g] = {c, dout, doff, no};
            nds[g] = nd;
        });
    for (auto &t : ts) t.join();
    for (int g = 0; g < G; ++g)
        if (rcs[g]) {
            fprintf(stderr, "openge: rank %d: %s\n", g, why[g].c_str());
            return -1;
        }
    cc.free_device(b);
    b.shards.clear();
    b.slices = sl;
    b.n = 0;
    for (auto &x : sl) b.n += x.n;
    b.host_valid = false;
    *n_dup = nds[0];
    return 0;
}

int AlgorithmModule::runChain(ChainContext &cc) {
    AlgorithmModule *head = this;
    while (head->source_) head = head->source_;
    ReadBatch b;
    bool marked = false;  // ReadSorter fused MarkDuplicates into its device pipeline
    for (AlgorithmModule *m = head; m; m = m->sink_) {
        if (marked && dynamic_cast<MarkDuplicates *>(m)) {
            b.drop_duplicates = static_cast<MarkDuplicates *>(m)->removeDuplicates;
            marked = false;
            continue;
        }
        if (verbose_) fprintf(stderr, "[openge] running %s on %llu records\n", m->name(), (unsigned long long)b.n);
        const auto t0 = std::chrono::steady_clock::now();
        int rc = m->runInternal(cc, b);
        if (verbose_)
            fprintf(stderr, "[openge] %s: %.3f s\n", m->name(),
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        if (rc) {
            cc.free_device(b);
            return rc;
        }
        if (dynamic_cast<ReadSorter *>(m) && static_cast<ReadSorter *>(m)->sortBy() == BamHeaderModel::COORDINATE &&
            dynamic_cast<MarkDuplicates *>(m->sink_))
            marked = true;
    }
    cc.free_device(b);
    return 0;
}

// ----------------------------------------------------------------------------------- FileReader
// The input read into host memory on helper threads while the process is still bringing up HIP (r06: the CLI
// starts this before oge_ctx_create, ~0.2 s, and the reader then only copies it up).  One file of 64 MiB to
// 8 GiB; OGE_PREFETCH=0 turns it off.
namespace {
struct Prefetch {
    std::string path;
    uint64_t size = 0;
    bytevec data;
    std::thread th;
    bool ok = false;
};
Prefetch *g_prefetch = nullptr;
bool g_prefetch_used = false;  // (the reader's -v line says so)
}  // namespace

void prefetch_input(const std::string &path) {
    const char *e = getenv("OGE_PREFETCH");
    if ((e && *e == '0') || g_prefetch) return;
    struct stat st;
    const char *mn = getenv("OGE_PREFETCH_MIN");  // smallest file prefetched (bytes; tests lower it)
    const long long pmin = mn && *mn ? atoll(mn) : (64ll << 20);
    if (stat(path.c_str(), &st) || !S_ISREG(st.st_mode) || st.st_size < pmin || st.st_size < 1 || st.st_size > (8ll << 30)) return;
    auto *P = new Prefetch();
    P->path = path;
    P->size = (uint64_t)st.st_size;
    P->th = std::thread([P]() {
        const int fd = open(P->path.c_str(), O_RDONLY);
        if (fd < 0) return;
        const uint64_t Z = P->size;
        try {
            P->data.reserve(Z + 16);
            want_huge_pages(P->data.data(), Z + 16);
            P->data.resize(Z + 16);  // uninitialised: the reads below fill it
        } catch (const std::bad_alloc &) {
            close(fd);
            return;
        }
        memset(P->data.data() + Z, 0, 16);
        std::atomic<bool> bad(false);
        const int T = 8;
        std::vector<std::thread> ts;
        for (int k = 0; k < T; ++k)
            ts.emplace_back([&, k]() {
                uint64_t o = Z * (uint64_t)k / T;
                const uint64_t end = Z * (uint64_t)(k + 1) / T;
                while (o < end) {
                    const ssize_t r = pread(fd, P->data.data() + o, end - o, (off_t)o);
                    if (r <= 0) {
                        bad = true;
                        return;
                    }
                    o += (uint64_t)r;
                }
            });
        for (auto &t : ts) t.join();
        close(fd);
        P->ok = !bad;
    });
    g_prefetch = P;
}

// the prefetched bytes of `path` when they match a file of Z bytes (the helper joined first)
static bool take_prefetch(const std::string &path, uint64_t Z, bytevec &out) {
    Prefetch *P = g_prefetch;
    if (!P || P->path != path) return false;
    g_prefetch = nullptr;
    if (P->th.joinable()) P->th.join();
    const bool ok = P->ok && P->size == Z;
    if (ok) out = std::move(P->data);
    delete P;
    return ok;
}

// The file streamed into HBM through two page-locked buffers (parallel preads of one while the other
// is copied), indexed on the device: no host copy of the whole file to allocate, fault in and unmap
// (a 29 GB file's unmap alone took 1.5 s).  Returns 2 when it does not apply (small files, inputs
// close to the HBM size, a framing the device index rejects) -- the caller then takes the host path.
static int stream_to_device(ChainContext &cc, const std::string &path, void **dz_out, uint64_t *zbytes) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return 2;
    struct stat stt;
    const char *mn = getenv("OGE_STREAM_MIN");  // smallest file streamed (bytes; tests lower it)
    const long long smin = mn && *mn ? atoll(mn) : (64ll << 20);
    if (fstat(fd, &stt) || !S_ISREG(stt.st_mode) || stt.st_size < smin || stt.st_size < 1) {
        close(fd);
        return 2;
    }
    const uint64_t Z = (uint64_t)stt.st_size;
    uint64_t fr = 0, tot = 0;
    if (oge_mem_info(cc.ctx, &fr, &tot) || Z / 10 * 40 > fr) {  // leave the host path to size what follows
        close(fd);
        return 2;
    }
    void *dz = nullptr, *hb[2] = {nullptr, nullptr};
    {
        bytevec pre;
        if (take_prefetch(path, Z, pre)) {  // read while HIP came up: one copy from the helper's buffer
            g_prefetch_used = true;
            const bool ok = !oge_dev_alloc(cc.ctx, Z + 16, &dz) && !oge_memcpy(cc.ctx, dz, pre.data(), Z, 1);
            std::thread([](bytevec v) { v = bytevec(); }, std::move(pre)).detach();  // unmapped beside what follows
            close(fd);
            if (!ok) {
                if (dz) oge_dev_free(cc.ctx, dz);
                return 2;
            }
            *dz_out = dz;
            *zbytes = Z;
            return 0;
        }
    }
    const uint64_t CH = getenv("OGE_STREAM_MIN") ? (64ull << 10) : (256ull << 20);  // tests: many small chunks
    auto cleanup = [&]() {
        for (void *h : hb)
            if (h) oge_host_free(cc.ctx, h);
        close(fd);
    };
    if (oge_dev_alloc(cc.ctx, Z + 16, &dz) || oge_host_alloc(cc.ctx, CH, &hb[0]) || oge_host_alloc(cc.ctx, CH, &hb[1])) {
        if (dz) oge_dev_free(cc.ctx, dz);
        cleanup();
        return 2;
    }
    const uint64_t nch = (Z + CH - 1) / CH;
    std::atomic<bool> bad(false);
    auto read_chunk = [&](uint64_t c) {  // chunk c into hb[c & 1], 8 preads of 32 MB in parallel
        const uint64_t o0 = c * CH, e0 = std::min(Z, o0 + CH);
        const uint64_t sl = 32ull << 20, ns = (e0 - o0 + sl - 1) / sl;
        std::vector<std::thread> ts;
        for (uint64_t k = 0; k < ns; ++k)
            ts.emplace_back([&, k]() {
                uint64_t o = o0 + k * sl;
                const uint64_t e = std::min(e0, o + sl);
                while (o < e) {
                    const ssize_t r = pread(fd, (uint8_t *)hb[c & 1] + (o - o0), e - o, (off_t)o);
                    if (r <= 0) {
                        bad = true;
                        return;
                    }
                    o += (uint64_t)r;
                }
            });
        for (auto &t : ts) t.join();
    };
    read_chunk(0);
    for (uint64_t c = 0; c < nch && !bad; ++c) {
        std::thread next;
        if (c + 1 < nch) next = std::thread(read_chunk, c + 1);
        const uint64_t o = c * CH, len = std::min(Z, o + CH) - o;
        if (oge_memcpy(cc.ctx, (uint8_t *)dz + o, hb[c & 1], len, 1)) bad = true;
        if (next.joinable()) next.join();
    }
    cleanup();
    if (bad) {
        oge_dev_free(cc.ctx, dz);
        return 2;
    }
    *dz_out = dz;
    *zbytes = Z;
    return 0;
}

int FileReader::read_device(ChainContext &cc, ReadBatch &b, const std::string &path) {
    auto clk = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
        return std::chrono::duration<double>(z - a).count();
    };
    const auto t0 = clk();
    const int threads = cc.threads > 0 ? cc.threads : 8;
    bytevec comp;
    std::string err;
    void *dz = nullptr, *di = nullptr, *dc = nullptr, *dout = nullptr, *doff = nullptr;
    auto release = [&]() {
        for (void *p : {dz, di, dc, dout, doff})
            if (p) oge_dev_free(cc.ctx, p);
    };
    uint64_t nb = 0, total = 0, zbytes = 0;
    bool streamed = false;
    if (!getenv("OGE_CHUNK_BYTES") && !(getenv("OGE_READER") && std::string(getenv("OGE_READER")) == "hostcopy") &&
        stream_to_device(cc, path, &dz, &zbytes) == 0) {
        // framing index on the device (count, then fill); anything it rejects goes to the host path
        streamed = oge_bgzf_index_dev(cc.ctx, (const uint8_t *)dz, zbytes, nullptr, nullptr, nullptr, nullptr, 0, &nb) == 0 &&
                   oge_dev_alloc(cc.ctx, (3 * nb + 1) * 8, &di) == 0 && oge_dev_alloc(cc.ctx, nb * 4 + 4, &dc) == 0;
        if (streamed) {
            uint64_t *dd = (uint64_t *)di;
            streamed = oge_bgzf_index_dev(cc.ctx, (const uint8_t *)dz, zbytes, dd, dd + nb, dd + 2 * nb, (uint32_t *)dc, nb, &nb) == 0 &&
                       oge_memcpy(cc.ctx, &total, dd + 3 * nb, 8, 2) == 0;
        }
        if (streamed && sink_sorts()) {
            uint64_t fr = 0, tot = 0;
            if (oge_mem_info(cc.ctx, &fr, &tot) || total / 10 * 25 > fr) streamed = false;
        }
        if (!streamed) {
            release();
            dz = di = dc = nullptr;
            nb = total = 0;
        }
    }
    auto t1 = clk();
    if (!streamed) {
        if (!read_file_bytes(path, comp, threads, err)) {
            fprintf(stderr, "openge: error reading %s: %s\n", path.c_str(), err.c_str());
            return -1;
        }
        oge_bgzf_index(comp.data(), comp.size(), nullptr, nullptr, nullptr, nullptr, 0, &nb);
        std::vector<uint64_t> idx(3 * nb + 1);
        std::vector<uint32_t> crc(nb);
        if (oge_bgzf_index(comp.data(), comp.size(), idx.data(), idx.data() + nb, idx.data() + 2 * nb, crc.data(), nb, &nb))
            return 1;  // not BGZF / truncated: the host reader reports it
        total = idx[3 * nb];
        if (sink_sorts()) {  // larger than HBM (or the chunked test knob): the sorter works from host memory
            uint64_t fr = 0, tot = 0;
            if (getenv("OGE_CHUNK_BYTES") || (!oge_mem_info(cc.ctx, &fr, &tot) && total / 10 * 25 > fr)) return 1;
        }
        t1 = clk();
        zbytes = comp.size();
        if (oge_dev_alloc(cc.ctx, comp.size() + 16, &dz) || oge_dev_alloc(cc.ctx, idx.size() * 8, &di) ||
            oge_dev_alloc(cc.ctx, crc.size() * 4 + 4, &dc)) {
            release();
            return cc.fail("device allocation");
        }
        if (oge_memcpy(cc.ctx, dz, comp.data(), comp.size(), 1) || oge_memcpy(cc.ctx, di, idx.data(), idx.size() * 8, 1) ||
            oge_memcpy(cc.ctx, dc, crc.data(), crc.size() * 4, 1)) {
            release();
            return cc.fail("host->device copy");
        }
    }
    if (oge_dev_alloc(cc.ctx, total + 64, &dout)) {
        release();
        return cc.fail("device allocation");
    }
    const auto t2 = clk();
    const uint64_t *dd = (const uint64_t *)di;
    if (nb && oge_bgzf_inflate_dev(cc.ctx, (const uint8_t *)dz, zbytes, dd, dd + nb, dd + 2 * nb, (const uint32_t *)dc, nb,
                                   (uint8_t *)dout)) {
        release();
        return 1;
    }
    double t_kern = -1;
    if (verbose_) oge_ctx_timing(cc.ctx, "bgzf_inflate", &t_kern);  // synchronises: the kernels' own time
    const auto t2b = clk();
    oge_dev_free(cc.ctx, dz);
    dz = nullptr;
    // the host path's copy of the compressed file (29 GB at 150M reads) takes ~1.5 s to unmap: on a
    // thread of its own, beside the device stages that follow
    if (!comp.empty()) std::thread([](bytevec v) { v = bytevec(); }, std::move(comp)).detach();
    comp = bytevec();
    const auto t3 = clk();
    // header from a prefix of the stream
    BamFile f;
    size_t rec_base = 0;
    for (uint64_t pre = std::min<uint64_t>(total, 1 << 20);; pre = std::min<uint64_t>(total, pre * 8)) {
        std::vector<uint8_t> h(pre);
        if (pre && oge_memcpy(cc.ctx, h.data(), dout, pre, 2)) {
            release();
            return cc.fail("device->host copy");
        }
        f = BamFile();
        if (bam_parse_header(h.data(), pre, f, err, &rec_base)) break;
        if (pre == total) {
            release();
            return 1;
        }
    }
    uint64_t n = 0;
    if (oge_bam_record_offsets_dev(cc.ctx, (const uint8_t *)dout, rec_base, total, (int32_t)f.ref_names.size(), nullptr, 0, &n) ||
        oge_dev_alloc(cc.ctx, (n + 1) * 8, &doff) ||
        oge_bam_record_offsets_dev(cc.ctx, (const uint8_t *)dout, rec_base, total, (int32_t)f.ref_names.size(), (uint64_t *)doff,
                                   n + 1, &n)) {
        release();
        return 1;
    }
    oge_dev_free(cc.ctx, di);
    oge_dev_free(cc.ctx, dc);
    b.header = f.header;
    b.ref_names = f.ref_names;
    b.n = n;
    b.d_recs = (uint8_t *)dout;
    b.d_offs = (uint64_t *)doff;
    b.d_bytes = total;
    b.dev_valid = true;
    b.host_valid = false;
    if (verbose_)
        fprintf(stderr,
                "[openge] FileReader (device%s): file %.3f s, upload %.3f s, inflate %.3f s (kernels %.3f s, release of the "
                "compressed copies %.3f s), records %.3f s\n",
                streamed ? (g_prefetch_used ? ", prefetched + device index" : ", streamed + device index") : "", sec(t0, t1),
                sec(t1, t2), sec(t2, t3), t_kern / 1e3, sec(t2b, t3),
                sec(t3, clk()));
    return 0;
}

// Bytes [off, off + len) of the open file into device memory dst (rank ctx's stream): parallel preads
// into one of two page-locked buffers while the other is copied.  0 = ok.
static int read_range_to_device(oge_ctx *ctx, int fd, uint64_t off, uint64_t len, uint8_t *dst) {
    if (!len) return 0;
    const uint64_t CH = std::min<uint64_t>(len, 128ull << 20);
    void *hb[2] = {nullptr, nullptr};
    if (oge_host_alloc(ctx, CH, &hb[0]) || oge_host_alloc(ctx, CH, &hb[1])) {
        for (void *h : hb)
            if (h) oge_host_free(ctx, h);
        return -1;
    }
    std::atomic<bool> bad(false);
    const uint64_t nch = (len + CH - 1) / CH;
    auto read_chunk = [&](uint64_t c) {
        const uint64_t o0 = c * CH, e0 = std::min(len, o0 + CH), sl = 16ull << 20, ns = (e0 - o0 + sl - 1) / sl;
        std::vector<std::thread> ts;
        for (uint64_t k = 0; k < ns; ++k)
            ts.emplace_back([&, k]() {
                uint64_t o = o0 + k * sl;
                const uint64_t e = std::min(e0, o + sl);
                while (o < e) {
                    const ssize_t r = pread(fd, (uint8_t *)hb[c & 1] + (o - o0), e - o, (off_t)(off + o));
                    if (r <= 0) {
                        bad = true;
                        return;
                    }
                    o += (uint64_t)r;
                }
            });
        for (auto &t : ts) t.join();
    };
    read_chunk(0);
    for (uint64_t c = 0; c < nch && !bad; ++c) {
        std::thread next;
        if (c + 1 < nch) next = std::thread(read_chunk, c + 1);
        const uint64_t o = c * CH, l = std::min(len, o + CH) - o;
        if (oge_memcpy(ctx, dst + o, hb[c & 1], l, 1)) bad = true;
        if (next.joinable()) next.join();
    }
    for (void *h : hb) oge_host_free(ctx, h);
    return bad ? -1 : 0;
}

// True when the next module takes per-rank input shards (run_ranks: the coordinate ReadSorter, or a
// standalone MarkDuplicates).
bool FileReader::sink_takes_shards() const {
    if (auto *rs = dynamic_cast<const ReadSorter *>(sink_)) return rs->sortBy() == BamHeaderModel::COORDINATE;
    return dynamic_cast<const MarkDuplicates *>(sink_) != nullptr;
}

// --gpus G with one input file (config 4): rank g reads the file's bytes [a_g, min(size, b_g + 64 KiB))
// into its own HBM and decodes the BGZF blocks that start in [a_g, b_g) (oge_bgzf_decode_shard: block and
// record boundaries joined with the neighbouring ranks), so the G ranks share the codec instead of rank 0
// inflating the whole file.  Returns 1 when the file cannot be opened or decoded this way (the
// whole-file readers take over and report it).
int FileReader::read_sharded(ChainContext &cc, ReadBatch &b, const std::string &path) {
    const auto t0 = std::chrono::steady_clock::now();
    const int fd = open(path.c_str(), O_RDONLY);
    struct stat stt;
    if (fd < 0) return 1;
    if (fstat(fd, &stt) || !S_ISREG(stt.st_mode)) {
        close(fd);
        return 1;
    }
    if (cc.init_ranks()) {
        close(fd);
        return -1;
    }
    const int G = cc.gpus;
    const uint64_t Z = (uint64_t)stt.st_size;
    std::vector<ReadBatch::Slice> sh(G);
    std::vector<int> rcs(G, 0);
    std::vector<std::string> why(G);
    std::vector<uint8_t> hdr(1 << 22);
    uint64_t hlen = 0;
    std::vector<double> t_read(G, 0), t_dec(G, 0);
    std::vector<std::thread> ts;
    for (int g = 0; g < G; ++g)
        ts.emplace_back([&, g]() {
            oge_ctx *c = cc.rank_ctx[g];
            const uint64_t a = Z * (uint64_t)g / (uint64_t)G, bnd = Z * (uint64_t)(g + 1) / (uint64_t)G;
            const uint64_t end = std::min<uint64_t>(Z, bnd + 65536), len = end - a;
            void *dz = nullptr;
            const auto r0 = std::chrono::steady_clock::now();
            int rc = oge_dev_alloc(c, len + 64, &dz);
            if (!rc && read_range_to_device(c, fd, a, len, (uint8_t *)dz)) rc = OGE_ERR_IO;
            if (rc) why[g] = rc == OGE_ERR_IO ? std::string("read failed") : std::string(oge_last_error(c));
            const auto r1 = std::chrono::steady_clock::now();
            const uint8_t *recs = nullptr;
            const uint64_t *offs = nullptr;
            uint64_t n = 0, hl = 0;
            // a rank whose read failed still takes part, with no buffer: its argument error fails every rank
            const int rd = oge_bgzf_decode_shard(cc.comms[g], rc ? nullptr : (const uint8_t *)dz, len, bnd - a, &recs, &offs, &n,
                                                 g == 0 ? hdr.data() : nullptr, g == 0 ? hdr.size() : 0, g == 0 ? &hl : nullptr);
            if (!rc && rd) why[g] = oge_last_error(c);
            rcs[g] = rc ? rc : rd;
            if (g == 0) hlen = hl;
            if (dz) oge_dev_free(c, dz);
            sh[g] = {c, const_cast<uint8_t *>(recs), const_cast<uint64_t *>(offs), n};
            t_read[g] = std::chrono::duration<double>(r1 - r0).count();
            t_dec[g] = std::chrono::duration<double>(std::chrono::steady_clock::now() - r1).count();
        });
    for (auto &t : ts) t.join();
    close(fd);
    // a file the sharded decode rejects goes to the whole-file readers, which report format errors with
    // the reference's messages (the ranks failed together, so their communicators are still in step)
    for (int g = 0; g < G; ++g)
        if (rcs[g]) {
            if (verbose_) fprintf(stderr, "[openge] FileReader: sharded decode failed on rank %d (%s); reading the whole file\n", g, why[g].c_str());
            return 1;
        }
    BamFile f;
    std::string err;
    size_t rec_base = 0;
    if (!bam_parse_header(hdr.data(), hlen, f, err, &rec_base)) return 1;
    b.header = f.header;
    b.ref_names = f.ref_names;
    b.shards = sh;
    b.n = 0;
    for (auto &s : sh) b.n += s.n;
    b.dev_valid = b.host_valid = false;
    if (verbose_) {
        std::string per;
        for (int g = 0; g < G; ++g) {
            uint64_t nb = 0;
            oge_ctx_counter(cc.rank_ctx[g], "shard_blocks", &nb);
            char tmp[160];
            snprintf(tmp, sizeof tmp, " [rank %d: read %.3f s, decode %.3f s, %llu blocks, %llu records]", g, t_read[g], t_dec[g],
                     (unsigned long long)nb, (unsigned long long)sh[g].n);
            per += tmp;
        }
        fprintf(stderr, "[openge] FileReader (sharded over %d ranks): %.3f s%s\n", G,
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), per.c_str());
    }
    return 0;
}

int FileReader::runInternal(ChainContext &cc, ReadBatch &b) {
    if (files_.empty()) files_.push_back("stdin");
    std::vector<uint64_t> file_end;  // record count after each file
    const char *rd = getenv("OGE_READER");
    // the byte-range sharded reader by default only over the host-staged transport, where every multi-rank
    // test ran; over RCCL (an 8-GPU node) it is opt-in (OGE_READER=sharded) until a G > 1 RCCL run of it has
    // been recorded: its rank joins and tail fetch are collectives that a fall-back cannot undo
    const bool want_shards = cc.gpus > 1 && files_.size() == 1 && files_[0] != "stdin" && files_[0] != "-" && sink_takes_shards() &&
                             !(rd && (std::string(rd) == "host" || std::string(rd) == "whole"));
    if (want_shards && cc.init_ranks()) return -1;  // the ranks (and so the transport) are needed here anyway
    const bool rccl = !cc.comms.empty() && cc.comms[0] && std::string(oge_comm_transport(cc.comms[0])) == "rccl";
    if (want_shards && (!rccl || (rd && std::string(rd) == "sharded"))) {
        const int r = read_sharded(cc, b, files_[0]);
        if (r <= 0) return r;  // 1: the host reader reports why the file cannot be read
    }
    if (files_.size() == 1 && files_[0] != "stdin" && files_[0] != "-" && !(rd && std::string(rd) == "host")) {
        const int r = read_device(cc, b, files_[0]);
        if (r <= 0) return r;  // 1: fall through to the host reader (it reports format errors)
    }
    for (size_t i = 0; i < files_.size(); ++i) {
        const std::string path = files_[i] == "stdin" ? "/dev/stdin" : files_[i];
        BamFile f;
        std::string err;
        if (!bam_read_file(path, f, cc.threads > 0 ? cc.threads : 8, err)) {
            fprintf(stderr, "openge: error reading %s: %s\n", files_[i].c_str(), err.c_str());
            return -1;
        }
        if (i == 0) {  // take the decompressed stream as it is: records start at rec_base
            b.header = f.header;
            b.ref_names = f.ref_names;
            const uint64_t base = f.rec_base;
            b.offs.resize(f.offsets.size());
            for (size_t k = 0; k < f.offsets.size(); ++k) b.offs[k] = base + f.offsets[k];
            b.recs = std::move(f.data);
        } else {
            if (f.header.sq.size() != b.header.sq.size() || f.ref_names != b.ref_names)  // read_stream_reader.h:116-124
                fprintf(stderr, "Warning; sequence headers vary between files. Data may be corrupt.\n");
            const uint64_t base = b.recs.size();
            b.recs.insert(b.recs.end(), f.recs(), f.recs() + f.rec_bytes());
            for (uint64_t o : f.offsets) b.offs.push_back(base + o);
        }
        file_end.push_back(b.offs.size());
    }
    b.n = b.offs.size();
    b.offs.push_back(b.recs.size());
    b.recs.resize(b.recs.size() + 16, 0);
    b.host_valid = true;
    if (files_.size() > 1 && !sink_sorts()) return merge_inputs(b, file_end, cc.threads);
    return 0;
}

// True when the records go straight (or through a Filter) into a ReadSorter: the sort then makes
// the MultiReader's interleaving irrelevant (records it would order differently are full ByPosition
// ties, ordered by heap address in the reference).
bool FileReader::sink_sorts() const {
    const AlgorithmModule *m = sink_;
    if (m && dynamic_cast<const Filter *>(m)) m = m->sink();
    return m && dynamic_cast<const ReadSorter *>(m);
}

// Sort::ByPosition (util/bamtools/Sort.h:116-133) down to the flag, as a three-way compare; refID
// -1 sorts last and is equivalent to every other refID -1 record.
static int bypos_cmp(const uint8_t *a, const uint8_t *b) {
    const int32_t ra = oge_rd_i32(a + 4), rb = oge_rd_i32(b + 4);
    if (ra == -1 || rb == -1) return (ra == -1) - (rb == -1);
    if (ra != rb) return ra < rb ? -1 : 1;
    const int32_t pa = oge_rd_i32(a + 8), pb = oge_rd_i32(b + 8);
    if (pa != pb) return pa < pb ? -1 : 1;
    const uint16_t fa = oge_rd_u16(a + 18), fb = oge_rd_u16(b + 18);
    const bool va = fa & 0x10, vb = fb & 0x10;
    if (va != vb) return va ? 1 : -1;
    const int la = a[12] - 1, lb = b[12] - 1;
    const int c = memcmp(a + 36, b + 36, (size_t)std::min(la, lb));
    if (c) return c < 0 ? -1 : 1;
    if (la != lb) return la < lb ? -1 : 1;
    if (fa != fb) return fa < fb ? -1 : 1;
    return 0;
}

// MultiReader::read (util/read_stream_reader.h:132-153): the inputs are interleaved by a
// std::multiset of one head per file ordered by ByPosition, so equivalent heads leave in insertion
// order.  A binary heap keyed on (ByPosition, insertion number) reproduces it exactly, for sorted
// and unsorted inputs alike (the reference's final address tie-break is replaced by insertion
// order, Q10).  The arena is then rewritten in that order.
int FileReader::merge_inputs(ReadBatch &b, const std::vector<uint64_t> &file_end, int threads) {
    struct Head {
        uint64_t rec, end, seq;
    };
    const uint8_t *base = b.recs.data();
    auto later = [&](const Head &x, const Head &y) {  // heap "less": x leaves after y
        const int c = bypos_cmp(base + b.offs[x.rec], base + b.offs[y.rec]);
        return c ? c > 0 : x.seq > y.seq;
    };
    std::vector<Head> heap;
    uint64_t seq = 0, begin = 0;
    for (uint64_t e : file_end) {  // MultiReader::open: one read from each file, in file order
        if (e > begin) heap.push_back({begin, e, seq++});
        begin = e;
    }
    std::make_heap(heap.begin(), heap.end(), later);
    std::vector<uint64_t> order;
    order.reserve(b.n);
    while (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), later);
        Head h = heap.back();
        heap.pop_back();
        order.push_back(h.rec);
        if (++h.rec < h.end) {
            h.seq = seq++;
            heap.push_back(h);
            std::push_heap(heap.begin(), heap.end(), later);
        }
    }
    bytevec out;
    out.resize(b.recs.size());
    std::vector<uint64_t> offs(b.n + 1);
    for (uint64_t k = 0; k < b.n; ++k) offs[k + 1] = offs[k] + (b.offs[order[k] + 1] - b.offs[order[k]]);
    const uint64_t shift = b.offs[0];  // keep the reader's leading bytes (header) where they were
    const int T = std::max(1, threads);
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t)
        ts.emplace_back([&, t]() {
            for (uint64_t k = (uint64_t)t; k < b.n; k += (uint64_t)T)
                memcpy(out.data() + shift + offs[k], base + b.offs[order[k]], offs[k + 1] - offs[k]);
        });
    for (auto &t : ts) t.join();
    memcpy(out.data(), base, shift);
    memset(out.data() + shift + offs[b.n], 0, out.size() - shift - offs[b.n]);
    for (auto &o : offs) o += shift;
    b.recs = std::move(out);
    b.offs = std::move(offs);
    return 0;
}

// ----------------------------------------------------------------------------------- dedup opts
// RG -> library table as MarkDuplicates::getLibraryName resolves it (mark_duplicates.cpp:301-318).
struct MdOpts {
    oge_markdup_opts o;
    std::string ids;
    std::vector<int16_t> libs;
};
static void markdup_opts(const ReadBatch &b, bool compat, int split, MdOpts &m) {
    std::map<std::string, int16_t> lib_ids;
    int16_t next = 1;
    for (auto &rg : b.header.rg) {
        std::string lib = rg.lb.empty() ? std::string("Unknown Library") : rg.lb;
        auto it = lib_ids.find(lib);
        if (it == lib_ids.end()) it = lib_ids.emplace(lib, next++).first;
        m.libs.push_back(it->second);
        m.ids += rg.id;
        m.ids.push_back('\0');
    }
    auto unk = lib_ids.find("Unknown Library");
    m.libs.push_back(0);
    memset(&m.o, 0, sizeof m.o);
    m.o.n_ref = (int32_t)b.ref_names.size();
    m.o.rg_ids = m.ids.c_str();
    m.o.rg_ids_bytes = m.ids.size();
    m.o.rg_lib = m.libs.data();
    m.o.n_rg = (int32_t)b.header.rg.size();
    m.o.unknown_lib = unk != lib_ids.end() ? unk->second : next;
    m.o.compat_nonverbose_index = compat ? 1 : 0;
    m.o.split_chains = split;
}

// ----------------------------------------------------------------------------------- Filter
bool Filter::setReadLengths(const std::string &s) {
    int a = 0, z = 0;
    char junk;
    bool ok;
    if (!s.empty() && s[0] == '+') {
        ok = sscanf(s.c_str(), "%c%d", &junk, &a) == 2;
        z = INT32_MAX;
    } else if (!s.empty() && s[0] == '-') {
        ok = sscanf(s.c_str(), "%c%d", &junk, &z) == 2;
        a = INT32_MIN;
    } else if (s.find('-') != std::string::npos) {
        ok = sscanf(s.c_str(), "%d%c%d", &a, &junk, &z) == 3;
    } else {
        ok = sscanf(s.c_str(), "%d", &a) == 1;
        z = a;
    }
    if (!ok) {  // filter.cpp:179-182
        fprintf(stderr, "Error parsing read length requirements. Aborting.\n"
                        "Valid ranges look like: 64, or 64-72, or -64, or +64.\n");
        exit(-1);
    }
    opts_.min_len = a;
    opts_.max_len = z;
    return true;
}

int Filter::runInternal(ChainContext &cc, ReadBatch &b) {
    oge_filter_opts o = opts_;
    if (has_region_) {
        if (verbose_) fprintf(stderr, "Filtering to region %s\n", region_.c_str());
        std::string names;
        std::vector<int64_t> lens;
        for (auto &sq : b.header.sq) {
            names += sq.name;
            names.push_back('\0');
            lens.push_back(sq.length);
        }
        if (oge_parse_region(region_.c_str(), names.data(), (int32_t)lens.size(), lens.data(), &o)) {
            // filter.cpp:243-247: the parse error, then the generic message, then exit(-1)
            const std::string why = oge_last_error(nullptr);
            if (why.rfind("ERROR: could not parse", 0) != 0) fprintf(stderr, "%s\n", why.c_str());
            fprintf(stderr, "ERROR: could not parse region'%s'\n"
                            "Check that region description is in valid format (see documentation) and that the "
                            "coordinates are valid\n", region_.c_str());
            return -1;
        }
    }
    if (cc.to_device(b)) return -1;
    void *out = nullptr, *out_off = nullptr;
    if (oge_dev_alloc(cc.ctx, b.d_bytes + 64, &out) || oge_dev_alloc(cc.ctx, (b.n + 1) * 8, &out_off))
        return cc.fail("device allocation");
    uint64_t m = 0, bytes = 0;
    int rc = oge_filter_records_dev(cc.ctx, b.d_recs, b.d_offs, b.n, &o, (uint8_t *)out, (uint64_t *)out_off, &m);
    if (!rc) rc = oge_memcpy(cc.ctx, &bytes, (uint64_t *)out_off + m, 8, 2);
    if (!rc) rc = oge_ctx_sync(cc.ctx);
    if (rc) {
        oge_dev_free(cc.ctx, out);
        oge_dev_free(cc.ctx, out_off);
        return cc.fail("Filter");
    }
    cc.free_device(b);
    b.d_recs = (uint8_t *)out;
    b.d_offs = (uint64_t *)out_off;
    b.d_bytes = bytes;
    b.n = m;
    b.dev_valid = true;
    b.host_valid = false;
    kept = m;
    if (verbose_) fprintf(stderr, "%llu alignments processed.\n", (unsigned long long)m);
    return 0;
}

// ----------------------------------------------------------------------------------- ReadSorter
// One GPU, and the chain's records (+ the sort's second arena and workspace) do not fit free HBM,
// or OGE_CHUNK_BYTES forces the chunked path (tests).
static bool use_chunked(ChainContext &cc, const ReadBatch &b) {
    if (cc.gpus > 1) return false;
    if (getenv("OGE_CHUNK_BYTES")) return true;
    if (b.dev_valid) return false;  // the reader already holds them in HBM
    uint64_t fr = 0, tot = 0;
    if (oge_mem_info(cc.ctx, &fr, &tot)) return false;
    return b.bytes() / 10 * 25 + b.n * 100 > fr;
}

int ReadSorter::runInternal(ChainContext &cc, ReadBatch &b) {
    if (order_ != BamHeaderModel::COORDINATE && order_ != BamHeaderModel::QUERYNAME) {
        fprintf(stderr, "openge: unsupported sort order\n");
        return -1;
    }
    MarkDuplicates *md = order_ == BamHeaderModel::COORDINATE ? dynamic_cast<MarkDuplicates *>(sink_) : nullptr;
    if (cc.gpus > 1 && order_ == BamHeaderModel::COORDINATE) {  // --gpus G: range-split sort (+ dedup) over G ranks
        MdOpts m;
        if (md) markdup_opts(b, md->compatNonverbose, md->splitChains, m);
        uint64_t nd = 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (run_ranks(cc, b, true, md ? &m.o : nullptr, &nd)) return -1;
        if (md) md->duplicates = nd;
        b.header.sort_order = order_;
        if (verbose_)
            fprintf(stderr, "[openge] ReadSorter: %d ranks, %.3f s\n", cc.gpus,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        return 0;
    }
    if (order_ == BamHeaderModel::COORDINATE && use_chunked(cc, b)) {
        // larger than HBM: sorted runs spilled into the host arena, key ranges sorted on the device,
        // produced range by range when the writer asks (oge_sort_markdup_chunked)
        if (cc.to_host(b)) return -1;
        cc.free_device(b);
        auto arena = std::make_shared<ReadBatch>();
        arena->recs = std::move(b.recs);
        arena->offs = std::move(b.offs);
        auto mo = std::make_shared<MdOpts>();
        if (md) markdup_opts(b, md->compatNonverbose, md->splitChains, *mo);
        const char *ce = getenv("OGE_CHUNK_BYTES");
        const uint64_t chunk = ce ? strtoull(ce, nullptr, 10) : 0, n = b.n;
        const int32_t n_ref = (int32_t)b.ref_names.size();
        b.produce = [arena, mo, md, chunk, n, n_ref](ChainContext &c, const ReadBatch::RangeSink &sink) -> int {
            struct Tramp {
                const ReadBatch::RangeSink *s;
                static int call(void *u, const uint8_t *r, const uint64_t *o, uint64_t m) { return (*((Tramp *)u)->s)(r, o, m); }
            } tr{&sink};
            uint64_t nd = 0, runs = 0, ranges = 0;
            const int rc = oge_sort_markdup_chunked(c.ctx, arena->recs.data(), arena->offs.data(), n, n_ref, md ? &mo->o : nullptr,
                                                    chunk, &Tramp::call, &tr, &nd, &runs, &ranges);
            if (rc) return c.fail("ReadSorter (chunked)");
            if (md) md->duplicates = nd;
            if (verbose_)
                fprintf(stderr, "[openge] ReadSorter: %llu records in %llu sorted runs, output in %llu key ranges\n",
                        (unsigned long long)n, (unsigned long long)runs, (unsigned long long)ranges);
            return 0;
        };
        b.host_valid = false;
        b.header.sort_order = order_;
        return 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (cc.to_device(b)) return -1;
    const auto t1 = std::chrono::steady_clock::now();
    void *perm = nullptr, *out = nullptr, *out_off = nullptr;
    if (oge_dev_alloc(cc.ctx, b.n * 4 + 4, &perm) || oge_dev_alloc(cc.ctx, b.d_bytes + 64, &out) ||
        oge_dev_alloc(cc.ctx, (b.n + 1) * 8, &out_off))
        return cc.fail("device allocation");
    if (verbose_) oge_ctx_sync(cc.ctx);
    const auto t1a = std::chrono::steady_clock::now();
    int rc;
    if (order_ == BamHeaderModel::QUERYNAME) {  // -b; a MarkDuplicates sink then runs on its own
        rc = oge_sort_name_dev(cc.ctx, b.d_recs, b.d_offs, b.n, (uint32_t *)perm);
        if (!rc) rc = oge_gather_records_dev(cc.ctx, b.d_recs, b.d_offs, (uint32_t *)perm, b.n, (uint8_t *)out, (uint64_t *)out_off);
    } else if (md) {  // mergesort -M: one fused device pipeline (sort, dedup, gather with 0x400 applied)
        MdOpts m;
        markdup_opts(b, md->compatNonverbose, md->splitChains, m);
        uint64_t nd = 0;
        rc = oge_sort_markdup_dev(cc.ctx, b.d_recs, b.d_offs, b.n, &m.o, (uint32_t *)perm, (uint8_t *)out,
                                  (uint64_t *)out_off, &nd);
        md->duplicates = nd;
    } else {
        rc = oge_sort_coord_dev(cc.ctx, b.d_recs, b.d_offs, b.n, (int32_t)b.ref_names.size(), (uint32_t *)perm);
        if (!rc) rc = oge_gather_records_dev(cc.ctx, b.d_recs, b.d_offs, (uint32_t *)perm, b.n, (uint8_t *)out, (uint64_t *)out_off);
    }
    if (!rc) rc = oge_ctx_sync(cc.ctx);
    if (verbose_) {
        fprintf(stderr, "[openge] ReadSorter: host->device %.3f s, output allocation %.3f s, device pipeline %.3f s\n",
                std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t1a - t1).count(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t1a).count());
        std::string st;  // HIP-event stage times of the device pipeline (ms)
        for (const char *s : {"input_pass", "sort_radix", "sort_ties", "meta_gather", "md_matejoin", "md_pairs", "md_frags",
                              "md_apply", "gather_offsets", "gather_records", "name_sort"}) {
            double ms = -1;
            if (!oge_ctx_timing(cc.ctx, s, &ms) && ms >= 0) st += std::string(" ") + s + "=" + std::to_string(ms).substr(0, 6);
        }
        fprintf(stderr, "[openge] ReadSorter stages (ms):%s\n", st.c_str());
    }
    oge_dev_free(cc.ctx, perm);
    if (rc) {
        oge_dev_free(cc.ctx, out);
        oge_dev_free(cc.ctx, out_off);
        return cc.fail("ReadSorter");
    }
    cc.free_device(b);
    b.d_recs = (uint8_t *)out;
    b.d_offs = (uint64_t *)out_off;
    b.dev_valid = true;
    b.host_valid = false;
    b.header.sort_order = order_;  // read_sorter.cpp:257-258
    return 0;
}

// ----------------------------------------------------------------------------------- MarkDuplicates
int MarkDuplicates::runInternal(ChainContext &cc, ReadBatch &b) {
    if (cc.gpus > 1) {  // --gpus G: every rank marks its input range in place order
        if (compatNonverbose) {
            fprintf(stderr, "openge: --compat-nonverbose-dedup is one-GPU only\n");
            return -1;
        }
        MdOpts m;
        markdup_opts(b, false, splitChains, m);
        uint64_t nd = 0;
        if (run_ranks(cc, b, false, &m.o, &nd)) return -1;
        duplicates = nd;
        b.drop_duplicates = removeDuplicates;
        return 0;
    }
    if (cc.to_device(b)) return -1;
    void *dup = nullptr;
    if (oge_dev_alloc(cc.ctx, b.n + 1, &dup)) return cc.fail("device allocation");
    MdOpts m;
    markdup_opts(b, compatNonverbose, splitChains, m);
    uint64_t nd = 0;
    int rc = oge_markdup_dev(cc.ctx, b.d_recs, b.d_offs, b.n, &m.o, (uint8_t *)dup, 1, &nd);
    if (!rc) rc = oge_ctx_sync(cc.ctx);
    oge_dev_free(cc.ctx, dup);
    if (rc) return cc.fail("MarkDuplicates");
    duplicates = nd;
    b.host_valid = false;
    b.drop_duplicates = removeDuplicates;
    return 0;
}

// ----------------------------------------------------------------------------------- LocalRealignment

// --gpus G: one realignment over the whole input whose per-interval device work (consensus
// generation, the offset scan) is spread over the G ranks' devices by interval ranges balanced by reads
// (oge_localrealign_multi) -- cuts fall inside contigs too, so a single-contig input shards; the binning,
// the decisions and the mate-fixing writer run once, on all host threads, so the output is the one-GPU
// output.  (Until r05 each rank realigned a range of whole contigs on its own, and a mate-fixer backlog at a
// shard boundary aborted the run.)
static int realign_ranks(ChainContext &cc, ReadBatch &b, const std::string &ht, const std::string &ref, const std::string &iv,
                         bool verbose) {
    if (cc.init_ranks()) return -1;
    const int G = cc.gpus;
    oge_realign_opts o;
    oge_realign_opts_init(&o);
    o.threads = cc.threads;
    oge_realign_result *r = nullptr;
    if (oge_localrealign_multi(cc.rank_ctx.data(), G, ht.data(), ht.size(), b.recs.data(), b.offs.data(), b.n, ref.c_str(), iv.c_str(),
                               &o, &r))
        return cc.fail("LocalRealignment");
    if (verbose) fprintf(stderr, "[openge] LocalRealignment over %d devices: %s\n", G, oge_realign_result_stats(r));
    const uint64_t m = oge_realign_result_count(r);
    oge_realign_result_take(r, b.recs, b.offs);  // the records and offsets, moved (offsets from 0, 16 bytes of slack)
    oge_realign_result_free(r);
    if (b.offs.size() != m + 1) b.offs.assign(m + 1, 0);
    b.n = m;
    return 0;
}

int LocalRealignment::runInternal(ChainContext &cc, ReadBatch &b) {
    const auto t0 = std::chrono::steady_clock::now();
    if (cc.to_host(b)) return -1;
    cc.free_device(b);
    const std::string ht = b.header.to_string();
    if (cc.gpus > 1) return realign_ranks(cc, b, ht, reference_, intervals_, verbose);
    oge_realign_opts o;
    oge_realign_opts_init(&o);
    o.threads = cc.threads;
    oge_realign_result *r = nullptr;
    const auto t1 = std::chrono::steady_clock::now();
    if (oge_localrealign(cc.ctx, ht.data(), ht.size(), b.recs.data(), b.offs.data(), b.n, reference_.c_str(),
                         intervals_.c_str(), &o, &r))
        return cc.fail("LocalRealignment");
    const auto t2 = std::chrono::steady_clock::now();
    uint64_t bytes = 0;
    const uint8_t *rp = oge_realign_result_records(r, &bytes);
    const uint64_t *op = oge_realign_result_offsets(r);
    const uint64_t n = oge_realign_result_count(r);
    // OGE_WRITE_DEVICE=1: the result goes straight up to the device when it fits and the writer deflates it
    // there (a host module downloads it again).  Otherwise (default) the host batch takes it in a threaded
    // copy into huge pages -- one thread copying into fresh 4 KiB pages took 0.52 s for the 1.1 GB C5 result
    // -- and the writer compresses it with the host codec (zlib-class level 6, as the reference writes).
    uint64_t fr = 0, tot = 0;
    const uint64_t base = n ? op[0] : 0, len = n ? op[n] - base : 0;
    void *dr = nullptr, *dof = nullptr;
    bool up = n && write_device_forced() && !bgzf_host_codec_forced() && !oge_mem_info(cc.ctx, &fr, &tot) &&
              2 * len + (n + 1) * 16 + (256ull << 20) < fr;
    if (up) {
        std::vector<uint64_t> ro(op, op + n + 1);
        for (auto &x : ro) x -= base;
        up = !oge_dev_alloc(cc.ctx, len + 64, &dr) && !oge_dev_alloc(cc.ctx, (n + 1) * 8, &dof) &&
             !oge_memcpy(cc.ctx, dr, rp + base, len, 1) && !oge_memcpy(cc.ctx, dof, ro.data(), (n + 1) * 8, 1);
        if (up) {
            b.recs.clear();
            b.recs.shrink_to_fit();
            b.offs.clear();
            b.offs.shrink_to_fit();
            b.d_recs = (uint8_t *)dr;
            b.d_offs = (uint64_t *)dof;
            b.d_bytes = len;
            b.dev_valid = true;
            b.host_valid = false;
        } else {
            if (dr) oge_dev_free(cc.ctx, dr);
            if (dof) oge_dev_free(cc.ctx, dof);
        }
    }
    if (verbose) fprintf(stderr, "[openge] LocalRealignment: %s\n", oge_realign_result_stats(r));
    if (!up) {
        // the host batch takes the result's own buffers (r06: no copy; r05 copied the 1.1 GB C5 result into
        // fresh huge pages on 16 threads, 0.06 s, and unmapped the library's copy, another 0.06 s)
        oge_realign_result_take(r, b.recs, b.offs);  // (the input's host copy is unmapped here: a background unmap
                                                     // measured slower, its mm lock stalling the writer's threads)
        if (b.offs.size() != n + 1) b.offs.assign(n + 1, 0);
    }
    (void)rp;
    b.n = n;
    const auto t3 = std::chrono::steady_clock::now();
    oge_realign_result_free(r);
    if (verbose) {
        auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
            return std::chrono::duration<double>(z - a).count();
        };
        fprintf(stderr, "[openge] LocalRealignment: records to host %.3f s, realign %.3f s, result %s %.3f s, release %.3f s\n",
                sec(t0, t1), sec(t1, t2), up ? "to the device" : "host copy", sec(t2, t3), sec(t3, std::chrono::steady_clock::now()));
    }
    return 0;
}

// ----------------------------------------------------------------------------------- FileWriter
int FileWriter::setFormat(const std::string &f) {
    if (f == "bam" || f == "BAM") return 0;
    fprintf(stderr, "openge: output format %s is not provided (BAM only)\n", f.c_str());
    return -1;
}

// the bin every record must carry (bam_serializer.h:112-116), recomputed in place by the workers
static void fix_bins(ReadBatch &b, int threads) {
    const uint64_t n = b.n, chunk = 1 << 16;
    const uint64_t nc = (n + chunk - 1) / chunk;
    std::atomic<uint64_t> next(0);
    std::vector<std::thread> ts;
    for (int t = 0; t < std::max(1, threads); ++t)
        ts.emplace_back([&]() {
            for (uint64_t c; (c = next.fetch_add(1)) < nc;)
                for (uint64_t k = c * chunk, e = std::min(n, k + chunk); k < e; ++k) {
                    uint8_t *r = b.recs.data() + b.offs[k];
                    oge_wr_u16(r + OGE_OFF_BIN, oge_rec_bin(r));
                }
        });
    for (auto &t : ts) t.join();
}

// Device-resident records: drop duplicates (-r/-R), recompute bins and BGZF-compress on the GPU;
// only the compressed stream crosses PCIe.  The records of a batch are back to back in its arena
// (the reader's stream, a gather's output), so the stream is the byte range [off[0], off[n]).
// Device-resident records -> BGZF file.  Bins are recomputed on the device, then the stream is
// deflated in segments of kSeg bytes (a multiple of the 65,280-byte block payload, so the blocks are
// exactly those of one whole-stream deflate); each segment's compressed bytes come down into one of
// two page-locked buffers and are written by a background thread while the next segment is
// deflated and copied.  Timings: device deflate, device->host, and time spent waiting for the disk.
int FileWriter::write_device(ChainContext &cc, ReadBatch &b, BgzfWriter &w, double *t_dev, double *t_d2h, double *t_wait) {
    auto clk = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
        return std::chrono::duration<double>(z - a).count();
    };
    *t_dev = *t_d2h = *t_wait = 0;
    if (const char *f = getenv("OGE_TEST_FAIL"); f && !strcmp(f, "write_device")) {  // test hook: a failed device write
        fprintf(stderr, "openge: FileWriter: injected failure (OGE_TEST_FAIL=write_device)\n");
        return -1;
    }
    uint8_t *recs = b.d_recs;
    uint64_t *offs = b.d_offs;
    uint64_t n = b.n;
    void *kept = nullptr, *kept_off = nullptr, *dz = nullptr, *hz[2] = {nullptr, nullptr};
    std::thread wr;
    auto release = [&]() {
        if (wr.joinable()) wr.join();
        if (kept) oge_dev_free(cc.ctx, kept);
        if (kept_off) oge_dev_free(cc.ctx, kept_off);
        if (dz) oge_dev_free(cc.ctx, dz);
        for (void *h : hz)
            if (h) oge_host_free(cc.ctx, h);
    };
    auto t = clk();
    if (b.drop_duplicates && n) {
        if (oge_dev_alloc(cc.ctx, b.d_bytes + 64, &kept) || oge_dev_alloc(cc.ctx, (n + 1) * 8, &kept_off)) {
            release();
            return cc.fail("device allocation");
        }
        uint64_t m = 0;
        if (oge_drop_flagged_dev(cc.ctx, recs, offs, n, OGE_F_DUP, (uint8_t *)kept, (uint64_t *)kept_off, &m)) {
            release();
            return cc.fail("FileWriter: drop duplicates");
        }
        recs = (uint8_t *)kept;
        offs = (uint64_t *)kept_off;
        n = m;
    }
    uint64_t ends[2] = {0, 0};
    if (n && (oge_fix_bins_dev(cc.ctx, recs, offs, n) || oge_memcpy(cc.ctx, &ends[0], offs, 8, 2) ||
              oge_memcpy(cc.ctx, &ends[1], offs + n, 8, 2))) {
        release();
        return cc.fail("FileWriter: bins");
    }
    *t_dev += sec(t, clk());
    const uint64_t len = ends[1] - ends[0];
    // segments of 1024-32768 payloads (67 MB - 2.14 GB of records), about an eighth of the stream: the
    // page-locked download buffers are sized by the segment and pinning / unpinning them costs ~0.25 s per
    // GB (a 1.1 GB realign output: 0.5 s in 2.1 GB segments, 0.04 s in 67 MB ones), while a large file keeps
    // full-size deflate calls.  OGE_WRITE_SEG_BLOCKS fixes the payloads per segment (tests).
    const char *se = getenv("OGE_WRITE_SEG_BLOCKS");
    const uint64_t want = se ? std::max(1ul, strtoul(se, nullptr, 10)) : std::min<uint64_t>(32768, std::max<uint64_t>(1024, len / 8 / 65280 + 1));
    const uint64_t kSeg = 65280ull * want;
    const uint64_t seg = std::min(len, kSeg);
    const uint64_t cap = oge_bgzf_bound(seg);
    t = clk();
    if (len && (oge_dev_alloc(cc.ctx, cap, &dz) || oge_host_alloc(cc.ctx, cap, &hz[0]) ||
                (len > seg && oge_host_alloc(cc.ctx, cap, &hz[1])))) {
        release();
        return cc.fail("FileWriter: buffers");
    }
    if (getenv("OGE_WRITE_TRACE")) fprintf(stderr, "[openge] FileWriter: buffers %.3f s\n", sec(t, clk()));
    w.write_compressed(nullptr, 0);  // flush the header as blocks of its own
    int k = 0;
    for (uint64_t s0 = 0; s0 < len; s0 += seg, k ^= 1) {
        const uint64_t sl = std::min(seg, len - s0);
        uint64_t zb = 0;
        t = clk();
        if (oge_bgzf_deflate_dev(cc.ctx, recs + ends[0] + s0, sl, std::max(0, std::min(9, level_)), (uint8_t *)dz, cap, &zb) ||
            oge_ctx_sync(cc.ctx)) {
            release();
            return cc.fail("FileWriter: BGZF on the device");
        }
        *t_dev += sec(t, clk());
        t = clk();
        if (wr.joinable()) wr.join();  // the buffer written two segments ago is free again
        *t_wait += sec(t, clk());
        t = clk();
        if (zb && oge_memcpy(cc.ctx, hz[k], dz, zb, 2)) {
            release();
            return cc.fail("device->host copy");
        }
        *t_d2h += sec(t, clk());
        const uint8_t *hp = (const uint8_t *)hz[k];
        wr = std::thread([&w, hp, zb]() { w.write_compressed(hp, zb); });
    }
    t = clk();
    if (wr.joinable()) wr.join();
    *t_wait += sec(t, clk());
    t = clk();
    release();
    if (getenv("OGE_WRITE_TRACE")) fprintf(stderr, "[openge] FileWriter: release %.3f s\n", sec(t, clk()));
    return 0;
}

// --gpus G: every rank drops its duplicates (-r / -R) and BGZF-compresses its own slice on its own
// GPU, concurrently; the compressed slices go to the file in rank order (a slice's last block may be
// short, the decompressed stream is the one-GPU stream).
int FileWriter::write_slices(ChainContext &cc, ReadBatch &b, BgzfWriter &w) {
    const int G = (int)b.slices.size();
    struct Out {
        void *host = nullptr;
        uint64_t zb = 0;
        int rc = 0;
        std::string why;
    };
    std::vector<Out> outs(G);
    const int level = std::max(0, std::min(9, level_));
    const bool drop = b.drop_duplicates;
    std::vector<std::thread> ts;
    for (int g = 0; g < G; ++g)
        ts.emplace_back([&, g]() {
            const ReadBatch::Slice &s = b.slices[g];
            Out &o = outs[g];
            oge_ctx *c = s.ctx;
            uint8_t *recs = s.d_recs;
            uint64_t *offs = s.d_offs, n = s.n;
            void *kept = nullptr, *kept_off = nullptr, *dz = nullptr;
            int rc = 0;
            if (drop && n) {
                rc = oge_dev_alloc(c, (n + 1) * 8, &kept_off);
                uint64_t e = 0, m = 0;
                if (!rc) rc = oge_memcpy(c, &e, offs + n, 8, 2);
                if (!rc) rc = oge_dev_alloc(c, e + 64, &kept);
                if (!rc) rc = oge_drop_flagged_dev(c, recs, offs, n, OGE_F_DUP, (uint8_t *)kept, (uint64_t *)kept_off, &m);
                recs = (uint8_t *)kept;
                offs = (uint64_t *)kept_off;
                n = m;
            }
            uint64_t ends[2] = {0, 0};
            if (!rc && n) rc = oge_memcpy(c, &ends[0], offs, 8, 2) || oge_memcpy(c, &ends[1], offs + n, 8, 2);
            const uint64_t len = ends[1] - ends[0], cap = oge_bgzf_bound(len);
            if (!rc && len) rc = oge_dev_alloc(c, cap, &dz);
            if (!rc && len) rc = oge_bgzf_deflate_dev(c, recs + ends[0], len, level, (uint8_t *)dz, cap, &o.zb);
            if (!rc && o.zb) rc = oge_host_alloc(c, o.zb, &o.host);
            if (!rc && o.zb) rc = oge_memcpy(c, o.host, dz, o.zb, 2);
            if (rc) o.why = oge_last_error(c);
            o.rc = rc;
            for (void *p : {kept, kept_off, dz})
                if (p) oge_dev_free(c, p);
        });
    w.write_compressed(nullptr, 0);  // the header's blocks first
    int ret = 0;
    for (int g = 0; g < G; ++g) {
        ts[g].join();
        if (outs[g].rc) {
            fprintf(stderr, "openge: FileWriter: rank %d: %s\n", g, outs[g].why.c_str());
            ret = -1;
        } else if (!ret && outs[g].zb) {
            w.write_compressed((const uint8_t *)outs[g].host, outs[g].zb);
        }
        if (outs[g].host) oge_host_free(b.slices[g].ctx, outs[g].host);
    }
    return ret;
}

// Inputs larger than HBM: every output range the sorter produces is (with -r / -R) compacted, BGZF
// compressed on the device and written before the next range is made.
int FileWriter::write_ranges(ChainContext &cc, ReadBatch &b, BgzfWriter &w) {
    w.write_compressed(nullptr, 0);  // the header's blocks first
    const int level = std::max(0, std::min(9, level_));
    const bool drop = b.drop_duplicates;
    struct Buf {
        oge_ctx *c;
        void *p = nullptr;
        uint64_t cap = 0;
        bool host = false;
        int need(uint64_t bytes) {
            if (bytes <= cap) return 0;
            if (p) host ? oge_host_free(c, p) : oge_dev_free(c, p);
            p = nullptr;
            cap = 0;
            const int rc = host ? oge_host_alloc(c, bytes, &p) : oge_dev_alloc(c, bytes, &p);
            if (!rc) cap = bytes;
            return rc;
        }
        ~Buf() {
            if (p) host ? oge_host_free(c, p) : oge_dev_free(c, p);
        }
    } kept{cc.ctx}, kept_off{cc.ctx}, dz{cc.ctx}, hz{cc.ctx};
    hz.host = true;
    auto sink = [&](const uint8_t *recs, const uint64_t *offs, uint64_t n) -> int {
        uint64_t ends[2] = {0, 0};
        if (n && (oge_memcpy(cc.ctx, &ends[0], offs, 8, 2) || oge_memcpy(cc.ctx, &ends[1], offs + n, 8, 2))) return -1;
        if (drop && n) {
            uint64_t m = 0;
            if (kept.need(ends[1] + 64) || kept_off.need((n + 1) * 8) ||
                oge_drop_flagged_dev(cc.ctx, recs, offs, n, OGE_F_DUP, (uint8_t *)kept.p, (uint64_t *)kept_off.p, &m))
                return -1;
            recs = (const uint8_t *)kept.p;
            offs = (const uint64_t *)kept_off.p;
            n = m;
            ends[0] = ends[1] = 0;
            if (n && (oge_memcpy(cc.ctx, &ends[0], offs, 8, 2) || oge_memcpy(cc.ctx, &ends[1], offs + n, 8, 2))) return -1;
        }
        const uint64_t len = ends[1] - ends[0];
        if (!len) return 0;
        const uint64_t cap = oge_bgzf_bound(len);
        uint64_t zb = 0;
        if (dz.need(cap) || oge_bgzf_deflate_dev(cc.ctx, recs + ends[0], len, level, (uint8_t *)dz.p, cap, &zb) || hz.need(zb) ||
            oge_memcpy(cc.ctx, hz.p, dz.p, zb, 2))
            return -1;
        w.write_compressed((const uint8_t *)hz.p, zb);
        return 0;
    };
    if (b.produce(cc, sink)) return -1;
    return 0;
}

int FileWriter::runInternal(ChainContext &cc, ReadBatch &b) {
    auto clk = [] { return std::chrono::steady_clock::now(); };
    auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
        return std::chrono::duration<double>(z - a).count();
    };
    const auto t0 = clk();
    const bool sliced = !b.slices.empty(), produced = (bool)b.produce;
    bool on_device = sliced || produced || (b.dev_valid && !b.host_valid && !bgzf_host_codec_forced());
    double t_dev = 0, t_d2h = 0, t_wait = 0;
    // OGE_WRITE_DEVICE=1: host records (the realigner's output) whose bytes sit back to back go up to the
    // device and out through the GPU deflate -- on the C5 set 1.1 GB of records take 0.78 s with 16
    // libdeflate threads (profiles/r05ap_realign_cli.txt), the upload and the device path a fraction of that,
    // for an 11 % larger file (the GPU deflate's greedy search).  Off by default: the host codec writes
    // zlib-class level 6 like the reference.  A device that cannot hold them leaves the host writer in charge.
    if (!on_device && b.host_valid && !b.dev_valid && b.n && write_device_forced() && !bgzf_host_codec_forced()) {
        bool contiguous = b.offs.size() == b.n + 1 && b.offs[b.n] + 16 <= b.recs.size();
        for (uint64_t k = 0; contiguous && k < b.n; ++k)
            contiguous = b.offs[k + 1] == b.offs[k] + 4 + oge_rd_u32(b.recs.data() + b.offs[k]);
        uint64_t fr = 0, tot = 0;
        const uint64_t bytes = contiguous ? b.offs[b.n] : 0;
        if (contiguous && !oge_mem_info(cc.ctx, &fr, &tot) && bytes + oge_bgzf_bound(std::min<uint64_t>(bytes, 65280ull * 32768)) +
                                                                      (b.n + 1) * 8 + (256ull << 20) < fr) {
            if (cc.to_device(b)) return -1;
            on_device = true;
            b.host_valid = false;  // write_device reads the device copy
        }
    }
    if (!on_device && cc.to_host(b)) return -1;
    const auto t1 = clk();
    if (!on_device) fix_bins(b, cc.threads);
    const auto t2 = clk();
    BamHeaderModel h = b.header;
    if (!program_line_.empty()) add_program_record(h, program_line_);  // file_writer.cpp:76-89
    FILE *f = filename_ == "stdout" || filename_ == "-" ? stdout : fopen(filename_.c_str(), "wb");
    if (!f) {
        fprintf(stderr, "Error opening BAM file to write.\n");
        return -1;
    }
    bool write_ok = true;
    {
        BgzfWriter w(f, level_, cc.threads > 0 ? cc.threads : 8);
        std::vector<uint8_t> hb = bam_encode_header(h);
        w.write(hb.data(), hb.size());
        if (on_device) {
            if (produced ? write_ranges(cc, b, w) : sliced ? write_slices(cc, b, w) : write_device(cc, b, w, &t_dev, &t_d2h, &t_wait)) {
                w.abandon();  // no EOF block and no write into the FILE closed below
                if (f != stdout) fclose(f);
                return -1;
            }
            w.close();
        }
        // maximal runs of records that sit back to back in memory go out as spans (no copy)
        uint64_t k = 0;
        while (!on_device && k < b.n) {
            const uint8_t *r = b.recs.data() + b.offs[k];
            if (b.drop_duplicates && (oge_rd_u16(r + OGE_OFF_FLAG) & OGE_F_DUP)) {
                ++k;
                continue;
            }
            const uint64_t s = b.offs[k];
            uint64_t e = s + 4 + oge_rd_u32(r);
            ++k;
            while (k < b.n && b.offs[k] == e) {
                const uint8_t *q = b.recs.data() + e;
                if (b.drop_duplicates && (oge_rd_u16(q + OGE_OFF_FLAG) & OGE_F_DUP)) break;
                e += 4 + oge_rd_u32(q);
                ++k;
            }
            w.write_span(b.recs.data() + s, e - s);
        }
        w.close();
        write_ok = w.ok();
    }
    if (f != stdout ? fclose(f) != 0 : fflush(f) != 0) write_ok = false;
    if (!write_ok) {  // a full disk or a closed pipe must not look like success
        fprintf(stderr, "openge: error writing %s: %s\n", filename_.c_str(), strerror(errno));
        return -1;
    }
    if (verbose_ && on_device)
        fprintf(stderr, "[openge] FileWriter: device bins + BGZF %.3f s (gpu, segmented), device->host %.3f s, waiting on the disk %.3f s, "
                "total %.3f s\n", t_dev, t_d2h, t_wait, sec(t2, clk()));
    else if (verbose_)
        fprintf(stderr, "[openge] FileWriter: device->host %.3f s, bins %.3f s, BGZF %.3f s (%s)\n", sec(t0, t1), sec(t1, t2),
                sec(t2, clk()), bgzf_codec_name());
    else fflush(stdout);
    return 0;
}

}  // namespace oge
