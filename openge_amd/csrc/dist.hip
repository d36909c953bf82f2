// dist.hip -- sort + duplicate marking over G GPUs (one rank per GPU), the MI355X replacement of the
// reference's split-by-chromosome parallelism (alg/split_by_chromosome.cpp:30-58 routes refID % K to
// K MarkDuplicates chains, alg/sorted_merge.cpp:66-101 re-merges them; driven from
// cmd/command_mergesort.cpp:118-179 and cmd/command_dedup.cpp:70-113).  The result equals the one-GPU
// `mergesort [-M] --nosplit` result record for record, for any G and any input split.
//
// Each rank enters with any shard of the input (contiguous input ranges in rank order keep the
// reference's input-order tie-break); the collectives go through an OgeTransport: RCCL over xGMI
// between processes or GPUs, or the in-process hub (dist_local.h) between contexts of one process.
//
//  1 range split   packed ByPosition keys (refID', pos, strand) of every record, kSamples per rank
//                  pooled into G-1 splitters (dist_plan.h); record -> owner of its key
//  2 exchange      records (stable by input order within each source), sizes; local sort of the
//                  received records = this rank's slice of the global order (ties share a key, so
//                  name/flag tie order is decided on one rank)
//  3 dedup         ReadEnds of the sorted slice (records.hip input pass), global index = padded
//                  (rank * stride + sorted position), monotone in the global sorted position:
//     fragments    routed by the owner of their 5' (refID, coord): a fragment group (equal lib,
//                  r1Seq, r1Coord, orient) lands on one rank, nearly always its own
//     mate join    every candidate end (paired, mate mapped: mark_duplicates.cpp:205-245) goes to
//                  hash(RG:name)'s rank with a minimal record (name + RG tag) for exact key compares;
//                  arrival order = global index order, so the ReadEndsMap pairs consecutive ends of a
//                  name exactly as on one GPU, for any number of primaries per name (0x800 included)
//     pair groups  completed pair ReadEnds go to the rank of a hash of their chunk key
//     reduce       dup marks, written at padded global indices, meet in a max reduce-scatter
//  4 gather        the slice written once with bin recomputed and 0x400 applied
#include "oge_ctx.h"
#include "bam_layout.h"
#include "dev_util.h"
#include "dist_local.h"
#include "dist_plan.h"
#include "dist_shm.h"
#include "markdup_stages.h"
#include "records.h"
#include "rec_parse.h"
#include "minirec.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

int oge_markdup_prepare(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, const char *name, RecMeta **meta,
                        OgeRgTable *rg);
int oge_sort_buffers(oge_ctx *ctx, uint64_t n, uint64_t **keys, uint32_t **vals);
unsigned int *oge_sort_counts(oge_ctx *ctx);
int oge_sort_keys_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                      bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out);

// ----------------------------------------------------------------------------------------- transport
struct OgeTransport {
    int rank = 0, size = 1;
    virtual ~OgeTransport() {}
    virtual const char *name() const = 0;
    // device buffers, stream-ordered on ctx->stream: complete on return (host-driven transports) or queued on
    // it (RCCL, r06) -- callers consume the results on ctx->stream or after synchronizing it
    virtual int alltoallv(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                          const uint64_t *rbytes, const uint64_t *roff) = 0;
    virtual int allgather_host(oge_ctx *ctx, const void *in, void *out, size_t bytes) = 0;
    virtual int reduce_scatter_max_u8(oge_ctx *ctx, const uint8_t *in, uint8_t *out, size_t chunk) = 0;
    // The peers' parts of an all-to-all (the caller moves its own part), ordered after everything already on
    // stream st.  On return the exchange is either complete (host-driven transports: their copies run on st
    // while ctx->stream keeps executing what was queued on it -- the overlap) or queued on st (RCCL); the
    // caller makes ctx->stream wait for st.  Default: the blocking all-to-all on ctx->stream (no overlap).
    virtual int alltoallv_peers(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                                const uint64_t *rbytes, const uint64_t *roff, hipStream_t st) {
        (void)st;
        return alltoallv(ctx, send, sbytes, soff, recv, rbytes, roff);
    }
    // whether alltoallv_peers really runs beside the context stream (the default above does not)
    virtual bool overlaps() const { return false; }
    // how allgather_host moves its bytes (the `mode` of its tags in the exchange stats)
    virtual const char *gather_mode() const { return "host_memory"; }
};

// One exchange site of a step: bytes this rank sent to / received from other ranks (and kept), and the
// host wall time of its collectives (a transport call returns when its data is complete on this rank, so
// the time includes waiting for the slowest peer).  `calls` collectives were made under the tag.
struct OgeXchg {
    std::string tag;
    uint64_t sent = 0, recv = 0, self = 0, calls = 0;
    double ms = 0;
    double dev_ms = 0;  // RCCL: the collectives' own time on their stream (HIP events; waiting for peers included)
    // "blocking": ms covers the data movement; "side_stream": the peers' parts moved on a side stream beside
    // the caller's own work (host transport: ms covers the staged copies, which ran beside it; RCCL: ms is
    // the time to queue them)
    const char *mode = "blocking";
};

struct oge_comm {
    oge_ctx *ctx = nullptr;
    std::unique_ptr<OgeTransport> tr;
    std::vector<OgeXchg> stats;  // since the last oge_sort_markdup_dist / oge_mergesort_bgzf_dist call
    // RCCL collectives are stream-ordered and not waited for (r06): their time per tag comes
    // from event pairs around them, read when the stats are (stats index, start, stop)
    struct Ev {
        size_t i;
        hipEvent_t a, b;
    };
    mutable std::vector<Ev> pend;
    ~oge_comm() { drop_events(); }
    bool rccl() const { return tr && strcmp(tr->name(), "rccl") == 0; }
    void drop_events() const {
        for (auto &e : pend) (void)hipEventDestroy(e.a), (void)hipEventDestroy(e.b);
        pend.clear();
    }
    void settle_events() const {  // the pending pairs' times into their stats (waits for the collectives)
        for (auto &e : pend) {
            float t = 0;
            if (hipEventSynchronize(e.b) == hipSuccess && hipEventElapsedTime(&t, e.a, e.b) == hipSuccess && e.i < stats.size())
                const_cast<OgeXchg &>(stats[e.i]).dev_ms += t;
        }
        drop_events();
    }
    void clear_stats() {
        drop_events();
        stats.clear();
    }
    // an event pair around a collective queued on `st` (RCCL only; null otherwise)
    struct Bracket {
        const oge_comm *c;
        hipStream_t st;
        hipEvent_t a = nullptr, b = nullptr;
        Bracket(const oge_comm *c_, hipStream_t s) : c(c_), st(s) {
            if (!c->rccl()) return;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess || hipEventRecord(a, st) != hipSuccess) {
                if (a) (void)hipEventDestroy(a);
                if (b) (void)hipEventDestroy(b);
                a = b = nullptr;
            }
        }
        void done(size_t i) {
            if (!a) return;
            if (hipEventRecord(b, st) == hipSuccess) c->pend.push_back({i, a, b});
            else (void)hipEventDestroy(a), (void)hipEventDestroy(b);
            a = b = nullptr;
        }
        ~Bracket() {
            if (a) (void)hipEventDestroy(a), (void)hipEventDestroy(b);
        }
    };
    size_t stat_index(const OgeXchg &x) const { return (size_t)(&x - stats.data()); }
    OgeXchg &stat(const char *tag) {
        for (auto &x : stats)
            if (x.tag == tag) return x;
        stats.push_back(OgeXchg());
        stats.back().tag = tag;
        return stats.back();
    }
    // the collectives, recorded per tag
    int alltoallv(const char *tag, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                  const uint64_t *rbytes, const uint64_t *roff) {
        const auto t0 = std::chrono::steady_clock::now();
        Bracket br(this, ctx->stream);
        const int rc = tr->alltoallv(ctx, send, sbytes, soff, recv, rbytes, roff);
        OgeXchg &x = stat(tag);
        br.done(stat_index(x));
        x.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        x.calls++;
        for (int p = 0; p < tr->size; ++p) {
            if (p == tr->rank) {
                x.self += sbytes[p];
            } else {
                x.sent += sbytes[p];
                x.recv += rbytes[p];
            }
        }
        return rc;
    }
    // the peers' parts only (sbytes / rbytes of this rank's own part are ignored), see OgeTransport
    int alltoallv_peers(const char *tag, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                        const uint64_t *rbytes, const uint64_t *roff, hipStream_t st) {
        std::vector<uint64_t> sb(sbytes, sbytes + tr->size), rb(rbytes, rbytes + tr->size);
        sb[tr->rank] = rb[tr->rank] = 0;
        const auto t0 = std::chrono::steady_clock::now();
        Bracket br(this, st);
        const int rc = tr->alltoallv_peers(ctx, send, sb.data(), soff, recv, rb.data(), roff, st);
        OgeXchg &x = stat(tag);
        br.done(stat_index(x));
        x.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        x.calls++;
        x.mode = tr->overlaps() ? "side_stream" : "blocking";
        x.self += sbytes[tr->rank];
        for (int p = 0; p < tr->size; ++p) x.sent += sb[p], x.recv += rb[p];
        return rc;
    }
    int allgather_host(const char *tag, const void *in, void *out, size_t bytes) {
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = tr->allgather_host(ctx, in, out, bytes);
        OgeXchg &x = stat(tag);
        x.mode = tr->gather_mode();
        x.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        x.calls++;
        x.sent += bytes * (tr->size - 1);
        x.recv += bytes * (tr->size - 1);
        x.self += bytes;
        return rc;
    }
    int reduce_scatter_max_u8(const char *tag, const uint8_t *in, uint8_t *out, size_t chunk) {
        const auto t0 = std::chrono::steady_clock::now();
        Bracket br(this, ctx->stream);
        const int rc = tr->reduce_scatter_max_u8(ctx, in, out, chunk);
        OgeXchg &x = stat(tag);
        br.done(stat_index(x));
        x.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        x.calls++;
        x.sent += chunk * (tr->size - 1);
        x.recv += chunk * (tr->size - 1);
        x.self += chunk;
        return rc;
    }
};

namespace {

constexpr int kT = 256;

int dist_hip_fail(oge_ctx *ctx, int line) {
    const hipError_t e = hipGetLastError();
    return oge_fail(ctx, OGE_ERR_HIP, ("dist.hip:" + std::to_string(line) + ": " + hipGetErrorString(e)).c_str());
}

__global__ __launch_bounds__(kT) void k_max_into(uint8_t *__restrict__ acc, const uint8_t *__restrict__ src, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kT) acc[i] = max(acc[i], src[i]);
}

// the in-process hub's memory operations on HBM
struct HipOps {
    oge_ctx *ctx;
    int copy(void *dst, const void *src, size_t n) {
        return hipMemcpyAsync(dst, src, n, hipMemcpyDefault, ctx->stream) == hipSuccess ? 0 : -1;
    }
    int sync() { return hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : -1; }
    int max_into(uint8_t *acc, const uint8_t *src, size_t n) {  // src may live on another GPU: stage it
        uint8_t *tmp = (uint8_t *)ctx->ws("comm_max_tmp", n);
        if (!tmp || copy(tmp, src, n)) return -1;
        hipLaunchKernelGGL(k_max_into, dim3(std::min<uint32_t>(oge_ceil_div(n, kT), 4096u)), dim3(kT), 0, ctx->stream, acc,
                           (const uint8_t *)tmp, (uint64_t)n);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
};

struct LocalTransport : OgeTransport {
    std::shared_ptr<oge_dist::Hub> hub;
    const char *name() const override { return "local"; }
    int alltoallv(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
                  const uint64_t *roff) override {
        HipOps ops{ctx};
        oge_dist::LocalColl<HipOps> c{*hub, rank, ops};
        return c.alltoallv(send, sbytes, soff, recv, rbytes, roff) ? oge_fail(ctx, OGE_ERR_HIP, "local transport: all-to-all failed")
                                                                   : OGE_OK;
    }
    int allgather_host(oge_ctx *ctx, const void *in, void *out, size_t bytes) override {
        HipOps ops{ctx};
        oge_dist::LocalColl<HipOps> c{*hub, rank, ops};
        return c.allgather_host(in, out, bytes);
    }
    int reduce_scatter_max_u8(oge_ctx *ctx, const uint8_t *in, uint8_t *out, size_t chunk) override {
        HipOps ops{ctx};
        oge_dist::LocalColl<HipOps> c{*hub, rank, ops};
        return c.reduce_scatter_max_u8(in, out, chunk) ? oge_fail(ctx, OGE_ERR_HIP, "local transport: reduce-scatter failed")
                                                       : OGE_OK;
    }
};

// the host-staged transport's memory operations (dist_shm.h), on the context stream
struct StageOps {
    oge_ctx *ctx;
    hipStream_t st = nullptr;  // null: the context stream
    hipStream_t s() const { return st ? st : ctx->stream; }
    int d2h(void *h, const void *d, size_t n) { return hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s()) == hipSuccess ? 0 : -1; }
    int h2d(void *d, const void *h, size_t n) { return hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s()) == hipSuccess ? 0 : -1; }
    int d2d(void *d, const void *s_, size_t n) { return hipMemcpyAsync(d, s_, n, hipMemcpyDeviceToDevice, s()) == hipSuccess ? 0 : -1; }
    int sync() { return hipStreamSynchronize(s()) == hipSuccess ? 0 : -1; }
};

struct ShmTransport : OgeTransport {
    std::unique_ptr<oge_dist::ShmSeg> seg;
    const char *name() const override { return "host"; }
    int alltoallv(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
                  const uint64_t *roff) override {
        return a2a_on(ctx, send, sbytes, soff, recv, rbytes, roff, nullptr);
    }
    int alltoallv_peers(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                        const uint64_t *rbytes, const uint64_t *roff, hipStream_t st) override {
        return a2a_on(ctx, send, sbytes, soff, recv, rbytes, roff, st);  // staged copies on st
    }
    bool overlaps() const override { return true; }
    int a2a_on(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
               const uint64_t *roff, hipStream_t st) {
        StageOps ops{ctx, st};
        oge_dist::ShmColl<StageOps> c{*seg, ops};
        const int rc = c.alltoallv(send, sbytes, soff, recv, rbytes, roff);
        return rc ? oge_fail(ctx, OGE_ERR_HIP, rc == -2 ? "host transport: all-to-all timed out (a rank did not arrive)"
                                                       : "host transport: all-to-all failed")
                  : OGE_OK;
    }
    int allgather_host(oge_ctx *ctx, const void *in, void *out, size_t bytes) override {
        StageOps ops{ctx};
        oge_dist::ShmColl<StageOps> c{*seg, ops};
        return c.allgather_host(in, out, bytes) ? oge_fail(ctx, OGE_ERR_HIP, "host transport: allgather timed out") : OGE_OK;
    }
    int reduce_scatter_max_u8(oge_ctx *ctx, const uint8_t *in, uint8_t *out, size_t chunk) override {
        StageOps ops{ctx};
        oge_dist::ShmColl<StageOps> c{*seg, ops};
        const int rc = c.reduce_scatter_max_u8(in, out, chunk);
        return rc ? oge_fail(ctx, OGE_ERR_HIP, rc == -2 ? "host transport: reduce-scatter timed out" : "host transport: reduce-scatter failed")
                  : OGE_OK;
    }
};

#define OGE_NCCL_TRY(ctx, expr)                                                                              \
    do {                                                                                                     \
        ncclResult_t _r = (expr);                                                                            \
        if (_r != ncclSuccess) return oge_fail((ctx), OGE_ERR_HIP, (std::string(#expr) + ": " + ncclGetErrorString(_r)).c_str()); \
    } while (0)

struct RcclTransport : OgeTransport {
    ncclComm_t comm = nullptr;
    // The small host-side exchanges (statuses, per-destination counts, splitter samples) go through host
    // memory when every rank is on this node (r06): the node's shared segment for ranks
    // in separate processes, the in-process hub for oge_comm_init's ranks.  Otherwise (ranks on several
    // hosts) a device round trip through ncclAllGather.
    std::unique_ptr<oge_dist::ShmSeg> hx_seg;
    std::shared_ptr<oge_dist::Hub> hx_hub;
    ~RcclTransport() override {
        hx_seg.reset();
        if (comm) ncclCommDestroy(comm);
    }
    const char *gather_mode() const override { return hx_seg || hx_hub ? "host_memory" : "device_round_trip"; }
    const char *name() const override { return "rccl"; }
    int alltoallv(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
                  const uint64_t *roff) override {
        OGE_NCCL_TRY(ctx, ncclGroupStart());
        for (int p = 0; p < size; ++p) {
            if (sbytes[p]) OGE_NCCL_TRY(ctx, ncclSend((const uint8_t *)send + soff[p], sbytes[p], ncclUint8, p, comm, ctx->stream));
            if (rbytes[p]) OGE_NCCL_TRY(ctx, ncclRecv((uint8_t *)recv + roff[p], rbytes[p], ncclUint8, p, comm, ctx->stream));
        }
        OGE_NCCL_TRY(ctx, ncclGroupEnd());
        // stream-ordered, not waited for (r06): every consumer of `recv` is queued on ctx->stream after it, and
        // anything the host reads goes through a copy + synchronize on that stream
        return OGE_OK;
    }
    int alltoallv_peers(oge_ctx *ctx, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                        const uint64_t *rbytes, const uint64_t *roff, hipStream_t st) override {
        OGE_NCCL_TRY(ctx, ncclGroupStart());  // queued on st, not waited for: the caller joins st
        for (int p = 0; p < size; ++p) {
            if (p == rank) continue;
            if (sbytes[p]) OGE_NCCL_TRY(ctx, ncclSend((const uint8_t *)send + soff[p], sbytes[p], ncclUint8, p, comm, st));
            if (rbytes[p]) OGE_NCCL_TRY(ctx, ncclRecv((uint8_t *)recv + roff[p], rbytes[p], ncclUint8, p, comm, st));
        }
        OGE_NCCL_TRY(ctx, ncclGroupEnd());
        return OGE_OK;
    }
    bool overlaps() const override { return true; }
    int allgather_host(oge_ctx *ctx, const void *in, void *out, size_t bytes) override {
        if (hx_hub) {
            HipOps ops{ctx};
            oge_dist::LocalColl<HipOps> c{*hx_hub, rank, ops};
            return c.allgather_host(in, out, bytes);
        }
        if (hx_seg) {
            StageOps ops{ctx};
            oge_dist::ShmColl<StageOps> c{*hx_seg, ops};
            return c.allgather_host(in, out, bytes) ? oge_fail(ctx, OGE_ERR_HIP, "rccl transport: host allgather timed out") : OGE_OK;
        }
        uint8_t *d = (uint8_t *)ctx->ws("comm_allgather", bytes * size);
        if (!d) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(d + bytes * rank, in, bytes, hipMemcpyHostToDevice, ctx->stream));
        OGE_NCCL_TRY(ctx, ncclAllGather(d + bytes * rank, d, bytes, ncclUint8, comm, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(out, d, bytes * size, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    }
    int reduce_scatter_max_u8(oge_ctx *ctx, const uint8_t *in, uint8_t *out, size_t chunk) override {
        if (chunk) OGE_NCCL_TRY(ctx, ncclReduceScatter(in, out, chunk, ncclUint8, ncclMax, comm, ctx->stream));
        return OGE_OK;  // stream-ordered (see alltoallv)
    }
};

// ------------------------------------------------------------------------------------------ kernels
// ByPosition key (sort.hip's k_keypack without the size payload)
__global__ __launch_bounds__(kT) void k_dist_keys(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                                                  int32_t n_ref, uint64_t *__restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[i];
    const int32_t ref = oge_rd_i32(r + OGE_OFF_REFID), pos = oge_rd_i32(r + OGE_OFF_POS);
    const uint32_t rev = (oge_rd_u16(r + OGE_OFF_FLAG) >> 4) & 1u;
    keys[i] = ref == -1 ? (uint64_t)(uint32_t)n_ref << 33
                        : ((uint64_t)(uint32_t)ref << 33) | ((uint64_t)(uint32_t)(pos + 1) << 1) | rev;
}

__global__ __launch_bounds__(kT) void k_sample(const uint64_t *__restrict__ keys, uint64_t n, uint32_t m, uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i < m) out[i] = keys[oge_dist::sample_pos(n, m, i)];
}

// destination of each record by its key; G = excluded
__global__ __launch_bounds__(kT) void k_dest_range(const uint64_t *__restrict__ keys, uint64_t n, const uint64_t *__restrict__ spl,
                                                   uint32_t nspl, uint64_t *__restrict__ dkey, uint32_t *__restrict__ dval) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    dkey[i] = oge_dist::owner_of(keys[i] & OGE_SORT_KEY_MASK, spl, nspl);
    dval[i] = (uint32_t)i;
}

// fragment ReadEnds -> owner of the 5' coordinate's key; other records excluded (G)
__global__ __launch_bounds__(kT) void k_dest_frag(const RecMeta *__restrict__ meta, uint64_t n, const uint64_t *__restrict__ spl,
                                                  uint32_t nspl, uint32_t G, uint64_t *__restrict__ dkey, uint32_t *__restrict__ dval) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const RecMeta &M = meta[i];
    uint32_t d = G;
    if (M.m & OGE_M_FRAG) {
        const int64_t c1 = (int64_t)M.coord + 1;
        const uint64_t cpos = c1 < 0 ? 0 : (uint64_t)c1;
        d = oge_dist::owner_of(((uint64_t)(uint32_t)M.seq << 33) | ((cpos > 0xffffffffull ? 0xffffffffull : cpos) << 1), spl, nspl);
    }
    dkey[i] = d;
    dval[i] = (uint32_t)i;
}

// mate-join candidates -> owner of their RG:name hash; other records excluded (G)
__global__ __launch_bounds__(kT) void k_dest_cand(const RecMeta *__restrict__ meta, uint64_t n, uint32_t G,
                                                  uint64_t *__restrict__ dkey, uint32_t *__restrict__ dval) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const RecMeta &M = meta[i];
    dkey[i] = (M.m & OGE_M_CAND) ? oge_dist::hash_owner(oge_meta_hash48(M), G) : G;
    dval[i] = (uint32_t)i;
}

__global__ __launch_bounds__(kT) void k_dest_pairs(const uint64_t *__restrict__ hk, uint32_t np, uint32_t G, uint64_t *__restrict__ dkey,
                                                   uint32_t *__restrict__ dval) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i >= np) return;
    dkey[i] = oge_dist::hash_owner(hk[i], G);
    dval[i] = i;
}

__global__ __launch_bounds__(kT) void k_count_dest(const uint64_t *__restrict__ dkey, uint64_t n, uint32_t G,
                                                   unsigned long long *__restrict__ cnt) {
    __shared__ unsigned int c[65];
    for (uint32_t g = threadIdx.x; g <= G; g += kT) c[g] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kT) atomicAdd(&c[dkey[i]], 1u);
    __syncthreads();
    for (uint32_t g = threadIdx.x; g <= G; g += kT)
        if (c[g]) atomicAdd(cnt + g, (unsigned long long)c[g]);
}

// out[k] = in[perm[k]] for elements of W 4-byte words
template <int W>
__global__ __launch_bounds__(kT) void k_gather_words(const uint32_t *__restrict__ in, const uint32_t *__restrict__ perm, uint64_t n,
                                                     uint32_t *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k >= n) return;
    const uint64_t s = perm[k];
#pragma unroll
    for (int w = 0; w < W; ++w) out[k * W + w] = in[s * W + w];
}

__global__ __launch_bounds__(kT) void k_sizes_u32(const uint64_t *__restrict__ off, uint64_t n, uint32_t *__restrict__ sz) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k < n) sz[k] = (uint32_t)(off[k + 1] - off[k]);
}

__global__ __launch_bounds__(kT) void k_off_from_u32(const uint32_t *__restrict__ sz, uint64_t n, uint64_t *__restrict__ off) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k < n) off[k] = sz[k];
    else if (k == n) off[k] = 0;
}

// received summaries from source s start at rcnt_off[s]; their records at rbyte_off[s]
__global__ __launch_bounds__(kT) void k_minirec_fix(RecMeta *__restrict__ cm, uint64_t n, const uint64_t *__restrict__ rcnt_off,
                                                    const uint64_t *__restrict__ rbyte_off, uint32_t G) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k >= n) return;
    uint32_t s = 0;
    while (s + 1 < G && k >= rcnt_off[s + 1]) ++s;
    cm[k].src += rbyte_off[s];
}

__global__ __launch_bounds__(kT) void k_padded_index(const uint32_t *__restrict__ local, uint64_t n, uint32_t base,
                                                     uint32_t *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k < n) out[k] = base + local[k];
}

__global__ __launch_bounds__(kT) void k_iota(uint64_t n, uint32_t *__restrict__ v) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k < n) v[k] = (uint32_t)k;
}

__global__ __launch_bounds__(kT) void k_map_pair_idx(uint2 *__restrict__ idx, uint32_t np, const uint32_t *__restrict__ gidx) {
    const uint32_t p = blockIdx.x * kT + threadIdx.x;
    if (p < np) idx[p] = make_uint2(gidx[idx[p].x], gidx[idx[p].y]);
}

// ------------------------------------------------------------------------------------------- driver
struct Dist {
    oge_comm *comm;
    oge_ctx *ctx;
    int G, rank;

    // device -> host, ordered after this rank's stream (the context's stream does not synchronise
    // with the null stream a plain hipMemcpy uses)
    int d2h(void *h, const void *d, size_t bytes) {
        if (hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return oge_fail(ctx, OGE_ERR_HIP, (std::string("multi-GPU: device->host copy: ") + hipGetErrorString(hipGetLastError())).c_str());
        return OGE_OK;
    }

    int agree(int rc) {  // every rank learns whether any rank failed; keeps the collectives in step
        std::vector<int> all(G);
        int r2 = comm->allgather_host("status", &rc, all.data(), sizeof(int));
        if (r2) return r2;
        for (int g = 0; g < G; ++g)
            if (all[g]) return rc ? rc : oge_fail(ctx, OGE_ERR_HIP, ("multi-GPU: rank " + std::to_string(g) + " failed").c_str());
        return OGE_OK;
    }

    // stable partition of n entries by destination (dkey in [0, G], G = not sent):
    // perm = entry order grouped by destination, cnt[G] = entries per destination
    int partition(uint64_t *dkey, uint32_t *dval, uint64_t n, const char *tag, uint32_t **perm, std::vector<uint64_t> &cnt) {
        cnt.assign(G, 0);
        *perm = dval;
        if (!n) return OGE_OK;
        unsigned long long *dc = (unsigned long long *)ctx->ws("dist_cnt", 8 * (G + 1));
        uint64_t *k2 = (uint64_t *)ctx->ws((std::string("dist_pk_") + tag).c_str(), n * 8);
        uint32_t *v2 = (uint32_t *)ctx->ws((std::string("dist_pv_") + tag).c_str(), n * 4);
        if (!dc || !k2 || !v2) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(dc, 0, 8 * (G + 1), ctx->stream));
        hipLaunchKernelGGL(k_count_dest, dim3(std::min<uint32_t>(oge_ceil_div(n, kT), 1024u)), dim3(kT), 0, ctx->stream,
                           (const uint64_t *)dkey, n, (uint32_t)G, dc);
        OGE_LAUNCH_CHECK(ctx);
        uint32_t b = 0;
        while ((1u << b) <= (uint32_t)G) ++b;
        uint64_t *ko;
        uint32_t *vo;
        int rc = oge_radix_sort_pairs(ctx, dkey, dval, k2, v2, n, (1ull << b) - 1, &ko, &vo);
        if (rc) return rc;
        std::vector<unsigned long long> h(G + 1);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h.data(), dc, 8 * (G + 1), hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (int g = 0; g < G; ++g) cnt[g] = h[g];
        *perm = vo;
        return OGE_OK;
    }

    // exchange plan for per-destination element counts
    int plan(const std::vector<uint64_t> &cnt, oge_dist::Plan *p) {
        std::vector<uint64_t> all((size_t)G * G);
        int rc = comm->allgather_host("plans", cnt.data(), all.data(), G * 8);
        if (rc) return rc;
        *p = oge_dist::plan_from_counts(all, G, rank);
        return OGE_OK;
    }

    // all-to-all of `elem`-byte elements laid out by the plan
    int a2a(const char *tag, const oge_dist::Plan &p, size_t elem, const void *send, void *recv) {
        std::vector<uint64_t> sb(G), so(G), rb(G), ro(G);
        for (int g = 0; g < G; ++g) {
            sb[g] = p.scnt[g] * elem;
            so[g] = p.soff[g] * elem;
            rb[g] = p.rcnt[g] * elem;
            ro[g] = p.roff[g] * elem;
        }
        return comm->alltoallv(tag, send, sb.data(), so.data(), recv, rb.data(), ro.data());
    }

    template <int W>
    int gather_words(const void *in, const uint32_t *perm, uint64_t n, void *out) {
        if (!n) return OGE_OK;
        hipLaunchKernelGGL(k_gather_words<W>, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint32_t *)in, perm, n,
                           (uint32_t *)out);
        OGE_LAUNCH_CHECK(ctx);
        return OGE_OK;
    }
};

}  // namespace

// The record exchange still to be made when dist_dedup starts (sort + dedup): the byte plan, the send
// buffer and the record plan (which records of rbuf came from which rank)
struct RecXchg {
    const oge_dist::Plan *pb, *pr;
    const uint8_t *sbuf;
};
static int dist_dedup(Dist &D, uint8_t *rbuf, const uint64_t *roff, uint64_t R, uint64_t RB, int32_t n_ref, const uint64_t *d_spl,
                      bool sorted, const oge_markdup_opts *opts, uint8_t **d_out, uint64_t **d_out_off, uint64_t *n_out,
                      uint64_t *n_dup_total, const RecXchg *xr = nullptr);

static int dist_run(oge_comm *comm, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref, int sort,
                    const oge_markdup_opts *opts, uint8_t **d_out, uint64_t **d_out_off, uint64_t *n_out, uint64_t *n_dup_total) {
    oge_ctx *ctx = comm->ctx;
    Dist D{comm, ctx, comm->tr->size, comm->tr->rank};
    const int G = D.G;
    const uint32_t nspl = (uint32_t)G - 1;
    int rc = OGE_OK;
    if (opts && opts->compat_nonverbose_index) rc = oge_fail(ctx, OGE_ERR_ARG, "multi-GPU dedup: compat_nonverbose_index is one-GPU only");
    if (n > 0xFFFFFFFEull) rc = oge_fail(ctx, OGE_ERR_LIMIT, "multi-GPU: more than 2^32-2 records on one rank");
    if (!sort && !opts) rc = oge_fail(ctx, OGE_ERR_ARG, "multi-GPU: nothing to do (no sort, no duplicate marking)");
    if ((rc = D.agree(rc))) return rc;

    // ---- 1. range split
    OgeStageTimer *t = ctx->begin_stage("dist_split");
    uint64_t *keys = (uint64_t *)ctx->ws("dist_keys", (n + 1) * 8);
    uint64_t *samp = (uint64_t *)ctx->ws("dist_samp", oge_dist::kSamples * 8);
    if (!keys || !samp) rc = OGE_ERR_HIP;
    const uint32_t m = (uint32_t)std::min<uint64_t>(n, oge_dist::kSamples);
    std::vector<uint64_t> hs(oge_dist::kSamples, 0);
    if (!rc && n) {
        hipLaunchKernelGGL(k_dist_keys, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, n, n_ref, keys);
        hipLaunchKernelGGL(k_sample, dim3(oge_ceil_div(m, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)keys, n, m, samp);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(hs.data(), samp, m * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            rc = oge_fail(ctx, OGE_ERR_HIP, "multi-GPU: key sampling failed");
    }
    if ((rc = D.agree(rc))) return rc;
    std::vector<uint64_t> allsamp((size_t)G * oge_dist::kSamples), alln(G);
    const uint64_t mm[2] = {n, m};
    std::vector<uint64_t> allmm(2 * G);
    if ((rc = comm->allgather_host("splitter_samples", hs.data(), allsamp.data(), oge_dist::kSamples * 8))) return rc;
    if ((rc = comm->allgather_host("splitter_samples", mm, allmm.data(), 16))) return rc;
    std::vector<std::vector<uint64_t>> per(G);
    for (int g = 0; g < G; ++g) {
        alln[g] = allmm[2 * g];
        per[g].assign(allsamp.begin() + (size_t)g * oge_dist::kSamples, allsamp.begin() + (size_t)g * oge_dist::kSamples + allmm[2 * g + 1]);
    }
    const std::vector<uint64_t> spl = oge_dist::choose_splitters(per, alln, G);
    uint64_t *d_spl = (uint64_t *)ctx->ws("dist_spl", 8 * (nspl + 1));
    if (!d_spl) rc = OGE_ERR_HIP;
    if (!rc && nspl) rc = hipMemcpyAsync(d_spl, spl.data(), 8 * nspl, hipMemcpyHostToDevice, ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    uint64_t total = 0, first = 0;
    if (!rc && n) rc = D.d2h(&total, d_off + n, 8);
    if (!rc && n) rc = D.d2h(&first, d_off, 8);
    if (!sort) {  // dedup: records stay where they are, in input order (record index = input position)
        ctx->end_stage(t);
        if ((rc = D.agree(rc))) return rc;
        return dist_dedup(D, const_cast<uint8_t *>(d_recs), d_off, n, total - first, n_ref, d_spl, false, opts, d_out, d_out_off,
                          n_out, n_dup_total);
    }
    uint64_t *dkey = (uint64_t *)ctx->ws("dist_dkey", (n + 1) * 8);
    uint32_t *dval = (uint32_t *)ctx->ws("dist_dval", (n + 1) * 4);
    uint32_t *perm = nullptr;
    std::vector<uint64_t> cnt;
    if (!dkey || !dval) rc = OGE_ERR_HIP;
    if (!rc && n) {
        hipLaunchKernelGGL(k_dest_range, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)keys, n,
                           (const uint64_t *)d_spl, nspl, dkey, dval);
        rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    }
    if (!rc) rc = D.partition(dkey, dval, n, "rec", &perm, cnt);
    // send buffer: records grouped by destination (stable), their sizes
    uint8_t *sbuf = (uint8_t *)ctx->ws("dist_sbuf", total - first + 64);
    uint64_t *soff = (uint64_t *)ctx->ws("dist_soff", (n + 1) * 8);
    uint32_t *ssz = (uint32_t *)ctx->ws("dist_ssz", (n + 1) * 4);
    if (!rc && (!sbuf || !soff || !ssz)) rc = OGE_ERR_HIP;
    if (!rc && n) rc = oge_gather_with_sizes(ctx, d_recs, d_off, perm, nullptr, n, sbuf, soff, nullptr, nullptr);
    if (!rc && n) {
        hipLaunchKernelGGL(k_sizes_u32, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)soff, n, ssz);
        rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    }
    // bytes per destination from the send offsets at the count boundaries
    std::vector<uint64_t> bcnt(G, 0);
    if (!rc) {
        std::vector<uint64_t> bnd(G + 1, 0);
        uint64_t c = 0;
        for (int g = 0; g <= G && !rc; ++g) {
            if (n) rc = D.d2h(&bnd[g], soff + c, 8);
            if (g < G) c += cnt[g];
        }
        for (int g = 0; g < G; ++g) bcnt[g] = bnd[g + 1] - bnd[g];
    }
    ctx->end_stage(t);
    if ((rc = D.agree(rc))) return rc;

    // ---- 2. exchange + local sort
    t = ctx->begin_stage("dist_exchange");
    oge_dist::Plan pr, pb;
    if ((rc = D.plan(cnt, &pr)) || (rc = D.plan(bcnt, &pb))) return rc;
    const uint64_t R = pr.rtot, RB = pb.rtot;
    uint8_t *rbuf = (uint8_t *)ctx->ws("dist_rbuf", RB + 64);
    uint32_t *rsz = (uint32_t *)ctx->ws("dist_rsz", (R + 1) * 4);
    uint64_t *roff = (uint64_t *)ctx->ws("dist_roff", (R + 1) * 8);
    if (!rbuf || !rsz || !roff) rc = OGE_ERR_HIP;
    if ((rc = D.agree(rc))) return rc;
    // every rank makes both exchanges; a failure goes to the agree() below, never straight out.  With
    // duplicate marking the records follow inside dist_dedup, overlapped with the local input pass
    // (OGE_DIST_RECORDS=blocking: before it, on the context stream -- the A/B and fallback of the overlap)
    const char *rmode = getenv("OGE_DIST_RECORDS");
    const bool overlap = opts && !(rmode && !strcmp(rmode, "blocking"));
    rc = D.a2a("record_sizes", pr, 4, ssz, rsz);
    if (!overlap)
        if (const int r2 = D.a2a("records", pb, 1, sbuf, rbuf)) rc = rc ? rc : r2;
    if (!rc) {
        hipLaunchKernelGGL(k_off_from_u32, dim3(oge_ceil_div(R + 1, kT)), dim3(kT), 0, ctx->stream, (const uint32_t *)rsz, R, roff);
        rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    }
    if (!rc) rc = oge_exclusive_scan_u64(ctx, roff, roff, R + 1);
    ctx->end_stage(t);
    if ((rc = D.agree(rc))) return rc;
    if (R > 0xFFFFFFFEull) rc = oge_fail(ctx, OGE_ERR_LIMIT, "multi-GPU: more than 2^32-2 records on one rank after the exchange");
    uint8_t *out = (uint8_t *)ctx->ws("dist_out", RB + 64);
    uint64_t *out_off = (uint64_t *)ctx->ws("dist_out_off", (R + 1) * 8);
    if (!out || !out_off) rc = OGE_ERR_HIP;
    if ((rc = D.agree(rc))) return rc;

    uint64_t *k = nullptr;
    uint32_t *v = nullptr;
    if (!opts) {  // sort only
        rc = oge_sort_keys_dev(ctx, rbuf, roff, R, n_ref, false, &k, &v, nullptr, nullptr);
        if (!rc) rc = oge_gather_with_sizes(ctx, rbuf, roff, v, k, R, out, out_off, nullptr, nullptr);
        if (!rc) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        if ((rc = D.agree(rc))) return rc;
        *d_out = out;
        *d_out_off = out_off;
        *n_out = R;
        if (n_dup_total) *n_dup_total = 0;
        return OGE_OK;
    }

    const RecXchg xr{&pb, &pr, sbuf};
    return dist_dedup(D, rbuf, roff, R, RB, n_ref, d_spl, true, opts, d_out, d_out_off, n_out, n_dup_total, overlap ? &xr : nullptr);
}

// Duplicate marking of this rank's records (its sorted slice when `sorted`, else its input shard in
// input order), then the gather of the records with bin recomputed and 0x400 applied.
static int dist_dedup(Dist &D, uint8_t *rbuf, const uint64_t *roff, uint64_t R, uint64_t RB, int32_t n_ref, const uint64_t *d_spl,
                      bool sorted, const oge_markdup_opts *opts, uint8_t **d_out, uint64_t **d_out_off, uint64_t *n_out,
                      uint64_t *n_dup_total, const RecXchg *xr) {
    oge_comm *comm = D.comm;
    oge_ctx *ctx = D.ctx;
    const int G = D.G;
    const uint32_t nspl = (uint32_t)G - 1;
    int rc = OGE_OK;
    OgeStageTimer *t = nullptr;
    uint8_t *out = (uint8_t *)ctx->ws("dist_out", RB + 64);
    uint64_t *out_off = (uint64_t *)ctx->ws("dist_out_off", (R + 1) * 8);
    if (!out || !out_off) rc = OGE_ERR_HIP;
    uint64_t *k = nullptr;
    uint32_t *v = nullptr;
    RecMeta *meta_in = nullptr, *meta = nullptr;
    OgeRgTable rg;
    if (!rc) rc = oge_markdup_prepare(ctx, opts, R, "md_meta_in", &meta_in, &rg);
    uint64_t *skeys = nullptr;
    uint32_t *svals = nullptr;
    unsigned int *counts = oge_sort_counts(ctx);
    if (!rc && (oge_sort_buffers(ctx, R, &skeys, &svals) || !counts)) rc = OGE_ERR_HIP;
    meta = (RecMeta *)ctx->ws("md_meta", (R + 1) * sizeof(RecMeta));
    if (!rc && !meta) rc = OGE_ERR_HIP;
    if (!rc) rc = hipMemsetAsync(counts, 0, 32, ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    // the ReadEnds / key pass over records [r0, r1) of rbuf
    auto pass = [&](uint64_t r0, uint64_t r1) {
        if (rc || r1 <= r0) return;
        OgePassArgs a = {};
        a.recs = rbuf;
        a.off = roff + r0;
        a.n = r1 - r0;
        a.ibase = r0;
        a.meta = meta_in + r0;
        a.rg = rg;
        a.keys = sorted ? skeys + r0 : nullptr;
        a.vals = sorted ? svals + r0 : nullptr;
        a.n_ref = n_ref;
        a.bad = counts + 2;
        a.keyred = (unsigned long long *)(counts + 4);
        rc = oge_input_pass(ctx, a);
    };
    if (xr) {
        // Records still to exchange: this rank's own records are copied and passed on
        // the context stream while the peers' parts move on a side stream (RCCL: queued there; the host
        // transport: its staged copies run there while this stream executes the pass), then the pass covers
        // the received records.  Every rank makes the exchange whatever happened before (agree() below).
        t = ctx->begin_stage("input_pass");
        const int me = D.rank;
        const oge_dist::Plan &pb = *xr->pb, &pr = *xr->pr;
        hipStream_t side = ctx->side_stream(0);
        hipEvent_t ev[2] = {nullptr, nullptr};
        for (auto &e : ev)
            if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = dist_hip_fail(ctx, __LINE__);
        if (!rc && !side) rc = OGE_ERR_HIP;
        // the send buffer (gathered on the context stream) before the side stream reads it
        if (!rc && (hipEventRecord(ev[0], ctx->stream) != hipSuccess || hipStreamWaitEvent(side, ev[0], 0) != hipSuccess))
            rc = dist_hip_fail(ctx, __LINE__);
        if (!rc && pb.scnt[me] &&
            hipMemcpyAsync(rbuf + pb.roff[me], xr->sbuf + pb.soff[me], pb.scnt[me], hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess)
            rc = dist_hip_fail(ctx, __LINE__);
        pass(pr.roff[me], pr.roff[me] + pr.rcnt[me]);
        std::vector<uint64_t> sb(D.G), so(D.G), rb(D.G), ro(D.G);
        for (int g = 0; g < D.G; ++g) sb[g] = pb.scnt[g], so[g] = pb.soff[g], rb[g] = pb.rcnt[g], ro[g] = pb.roff[g];
        const int rx = comm->alltoallv_peers("records", xr->sbuf, sb.data(), so.data(), rbuf, rb.data(), ro.data(),
                                             side ? side : ctx->stream);
        if (!rc) rc = rx;
        if (!rc && (hipEventRecord(ev[1], side) != hipSuccess || hipStreamWaitEvent(ctx->stream, ev[1], 0) != hipSuccess))
            rc = dist_hip_fail(ctx, __LINE__);
        pass(0, pr.roff[me]);
        pass(pr.roff[me] + pr.rcnt[me], R);
        if (side) (void)hipStreamSynchronize(side);  // the events may go: nothing is left on the side stream
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        ctx->end_stage(t);
    } else if (!rc) {
        t = ctx->begin_stage("input_pass");
        pass(0, R);
        ctx->end_stage(t);
    }
    if (sorted) {
        if (!rc) rc = oge_sort_keys_dev(ctx, rbuf, roff, R, n_ref, true, &k, &v, meta_in, meta);
    } else {  // input order: the summaries as they are, the identity permutation for the gather
        v = svals;
        if (!rc && R) rc = hipMemcpyAsync(meta, meta_in, R * sizeof(RecMeta), hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess
                               ? 0 : dist_hip_fail(ctx, __LINE__);
        if (!rc && R) {
            hipLaunchKernelGGL(k_iota, dim3(oge_ceil_div(R, kT)), dim3(kT), 0, ctx->stream, R, v);
            rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        }
    }
    if ((rc = D.agree(rc))) return rc;

    // ---- 3. dedup: global indices
    std::vector<uint64_t> allR(G);
    if ((rc = comm->allgather_host("plans", &R, allR.data(), 8))) return rc;
    uint64_t stride = 1, Ntot = 0;
    for (int g = 0; g < G; ++g) stride = std::max<uint64_t>(stride, allR[g]), Ntot += allR[g];
    if ((uint64_t)G * stride > 0xFFFFFFFFull)
        return oge_fail(ctx, OGE_ERR_LIMIT, "multi-GPU dedup: G x the largest slice exceeds 2^32 records");
    const uint32_t base = (uint32_t)((uint64_t)D.rank * stride);
    (void)Ntot;
    (void)nspl;
    uint8_t *dup_pad = (uint8_t *)ctx->ws("dist_dup_pad", (size_t)G * stride);
    uint8_t *dup = (uint8_t *)ctx->ws("dist_dup", stride + 1);
    uint64_t *desc = (uint64_t *)ctx->ws("dist_desc", (R + 1) * 8);
    uint64_t *desc0 = (uint64_t *)ctx->ws("dist_desc0", (R + 1) * 8);
    if (!dup_pad || !dup || !desc || !desc0) rc = OGE_ERR_HIP;
    if (!rc) rc = hipMemsetAsync(dup_pad, 0, (size_t)G * stride, ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    OgeMdFrags F;
    t = ctx->begin_stage("dist_frags");
    if (!rc) rc = oge_md_cand_frag(ctx, opts, meta, R, true, &F);
    if (!rc && F.desc_ovf) rc = oge_fail(ctx, OGE_ERR_LIMIT, "multi-GPU dedup: a record offset exceeds 2^39");
    if (!rc && R) rc = hipMemcpyAsync(desc0, F.desc0, R * 8, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    if ((rc = D.agree(rc))) return rc;

    // fragments -> owner of their 5' coordinate
    {
        uint64_t *fdk = (uint64_t *)ctx->ws("dist_fdk", (R + 1) * 8);
        uint32_t *fdv = (uint32_t *)ctx->ws("dist_fdv", (R + 1) * 4);
        uint64_t *fks = (uint64_t *)ctx->ws("dist_fks", (R + 1) * 8);
        uint32_t *fvs = (uint32_t *)ctx->ws("dist_fvs", (R + 1) * 4);
        if (!fdk || !fdv || !fks || !fvs) rc = OGE_ERR_HIP;
        if (!rc && R) {
            hipLaunchKernelGGL(k_dest_frag, dim3(oge_ceil_div(R, kT)), dim3(kT), 0, ctx->stream, (const RecMeta *)meta, R,
                               (const uint64_t *)d_spl, nspl, (uint32_t)G, fdk, fdv);
            rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        }
        uint32_t *fperm = nullptr;
        std::vector<uint64_t> fc;
        if (!rc) rc = D.partition(fdk, fdv, R, "frag", &fperm, fc);
        uint64_t ns = 0;
        for (uint64_t c : fc) ns += c;
        if (!rc && ns) {  // fragment keys and padded global indices in destination order
            rc = D.gather_words<2>(F.fk, fperm, ns, fks);
            if (!rc) {
                hipLaunchKernelGGL(k_padded_index, dim3(oge_ceil_div(ns, kT)), dim3(kT), 0, ctx->stream, (const uint32_t *)fperm, ns, base,
                                   fvs);
                rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
            }
        }
        if ((rc = D.agree(rc))) return rc;
        oge_dist::Plan pf;
        if ((rc = D.plan(fc, &pf))) return rc;
        uint64_t *fkr = (uint64_t *)ctx->ws("dist_fkr", (pf.rtot + 1) * 8);
        uint32_t *fvr = (uint32_t *)ctx->ws("dist_fvr", (pf.rtot + 1) * 4);
        if (!fkr || !fvr) rc = OGE_ERR_HIP;
        if ((rc = D.agree(rc))) return rc;
        rc = D.a2a("fragments", pf, 8, fks, fkr);
        if (const int r2 = D.a2a("fragments", pf, 4, fvs, fvr)) rc = rc ? rc : r2;
        if (!rc) rc = oge_md_frag_groups(ctx, fkr, fvr, pf.rtot, dup_pad);
        if ((rc = D.agree(rc))) return rc;
    }
    ctx->end_stage(t);

    // mate-join candidates -> owner of their RG:name hash, with their minimal records
    t = ctx->begin_stage("dist_join");
    OgeMdPairs P;
    {
        uint64_t *cdk = (uint64_t *)ctx->ws("dist_cdk", (R + 1) * 8);
        uint32_t *cdv = (uint32_t *)ctx->ws("dist_cdv", (R + 1) * 4);
        if (!cdk || !cdv) rc = OGE_ERR_HIP;
        if (!rc && R) {
            hipLaunchKernelGGL(k_dest_cand, dim3(oge_ceil_div(R, kT)), dim3(kT), 0, ctx->stream, (const RecMeta *)meta, R, (uint32_t)G,
                               cdk, cdv);
            rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        }
        uint32_t *cperm = nullptr;
        std::vector<uint64_t> cc;
        if (!rc) rc = D.partition(cdk, cdv, R, "cand", &cperm, cc);
        uint64_t ns = 0;
        for (uint64_t c : cc) ns += c;
        RecMeta *cms = (RecMeta *)ctx->ws("dist_cms", (ns + 1) * sizeof(RecMeta));
        uint32_t *cgs = (uint32_t *)ctx->ws("dist_cgs", (ns + 1) * 4);
        uint64_t *moff = (uint64_t *)ctx->ws("dist_moff", (ns + 1) * 8);
        uint64_t *dend = (uint64_t *)ctx->ws("dist_dend", 8 * (G + 1));
        if (!cms || !cgs || !moff || !dend) rc = OGE_ERR_HIP;
        std::vector<uint64_t> mb(G, 0);
        if (!rc && ns) {
            rc = D.gather_words<sizeof(RecMeta) / 4>(meta, cperm, ns, cms);
            if (!rc) {
                hipLaunchKernelGGL(k_padded_index, dim3(oge_ceil_div(ns, kT)), dim3(kT), 0, ctx->stream, (const uint32_t *)cperm, ns, base,
                                   cgs);
                hipLaunchKernelGGL(k_minirec_sizes, dim3(oge_ceil_div(ns + 1, kT)), dim3(kT), 0, ctx->stream, rbuf, (const RecMeta *)cms,
                                   ns, false, moff);
                rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
            }
            if (!rc) rc = oge_exclusive_scan_u64(ctx, moff, moff, ns + 1);
            std::vector<uint64_t> de(G), mo(G + 1, 0);
            uint64_t c = 0;
            for (int g = 0; g < G; ++g) c += cc[g], de[g] = c;
            for (int g = 0; g <= G && !rc; ++g) {
                const uint64_t at = g ? de[g - 1] : 0;
                rc = D.d2h(&mo[g], moff + at, 8);
            }
            for (int g = 0; g < G; ++g) mb[g] = mo[g + 1] - mo[g];
            uint8_t *mrec = nullptr;
            if (!rc) {
                mrec = (uint8_t *)ctx->ws("dist_mrec", mo[G] + 64);
                if (!mrec) rc = OGE_ERR_HIP;
            }
            if (!rc) rc = hipMemcpyAsync(dend, de.data(), 8 * G, hipMemcpyHostToDevice, ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
            if (!rc) {
                hipLaunchKernelGGL(k_minirec_write, dim3(oge_ceil_div(ns, kT)), dim3(kT), 0, ctx->stream, rbuf, cms, ns,
                                   (const uint64_t *)moff, (const uint64_t *)dend, (uint32_t)G, mrec);
                rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
            }
            // `de` (the source of the dend upload) leaves scope here
            if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = dist_hip_fail(ctx, __LINE__);
        }
        if ((rc = D.agree(rc))) return rc;
        oge_dist::Plan pc, pm;
        if ((rc = D.plan(cc, &pc)) || (rc = D.plan(mb, &pm))) return rc;
        const uint64_t nr = pc.rtot;
        RecMeta *cmr = (RecMeta *)ctx->ws("dist_cmr", (nr + 1) * sizeof(RecMeta));
        uint32_t *cgr = (uint32_t *)ctx->ws("dist_cgr", (nr + 1) * 4);
        uint8_t *mrr = (uint8_t *)ctx->ws("dist_mrr", pm.rtot + 64);
        uint64_t *rco = (uint64_t *)ctx->ws("dist_rco", 8 * (G + 1));
        uint64_t *rbo = (uint64_t *)ctx->ws("dist_rbo", 8 * (G + 1));
        if (!cmr || !cgr || !mrr || !rco || !rbo) rc = OGE_ERR_HIP;
        if ((rc = D.agree(rc))) return rc;
        uint8_t *mrec = (uint8_t *)ctx->ws("dist_mrec", 64);
        rc = D.a2a("matejoin_candidates", pc, sizeof(RecMeta), cms, cmr);
        if (const int r2 = D.a2a("matejoin_candidates", pc, 4, cgs, cgr)) rc = rc ? rc : r2;
        if (const int r3 = D.a2a("matejoin_minirecs", pm, 1, mrec, mrr)) rc = rc ? rc : r3;
        if (!rc && nr) {
            if (hipMemcpyAsync(rco, pc.roff.data(), 8 * (G + 1), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
                hipMemcpyAsync(rbo, pm.roff.data(), 8 * (G + 1), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
                rc = dist_hip_fail(ctx, __LINE__);
            if (!rc) {
                hipLaunchKernelGGL(k_minirec_fix, dim3(oge_ceil_div(nr, kT)), dim3(kT), 0, ctx->stream, cmr, nr, (const uint64_t *)rco,
                                   (const uint64_t *)rbo, (uint32_t)G);
                rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
            }
        }
        // the owner's join: arrival order (source rank, then sorted position) = global order
        OgeMdFrags F2;
        if (!rc) rc = oge_md_cand_frag(ctx, opts, cmr, nr, false, &F2);
        if (!rc) rc = oge_md_join_build(ctx, opts, mrr, cmr, nr, F2, &P);
        if (!rc && P.np) {
            hipLaunchKernelGGL(k_map_pair_idx, dim3(oge_ceil_div(P.np, kT)), dim3(kT), 0, ctx->stream, P.idx, P.np, (const uint32_t *)cgr);
            rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        }
        if ((rc = D.agree(rc))) return rc;
    }
    ctx->end_stage(t);

    // pair ReadEnds -> owner of their chunk-key hash
    t = ctx->begin_stage("dist_pairs");
    {
        const uint32_t np = P.np;
        uint64_t *pdk = (uint64_t *)ctx->ws("dist_pdk", ((uint64_t)np + 1) * 8);
        uint32_t *pdv = (uint32_t *)ctx->ws("dist_pdv", ((uint64_t)np + 1) * 4);
        uint64_t *shi = (uint64_t *)ctx->ws("dist_shi", ((uint64_t)np + 1) * 8);
        uint64_t *slo = (uint64_t *)ctx->ws("dist_slo", ((uint64_t)np + 1) * 8);
        uint2 *sidx = (uint2 *)ctx->ws("dist_sidx", ((uint64_t)np + 1) * 8);
        if (!pdk || !pdv || !shi || !slo || !sidx) rc = OGE_ERR_HIP;
        if (!rc && np) {
            hipLaunchKernelGGL(k_dest_pairs, dim3(oge_ceil_div(np, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)P.hk, np, (uint32_t)G,
                               pdk, pdv);
            rc = hipGetLastError() == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
        }
        uint32_t *pperm = nullptr;
        std::vector<uint64_t> pc2;
        if (!rc) rc = D.partition(pdk, pdv, np, "pair", &pperm, pc2);
        if (!rc && np) {
            rc = D.gather_words<2>(P.hi, pperm, np, shi);
            if (!rc) rc = D.gather_words<2>(P.lo, pperm, np, slo);
            if (!rc) rc = D.gather_words<2>(P.idx, pperm, np, sidx);
        }
        if ((rc = D.agree(rc))) return rc;
        oge_dist::Plan pp;
        if ((rc = D.plan(pc2, &pp))) return rc;
        OgeMdPairs Q;
        Q.np = (uint32_t)pp.rtot;
        Q.hi = (uint64_t *)ctx->ws("dist_rhi", (pp.rtot + 1) * 8);
        Q.lo = (uint64_t *)ctx->ws("dist_rlo", (pp.rtot + 1) * 8);
        Q.idx = (uint2 *)ctx->ws("dist_ridx", (pp.rtot + 1) * 8);
        if (!Q.hi || !Q.lo || !Q.idx) rc = OGE_ERR_HIP;
        if ((rc = D.agree(rc))) return rc;
        rc = D.a2a("pair_ends", pp, 8, shi, Q.hi);
        if (const int r2 = D.a2a("pair_ends", pp, 8, slo, Q.lo)) rc = rc ? rc : r2;
        if (const int r3 = D.a2a("pair_ends", pp, 8, sidx, Q.idx)) rc = rc ? rc : r3;
        if (!rc) rc = oge_md_pairs_rehash(ctx, &Q);
        if (!rc) rc = oge_md_pair_groups(ctx, opts, Q, dup_pad);
        if ((rc = D.agree(rc))) return rc;
    }
    ctx->end_stage(t);

    // ---- dup marks meet; 4. apply + gather
    t = ctx->begin_stage("dist_reduce");
    rc = comm->reduce_scatter_max_u8("dup_marks", dup_pad, dup, stride);
    ctx->end_stage(t);
    t = ctx->begin_stage("md_apply");
    uint64_t nd = 0;
    if (!rc) rc = oge_md_apply_desc(ctx, desc0, R, dup, desc, &nd);
    ctx->end_stage(t);
    if (!rc) rc = oge_gather_with_sizes(ctx, rbuf, roff, v, k, R, out, out_off, meta, dup, desc);
    if (!rc) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : dist_hip_fail(ctx, __LINE__);
    if ((rc = D.agree(rc))) return rc;
    std::vector<uint64_t> alld(G);
    if ((rc = comm->allgather_host("status", &nd, alld.data(), 8))) return rc;
    uint64_t tot = 0;
    for (uint64_t x : alld) tot += x;
    *d_out = out;
    *d_out_off = out_off;
    *n_out = R;
    if (n_dup_total) *n_dup_total = tot;
    return OGE_OK;
}

oge_ctx *oge_comm_ctx(oge_comm *comm) { return comm ? comm->ctx : nullptr; }

int oge_comm_sum_u64(oge_comm *comm, uint64_t *v, int count) {
    const int G = comm->tr->size;
    std::vector<uint64_t> all((size_t)G * count);
    const int rc = comm->allgather_host("status", v, all.data(), 8 * (size_t)count);
    if (rc) return rc;
    for (int k = 0; k < count; ++k) {
        v[k] = 0;
        for (int g = 0; g < G; ++g) v[k] += all[(size_t)g * count + k];
    }
    return OGE_OK;
}

int oge_comm_allgather(oge_comm *comm, const char *tag, const void *in, void *out, size_t bytes) {
    return comm->allgather_host(tag, in, out, bytes);
}

int oge_comm_alltoallv_dev(oge_comm *comm, const char *tag, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                           const uint64_t *rbytes, const uint64_t *roff) {
    return comm->alltoallv(tag, send, sbytes, soff, recv, rbytes, roff);
}

void oge_comm_reset_stats(oge_comm *comm) { comm->clear_stats(); }

// ---------------------------------------------------------------------------------------------- ABI
extern "C" {

// The id = RCCL's unique id + 16 random bytes that name the node-local meeting of ranks sharing a GPU.
constexpr size_t kIdNonce = 16;

int oge_comm_unique_id(uint8_t *id_out, uint64_t bytes) {
    if (!id_out || bytes < sizeof(ncclUniqueId) + kIdNonce) return oge_fail(nullptr, OGE_ERR_ARG, "oge_comm_unique_id: buffer too small");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return oge_fail(nullptr, OGE_ERR_HIP, ncclGetErrorString(r));
    memcpy(id_out, &id, sizeof id);
    std::random_device rd;
    for (size_t i = 0; i < kIdNonce; i += 4) {
        const uint32_t v = rd();
        memcpy(id_out + sizeof id + i, &v, 4);
    }
    return OGE_OK;
}

uint64_t oge_comm_unique_id_bytes(void) { return sizeof(ncclUniqueId) + kIdNonce; }

// Number of ranks the launcher placed on this node, when it says (torchrun LOCAL_WORLD_SIZE, Open MPI,
// MPICH / Hydra); 0 = unknown.
static int launcher_local_ranks() {
    for (const char *v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", "SLURM_NTASKS_PER_NODE",
                          "SLURM_STEP_TASKS_PER_NODE"}) {
        const char *e = getenv(v);
        if (e && *e) return atoi(e);
    }
    return 0;
}

// OGE_COMM_HOSTX=0: RCCL's host exchanges take the device round trip even on one node
static bool hostx_enabled() {
    const char *e = getenv("OGE_COMM_HOSTX");
    return !(e && *e == '0');
}

// Transport of one rank.  mode: "rccl", "host" or "auto" (nullptr / "": OGE_COMM, default auto).  RCCL
// between distinct GPUs, the host-staged transport (dist_shm.h) when ranks share one.  auto: a process
// that sees at least `nranks` devices takes RCCL at once (bench.py / the CLI give rank r device r %
// count).  With fewer visible devices than ranks, the shared-segment meeting (which compares the ranks'
// PCI bus ids: all distinct -> RCCL, else host) is only tried when every rank is known to be on this
// node -- the launcher's local rank count equals nranks (torchrun's LOCAL_WORLD_SIZE, ...), or the caller
// runs every rank itself (the CLI's threads pass "host" when ranks share devices, else "node" = auto on one
// node); otherwise (a multi-node job, 2 x 8 GPUs with a device-isolating launcher) RCCL, which is the only
// transport that reaches other hosts.  RCCL ranks known to be on one node also meet in a small shared
// segment for their host exchanges (RcclTransport::hx_seg; OGE_COMM_HOSTX=0 turns that off).
static int comm_init_rank(oge_ctx *ctx, int nranks, int rank, const uint8_t *id, const char *want, oge_comm **out) {
    if (!ctx || !id || !out || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        return oge_fail(ctx, OGE_ERR_ARG, "oge_comm_init_rank: bad arguments");
    (void)hipSetDevice(ctx->device);
    const bool node = want && !strcmp(want, "node");  // the caller runs every rank on this node (the CLI's threads)
    const char *e = want && *want && !node ? want : getenv("OGE_COMM");
    std::string mode = e && *e ? e : "auto";
    if (mode == "local") mode = "host";  // oge_comm_init's in-process name for "ranks share a GPU"
    const bool one_node = node || launcher_local_ranks() == nranks;
    if (mode != "auto" && mode != "rccl" && mode != "host")
        return oge_fail(ctx, OGE_ERR_ARG, "OGE_COMM must be auto, rccl or host");
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    std::unique_ptr<oge_dist::ShmSeg> seg, hx;
    if (mode == "host" || (mode == "auto" && ndev < nranks && one_node)) {
        char bus[64] = {0};
        (void)hipDeviceGetPCIBusId(bus, sizeof bus - 1, ctx->device);
        uint64_t h = 1469598103934665603ull;  // FNV-1a of the whole id names the meeting
        for (size_t i = 0; i < sizeof(ncclUniqueId) + kIdNonce; ++i) h = (h ^ id[i]) * 1099511628211ull;
        char name[64];
        snprintf(name, sizeof name, "oge_comm_%016llx", (unsigned long long)h);
        std::string err;
        seg.reset(oge_dist::ShmSeg::open(name, nranks, rank, oge_dist::ShmSeg::default_stage_bytes(), bus, &err));
        if (!seg) {
            err += " (the host transport meets node-local ranks only: a job spanning several hosts needs OGE_COMM=rccl)";
            return oge_fail(ctx, OGE_ERR_HIP, err.c_str());
        }
        bool shared = false;
        for (int a = 0; a < nranks; ++a)
            for (int b = a + 1; b < nranks; ++b) shared = shared || !strcmp(seg->post(a).bus, seg->post(b).bus);
        if (mode == "auto" && !shared) hx = std::move(seg);  // distinct GPUs: RCCL after all (the segment stays for
                                                             // the host exchanges)
    }
    oge_comm *c = new oge_comm();
    c->ctx = ctx;
    if (seg) {
        auto t = std::make_unique<ShmTransport>();
        t->seg = std::move(seg);
        t->rank = rank;
        t->size = nranks;
        c->tr = std::move(t);
    } else {
        auto t = std::make_unique<RcclTransport>();
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof uid);
        ncclResult_t r = ncclCommInitRank(&t->comm, nranks, uid, rank);
        if (r != ncclSuccess) {
            delete c;
            std::string m = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            if (mode == "auto" && ndev < nranks)  // ranks that may share a device, started by a launcher we do not know
                m += " (fewer visible devices than ranks: ranks sharing a GPU need the host transport, OGE_COMM=host)";
            return oge_fail(ctx, OGE_ERR_HIP, m.c_str());
        }
        t->rank = rank;
        t->size = nranks;
        if (one_node && hostx_enabled()) {
            // the host exchanges' segment (RcclTransport::hx_seg): met right after ncclCommInitRank, which every
            // rank has passed, so the meeting takes milliseconds (bounded at 60 s); then one allreduce makes
            // every rank take the same route
            if (!hx) {
                char bus[64] = {0};
                (void)hipDeviceGetPCIBusId(bus, sizeof bus - 1, ctx->device);
                uint64_t h = 1469598103934665603ull;
                for (size_t i = 0; i < sizeof(ncclUniqueId) + kIdNonce; ++i) h = (h ^ id[i]) * 1099511628211ull;
                char name[64];
                snprintf(name, sizeof name, "oge_hx_%016llx", (unsigned long long)h);
                std::string err;
                hx.reset(oge_dist::ShmSeg::open(name, nranks, rank, 1ull << 20, bus, &err, 60.0));
            }
            int have = hx ? 1 : 0;
            int *d = (int *)ctx->ws("comm_hx_agree", sizeof(int));
            if (!d || hipMemcpyAsync(d, &have, sizeof have, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
                ncclAllReduce(d, d, 1, ncclInt32, ncclMin, t->comm, ctx->stream) != ncclSuccess ||
                hipMemcpyAsync(&have, d, sizeof have, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                hipStreamSynchronize(ctx->stream) != hipSuccess)
                have = 0;
            if (!have) hx.reset();
            t->hx_seg = std::move(hx);
        }
        c->tr = std::move(t);
    }
    *out = c;
    return OGE_OK;
}

int oge_comm_init_rank(oge_ctx *ctx, int nranks, int rank, const uint8_t *id, oge_comm **out) {
    return comm_init_rank(ctx, nranks, rank, id, nullptr, out);
}

int oge_comm_init_rank_mode(oge_ctx *ctx, int nranks, int rank, const uint8_t *id, const char *mode, oge_comm **out) {
    return comm_init_rank(ctx, nranks, rank, id, mode, out);
}

int oge_comm_init(oge_ctx **ctxs, int n, oge_comm **out) {
    if (!ctxs || !out || n < 1 || n > 64) return oge_fail(nullptr, OGE_ERR_ARG, "oge_comm_init: bad arguments");
    for (int g = 0; g < n; ++g)
        if (!ctxs[g]) return oge_fail(nullptr, OGE_ERR_ARG, "oge_comm_init: null context");
    bool distinct = true;
    for (int a = 0; a < n; ++a)
        for (int b = a + 1; b < n; ++b) distinct = distinct && ctxs[a]->device != ctxs[b]->device;
    const char *e = getenv("OGE_COMM");
    const bool local = !distinct || n == 1 || (e && !strcmp(e, "local"));
    if (local) {  // contexts sharing a GPU (or forced): the in-process hub
        auto hub = std::make_shared<oge_dist::Hub>(n);
        for (int g = 0; g < n; ++g) {
            auto t = std::make_unique<LocalTransport>();
            t->hub = hub;
            t->rank = g;
            t->size = n;
            out[g] = new oge_comm();
            out[g]->ctx = ctxs[g];
            out[g]->tr = std::move(t);
        }
        return OGE_OK;
    }
    std::vector<ncclComm_t> cs(n);
    std::vector<int> devs(n);
    for (int g = 0; g < n; ++g) devs[g] = ctxs[g]->device;
    ncclResult_t r = ncclCommInitAll(cs.data(), n, devs.data());
    if (r != ncclSuccess) return oge_fail(nullptr, OGE_ERR_HIP, (std::string("ncclCommInitAll: ") + ncclGetErrorString(r)).c_str());
    // the ranks are threads of this process: their host exchanges meet at one hub (RcclTransport::hx_hub)
    std::shared_ptr<oge_dist::Hub> hx_hub = hostx_enabled() ? std::make_shared<oge_dist::Hub>(n) : nullptr;
    for (int g = 0; g < n; ++g) {
        auto t = std::make_unique<RcclTransport>();
        t->comm = cs[g];
        t->rank = g;
        t->size = n;
        t->hx_hub = hx_hub;
        out[g] = new oge_comm();
        out[g]->ctx = ctxs[g];
        out[g]->tr = std::move(t);
    }
    return OGE_OK;
}

void oge_comm_destroy(oge_comm *c) { delete c; }

int oge_comm_rank(const oge_comm *c) { return c ? c->tr->rank : -1; }
int oge_comm_size(const oge_comm *c) { return c ? c->tr->size : -1; }
const char *oge_comm_transport(const oge_comm *c) { return c ? c->tr->name() : ""; }

int64_t oge_comm_stats_json(const oge_comm *c, char *buf, uint64_t cap) {
    if (!c) return -1;
    c->settle_events();
    std::string j = "[";
    char tmp[448];
    for (size_t i = 0; i < c->stats.size(); ++i) {
        const OgeXchg &x = c->stats[i];
        snprintf(tmp, sizeof tmp,
                 "%s{\"tag\":\"%s\",\"calls\":%llu,\"bytes_sent\":%llu,\"bytes_recv\":%llu,\"bytes_self\":%llu,\"ms\":%.3f,"
                 "\"device_ms\":%.3f,\"mode\":\"%s\"}",
                 i ? "," : "", x.tag.c_str(), (unsigned long long)x.calls, (unsigned long long)x.sent, (unsigned long long)x.recv,
                 (unsigned long long)x.self, x.ms, x.dev_ms, x.mode);
        j += tmp;
    }
    j += "]";
    if (buf && cap > j.size()) memcpy(buf, j.c_str(), j.size() + 1);
    return (int64_t)j.size();
}

int oge_sort_markdup_dist(oge_comm *comm, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref, int sort,
                          const oge_markdup_opts *opts, uint8_t **d_out, uint64_t **d_out_off, uint64_t *n_out,
                          uint64_t *n_dup_total) {
    if (!comm || !d_out || !d_out_off || !n_out || (n && (!d_recs || !d_off)))
        return oge_fail(comm ? comm->ctx : nullptr, OGE_ERR_ARG, "oge_sort_markdup_dist: bad arguments");
    oge_ctx *ctx = comm->ctx;
    (void)hipSetDevice(ctx->device);
    ctx->reset_timing();
    if (!ctx->timing_hold) comm->clear_stats();  // a composite entry point (pipeline.hip) keeps its earlier exchanges
    if (opts && opts->n_ref != n_ref) return oge_fail(ctx, OGE_ERR_ARG, "oge_sort_markdup_dist: opts->n_ref differs from n_ref");
    return dist_run(comm, d_recs, d_off, n, n_ref, sort, opts, d_out, d_out_off, n_out, n_dup_total);
}

}  // extern "C"
