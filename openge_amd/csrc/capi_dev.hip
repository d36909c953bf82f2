// capi_dev.hip -- C-ABI entry points that run on the GPU, the context implementation, and the
// device-side synthetic generator.
#include <chrono>
#include "oge_ctx.h"
#include "bam_layout.h"
#include "synth.h"
#include "records.h"
#include "markdup_stages.h"

#include <cstdio>
#include <cstring>
#include <string>

// implemented in sort.hip / markdup.hip
int oge_sort_buffers(oge_ctx *ctx, uint64_t n, uint64_t **keys, uint32_t **vals);
unsigned int *oge_sort_counts(oge_ctx *ctx);
int oge_sort_keys_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                      bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in = nullptr,
                      RecMeta *meta_out = nullptr);
int oge_markdup_prepare(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, const char *name, RecMeta **meta,
                        OgeRgTable *rg);
int oge_markdup_finish(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                       const RecMeta *meta, uint8_t *d_dup, int apply, uint64_t *n_dup_out, uint64_t *d_desc, bool *desc_ok,
                       const uint64_t *skeys);
int oge_meta_gather(oge_ctx *ctx, const RecMeta *in, const uint32_t *perm, uint64_t n, RecMeta *out);
int oge_sort_keys_dev_hook(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                           bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out,
                           const OgeSortGatherHook *hook);
int oge_markdup_run(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                    uint8_t *d_dup, int apply, uint64_t *n_dup_out);

static thread_local std::string g_last_error;

int oge_fail(oge_ctx *ctx, int code, const char *msg) {
    g_last_error = msg ? msg : "";
    if (ctx) ctx->err = g_last_error;
    return code;
}

// ---------------------------------------------------------------- context
// With `pool` (oge_ctx_set_pool), buffers come from the device's default stream-ordered pool with
// an unlimited release threshold: memory one module frees is handed to the next module's buffers
// without going back to the driver (each fresh hipMalloc of tens of GB maps new pages, which on
// some boxes costs seconds in a CLI run).
void *oge_ctx::alloc(size_t bytes) {
    void *p = nullptr;
    if (pool) {
        if (hipMallocAsync(&p, bytes, stream) != hipSuccess) return nullptr;
        return p;
    }
    // experiment (OGE_ALLOC_CONTIG=1): physically contiguous buffers, i.e. the largest page fragments
    static const bool contig = getenv("OGE_ALLOC_CONTIG") && atoi(getenv("OGE_ALLOC_CONTIG")) == 1;
    if (contig && hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) == hipSuccess) return p;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}

void oge_ctx::release(void *p) {
    if (!p) return;
    if (pool) hipFreeAsync(p, stream);
    else hipFree(p);
}

void *oge_ctx::ws(const char *name, size_t bytes) {
    Buf &b = bufs[name];
    if (bytes == 0) bytes = 1;
    if (b.cap >= bytes) return b.p;
    // host time of (re)allocations, per call (oge_ctx_counter "ws_alloc_us" / "ws_allocs"); OGE_TRACE_ALLOC
    // prints each one
    const auto t0 = std::chrono::steady_clock::now();
    struct Note {
        oge_ctx *c;
        const char *nm;
        size_t sz;
        std::chrono::steady_clock::time_point t0;
        ~Note() {
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            c->counters["ws_alloc_us"] += (uint64_t)us;
            c->counters["ws_allocs"] += 1;
            static const bool tr = getenv("OGE_TRACE_ALLOC") != nullptr;
            if (tr) fprintf(stderr, "[oge ws] %s %.3f GB: %.1f ms\n", nm, sz / 1e9, us / 1e3);
        }
    } note{this, name, bytes, t0};
    if (b.p) {
        hipStreamSynchronize(stream);
        release(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    size_t cap = bytes + 64;  // slack so 4-byte over-reads at the end stay inside the allocation
    b.p = alloc(cap);
    hipError_t e = b.p ? hipSuccess : hipErrorOutOfMemory;
    if (e != hipSuccess) {
        b.p = nullptr;
        std::string m = std::string("hipMalloc(") + name + ", " + std::to_string(cap) + " B): " + hipGetErrorString(e);
        oge_fail(this, OGE_ERR_HIP, m.c_str());
        return nullptr;
    }
    b.cap = cap;
    return b.p;
}

// side stream 3 carries the host pipeline's PCIe copies, which the runtime runs as blit kernels: it is
// created with the highest priority so it does not share a hardware queue with (and wait behind) the
// codec kernels on streams 0-2 (r05o: a 1.4 GB copy held each 10 ms segment deflate to 31 ms)
hipStream_t oge_ctx::side_stream(int i) {
    if (side[i]) return side[i];
    int lo = 0, hi = 0;
    const bool prio = i == 3 && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess;
    if ((prio ? hipStreamCreateWithPriority(&side[i], hipStreamNonBlocking, hi) : hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking)) !=
        hipSuccess)
        side[i] = nullptr;
    return side[i];
}

void *oge_ctx::scratch(const char *name, size_t bytes) {
    const size_t a = (loan_used + 255) & ~(size_t)255;
    if (loan_base && a + bytes + 64 <= loan_cap) {
        loan_used = a + bytes + 64;
        return loan_base + a;
    }
    return ws(name, bytes);
}

OgeStageTimer *oge_ctx::begin_stage(const char *name) {
    if (!timing) return nullptr;
    if (event_pool_used == event_pool.size()) {
        OgeStageTimer t;
        hipEventCreate(&t.start);
        hipEventCreate(&t.stop);
        event_pool.push_back(t);
    }
    OgeStageTimer *t = &event_pool[event_pool_used++];
    hipEventRecord(t->start, stream);
    stage_events[name].push_back(*t);
    return t;
}

void oge_ctx::end_stage(OgeStageTimer *t) {
    if (t) hipEventRecord(t->stop, stream);
}

void oge_ctx::reset_timing() {
    // every top-level entry point starts here: drop a sticky error some other HIP user of this thread
    // left behind (torch in a worker thread, say), so OGE_LAUNCH_CHECK reports only our launches
    (void)hipGetLastError();
    if (timing_hold) return;
    stage_events.clear();
    counters.clear();
    event_pool_used = 0;
}

extern "C" {

const char *oge_version(void) { return "openge_amd 0.1 (gfx950)"; }

const char *oge_last_error(const oge_ctx *ctx) { return ctx ? ctx->err.c_str() : g_last_error.c_str(); }

int oge_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int oge_ctx_create(int device, oge_ctx **out) {
    if (!out) return oge_fail(nullptr, OGE_ERR_ARG, "oge_ctx_create: out is NULL");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0)
        return oge_fail(nullptr, OGE_ERR_HIP, "oge_ctx_create: no HIP device (the GPU path has no CPU fallback)");
    if (device < 0 || device >= ndev) return oge_fail(nullptr, OGE_ERR_ARG, "oge_ctx_create: bad device index");
    e = hipSetDevice(device);
    if (e != hipSuccess) return oge_fail(nullptr, OGE_ERR_HIP, hipGetErrorString(e));
    oge_ctx *c = new oge_ctx();
    c->device = device;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return oge_fail(nullptr, OGE_ERR_HIP, hipGetErrorString(e));
    }
    c->own_stream = true;
    *out = c;
    return OGE_OK;
}

int oge_ctx_set_stream(oge_ctx *ctx, void *stream) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    if (stream) {
        // the old stream's work ends before the new stream's starts: the inflate's bitmap carry-over
        // (phase 2 clears what phase 1 of the next call relies on) and the record walk's cached starts
        // are only valid in stream order, so both are also forgotten
        (void)hipStreamSynchronize(ctx->stream);
        ctx->infl_clean_ptr = nullptr;
        ctx->infl_clean_bytes = ctx->infl_clean_next = 0;
        ctx->recwalk = oge_ctx::RecWalk{};
        if (ctx->own_stream) hipStreamDestroy(ctx->stream);
        ctx->stream = (hipStream_t)stream;
        ctx->own_stream = false;
    }
    return OGE_OK;
}

void *oge_ctx_stream(oge_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int oge_ctx_sync(oge_ctx *ctx) {
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

void oge_ctx_destroy(oge_ctx *ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (auto &kv : ctx->bufs) ctx->release(kv.second.p);
    hipStreamSynchronize(ctx->stream);
    for (auto &t : ctx->event_pool) {
        hipEventDestroy(t.start);
        hipEventDestroy(t.stop);
    }
    for (hipStream_t s : ctx->side)
        if (s) hipStreamDestroy(s);
    if (ctx->own_stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

int oge_ctx_counter(oge_ctx *ctx, const char *name, uint64_t *value) {
    if (!ctx || !name || !value) return oge_fail(ctx, OGE_ERR_ARG, "oge_ctx_counter: null argument");
    auto it = ctx->counters.find(name);
    if (it == ctx->counters.end()) return OGE_ERR_ARG;
    *value = it->second;
    return OGE_OK;
}

int oge_ctx_timing(oge_ctx *ctx, const char *stage, double *ms_out) {
    if (!ctx || !stage || !ms_out) return oge_fail(ctx, OGE_ERR_ARG, "oge_ctx_timing: null argument");
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    double tot = 0;
    auto it = ctx->stage_events.find(stage);
    if (it == ctx->stage_events.end()) { *ms_out = -1; return OGE_OK; }
    for (auto &t : it->second) {
        float ms = 0;
        OGE_HIP_TRY(ctx, hipEventElapsedTime(&ms, t.start, t.stop));
        tot += ms;
    }
    *ms_out = tot;
    return OGE_OK;
}

// ---------------------------------------------------------------- device buffers
int oge_dev_alloc(oge_ctx *ctx, uint64_t bytes, void **out) {
    if (!ctx || !out) return oge_fail(ctx, OGE_ERR_ARG, "oge_dev_alloc: null argument");
    hipSetDevice(ctx->device);
    *out = ctx->alloc(bytes ? bytes : 1);
    if (!*out) return oge_fail(ctx, OGE_ERR_HIP, ("oge_dev_alloc: out of device memory (" + std::to_string(bytes) + " B)").c_str());
    return OGE_OK;
}

int oge_dev_free(oge_ctx *ctx, void *p) {
    if (!ctx) return oge_fail(ctx, OGE_ERR_ARG, "oge_dev_free: null ctx");
    hipSetDevice(ctx->device);
    ctx->release(p);
    return OGE_OK;
}

int oge_mem_info(oge_ctx *ctx, uint64_t *free_bytes, uint64_t *total_bytes) {
    if (!ctx || !free_bytes || !total_bytes) return oge_fail(ctx, OGE_ERR_ARG, "oge_mem_info: null argument");
    (void)hipSetDevice(ctx->device);
    size_t f = 0, t = 0;
    OGE_HIP_TRY(ctx, hipMemGetInfo(&f, &t));
    *free_bytes = f;
    *total_bytes = t;
    return OGE_OK;
}

int oge_ctx_set_pool(oge_ctx *ctx, int enable) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    if (enable) {
        hipMemPool_t mp;
        OGE_HIP_TRY(ctx, hipDeviceGetDefaultMemPool(&mp, ctx->device));
        uint64_t thr = ~0ull;
        OGE_HIP_TRY(ctx, hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &thr));
    }
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->pool = enable != 0;
    return OGE_OK;
}

int oge_host_alloc(oge_ctx *ctx, uint64_t bytes, void **out) {
    if (!ctx || !out) return oge_fail(ctx, OGE_ERR_ARG, "oge_host_alloc: null argument");
    hipSetDevice(ctx->device);
    *out = nullptr;
    OGE_HIP_TRY(ctx, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return OGE_OK;
}

int oge_host_free(oge_ctx *ctx, void *p) {
    if (!ctx) return oge_fail(ctx, OGE_ERR_ARG, "oge_host_free: null ctx");
    if (p) OGE_HIP_TRY(ctx, hipHostFree(p));
    return OGE_OK;
}

int oge_memcpy(oge_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind) {
    if (!ctx || (bytes && (!dst || !src))) return oge_fail(ctx, OGE_ERR_ARG, "oge_memcpy: null argument");
    hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost
                    : kind == 3 ? hipMemcpyDeviceToDevice : hipMemcpyDefault;
    if (kind < 1 || kind > 4) return oge_fail(ctx, OGE_ERR_ARG, "oge_memcpy: bad kind");
    hipSetDevice(ctx->device);
    if (bytes) OGE_HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

// ---------------------------------------------------------------- sort
int oge_sort_coord_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref, uint32_t *d_perm) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    uint64_t *k;
    uint32_t *v;
    int rc = oge_sort_keys_dev(ctx, d_recs, d_off, n, n_ref, false, &k, &v);
    if (rc) return rc;
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_perm, v, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    return OGE_OK;
}

int oge_gather_records_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, const uint32_t *d_perm, uint64_t n,
                           uint8_t *d_out, uint64_t *d_out_off) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    return oge_gather_with_sizes(ctx, d_recs, d_off, d_perm, nullptr, n, d_out, d_out_off, nullptr, nullptr);
}

static int upload(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n, uint8_t **d_recs,
                  uint64_t **d_off) {
    *d_recs = (uint8_t *)ctx->ws("host_recs", rec_bytes + 16);
    *d_off = (uint64_t *)ctx->ws("host_off", (n + 1) * 8);
    if (!*d_recs || !*d_off) return OGE_ERR_HIP;
    if (rec_bytes) OGE_HIP_TRY(ctx, hipMemcpyAsync(*d_recs, recs, rec_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(*d_off, rec_off, n * 8, hipMemcpyHostToDevice, ctx->stream));
    return OGE_OK;
}

int oge_sort_coord(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n, int32_t n_ref,
                   uint32_t *perm_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    uint8_t *dr;
    uint64_t *dof;
    int rc = upload(ctx, recs, rec_bytes, rec_off, n, &dr, &dof);
    if (rc) return rc;
    uint32_t *dp = (uint32_t *)ctx->ws("host_perm", (n + 1) * 4);
    if (!dp) return OGE_ERR_HIP;
    rc = oge_sort_coord_dev(ctx, dr, dof, n, n_ref, dp);
    if (rc) return rc;
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(perm_out, dp, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

int oge_sort_name(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n,
                  uint32_t *perm_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    uint8_t *dr;
    uint64_t *dof;
    int rc = upload(ctx, recs, rec_bytes, rec_off, n, &dr, &dof);
    if (rc) return rc;
    uint32_t *dp = (uint32_t *)ctx->ws("host_perm", (n + 1) * 4);
    if (!dp) return OGE_ERR_HIP;
    rc = oge_sort_name_dev(ctx, dr, dof, n, dp);
    if (rc) return rc;
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(perm_out, dp, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

// ---------------------------------------------------------------- markdup
int oge_markdup_dev(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                    uint8_t *d_dup, int apply, uint64_t *n_dup_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    uint64_t nd = 0;
    int rc = oge_markdup_run(ctx, d_recs, d_off, n, opts, d_dup, apply, &nd);
    if (n_dup_out) *n_dup_out = nd;
    return rc;
}

int oge_markdup(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n,
                const oge_markdup_opts *opts, uint8_t *dup_out, uint64_t *n_dup_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    uint8_t *dr;
    uint64_t *dof;
    int rc = upload(ctx, recs, rec_bytes, rec_off, n, &dr, &dof);
    if (rc) return rc;
    uint8_t *dd = (uint8_t *)ctx->ws("host_dup", n + 1);
    if (!dd) return OGE_ERR_HIP;
    rc = oge_markdup_dev(ctx, dr, dof, n, opts, dd, 0, n_dup_out);
    if (rc) return rc;
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(dup_out, dd, n, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

int oge_sort_markdup_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                         uint32_t *d_perm, uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_dup_out) {
    // mergesort -M --nosplit on device:
    //   1 input pass   : sort keys + 32-byte ReadEnds summaries, records read once in input order
    //   2 sort         : radix sort of the coordinate keys, name/flag tie runs
    //   3 meta gather  : summaries into sorted order (record index = sorted position, as in the
    //                    reference where MarkDuplicates consumes the sorter's output stream)
    //   4 markdup      : mate join, pair/fragment groups -> dup[] in sorted order
    //   5 record gather: sorted records written once with bin recomputed and 0x400 applied
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!opts) return oge_fail(ctx, OGE_ERR_ARG, "sort_markdup: opts is NULL");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    // d_out holds the records' byte total and is only written by the final gather: until then it is
    // the scratch arena of the pipeline (input summaries, mate-join and group buffers), which keeps
    // the 300M-read footprint at the two record arenas + ~30 GB
    if (n) {
        uint64_t span[2] = {0, 0};
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&span[0], d_off, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&span[1], d_off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        ctx->lend(d_out, span[1] - span[0]);
    }
    struct Loan {
        oge_ctx *c;
        ~Loan() { c->end_loan(); }
    } loan{ctx};
    RecMeta *meta_in;
    OgeRgTable rg;
    int rc = oge_markdup_prepare(ctx, opts, n, "md_meta_in", &meta_in, &rg);
    if (rc) return rc;
    uint64_t *keys;
    uint32_t *vals;
    if (oge_sort_buffers(ctx, n, &keys, &vals)) return OGE_ERR_HIP;
    unsigned int *counts = oge_sort_counts(ctx);
    if (!counts) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(counts, 0, 32, ctx->stream));
    OgeStageTimer *t = ctx->begin_stage("input_pass");
    OgePassArgs a = {};
    a.recs = d_recs;
    a.off = d_off;
    a.n = n;
    a.meta = meta_in;
    a.rg = rg;
    a.keys = keys;
    a.vals = vals;
    a.n_ref = opts->n_ref;
    a.bad = counts + 2;
    a.keyred = (unsigned long long *)(counts + 4);
    rc = oge_input_pass(ctx, a);
    if (rc) return rc;
    ctx->end_stage(t);
    uint64_t *k;
    uint32_t *v;
    RecMeta *meta = (RecMeta *)ctx->ws("md_meta", (n + 1) * sizeof(RecMeta));
    uint8_t *dd = (uint8_t *)ctx->ws("sm_dup", n + 1);
    if (!meta || !dd) return OGE_ERR_HIP;
    // the summaries are gathered after the tie sort, in final order, by the same pass that derives the
    // mate-join / fragment / descriptor words from them (oge_md_cand_frag_gather: one pass over the rows)
    // the descriptors in a workspace, not in scratch: scratch lives in the lent output buffer, which the gather
    // overwrites while it reads them (the deferred apply)
    uint64_t *desc = (uint64_t *)ctx->ws("sm_desc", (n + 1) * 8);
    if (!desc) return OGE_ERR_HIP;
    struct Cf {
        const oge_markdup_opts *opts;
        const RecMeta *in;
        RecMeta *out;
        uint64_t n;
        uint64_t *desc0;
        OgeMdFrags F;
    } cf{opts, meta_in, meta, n, desc, {}};
    OgeSortGatherHook hook{[](void *u, oge_ctx *c, const uint32_t *perm, const uint64_t *skeys) {
                               Cf *x = (Cf *)u;
                               return oge_md_cand_frag_gather(c, x->opts, x->in, perm, x->n, x->out, true, skeys, &x->F, x->desc0);
                           },
                           &cf};
    rc = oge_sort_keys_dev_hook(ctx, d_recs, d_off, n, opts->n_ref, true, &k, &v, meta_in, meta, &hook);
    if (rc) return rc;
    if (n) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_perm, v, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    uint64_t nd = 0;
    bool desc_ok = false;
    cf.F.defer_apply = true;  // the gather finishes the descriptors and counts the duplicates (MODE 3)
    rc = oge_markdup_finish_pre(ctx, (uint8_t *)d_recs, d_off, n, opts, meta, dd, 0, &nd, desc, &desc_ok, k, n ? &cf.F : nullptr);
    if (rc) return rc;
    const bool deferred = n && nd == ~0ull;
    unsigned int *nds = deferred ? (unsigned int *)ctx->ws("sm_ndup", 64 * 32 * 4) : nullptr;
    if (deferred) {
        if (!nds) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(nds, 0, 64 * 32 * 4, ctx->stream));
    }
    ctx->end_loan();  // the gather below writes d_out
    rc = oge_gather_with_sizes(ctx, d_recs, d_off, v, k, n, d_out, d_out_off, meta, dd,
                               deferred ? cf.F.desc0 : desc_ok ? desc : nullptr, nds);
    if (rc) return rc;
    if (deferred) {
        uint32_t h[64 * 32];
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h, nds, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        nd = 0;
        for (int q = 0; q < 64; ++q) nd += h[q * 32];
    }
    if (n_dup_out) *n_dup_out = nd;
    return OGE_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device synth
namespace {
__global__ __launch_bounds__(256) void k_synth_sizes(oge_synth_params P, uint64_t s0, uint64_t n, uint64_t *offs) {
    uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s < n) offs[s] = oge_synth_slot_bytes(&P, s0 + s);
    else if (s == n) offs[s] = 0;
}
__global__ __launch_bounds__(256) void k_synth_write(oge_synth_params P, uint64_t s0, uint64_t n, const uint64_t *offs,
                                                     uint8_t *out) {
    uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s < n) oge_synth_write_slot(&P, s0 + s, out + offs[s]);
}
}  // namespace

extern "C" {
int oge_synth_offsets_range_dev(oge_ctx *ctx, const void *params, uint64_t slot0, uint64_t n, uint64_t *d_offs) {
    if (!ctx || !params) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    const oge_synth_params *P = (const oge_synth_params *)params;
    if (slot0 + n > 2 * P->n_pairs) return oge_fail(ctx, OGE_ERR_ARG, "synth: slot range outside the data set");
    hipSetDevice(ctx->device);
    hipLaunchKernelGGL(k_synth_sizes, dim3(oge_ceil_div(n + 1, 256)), dim3(256), 0, ctx->stream, *P, slot0, n, d_offs);
    OGE_LAUNCH_CHECK(ctx);
    return oge_exclusive_scan_u64(ctx, d_offs, d_offs, n + 1);
}
int oge_synth_records_range_dev(oge_ctx *ctx, const void *params, uint64_t slot0, uint64_t n, const uint64_t *d_offs,
                                uint8_t *d_out) {
    if (!ctx || !params) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    const oge_synth_params *P = (const oge_synth_params *)params;
    if (slot0 + n > 2 * P->n_pairs) return oge_fail(ctx, OGE_ERR_ARG, "synth: slot range outside the data set");
    hipSetDevice(ctx->device);
    if (n) {
        hipLaunchKernelGGL(k_synth_write, dim3(oge_ceil_div(n, 256)), dim3(256), 0, ctx->stream, *P, slot0, n, d_offs, d_out);
        OGE_LAUNCH_CHECK(ctx);
    }
    return OGE_OK;
}
int oge_synth_offsets_dev(oge_ctx *ctx, const void *params, uint64_t *d_offs) {
    if (!params) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    return oge_synth_offsets_range_dev(ctx, params, 0, 2 * ((const oge_synth_params *)params)->n_pairs, d_offs);
}
int oge_synth_records_dev(oge_ctx *ctx, const void *params, const uint64_t *d_offs, uint8_t *d_out) {
    if (!params) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    return oge_synth_records_range_dev(ctx, params, 0, 2 * ((const oge_synth_params *)params)->n_pairs, d_offs, d_out);
}
}  // extern "C"

extern "C" int oge_radix_sort_pairs_dev(oge_ctx *ctx, uint64_t *d_keys, uint32_t *d_vals, uint64_t *d_ktmp, uint32_t *d_vtmp,
                                        uint64_t n, uint64_t bit_mask, int *in_tmp_out) {
    if (!ctx || (n && (!d_keys || !d_ktmp)) || ((d_vals == nullptr) != (d_vtmp == nullptr)) || !in_tmp_out)
        return oge_fail(ctx, OGE_ERR_ARG, "oge_radix_sort_pairs_dev: bad arguments");
    hipSetDevice(ctx->device);
    uint64_t *ko = d_keys;
    uint32_t *vo = d_vals;
    int rc = oge_radix_sort_pairs(ctx, d_keys, d_vals, d_ktmp, d_vtmp, n, bit_mask, &ko, d_vals ? &vo : nullptr);
    if (rc) return rc;
    *in_tmp_out = ko != d_keys;
    return OGE_OK;
}
