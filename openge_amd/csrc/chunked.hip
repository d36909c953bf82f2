// chunked.hip -- sort (+ duplicate marking) of inputs larger than HBM on one GPU: the MI355X form of
// the reference's runs + merge (alg/read_sorter.cpp:48-190: runs of -n reads sorted and spilled as
// temp BAM files, then a k-way std::multiset merge of the run heads, util/read_stream_reader.h:132-153).
//
//  1 runs     the input (host memory, any size) in chunks of <= chunk_bytes: upload, device sort +
//             gather, and the sorted run written back over the chunk it came from (the host arena
//             is the spill space: no second copy); the run's sorted keys and offsets stay on the host.
//  2 ranges   splitters on the ByPosition key (pooled run samples, refined by bisection until every
//             range fits) cut every run into one contiguous segment per range; equal keys never
//             straddle ranges.  A range = the concatenation of its segments in run order, so a
//             device sort of it is the global order of its records (full ties: run order = input
//             order, within a run the stable sort kept it).  This replaces the k-way merge.
//  3 dedup    (-M) range by range: ReadEnds summaries of the sorted range into one device-resident
//             array for the whole input (64 B/read; 600M reads = 38 GB), minimal records for the
//             mate-join candidates (exact key compares without the arena), then the one-GPU dedup
//             stages over the whole array: the same marks as oge_sort_markdup_dev.
//  4 output   range by range again: device sort + gather (bins recomputed), 0x400 applied from the
//             global marks, handed to the caller's callback (the writer deflates it on the device).
#include "oge_ctx.h"
#include "bam_layout.h"
#include "dev_util.h"
#include "dist_plan.h"
#include "markdup_stages.h"
#include "minirec.h"
#include "records.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int oge_markdup_prepare(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, const char *name, RecMeta **meta,
                        OgeRgTable *rg);
int oge_sort_buffers(oge_ctx *ctx, uint64_t n, uint64_t **keys, uint32_t **vals);
unsigned int *oge_sort_counts(oge_ctx *ctx);
int oge_sort_keys_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                      bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out);

namespace {

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void k_add_src(RecMeta *__restrict__ meta, uint64_t n, uint64_t add) {
    const uint64_t k = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (k < n && (meta[k].m & OGE_M_CAND)) meta[k].src += add;
}

struct Run {
    uint64_t base = 0;            // host byte offset of the run's region (= h_off of its first record)
    std::vector<uint64_t> keys;   // sorted ByPosition keys (size payload stripped)
    std::vector<uint64_t> offs;   // m + 1 byte offsets of the sorted records, relative to base
};

struct Range {
    std::vector<uint64_t> lo, hi;  // per run: record index range of the segment
    uint64_t n = 0, bytes = 0;
};

// Device buffer that keeps its contents when it grows (the global minimal-record arena).
struct GrowBuf {
    oge_ctx *ctx;
    uint8_t *p = nullptr;
    uint64_t cap = 0;
    ~GrowBuf() {
        if (p) ctx->release(p);
    }
    int reserve(uint64_t need, uint64_t used) {
        if (need <= cap) return OGE_OK;
        const uint64_t nc = std::max<uint64_t>(need + (need >> 2), 1 << 20);
        uint8_t *q = (uint8_t *)ctx->alloc(nc);
        if (!q) return oge_fail(ctx, OGE_ERR_HIP, "chunked: out of device memory for the minimal records");
        if (used) OGE_HIP_TRY(ctx, hipMemcpyAsync(q, p, used, hipMemcpyDeviceToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (p) ctx->release(p);
        p = q;
        cap = nc;
        return OGE_OK;
    }
};

// Upload a range (its segments back to back, run order) into A with its rebased offsets in d_off.
int upload_range(oge_ctx *ctx, const uint8_t *h_recs, const std::vector<Run> &runs, const Range &R, uint8_t *A, uint64_t *d_off,
                 std::vector<uint64_t> &hoff) {
    hoff.clear();
    hoff.reserve(R.n + 1);
    uint64_t at = 0;
    for (size_t j = 0; j < runs.size(); ++j) {
        const Run &r = runs[j];
        const uint64_t lo = R.lo[j], hi = R.hi[j];
        if (hi == lo) continue;
        const uint64_t b0 = r.offs[lo], b1 = r.offs[hi];
        OGE_HIP_TRY(ctx, hipMemcpyAsync(A + at, h_recs + r.base + b0, b1 - b0, hipMemcpyHostToDevice, ctx->stream));
        for (uint64_t i = lo; i < hi; ++i) hoff.push_back(at + r.offs[i] - b0);
        at += b1 - b0;
    }
    hoff.push_back(at);
    OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // hoff and pageable sources are reused
    return OGE_OK;
}

// Segments of the key range [klo, khi) (khi = ~0: to the end) in every run.
Range make_range(const std::vector<Run> &runs, uint64_t klo, uint64_t khi, bool last) {
    Range R;
    for (const Run &r : runs) {
        const uint64_t lo = (uint64_t)(std::lower_bound(r.keys.begin(), r.keys.end(), klo) - r.keys.begin());
        const uint64_t hi = last ? r.keys.size() : (uint64_t)(std::lower_bound(r.keys.begin(), r.keys.end(), khi) - r.keys.begin());
        R.lo.push_back(lo);
        R.hi.push_back(hi);
        R.n += hi - lo;
        R.bytes += r.offs[hi] - r.offs[lo];
    }
    return R;
}

// Key ranges whose records fit `cap` bytes: pooled weighted quantiles, then bisection of any range
// that is still too big (a range holding a single key cannot be cut: ties must stay together).
int plan_ranges(oge_ctx *ctx, const std::vector<Run> &runs, uint64_t total, uint64_t cap, std::vector<Range> &out) {
    std::vector<std::vector<uint64_t>> samples(runs.size());
    std::vector<uint64_t> counts(runs.size());
    for (size_t j = 0; j < runs.size(); ++j) {
        const uint64_t m = runs[j].keys.size();
        const uint32_t s = (uint32_t)std::min<uint64_t>(m, oge_dist::kSamples);
        for (uint32_t i = 0; i < s; ++i) samples[j].push_back(runs[j].keys[oge_dist::sample_pos(m, s, i)]);
        counts[j] = m;
    }
    const int K = (int)std::min<uint64_t>(1u << 20, std::max<uint64_t>(1, (total + total / 4) / cap + 1));
    std::vector<uint64_t> spl = oge_dist::choose_splitters(samples, counts, K);
    spl.erase(std::unique(spl.begin(), spl.end()), spl.end());
    // work list of key intervals [a, b) in order; b == ~0 with last = true means "to the end"
    struct Iv { uint64_t a, b; bool last; };
    std::vector<Iv> work;
    uint64_t prev = 0;
    for (uint64_t s : spl) {
        if (s == ~0ull) break;
        work.push_back({prev, s, false});
        prev = s;
    }
    work.push_back({prev, ~0ull, true});
    out.clear();
    while (!work.empty()) {
        const Iv iv = work.front();
        work.erase(work.begin());
        Range R = make_range(runs, iv.a, iv.b, iv.last);
        if (R.bytes <= cap || R.n == 0) {
            if (R.n) out.push_back(std::move(R));
            continue;
        }
        // bisect at the median key of the interval (by record count)
        std::vector<uint64_t> keys;
        for (size_t j = 0; j < runs.size(); ++j) {
            const uint64_t lo = R.lo[j], hi = R.hi[j], step = std::max<uint64_t>(1, (hi - lo) / 4096);
            for (uint64_t i = lo; i < hi; i += step) keys.push_back(runs[j].keys[i]);
        }
        std::sort(keys.begin(), keys.end());
        uint64_t mid = keys[keys.size() / 2];
        if (mid == iv.a) {  // the lower half is one key: cut just above it
            auto it = std::upper_bound(keys.begin(), keys.end(), mid);
            if (it != keys.end()) {
                mid = *it;
            } else {  // no larger key among the samples: the smallest larger key of any run's whole segment
                uint64_t nxt = ~0ull;
                bool found = false;
                for (size_t j = 0; j < runs.size(); ++j) {
                    const uint64_t *b = runs[j].keys.data() + R.lo[j], *e = runs[j].keys.data() + R.hi[j];
                    const uint64_t *u = std::upper_bound(b, e, mid);
                    if (u != e) nxt = std::min(nxt, *u), found = true;
                }
                if (!found)
                    return oge_fail(ctx, OGE_ERR_LIMIT, ("chunked sort: " + std::to_string(R.n) + " records share one sort key (" +
                                                         std::to_string(R.bytes) + " bytes), more than the chunk size").c_str());
                mid = nxt;
            }
        }
        work.insert(work.begin(), {mid, iv.b, iv.last});
        work.insert(work.begin(), {iv.a, mid, false});
    }
    return OGE_OK;
}

}  // namespace

extern "C" int oge_sort_markdup_chunked(oge_ctx *ctx, uint8_t *h_recs, const uint64_t *h_off, uint64_t n, int32_t n_ref,
                                        const oge_markdup_opts *opts, uint64_t chunk_bytes, oge_range_cb cb, void *user,
                                        uint64_t *n_dup, uint64_t *n_runs, uint64_t *n_ranges) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!cb || (n && (!h_recs || !h_off))) return oge_fail(ctx, OGE_ERR_ARG, "oge_sort_markdup_chunked: null argument");
    if (opts && opts->compat_nonverbose_index) return oge_fail(ctx, OGE_ERR_ARG, "chunked dedup: compat_nonverbose_index is not supported");
    if (opts && opts->n_ref != n_ref) return oge_fail(ctx, OGE_ERR_ARG, "oge_sort_markdup_chunked: opts->n_ref differs from n_ref");
    if (n > 0xFFFFFFFEull) return oge_fail(ctx, OGE_ERR_LIMIT, "chunked: more than 2^32-2 records");
    (void)hipSetDevice(ctx->device);
    ctx->reset_timing();
    if (n_dup) *n_dup = 0;
    const uint64_t total = n ? h_off[n] - h_off[0] : 0;
    // per-read bytes the dedup keeps for the whole input: summary 64, minimal record <= 64 (typical
    // names), the stages' scratch ~72, the marks 1
    const uint64_t per_read = opts ? 64 + 64 + 72 + 1 : 0;
    if (!chunk_bytes) {
        size_t fr = 0, tot = 0;
        OGE_HIP_TRY(ctx, hipMemGetInfo(&fr, &tot));
        const uint64_t keep = per_read * n + (2ull << 30);
        if (fr <= keep) return oge_fail(ctx, OGE_ERR_LIMIT, "chunked: the per-read dedup state alone exceeds free HBM; use --gpus");
        chunk_bytes = (uint64_t)((fr - keep) / 2.8);  // two record buffers + sort workspace (~0.4 B/B + 24 B/read)
    }
    chunk_bytes = std::max<uint64_t>(chunk_bytes, 1 << 16);
    uint64_t max_rec = 0;
    for (uint64_t i = 0; i < n; ++i) max_rec = std::max(max_rec, h_off[i + 1] - h_off[i]);
    chunk_bytes = std::max(chunk_bytes, max_rec);

    // ---- 1. sorted runs, spilled in place
    std::vector<Run> runs;
    uint8_t *A = (uint8_t *)ctx->ws("chk_a", chunk_bytes + 64);
    uint8_t *B = (uint8_t *)ctx->ws("chk_b", chunk_bytes + 64);
    if (!A || !B) return OGE_ERR_HIP;
    OgeStageTimer *t = ctx->begin_stage("chunk_runs");
    for (uint64_t r0 = 0; r0 < n;) {
        uint64_t r1 = r0 + 1;
        while (r1 < n && h_off[r1 + 1] - h_off[r0] <= chunk_bytes) ++r1;
        const uint64_t m = r1 - r0, bytes = h_off[r1] - h_off[r0];
        uint64_t *d_off = (uint64_t *)ctx->ws("chk_off", (m + 1) * 8);
        uint64_t *b_off = (uint64_t *)ctx->ws("chk_boff", (m + 1) * 8);
        if (!d_off || !b_off) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(A, h_recs + h_off[r0], bytes, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off, h_off + r0, (m + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        uint64_t *k;
        uint32_t *v;
        const uint8_t *Ash = A - h_off[r0];  // the offsets stay absolute
        int rc = oge_sort_keys_dev(ctx, Ash, d_off, m, n_ref, false, &k, &v, nullptr, nullptr);
        if (!rc) rc = oge_gather_with_sizes(ctx, Ash, d_off, v, k, m, B, b_off, nullptr, nullptr);
        if (rc) return rc;
        Run run;
        run.base = h_off[r0];
        run.keys.resize(m);
        run.offs.resize(m + 1);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h_recs + h_off[r0], B, bytes, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(run.keys.data(), k, m * 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(run.offs.data(), b_off, (m + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (auto &x : run.keys) x &= OGE_SORT_KEY_MASK;
        runs.push_back(std::move(run));
        r0 = r1;
    }
    ctx->end_stage(t);
    if (n_runs) *n_runs = runs.size();

    // ---- 2. key ranges that fit
    std::vector<Range> ranges;
    int rc = plan_ranges(ctx, runs, total, chunk_bytes, ranges);
    if (rc) return rc;
    if (n_ranges) *n_ranges = ranges.size();
    std::vector<uint64_t> hoff;

    // ---- 3. dedup over the whole input, range by range
    RecMeta *meta_all = nullptr;
    uint8_t *dup_all = nullptr;
    GrowBuf mrec{ctx};
    if (opts && n) {
        t = ctx->begin_stage("chunk_dedup");
        meta_all = (RecMeta *)ctx->ws("chk_meta", (n + 1) * sizeof(RecMeta));
        dup_all = (uint8_t *)ctx->ws("chk_dup", n + 1);
        if (!meta_all || !dup_all) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(dup_all, 0, n + 1, ctx->stream));
        uint64_t gbase = 0, used = 0;
        for (const Range &R : ranges) {
            uint64_t *d_off = (uint64_t *)ctx->ws("chk_off", (R.n + 1) * 8);
            uint64_t *msz = (uint64_t *)ctx->ws("chk_msz", (R.n + 1) * 8);
            if (!d_off || !msz) return OGE_ERR_HIP;
            if ((rc = upload_range(ctx, h_recs, runs, R, A, d_off, hoff))) return rc;
            RecMeta *meta_in;
            OgeRgTable rg;
            if ((rc = oge_markdup_prepare(ctx, opts, R.n, "md_meta_in", &meta_in, &rg))) return rc;
            uint64_t *skeys;
            uint32_t *svals;
            unsigned int *counts = oge_sort_counts(ctx);
            if (oge_sort_buffers(ctx, R.n, &skeys, &svals) || !counts) return OGE_ERR_HIP;
            OGE_HIP_TRY(ctx, hipMemsetAsync(counts, 0, 32, ctx->stream));
            OgePassArgs a = {};
            a.recs = A;
            a.off = d_off;
            a.n = R.n;
            a.meta = meta_in;
            a.rg = rg;
            a.keys = skeys;
            a.vals = svals;
            a.n_ref = n_ref;
            a.bad = counts + 2;
            a.keyred = (unsigned long long *)(counts + 4);
            if ((rc = oge_input_pass(ctx, a))) return rc;
            uint64_t *k;
            uint32_t *v;
            RecMeta *mo = meta_all + gbase;  // summaries land in global sorted order
            if ((rc = oge_sort_keys_dev(ctx, A, d_off, R.n, n_ref, true, &k, &v, meta_in, mo))) return rc;
            // minimal records of the candidates; their src then points into the global arena
            hipLaunchKernelGGL(k_minirec_sizes, dim3(oge_ceil_div(R.n + 1, kT)), dim3(kT), 0, ctx->stream, (const uint8_t *)A,
                               (const RecMeta *)mo, R.n, true, msz);
            OGE_LAUNCH_CHECK(ctx);
            if ((rc = oge_exclusive_scan_u64(ctx, msz, msz, R.n + 1))) return rc;
            uint64_t tb = 0;
            OGE_HIP_TRY(ctx, hipMemcpyAsync(&tb, msz + R.n, 8, hipMemcpyDeviceToHost, ctx->stream));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if ((rc = mrec.reserve(used + tb + 64, used))) return rc;
            uint64_t *dend = (uint64_t *)ctx->ws("chk_dend", 16);
            if (!dend) return OGE_ERR_HIP;
            const uint64_t de = R.n;
            OGE_HIP_TRY(ctx, hipMemcpyAsync(dend, &de, 8, hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(k_minirec_write, dim3(oge_ceil_div(R.n, kT)), dim3(kT), 0, ctx->stream, (const uint8_t *)A, mo, R.n,
                               (const uint64_t *)msz, (const uint64_t *)dend, 1u, mrec.p + used);
            OGE_LAUNCH_CHECK(ctx);
            if (used) {
                hipLaunchKernelGGL(k_add_src, dim3(oge_ceil_div(R.n, kT)), dim3(kT), 0, ctx->stream, mo, R.n, used);
                OGE_LAUNCH_CHECK(ctx);
            }
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // `de` leaves scope
            used += tb;
            gbase += R.n;
        }
        OgeMdFrags F;
        OgeMdPairs P;
        if ((rc = oge_md_cand_frag(ctx, opts, meta_all, n, false, &F))) return rc;
        if ((rc = oge_md_join_build(ctx, opts, mrec.p, meta_all, n, F, &P))) return rc;
        if ((rc = oge_md_pair_groups(ctx, opts, P, dup_all))) return rc;
        if ((rc = oge_md_frag_groups(ctx, F.fk, F.fv, n, dup_all))) return rc;
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        ctx->end_stage(t);
    }

    // ---- 4. output, range by range
    t = ctx->begin_stage("chunk_output");
    uint64_t gbase = 0, nd = 0;
    for (const Range &R : ranges) {
        uint64_t *d_off = (uint64_t *)ctx->ws("chk_off", (R.n + 1) * 8);
        uint64_t *b_off = (uint64_t *)ctx->ws("chk_boff", (R.n + 1) * 8);
        if (!d_off || !b_off) return OGE_ERR_HIP;
        if ((rc = upload_range(ctx, h_recs, runs, R, A, d_off, hoff))) return rc;
        uint64_t *k;
        uint32_t *v;
        if ((rc = oge_sort_keys_dev(ctx, A, d_off, R.n, n_ref, false, &k, &v, nullptr, nullptr))) return rc;
        if ((rc = oge_gather_with_sizes(ctx, A, d_off, v, k, R.n, B, b_off, nullptr, nullptr))) return rc;
        if (opts) {
            uint64_t d = 0;
            if ((rc = oge_md_apply_inplace(ctx, B, b_off, R.n, meta_all + gbase, dup_all + gbase, &d))) return rc;
            nd += d;
        }
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if ((rc = cb(user, B, b_off, R.n))) return oge_fail(ctx, rc, "chunked: the output callback failed");
        gbase += R.n;
    }
    ctx->end_stage(t);
    if (n_dup) *n_dup = nd;
    return OGE_OK;
}
