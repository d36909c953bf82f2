// filter.hip -- record compaction on the device: mergesort's Filter module (-r region / -q mapq,
// algorithms/filter.cpp:205-249) and the writer side of -r/-R duplicate removal
// (algorithms/mark_duplicates.cpp:456-458).
//
// Both are a keep predicate over the record core (one thread per record, 24 bytes of the 32-byte
// core read), an exclusive scan of the keep flags, a keep -> output-position permutation, and the
// shared permutation gather of sort.hip (records copied once, bins recomputed in flight).  The
// predicate costs ~0.1 B/record of HBM against the gather's 2 x record size, so the whole module is
// bound by the gather.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "bam_layout.h"
#include "oge_ctx.h"
#include "records.h"

namespace {

__global__ void k_keep_flags(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n, uint16_t mask,
                             uint32_t *__restrict__ keep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keep[i] = (oge_rd_u16(recs + off[i] + OGE_OFF_FLAG) & mask) ? 0u : 1u;
}

// Filter::runInternal (filter.cpp:213-242).  getPosition() + getLength() is int arithmetic in the
// reference (int32 pos + int32 l_seq); getMapQuality() is the unsigned MAPQ byte.
__global__ void k_keep_filter(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                              oge_filter_opts o, uint32_t *__restrict__ keep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[i];
    const int32_t len = oge_rd_i32(r + OGE_OFF_LSEQ);
    const int32_t mapq = r[OGE_OFF_MAPQ];
    bool k = mapq >= o.mapq_min && len >= o.min_len && len <= o.max_len && len > o.trim_total;
    if (o.has_region) {
        const int32_t ref = oge_rd_i32(r + OGE_OFF_REFID);
        const int32_t pos = oge_rd_i32(r + OGE_OFF_POS);
        k = k && ref >= o.ref_id && ref <= o.ref_id && (int32_t)((uint32_t)pos + (uint32_t)len) >= o.left_pos &&
            pos <= o.right_pos;
    }
    keep[i] = k ? 1u : 0u;
}

__global__ void k_keep_perm(const uint32_t *__restrict__ keep, const uint32_t *__restrict__ pos, uint64_t n,
                            uint32_t *__restrict__ perm) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (keep[i]) perm[pos[i]] = (uint32_t)i;
}

}  // namespace

// keep[] (n flags, already written on the stream) -> the first `limit` kept records, in order.
static int compact_kept(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, uint32_t *keep,
                        uint64_t limit, uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_out) {
    uint32_t *pos = (uint32_t *)ctx->ws("keep_pos", (n + 1) * 4);
    uint32_t *perm = (uint32_t *)ctx->ws("keep_perm", (n + 1) * 4);
    if (!pos || !perm) return OGE_ERR_HIP;
    int rc = oge_exclusive_scan_u32(ctx, keep, pos, n);
    if (rc) return rc;
    k_keep_perm<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(keep, pos, n, perm);
    OGE_LAUNCH_CHECK(ctx);
    uint32_t last[2];
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&last[0], pos + n - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&last[1], keep + n - 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t m = (uint64_t)last[0] + last[1];
    if (m > limit) m = limit;  // the reference stops pulling records once count_limit were kept
    if (m) {
        rc = oge_gather_with_sizes(ctx, d_recs, d_off, perm, nullptr, m, d_out, d_out_off, nullptr, nullptr);
        if (rc) return rc;
    } else {
        OGE_HIP_TRY(ctx, hipMemsetAsync(d_out_off, 0, 8, ctx->stream));
    }
    *n_out = m;
    return OGE_OK;
}

extern "C" int oge_drop_flagged_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, uint16_t flag_mask,
                                    uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!n_out) return oge_fail(ctx, OGE_ERR_ARG, "null n_out");
    if (n >= 0xffffffffull) return oge_fail(ctx, OGE_ERR_ARG, "too many records");
    hipSetDevice(ctx->device);
    *n_out = 0;
    if (!n) return OGE_OK;
    uint32_t *keep = (uint32_t *)ctx->ws("keep_flags", (n + 1) * 4);
    if (!keep) return OGE_ERR_HIP;
    k_keep_flags<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_recs, d_off, n, flag_mask, keep);
    OGE_LAUNCH_CHECK(ctx);
    return compact_kept(ctx, d_recs, d_off, n, keep, ~0ull, d_out, d_out_off, n_out);
}

extern "C" int oge_filter_records_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                                      const oge_filter_opts *o, uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!n_out || !o) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    if (n >= 0xffffffffull) return oge_fail(ctx, OGE_ERR_ARG, "too many records");
    hipSetDevice(ctx->device);
    *n_out = 0;
    if (!n || !o->count_limit) {
        if (d_out_off) OGE_HIP_TRY(ctx, hipMemsetAsync(d_out_off, 0, 8, ctx->stream));
        return OGE_OK;
    }
    uint32_t *keep = (uint32_t *)ctx->ws("keep_flags", (n + 1) * 4);
    if (!keep) return OGE_ERR_HIP;
    OgeStageTimer *t = ctx->begin_stage("filter");
    k_keep_filter<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_recs, d_off, n, *o, keep);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    return compact_kept(ctx, d_recs, d_off, n, keep, o->count_limit, d_out, d_out_off, n_out);
}
