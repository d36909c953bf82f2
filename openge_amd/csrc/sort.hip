// sort.hip -- coordinate sort of BAM records (ReadSorter + Sort::ByPosition) and the permutation
// gather that re-encodes records in sorted order (BamSerializer::write with bin recompute).
//
// Sort key (u64) per record, packed by k_keypack:
//   bits [0]      reverse strand (forward sorts first, util/bamtools/Sort.h:126-127)
//   bits [1,33)   pos + 1  (pos >= -1)
//   bits [33,50)  refID, with refID == -1 mapped to n_ref so unmapped reads sort last (:119-120)
//   bits [50,64)  record byte size (payload: not sorted; feeds the output offset scan)
// Only the key bits that actually vary across the input are radix-sorted (OR/AND reduction).
// Equal (refID,pos,strand) runs are then ordered by read name bytes, flag and input index
// (Sort.h:128-132; input index stands in for the heap-address tie-break) in k_tie_small
// (thread per run <= 32) and k_tie_large (workgroup bitonic per longer run).  The refID == -1
// run keeps input order.
#include "oge_ctx.h"
#include "bam_layout.h"

#include <algorithm>
#include <vector>

namespace {

constexpr uint64_t kSortKeyMask = (1ull << 50) - 1;
constexpr int kT = 256;

__global__ __launch_bounds__(kT) void k_keypack(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                 uint64_t n, int32_t n_ref, uint64_t *__restrict__ keys,
                                                 uint32_t *__restrict__ vals, unsigned int *__restrict__ bad) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[i];
    uint32_t bs = oge_rd_u32(r);
    int32_t ref = oge_rd_i32(r + OGE_OFF_REFID);
    int32_t pos = oge_rd_i32(r + OGE_OFF_POS);
    uint32_t rev = (oge_rd_u16(r + OGE_OFF_FLAG) >> 4) & 1u;
    uint64_t k;
    if (ref == -1) {
        k = (uint64_t)(uint32_t)n_ref << 33;
    } else {
        if (ref < -1 || ref >= n_ref || pos < -1) atomicOr(bad, 1u);
        k = ((uint64_t)(uint32_t)ref << 33) | ((uint64_t)(uint32_t)(pos + 1) << 1) | rev;
    }
    if (bs < 32 || bs > 10000) atomicOr(bad, 2u);
    keys[i] = k | ((uint64_t)(bs + 4) << 50);
    vals[i] = (uint32_t)i;
}

// (name bytes, flag, input index) order inside an equal-coordinate run
__device__ __forceinline__ bool tie_less(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint32_t a,
                                         uint32_t b) {
    if (a == 0xFFFFFFFFu) return false;
    if (b == 0xFFFFFFFFu) return true;
    const uint8_t *ra = recs + off[a], *rb = recs + off[b];
    uint32_t la = ra[OGE_OFF_LNAME], lb = rb[OGE_OFF_LNAME];
    uint32_t m = la < lb ? la : lb;
    const uint8_t *na = ra + OGE_OFF_NAME, *nb = rb + OGE_OFF_NAME;
    for (uint32_t i = 0; i < m; ++i) {
        uint8_t x = na[i], y = nb[i];
        if (x != y) return x < y;
    }
    if (la != lb) return la < lb;
    uint16_t fa = oge_rd_u16(ra + OGE_OFF_FLAG), fb = oge_rd_u16(rb + OGE_OFF_FLAG);
    if (fa != fb) return fa < fb;
    return a < b;
}

__global__ __launch_bounds__(kT) void k_find_ties(const uint64_t *__restrict__ keys, uint64_t n, int32_t n_ref,
                                                   uint2 *__restrict__ small, uint2 *__restrict__ large,
                                                   unsigned int *__restrict__ counts) {
    uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (p + 1 >= n) return;
    uint64_t k = keys[p] & kSortKeyMask;
    if (p > 0 && (keys[p - 1] & kSortKeyMask) == k) return;
    if ((keys[p + 1] & kSortKeyMask) != k) return;
    if ((k >> 33) == (uint64_t)(uint32_t)n_ref) return;  // refID == -1 tail keeps input order
    uint64_t e = p + 2;
    while (e < n && (keys[e] & kSortKeyMask) == k) ++e;
    uint32_t len = (uint32_t)(e - p);
    if (len <= 32) {
        unsigned int s = atomicAdd(&counts[0], 1u);
        small[s] = make_uint2((uint32_t)p, len);
    } else {
        unsigned int s = atomicAdd(&counts[1], 1u);
        large[s] = make_uint2((uint32_t)p, len);
    }
}

__global__ __launch_bounds__(kT) void k_tie_small(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                   const uint2 *__restrict__ segs, uint32_t nseg) {
    uint32_t s = blockIdx.x * kT + threadIdx.x;
    if (s >= nseg) return;
    uint2 sg = segs[s];
    uint64_t *k = keys + sg.x;
    uint32_t *v = vals + sg.x;
    for (uint32_t i = 1; i < sg.y; ++i) {
        uint32_t vi = v[i];
        uint64_t ki = k[i];
        int j = (int)i - 1;
        while (j >= 0 && tie_less(recs, off, vi, v[j])) {
            v[j + 1] = v[j];
            k[j + 1] = k[j];
            --j;
        }
        v[j + 1] = vi;
        k[j + 1] = ki;
    }
}

// One workgroup per long run: bitonic sort of (key,val) in a power-of-two scratch region.
__global__ __launch_bounds__(kT) void k_tie_large(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                   const uint2 *__restrict__ segs, const uint64_t *__restrict__ scratch_off,
                                                   uint64_t *__restrict__ sk, uint32_t *__restrict__ sv) {
    const uint2 sg = segs[blockIdx.x];
    const uint64_t so = scratch_off[blockIdx.x];
    uint32_t P = 1;
    while (P < sg.y) P <<= 1;
    uint64_t *K = sk + so;
    uint32_t *V = sv + so;
    for (uint32_t i = threadIdx.x; i < P; i += kT) {
        if (i < sg.y) { K[i] = keys[sg.x + i]; V[i] = vals[sg.x + i]; }
        else { K[i] = 0; V[i] = 0xFFFFFFFFu; }
    }
    __syncthreads();
    for (uint32_t kk = 2; kk <= P; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += kT) {
                uint32_t l = i ^ j;
                if (l > i) {
                    bool up = (i & kk) == 0;
                    uint32_t vi = V[i], vl = V[l];
                    bool sw = up ? tie_less(recs, off, vl, vi) : tie_less(recs, off, vi, vl);
                    if (sw) {
                        V[i] = vl; V[l] = vi;
                        uint64_t t = K[i]; K[i] = K[l]; K[l] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < sg.y; i += kT) {
        keys[sg.x + i] = K[i];
        vals[sg.x + i] = V[i];
    }
}

__global__ __launch_bounds__(kT) void k_sizes_from_keys(const uint64_t *__restrict__ keys, uint64_t n,
                                                         uint64_t *__restrict__ sizes) {
    uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (p < n) sizes[p] = keys[p] >> 50;
    else if (p == n) sizes[p] = 0;
}

__global__ __launch_bounds__(kT) void k_sizes_from_perm(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                         const uint32_t *__restrict__ perm, uint64_t n,
                                                         uint64_t *__restrict__ sizes) {
    uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (p < n) sizes[p] = 4ull + oge_rd_u32(recs + off[perm[p]]);
    else if (p == n) sizes[p] = 0;
}

// One wave per record: dword-granular copy with funnel shifts for any src/dst alignment, byte
// stores only on the two edge dwords shared with neighbouring records.  The bin field (record
// bytes 14-15) is replaced by the recomputed bin as BamSerializer::write does.
__global__ __launch_bounds__(kT) void k_gather_records(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                        const uint32_t *__restrict__ perm, uint64_t n,
                                                        uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * kT + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * kT) >> 6;
    for (uint64_t rec = wave; rec < n; rec += nwaves) {
        const uint8_t *src = recs + off[perm[rec]];
        const uint64_t d0 = out_off[rec];
        const uint64_t len = out_off[rec + 1] - d0;
        uint32_t bin = 0;
        if (lane == 0) bin = oge_rec_bin(src);
        bin = __shfl(bin, 0, 64);
        const uint64_t a0 = d0 & ~3ull;
        const uint64_t dend = d0 + len;
        const uint64_t nwords = (((dend + 3) & ~3ull) - a0) >> 2;
        const uintptr_t sbase = (uintptr_t)src;
        for (uint64_t w = lane; w < nwords; w += 64) {
            const uint64_t A = a0 + 4 * w;
            if (A >= d0 && A + 4 <= dend) {
                const uint64_t ro = A - d0;  // record byte offset of this dword
                const uintptr_t s = sbase + ro;
                const uint32_t sh = (uint32_t)(s & 3);
                const uint32_t *sp = (const uint32_t *)(s & ~(uintptr_t)3);
                uint32_t lo = sp[0];
                uint32_t v = lo;
                if (sh) {
                    uint32_t hi = sp[1];
                    v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
                }
                if (ro <= 15 && ro + 4 > 14) {
#pragma unroll
                    for (uint32_t b = 0; b < 4; ++b) {
                        uint64_t x = ro + b;
                        if (x == 14 || x == 15) {
                            uint32_t byte = (x == 14) ? (bin & 0xff) : ((bin >> 8) & 0xff);
                            v = (v & ~(0xffu << (8 * b))) | (byte << (8 * b));
                        }
                    }
                }
                *(uint32_t *)(out + A) = v;
            } else {
                for (uint64_t x = (A > d0 ? A : d0); x < A + 4 && x < dend; ++x) {
                    uint64_t ro = x - d0;
                    uint8_t byte = src[ro];
                    if (ro == 14) byte = (uint8_t)(bin & 0xff);
                    if (ro == 15) byte = (uint8_t)(bin >> 8);
                    out[x] = byte;
                }
            }
        }
    }
}

}  // namespace

// Sort keys/vals for records; on return *kout/*vout hold the sorted (key, input index) pairs.
int oge_sort_keys_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                      uint64_t **kout, uint32_t **vout) {
    if (n_ref < 0 || n_ref >= (1 << 17)) return oge_fail(ctx, OGE_ERR_LIMIT, "sort: n_ref outside [0, 131072)");
    if (n > 0xFFFFFFFEull) return oge_fail(ctx, OGE_ERR_LIMIT, "sort: more than 2^32-2 records");
    uint64_t *keys = (uint64_t *)ctx->ws("sort_keys", (n + 1) * 8);
    uint32_t *vals = (uint32_t *)ctx->ws("sort_vals", (n + 1) * 4);
    uint64_t *ktmp = (uint64_t *)ctx->ws("sort_ktmp", (n + 1) * 8);
    uint32_t *vtmp = (uint32_t *)ctx->ws("sort_vtmp", (n + 1) * 4);
    unsigned int *counts = (unsigned int *)ctx->ws("sort_counts", 16);
    if (!keys || !vals || !ktmp || !vtmp || !counts) return OGE_ERR_HIP;
    OgeStageTimer *t = ctx->begin_stage("sort_keypack");
    OGE_HIP_TRY(ctx, hipMemsetAsync(counts, 0, 16, ctx->stream));
    if (n) {
        hipLaunchKernelGGL(k_keypack, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, n, n_ref, keys,
                           vals, counts + 2);
        OGE_LAUNCH_CHECK(ctx);
    }
    ctx->end_stage(t);
    uint64_t o = 0, a = 0;
    int rc = oge_reduce_or_and_u64(ctx, keys, n, kSortKeyMask, &o, &a);
    if (rc) return rc;
    unsigned int bad = 0;
    OGE_HIP_TRY(ctx, hipMemcpy(&bad, counts + 2, 4, hipMemcpyDeviceToHost));
    if (bad & 1) return oge_fail(ctx, OGE_ERR_ARG, "sort: record with refID outside [-1, n_ref) or pos < -1");
    if (bad & 2) return oge_fail(ctx, OGE_ERR_ARG, "sort: record block_size outside [32, 10000] (util/bam_deserializer.h:160)");
    t = ctx->begin_stage("sort_radix");
    rc = oge_radix_sort_pairs(ctx, keys, vals, ktmp, vtmp, n, (o ^ a) & kSortKeyMask, kout, vout);
    if (rc) return rc;
    ctx->end_stage(t);

    // equal-coordinate runs -> (name, flag, index) order
    t = ctx->begin_stage("sort_ties");
    uint2 *small = (uint2 *)ctx->ws("sort_small", (n / 2 + 1) * sizeof(uint2));
    uint2 *large = (uint2 *)ctx->ws("sort_large", (n / 33 + 1) * sizeof(uint2));
    if (!small || !large) return OGE_ERR_HIP;
    if (n > 1) {
        hipLaunchKernelGGL(k_find_ties, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)*kout, n,
                           n_ref, small, large, counts);
        OGE_LAUNCH_CHECK(ctx);
    }
    unsigned int cnt[2];
    OGE_HIP_TRY(ctx, hipMemcpyAsync(cnt, counts, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (cnt[0]) {
        hipLaunchKernelGGL(k_tie_small, dim3(oge_ceil_div(cnt[0], kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, *kout,
                           *vout, (const uint2 *)small, cnt[0]);
        OGE_LAUNCH_CHECK(ctx);
    }
    if (cnt[1]) {
        std::vector<uint2> h(cnt[1]);
        OGE_HIP_TRY(ctx, hipMemcpy(h.data(), large, cnt[1] * sizeof(uint2), hipMemcpyDeviceToHost));
        std::vector<uint64_t> so(cnt[1]);
        uint64_t tot = 0;
        for (unsigned i = 0; i < cnt[1]; ++i) {
            uint64_t P = 1;
            while (P < h[i].y) P <<= 1;
            so[i] = tot;
            tot += P;
        }
        uint64_t *dso = (uint64_t *)ctx->ws("sort_large_off", cnt[1] * 8);
        uint64_t *sk = (uint64_t *)ctx->ws("sort_large_k", tot * 8);
        uint32_t *sv = (uint32_t *)ctx->ws("sort_large_v", tot * 4);
        if (!dso || !sk || !sv) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dso, so.data(), cnt[1] * 8, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_tie_large, dim3(cnt[1]), dim3(kT), 0, ctx->stream, d_recs, d_off, *kout, *vout,
                           (const uint2 *)large, (const uint64_t *)dso, sk, sv);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->end_stage(t);
    return OGE_OK;
}

int oge_gather_with_sizes(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, const uint32_t *d_perm,
                          const uint64_t *sorted_keys, uint64_t n, uint8_t *d_out, uint64_t *d_out_off) {
    OgeStageTimer *t = ctx->begin_stage("gather_offsets");
    if (sorted_keys)
        hipLaunchKernelGGL(k_sizes_from_keys, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, sorted_keys, n,
                           d_out_off);
    else
        hipLaunchKernelGGL(k_sizes_from_perm, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off,
                           d_perm, n, d_out_off);
    OGE_LAUNCH_CHECK(ctx);
    int rc = oge_exclusive_scan_u64(ctx, d_out_off, d_out_off, n + 1);
    if (rc) return rc;
    ctx->end_stage(t);
    if (!n) return OGE_OK;
    t = ctx->begin_stage("gather_records");
    uint32_t blocks = (uint32_t)std::min<uint64_t>(oge_ceil_div(n, kT / 64), 256u * 32u);
    hipLaunchKernelGGL(k_gather_records, dim3(blocks), dim3(kT), 0, ctx->stream, d_recs, d_off, d_perm, n, d_out,
                       (const uint64_t *)d_out_off);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    return OGE_OK;
}
