// sort_name.hip -- mergesort -b: records in Sort::ByName order (util/bamtools/Sort.h:67-90, used by
// ReadSorter for SORT_QUERYNAME, algorithms/read_sorter.cpp:202-203).
//
// std::string operator< on the read names is an unsigned bytewise compare with "shorter prefix
// first"; names never contain NUL, so it equals the compare of the names zero-padded to a common
// length.  The sort is an LSD radix sort over the padded name read as big-endian u64 words, last
// word first: each word pass packs word w of every record (in the current order) into a key and
// runs the stable pair radix sort (prims.hip) on the key bits that vary, so the final order is
// lexicographic with ties (mates share a name) in input order.  Words that are equal over all
// records cost only the key pack.  HBM per word pass: the key pack touches one name line per record
// plus 12 B/record of key + index, and the radix passes move 12 B/record per 8 varying bits.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bam_layout.h"
#include "oge_ctx.h"

namespace {

__global__ void k_name_maxlen(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                              uint32_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t l = i < n ? recs[off[i] + OGE_OFF_LNAME] : 0u;
    for (int s = 32; s > 0; s >>= 1) l = max(l, (uint32_t)__shfl_xor((int)l, s));
    if ((threadIdx.x & 63) == 0 && l) atomicMax(out, l);
}

__global__ void k_iota(uint32_t *__restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// key[i] = bytes [8w, 8w + 8) of the name of record idx[i], big-endian, zero past the name's end
// (l_read_name counts the NUL, bam_layout.h).
__global__ void k_name_word(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                            const uint32_t *__restrict__ idx, uint64_t n, uint32_t w, uint64_t *__restrict__ key) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[idx ? idx[i] : i];
    const int32_t len = (int32_t)r[OGE_OFF_LNAME] - 1;
    const uint8_t *nm = r + OGE_OFF_NAME;
    uint64_t k = 0;
    const int32_t b0 = 8 * (int32_t)w;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint64_t c = b0 + b < len ? nm[b0 + b] : 0;
        k |= c << (56 - 8 * b);
    }
    key[i] = k;
}

}  // namespace

extern "C" int oge_sort_name_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, uint32_t *d_perm) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (n && (!d_recs || !d_off || !d_perm)) return oge_fail(ctx, OGE_ERR_ARG, "null buffer");
    if (n >= 0xffffffffull) return oge_fail(ctx, OGE_ERR_ARG, "too many records");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    if (!n) return OGE_OK;
    uint32_t *dmax = (uint32_t *)ctx->ws("name_maxlen", 16);
    uint64_t *keys = (uint64_t *)ctx->ws("name_keys", n * 8);
    uint64_t *ktmp = (uint64_t *)ctx->ws("name_ktmp", n * 8);
    uint32_t *vtmp = (uint32_t *)ctx->ws("name_vtmp", n * 4);
    if (!dmax || !keys || !ktmp || !vtmp) return OGE_ERR_HIP;
    OgeStageTimer *t = ctx->begin_stage("name_sort");
    OGE_HIP_TRY(ctx, hipMemsetAsync(dmax, 0, 4, ctx->stream));
    k_name_maxlen<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_recs, d_off, n, dmax);
    OGE_LAUNCH_CHECK(ctx);
    k_iota<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_perm, n);
    OGE_LAUNCH_CHECK(ctx);
    uint32_t maxlen = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&maxlen, dmax, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t words = maxlen > 1 ? (maxlen - 1 + 7) / 8 : 0;
    uint32_t *vals = d_perm;
    bool identity = true;  // vals still equals iota: the key pack can walk the records in order
    for (uint32_t w = words; w-- > 0;) {
        k_name_word<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_recs, d_off, identity ? nullptr : vals, n, w, keys);
        OGE_LAUNCH_CHECK(ctx);
        uint64_t o = 0, a = 0;
        int rc = oge_reduce_or_and_u64(ctx, keys, n, ~0ull, &o, &a);
        if (rc) return rc;
        if (!(o ^ a)) continue;  // this word is the same in every name
        uint64_t *ko = keys;
        uint32_t *vo = vals;
        rc = oge_radix_sort_pairs(ctx, keys, vals, ktmp, vals == d_perm ? vtmp : d_perm, n, o ^ a, &ko, &vo);
        if (rc) return rc;
        if (vo != vals) {  // ping-pong between d_perm and vtmp
            vtmp = vals;
            vals = vo;
        }
        identity = false;
    }
    if (vals != d_perm) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_perm, vals, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
    ctx->end_stage(t);
    return OGE_OK;
}
