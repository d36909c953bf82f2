// md_keys.h -- the per-record key words of the device MarkDuplicates, shared by markdup.hip (the summary
// passes) and records.hip (the in-place dedup's input pass, which derives them from the summary it has just
// built instead of re-reading it).  See markdup.hip for where each word is consumed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "records.h"

namespace {

// --- compaction of pair candidates (order-preserving) ---
// candidate key = top hb bits of the 48-bit pair-key hash << ib | record index (ib = bits for an
// index, hb = min(48, 64 - ib)): the hash takes every key bit the index leaves free, so collision
// runs (which fall to the exact slow path of k_pair_runs) stay rare at full-GPU sizes.  Only the hash
// bits are radix-sorted; the stable LSD sort keeps record order inside a hash run (the
// ReadEndsMap's first/second-seen).
struct CandKey {
    uint32_t ib, hb;
    int32_t split_k;
    __host__ __device__ uint64_t idx_mask() const { return (1ull << ib) - 1; }
    __host__ __device__ uint64_t hash_of(uint64_t k) const { return k >> ib; }
};

struct KeyLayout {
    uint32_t sb, lb;  // bits for refID and library id
    int32_t split_k;
};

// ---- windowed grouping support (records in ByPosition order, one GPU) ----
// A record's 5' coordinate (its fragment / pair group coordinate) lies within a few read lengths of
// its sort position, so in sorted order every group's members sit inside a short window.  Positions
// are compared as X(ref, v) = ref * 2^34 + v + 2^32 (v = pos + 1 or 5' coordinate + 1, |v| < 2^32).
__device__ __forceinline__ int64_t win_x(uint32_t ref, int64_t v) { return ((int64_t)ref << 34) + v + (1ll << 32); }
// the anchor of a sorted record: (refID', pos + 1) of its coordinate sort key (records.hip)
__device__ __forceinline__ int64_t anchor_of_key(uint64_t k) {
    return win_x((uint32_t)(k >> 33) & 0x1ffffu, (int64_t)((k >> 1) & 0xffffffffu));
}
constexpr int64_t kDevBias = 1ll << 40;  // deviations are kept as D + 2^40 (0 = none seen)
// fragment key: bit 63 paired, bits [47,63) score, bit 46 "not a fragment",
// lib << (sb+33) | refID << 33 | biased coord << 1 | reverse
__device__ __forceinline__ uint64_t frag_key(const RecMeta &R, KeyLayout L) {
    const uint64_t m = R.m;
    uint64_t k;
    if (!(m & OGE_M_FRAG)) {
        k = 1ull << 46;
    } else {
        const uint64_t lib = (m >> 16) & 0xFFFF;
        k = (lib << (L.sb + 33)) | ((uint64_t)(uint32_t)R.seq << 33) | ((uint64_t)((uint32_t)R.coord ^ 0x80000000u) << 1) |
            ((m & OGE_M_REV) ? 1ull : 0ull);
        k |= ((m & 0xFFFF) << 47) | ((m & OGE_M_PAIRED) ? (1ull << 63) : 0ull);
    }
    return k;
}


// the products of record i from its summary (only the first 32 bytes of R are read: m, src, seq, coord, hash)
__device__ __forceinline__ void cand_frag_one(const RecMeta &R, uint64_t i, KeyLayout L, CandKey ck, uint32_t *__restrict__ f,
                                              uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                              uint64_t *__restrict__ cval, uint64_t *__restrict__ desc0,
                                              unsigned int *__restrict__ ovf, const uint64_t *__restrict__ skeys, bool &has,
                                              int64_t &ax, int64_t &cx) {
    f[i] = (R.m & OGE_M_CAND) ? 1u : 0u;
    keys[i] = frag_key(R, L);
    vals[i] = (uint32_t)i;
    cval[i] = ((oge_meta_hash48(R) >> (48 - ck.hb)) << ck.ib) | i;
    if (desc0) {
        if (R.src >> 39) atomicOr(ovf, 1u);
        desc0[i] = (R.src & ((1ull << 39) - 1)) | ((R.m & OGE_M_PRIMARY) ? (1ull << 39) : 0ull) |
                   ((R.m >> 48) << 40) | (((R.m >> 40) & 0xff) << 56);
    }
    if (skeys && (R.m & OGE_M_FRAG)) {
        has = true;
        ax = anchor_of_key(skeys[i]);
        cx = win_x((uint32_t)R.seq, (int64_t)R.coord + 1);
    }
}

// Per-thread maxima of (anchor - coordinate + 2^40) and (coordinate - anchor + 2^40) into slot
// (blockIdx & 255) of dev[0..511] (pairs of words), reduced over the block first.  Every thread of the block
// calls it (barriers inside).
__device__ __forceinline__ void md_dev_slots(uint64_t d0, uint64_t d1, unsigned long long *dev) {
    __shared__ uint64_t wd[2][16];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o0 = ((uint64_t)__shfl_xor((unsigned)(d0 >> 32), d, 64) << 32) | (uint64_t)__shfl_xor((unsigned)d0, d, 64);
        const uint64_t o1 = ((uint64_t)__shfl_xor((unsigned)(d1 >> 32), d, 64) << 32) | (uint64_t)__shfl_xor((unsigned)d1, d, 64);
        d0 = o0 > d0 ? o0 : d0;
        d1 = o1 > d1 ? o1 : d1;
    }
    if ((threadIdx.x & 63) == 0) wd[0][threadIdx.x >> 6] = d0, wd[1][threadIdx.x >> 6] = d1;
    __syncthreads();
    if (threadIdx.x < 2) {
        uint64_t m = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) m = max(m, wd[threadIdx.x][w]);
        if (m) atomicMax(dev + 2 * (blockIdx.x & 255) + threadIdx.x, (unsigned long long)m);
    }
}

}  // namespace
