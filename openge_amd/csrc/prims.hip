// prims.hip -- device primitives for gfx950: exclusive scans, OR/AND reduction, and a stable
// LSD radix sort of (u64 key, u32 value) pairs with wave64 ballot-based digit ranking.
//
// Radix pass anatomy (reduce-then-scan, three launches per digit):
//   1. k_radix_hist   : each 256-thread block ranks one 4096-key tile, per-wave LDS histograms
//   2. exclusive scan : over the digit-major [digit][block] count matrix
//   3. k_radix_scatter: re-reads the tile, ranks every key stably inside its wave with 64-lane
//                       __ballot peer masks (one ballot per digit bit), prefix-sums the per-wave
//                       counts in LDS and scatters (key, value) to its global slot.
// Tile order is (wave, item j, lane) -> index = tile + wave*1024 + j*64 + lane, so global loads
// are 512-byte coalesced per wave instruction and ranks follow input order (stability).
#include "oge_ctx.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;  // 4096 keys per block

constexpr int kScanItems = 8;
constexpr int kScanTile = kThreads * kScanItems;  // 2048 values per block

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T t = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += t;
    }
    return v;
}

// Exclusive block-wide scan of one value per thread; *total gets the block sum.
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, T *total) {
    __shared__ T wsum[kWaves];
    const uint32_t w = threadIdx.x >> 6;
    T inc = wave_incl_scan(v);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {
        T s = wsum[i];
        if ((uint32_t)i < w) off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

template <class T>
__global__ __launch_bounds__(kThreads) void k_scan_tiles(const T *__restrict__ in, T *__restrict__ out, uint64_t n,
                                                          T *__restrict__ sums) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        uint64_t idx = base + i;
        v[i] = idx < n ? in[idx] : (T)0;
        s += v[i];
    }
    T total;
    T run = block_excl_scan(s, &total);
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        uint64_t idx = base + i;
        if (idx < n) out[idx] = run;
        run += v[i];
    }
    if (threadIdx.x == 0 && sums) sums[blockIdx.x] = total;
}

template <class T>
__global__ __launch_bounds__(kThreads) void k_scan_add(T *__restrict__ out, uint64_t n, const T *__restrict__ sums) {
    const T add = sums[blockIdx.x];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        uint64_t idx = base + (uint64_t)i * kThreads + threadIdx.x;
        if (idx < n) out[idx] += add;
    }
}

// Reduce-then-scan over 16-byte chunks (r05; in and out 16-byte aligned): a block owns 1024 chunks
// (16 KiB: 4096 u32 / 2048 u64), lane l of wave w the chunks w*256 + j*64 + l (j < 4), so every load and
// store instruction of a wave covers 1 KiB contiguously.  k_scanv_reduce reads the tile and writes its sum;
// k_scanv_down reads it again, scans it in registers (a wave scan over the lanes per j, then the waves) and
// writes it with the tile's offset: 3n element moves and full 16-byte lanes, against 4n for k_scan_tiles +
// k_scan_add with each thread's 8 elements in 8 narrow loads (300M u32: 1.55 ms).  A chunk that ends past n
// is read and written element by element.
constexpr int kVJ = 4;                      // chunks per lane
constexpr int kVTile = kThreads * kVJ;      // chunks per block

// SH: the element is in[i] >> SH (SH = 50: a sort key's record-size payload, sort.hip); elements at or past
// n_in read as 0
template <class T, int SH = 0>
__device__ __forceinline__ void load_chunk(const T *__restrict__ in, uint64_t c, uint64_t n_in, T (&v)[16 / sizeof(T)]) {
    constexpr int E = 16 / sizeof(T);
    const uint64_t e0 = c * E;
    if (e0 + E <= n_in) {
        const uint4 q = *(const uint4 *)(in + e0);
        __builtin_memcpy(v, &q, 16);
    } else {
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] = e0 + k < n_in ? in[e0 + k] : (T)0;
    }
    if (SH) {
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] >>= SH;
    }
}

template <class T, int SH = 0>
__global__ __launch_bounds__(kThreads) void k_scanv_reduce(const T *__restrict__ in, uint64_t n_in, T *__restrict__ sums) {
    constexpr int E = 16 / sizeof(T);
    const uint64_t c0 = (uint64_t)blockIdx.x * kVTile + (threadIdx.x >> 6) * 256 + lane_id();
    T s = 0;
#pragma unroll
    for (int j = 0; j < kVJ; ++j) {
        T v[E];
        load_chunk<T, SH>(in, c0 + 64 * j, n_in, v);
#pragma unroll
        for (int k = 0; k < E; ++k) s += v[k];
    }
    T total;
    (void)block_excl_scan(s, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

template <class T, int SH = 0>
__global__ __launch_bounds__(kThreads) void k_scanv_down(const T *in, T *out, uint64_t n, uint64_t n_in, const T *__restrict__ sums) {
    constexpr int E = 16 / sizeof(T);
    __shared__ T wt[kWaves];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint64_t c0 = (uint64_t)blockIdx.x * kVTile + w * 256 + lane;
    T v[kVJ][E], ex[kVJ];
#pragma unroll
    for (int j = 0; j < kVJ; ++j) load_chunk<T, SH>(in, c0 + 64 * j, n_in, v[j]);  // all loads before any store: out may be in
    T run = 0;  // the wave's running total over its stripes j
#pragma unroll
    for (int j = 0; j < kVJ; ++j) {
        T cs = 0;
#pragma unroll
        for (int k = 0; k < E; ++k) cs += v[j][k];
        const T inc = wave_incl_scan(cs);
        ex[j] = run + inc - cs;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) wt[w] = run;
    __syncthreads();
    T off = sums ? sums[blockIdx.x] : (T)0;
    for (uint32_t i = 0; i < w; ++i) off += wt[i];
#pragma unroll
    for (int j = 0; j < kVJ; ++j) {
        const uint64_t e0 = (c0 + 64 * j) * E;
        T o[E];
        T x = off + ex[j];
#pragma unroll
        for (int k = 0; k < E; ++k) o[k] = x, x += v[j][k];
        if (e0 + E <= n) {
            uint4 q;
            __builtin_memcpy(&q, o, 16);
            *(uint4 *)(out + e0) = q;
        } else {
#pragma unroll
            for (int k = 0; k < E; ++k)
                if (e0 + k < n) out[e0 + k] = o[k];
        }
    }
}

template <class T, int SH = 0>
int scanv_impl(oge_ctx *ctx, const T *in, T *out, uint64_t n, uint64_t n_in, int level);

template <class T>
int scan_impl(oge_ctx *ctx, const T *in, T *out, uint64_t n, int level) {
    if (n == 0) return OGE_OK;
    if (!(((uintptr_t)in | (uintptr_t)out) & 15)) return scanv_impl<T>(ctx, in, out, n, n, level);
    uint32_t nb = oge_ceil_div(n, kScanTile);
    if (nb == 1) {
        hipLaunchKernelGGL(k_scan_tiles<T>, dim3(1), dim3(kThreads), 0, ctx->stream, in, out, n, (T *)nullptr);
        OGE_LAUNCH_CHECK(ctx);
        return OGE_OK;
    }
    char name[32];
    snprintf(name, sizeof(name), "scan_sums_%d_%zu", level, sizeof(T));
    T *sums = (T *)ctx->ws(name, (size_t)nb * sizeof(T));
    if (!sums) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3(nb), dim3(kThreads), 0, ctx->stream, in, out, n, sums);
    OGE_LAUNCH_CHECK(ctx);
    int rc = scan_impl<T>(ctx, sums, sums, nb, level + 1);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add<T>, dim3(nb), dim3(kThreads), 0, ctx->stream, out, n, (const T *)sums);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

template <class T, int SH>
int scanv_impl(oge_ctx *ctx, const T *in, T *out, uint64_t n, uint64_t n_in, int level) {
    constexpr uint64_t per = (uint64_t)kVTile * (16 / sizeof(T));
    const uint32_t nb = oge_ceil_div(n, per);
    if (nb == 1) {
        hipLaunchKernelGGL((k_scanv_down<T, SH>), dim3(1), dim3(kThreads), 0, ctx->stream, in, out, n, n_in, (const T *)nullptr);
        OGE_LAUNCH_CHECK(ctx);
        return OGE_OK;
    }
    char name[32];
    snprintf(name, sizeof(name), "scan_sums_%d_%zu", level, sizeof(T));
    T *sums = (T *)ctx->ws(name, (size_t)nb * sizeof(T));
    if (!sums) return OGE_ERR_HIP;
    hipLaunchKernelGGL((k_scanv_reduce<T, SH>), dim3(nb), dim3(kThreads), 0, ctx->stream, in, n_in, sums);
    OGE_LAUNCH_CHECK(ctx);
    int rc = scan_impl<T>(ctx, sums, sums, nb, level + 1);
    if (rc) return rc;
    hipLaunchKernelGGL((k_scanv_down<T, SH>), dim3(nb), dim3(kThreads), 0, ctx->stream, in, out, n, n_in, (const T *)sums);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

// ---------------------------------------------------------------- OR / AND reduction
__global__ __launch_bounds__(kThreads) void k_or_and(const uint64_t *__restrict__ in, uint64_t n, uint64_t mask,
                                                      unsigned long long *res) {
    uint64_t o = 0, a = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads) {
        uint64_t v = in[i] & mask;
        o |= v;
        a &= v;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        o |= __shfl_xor(o, d, 64);
        a &= __shfl_xor(a, d, 64);
    }
    if (lane_id() == 0) {
        atomicOr(&res[0], (unsigned long long)o);
        atomicAnd(&res[1], (unsigned long long)a);
    }
}

// ---------------------------------------------------------------- radix sort
struct Digit {
    uint32_t s0, w0, s1, w1;  // digit = bits [s0, s0+w0) | bits [s1, s1+w1) << w0
};

__device__ __forceinline__ uint32_t digit_of(uint64_t k, const Digit d) {
    uint32_t lo = (uint32_t)(k >> d.s0) & ((1u << d.w0) - 1u);
    uint32_t hi = d.w1 ? ((uint32_t)(k >> d.s1) & ((1u << d.w1) - 1u)) : 0u;
    return lo | (hi << d.w0);
}

template <int NB>
__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint64_t *__restrict__ keys, uint64_t n, Digit dg,
                                                          uint32_t nbins, uint32_t *__restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[kWaves][NB];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    for (uint32_t i = tid; i < kWaves * NB; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)w * (kItems * 64);
#pragma unroll 4
    for (int j = 0; j < kItems; ++j) {
        uint64_t idx = base + (uint64_t)j * 64 + lane;
        if (idx < n) atomicAdd(&h[w][digit_of(keys[idx], dg)], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < nbins; d += kThreads) {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < kWaves; ++i) s += h[i][d];
        hist[(uint64_t)d * nblocks + blockIdx.x] = s;
    }
}

// Stable scatter of one 4096-key tile.  Ranks come from 64-lane ballot peer masks per wave; the
// tile is then re-ordered by digit in LDS so that the global writes of each digit bucket are
// contiguous runs written by consecutive lanes (instead of 16 scattered 8-byte writes per bucket).
template <bool HAS_V, int NB>
__global__ __launch_bounds__(kThreads) void k_radix_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                             uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, uint64_t n,
                                                             Digit dg, uint32_t nbins, const uint32_t *__restrict__ offs,
                                                             uint32_t nblocks) {
    constexpr int DPT = NB / kThreads > 0 ? NB / kThreads : 1;  // digits per thread in the digit scan
    __shared__ uint64_t sk[kTile];
    __shared__ uint32_t sv[HAS_V ? kTile : 1];
    __shared__ uint32_t wcnt[kWaves][NB];
    __shared__ uint32_t dstart[NB];
    __shared__ uint32_t gbase[NB];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t nbits = dg.w0 + dg.w1;
    for (uint32_t i = tid; i < kWaves * NB; i += kThreads) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tile0 = (uint64_t)blockIdx.x * kTile;
    const uint64_t base = tile0 + (uint64_t)w * (kItems * 64);
    const uint64_t lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    uint64_t key[kItems];
    uint32_t val[kItems];
    uint32_t rank[kItems];
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint64_t idx = base + (uint64_t)j * 64 + lane;
        const bool valid = idx < n;
        key[j] = valid ? kin[idx] : 0ull;
        if (HAS_V) val[j] = valid ? vin[idx] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint64_t idx = base + (uint64_t)j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = digit_of(key[j], dg);
        uint64_t peers = __ballot(valid);
        for (uint32_t b = 0; b < nbits; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
        const uint32_t cnt = (uint32_t)__popcll(peers);
        const uint32_t leader = (uint32_t)(__ffsll((long long)peers) - 1);
        const uint32_t prev = valid ? wcnt[w][d] : 0u;
        // all peers of the wave read wcnt[w][d] in the same ds_read before the leader's write
        __builtin_amdgcn_wave_barrier();
        if (valid && lane == leader) wcnt[w][d] = prev + cnt;
        __builtin_amdgcn_wave_barrier();
        rank[j] = prev + below;
    }
    __syncthreads();
    // per digit: tile total -> exclusive scan over digits (block-local bucket starts); thread t owns
    // digits [t*DPT, t*DPT + DPT)
    uint32_t tot[DPT];
    uint32_t tsum = 0;
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const uint32_t d = tid * DPT + k;
        tot[k] = 0;
        if (d < nbins) {
#pragma unroll
            for (int i = 0; i < kWaves; ++i) tot[k] += wcnt[i][d];
        }
        tsum += tot[k];
    }
    uint32_t dummy;
    uint32_t ds = block_excl_scan(tsum, &dummy);
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const uint32_t d = tid * DPT + k;
        if (d < nbins) {
            dstart[d] = ds;
            gbase[d] = offs[(uint64_t)d * nblocks + blockIdx.x];
            uint32_t run = ds;
#pragma unroll
            for (int i = 0; i < kWaves; ++i) {
                const uint32_t c = wcnt[i][d];
                wcnt[i][d] = run;
                run += c;
            }
        }
        ds += tot[k];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint64_t idx = base + (uint64_t)j * 64 + lane;
        if (idx < n) {
            const uint32_t lpos = wcnt[w][digit_of(key[j], dg)] + rank[j];
            sk[lpos] = key[j];
            if (HAS_V) sv[lpos] = val[j];
        }
    }
    __syncthreads();
    const uint32_t cnt_tile = (uint32_t)((n - tile0) < (uint64_t)kTile ? (n - tile0) : (uint64_t)kTile);
    for (uint32_t i = tid; i < cnt_tile; i += kThreads) {
        const uint64_t k = sk[i];
        const uint32_t d = digit_of(k, dg);
        const uint32_t g = gbase[d] + (i - dstart[d]);
        kout[g] = k;
        if (HAS_V) vout[g] = sv[i];
    }
}

std::vector<Digit> plan_digits(uint64_t mask, uint32_t maxw) {
    // contiguous runs of set bits
    std::vector<std::pair<uint32_t, uint32_t>> runs;  // (start, width)
    for (uint32_t b = 0; b < 64;) {
        if (!((mask >> b) & 1)) { ++b; continue; }
        uint32_t s = b;
        while (b < 64 && ((mask >> b) & 1)) ++b;
        runs.push_back({s, b - s});
    }
    uint32_t total = 0;
    for (auto &r : runs) total += r.second;
    std::vector<Digit> out;
    if (!total) return out;
    uint32_t passes = (total + maxw - 1) / maxw;
    uint32_t per = (total + passes - 1) / passes;  // balanced digit width
    size_t ri = 0;
    uint32_t roff = 0;
    while (ri < runs.size()) {
        Digit d = {0, 0, 0, 0};
        uint32_t need = per;
        // field 0
        uint32_t take = std::min(need, runs[ri].second - roff);
        d.s0 = runs[ri].first + roff; d.w0 = take; need -= take; roff += take;
        if (roff == runs[ri].second) { ++ri; roff = 0; }
        // field 1 (next run) if room left
        if (need && ri < runs.size()) {
            take = std::min(need, runs[ri].second - roff);
            d.s1 = runs[ri].first + roff; d.w1 = take; roff += take;
            if (roff == runs[ri].second) { ++ri; roff = 0; }
        }
        out.push_back(d);
    }
    return out;
}

}  // namespace

extern "C" int oge_exclusive_scan_dev(oge_ctx *ctx, const void *d_in, void *d_out, uint64_t n, int elem_bytes) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if ((elem_bytes != 4 && elem_bytes != 8) || (n && (!d_in || !d_out)) || ((uintptr_t)d_in | (uintptr_t)d_out) % elem_bytes)
        return oge_fail(ctx, OGE_ERR_ARG, "oge_exclusive_scan_dev: bad arguments");
    hipSetDevice(ctx->device);
    const int rc = elem_bytes == 4 ? scan_impl<uint32_t>(ctx, (const uint32_t *)d_in, (uint32_t *)d_out, n, 0)
                                   : scan_impl<uint64_t>(ctx, (const uint64_t *)d_in, (uint64_t *)d_out, n, 0);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

int oge_exclusive_scan_u32(oge_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n) {
    return scan_impl<uint32_t>(ctx, in, out, n, 0);
}
int oge_exclusive_scan_u64(oge_ctx *ctx, const uint64_t *in, uint64_t *out, uint64_t n) {
    return scan_impl<uint64_t>(ctx, in, out, n, 0);
}
int oge_offsets_from_keys(oge_ctx *ctx, const uint64_t *keys, uint64_t n, uint64_t *out) {
    if (((uintptr_t)keys | (uintptr_t)out) & 15) return 1;  // the caller takes the two-kernel path
    return scanv_impl<uint64_t, 50>(ctx, keys, out, n + 1, n, 0);
}

int oge_reduce_or_and_u64(oge_ctx *ctx, const uint64_t *in, uint64_t n, uint64_t mask, uint64_t *or_out, uint64_t *and_out) {
    unsigned long long *res = (unsigned long long *)ctx->ws("reduce_or_and", 2 * sizeof(uint64_t));
    if (!res) return OGE_ERR_HIP;
    unsigned long long init[2] = {0ull, ~0ull};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(res, init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
    if (n) {
        uint32_t nb = std::min<uint32_t>(oge_ceil_div(n, kThreads), 2048);
        hipLaunchKernelGGL(k_or_and, dim3(nb), dim3(kThreads), 0, ctx->stream, in, n, mask, res);
        OGE_LAUNCH_CHECK(ctx);
    }
    unsigned long long h[2];
    OGE_HIP_TRY(ctx, hipMemcpyAsync(h, res, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *or_out = h[0];
    *and_out = n ? h[1] : 0;
    return OGE_OK;
}

int oge_radix_sort_pairs(oge_ctx *ctx, uint64_t *keys, uint32_t *vals, uint64_t *ktmp, uint32_t *vtmp, uint64_t n,
                         uint64_t bit_mask, uint64_t **kout, uint32_t **vout) {
    *kout = keys;
    if (vout) *vout = vals;
    if (n < 2 || bit_mask == 0) return OGE_OK;
    if (n > 0xFFFFFFFFull) return oge_fail(ctx, OGE_ERR_LIMIT, "radix sort: more than 2^32-1 elements");
    const bool has_v = vals != nullptr;
    // widest digit 8 bits: the measured optimum on C2 at 300M reads (r01: 9- and 10-bit digits save
    // passes but every 4096-key tile then spreads over 512/1024 buckets, the scatter's per-bucket runs
    // shrink below a cache line, and the step got slower: 185 -> 192 / 196 ms)
    constexpr uint32_t maxw = 8;
    std::vector<Digit> digits = plan_digits(bit_mask, maxw);
    const uint32_t nblocks = oge_ceil_div(n, kTile);
    uint32_t *hist = (uint32_t *)ctx->ws("radix_hist", (size_t)1024 * nblocks * sizeof(uint32_t));
    if (!hist) return OGE_ERR_HIP;
    uint64_t *ka = keys, *kb = ktmp;
    uint32_t *va = vals, *vb = vtmp;
    for (const Digit &d : digits) {
        const uint32_t nbins = 1u << (d.w0 + d.w1);
        auto pass = [&](auto nb_tag) -> int {
            constexpr int NB = decltype(nb_tag)::value;
            hipLaunchKernelGGL(k_radix_hist<NB>, dim3(nblocks), dim3(kThreads), 0, ctx->stream, (const uint64_t *)ka, n, d,
                               nbins, hist, nblocks);
            OGE_LAUNCH_CHECK(ctx);
            int rc = oge_exclusive_scan_u32(ctx, hist, hist, (uint64_t)nbins * nblocks);
            if (rc) return rc;
            if (has_v)
                hipLaunchKernelGGL((k_radix_scatter<true, NB>), dim3(nblocks), dim3(kThreads), 0, ctx->stream,
                                   (const uint64_t *)ka, (const uint32_t *)va, kb, vb, n, d, nbins, (const uint32_t *)hist,
                                   nblocks);
            else
                hipLaunchKernelGGL((k_radix_scatter<false, NB>), dim3(nblocks), dim3(kThreads), 0, ctx->stream,
                                   (const uint64_t *)ka, (const uint32_t *)nullptr, kb, (uint32_t *)nullptr, n, d, nbins,
                                   (const uint32_t *)hist, nblocks);
            OGE_LAUNCH_CHECK(ctx);
            return OGE_OK;
        };
        int rc = nbins <= 256   ? pass(std::integral_constant<int, 256>())
                 : nbins <= 512 ? pass(std::integral_constant<int, 512>())
                                : pass(std::integral_constant<int, 1024>());
        if (rc) return rc;
        std::swap(ka, kb);
        std::swap(va, vb);
    }
    *kout = ka;
    if (vout) *vout = va;
    return OGE_OK;
}
