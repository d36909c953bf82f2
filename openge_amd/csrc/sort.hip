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
#include "dev_util.h"
#include "records.h"

#include <algorithm>
#include <vector>

unsigned int *oge_sort_counts(oge_ctx *ctx);

namespace {

constexpr uint64_t kSortKeyMask = OGE_SORT_KEY_MASK;
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

// (name, flag, index) order of two records from their sorted summaries: the 32-byte name slots
// (NUL-terminated, zero-padded: byte order of the slots = std::string order of the names) when
// both names fit; the record bytes otherwise, and for the flag when the names are equal.
__device__ __forceinline__ bool tie_less_meta(const uint8_t *__restrict__ recs, const RecMeta &A, const RecMeta &B,
                                              uint32_t ia, uint32_t ib) {
    if (A.m & B.m & OGE_M_NAMEFIT) {
        const uint32_t *x = (const uint32_t *)A.name, *y = (const uint32_t *)B.name;
#pragma unroll
        for (int q = 0; q < OGE_NAME_SLOT / 4; ++q) {
            if (x[q] != y[q]) return __builtin_bswap32(x[q]) < __builtin_bswap32(y[q]);
        }
        const uint16_t fa = oge_rd_u16(recs + A.src + OGE_OFF_FLAG), fb = oge_rd_u16(recs + B.src + OGE_OFF_FLAG);
        if (fa != fb) return fa < fb;
        return ia < ib;
    }
    const uint8_t *ra = recs + A.src, *rb = recs + B.src;
    uint32_t la = ra[OGE_OFF_LNAME], lb = rb[OGE_OFF_LNAME];
    uint32_t m = la < lb ? la : lb;
    for (uint32_t i = 0; i < m; ++i) {
        const uint8_t u = ra[OGE_OFF_NAME + i], v = rb[OGE_OFF_NAME + i];
        if (u != v) return u < v;
    }
    if (la != lb) return la < lb;
    const uint16_t fa = oge_rd_u16(ra + OGE_OFF_FLAG), fb = oge_rd_u16(rb + OGE_OFF_FLAG);
    if (fa != fb) return fa < fb;
    return ia < ib;
}

// Tie runs on the output-order summaries.  A block owns a 4096-position tile: it finds the run
// heads of its tile (16 positions per thread, coalesced), collects the small runs (2..32 equal keys)
// in LDS and then sorts them with every lane busy -- one run per lane, rows of a run contiguous.
// Runs longer than 32 are appended to `large` (rare) for k_tie_large.  Keys, input indices and
// rows move together.
constexpr uint32_t kTieTile = 2048;
constexpr uint32_t kTieHalo = 34;  // keys staged past the tile: a run starting in it is seen up to 33 long
// ROWS = false (r06, the gather-fused pipeline): the summaries are not in output order yet; a run's rows are
// read through its input indices (meta_in[vals[p]]) and only keys and indices move -- the rows are gathered
// once, in final order, after the tie sort.
template <bool ROWS>
__global__ __launch_bounds__(kT) void k_ties_meta(const uint8_t *__restrict__ recs, uint64_t *__restrict__ keys,
                                                   uint32_t *__restrict__ vals, RecMeta *__restrict__ smeta, uint64_t n,
                                                   int32_t n_ref, uint2 *__restrict__ large, unsigned int *__restrict__ nlarge,
                                                   const RecMeta *__restrict__ meta_in) {
    // the tile's masked keys with one before and kTieHalo after, staged by coalesced loads (r05: every
    // position read its neighbours and the run's tail from global memory, ~2 ms of the stage at 300M);
    // ~0 marks positions outside [0, n) (a masked key is below 2^50)
    __shared__ uint64_t sk[kTieTile + 1 + kTieHalo];
    __shared__ uint32_t hp[kTieTile / 2];
    __shared__ uint8_t hl[kTieTile / 2];
    __shared__ unsigned int nh;
    if (threadIdx.x == 0) nh = 0;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kTieTile;
    for (uint32_t i = threadIdx.x; i < kTieTile + 1 + kTieHalo; i += kT) {
        const uint64_t q = tile0 + i;  // position q - 1
        sk[i] = (q >= 1 && q - 1 < n) ? (keys[q - 1] & kSortKeyMask) : ~0ull;
    }
    __syncthreads();
    const uint64_t unm = (uint64_t)(uint32_t)n_ref << 33;  // the unmapped run keeps input order
    for (uint32_t j = 0; j < kTieTile / kT; ++j) {
        const uint32_t li = j * kT + threadIdx.x;  // position tile0 + li at sk[li + 1]
        const uint64_t p = tile0 + li;
        uint32_t len = 0;
        if (p + 1 < n) {
            const uint64_t k0 = sk[li + 1];
            if (sk[li] != k0 && sk[li + 2] == k0 && (k0 >> 33) != (unm >> 33)) {
                uint32_t e = li + 3;  // sk index of position p + 2
                while (e < kTieTile + 1 + kTieHalo && e - (li + 1) <= 32 && sk[e] == k0) ++e;
                uint64_t ee = tile0 + e - 1;  // the first position past the run seen so far
                if (ee - p > 32) { while (ee < n && (keys[ee] & kSortKeyMask) == k0) ++ee; }
                len = (uint32_t)(ee - p);
            }
        }
        const bool is_large = len > 32;
        const uint32_t l = oge_wave_append(is_large, nlarge);
        if (is_large) large[l] = make_uint2((uint32_t)p, len);
        if (len >= 2 && len <= 32) {
            const unsigned int h = atomicAdd(&nh, 1u);
            hp[h] = (uint32_t)(p - tile0);
            hl[h] = (uint8_t)len;
        }
    }
    __syncthreads();
    for (uint32_t h = threadIdx.x; h < nh; h += kT) {
        const uint64_t p = tile0 + hp[h];
        const uint32_t len = hl[h];
        uint64_t *k = keys + p;
        uint32_t *v = vals + p;
        RecMeta *M = ROWS ? smeta + p : nullptr;
        if (len == 2) {
            // pairs (92 % of the runs on C2): both rows loaded together, one compare, written back only when
            // they swap.  r05: the insertion sort's row moves were chains of dependent global round trips
            // (the small-run sort was 4.9 of the stage's 7.8 ms at 300M reads).
            const uint32_t va = v[0], vb = v[1];
            const RecMeta A = ROWS ? M[0] : meta_in[va], B = ROWS ? M[1] : meta_in[vb];
            if (tie_less_meta(recs, B, A, vb, va)) {
                const uint64_t ka = k[0], kb = k[1];
                if (ROWS) M[0] = B, M[1] = A;
                v[0] = vb, v[1] = va;
                k[0] = kb, k[1] = ka;
            }
            continue;
        }
        for (uint32_t i = 1; i < len; ++i) {
            const uint32_t vi = v[i];
            const RecMeta mi = ROWS ? M[i] : meta_in[vi];
            const uint64_t ki = k[i];
            int jj = (int)i - 1;
            while (jj >= 0 && tie_less_meta(recs, mi, ROWS ? M[jj] : meta_in[v[jj]], vi, v[jj])) {
                if (ROWS) M[jj + 1] = M[jj];
                v[jj + 1] = v[jj];
                k[jj + 1] = k[jj];
                --jj;
            }
            if (ROWS) M[jj + 1] = mi;
            v[jj + 1] = vi;
            k[jj + 1] = ki;
        }
    }
}

// after k_tie_large re-ordered a long run's input indices: its rows again
__global__ __launch_bounds__(kT) void k_meta_refill(const RecMeta *__restrict__ meta_in, const uint32_t *__restrict__ vals,
                                                     const uint2 *__restrict__ large, RecMeta *__restrict__ smeta) {
    const uint2 L = large[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < L.y; i += kT) smeta[L.x + i] = meta_in[vals[L.x + i]];
}

// One thread per sorted position: a run head with 2..32 equal keys insertion-sorts its run in place
// by (name, flag, index); longer runs go to `large` (rare; one wave-aggregated append).  No
// counter is touched for the common case, so nothing serialises on an atomic.
__global__ __launch_bounds__(kT) void k_ties(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                              uint64_t *__restrict__ keys, uint32_t *__restrict__ vals, uint64_t n,
                                              int32_t n_ref, uint2 *__restrict__ large, unsigned int *__restrict__ nlarge,
                                              bool sort_small) {
    const uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    uint32_t len = 0;
    if (p + 1 < n) {
        const uint64_t k = keys[p] & kSortKeyMask;
        const bool head = (p == 0 || (keys[p - 1] & kSortKeyMask) != k) && (keys[p + 1] & kSortKeyMask) == k &&
                          (k >> 33) != (uint64_t)(uint32_t)n_ref;  // refID == -1 tail keeps input order
        if (head) {
            uint64_t e = p + 2;
            while (e < n && e - p <= 32 && (keys[e] & kSortKeyMask) == k) ++e;
            if (e - p > 32) { while (e < n && (keys[e] & kSortKeyMask) == k) ++e; }
            len = (uint32_t)(e - p);
        }
    }
    const bool is_large = len > 32;
    const uint32_t l = oge_wave_append(is_large, nlarge);
    if (is_large) large[l] = make_uint2((uint32_t)p, len);
    if (len < 2 || len > 32 || !sort_small) return;
    uint64_t *k = keys + p;
    uint32_t *v = vals + p;
    for (uint32_t i = 1; i < len; ++i) {
        const uint32_t vi = v[i];
        const uint64_t ki = k[i];
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

// One workgroup per long run, with the summaries (r06): when every member's name fits its 32-byte slot and
// the run has at most kLongMax members, the (name slot, flag) rows are staged in LDS once and a bitonic sort
// of member positions runs on them -- each compare reads LDS only.  k_tie_large compares through the record
// bytes, a chain of dependent global loads per compare (1.2 ms at 300M C2 reads for ~50 runs of ~1,000
// members at position 0 of the contigs).  Other runs take the k_tie_large path in the same workgroup.
constexpr uint32_t kLongMax = 2048;
__global__ __launch_bounds__(kT) void k_tie_large_meta(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                        uint64_t *__restrict__ keys, uint32_t *__restrict__ vals,
                                                        const uint2 *__restrict__ segs, const uint64_t *__restrict__ scratch_off,
                                                        uint64_t *__restrict__ sk, uint32_t *__restrict__ sv,
                                                        const RecMeta *__restrict__ meta_in) {
    __shared__ uint32_t nm[kLongMax][OGE_NAME_SLOT / 4];  // name slots, bytes in compare order (bswapped words)
    __shared__ uint64_t kk[kLongMax];
    __shared__ uint32_t vv[kLongMax];
    __shared__ uint16_t fl[kLongMax];
    __shared__ uint16_t pm[kLongMax];
    const uint2 sg = segs[blockIdx.x];
    bool fit = sg.y <= kLongMax;
    if (fit) {
        for (uint32_t i = threadIdx.x; i < sg.y; i += kT) {
            const uint32_t v = vals[sg.x + i];
            const RecMeta &M = meta_in[v];
            fit = fit && (M.m & OGE_M_NAMEFIT);
            const uint32_t *w = (const uint32_t *)M.name;
#pragma unroll
            for (uint32_t q = 0; q < OGE_NAME_SLOT / 4; ++q) nm[i][q] = __builtin_bswap32(w[q]);
            fl[i] = oge_rd_u16(recs + M.src + OGE_OFF_FLAG);
            kk[i] = keys[sg.x + i];
            vv[i] = v;
            pm[i] = (uint16_t)i;
        }
    }
    if (!__syncthreads_and(fit)) {  // uniform: the record-byte path
        uint32_t P = 1;
        while (P < sg.y) P <<= 1;
        uint64_t *K = sk + scratch_off[blockIdx.x];
        uint32_t *V = sv + scratch_off[blockIdx.x];
        for (uint32_t i = threadIdx.x; i < P; i += kT) {
            if (i < sg.y) { K[i] = keys[sg.x + i]; V[i] = vals[sg.x + i]; }
            else { K[i] = 0; V[i] = 0xFFFFFFFFu; }
        }
        __syncthreads();
        for (uint32_t k2 = 2; k2 <= P; k2 <<= 1) {
            for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
                for (uint32_t i = threadIdx.x; i < P; i += kT) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const bool up = (i & k2) == 0;
                        const uint32_t vi = V[i], vl = V[l];
                        if (up ? tie_less(recs, off, vl, vi) : tie_less(recs, off, vi, vl)) {
                            V[i] = vl; V[l] = vi;
                            const uint64_t t = K[i]; K[i] = K[l]; K[l] = t;
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
        return;
    }
    uint32_t P = 1;
    while (P < sg.y) P <<= 1;
    for (uint32_t i = sg.y + threadIdx.x; i < P; i += kT) pm[i] = (uint16_t)i;  // pads: after every member
    __syncthreads();
    const uint32_t n = sg.y;
    auto less = [&](uint32_t a, uint32_t b) {  // member a before member b (tie_less_meta's order)
        if (a >= n) return false;
        if (b >= n) return true;
#pragma unroll
        for (uint32_t q = 0; q < OGE_NAME_SLOT / 4; ++q) {
            const uint32_t x = nm[a][q], y = nm[b][q];
            if (x != y) return x < y;
        }
        if (fl[a] != fl[b]) return fl[a] < fl[b];
        return vv[a] < vv[b];
    };
    for (uint32_t k2 = 2; k2 <= P; k2 <<= 1) {
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += kT) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const bool up = (i & k2) == 0;
                    const uint32_t a = pm[i], b = pm[l];
                    if (up ? less(b, a) : less(a, b)) pm[i] = (uint16_t)b, pm[l] = (uint16_t)a;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += kT) {
        const uint32_t s = pm[i];
        keys[sg.x + i] = kk[s];
        vals[sg.x + i] = vv[s];
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

}  // namespace

// Buffers the coordinate sort reads its (key, value) input from.
int oge_sort_buffers(oge_ctx *ctx, uint64_t n, uint64_t **keys, uint32_t **vals) {
    *keys = (uint64_t *)ctx->ws("sort_keys", (n + 1) * 8);
    *vals = (uint32_t *)ctx->ws("sort_vals", (n + 1) * 4);
    return (*keys && *vals) ? OGE_OK : OGE_ERR_HIP;
}

// Sort keys/vals for records; on return *kout/*vout hold the sorted (key, input index) pairs.
// keys_ready: the KEYS pass (records.hip) already filled oge_sort_buffers and the `bad` word.
int oge_meta_gather(oge_ctx *ctx, const RecMeta *in, const uint32_t *perm, uint64_t n, RecMeta *out);

// With meta_in/meta_out, meta_out receives the summaries in output order, and the small tie runs
// are ordered on them (k_ties_meta) instead of on the record bytes.
// With a gather hook (the fused sort + dedup pipeline): the summaries are gathered by hook->fn AFTER the
// tie sort, in final order, instead of by oge_meta_gather before it (see k_ties_meta<false>); meta_out is
// then not written here.
int oge_sort_keys_dev_hook(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                           bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out,
                           const OgeSortGatherHook *hook);
int oge_sort_keys_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                      bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out) {
    return oge_sort_keys_dev_hook(ctx, d_recs, d_off, n, n_ref, keys_ready, kout, vout, meta_in, meta_out, nullptr);
}
int oge_sort_keys_dev_hook(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref,
                           bool keys_ready, uint64_t **kout, uint32_t **vout, const RecMeta *meta_in, RecMeta *meta_out,
                           const OgeSortGatherHook *hook) {
    if (hook && !meta_in) return oge_fail(ctx, OGE_ERR_ARG, "sort: a gather hook needs the input summaries");
    if (n_ref < 0 || n_ref >= (1 << 17)) return oge_fail(ctx, OGE_ERR_LIMIT, "sort: n_ref outside [0, 131072)");
    if (n > 0xFFFFFFFEull) return oge_fail(ctx, OGE_ERR_LIMIT, "sort: more than 2^32-2 records");
    uint64_t *keys;
    uint32_t *vals;
    if (oge_sort_buffers(ctx, n, &keys, &vals)) return OGE_ERR_HIP;
    uint64_t *ktmp = (uint64_t *)ctx->ws("sort_ktmp", (n + 1) * 8);
    uint32_t *vtmp = (uint32_t *)ctx->ws("sort_vtmp", (n + 1) * 4);
    unsigned int *counts = oge_sort_counts(ctx);
    if (!ktmp || !vtmp || !counts) return OGE_ERR_HIP;
    if (!keys_ready) {
        OgeStageTimer *t = ctx->begin_stage("sort_keypack");
        OGE_HIP_TRY(ctx, hipMemsetAsync(counts, 0, 32, ctx->stream));
        if (n) {
            hipLaunchKernelGGL(k_keypack, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, n, n_ref, keys,
                               vals, counts + 2);
            OGE_LAUNCH_CHECK(ctx);
        }
        ctx->end_stage(t);
    }
    // the varying key bits: from the input pass when it reduced them (keys_ready, counts[3] set), else a
    // reduction pass over the keys
    unsigned int c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(c, counts, 32, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const unsigned int bad = c[2];
    uint64_t o = 0, a = 0;
    int rc = 0;
    if (keys_ready && c[3] == 1) {
        o = (uint64_t)c[4] | ((uint64_t)c[5] << 32);
        a = ~((uint64_t)c[6] | ((uint64_t)c[7] << 32));  // AND = complement of the complements' OR
    } else {
        rc = oge_reduce_or_and_u64(ctx, keys, n, kSortKeyMask, &o, &a);
        if (rc) return rc;
    }
    if (bad & 1) return oge_fail(ctx, OGE_ERR_ARG, "sort: record with refID outside [-1, n_ref) or pos < -1");
    if (bad & 2) return oge_fail(ctx, OGE_ERR_ARG, "sort: record block_size outside [32, 10000] (util/bam_deserializer.h:160)");
    OgeStageTimer *t = ctx->begin_stage("sort_radix");
    rc = oge_radix_sort_pairs(ctx, keys, vals, ktmp, vtmp, n, (o ^ a) & kSortKeyMask, kout, vout);
    if (rc) return rc;
    ctx->end_stage(t);

    // equal-coordinate runs -> (name, flag, index) order.  With summaries: gather them first and
    // order the small runs on them (k_ties_meta); long runs on the record bytes (k_tie_large), whose
    // rows are then re-gathered.
    uint2 *large = (uint2 *)ctx->scratch("sort_large", (n / 33 + 1) * sizeof(uint2));
    if (!large) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(counts, 0, 8, ctx->stream));
    if (meta_out && !hook) {
        t = ctx->begin_stage("meta_gather");
        rc = oge_meta_gather(ctx, meta_in, *vout, n, meta_out);
        if (rc) return rc;
        ctx->end_stage(t);
    }
    t = ctx->begin_stage("sort_ties");
    if (n > 1) {
        if (hook)
            hipLaunchKernelGGL(k_ties_meta<false>, dim3(oge_ceil_div(n, kTieTile)), dim3(kT), 0, ctx->stream, d_recs, *kout,
                               *vout, (RecMeta *)nullptr, n, n_ref, large, counts + 1, meta_in);
        else if (meta_out)
            hipLaunchKernelGGL(k_ties_meta<true>, dim3(oge_ceil_div(n, kTieTile)), dim3(kT), 0, ctx->stream, d_recs, *kout,
                               *vout, meta_out, n, n_ref, large, counts + 1, (const RecMeta *)nullptr);
        else
            hipLaunchKernelGGL(k_ties, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, *kout, *vout, n,
                               n_ref, large, counts + 1, true);
        OGE_LAUNCH_CHECK(ctx);
    }
    unsigned int nlarge = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&nlarge, counts + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (nlarge) {
        std::vector<uint2> h(nlarge);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h.data(), large, nlarge * sizeof(uint2), hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        std::vector<uint64_t> so(nlarge);
        uint64_t tot = 0;
        for (unsigned i = 0; i < nlarge; ++i) {
            uint64_t P = 1;
            while (P < h[i].y) P <<= 1;
            so[i] = tot;
            tot += P;
        }
        uint64_t *dso = (uint64_t *)ctx->scratch("sort_large_off", nlarge * 8);
        uint64_t *sk = (uint64_t *)ctx->scratch("sort_large_k", tot * 8);
        uint32_t *sv = (uint32_t *)ctx->scratch("sort_large_v", tot * 4);
        if (!dso || !sk || !sv) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dso, so.data(), nlarge * 8, hipMemcpyHostToDevice, ctx->stream));
        if (meta_in)
            hipLaunchKernelGGL(k_tie_large_meta, dim3(nlarge), dim3(kT), 0, ctx->stream, d_recs, d_off, *kout, *vout,
                               (const uint2 *)large, (const uint64_t *)dso, sk, sv, meta_in);
        else
            hipLaunchKernelGGL(k_tie_large, dim3(nlarge), dim3(kT), 0, ctx->stream, d_recs, d_off, *kout, *vout,
                               (const uint2 *)large, (const uint64_t *)dso, sk, sv);
        OGE_LAUNCH_CHECK(ctx);
        if (meta_out && !hook) {
            hipLaunchKernelGGL(k_meta_refill, dim3(nlarge), dim3(kT), 0, ctx->stream, meta_in, (const uint32_t *)*vout,
                               (const uint2 *)large, meta_out);
            OGE_LAUNCH_CHECK(ctx);
        }
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->end_stage(t);
    if (hook) {
        t = ctx->begin_stage("meta_gather");
        if ((rc = hook->fn(hook->user, ctx, *vout, *kout))) return rc;
        ctx->end_stage(t);
    }
    return OGE_OK;
}

// [1] long tie runs, [2] bad-record bits, [3] keyred written, [4..8) the input pass's key OR / complement OR
unsigned int *oge_sort_counts(oge_ctx *ctx) { return (unsigned int *)ctx->ws("sort_counts", 32); }

// Output offsets (from the size payload of the sorted keys, or from the records) and the gather.
// smeta (output-order summaries) and dup are optional (see OgePassArgs).
int oge_gather_with_sizes(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, const uint32_t *d_perm,
                          const uint64_t *sorted_keys, uint64_t n, uint8_t *d_out, uint64_t *d_out_off,
                          const RecMeta *smeta, const uint8_t *d_dup, const uint64_t *desc, unsigned int *ndup) {
    OgeStageTimer *t = ctx->begin_stage("gather_offsets");
    // the sizes straight from the sorted keys' payload inside the scan (r05: a sizes kernel first, 0.8 ms)
    int rc = sorted_keys ? oge_offsets_from_keys(ctx, sorted_keys, n, d_out_off) : 1;
    if (rc < 0) return rc;
    if (rc) {
        if (sorted_keys)
            hipLaunchKernelGGL(k_sizes_from_keys, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, sorted_keys, n,
                               d_out_off);
        else
            hipLaunchKernelGGL(k_sizes_from_perm, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off,
                               d_perm, n, d_out_off);
        OGE_LAUNCH_CHECK(ctx);
        rc = oge_exclusive_scan_u64(ctx, d_out_off, d_out_off, n + 1);
        if (rc) return rc;
    }
    ctx->end_stage(t);
    if (!n) return OGE_OK;
    t = ctx->begin_stage("gather_records");
    OgePassArgs a = {};
    a.recs = d_recs;
    a.off = d_off;
    a.perm = d_perm;
    a.n = n;
    a.out = d_out;
    a.out_off = d_out_off;
    a.smeta = desc ? nullptr : smeta;
    a.dup = desc && !ndup ? nullptr : d_dup;
    a.desc = desc;
    a.ndup = desc ? ndup : nullptr;
    rc = oge_gather_pass(ctx, a);
    if (rc) return rc;
    ctx->end_stage(t);
    return OGE_OK;
}
