// realign.hip -- local-realignment offset scan on gfx950 and the realign C-ABI entry points.
//
// The reference's hot loop is LocalRealignment::findBestOffset (algorithms/local_realignment.cpp:
// 1126-1164) calling mismatchQualitySumIgnoreCigar (:641-679) for every offset of every altRead
// against every alternate consensus.  It is an ungapped sliding mismatch-quality sum (the reference
// has no Smith-Waterman).  Score of read r at consensus offset k:
//     S(k) = sum_{i < L, k+i < C} [both bases regular, bases differ] * w_i  +  99 * #{i : k+i >= C}
// with w_i = (signed char)(q_i + 33) - 33 (qualities are kept as ASCII chars), "regular" =
// ACGTacgt* (BaseUtils::isRegularBase).  findBestOffset visits offsets in the order
// orig, 0..orig-1, orig+1..maxStart and keeps strict improvements (returning at the first 0), so
// while every weight is >= 0 its answer is the minimum of (score, visit rank) -- early exits never
// change it.  A quality >= 95 makes its weight negative; such reads take the literal scan (lit_best).
//
// Kernels.  k_planes turns every consensus and altRead into bit planes, 64 positions per word
// (wave ballots): base-code bits b0,b1 and a "regular base" mask v; for reads also the 7 bit planes
// of the weight.  k_scan_bp then gives each (consensus, read) pair one wave; lane l owns offsets
// k = 64a + l, so its consensus window is a fixed l-bit funnel shift of consecutive plane words, and
// the plane words every lane needs are the same (scalar loads).  Per 64 read positions and offset:
//     m = win(v) & rv & ((win(b0) ^ r0) | (win(b1) ^ r1));   S += sum_b popcount(m & W_b) << b
// (~50 VALU ops instead of ~450 byte-wise).  A wave min-reduction over the packed (score, rank) key
// gives the answer.  Integer VALU bound; no MFMA (no dense contraction), no LDS.
// k_realign_scan (byte-wise, one workgroup per consensus, LDS-staged) remains for batches holding
// lower-case bases or '*' (codes 4..8, which the 2-bit planes do not carry).
#include "oge_ctx.h"
#include "bamio.h"
#include "realign.h"
#include "realign_dev.h"

#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kT = 256;
constexpr uint32_t kConsCap = 40960;  // consensus bytes staged in LDS
constexpr uint32_t kReadCap = 4096;   // read bases staged in LDS (reads > 3000 bp are never cleaned)

__device__ __forceinline__ uint32_t base_code(uint32_t c) {
    switch (c) {
        case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
        case 'a': return 4; case 'c': return 5; case 'g': return 6; case 't': return 7;
        case '*': return 8;
        default: return 0x80;  // not a regular base: never counted
    }
}

struct ScanJob {
    uint32_t cons, first, count, pad;
};

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, d, 64), hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

// Literal findBestOffset / mismatchQualitySumIgnoreCigar control flow (early exits included), run by
// one lane.  Needed only for reads with a quality >= 95: their weight (signed char)(q + 33) - 33 is
// negative, partial sums are no longer monotone and the early exits change the answer.
template <class CodeC, class ReadV>
__device__ int lit_sum(CodeC cc, ReadV rv, int L, int C, int k, int quit) {
    int sum = 0, i = 0;
    const int common = k >= C ? 0 : (L < C - k - 1 ? L : C - k - 1);
    for (; i < common && sum <= quit; ++i, ++k) {
        const int32_t v = rv(i);
        const uint32_t c = cc(k), r = (uint32_t)v & 0xFF;
        if (((r | c) & 0x80u) == 0 && r != c) sum += v >> 16;
    }
    for (; i < L && sum <= quit; ++i, ++k) {
        if (k >= C) {
            sum += 99;
        } else {
            const int32_t v = rv(i);
            const uint32_t c = cc(k), r = (uint32_t)v & 0xFF;
            if (((r | c) & 0x80u) == 0 && r != c) sum += v >> 16;
        }
    }
    return sum;
}
template <class CodeC, class ReadV>
__device__ void lit_best(CodeC cc, ReadV rv, int L, int C, int orig, int maxStart, int *bi, int *bs) {
    int best = lit_sum(cc, rv, L, C, orig, 0x7FFFFFFF), idx = orig;
    if (best != 0) {
        for (int i = 0; i < orig && best != 0; i++) {
            const int s = lit_sum(cc, rv, L, C, i, best);
            if (s < best) { best = s; idx = i; }
        }
        for (int i = orig + 1; i <= maxStart && best != 0; i++) {
            const int s = lit_sum(cc, rv, L, C, i, best);
            if (s < best) { best = s; idx = i; }
        }
    }
    *bi = idx;
    *bs = best;
}

__device__ __forceinline__ int32_t read_word(const uint8_t *bg, const uint8_t *qg, int i) {
    const int w = (int)(signed char)(uint8_t)(qg[i] + 33) - 33;
    return (int32_t)(base_code(bg[i]) | ((uint32_t)w << 16));
}

// BIG = consensus or read too long for LDS: read codes straight from global memory.
template <bool BIG>
__global__ __launch_bounds__(kT) void k_realign_scan(const uint8_t *__restrict__ cons, const uint64_t *__restrict__ cons_off,
                                                      const uint8_t *__restrict__ bases, const uint8_t *__restrict__ quals,
                                                      const uint64_t *__restrict__ read_off, const int4 *__restrict__ pairs,
                                                      const ScanJob *__restrict__ jobs, int32_t *__restrict__ best_idx,
                                                      int32_t *__restrict__ best_score) {
    __shared__ uint8_t cs[BIG ? 4 : kConsCap];
    __shared__ int32_t rd[BIG ? 4 : kReadCap];
    __shared__ uint64_t red[kT / 64];
    const ScanJob J = jobs[blockIdx.x];
    const uint8_t *cg = cons + cons_off[J.cons];
    const int C = (int)(cons_off[J.cons + 1] - cons_off[J.cons]);
    if (!BIG) {
        for (int i = threadIdx.x; i < C; i += kT) cs[i] = (uint8_t)base_code(cg[i]);
    }
    for (uint32_t p = 0; p < J.count; ++p) {
        const int4 P = pairs[J.first + p];  // (cons, read, orig, max_start)
        const uint8_t *bg = bases + read_off[P.y];
        const uint8_t *qg = quals + read_off[P.y];
        const int L = (int)(read_off[P.y + 1] - read_off[P.y]);
        const int orig = P.z;
        __syncthreads();  // previous read's slots are free (and the consensus is staged)
        int neg = 0;
        for (int i = threadIdx.x; i < L; i += kT) {
            const int32_t v = read_word(bg, qg, i);
            neg |= v < 0;
            if (!BIG) rd[i] = v;
        }
        if (__syncthreads_or(neg)) {  // a negative weight: literal scan (one lane, rare)
            if (threadIdx.x == 0) {
                int bi, bs;
                if (BIG)
                    lit_best([&](int k) { return base_code(cg[k]); }, [&](int i) { return read_word(bg, qg, i); }, L, C, orig,
                             P.w, &bi, &bs);
                else
                    lit_best([&](int k) { return (uint32_t)cs[k]; }, [&](int i) { return rd[i]; }, L, C, orig, P.w, &bi, &bs);
                best_idx[J.first + p] = bi;
                best_score[J.first + p] = bs;
            }
            continue;
        }
        const int nOff = (orig > P.w ? orig : P.w) + 1;
        uint64_t best = ~0ull;
        for (int k = threadIdx.x; k < nOff; k += kT) {
            int lim = C - k;
            lim = lim < L ? lim : L;
            lim = lim > 0 ? lim : 0;
            int s = 0;
            if (!BIG) {
                const uint8_t *c = cs + k;
                for (int i = 0; i < lim; ++i) {
                    const int32_t v = rd[i];
                    const uint32_t cc = c[i], rc = (uint32_t)v & 0xFF;
                    s += (((rc | cc) & 0x80u) == 0 && rc != cc) ? (v >> 16) : 0;
                }
            } else {
                for (int i = 0; i < lim; ++i) {
                    const int32_t v = read_word(bg, qg, i);
                    const uint32_t cc = base_code(cg[k + i]), rc = (uint32_t)v & 0xFF;
                    s += (((rc | cc) & 0x80u) == 0 && rc != cc) ? (v >> 16) : 0;
                }
            }
            s += 99 * (L - lim);  // MAX_QUAL for read bases past the consensus end
            const uint32_t rank = k == orig ? 0u : (k < orig ? (uint32_t)k + 1u : (uint32_t)k);
            const uint64_t key = ((uint64_t)(uint32_t)(s + 0x40000000) << 32) | rank;
            best = key < best ? key : best;
        }
        best = wave_min_u64(best);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t b = red[0];
#pragma unroll
            for (int w = 1; w < kT / 64; ++w) b = red[w] < b ? red[w] : b;
            const uint32_t rank = (uint32_t)b;
            best_idx[J.first + p] = rank == 0 ? orig : (rank <= (uint32_t)orig ? (int)rank - 1 : (int)rank);
            best_score[J.first + p] = (int)(uint32_t)(b >> 32) - 0x40000000;
        }
    }
}

// ---------------------------------------------------------------- bit-parallel path
struct CPlane {  // 64 consensus positions
    uint64_t b0, b1, v, pad;
};
struct RPlane {  // 64 read positions
    uint64_t b0, b1, v, w[7];
};

__device__ __forceinline__ uint64_t ballot64(bool x) { return __ballot(x); }

// one wave per consensus (g < n_cons) or altRead (g - n_cons); *generic set when a code 4..8 occurs
__global__ __launch_bounds__(kT) void k_planes(const uint8_t *__restrict__ cons, const uint64_t *__restrict__ cons_off,
                                               uint32_t n_cons, const uint64_t *__restrict__ cons_woff,
                                               const uint8_t *__restrict__ bases, const uint8_t *__restrict__ quals,
                                               const uint64_t *__restrict__ read_off, uint32_t n_reads,
                                               const uint64_t *__restrict__ read_woff, CPlane *__restrict__ cp,
                                               RPlane *__restrict__ rp, uint32_t *__restrict__ rflags,
                                               uint32_t *__restrict__ generic) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * (kT / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    bool gen = false;
    if (g < n_cons) {
        const uint8_t *c = cons + cons_off[g];
        const uint64_t C = cons_off[g + 1] - cons_off[g];
        const uint64_t w0 = cons_woff[g], nw = cons_woff[g + 1] - w0;
        for (uint64_t w = 0; w < nw; ++w) {
            const uint64_t i = 64 * w + lane;
            const uint32_t code = i < C ? base_code(c[i]) : 0x80u;
            gen |= code >= 4 && code <= 8;
            const bool ok = code < 4;
            const uint64_t b0 = ballot64(ok && (code & 1)), b1 = ballot64(ok && (code & 2)), v = ballot64(ok);
            if (lane < 3) (&cp[w0 + w].b0)[lane] = lane == 0 ? b0 : (lane == 1 ? b1 : v);
            if (lane == 3) cp[w0 + w].pad = 0;
        }
    } else if (g < (uint64_t)n_cons + n_reads) {
        const uint64_t r = g - n_cons;
        const uint8_t *b = bases + read_off[r], *q = quals + read_off[r];
        const uint64_t L = read_off[r + 1] - read_off[r];
        const uint64_t w0 = read_woff[r], nw = read_woff[r + 1] - w0;
        bool neg = false;
        int32_t orw = 0;
        for (uint64_t w = 0; w < nw; ++w) {
            const uint64_t i = 64 * w + lane;
            uint32_t code = 0x80u;
            int32_t wt = 0;
            if (i < L) {
                code = base_code(b[i]);
                wt = (int32_t)(signed char)(uint8_t)(q[i] + 33) - 33;
            }
            gen |= code >= 4 && code <= 8;
            neg |= wt < 0;
            if (wt > 0) orw |= wt;
            const bool ok = code < 4;
            uint64_t pl = 0;
            const uint64_t b0 = ballot64(ok && (code & 1)), b1 = ballot64(ok && (code & 2)), v = ballot64(ok);
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                const uint64_t wk = ballot64(wt > 0 && ((wt >> k) & 1));
                if (lane == 3 + k) pl = wk;
            }
            if (lane == 0) pl = b0;
            if (lane == 1) pl = b1;
            if (lane == 2) pl = v;
            if (lane < 10) (&rp[w0 + w].b0)[lane] = pl;
        }
        const bool anyneg = ballot64(neg) != 0;
        int32_t o = orw;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) o |= __shfl_xor(o, d, 64);
        if (lane == 0) rflags[r] = (anyneg ? 1u : 0u) | ((uint32_t)(o ? 32 - __clz(o) : 0) << 8);
    }
    if (ballot64(gen) && lane == 0) atomicOr(generic, 1u);
}

// bits [sh, sh + 64) of hi:lo
__device__ __forceinline__ uint64_t win64(uint64_t lo, uint64_t hi, uint32_t sh) {
    return (lo >> sh) | ((hi << (63 - sh)) << 1);
}

__global__ __launch_bounds__(kT) void k_scan_bp(const int4 *__restrict__ pairs, uint64_t n_pairs,
                                                const uint64_t *__restrict__ cons_off, const uint64_t *__restrict__ cons_woff,
                                                const CPlane *__restrict__ cp, const uint64_t *__restrict__ read_off,
                                                const uint64_t *__restrict__ read_woff, const RPlane *__restrict__ rp,
                                                const uint32_t *__restrict__ rflags, const uint8_t *__restrict__ cons,
                                                const uint8_t *__restrict__ bases, const uint8_t *__restrict__ quals,
                                                int32_t *__restrict__ best_idx, int32_t *__restrict__ best_score) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t p = (uint64_t)blockIdx.x * (kT / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (p >= n_pairs) return;
    const int4 P = pairs[p];  // (cons, read, orig, max_start)
    const int C = (int)(cons_off[P.x + 1] - cons_off[P.x]);
    const int L = (int)(read_off[P.y + 1] - read_off[P.y]);
    const uint32_t fl = rflags[P.y];
    const int orig = P.z;
    if (fl & 1u) {  // a negative weight: literal scan (one lane, rare)
        if (lane == 0) {
            const uint8_t *cg = cons + cons_off[P.x], *bg = bases + read_off[P.y], *qg = quals + read_off[P.y];
            int bi, bs;
            lit_best([&](int k) { return base_code(cg[k]); }, [&](int i) { return read_word(bg, qg, i); }, L, C, orig, P.w,
                     &bi, &bs);
            best_idx[p] = bi;
            best_score[p] = bs;
        }
        return;
    }
    const int nb = (int)(fl >> 8);
    const CPlane *c = cp + cons_woff[P.x];
    const uint64_t Wc = cons_woff[P.x + 1] - cons_woff[P.x];
    const RPlane *r = rp + read_woff[P.y];
    const uint64_t RW = read_woff[P.y + 1] - read_woff[P.y];
    const int nOff = (orig > P.w ? orig : P.w) + 1;
    uint64_t best = ~0ull;
    for (int a = 0; 64 * a < nOff; ++a) {
        const int k = 64 * a + (int)lane;
        uint32_t s = 0;
        CPlane cur = (uint64_t)a < Wc ? c[a] : CPlane{0, 0, 0, 0};
        for (uint64_t j = 0; j < RW; ++j) {
            const CPlane nxt = (uint64_t)a + j + 1 < Wc ? c[a + j + 1] : CPlane{0, 0, 0, 0};
            const RPlane R = r[j];
            const uint64_t m = win64(cur.v, nxt.v, lane) & R.v &
                               ((win64(cur.b0, nxt.b0, lane) ^ R.b0) | (win64(cur.b1, nxt.b1, lane) ^ R.b1));
            uint32_t t = 0;
#pragma unroll
            for (int b = 6; b >= 0; --b)  // constant plane indices keep R in scalar registers
                if (b < nb) t = 2 * t + (uint32_t)__popcll(m & R.w[b]);
            s += t;
            cur = nxt;
        }
        int lim = C - k;
        lim = lim < L ? lim : L;
        lim = lim > 0 ? lim : 0;
        const int sc = (int)s + 99 * (L - lim);
        const uint32_t rank = k == orig ? 0u : (k < orig ? (uint32_t)k + 1u : (uint32_t)k);
        const uint64_t key = ((uint64_t)(uint32_t)(sc + 0x40000000) << 32) | rank;
        if (k < nOff && key < best) best = key;
    }
    best = wave_min_u64(best);
    if (lane == 0) {
        const uint32_t rank = (uint32_t)best;
        best_idx[p] = rank == 0 ? orig : (rank <= (uint32_t)orig ? (int)rank - 1 : (int)rank);
        best_score[p] = (int)(uint32_t)(best >> 32) - 0x40000000;
    }
}

}  // namespace

// The scan over a batch already in device memory: planes, then k_scan_bp -- or, when the batch holds codes
// the 2-bit planes do not carry (lower-case bases, '*'), the byte-wise kernel, whose per-consensus jobs are
// cut on the host from the offsets and pairs (copied down for it when they only live on the device).
static int scan_core(oge_ctx *ctx, const RsDevBatch &b, const uint64_t *h_cons_off, const uint64_t *h_read_off, const int32_t *h_pairs,
                     int32_t *di, int32_t *ds, bool *generic_out) {
    hipStream_t s = ctx->stream;
    CPlane *dcp = (CPlane *)ctx->ws("rs_cplanes", (b.cons_words + 1) * sizeof(CPlane));
    RPlane *drp = (RPlane *)ctx->ws("rs_rplanes", (b.read_words + 1) * sizeof(RPlane));
    uint32_t *drf = (uint32_t *)ctx->ws("rs_rflags", ((uint64_t)b.n_reads + 1) * 4);
    uint32_t *dgen = (uint32_t *)ctx->ws("rs_generic", 4);
    if (!dcp || !drp || !drf || !dgen) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(dgen, 0, 4, s));
    uint32_t generic = 0;
    OgeStageTimer *t = ctx->begin_stage("realign_scan");
    const uint64_t items = (uint64_t)b.n_cons + b.n_reads;
    hipLaunchKernelGGL(k_planes, dim3((uint32_t)((items + 3) / 4)), dim3(kT), 0, s, b.cons, b.cons_off, b.n_cons, b.cwo, b.bases, b.quals,
                       b.read_off, b.n_reads, b.rwo, dcp, drp, drf, dgen);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&generic, dgen, 4, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    if (!generic) {
        hipLaunchKernelGGL(k_scan_bp, dim3((uint32_t)((b.n_pairs + 3) / 4)), dim3(kT), 0, s, b.pairs, b.n_pairs, b.cons_off, b.cwo, dcp,
                           b.read_off, b.rwo, drp, drf, b.cons, b.bases, b.quals, di, ds);
        OGE_LAUNCH_CHECK(ctx);
    } else {
        // lower-case bases or '*' present: byte-wise kernel, one workgroup per run of same-consensus pairs
        std::vector<uint64_t> co, ro;
        std::vector<int32_t> pr;
        if (!h_cons_off) {
            co.resize((uint64_t)b.n_cons + 1), ro.resize((uint64_t)b.n_reads + 1), pr.resize(4 * b.n_pairs);
            OGE_HIP_TRY(ctx, hipMemcpyAsync(co.data(), b.cons_off, co.size() * 8, hipMemcpyDeviceToHost, s));
            OGE_HIP_TRY(ctx, hipMemcpyAsync(ro.data(), b.read_off, ro.size() * 8, hipMemcpyDeviceToHost, s));
            OGE_HIP_TRY(ctx, hipMemcpyAsync(pr.data(), b.pairs, pr.size() * 4, hipMemcpyDeviceToHost, s));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
            h_cons_off = co.data(), h_read_off = ro.data(), h_pairs = pr.data();
        }
        std::vector<ScanJob> small, big;
        for (uint64_t i = 0; i < b.n_pairs;) {
            const uint32_t c = (uint32_t)h_pairs[4 * i];
            uint64_t j = i;
            bool isbig = h_cons_off[c + 1] - h_cons_off[c] > kConsCap;
            for (; j < b.n_pairs && (uint32_t)h_pairs[4 * j] == c; ++j) {
                const uint32_t rd = (uint32_t)h_pairs[4 * j + 1];
                if (h_read_off[rd + 1] - h_read_off[rd] > kReadCap) isbig = true;
            }
            (isbig ? big : small).push_back({c, (uint32_t)i, (uint32_t)(j - i), 0});
            i = j;
        }
        ScanJob *dj = (ScanJob *)ctx->ws("rs_jobs", (small.size() + big.size() + 1) * sizeof(ScanJob));
        if (!dj) return OGE_ERR_HIP;
        std::vector<ScanJob> all(small);
        all.insert(all.end(), big.begin(), big.end());
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dj, all.data(), all.size() * sizeof(ScanJob), hipMemcpyHostToDevice, s));
        if (!small.empty()) {
            hipLaunchKernelGGL(k_realign_scan<false>, dim3((uint32_t)small.size()), dim3(kT), 0, s, b.cons, b.cons_off, b.bases, b.quals,
                               b.read_off, b.pairs, dj, di, ds);
            OGE_LAUNCH_CHECK(ctx);
        }
        if (!big.empty()) {
            hipLaunchKernelGGL(k_realign_scan<true>, dim3((uint32_t)big.size()), dim3(kT), 0, s, b.cons, b.cons_off, b.bases, b.quals,
                               b.read_off, b.pairs, dj + small.size(), di, ds);
            OGE_LAUNCH_CHECK(ctx);
        }
        OGE_HIP_TRY(ctx, hipStreamSynchronize(s));  // `all` must outlive the upload
    }
    ctx->end_stage(t);
    ctx->last_scan_generic = generic != 0;
    if (generic_out) *generic_out = generic != 0;
    return OGE_OK;
}

int realign_scan_devbatch(oge_ctx *ctx, const RsDevBatch &b, int32_t *best_index, int32_t *best_score, bool *generic) {
    if (!b.n_pairs) return OGE_OK;
    int32_t *di = (int32_t *)ctx->ws("rs_idx", b.n_pairs * 4);
    int32_t *ds = (int32_t *)ctx->ws("rs_score", b.n_pairs * 4);
    if (!di || !ds) return OGE_ERR_HIP;
    int rc = scan_core(ctx, b, nullptr, nullptr, nullptr, di, ds, generic);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_index, di, b.n_pairs * 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_score, ds, b.n_pairs * 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

// Device scan over a host batch: validate, upload, scan_core, download.
static int realign_scan_host(oge_ctx *ctx, const uint8_t *cons, uint64_t cons_bytes, const uint64_t *cons_off, uint32_t n_cons,
                             const uint8_t *bases, const uint8_t *quals, uint64_t read_bytes, const uint64_t *read_off,
                             uint32_t n_reads, const int32_t *pairs, uint64_t n_pairs, int32_t *best_index, int32_t *best_score) {
    if (!n_pairs) return OGE_OK;
    auto clk = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double h0 = clk();
    if (n_pairs > 0x7FFFFFFFull) return oge_fail(ctx, OGE_ERR_LIMIT, "realign_scan: too many pairs");
    // validate on the host: the kernel trusts every index it is given
    if (cons_off[0] != 0 || cons_off[n_cons] != cons_bytes || read_off[0] != 0 || read_off[n_reads] != read_bytes)
        return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: offset tables do not match the byte counts");
    for (uint64_t i = 0; i < n_pairs; ++i) {
        const int32_t *q = pairs + 4 * i;
        if ((uint32_t)q[0] >= n_cons || (uint32_t)q[1] >= n_reads || q[2] < 0 || q[2] > (1 << 28) || q[3] > (1 << 28))
            return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: pair out of range");
    }
    for (uint32_t c = 0; c < n_cons; ++c)
        if (cons_off[c + 1] < cons_off[c]) return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: offsets not increasing");
    for (uint32_t r = 0; r < n_reads; ++r)
        if (read_off[r + 1] < read_off[r]) return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: offsets not increasing");
    // plane word offsets: a consensus gets one zero word past its end (the last window's high half)
    std::vector<uint64_t> cwo(n_cons + 1, 0), rwo(n_reads + 1, 0);
    for (uint32_t c = 0; c < n_cons; ++c) cwo[c + 1] = cwo[c] + (cons_off[c + 1] - cons_off[c] + 63) / 64 + 1;
    for (uint32_t r = 0; r < n_reads; ++r) rwo[r + 1] = rwo[r] + (read_off[r + 1] - read_off[r] + 63) / 64;
    const double h1 = clk();
    uint8_t *dc = (uint8_t *)ctx->ws("rs_cons", cons_bytes + 16);
    uint64_t *dco = (uint64_t *)ctx->ws("rs_cons_off", (n_cons + 1) * 8);
    uint8_t *db = (uint8_t *)ctx->ws("rs_bases", read_bytes + 16);
    uint8_t *dq = (uint8_t *)ctx->ws("rs_quals", read_bytes + 16);
    uint64_t *dro = (uint64_t *)ctx->ws("rs_read_off", (n_reads + 1) * 8);
    int4 *dp = (int4 *)ctx->ws("rs_pairs", n_pairs * 16);
    int32_t *di = (int32_t *)ctx->ws("rs_idx", n_pairs * 4);
    int32_t *ds = (int32_t *)ctx->ws("rs_score", n_pairs * 4);
    uint64_t *dcwo = (uint64_t *)ctx->ws("rs_cwo", (n_cons + 1) * 8);
    uint64_t *drwo = (uint64_t *)ctx->ws("rs_rwo", (n_reads + 1) * 8);
    if (!dc || !dco || !db || !dq || !dro || !dp || !di || !ds || !dcwo || !drwo) return OGE_ERR_HIP;
    hipStream_t s = ctx->stream;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dc, cons, cons_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dco, cons_off, (n_cons + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(db, bases, read_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dq, quals, read_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dro, read_off, (n_reads + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dp, pairs, n_pairs * 16, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dcwo, cwo.data(), (n_cons + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(drwo, rwo.data(), (n_reads + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    const double h2 = clk();
    const RsDevBatch b{dc, dco, n_cons, dcwo, cwo[n_cons], db, dq, dro, n_reads, drwo, rwo[n_reads], dp, n_pairs};
    int rc = scan_core(ctx, b, cons_off, read_off, pairs, di, ds, nullptr);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_index, di, n_pairs * 4, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_score, ds, n_pairs * 4, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    ctx->scan_t[0] = h1 - h0;
    ctx->scan_t[1] = h2 - h1;
    ctx->scan_t[2] = clk() - h2;
    return OGE_OK;
}

struct oge_realign_result {
    oge::ByteBuf recs;
    std::vector<uint64_t> offs;
    std::string stats;
};

extern "C" {

int oge_realign_scan(oge_ctx *ctx, const oge_realign_scan_batch *b, int32_t *best_index, int32_t *best_score) {
    if (!ctx || !b) return oge_fail(ctx, OGE_ERR_ARG, "oge_realign_scan: null argument");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    return realign_scan_host(ctx, b->cons, b->cons_bytes, b->cons_off, b->n_cons, b->bases, b->quals, b->read_bytes,
                             b->read_off, b->n_reads, b->pairs, b->n_pairs, best_index, best_score);
}

void oge_realign_opts_init(oge_realign_opts *o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    oge::RealignParams d;
    o->lod_threshold = d.lod_threshold;
    o->mismatch_threshold = d.mismatch_threshold;
    o->max_records_in_memory = d.max_records_in_memory;
    o->max_isize_for_movement = d.max_isize_for_movement;
    o->max_pos_move_allowed = d.max_pos_move_allowed;
    o->max_reads = d.max_reads;
    o->no_original_alignment_tags = 0;
    o->threads = 0;
}

static int localrealign_on(oge_ctx *const *ctxs, int G, const char *header_text, uint64_t header_len, const uint8_t *recs,
                           const uint64_t *rec_off, uint64_t n, const char *fasta_path, const char *intervals_path,
                           const oge_realign_opts *opts, oge_realign_result **out) {
    oge_ctx *ctx = ctxs[0];
    if (!header_text || (!recs && n) || (!rec_off && n) || !fasta_path || !intervals_path || !out)
        return oge_fail(ctx, OGE_ERR_ARG, "oge_localrealign: null argument");
    for (int g = 0; g < G; ++g)
        if (!ctxs[g]) return oge_fail(ctx, OGE_ERR_ARG, "oge_localrealign: null context");
    hipSetDevice(ctx->device);
    for (int g = 0; g < G; ++g) ctxs[g]->reset_timing();
    oge::BamHeaderModel h;
    std::string err;
    if (!h.parse(std::string(header_text, header_len), err)) return oge_fail(ctx, OGE_ERR_ARG, ("oge_localrealign: " + err).c_str());
    std::vector<std::string> names;
    for (auto &sq : h.sq) names.push_back(sq.name);
    oge::RealignParams P;
    if (opts) {
        P.lod_threshold = opts->lod_threshold;
        P.mismatch_threshold = opts->mismatch_threshold;
        P.max_records_in_memory = opts->max_records_in_memory;
        P.max_isize_for_movement = opts->max_isize_for_movement;
        P.max_pos_move_allowed = opts->max_pos_move_allowed;
        P.max_reads = opts->max_reads;
        P.no_original_alignment_tags = opts->no_original_alignment_tags != 0;
        P.threads = opts->threads;
    }
    if (P.lod_threshold < 0.0) return oge_fail(ctx, OGE_ERR_ARG, "LOD threshold cannot be a negative number");
    if (P.mismatch_threshold <= 0.0 || P.mismatch_threshold > 1.0)
        return oge_fail(ctx, OGE_ERR_ARG, "Entropy threshold must be a fraction between 0 and 1");
    double scan_kernel_ms = 0;
    int scan_rc = 0;
    oge::ScanFn scan = [&](const oge::ScanBatch &B, std::vector<int32_t> &bi, std::vector<int32_t> &bs) -> int {
        bi.assign(B.pairs.size(), 0);
        bs.assign(B.pairs.size(), 0);
        scan_rc = realign_scan_host(ctx, B.cons.data(), B.cons.size(), B.cons_off.data(), (uint32_t)(B.cons_off.size() - 1),
                                    B.bases.data(), B.quals.data(), B.bases.size(), B.read_off.data(),
                                    (uint32_t)(B.read_off.size() - 1), (const int32_t *)B.pairs.data(), B.pairs.size(),
                                    bi.data(), bs.data());
        if (!scan_rc) oge_ctx_timing(ctx, "realign_scan", &scan_kernel_ms);
        return scan_rc;
    };
    // phase B on the device(s) (realign_prep.hip; OGE_REALIGN_DEVICE_PREP=0: the host threads): the record
    // arena is copied to every device by a helper thread while the host loads the FASTA, decodes and bins
    struct Stager {
        std::thread th;
        uint8_t *d = nullptr;
        hipError_t e = hipSuccess;
        ~Stager() {
            if (th.joinable()) th.join();
        }
    };
    std::vector<Stager> stg((size_t)G);
    std::vector<int> prep_rcs((size_t)G, 0);
    oge::DevPrep dp;
    dp.ndev = G;
    dp.stage = [&](int g, const uint8_t *rp, uint64_t lo, uint64_t hi) -> int {
        oge_ctx *c = ctxs[g];
        Stager &sg = stg[(size_t)g];
        (void)hipSetDevice(c->device);
        sg.d = (uint8_t *)c->ws("rp_recs", hi - lo + 64);
        if (!sg.d) return prep_rcs[(size_t)g] = OGE_ERR_HIP;
        const int dev = c->device;
        sg.th = std::thread([&sg, rp, lo, hi, dev]() {
            (void)hipSetDevice(dev);
            sg.e = hipMemcpy(sg.d, rp + lo, hi - lo, hipMemcpyHostToDevice);
        });
        (void)hipSetDevice(ctx->device);
        return 0;
    };
    dp.run = [&](int g, const oge::DevPrepBatch &B, oge::DevPrepOut &O) -> int {
        oge_ctx *c = ctxs[g];
        Stager &sg = stg[(size_t)g];
        if (sg.th.joinable()) sg.th.join();
        (void)hipSetDevice(c->device);
        int &rc = prep_rcs[(size_t)g];
        if (sg.e != hipSuccess) return rc = oge_fail(c, OGE_ERR_HIP, (std::string("realign: record upload: ") + hipGetErrorString(sg.e)).c_str());
        return rc = oge_realign_prep_run(c, sg.d, B, O);
    };
    const char *pe = getenv("OGE_REALIGN_DEVICE_PREP");
    const bool use_dev = !(pe && pe[0] == '0');
    std::unique_ptr<oge_realign_result> r(new oge_realign_result());
    oge::RealignStats st;
    const auto tr0 = std::chrono::steady_clock::now();
    int rc = oge::realign_run(names, recs, rec_off, n, fasta_path, intervals_path, P, scan, r->recs, r->offs, st, err,
                              use_dev ? &dp : nullptr);
    st.t_run = std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count();
    for (auto &sg : stg)
        if (sg.th.joinable()) sg.th.join();
    (void)hipSetDevice(ctx->device);
    if (rc) {
        if (scan_rc) return scan_rc;
        for (int g = 0; g < G; ++g)
            if (prep_rcs[(size_t)g]) {
                if (g) oge_fail(ctx, prep_rcs[(size_t)g], oge_last_error(ctxs[g]));
                return prep_rcs[(size_t)g];
            }
        return oge_fail(ctx, rc, ("oge_localrealign: " + err).c_str());
    }
    double prep_ms = 0;
    scan_kernel_ms = 0;
    for (int g = 0; g < G; ++g) {  // summed over the devices
        double a = 0, b = 0;
        oge_ctx_timing(ctxs[g], "realign_scan", &a);
        oge_ctx_timing(ctxs[g], "realign_prep", &b);
        scan_kernel_ms += a > 0 ? a : 0.0;
        prep_ms += b > 0 ? b : 0.0;
    }
    st.more.emplace_back("prep_kernel_ms", prep_ms > 0 ? prep_ms : 0.0);
    st.more.emplace_back("device_prep", use_dev ? 1.0 : 0.0);
    char buf[2048];
    snprintf(buf, sizeof buf,
             "{\"intervals\": %llu, \"intervals_cleaned\": %llu, \"reads_realigned\": %llu, \"scan_pairs\": %llu, "
             "\"scan_ops\": %llu, \"scan_kernel_ms\": %.4f, \"t_bin\": %.4f, \"t_prepare\": %.4f, \"t_scan\": %.4f, "
             "\"t_decide\": %.4f, \"t_emit\": %.4f, \"t_run\": %.4f, \"t_fasta\": %.4f, \"t_decode\": %.4f, "
             "\"t_mate\": %.4f, \"t_release\": %.4f, \"t_scan_build\": %.4f, \"t_scan_validate\": %.4f, \"t_scan_upload\": %.4f, "
             "\"t_scan_device\": %.4f, \"mate_segments\": %llu, \"tail_waiting\": %llu, \"scan_kernel\": \"%s\"}",
             (unsigned long long)st.intervals, (unsigned long long)st.intervals_cleaned, (unsigned long long)st.reads_realigned,
             (unsigned long long)st.scan_pairs, (unsigned long long)st.scan_ops, scan_kernel_ms, st.t_bin, st.t_prepare,
             st.t_scan, st.t_decide, st.t_emit, st.t_run, st.t_fasta, st.t_decode, st.t_mate, st.t_release, st.t_scan_build, ctx->scan_t[0], ctx->scan_t[1], ctx->scan_t[2],
             (unsigned long long)st.mate_segments, (unsigned long long)st.tail_waiting, ctx->last_scan_generic ? "k_realign_scan (byte-wise)" : "k_planes + k_scan_bp");
    r->stats = buf;
    if (!st.more.empty()) {  // the finer timers, appended before the closing brace
        r->stats.pop_back();
        for (auto &m : st.more) {
            snprintf(buf, sizeof buf, ", \"%s\": %.4f", m.first.c_str(), m.second);
            r->stats += buf;
        }
        r->stats += "}";
    }
    *out = r.release();
    return OGE_OK;
}

int oge_localrealign(oge_ctx *ctx, const char *header_text, uint64_t header_len, const uint8_t *recs, const uint64_t *rec_off,
                     uint64_t n, const char *fasta_path, const char *intervals_path, const oge_realign_opts *opts,
                     oge_realign_result **out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "oge_localrealign: null context");
    return localrealign_on(&ctx, 1, header_text, header_len, recs, rec_off, n, fasta_path, intervals_path, opts, out);
}

int oge_localrealign_multi(oge_ctx *const *ctxs, int n_ctx, const char *header_text, uint64_t header_len, const uint8_t *recs,
                           const uint64_t *rec_off, uint64_t n, const char *fasta_path, const char *intervals_path,
                           const oge_realign_opts *opts, oge_realign_result **out) {
    if (!ctxs || n_ctx < 1 || !ctxs[0]) return oge_fail(nullptr, OGE_ERR_ARG, "oge_localrealign_multi: no contexts");
    return localrealign_on(ctxs, n_ctx, header_text, header_len, recs, rec_off, n, fasta_path, intervals_path, opts, out);
}

uint64_t oge_realign_result_count(const oge_realign_result *r) { return r && !r->offs.empty() ? r->offs.size() - 1 : 0; }
const uint8_t *oge_realign_result_records(const oge_realign_result *r, uint64_t *bytes_out) {
    if (bytes_out) *bytes_out = r ? r->recs.size() : 0;
    return r ? r->recs.data() : nullptr;
}
const uint64_t *oge_realign_result_offsets(const oge_realign_result *r) { return r ? r->offs.data() : nullptr; }
const char *oge_realign_result_stats(const oge_realign_result *r) { return r ? r->stats.c_str() : ""; }
void oge_realign_result_free(oge_realign_result *r) { delete r; }

}  // extern "C"

// (C++, the library's own modules) the result's records and offsets moved out without a copy: recs gets
// the records + 16 bytes of zeroed slack (ReadBatch's layout), offs the n + 1 offsets (offs[0] = 0)
void oge_realign_result_take(oge_realign_result *r, oge::bytevec &recs, std::vector<uint64_t> &offs) {
    r->recs.take(recs);
    offs = std::move(r->offs);
    r->offs = std::vector<uint64_t>();
}

