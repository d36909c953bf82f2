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
// Kernel: one 256-thread workgroup per consensus (all altReads of an interval share it).  The
// consensus is staged in LDS as 1-byte base codes; each read in turn is staged as packed
// (code | weight << 16) words that every lane reads at the same address (LDS broadcast).  Lanes own
// offsets; a wave/workgroup min-reduction over the packed (score, rank) key gives the answer.
// Integer VALU + LDS bound; no MFMA (no dense contraction).
#include "oge_ctx.h"
#include "bamio.h"
#include "realign.h"

#include <chrono>
#include <cstring>
#include <memory>
#include <string>
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

}  // namespace

// Device scan over a host batch: upload, one launch per job class, download.  Jobs are maximal runs
// of pairs with the same consensus.
static int realign_scan_host(oge_ctx *ctx, const uint8_t *cons, uint64_t cons_bytes, const uint64_t *cons_off, uint32_t n_cons,
                             const uint8_t *bases, const uint8_t *quals, uint64_t read_bytes, const uint64_t *read_off,
                             uint32_t n_reads, const int32_t *pairs, uint64_t n_pairs, int32_t *best_index, int32_t *best_score) {
    if (!n_pairs) return OGE_OK;
    if (n_pairs > 0x7FFFFFFFull) return oge_fail(ctx, OGE_ERR_LIMIT, "realign_scan: too many pairs");
    // validate on the host: the kernel trusts every index it is given
    if (cons_off[0] != 0 || cons_off[n_cons] != cons_bytes || read_off[0] != 0 || read_off[n_reads] != read_bytes)
        return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: offset tables do not match the byte counts");
    std::vector<ScanJob> small, big;
    for (uint64_t i = 0; i < n_pairs;) {
        const int32_t *p = pairs + 4 * i;
        const uint32_t c = (uint32_t)p[0];
        uint64_t j = i;
        bool isbig = false;
        for (; j < n_pairs && (uint32_t)pairs[4 * j] == c; ++j) {
            const int32_t *q = pairs + 4 * j;
            if ((uint32_t)q[0] >= n_cons || (uint32_t)q[1] >= n_reads || q[2] < 0 || q[2] > (1 << 28) || q[3] > (1 << 28))
                return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: pair out of range");
            if (cons_off[c + 1] < cons_off[c] || read_off[q[1] + 1] < read_off[q[1]])
                return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: offsets not increasing");
            if (read_off[q[1] + 1] - read_off[q[1]] > kReadCap) isbig = true;
        }
        if (c >= n_cons) return oge_fail(ctx, OGE_ERR_ARG, "realign_scan: pair out of range");
        if (cons_off[c + 1] - cons_off[c] > kConsCap) isbig = true;
        (isbig ? big : small).push_back({c, (uint32_t)i, (uint32_t)(j - i), 0});
        i = j;
    }
    uint8_t *dc = (uint8_t *)ctx->ws("rs_cons", cons_bytes + 16);
    uint64_t *dco = (uint64_t *)ctx->ws("rs_cons_off", (n_cons + 1) * 8);
    uint8_t *db = (uint8_t *)ctx->ws("rs_bases", read_bytes + 16);
    uint8_t *dq = (uint8_t *)ctx->ws("rs_quals", read_bytes + 16);
    uint64_t *dro = (uint64_t *)ctx->ws("rs_read_off", (n_reads + 1) * 8);
    int4 *dp = (int4 *)ctx->ws("rs_pairs", n_pairs * 16);
    ScanJob *dj = (ScanJob *)ctx->ws("rs_jobs", (small.size() + big.size() + 1) * sizeof(ScanJob));
    int32_t *di = (int32_t *)ctx->ws("rs_idx", n_pairs * 4);
    int32_t *ds = (int32_t *)ctx->ws("rs_score", n_pairs * 4);
    if (!dc || !dco || !db || !dq || !dro || !dp || !dj || !di || !ds) return OGE_ERR_HIP;
    hipStream_t s = ctx->stream;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dc, cons, cons_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dco, cons_off, (n_cons + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(db, bases, read_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dq, quals, read_bytes, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dro, read_off, (n_reads + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dp, pairs, n_pairs * 16, hipMemcpyHostToDevice, s));
    std::vector<ScanJob> all(small);
    all.insert(all.end(), big.begin(), big.end());
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dj, all.data(), all.size() * sizeof(ScanJob), hipMemcpyHostToDevice, s));
    OgeStageTimer *t = ctx->begin_stage("realign_scan");
    if (!small.empty()) {
        hipLaunchKernelGGL(k_realign_scan<false>, dim3((uint32_t)small.size()), dim3(kT), 0, s, dc, dco, db, dq, dro, dp, dj, di, ds);
        OGE_LAUNCH_CHECK(ctx);
    }
    if (!big.empty()) {
        hipLaunchKernelGGL(k_realign_scan<true>, dim3((uint32_t)big.size()), dim3(kT), 0, s, dc, dco, db, dq, dro, dp,
                           dj + small.size(), di, ds);
        OGE_LAUNCH_CHECK(ctx);
    }
    ctx->end_stage(t);
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_index, di, n_pairs * 4, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(best_score, ds, n_pairs * 4, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
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

int oge_localrealign(oge_ctx *ctx, const char *header_text, uint64_t header_len, const uint8_t *recs, const uint64_t *rec_off,
                     uint64_t n, const char *fasta_path, const char *intervals_path, const oge_realign_opts *opts,
                     oge_realign_result **out) {
    if (!ctx || !header_text || (!recs && n) || (!rec_off && n) || !fasta_path || !intervals_path || !out)
        return oge_fail(ctx, OGE_ERR_ARG, "oge_localrealign: null argument");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
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
    std::unique_ptr<oge_realign_result> r(new oge_realign_result());
    oge::RealignStats st;
    const auto tr0 = std::chrono::steady_clock::now();
    int rc = oge::realign_run(names, recs, rec_off, n, fasta_path, intervals_path, P, scan, r->recs, r->offs, st, err);
    st.t_run = std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count();
    if (rc) return scan_rc ? scan_rc : oge_fail(ctx, rc, ("oge_localrealign: " + err).c_str());
    char buf[1024];
    snprintf(buf, sizeof buf,
             "{\"intervals\": %llu, \"intervals_cleaned\": %llu, \"reads_realigned\": %llu, \"scan_pairs\": %llu, "
             "\"scan_ops\": %llu, \"scan_kernel_ms\": %.4f, \"t_bin\": %.4f, \"t_prepare\": %.4f, \"t_scan\": %.4f, "
             "\"t_decide\": %.4f, \"t_emit\": %.4f, \"t_run\": %.4f, \"t_fasta\": %.4f, \"t_decode\": %.4f, "
             "\"t_mate\": %.4f, \"t_release\": %.4f}",
             (unsigned long long)st.intervals, (unsigned long long)st.intervals_cleaned, (unsigned long long)st.reads_realigned,
             (unsigned long long)st.scan_pairs, (unsigned long long)st.scan_ops, scan_kernel_ms, st.t_bin, st.t_prepare,
             st.t_scan, st.t_decide, st.t_emit, st.t_run, st.t_fasta, st.t_decode, st.t_mate, st.t_release);
    r->stats = buf;
    *out = r.release();
    return OGE_OK;
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
