// realign_prep.hip -- LocalRealignment's consensus generation (phase B) on gfx950, feeding the offset scan
// (realign.hip) without a host round trip (r06).
//
// Reference: determineReadsThatNeedCleaning (algorithms/local_realignment.cpp:918-999) for every toClean
// read of an interval -- getUnclippedBases (:137-164), leftAlignIndel of the two-block reads
// (util/gatk/AlignmentUtils.cpp:632-677 with createIndelString :724-783, moveCigarLeft :700-722,
// cleanUpCigar :687-698), mismatchQualitySumIgnoreCigar (:641-679) at the original start,
// getMismatchCount's quality sum (AlignmentUtils.cpp:58-108) and createAlternateConsensus (:1022-1088) --
// and the interval's consensus set: the distinct strings in creation order.  realign.cpp restates the same
// steps on the host (left_align_indel, mismatch_sum_ignore_cigar, create_consensus ...); the two must agree
// on every read, which the rl_* / c5_50k goldens and tests/test_gpu_realign.py check through both paths.
//
// Layout.  The record arena is staged once (the module's input, copied beside the binning phase); the host
// hands over each interval's reference window and its toClean reads (record offsets, start on the window).
//   k_r2_read   one thread per read: cigar walks, left-alignment (strings compared position by position
//               through their definition -- reference prefix, indel, reference suffix -- never built),
//               mismatch sums, the consensus length
//   k_r2_cand   one thread per consensus candidate: the string, written once, and its 64-bit FNV-1a hash
//   k_r2_iv     one wave per interval: altRead counts and sums, the consensus set (a candidate is kept
//               unless an earlier one has the same hash, length and bytes -- compared by the whole wave)
//   scans       per-interval bases of the batch (consensuses, altReads, pairs, plane words)
//   k_r2_batch  one wave per interval: kept consensus bytes, altRead bases / qualities, the pairs of
//               findBestOffset with orig and maxStart -- the batch k_planes / k_scan_bp read in place
// Anything outside the shapes handled here (more than 8 cigar operations, a newCigar of more than 4, more
// than kCandCap candidates in one interval, ...) marks the interval for the host path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "oge_ctx.h"
#include "realign.h"
#include "realign_dev.h"

namespace {

using oge::DevPrepRead;
constexpr int kT = 256;
constexpr int kMaxIn = 8;       // cigar operations of a read handled on the device
constexpr int kMaxOps = 12;     // working cigar (unclipped, moved, one M appended)
constexpr uint32_t kCandCap = 2048;  // consensus candidates of one interval handled on the device

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };

__constant__ char kSeqC[17] = "=ACMGRSVTWYHKDBN";

struct Cig {
    int n;
    uint32_t len[kMaxOps];
    uint8_t code[kMaxOps];
};

__device__ __forceinline__ bool regular(char b) {  // BaseUtils::isRegularBase
    return b == 'A' || b == 'C' || b == 'G' || b == 'T' || b == 'a' || b == 'c' || b == 'g' || b == 't' || b == '*';
}

struct Read {
    const uint8_t *seq4, *qual;
    int64_t lseq;
    __device__ char base(int64_t i) const { return kSeqC[(seq4[i >> 1] >> ((i & 1) ? 0 : 4)) & 15]; }
};

// createIndelString's parameters for cigar c, indel at idx (the string is never built: alt_at)
struct Alt {
    bool ok, del;
    int64_t sz, R, L, ri;  // length, reference index of the indel, its (truncated) length, read index
};
__device__ Alt alt_params(const Cig &c, int idx, int64_t rsz, int64_t refIndex, int64_t readIndex) {
    Alt a;
    int64_t L = c.len[idx], total = 0;
    for (int i = 0; i < idx; ++i) {
        const int64_t n = c.len[i];
        switch (c.code[i]) {
            case OP_M: readIndex += n, refIndex += n, total += n; break;
            case OP_S: readIndex += n; break;
            case OP_N: refIndex += n, total += n; break;
            default: break;
        }
    }
    if (total + L > rsz) L -= (total + L - rsz);
    a.del = c.code[idx] == OP_D;
    a.sz = rsz + (a.del ? -L : L);
    a.R = refIndex, a.L = L, a.ri = readIndex;
    a.ok = !(a.sz < 0 || refIndex < 0 || refIndex > a.sz || refIndex > rsz);
    if (a.ok) {
        const int64_t ri = refIndex + (a.del ? L : 0), cur = refIndex + (a.del ? 0 : L);
        a.ok = !((uint64_t)(rsz - ri) > (uint64_t)(a.sz - cur));
    }
    return a;
}
// character k of createIndelString's result (see realign.cpp create_indel_string: the prefix copy, the
// insertion or the deletion, the suffix copy -- which for a negative truncated length overwrites the
// prefix's tail)
__device__ __forceinline__ char alt_at(const Alt &a, int64_t k, const char *ref, const Read &rd) {
    if (a.del) return k < a.R ? ref[k] : ref[k + a.L];
    if (k >= a.R + a.L) return ref[k - a.L];
    if (k >= a.R) {
        const int64_t j = a.ri + (k - a.R);
        return j < rd.lseq ? rd.base(j) : '\0';
    }
    return ref[k];
}
// a == b as strings.  Both are the same reference with one indel of the same kind spliced in (left_align
// compares moves of one indel), so with equal lengths L they agree outside the span the two indels cover:
// below min(R) + min(L, 0) both are the reference prefix, from max(R) + max(L, 0) on (insertion) or max(R)
// on (deletion) both are the same shifted reference suffix -- only that span is compared (a memcmp of the
// whole window in the reference).
__device__ bool alt_equal(const Alt &a, const Alt &b, const char *ref, const Read &rd) {
    if (a.sz != b.sz) return false;
    int64_t k0 = 0, k1 = a.sz;
    if (a.del == b.del && a.L == b.L) {
        k0 = max(min(a.R, b.R) + min(a.L, (int64_t)0), (int64_t)0);
        k1 = min(max(a.R, b.R) + (a.del ? 0 : max(a.L, (int64_t)0)), a.sz);
    }
    for (int64_t k = k0; k < k1; ++k)
        if (alt_at(a, k, ref, rd) != alt_at(b, k, ref, rd)) return false;
    return true;
}

// AlignmentUtils::leftAlignIndel (:632-677); false: the working cigar outgrew kMaxOps (host path)
__device__ bool left_align(Cig &cig, const char *ref, int64_t rsz, const Read &rd, int64_t refIndex) {
    int idx = -1;
    for (int i = 0; i < cig.n; ++i) {
        if (cig.code[i] == OP_D || cig.code[i] == OP_I) {
            if (idx != -1) return true;
            idx = i;
        }
    }
    if (idx < 1) return true;
    const int indelLength = (int)cig.len[idx];
    const Alt a0 = alt_params(cig, idx, rsz, refIndex, 0);
    if (!a0.ok || a0.sz == 0) return true;
    Cig nc = cig;
    for (int i = 0; i < indelLength; ++i) {
        // moveCigarLeft (:700-722)
        {
            Cig e;
            e.n = 0;
            for (int k = 0; k < idx - 1; ++k) e.len[e.n] = nc.len[k], e.code[e.n++] = nc.code[k];
            e.len[e.n] = nc.len[idx - 1] - 1, e.code[e.n++] = nc.code[idx - 1];
            e.len[e.n] = nc.len[idx], e.code[e.n++] = nc.code[idx];
            if (idx + 1 < nc.n) e.len[e.n] = nc.len[idx + 1] + 1, e.code[e.n++] = nc.code[idx + 1];
            else e.len[e.n] = 1, e.code[e.n++] = OP_M;
            if (nc.n - (idx + 2) + e.n > kMaxOps) return false;
            for (int k = idx + 2; k < nc.n; ++k) e.len[e.n] = nc.len[k], e.code[e.n++] = nc.code[k];
            nc = e;
        }
        const Alt an = alt_params(nc, idx, rsz, refIndex, 0);
        bool reachedEnd = false;
        for (int k = 0; k < nc.n; ++k) reachedEnd |= nc.len[k] == 0;
        if (an.ok && alt_equal(a0, an, ref, rd)) {
            cig = nc;
            i = -1;
            if (reachedEnd) {  // cleanUpCigar (:687-698)
                Cig e;
                e.n = 0;
                for (int k = 0; k < cig.n; ++k)
                    if (cig.len[k] != 0 && (e.n || cig.code[k] != OP_D)) e.len[e.n] = cig.len[k], e.code[e.n++] = cig.code[k];
                cig = e;
            }
        }
        if (reachedEnd) break;
    }
    return true;
}

// the read's i-th unclipped base (getUnclippedBases: the M and I operations of the ORIGINAL cigar, each
// clipped to the read); -1 past the end
__device__ int64_t unclipped_pos(const Cig &orig, int64_t i, int64_t lseq) {
    int64_t from = 0, k = 0;
    for (int j = 0; j < orig.n; ++j) {
        const int64_t n = orig.len[j];
        if (orig.code[j] == OP_S) {
            from += n;
        } else if (orig.code[j] == OP_M || orig.code[j] == OP_I) {
            const int64_t m = from < lseq ? min(n, lseq - from) : 0;
            if (i < k + m) return from + (i - k);
            k += m;
            from += n;
        }
    }
    return -1;
}

// createAlternateConsensus's string as pieces: [ref 0, p0) then per operation, then [ref refEnd, rsz).
// Returns the length, or -1 when the reference returns null.  emit(piece kind, a, n): kind 0 = reference
// bytes [a, a + n), 1 = unclipped read bases [a, a + n)
template <class Emit>
__device__ int64_t consensus(int64_t indexOnRef, const Cig &c, int64_t rsz, const Cig &orig, const Read &rd, int64_t ul, Emit emit) {
    if (indexOnRef < 0) return -1;
    if (c.n == 1 && c.code[0] == OP_M) return -1;
    int64_t len = min(indexOnRef, rsz);
    emit(0, 0, len);
    int indelCount = 0;
    int64_t altIdx = 0, refIdx = indexOnRef;
    bool ok = true;
    for (int k = 0; k < c.n; ++k) {
        const int64_t n = c.len[k];
        switch (c.code[k]) {
            case OP_D:
                refIdx += n;
                indelCount++;
                break;
            case OP_M:
            case OP_N:
                if (c.code[k] == OP_M) altIdx += n;
                if (rsz < refIdx + n) {
                    ok = false;
                } else {
                    emit(0, refIdx, n);
                    len += n;
                }
                refIdx += n;
                break;
            case OP_I: {
                int64_t j = 0;
                for (; j < n; ++j) {
                    const int64_t u = altIdx + j;
                    const int64_t p = u < ul ? unclipped_pos(orig, u, rd.lseq) : -1;
                    if (!regular(p >= 0 ? rd.base(p) : '\0')) {
                        ok = false;
                        break;
                    }
                }
                emit(1, altIdx, j);
                len += j;
                altIdx += n;
                indelCount++;
                break;
            }
            default: break;
        }
    }
    if (!ok || indelCount != 1 || rsz < refIdx) return -1;
    emit(0, refIdx, rsz - refIdx);
    return len + (rsz - refIdx);
}

struct ReadArgs {
    const uint8_t *recs;
    const uint64_t *rec;
    const int32_t *start;
    const uint64_t *rd_off;
    uint32_t n_iv;
    uint64_t n;
    const uint8_t *ref;
    const uint64_t *ref_off;
    DevPrepRead *out;
    uint64_t *cand_len;  // consensus length of a candidate read, else 0
};

__device__ uint32_t iv_of(const uint64_t *rd_off, uint32_t n_iv, uint64_t r) {  // the interval holding read r
    uint32_t lo = 0, hi = n_iv;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rd_off[mid] <= r) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t rd_u32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ void load_read(const uint8_t *R, Cig &orig, Read &rd, uint32_t *flag, bool *fits) {
    const uint32_t lname = R[12], nc = (uint32_t)R[16] | ((uint32_t)R[17] << 8);
    *flag = (uint32_t)R[18] | ((uint32_t)R[19] << 8);
    rd.lseq = rd_u32(R + 20);
    const uint8_t *cg = R + 36 + lname;
    rd.seq4 = cg + 4 * nc;
    rd.qual = rd.seq4 + (rd.lseq + 1) / 2;
    *fits = nc <= (uint32_t)kMaxIn;
    orig.n = (int)min(nc, (uint32_t)kMaxIn);
    for (int i = 0; i < orig.n; ++i) {
        const uint32_t op = rd_u32(cg + 4 * i);
        orig.len[i] = op >> 4;
        orig.code[i] = (uint8_t)((op & 15) < 9 ? (op & 15) : 0);
    }
}

__global__ __launch_bounds__(kT) void k_r2_read(ReadArgs A) {
    const uint64_t r = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (r >= A.n) return;
    DevPrepRead o = {};
    A.cand_len[r] = 0;
    const uint8_t *R = A.recs + A.rec[r];
    Cig orig;
    Read rd;
    uint32_t flag;
    bool fits;
    load_read(R, orig, rd, &flag, &fits);
    const uint32_t nc = (uint32_t)R[16] | ((uint32_t)R[17] << 8);
    if (flag & 0x400) o.flags |= oge::DP_DUP;
    if (nc == 0) {  // refReads: skipped
        o.flags |= oge::DP_SKIP;
        A.out[r] = o;
        return;
    }
    if (!fits || rd.lseq > 65535) {
        o.flags |= oge::DP_HOST;
        A.out[r] = o;
        return;
    }
    const uint32_t w = iv_of(A.rd_off, A.n_iv, r);
    const char *ref = (const char *)A.ref + A.ref_off[w];
    const int64_t rsz = (int64_t)(A.ref_off[w + 1] - A.ref_off[w]);
    const int64_t startOnRef = A.start[r];
    int blocks = 0;
    int64_t ul = 0, from = 0;
    for (int i = 0; i < orig.n; ++i) {
        const uint8_t c = orig.code[i];
        if (c == OP_M || c == OP_EQ || c == OP_X) blocks++;
        if (c == OP_S) from += orig.len[i];
        else if (c == OP_M || c == OP_I) {
            if (from < rd.lseq) ul += min((int64_t)orig.len[i], rd.lseq - from);
            from += orig.len[i];
        }
    }
    o.ul = (uint16_t)ul;
    // the current cigar: the left-aligned one when it differs from the original (AlignedRead::setCigar with
    // fixClipped = false), else the original
    Cig cur = orig;
    if (blocks == 2) {
        Cig u;
        u.n = 0;
        for (int i = 0; i < orig.n; ++i)
            if (!(orig.code[i] == OP_S || orig.code[i] == OP_H || orig.code[i] == OP_P)) u.len[u.n] = orig.len[i], u.code[u.n++] = orig.code[i];
        if (!left_align(u, ref, rsz, rd, startOnRef)) {
            o.flags |= oge::DP_HOST;
            A.out[r] = o;
            return;
        }
        bool same = u.n == orig.n;
        for (int i = 0; same && i < u.n; ++i) same = u.len[i] == orig.len[i] && u.code[i] == orig.code[i];
        if (!same) {
            if (u.n > 4) {
                o.flags |= oge::DP_HOST;
                A.out[r] = o;
                return;
            }
            for (int i = 0; i < u.n; ++i) {
                if (u.len[i] >= (1u << 28)) {
                    o.flags |= oge::DP_HOST;
                    A.out[r] = o;
                    return;
                }
                o.ops[i] = (u.len[i] << 4) | u.code[i];
            }
            o.n_ops = (uint8_t)u.n;
            o.flags |= oge::DP_NEWCIG;
            cur = u;
        }
    }
    // getCigarLength of the current cigar
    uint64_t cl = 0;
    for (int i = 0; i < cur.n; ++i)
        if (!(cur.code[i] == OP_H || cur.code[i] == OP_S || cur.code[i] == OP_D)) cl += cur.len[i];
    o.cig_len = (uint32_t)cl;
    // mismatchQualitySumIgnoreCigar over the unclipped bases at the original start (quit = INT_MAX)
    int32_t raw = 0;
    {
        int64_t i = 0;
        from = 0;
        for (int j = 0; j < orig.n; ++j) {
            const int64_t n = orig.len[j];
            if (orig.code[j] == OP_S) {
                from += n;
            } else if (orig.code[j] == OP_M || orig.code[j] == OP_I) {
                const int64_t m = from < rd.lseq ? min(n, rd.lseq - from) : 0;
                for (int64_t t = 0; t < m; ++t, ++i) {
                    const int64_t k = startOnRef + i;
                    if (k >= rsz) {
                        raw += 99;
                        continue;
                    }
                    if (k < 0) continue;
                    const char rc = ref[k], bc = rd.base(from + t);
                    if (!regular(bc) || !regular(rc)) continue;
                    if (bc != rc) raw += (int)(signed char)(uint8_t)(rd.qual[from + t] + 33) - 33;
                }
                from += n;
            }
        }
    }
    o.raw = raw;
    if (raw > 0) {
        o.flags |= oge::DP_ALT;
        // getMismatchCount's mismatch-quality sum over the original cigar
        int32_t mq = 0;
        int64_t readIdx = 0, refIndex = startOnRef;
        const int64_t endOnRead = rd.lseq - 1;
        for (int j = 0; j < orig.n; ++j) {
            if (readIdx > endOnRead) break;
            const int64_t n = orig.len[j];
            switch (orig.code[j]) {
                case OP_M:
                    for (int64_t t = 0; t < n; ++t, ++refIndex, ++readIdx) {
                        if (refIndex < 0 || refIndex >= rsz) continue;
                        if (readIdx > endOnRead) break;
                        if (rd.base(readIdx) != ref[refIndex]) mq += (int)(signed char)(uint8_t)(rd.qual[readIdx] + 33) - 33;
                    }
                    break;
                case OP_I: case OP_S: readIdx += n; break;
                case OP_D: case OP_N: refIndex += n; break;
                default: break;
            }
        }
        o.aligner = mq;
        if (blocks == 2) {
            const int64_t len = consensus(startOnRef, cur, rsz, orig, rd, ul, [](int, int64_t, int64_t) {});
            if (len >= 0) {
                if (len >= (1ll << 31)) {
                    o.flags |= oge::DP_HOST;
                } else {
                    o.flags |= oge::DP_CAND;
                    A.cand_len[r] = (uint64_t)len;
                }
            }
        }
    }
    A.out[r] = o;
}

// the current cigar of a read from its result (NEWCIG) or its record
__device__ void cur_cigar(const DevPrepRead &o, const Cig &orig, Cig &cur) {
    if (o.flags & oge::DP_NEWCIG) {
        cur.n = o.n_ops;
        for (int i = 0; i < cur.n; ++i) cur.len[i] = o.ops[i] >> 4, cur.code[i] = (uint8_t)(o.ops[i] & 15);
    } else {
        cur = orig;
    }
}

// one thread per candidate: its consensus string at cand_off[r] and its FNV-1a hash
__global__ __launch_bounds__(kT) void k_r2_cand(ReadArgs A, const uint64_t *__restrict__ cand_off, uint8_t *__restrict__ cand,
                                                uint64_t *__restrict__ cand_hash) {
    const uint64_t r = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (r >= A.n) return;
    const DevPrepRead o = A.out[r];
    if (!(o.flags & oge::DP_CAND)) return;
    const uint8_t *R = A.recs + A.rec[r];
    Cig orig, cur;
    Read rd;
    uint32_t flag;
    bool fits;
    load_read(R, orig, rd, &flag, &fits);
    cur_cigar(o, orig, cur);
    const uint32_t w = iv_of(A.rd_off, A.n_iv, r);
    const char *ref = (const char *)A.ref + A.ref_off[w];
    const int64_t rsz = (int64_t)(A.ref_off[w + 1] - A.ref_off[w]);
    uint8_t *dst = cand + cand_off[r];
    uint64_t h = 14695981039346656037ull;
    consensus(A.start[r], cur, rsz, orig, rd, o.ul, [&](int kind, int64_t a, int64_t n) {
        for (int64_t k = 0; k < n; ++k) {
            char c;
            if (kind == 0) {
                c = ref[a + k];
            } else {
                const int64_t p = unclipped_pos(orig, a + k, rd.lseq);
                c = p >= 0 ? rd.base(p) : '\0';
            }
            *dst++ = (uint8_t)c;
            h = (h ^ (uint8_t)c) * 1099511628211ull;
        }
    });
    cand_hash[r] = h;
}

// per interval (one wave): counts, sums and the consensus set.  Outputs in separate arrays so that their
// exclusive scans give the batch bases: kc kb kw (kept consensuses, bytes, plane words), ac ab aw (altReads
// in the batch, bytes, words), pc (pairs).
struct IvArgs {
    const uint64_t *rd_off;
    uint32_t n_iv;
    DevPrepRead *out;
    const uint64_t *cand_len, *cand_off, *cand_hash;
    const uint8_t *cand;
    uint64_t *kc, *kb, *kw, *ac, *ab, *aw, *pc;
    int64_t *total_raw;
    uint8_t *host;
};

__global__ __launch_bounds__(64) void k_r2_iv(IvArgs A) {
    __shared__ uint32_t cidx[kCandCap];
    const uint32_t w = blockIdx.x, lane = threadIdx.x;
    const uint64_t a = A.rd_off[w], b = A.rd_off[w + 1];
    uint64_t n_alt = 0, alt_bytes = 0, alt_words = 0;
    int64_t traw = 0;
    bool host = false;
    uint32_t ncand = 0;
    // pass 1: sums, the candidates in read order into LDS
    for (uint64_t r0 = a; r0 < b; r0 += 64) {
        const uint64_t r = r0 + lane;
        uint8_t f = 0;
        uint32_t ul = 0;
        int32_t raw = 0;
        if (r < b) {
            const DevPrepRead &o = A.out[r];
            f = o.flags, ul = o.ul, raw = o.raw;
        }
        host |= (f & oge::DP_HOST) != 0;
        if (f & oge::DP_ALT) {
            n_alt++, alt_bytes += ul, alt_words += (ul + 63) / 64;
            if (!(f & oge::DP_DUP)) traw += raw;
        }
        const uint64_t m = __ballot((f & oge::DP_CAND) != 0);
        if ((f & oge::DP_CAND) && ncand + __popcll(m & ((1ull << lane) - 1)) < kCandCap)
            cidx[ncand + __popcll(m & ((1ull << lane) - 1))] = (uint32_t)(r - a);
        ncand += (uint32_t)__popcll(m);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        n_alt += __shfl_xor((unsigned long long)n_alt, d, 64);
        alt_bytes += __shfl_xor((unsigned long long)alt_bytes, d, 64);
        alt_words += __shfl_xor((unsigned long long)alt_words, d, 64);
        traw += __shfl_xor((long long)traw, d, 64);
    }
    host = __ballot(host) != 0 || ncand > kCandCap;
    __syncthreads();
    // pass 2: a candidate is kept unless an earlier one has the same string (hash + length, then the bytes)
    uint64_t n_kept = 0, kept_bytes = 0, kept_words = 0;
    if (!host) {
        for (uint32_t j = 0; j < ncand; ++j) {
            const uint64_t rj = a + cidx[j];
            const uint64_t hj = A.cand_hash[rj], lj = A.cand_len[rj];
            bool dup = false;
            for (uint32_t i0 = 0; i0 < j && !dup; i0 += 64) {
                const uint32_t i = i0 + lane;
                bool m = false;
                uint64_t ri = 0;
                if (i < j) {
                    ri = a + cidx[i];
                    m = A.cand_hash[ri] == hj && A.cand_len[ri] == lj;
                }
                uint64_t mb = __ballot(m);
                while (mb && !dup) {  // candidates with the same hash and length: compare the bytes
                    const int src = __builtin_ctzll(mb);
                    mb &= mb - 1;
                    const uint64_t rs = __shfl((unsigned long long)ri, src, 64);
                    const uint8_t *x = A.cand + A.cand_off[rs], *y = A.cand + A.cand_off[rj];
                    bool diff = false;
                    for (uint64_t k = lane; k < lj; k += 64) diff |= x[k] != y[k];
                    dup = __ballot(diff) == 0;
                }
            }
            if (!dup) {
                n_kept++, kept_bytes += lj, kept_words += (lj + 63) / 64 + 1;
                if (lane == 0) A.out[rj].flags |= oge::DP_KEPT;
            }
        }
    }
    if (lane == 0) {
        const bool on = !host && n_kept > 0;  // an interval without consensuses adds nothing to the batch
        A.host[w] = host;
        A.total_raw[w] = traw;
        A.kc[w] = on ? n_kept : 0;
        A.kb[w] = on ? kept_bytes : 0;
        A.kw[w] = on ? kept_words : 0;
        A.ac[w] = on ? n_alt : 0;
        A.ab[w] = on ? alt_bytes : 0;
        A.aw[w] = on ? alt_words : 0;
        A.pc[w] = on ? n_kept * n_alt : 0;
        if (w == 0) A.kc[A.n_iv] = A.kb[A.n_iv] = A.kw[A.n_iv] = A.ac[A.n_iv] = A.ab[A.n_iv] = A.aw[A.n_iv] = A.pc[A.n_iv] = 0;
    }
}

// per batch altRead (one wave per interval, before k_r2_batch): its start on the window and its cigar length
__global__ __launch_bounds__(64) void k_r2_readcl(ReadArgs R, const uint8_t *__restrict__ host, const uint64_t *__restrict__ kc,
                                                  const uint64_t *__restrict__ ac, uint32_t *__restrict__ read_cl,
                                                  int32_t *__restrict__ read_start) {
    const uint32_t w = blockIdx.x, lane = threadIdx.x;
    if (host[w] || kc[w + 1] == kc[w]) return;
    const uint64_t a = R.rd_off[w], b = R.rd_off[w + 1];
    uint64_t ri = ac[w];
    for (uint64_t r0 = a; r0 < b; r0 += 64) {
        const uint64_t r = r0 + lane;
        const bool alt = r < b && (R.out[r].flags & oge::DP_ALT);
        const uint64_t m = __ballot(alt);
        if (alt) {
            const uint64_t k = ri + __popcll(m & ((1ull << lane) - 1));
            read_cl[k] = R.out[r].cig_len;
            read_start[k] = R.start[r];
        }
        ri += __popcll(m);
    }
}

// per interval (one wave): the batch -- kept consensus bytes, altRead bases / raw qualities, offsets, plane
// word offsets, and the pairs (consensus-major, as the host batch) with orig and maxStart (:1149-1150)
struct BatchArgs {
    ReadArgs R;
    const uint64_t *cand_off, *cand_len;
    const uint8_t *cand, *host;
    const uint64_t *kc, *kb, *kw, *ac, *ab, *aw, *pc;  // exclusive scans
    const uint32_t *read_cl;
    const int32_t *read_start;
    uint8_t *cons;
    uint64_t *cons_off, *cwo;
    uint8_t *bases, *quals;
    uint64_t *read_off, *rwo;
    int4 *pairs;
};

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v, uint32_t lane) {  // inclusive prefix sum over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = ((uint64_t)__shfl_up((unsigned)(v >> 32), d, 64) << 32) | (uint64_t)__shfl_up((unsigned)v, d, 64);
        if (lane >= (uint32_t)d) v += o;
    }
    return v;
}

// A chunk of 64 reads at a time: each lane loads its own read's summary, record header and cigar and takes
// its offsets from the wave's prefix sums; then the chunk's kept consensuses and altReads are copied one after
// the other by the whole wave (consecutive bytes per lane), each read's pointers, offsets and cigar handed to
// the wave by shuffles.  (r06: one read at a time with every lane loading the same summary and header --
// dependent round trips per read -- took 3.4 ms of C5; a lane copying its own read's bytes, 9 ms.)
__global__ __launch_bounds__(64) void k_r2_batch(BatchArgs A) {
    __shared__ uint32_t clen_s[kCandCap];
    const uint32_t w = blockIdx.x, lane = threadIdx.x;
    if (A.host[w] || A.kc[w + 1] == A.kc[w]) return;
    const uint64_t a = A.R.rd_off[w], b = A.R.rd_off[w + 1];
    const uint64_t n_alt = A.ac[w + 1] - A.ac[w], n_kept = A.kc[w + 1] - A.kc[w];
    uint64_t ci = A.kc[w], cb = A.kb[w], cw = A.kw[w];
    uint64_t ri = A.ac[w], rb = A.ab[w], rw = A.aw[w];
    uint64_t c0 = 0;
    auto bc64 = [](uint64_t v, int src) {
        return ((uint64_t)__shfl((unsigned)(v >> 32), src, 64) << 32) | (uint64_t)__shfl((unsigned)v, src, 64);
    };
    for (uint64_t r0 = a; r0 < b; r0 += 64) {
        const uint64_t r = r0 + lane;
        uint8_t f = 0;
        uint32_t ul = 0;
        uint64_t len = 0;
        if (r < b) {
            f = A.R.out[r].flags;
            if (f & oge::DP_ALT) ul = A.R.out[r].ul;
            if (f & oge::DP_KEPT) len = A.cand_len[r];
        }
        const bool kept = f & oge::DP_KEPT, alt = f & oge::DP_ALT;
        const uint64_t kw1 = kept ? (len + 63) / 64 + 1 : 0, aw1 = alt ? (ul + 63) / 64 : 0;
        const uint64_t ik = wave_incl_u64(kept, lane), il = wave_incl_u64(len, lane), iw = wave_incl_u64(kw1, lane);
        const uint64_t ia = wave_incl_u64(alt, lane), iu = wave_incl_u64(ul, lane), iaw = wave_incl_u64(aw1, lane);
        // this lane's read: offsets, and for an altRead its header and cigar (packed len << 4 | code)
        uint64_t src_c = 0, dst_c = cb + il - len, dst_r = rb + iu - ul, seq4 = 0, qual = 0;
        uint32_t ops[kMaxIn], nops = 0;
        int64_t lseq = 0;
        if (kept) {
            src_c = (uint64_t)(uintptr_t)(A.cand + A.cand_off[r]);
            A.cons_off[ci + ik - 1] = dst_c;
            A.cwo[ci + ik - 1] = cw + iw - kw1;
            clen_s[c0 + ik - 1] = (uint32_t)len;
        }
        if (alt) {
            Cig orig;
            Read rd;
            uint32_t flag;
            bool fits;
            load_read(A.R.recs + A.R.rec[r], orig, rd, &flag, &fits);
            seq4 = (uint64_t)(uintptr_t)rd.seq4, qual = (uint64_t)(uintptr_t)rd.qual, lseq = rd.lseq;
            nops = (uint32_t)orig.n;
#pragma unroll
            for (int j = 0; j < kMaxIn; ++j) ops[j] = j < orig.n ? (orig.len[j] << 4) | orig.code[j] : 0u;
            A.read_off[ri + ia - 1] = dst_r;
            A.rwo[ri + ia - 1] = rw + iaw - aw1;
        }
        // the copies, read by read, by the whole wave
        uint64_t mk = __ballot(kept);
        while (mk) {
            const int src = __builtin_ctzll(mk);
            mk &= mk - 1;
            const uint8_t *from = (const uint8_t *)(uintptr_t)bc64(src_c, src);
            const uint64_t to = bc64(dst_c, src), n = bc64(len, src);
            for (uint64_t k = lane; k < n; k += 64) A.cons[to + k] = from[k];
        }
        uint64_t ma = __ballot(alt);
        while (ma) {
            const int src = __builtin_ctzll(ma);
            ma &= ma - 1;
            Cig orig;
            orig.n = (int)__shfl(nops, src, 64);
#pragma unroll
            for (int j = 0; j < kMaxIn; ++j) {
                const uint32_t o = __shfl(ops[j], src, 64);
                orig.len[j] = o >> 4, orig.code[j] = (uint8_t)(o & 15);
            }
            Read rd;
            rd.seq4 = (const uint8_t *)(uintptr_t)bc64(seq4, src);
            rd.qual = (const uint8_t *)(uintptr_t)bc64(qual, src);
            rd.lseq = (int64_t)bc64((uint64_t)lseq, src);
            const uint64_t to = bc64(dst_r, src), n = __shfl(ul, src, 64);
            for (uint64_t k = lane; k < n; k += 64) {
                const int64_t p = unclipped_pos(orig, (int64_t)k, rd.lseq);
                A.bases[to + k] = (uint8_t)rd.base(p);
                A.quals[to + k] = rd.qual[p];
            }
        }
        auto last = [](uint64_t v) { return (uint64_t)__shfl((unsigned long long)v, 63, 64); };
        ci += last(ik), cb += last(il), cw += last(iw), c0 += last(ik);
        ri += last(ia), rb += last(iu), rw += last(iaw);
    }
    __syncthreads();
    const uint64_t np = n_kept * n_alt;
    for (uint64_t p = lane; p < np; p += 64) {
        const uint64_t cc = p / n_alt, j = p % n_alt, gj = A.ac[w] + j;
        int4 q;
        q.x = (int)(A.kc[w] + cc);
        q.y = (int)gj;
        q.z = A.read_start[gj];
        q.w = (int)clen_s[cc] - (int)A.read_cl[gj];
        A.pairs[A.pc[w] + p] = q;
    }
}

}  // namespace

// Phase B + the batch on the device; then the offset scan (realign.hip).  d_recs: the staged arena.
int oge_realign_prep_run(oge_ctx *ctx, const uint8_t *d_recs, const oge::DevPrepBatch &B, oge::DevPrepOut &O) {
    auto clk = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = clk();
    const uint32_t nw = (uint32_t)(B.rd_off.size() - 1);
    const uint64_t nr = B.rec.size();
    O.reads.resize(nr);  // (every entry copied back from the device below)
    O.iv_host.assign(nw, 0);
    O.iv_total_raw.assign(nw, 0);
    O.iv_pair_base.assign(nw, 0);
    O.best_index.clear(), O.best_score.clear();
    O.pairs = O.ops = 0;
    O.generic = false;
    if (!nw) return OGE_OK;
    hipStream_t s = ctx->stream;
    // inputs
    uint8_t *dref = (uint8_t *)ctx->ws("rp_ref", B.ref.size() + 16);
    uint64_t *dref_off = (uint64_t *)ctx->ws("rp_ref_off", (nw + 1) * 8);
    uint64_t *drd_off = (uint64_t *)ctx->ws("rp_rd_off", (nw + 1) * 8);
    uint64_t *drec = (uint64_t *)ctx->ws("rp_rec", (nr + 1) * 8);
    int32_t *dstart = (int32_t *)ctx->ws("rp_start", (nr + 1) * 4);
    DevPrepRead *dout = (DevPrepRead *)ctx->ws("rp_out", (nr + 1) * sizeof(DevPrepRead));
    uint64_t *dclen = (uint64_t *)ctx->ws("rp_clen", (nr + 1) * 8);
    uint64_t *dcoff = (uint64_t *)ctx->ws("rp_coff", (nr + 1) * 8);
    uint64_t *dchash = (uint64_t *)ctx->ws("rp_chash", (nr + 1) * 8);
    uint64_t *iva = (uint64_t *)ctx->ws("rp_iv", 7 * (uint64_t)(nw + 1) * 8);
    int64_t *dtraw = (int64_t *)ctx->ws("rp_traw", (nw + 1) * 8);
    uint8_t *dhost = (uint8_t *)ctx->ws("rp_host", nw + 1);
    if (!dref || !dref_off || !drd_off || !drec || !dstart || !dout || !dclen || !dcoff || !dchash || !iva || !dtraw || !dhost)
        return OGE_ERR_HIP;
    if (!B.ref.empty()) OGE_HIP_TRY(ctx, hipMemcpyAsync(dref, B.ref.data(), B.ref.size(), hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dref_off, B.ref_off.data(), (nw + 1) * 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(drd_off, B.rd_off.data(), (nw + 1) * 8, hipMemcpyHostToDevice, s));
    if (nr) {
        OGE_HIP_TRY(ctx, hipMemcpyAsync(drec, B.rec.data(), nr * 8, hipMemcpyHostToDevice, s));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dstart, B.start.data(), nr * 4, hipMemcpyHostToDevice, s));
    }
    OgeStageTimer *tm = ctx->begin_stage("realign_prep");
    ReadArgs RA{d_recs, drec, dstart, drd_off, nw, nr, dref, dref_off, dout, dclen};
    if (nr) {
        hipLaunchKernelGGL(k_r2_read, dim3((uint32_t)((nr + kT - 1) / kT)), dim3(kT), 0, s, RA);
        OGE_LAUNCH_CHECK(ctx);
    }
    OGE_HIP_TRY(ctx, hipMemsetAsync(dclen + nr, 0, 8, s));
    int rc = oge_exclusive_scan_u64(ctx, dclen, dcoff, nr + 1);
    if (rc) return rc;
    uint64_t cand_bytes = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&cand_bytes, dcoff + nr, 8, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    uint8_t *dcand = (uint8_t *)ctx->ws("rp_cand", cand_bytes + 16);
    if (!dcand) return OGE_ERR_HIP;
    if (nr) {
        hipLaunchKernelGGL(k_r2_cand, dim3((uint32_t)((nr + kT - 1) / kT)), dim3(kT), 0, s, RA, (const uint64_t *)dcoff, dcand, dchash);
        OGE_LAUNCH_CHECK(ctx);
    }
    uint64_t *kc = iva, *kb = iva + (nw + 1), *kw = iva + 2 * (nw + 1), *ac = iva + 3 * (nw + 1), *ab = iva + 4 * (nw + 1),
             *aw = iva + 5 * (nw + 1), *pc = iva + 6 * (nw + 1);
    IvArgs IA{drd_off, nw, dout, dclen, dcoff, dchash, dcand, kc, kb, kw, ac, ab, aw, pc, dtraw, dhost};
    hipLaunchKernelGGL(k_r2_iv, dim3(nw), dim3(64), 0, s, IA);
    OGE_LAUNCH_CHECK(ctx);
    for (uint64_t *x : {kc, kb, kw, ac, ab, aw, pc})
        if ((rc = oge_exclusive_scan_u64(ctx, x, x, nw + 1))) return rc;
    uint64_t tot[7];
    for (int k = 0; k < 7; ++k) OGE_HIP_TRY(ctx, hipMemcpyAsync(&tot[k], iva + k * (uint64_t)(nw + 1) + nw, 8, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    const uint64_t n_cons = tot[0], cons_bytes = tot[1], cons_words = tot[2], n_reads = tot[3], read_bytes = tot[4],
                   read_words = tot[5], n_pairs = tot[6];
    if (n_cons > 0x7FFFFFFFull || n_reads > 0x7FFFFFFFull || n_pairs > 0x7FFFFFFFull)
        return oge_fail(ctx, OGE_ERR_LIMIT, "realign prep: batch too large");
    // the batch
    uint8_t *dc = (uint8_t *)ctx->ws("rs_cons", cons_bytes + 16);
    uint64_t *dco = (uint64_t *)ctx->ws("rs_cons_off", (n_cons + 1) * 8);
    uint64_t *dcwo = (uint64_t *)ctx->ws("rs_cwo", (n_cons + 1) * 8);
    uint8_t *db = (uint8_t *)ctx->ws("rs_bases", read_bytes + 16);
    uint8_t *dq = (uint8_t *)ctx->ws("rs_quals", read_bytes + 16);
    uint64_t *dro = (uint64_t *)ctx->ws("rs_read_off", (n_reads + 1) * 8);
    uint64_t *drwo = (uint64_t *)ctx->ws("rs_rwo", (n_reads + 1) * 8);
    int4 *dp = (int4 *)ctx->ws("rs_pairs", (n_pairs + 1) * 16);
    uint32_t *drcl = (uint32_t *)ctx->ws("rp_rcl", (n_reads + 1) * 4);
    int32_t *drst = (int32_t *)ctx->ws("rp_rst", (n_reads + 1) * 4);
    if (!dc || !dco || !dcwo || !db || !dq || !dro || !drwo || !dp || !drcl || !drst) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_r2_readcl, dim3(nw), dim3(64), 0, s, RA, (const uint8_t *)dhost, (const uint64_t *)kc, (const uint64_t *)ac, drcl,
                       drst);
    OGE_LAUNCH_CHECK(ctx);
    BatchArgs BA{RA, dcoff, dclen, dcand, dhost, kc, kb, kw, ac, ab, aw, pc, drcl, drst, dc, dco, dcwo, db, dq, dro, drwo, dp};
    hipLaunchKernelGGL(k_r2_batch, dim3(nw), dim3(64), 0, s, BA);
    OGE_LAUNCH_CHECK(ctx);
    const uint64_t ends[4] = {cons_bytes, cons_words, read_bytes, read_words};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dco + n_cons, &ends[0], 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dcwo + n_cons, &ends[1], 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dro + n_reads, &ends[2], 8, hipMemcpyHostToDevice, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(drwo + n_reads, &ends[3], 8, hipMemcpyHostToDevice, s));
    ctx->end_stage(tm);
    const double t1 = clk();
    // the offset scan over the batch in place
    O.best_index.resize(n_pairs);  // (written by the scan)
    O.best_score.resize(n_pairs);
    RsDevBatch S{dc, dco, (uint32_t)n_cons, dcwo, cons_words, db, dq, dro, (uint32_t)n_reads, drwo, read_words, dp, n_pairs};
    if (n_pairs) {
        if ((rc = realign_scan_devbatch(ctx, S, O.best_index.data(), O.best_score.data(), &O.generic))) return rc;
    }
    const double t2 = clk();
    // results
    if (nr) OGE_HIP_TRY(ctx, hipMemcpyAsync(O.reads.data(), dout, nr * sizeof(DevPrepRead), hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(O.iv_host.data(), dhost, nw, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(O.iv_total_raw.data(), dtraw, nw * 8, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(O.iv_pair_base.data(), pc, nw * 8, hipMemcpyDeviceToHost, s));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(s));
    O.pairs = n_pairs;
    O.t_device = t1 - t0;
    O.t_download = clk() - t2;
    return OGE_OK;
}
