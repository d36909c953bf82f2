// markdup.hip -- Picard-style duplicate marking (MarkDuplicates, algorithms/mark_duplicates.cpp)
// as data-parallel HIP kernels on gfx950.
//
//  k_readends   : one thread per record builds the fragment ReadEnds fields
//                 (buildReadEnds :147-164 with getUnclippedStart/End :88-129, getScore :135-144,
//                 getLibraryId/Name :282-318) plus a 32-bit hash of the pair key RG ":" name (:210-213)
//  mate join    : pair candidates sorted by hash (stable, so record order inside a hash run);
//                 k_pair_runs pairs consecutive occurrences of each exact key (the first-seen /
//                 second-seen semantics of the ReadEndsMap at :214-245)
//  k_pair_build : read1/read2 choice, orientation byte and int16 score sum of :222-243
//  groups       : pairs sorted by (lib,r1Seq,r1Coord,orient,r2Seq,r2Coord), fragments by
//                 (lib,r1Seq,r1Coord,orient); one thread per group head applies
//                 markDuplicatePairs / markDuplicateFragments (:488-540): best = first strict max
//                 score in index order; fragments only when the chunk holds an unpaired end.
//  k_apply      : every primary record gets 0x400 set/cleared, others untouched (:443-465).
#include "oge_ctx.h"
#include "bam_layout.h"

#include <algorithm>
#include <vector>

namespace {

constexpr int kT = 256;
enum { RE_F = 1, RE_R = 2, RE_FF = 3, RE_RR = 4, RE_FR = 5, RE_RF = 6 };

// meta bit layout (u64 per record)
constexpr uint64_t M_FRAG = 1ull << 32, M_REV = 1ull << 33, M_CAND = 1ull << 34, M_PRIMARY = 1ull << 35,
                   M_PAIRED = 1ull << 36;
// meta[15:0] score (int16), meta[31:16] library id

__device__ __forceinline__ const uint8_t *cigar_ptr(const uint8_t *r) { return r + OGE_OFF_NAME + r[OGE_OFF_LNAME]; }

// BamAlignment::GetTag<std::string>("RG") -- FindTag/SkipToNextTag semantics
// (util/bamtools/BamAlignment.cpp:270-294,699-780; BamAlignment.h:576-606)
__device__ bool get_rg(const uint8_t *r, const uint8_t **val, uint32_t *len) {
    uint32_t bs = oge_rd_u32(r);
    uint32_t lseq = oge_rd_u32(r + OGE_OFF_LSEQ), nc = oge_rd_u16(r + OGE_OFF_NCIGAR);
    const uint8_t *p = cigar_ptr(r) + 4 * nc + (lseq + 1) / 2 + lseq;
    const uint8_t *end = r + 4 + bs;
    while (p + 3 <= end) {
        const uint8_t *tag = p;
        uint8_t type = p[2];
        p += 3;
        if (tag[0] == 'R' && tag[1] == 'G') {
            const uint8_t *s = p;
            while (s < end && *s) ++s;
            *val = p;
            *len = (uint32_t)(s - p);
            return true;
        }
        if (type == 0) return false;
        switch (type) {
        case 'A': case 'c': case 'C': p += 1; break;
        case 's': case 'S': p += 2; break;
        case 'f': case 'i': case 'I': p += 4; break;
        case 'Z': case 'H':
            while (p < end && *p) ++p;
            ++p;
            break;
        case 'B': {
            if (p + 5 > end) return false;
            uint8_t at = p[0];
            int32_t cnt = oge_rd_i32(p + 1);
            p += 5;
            int sz = (at == 'c' || at == 'C') ? 1 : (at == 's' || at == 'S') ? 2 : (at == 'f' || at == 'i' || at == 'I') ? 4 : 0;
            if (!sz) return false;
            p += (int64_t)cnt * sz;
            break;
        }
        default: return false;
        }
        if (p >= end || *p == 0) return false;
    }
    return false;
}

__device__ __forceinline__ uint32_t fnv_step(uint32_t h, uint8_t b) { return (h ^ b) * 16777619u; }

__global__ __launch_bounds__(kT) void k_readends(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                                                  const uint8_t *__restrict__ rg_ids, const int16_t *__restrict__ rg_lib,
                                                  int32_t n_rg, int16_t unknown_lib, uint64_t *__restrict__ meta,
                                                  int32_t *__restrict__ seq, int32_t *__restrict__ coord,
                                                  int32_t *__restrict__ r2seq, uint32_t *__restrict__ hash) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[i];
    uint32_t flag = oge_rd_u16(r + OGE_OFF_FLAG);
    int32_t ref = oge_rd_i32(r + OGE_OFF_REFID);
    uint64_t m = 0;
    if (!(flag & OGE_F_SECONDARY)) m |= M_PRIMARY;
    if ((flag & OGE_F_UNMAP) || ref == -1 || (flag & OGE_F_SECONDARY)) {
        meta[i] = m;
        return;
    }
    m |= M_FRAG;
    bool rev = (flag & OGE_F_REVERSE) != 0;
    if (rev) m |= M_REV;
    int32_t pos = oge_rd_i32(r + OGE_OFF_POS);
    uint32_t nc = oge_rd_u16(r + OGE_OFF_NCIGAR);
    const uint8_t *c = cigar_ptr(r);
    int32_t cd;
    if (!rev) {  // getUnclippedStart
        cd = pos;
        for (uint32_t k = 0; k < nc; ++k) {
            uint32_t op = oge_rd_u32(c + 4 * k), t = op & 0xF;
            if (t == OGE_CIG_S || t == OGE_CIG_H) cd -= (int32_t)(op >> 4); else break;
        }
    } else {  // getUnclippedEnd = getAlignmentEnd + trailing clips
        int32_t rl = 0;
        for (uint32_t k = 0; k < nc; ++k) {
            uint32_t op = oge_rd_u32(c + 4 * k), t = op & 0xF;
            if (t == OGE_CIG_M || t == OGE_CIG_D || t == OGE_CIG_N || t == OGE_CIG_EQ || t == OGE_CIG_X) rl += (int32_t)(op >> 4);
        }
        cd = pos + rl - 1;
        for (int k = (int)nc - 1; k >= 0; --k) {
            uint32_t op = oge_rd_u32(c + 4 * k), t = op & 0xF;
            if (t == OGE_CIG_S || t == OGE_CIG_H) cd += (int32_t)(op >> 4); else break;
        }
    }
    // getScore: int16 sum of raw qual bytes >= 15
    uint32_t lseq = oge_rd_u32(r + OGE_OFF_LSEQ);
    const uint8_t *q = c + 4 * nc + (lseq + 1) / 2;
    uint32_t sc = 0;
    uint32_t k = 0;
    const uint32_t qmis = (uint32_t)((uintptr_t)q & 3);
    for (; k < lseq && ((k + qmis) & 3); ++k) { uint32_t b = q[k]; sc += b >= 15 ? b : 0; }
    for (; k + 4 <= lseq; k += 4) {
        uint32_t w = *(const uint32_t *)(q + k);
#pragma unroll
        for (int s = 0; s < 4; ++s) { uint32_t b = (w >> (8 * s)) & 0xff; sc += b >= 15 ? b : 0; }
    }
    for (; k < lseq; ++k) { uint32_t b = q[k]; sc += b >= 15 ? b : 0; }
    // library via RG
    const uint8_t *rgv = nullptr;
    uint32_t rgl = 0;
    bool has = get_rg(r, &rgv, &rgl);
    if (!has) rgl = 0;
    int16_t lib = unknown_lib;
    if (has && rgl) {
        const uint8_t *p = rg_ids;
        for (int32_t g = 0; g < n_rg; ++g) {
            uint32_t L = 0;
            while (p[L]) ++L;
            if (L == rgl) {
                bool eq = true;
                for (uint32_t x = 0; x < L && eq; ++x) eq = p[x] == rgv[x];
                if (eq) { lib = rg_lib[g]; break; }
            }
            p += L + 1;
        }
    }
    m |= (uint64_t)(uint16_t)(int16_t)sc | ((uint64_t)(uint16_t)lib << 16);
    bool paired_mm = (flag & OGE_F_PAIRED) && !(flag & OGE_F_MUNMAP);
    int32_t mref = oge_rd_i32(r + OGE_OFF_MREFID);
    int32_t r2 = paired_mm ? mref : -1;
    if (r2 != -1) m |= M_PAIRED;
    if (paired_mm) {
        m |= M_CAND;
        uint32_t h = 2166136261u;
        for (uint32_t x = 0; x < rgl; ++x) h = fnv_step(h, rgv[x]);
        h = fnv_step(h, ':');
        uint32_t nl = r[OGE_OFF_LNAME] ? r[OGE_OFF_LNAME] - 1u : 0u;
        for (uint32_t x = 0; x < nl; ++x) h = fnv_step(h, r[OGE_OFF_NAME + x]);
        hash[i] = h;
    }
    meta[i] = m;
    seq[i] = ref;
    coord[i] = cd;
    r2seq[i] = r2;
}

// --- compaction of pair candidates (order-preserving) ---
__global__ __launch_bounds__(kT) void k_cand_flags(const uint64_t *__restrict__ meta, uint64_t n, uint32_t *__restrict__ f) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n) f[i] = (meta[i] & M_CAND) ? 1u : 0u;
    else if (i == n) f[i] = 0;
}
__global__ __launch_bounds__(kT) void k_cand_scatter(const uint64_t *__restrict__ meta, const uint32_t *__restrict__ hash,
                                                      uint64_t n, const uint32_t *__restrict__ pos,
                                                      uint64_t *__restrict__ ckey, uint32_t *__restrict__ cval) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n && (meta[i] & M_CAND)) {
        uint32_t p = pos[i];
        ckey[p] = hash[i];
        cval[p] = (uint32_t)i;
    }
}

// key byte k of RG ":" name for record r
__device__ __forceinline__ uint8_t key_byte(const uint8_t *rgv, uint32_t rgl, const uint8_t *name, uint32_t k) {
    return k < rgl ? rgv[k] : (k == rgl ? (uint8_t)':' : name[k - rgl - 1]);
}
__device__ bool same_pair_key(const uint8_t *recs, const uint64_t *off, uint32_t a, uint32_t b) {
    const uint8_t *ra = recs + off[a], *rb = recs + off[b];
    const uint8_t *ga = nullptr, *gb = nullptr;
    uint32_t la = 0, lb = 0;
    if (!get_rg(ra, &ga, &la)) la = 0;
    if (!get_rg(rb, &gb, &lb)) lb = 0;
    uint32_t na = ra[OGE_OFF_LNAME] ? ra[OGE_OFF_LNAME] - 1u : 0u, nb = rb[OGE_OFF_LNAME] ? rb[OGE_OFF_LNAME] - 1u : 0u;
    if (la + na != lb + nb) return false;
    uint32_t L = la + 1 + na;
    for (uint32_t k = 0; k < L; ++k)
        if (key_byte(ga, la, ra + OGE_OFF_NAME, k) != key_byte(gb, lb, rb + OGE_OFF_NAME, k)) return false;
    return true;
}

// One thread per hash run: pair consecutive occurrences of each exact key (in record order).
__global__ __launch_bounds__(kT) void k_pair_runs(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off,
                                                   const uint64_t *__restrict__ ckey, const uint32_t *__restrict__ cval,
                                                   uint64_t nc, uint8_t *__restrict__ used, uint2 *__restrict__ pairs,
                                                   unsigned int *__restrict__ npairs) {
    uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (p >= nc) return;
    uint64_t h = ckey[p];
    if (p > 0 && ckey[p - 1] == h) return;
    uint64_t e = p + 1;
    while (e < nc && ckey[e] == h) ++e;
    if (e - p == 2) {  // common case: exactly two candidates share the hash
        if (same_pair_key(recs, off, cval[p], cval[p + 1])) {
            unsigned int s = atomicAdd(npairs, 1u);
            pairs[s] = make_uint2(cval[p], cval[p + 1]);
        }
        return;
    }
    for (uint64_t a = p; a < e; ++a) {
        if (used[a]) continue;
        for (uint64_t b = a + 1; b < e; ++b) {
            if (used[b]) continue;
            if (same_pair_key(recs, off, cval[a], cval[b])) {
                used[a] = used[b] = 1;
                unsigned int s = atomicAdd(npairs, 1u);
                pairs[s] = make_uint2(cval[a], cval[b]);
                break;
            }
        }
    }
}

struct KeyLayout {
    uint32_t sb, lb;  // bits for refID and library id
};

__device__ __forceinline__ int orient_byte(bool r1neg, bool r2neg) {
    return r1neg ? (r2neg ? RE_RR : RE_RF) : (r2neg ? RE_FR : RE_FF);
}

// hi = score(16) << 48 | lib << (sb+32) | r1Seq << 32 | biased r1Coord
// lo = (orient-3) << (sb+32) | r2Seq << 32 | biased r2Coord
__global__ __launch_bounds__(kT) void k_pair_build(const uint2 *__restrict__ pairs, uint32_t np,
                                                    const uint64_t *__restrict__ meta, const int32_t *__restrict__ seq,
                                                    const int32_t *__restrict__ coord, KeyLayout L, uint64_t *__restrict__ hi,
                                                    uint64_t *__restrict__ lo, uint2 *__restrict__ idx, uint32_t *__restrict__ val) {
    uint32_t p = blockIdx.x * kT + threadIdx.x;
    if (p >= np) return;
    uint32_t a = pairs[p].x, b = pairs[p].y;  // a seen first (smaller record index)
    if (a > b) { uint32_t t = a; a = b; b = t; }
    uint64_t ma = meta[a], mb = meta[b];
    int32_t sa = seq[a], ca = coord[a], sb_ = seq[b], cb = coord[b];
    bool reva = (ma & M_REV) != 0, revb = (mb & M_REV) != 0;
    int32_t r1s, r1c, r2s, r2c;
    uint32_t i1, i2;
    int o;
    if (sb_ > sa || (sb_ == sa && cb >= ca)) {
        r1s = sa; r1c = ca; r2s = sb_; r2c = cb; i1 = a; i2 = b;
        o = orient_byte(reva, revb);
    } else {
        r1s = sb_; r1c = cb; r2s = sa; r2c = ca; i1 = b; i2 = a;
        o = orient_byte(revb, reva);
    }
    uint16_t score = (uint16_t)((int16_t)(uint16_t)(ma & 0xFFFF) + (int16_t)(uint16_t)(mb & 0xFFFF));
    uint64_t lib = (ma >> 16) & 0xFFFF;
    hi[p] = ((uint64_t)score << 48) | (lib << (L.sb + 32)) | ((uint64_t)(uint32_t)r1s << 32) |
            (uint64_t)((uint32_t)r1c ^ 0x80000000u);
    lo[p] = ((uint64_t)(o - RE_FF) << (L.sb + 32)) | ((uint64_t)(uint32_t)r2s << 32) | (uint64_t)((uint32_t)r2c ^ 0x80000000u);
    idx[p] = make_uint2(i1, i2);
    val[p] = p;
}

__global__ __launch_bounds__(kT) void k_gather_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ by,
                                                    uint32_t n, uint64_t *__restrict__ dst) {
    uint32_t p = blockIdx.x * kT + threadIdx.x;
    if (p < n) dst[p] = src[by[p]];
}

// One thread per pair group (sorted by (hi, lo)): best = max score, ties -> smallest read1 index.
__global__ __launch_bounds__(kT) void k_pair_groups(const uint64_t *__restrict__ shi, const uint32_t *__restrict__ sval,
                                                     const uint64_t *__restrict__ lo, const uint2 *__restrict__ idx, uint32_t np,
                                                     uint8_t *__restrict__ dup) {
    uint32_t q = blockIdx.x * kT + threadIdx.x;
    if (q >= np) return;
    const uint64_t kmask = (1ull << 48) - 1;
    uint64_t h = shi[q] & kmask, l = lo[sval[q]];
    if (q > 0 && (shi[q - 1] & kmask) == h && lo[sval[q - 1]] == l) return;
    uint32_t e = q + 1;
    while (e < np && (shi[e] & kmask) == h && lo[sval[e]] == l) ++e;
    if (e - q < 2) return;
    uint32_t best = q;
    int16_t bs = (int16_t)(uint16_t)(shi[q] >> 48);
    uint32_t bi = idx[sval[q]].x;
    for (uint32_t x = q + 1; x < e; ++x) {
        int16_t s = (int16_t)(uint16_t)(shi[x] >> 48);
        uint32_t i1 = idx[sval[x]].x;
        if (s > bs || (s == bs && i1 < bi)) { best = x; bs = s; bi = i1; }
    }
    for (uint32_t x = q; x < e; ++x) {
        if (x == best) continue;
        uint2 ii = idx[sval[x]];
        dup[ii.x] = 1;
        dup[ii.y] = 1;
    }
}

// fragment key: bit 63 paired, bits [47,63) score, bit 46 "not a fragment",
// lib << (sb+33) | refID << 33 | biased coord << 1 | reverse
__global__ __launch_bounds__(kT) void k_frag_keys(const uint64_t *__restrict__ meta, const int32_t *__restrict__ seq,
                                                   const int32_t *__restrict__ coord, uint64_t n, KeyLayout L,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    uint64_t m = meta[i];
    uint64_t k;
    if (!(m & M_FRAG)) {
        k = 1ull << 46;
    } else {
        uint64_t lib = (m >> 16) & 0xFFFF;
        k = (lib << (L.sb + 33)) | ((uint64_t)(uint32_t)seq[i] << 33) | ((uint64_t)((uint32_t)coord[i] ^ 0x80000000u) << 1) |
            ((m & M_REV) ? 1ull : 0ull);
        k |= ((m & 0xFFFF) << 47) | ((m & M_PAIRED) ? (1ull << 63) : 0ull);
    }
    keys[i] = k;
    vals[i] = (uint32_t)i;
}

__global__ __launch_bounds__(kT) void k_frag_groups(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                     uint64_t n, uint8_t *__restrict__ dup) {
    uint64_t q = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (q >= n) return;
    const uint64_t gmask = (1ull << 47) - 1;
    uint64_t g = keys[q] & gmask;
    if (g & (1ull << 46)) return;
    if (q > 0 && (keys[q - 1] & gmask) == g) return;
    uint64_t e = q + 1;
    bool paired = (keys[q] >> 63) != 0;
    while (e < n && (keys[e] & gmask) == g) { paired |= (keys[e] >> 63) != 0; ++e; }
    if (e - q < 2) return;
    if (paired) {  // markDuplicateFragments with containsPairs: every unpaired end
        for (uint64_t x = q; x < e; ++x)
            if (!(keys[x] >> 63)) dup[vals[x]] = 1;
        return;
    }
    uint64_t best = q;
    int16_t bs = (int16_t)(uint16_t)((keys[q] >> 47) & 0xFFFF);
    for (uint64_t x = q + 1; x < e; ++x) {
        int16_t s = (int16_t)(uint16_t)((keys[x] >> 47) & 0xFFFF);
        if (s > bs) { best = x; bs = s; }
    }
    for (uint64_t x = q; x < e; ++x)
        if (x != best) dup[vals[x]] = 1;
}

__global__ __launch_bounds__(kT) void k_any(const uint8_t *__restrict__ dup, uint64_t n, unsigned int *__restrict__ any) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n && dup[i]) atomicOr(any, 1u);
}

__global__ __launch_bounds__(kT) void k_apply(uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                                               const uint64_t *__restrict__ meta, uint8_t *__restrict__ dup, int apply,
                                               int compat, const unsigned int *__restrict__ any,
                                               unsigned long long *__restrict__ ndup) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    uint32_t mine = 0;
    if (i < n) {
        uint8_t d = compat ? (uint8_t)(i == 0 && *any) : dup[i];
        if (!(meta[i] & M_PRIMARY)) {
            dup[i] = 2;
        } else {
            dup[i] = d;
            mine = d;
            if (apply) {
                uint8_t *f = recs + off[i] + OGE_OFF_FLAG;
                uint16_t flag = oge_rd_u16(f);
                uint16_t nf = d ? (uint16_t)(flag | OGE_F_DUP) : (uint16_t)(flag & ~OGE_F_DUP);
                if (nf != flag) oge_wr_u16(f, nf);
            }
        }
    }
    // per-wave count -> one atomic per wave
    unsigned long long b = __ballot(mine != 0);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ndup, (unsigned long long)__popcll(b));
}

uint32_t bits_for(uint64_t v) {  // bits to hold values 0..v
    uint32_t b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b ? b : 1;
}

}  // namespace

int oge_markdup_run(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                    uint8_t *d_dup, int apply, uint64_t *n_dup_out) {
    if (!opts) return oge_fail(ctx, OGE_ERR_ARG, "markdup: opts is NULL");
    if (n > 0xFFFFFFFEull) return oge_fail(ctx, OGE_ERR_LIMIT, "markdup: more than 2^32-2 records");
    int16_t maxlib = opts->unknown_lib;
    for (int32_t g = 0; g < opts->n_rg; ++g) maxlib = std::max(maxlib, opts->rg_lib[g]);
    if (opts->unknown_lib < 0 || maxlib < 0) return oge_fail(ctx, OGE_ERR_ARG, "markdup: negative library id");
    for (int32_t g = 0; g < opts->n_rg; ++g)
        if (opts->rg_lib[g] < 0) return oge_fail(ctx, OGE_ERR_ARG, "markdup: negative library id");
    KeyLayout L{bits_for((uint64_t)std::max(opts->n_ref, 1)), bits_for((uint64_t)maxlib)};
    if (L.sb + L.lb + 34 > 47 || L.sb + L.lb > 16)
        return oge_fail(ctx, OGE_ERR_LIMIT, "markdup: too many references x libraries for the packed group key");

    uint64_t *meta = (uint64_t *)ctx->ws("md_meta", (n + 1) * 8);
    int32_t *seq = (int32_t *)ctx->ws("md_seq", (n + 1) * 4);
    int32_t *coord = (int32_t *)ctx->ws("md_coord", (n + 1) * 4);
    int32_t *r2seq = (int32_t *)ctx->ws("md_r2seq", (n + 1) * 4);
    uint32_t *hash = (uint32_t *)ctx->ws("md_hash", (n + 1) * 4);
    uint8_t *rgtab = (uint8_t *)ctx->ws("md_rgtab", opts->rg_ids_bytes + 16);
    int16_t *rglib = (int16_t *)ctx->ws("md_rglib", (size_t)(opts->n_rg + 1) * 2);
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    unsigned long long *ndup = (unsigned long long *)ctx->ws("md_ndup", 8);
    if (!meta || !seq || !coord || !r2seq || !hash || !rgtab || !rglib || !cnt || !ndup) return OGE_ERR_HIP;
    if (opts->rg_ids_bytes)
        OGE_HIP_TRY(ctx, hipMemcpyAsync(rgtab, opts->rg_ids, opts->rg_ids_bytes, hipMemcpyHostToDevice, ctx->stream));
    if (opts->n_rg)
        OGE_HIP_TRY(ctx, hipMemcpyAsync(rglib, opts->rg_lib, (size_t)opts->n_rg * 2, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(ndup, 0, 8, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(d_dup, 0, n ? n : 1, ctx->stream));
    if (!n) { *n_dup_out = 0; return OGE_OK; }
    const uint32_t nb = oge_ceil_div(n, kT);

    OgeStageTimer *t = ctx->begin_stage("md_readends");
    hipLaunchKernelGGL(k_readends, dim3(nb), dim3(kT), 0, ctx->stream, (const uint8_t *)d_recs, d_off, n,
                       (const uint8_t *)rgtab, (const int16_t *)rglib, opts->n_rg, opts->unknown_lib, meta, seq, coord, r2seq,
                       hash);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);

    // ---- mate join ----
    t = ctx->begin_stage("md_matejoin");
    uint32_t *cpos = (uint32_t *)ctx->ws("md_cpos", (n + 1) * 4);
    if (!cpos) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_cand_flags, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)meta, n, cpos);
    OGE_LAUNCH_CHECK(ctx);
    int rc = oge_exclusive_scan_u32(ctx, cpos, cpos, n + 1);
    if (rc) return rc;
    uint32_t nc = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&nc, cpos + n, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t *ck = (uint64_t *)ctx->ws("md_ck", ((uint64_t)nc + 1) * 8);
    uint32_t *cv = (uint32_t *)ctx->ws("md_cv", ((uint64_t)nc + 1) * 4);
    uint64_t *ck2 = (uint64_t *)ctx->ws("md_ck2", ((uint64_t)nc + 1) * 8);
    uint32_t *cv2 = (uint32_t *)ctx->ws("md_cv2", ((uint64_t)nc + 1) * 4);
    uint8_t *used = (uint8_t *)ctx->ws("md_used", (uint64_t)nc + 1);
    uint2 *pairs = (uint2 *)ctx->ws("md_pairs", ((uint64_t)nc / 2 + 1) * sizeof(uint2));
    if (!ck || !cv || !ck2 || !cv2 || !used || !pairs) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_cand_scatter, dim3(nb), dim3(kT), 0, ctx->stream, (const uint64_t *)meta, (const uint32_t *)hash, n,
                       (const uint32_t *)cpos, ck, cv);
    OGE_LAUNCH_CHECK(ctx);
    uint64_t *sk;
    uint32_t *sv;
    rc = oge_radix_sort_pairs(ctx, ck, cv, ck2, cv2, nc, 0xFFFFFFFFull, &sk, &sv);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipMemsetAsync(used, 0, (uint64_t)nc + 1, ctx->stream));
    if (nc) {
        hipLaunchKernelGGL(k_pair_runs, dim3(oge_ceil_div(nc, kT)), dim3(kT), 0, ctx->stream, (const uint8_t *)d_recs, d_off,
                           (const uint64_t *)sk, (const uint32_t *)sv, (uint64_t)nc, used, pairs, cnt);
        OGE_LAUNCH_CHECK(ctx);
    }
    uint32_t np = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&np, cnt, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->end_stage(t);

    // ---- pair groups ----
    t = ctx->begin_stage("md_pairs");
    if (np) {
        uint64_t *hi = (uint64_t *)ctx->ws("md_hi", (uint64_t)np * 8);
        uint64_t *lo = (uint64_t *)ctx->ws("md_lo", (uint64_t)np * 8);
        uint64_t *lo2 = (uint64_t *)ctx->ws("md_lo2", (uint64_t)np * 8);
        uint64_t *hi2 = (uint64_t *)ctx->ws("md_hi2", (uint64_t)np * 8);
        uint2 *pidx = (uint2 *)ctx->ws("md_pidx", (uint64_t)np * sizeof(uint2));
        uint32_t *pv = (uint32_t *)ctx->ws("md_pv", (uint64_t)np * 4);
        uint32_t *pv2 = (uint32_t *)ctx->ws("md_pv2", (uint64_t)np * 4);
        if (!hi || !lo || !lo2 || !hi2 || !pidx || !pv || !pv2) return OGE_ERR_HIP;
        const uint32_t pb = oge_ceil_div(np, kT);
        hipLaunchKernelGGL(k_pair_build, dim3(pb), dim3(kT), 0, ctx->stream, (const uint2 *)pairs, np, (const uint64_t *)meta,
                           (const int32_t *)seq, (const int32_t *)coord, L, hi, lo, pidx, pv);
        OGE_LAUNCH_CHECK(ctx);
        // LSD over (hi, lo): sort by lo first (copy lo so the unsorted lo stays addressable by pair index)
        OGE_HIP_TRY(ctx, hipMemcpyAsync(lo2, lo, (uint64_t)np * 8, hipMemcpyDeviceToDevice, ctx->stream));
        uint64_t o = 0, a = 0;
        rc = oge_reduce_or_and_u64(ctx, lo2, np, ~0ull, &o, &a);
        if (rc) return rc;
        uint64_t *k1;
        uint32_t *v1;
        rc = oge_radix_sort_pairs(ctx, lo2, pv, hi2, pv2, np, o ^ a, &k1, &v1);
        if (rc) return rc;
        // gather hi in lo-sorted order, then stable sort by hi's key bits
        uint64_t *hk = (k1 == lo2) ? hi2 : lo2;
        hipLaunchKernelGGL(k_gather_u64, dim3(pb), dim3(kT), 0, ctx->stream, (const uint64_t *)hi, (const uint32_t *)v1, np, hk);
        OGE_LAUNCH_CHECK(ctx);
        rc = oge_reduce_or_and_u64(ctx, hk, np, (1ull << 48) - 1, &o, &a);
        if (rc) return rc;
        uint64_t *kt2 = (hk == lo2) ? hi2 : lo2;  // the other scratch key buffer (free now)
        uint32_t *vt2 = (v1 == pv) ? pv2 : pv;
        uint64_t *k2;
        uint32_t *v2;
        rc = oge_radix_sort_pairs(ctx, hk, v1, kt2, vt2, np, (o ^ a) & ((1ull << 48) - 1), &k2, &v2);
        if (rc) return rc;
        hipLaunchKernelGGL(k_pair_groups, dim3(pb), dim3(kT), 0, ctx->stream, (const uint64_t *)k2, (const uint32_t *)v2,
                           (const uint64_t *)lo, (const uint2 *)pidx, np, d_dup);
        OGE_LAUNCH_CHECK(ctx);
    }
    ctx->end_stage(t);

    // ---- fragment groups ----
    t = ctx->begin_stage("md_frags");
    uint64_t *fk = (uint64_t *)ctx->ws("md_fk", (n + 1) * 8);
    uint32_t *fv = (uint32_t *)ctx->ws("md_fv", (n + 1) * 4);
    uint64_t *fk2 = (uint64_t *)ctx->ws("md_fk2", (n + 1) * 8);
    uint32_t *fv2 = (uint32_t *)ctx->ws("md_fv2", (n + 1) * 4);
    if (!fk || !fv || !fk2 || !fv2) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_frag_keys, dim3(nb), dim3(kT), 0, ctx->stream, (const uint64_t *)meta, (const int32_t *)seq,
                       (const int32_t *)coord, n, L, fk, fv);
    OGE_LAUNCH_CHECK(ctx);
    {
        uint64_t o = 0, a = 0;
        rc = oge_reduce_or_and_u64(ctx, fk, n, (1ull << 47) - 1, &o, &a);
        if (rc) return rc;
        uint64_t *k;
        uint32_t *v;
        rc = oge_radix_sort_pairs(ctx, fk, fv, fk2, fv2, n, (o ^ a) & ((1ull << 47) - 1), &k, &v);
        if (rc) return rc;
        hipLaunchKernelGGL(k_frag_groups, dim3(nb), dim3(kT), 0, ctx->stream, (const uint64_t *)k, (const uint32_t *)v, n, d_dup);
        OGE_LAUNCH_CHECK(ctx);
    }
    ctx->end_stage(t);

    // ---- apply ----
    t = ctx->begin_stage("md_apply");
    if (opts->compat_nonverbose_index) {
        hipLaunchKernelGGL(k_any, dim3(nb), dim3(kT), 0, ctx->stream, (const uint8_t *)d_dup, n, cnt + 1);
        OGE_LAUNCH_CHECK(ctx);
    }
    hipLaunchKernelGGL(k_apply, dim3(nb), dim3(kT), 0, ctx->stream, d_recs, d_off, n, (const uint64_t *)meta, d_dup, apply,
                       opts->compat_nonverbose_index, (const unsigned int *)(cnt + 1), ndup);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    unsigned long long h = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&h, ndup, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_dup_out = h;
    return OGE_OK;
}
