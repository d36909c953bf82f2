// markdup.hip -- Picard-style duplicate marking (MarkDuplicates, algorithms/mark_duplicates.cpp)
// as data-parallel HIP kernels on gfx950.
//
//  readends     : per-record fragment ReadEnds fields (records.hip, k_records<*, META>): buildReadEnds
//                 :147-164, getUnclippedStart/End :88-129, getScore :135-144, getLibraryId :282-318,
//                 plus a 32-bit hash of the pair key RG ":" name (:210-213)
//  k_cand_frag  : one pass over the sorted summaries -> candidate flags, candidate hash keys,
//                 fragment sort keys and the gather descriptors (8-byte words for later passes)
//  mate join    : pair candidates sorted by hash (stable, so record order inside a hash run);
//                 k_pair_runs pairs consecutive occurrences of each exact key (the first-seen /
//                 second-seen semantics of the ReadEndsMap at :214-245)
//  k_pair_build : read1/read2 choice, orientation byte and int16 score sum of :222-243
//  groups       : pairs sorted by (lib,r1Seq,r1Coord,orient,r2Seq,r2Coord), fragments by
//                 (lib,r1Seq,r1Coord,orient); one thread per group head applies
//                 markDuplicatePairs / markDuplicateFragments (:488-540): best = first strict max
//                 score in index order; fragments only when the chunk holds an unpaired end.
//  k_apply      : every primary record gets 0x400 set/cleared, others untouched (:443-465); only
//                 records whose flag byte changes are written (standalone dedup); k_apply_desc
//                 finishes the gather descriptors instead in the fused sort + dedup pipeline.
#include "oge_ctx.h"
#include "bam_layout.h"
#include "dev_util.h"
#include "records.h"
#include "rec_parse.h"
#include "markdup_stages.h"
#include "md_keys.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr int kT = 256;
enum { RE_F = 1, RE_R = 2, RE_FF = 3, RE_RR = 4, RE_FR = 5, RE_RF = 6 };

__device__ bool pair_key_of(const uint8_t *r, const uint8_t **rg, uint32_t *rgl, uint32_t *nl) {
    const uint32_t bs = oge_ldu32(r);
    const uint32_t lname = r[OGE_OFF_LNAME], nc = oge_ldu16(r + OGE_OFF_NCIGAR), lseq = oge_ldu32(r + OGE_OFF_LSEQ);
    const uint8_t *tags = r + OGE_OFF_NAME + lname + 4 * nc + (lseq + 1) / 2 + lseq;
    if (!find_rg(tags, r + 4 + bs, rg, rgl)) *rgl = 0;
    *nl = lname ? lname - 1u : 0u;
    return true;
}

// key byte k of RG ":" name
__device__ __forceinline__ uint8_t key_byte(const uint8_t *rgv, uint32_t rgl, const uint8_t *name, uint32_t k) {
    return k < rgl ? rgv[k] : (k == rgl ? (uint8_t)':' : name[k - rgl - 1]);
}
// Exact RG ":" name comparison (the ReadEndsMap key, mark_duplicates.cpp:210-213) of the records
// summarised by A and B.  Same listed read group -> the keys are equal iff the names are, which is
// one 16-byte-chunked compare at record byte 36; anything else compares the whole key strings.
// With split_k > 1 the key also carries the chain (refID % K): SplitByChromosome gives every chain
// its own MarkDuplicates, so mates routed to different chains never meet.
__device__ bool same_pair_key(const uint8_t *recs, const RecMeta &A, const RecMeta &B, int32_t split_k) {
    if (split_k > 1 && A.seq % split_k != B.seq % split_k) return false;
    if (A.rgi == B.rgi && A.rgi != OGE_RGI_UNLISTED && (A.m & B.m & OGE_M_NAMEFIT)) {
        // same listed read group: keys equal iff names equal; both names sit NUL-terminated and
        // zero-padded in the metadata slots
        const uint4 *x = (const uint4 *)A.name, *y = (const uint4 *)B.name;
#pragma unroll
        for (uint32_t q = 0; q < OGE_NAME_SLOT / 16; ++q)
            if (x[q].x != y[q].x || x[q].y != y[q].y || x[q].z != y[q].z || x[q].w != y[q].w) return false;
        return true;
    }
    const uint8_t *ra = recs + A.src, *rb = recs + B.src;
    if (A.rgi == B.rgi && A.rgi != OGE_RGI_UNLISTED) {
        const uint32_t la = ra[OGE_OFF_LNAME];
        if (la != rb[OGE_OFF_LNAME]) return false;
        for (uint32_t k = 0; k < la; ++k)
            if (ra[OGE_OFF_NAME + k] != rb[OGE_OFF_NAME + k]) return false;
        return true;
    }
    const uint8_t *ga = nullptr, *gb = nullptr;
    uint32_t la = 0, lb = 0, na = 0, nb = 0;
    pair_key_of(ra, &ga, &la, &na);
    pair_key_of(rb, &gb, &lb, &nb);
    if (la + na != lb + nb) return false;
    const uint32_t L = la + 1 + na;
    for (uint32_t k = 0; k < L; ++k)
        if (key_byte(ga, la, ra + OGE_OFF_NAME, k) != key_byte(gb, lb, rb + OGE_OFF_NAME, k)) return false;
    return true;
}

// One thread per sorted candidate position p (a run = equal hash bits, in record order).  Common
// case, a run of exactly two: a provisional pair (first-seen a < b, confirmed by k_pair_build) at
// flag[p] / sparse[p], compacted later by a scan with no atomics.  Longer runs (hash collisions,
// supplementary records) are queued (one wave-aggregated atomic) for k_pair_runs_slow, so no wave
// waits on exact key compares.
__global__ __launch_bounds__(kT) void k_pair_runs(const uint64_t *__restrict__ ckey, uint64_t nc, CandKey ck,
                                                   uint32_t *__restrict__ flag, uint64_t *__restrict__ sparse,
                                                   uint32_t *__restrict__ slow, unsigned int *__restrict__ nslow) {
    const uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    bool queue = false;
    if (p < nc) {
        uint32_t f = 0;
        uint64_t sp = 0;
        const uint64_t kp = ckey[p];
        const uint64_t h = ck.hash_of(kp);
        if (p == 0 || ck.hash_of(ckey[p - 1]) != h) {
            uint64_t e = p + 1;
            while (e < nc && e - p <= 2 && ck.hash_of(ckey[e]) == h) ++e;
            if (e - p == 2) {
                f = 1;
                sp = ((kp & ck.idx_mask()) << 32) | (ckey[p + 1] & ck.idx_mask());
            } else if (e - p > 2) {
                queue = true;
            }
        }
        flag[p] = f;
        sparse[p] = sp;  // every slot written: whole-line stores, no partial-line read-modify-write
    } else if (p == nc) {
        flag[p] = 0;
    }
    const uint64_t m = __ballot(queue);
    if (m) {
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(nslow, (unsigned int)__popcll(m));
        base = __shfl(base, (int)leader, 64);
        if (queue) slow[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)p;
    }
}

// One thread per long run: the exact consecutive-occurrence pairing (ReadEndsMap first-seen /
// second-seen, mark_duplicates.cpp:214-245) with full key compares; a pair is stored at the
// sorted position of its first member, like the fast path.
__global__ __launch_bounds__(kT) void k_pair_runs_slow(const uint8_t *__restrict__ recs, const RecMeta *__restrict__ meta,
                                                        const uint64_t *__restrict__ ckey, uint64_t nc, CandKey ck,
                                                        const uint32_t *__restrict__ slow, uint32_t nslow,
                                                        uint8_t *__restrict__ used, uint32_t *__restrict__ flag,
                                                        uint64_t *__restrict__ sparse) {
    const uint32_t t = blockIdx.x * kT + threadIdx.x;
    if (t >= nslow) return;
    const uint64_t p = slow[t];
    const uint64_t h = ck.hash_of(ckey[p]);
    uint64_t e = p + 1;
    while (e < nc && ck.hash_of(ckey[e]) == h) ++e;
    for (uint64_t x = p; x < e; ++x) {
        if (used[x]) continue;
        const uint32_t a = (uint32_t)(ckey[x] & ck.idx_mask());
        const RecMeta A = meta[a];
        for (uint64_t y = x + 1; y < e; ++y) {
            if (used[y]) continue;
            const uint32_t b = (uint32_t)(ckey[y] & ck.idx_mask());
            if (same_pair_key(recs, A, meta[b], ck.split_k)) {
                used[x] = used[y] = 1;
                flag[x] = 1;
                sparse[x] = ((uint64_t)a << 32) | b;
                break;
            }
        }
    }
}

// after the exclusive scan, position p holds a pair iff pos[p+1] != pos[p]
__global__ __launch_bounds__(kT) void k_pair_compact_scan(const uint32_t *__restrict__ pos, const uint64_t *__restrict__ sparse,
                                                           uint64_t nc, uint64_t *__restrict__ pairs) {
    const uint64_t p = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (p < nc && pos[p + 1] != pos[p]) pairs[pos[p]] = sparse[p];
}

__device__ __forceinline__ int orient_byte(bool r1neg, bool r2neg) {
    return r1neg ? (r2neg ? RE_RR : RE_RF) : (r2neg ? RE_FR : RE_FF);
}

// Pairs (a << 32 | b, sorted by a) -> pair ReadEnds group keys.  The pair key is confirmed here
// (same_pair_key); a hash-collision "pair" gets bit 63 of lo and is ignored by k_pair_groups_h.
// hi = score(16) << 48 | lib << (sb+32) | r1Seq << 32 | biased r1Coord
// lo = invalid << 63 | (orient-3) << (sb+32) | r2Seq << 32 | biased r2Coord
// 64-bit mix of the whole chunk key (hi without score, lo): k_pair_groups_h's sort key
__device__ __forceinline__ uint64_t mix64(uint64_t h) {
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; return h ^ (h >> 33);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = ((uint64_t)__shfl_xor((unsigned)(v >> 32), d, 64) << 32) | (uint64_t)__shfl_xor((unsigned)v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}
// max(anchor - coord) and max(coord - anchor) over the items, reduced per block into slot
// (blockIdx & 255) of dev[0..511] (pairs of words); k_dev_fold folds the slots.  A single word
// would serialise millions of atomics at one L2 channel.  Every thread of the block must call it.
constexpr int kDevSlots = 256;
__device__ __forceinline__ void win_dev_update(bool has, int64_t a, int64_t c, unsigned long long *dev) {
    __shared__ uint64_t wd[2][kT / 64];
    const uint64_t d0 = wave_max_u64(has ? (uint64_t)(a - c + kDevBias) : 0ull);
    const uint64_t d1 = wave_max_u64(has ? (uint64_t)(c - a + kDevBias) : 0ull);
    if ((threadIdx.x & 63) == 0) {
        wd[0][threadIdx.x >> 6] = d0;
        wd[1][threadIdx.x >> 6] = d1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint64_t m = 0;
        for (int w = 0; w < kT / 64; ++w) m = max(m, wd[threadIdx.x][w]);
        if (m) atomicMax(dev + 2 * (blockIdx.x & (kDevSlots - 1)) + threadIdx.x, (unsigned long long)m);
    }
}
// out[0..1] = the maxima over the slots
__global__ __launch_bounds__(kDevSlots) void k_dev_fold(const unsigned long long *__restrict__ slots,
                                                        unsigned long long *__restrict__ out) {
    __shared__ unsigned long long m[2][kDevSlots];
    m[0][threadIdx.x] = slots[2 * threadIdx.x];
    m[1][threadIdx.x] = slots[2 * threadIdx.x + 1];
    __syncthreads();
    for (int h = kDevSlots / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            m[0][threadIdx.x] = max(m[0][threadIdx.x], m[0][threadIdx.x + h]);
            m[1][threadIdx.x] = max(m[1][threadIdx.x], m[1][threadIdx.x + h]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 2) out[threadIdx.x] = m[threadIdx.x][0];
}

// skeys (optional, records in sorted order): pax[p] = anchor of the pair's first record a (pairs
// arrive sorted by a) and the deviation of read1's 5' coordinate from it into dev[0..1].
// The pair ReadEnds of pair (a, b) at slot p (a seen first: the smaller record index; with win_bad, b may
// carry kSortPair).  *has / *ax / *cx: the deviation sample for win_dev_update.
__device__ __forceinline__ void pair_entry(uint32_t p, uint32_t a, uint32_t b, const uint8_t *__restrict__ recs,
                                           const RecMeta *__restrict__ meta, KeyLayout L, uint64_t *__restrict__ hi,
                                           uint64_t *__restrict__ lo, uint2 *__restrict__ idx, uint32_t *__restrict__ val,
                                           uint64_t *__restrict__ hk, const uint64_t *__restrict__ skeys,
                                           int64_t *__restrict__ pax, unsigned int *__restrict__ win_bad, bool &has,
                                           int64_t &ax, int64_t &cx) {
    // win_bad: pairs from the windowed join (b without kSortPair) whose names differ are counted
    const bool from_sort = win_bad && (b & 0x80000000u);
    if (win_bad) b &= 0x7fffffffu;
    if (a > b) { uint32_t t = a; a = b; b = t; }
    const RecMeta A = meta[a], B = meta[b];
    const uint64_t bad = same_pair_key(recs, A, B, L.split_k) ? 0ull : (1ull << 63);
    if (bad && win_bad && !from_sort) atomicAdd(win_bad, 1u);
    const uint64_t ma = A.m, mb = B.m;
    const int32_t sa = A.seq, ca = A.coord, sb_ = B.seq, cb = B.coord;
    const bool reva = (ma & OGE_M_REV) != 0, revb = (mb & OGE_M_REV) != 0;
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
    const uint16_t score = (uint16_t)((int16_t)(uint16_t)(ma & 0xFFFF) + (int16_t)(uint16_t)(mb & 0xFFFF));
    const uint64_t lib = (ma >> 16) & 0xFFFF;
    const uint64_t kh = (lib << (L.sb + 32)) | ((uint64_t)(uint32_t)r1s << 32) | (uint64_t)((uint32_t)r1c ^ 0x80000000u);
    const uint64_t kl = bad | ((uint64_t)(o - RE_FF) << (L.sb + 32)) | ((uint64_t)(uint32_t)r2s << 32) |
                        (uint64_t)((uint32_t)r2c ^ 0x80000000u);
    hi[p] = ((uint64_t)score << 48) | kh;
    lo[p] = kl;
    if (hk) {  // (the windowed join leaves them to the fallback paths that sort by them: pairs_hk)
        hk[p] = mix64(mix64(kh) ^ kl);
        val[p] = p;
    }
    idx[p] = make_uint2(i1, i2);
    if (skeys) {
        ax = anchor_of_key(skeys[a]);
        cx = win_x((uint32_t)r1s, (int64_t)r1c + 1);
        pax[p] = ax;
        has = !bad;
    }
}

__global__ __launch_bounds__(kT) void k_pair_build(const uint64_t *__restrict__ pairs, uint32_t np, const uint8_t *__restrict__ recs,
                                                    const RecMeta *__restrict__ meta, KeyLayout L, uint64_t *__restrict__ hi,
                                                    uint64_t *__restrict__ lo, uint2 *__restrict__ idx, uint32_t *__restrict__ val,
                                                    uint64_t *__restrict__ hk, const uint64_t *__restrict__ skeys,
                                                    int64_t *__restrict__ pax, unsigned long long *__restrict__ dev,
                                                    unsigned int *__restrict__ win_bad) {
    const uint32_t p = blockIdx.x * kT + threadIdx.x;
    bool has = false;
    int64_t ax = 0, cx = 0;
    if (p < np) {
        const uint64_t pr = pairs[p];
        pair_entry(p, (uint32_t)(pr >> 32), (uint32_t)pr, recs, meta, L, hi, lo, idx, val, hk, skeys, pax, win_bad, has, ax, cx);
    }
    if (skeys) win_dev_update(has, ax, cx, dev);
}

// Pair chunks (markDuplicatePairs, :488-507) need equal (lib, r1Seq, r1Coord, orient, r2Seq, r2Coord)
// contiguous, not ordered: the best of a chunk is chosen explicitly (max score, then smallest read1
// index, which is the reference's "first strict max" in its index-ordered chunk).  So pairs are
// sorted on 32 bits of a 64-bit hash of the full key (4 radix passes instead of 10 for the two
// 48-bit key words) and every run of equal hash bits is split into its exact keys here.
// (the pair's hash sort key, 32 bits of which group equal chunk keys, is written by k_pair_build)

__device__ __forceinline__ void pair_chunk(const uint32_t *__restrict__ sval, const uint64_t *__restrict__ hi,
                                           const uint64_t *__restrict__ lo, const uint2 *__restrict__ idx, uint32_t q,
                                           uint32_t e, uint64_t kh, uint64_t kl, uint8_t *__restrict__ dup) {
    const uint64_t kmask = (1ull << 48) - 1;
    uint32_t cnt = 0, best = 0xffffffffu, bi = 0;
    int16_t bs = 0;
    for (uint32_t x = q; x < e; ++x) {
        const uint32_t v = sval[x];
        const uint64_t h = hi[v];
        if ((h & kmask) != kh || lo[v] != kl) continue;
        ++cnt;
        const int16_t s = (int16_t)(uint16_t)(h >> 48);
        const uint32_t i1 = idx[v].x;
        if (best == 0xffffffffu || s > bs || (s == bs && i1 < bi)) { best = x; bs = s; bi = i1; }
    }
    if (cnt < 2) return;
    for (uint32_t x = q; x < e; ++x) {
        const uint32_t v = sval[x];
        if (x == best || (hi[v] & kmask) != kh || lo[v] != kl) continue;
        const uint2 ii = idx[v];
        dup[ii.x] = 1;
        dup[ii.y] = 1;
    }
}

__global__ __launch_bounds__(kT) void k_pair_groups_h(const uint64_t *__restrict__ shk, const uint32_t *__restrict__ sval,
                                                       const uint64_t *__restrict__ hi, const uint64_t *__restrict__ lo,
                                                       const uint2 *__restrict__ idx, uint32_t np, uint64_t rmask,
                                                       uint8_t *__restrict__ dup) {
    const uint32_t q = blockIdx.x * kT + threadIdx.x;
    if (q >= np) return;
    const uint64_t top = shk[q] & rmask, kmask = (1ull << 48) - 1;
    if (q > 0 && (shk[q - 1] & rmask) == top) return;  // one thread per run of equal sorted hash bits
    uint32_t e = q + 1;
    while (e < np && (shk[e] & rmask) == top) ++e;
    if (e - q < 2) return;
    // the common case: one exact key fills the run.  Its best pair is found in the same walk that
    // checks the keys (score, then read1 index, as pair_chunk), so each pair is gathered once.
    const uint32_t v0 = sval[q];
    const uint64_t h0 = hi[v0], qh = h0 & kmask, ql = lo[v0];
    uint32_t best = q, bi = idx[v0].x;
    int16_t bs = (int16_t)(uint16_t)(h0 >> 48);
    bool pure = true;
    for (uint32_t x = q + 1; x < e; ++x) {
        const uint32_t v = sval[x];
        const uint64_t h = hi[v];
        if ((h & kmask) != qh || lo[v] != ql) { pure = false; break; }
        const int16_t s = (int16_t)(uint16_t)(h >> 48);
        const uint32_t i1 = idx[v].x;
        if (s > bs || (s == bs && i1 < bi)) { best = x; bs = s; bi = i1; }
    }
    if (pure) {
        if (ql >> 63) return;  // unconfirmed pair key (hash collision): not a pair
        for (uint32_t x = q; x < e; ++x) {
            if (x == best) continue;
            const uint2 ii = idx[sval[x]];
            dup[ii.x] = 1;
            dup[ii.y] = 1;
        }
        return;
    }
    for (uint32_t x = q; x < e; ++x) {  // each exact key once, at its first occurrence in the run
        const uint32_t v = sval[x];
        const uint64_t kh = hi[v] & kmask, kl = lo[v];
        if (kl >> 63) continue;  // unconfirmed pair key (hash collision): not a pair
        bool seen = false;
        for (uint32_t y = q; y < x && !seen; ++y) seen = (hi[sval[y]] & kmask) == kh && lo[sval[y]] == kl;
        if (!seen) pair_chunk(sval, hi, lo, idx, x, e, kh, kl, dup);
    }
}

// One pass over the summaries for the two per-record products that need nothing else: the
// mate-join candidate flag and the fragment key, so the 64-byte rows
// are streamed once instead of twice.
// Also written here, so later kernels stream 8 bytes per record instead of the 64-byte row:
//   cval[i]  = the record's mate-join candidate key (see CandKey), scattered by k_cand_pack
//   desc0[i] = src (39 bits) | primary << 39 | bin << 40 | FLAG high byte << 56 (optional), finished
//              by k_apply_desc once the dup bits are known; a src past 39 bits sets *ovf.
// skeys (optional): the records' sorted coordinate keys; then the fragment coordinates' deviation
// from the anchors is reduced into dev[0..1] for the windowed fragment groups.
__global__ __launch_bounds__(kT) void k_cand_frag(const RecMeta *__restrict__ meta, uint64_t n, KeyLayout L, CandKey ck,
                                                   uint32_t *__restrict__ f, uint64_t *__restrict__ keys,
                                                   uint32_t *__restrict__ vals, uint64_t *__restrict__ cval,
                                                   uint64_t *__restrict__ desc0, unsigned int *__restrict__ ovf,
                                                   const uint64_t *__restrict__ skeys, unsigned long long *__restrict__ dev) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    bool has = false;
    int64_t ax = 0, cx = 0;
    if (i < n) {
        const RecMeta R = meta[i];
        cand_frag_one(R, i, L, ck, f, keys, vals, cval, desc0, ovf, skeys, has, ax, cx);
    } else if (i == n) {
        f[i] = 0;
    }
    if (skeys) win_dev_update(has, ax, cx, dev);
}

// k_cand_frag fused into the summary gather (r06, the one-GPU sort + dedup pipeline): out[i] = in[perm[i]]
// with four lanes per 64-byte row (as k_meta_gather), and the first lane of each four, given the second
// lane's 16 bytes by a shuffle, writes k_cand_frag's products for output record i -- the sorted rows are not
// streamed a second time.  perm is the FINAL order (the tie sort ran on perm first: k_ties_meta<false>).
__global__ __launch_bounds__(kT) void k_meta_gather_cf(const RecMeta *__restrict__ in, const uint32_t *__restrict__ perm,
                                                        uint64_t n, RecMeta *__restrict__ out, KeyLayout L, CandKey ck,
                                                        uint32_t *__restrict__ f, uint64_t *__restrict__ keys,
                                                        uint32_t *__restrict__ vals, uint64_t *__restrict__ cval,
                                                        uint64_t *__restrict__ desc0, unsigned int *__restrict__ ovf,
                                                        const uint64_t *__restrict__ skeys, unsigned long long *__restrict__ dev) {
    static_assert(sizeof(RecMeta) == 64 && offsetof(RecMeta, seq) == 16 && offsetof(RecMeta, hash) == 28,
                  "m, src in the first 16 bytes; seq, coord, rgi, hash_hi, hash in the next 16");
    const uint64_t g = (uint64_t)blockIdx.x * kT + threadIdx.x, i = g >> 2;
    const uint32_t part = (uint32_t)g & 3, lane = threadIdx.x & 63;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i < n) {
        v = ((const uint4 *)(in + perm[i]))[part];
        ((uint4 *)(out + i))[part] = v;
    }
    const uint32_t b0 = __shfl(v.x, (int)lane + 1, 64), b1 = __shfl(v.y, (int)lane + 1, 64);
    const uint32_t b2 = __shfl(v.z, (int)lane + 1, 64), b3 = __shfl(v.w, (int)lane + 1, 64);
    bool has = false;
    int64_t ax = 0, cx = 0;
    if (part == 0) {
        if (i < n) {
            RecMeta R;
            R.m = (uint64_t)v.x | ((uint64_t)v.y << 32);
            R.src = (uint64_t)v.z | ((uint64_t)v.w << 32);
            R.seq = (int32_t)b0;
            R.coord = (int32_t)b1;
            R.rgi = (int16_t)(b2 & 0xffff);
            R.hash_hi = (uint16_t)(b2 >> 16);
            R.hash = b3;
            cand_frag_one(R, i, L, ck, f, keys, vals, cval, desc0, ovf, skeys, has, ax, cx);
        } else if (i == n) {
            f[n] = 0;
        }
    }
    if (skeys) win_dev_update(has, ax, cx, dev);
}

// candidate i (flag = its exclusive-scan slot differs from the next one's) -> its compacted slot
__global__ __launch_bounds__(kT) void k_cand_pack(const uint32_t *__restrict__ pos, const uint64_t *__restrict__ cval,
                                                   uint64_t n, uint64_t *__restrict__ ckey) {
    uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i < n && pos[i + 1] != pos[i]) ckey[pos[i]] = cval[i];
}

__global__ __launch_bounds__(kT) void k_frag_groups(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                     uint64_t n, uint8_t *__restrict__ dup) {
    const uint64_t q = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (q >= n) return;
    const uint64_t gmask = (1ull << 47) - 1;
    const uint64_t g = keys[q] & gmask;
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
    // best = max score, then smallest record index (the reference's first strict max in index
    // order; explicit, so the group's order in the array does not matter)
    uint64_t best = q;
    int16_t bs = (int16_t)(uint16_t)((keys[q] >> 47) & 0xFFFF);
    uint32_t bv = vals[q];
    for (uint64_t x = q + 1; x < e; ++x) {
        const int16_t s = (int16_t)(uint16_t)((keys[x] >> 47) & 0xFFFF);
        const uint32_t v = vals[x];
        if (s > bs || (s == bs && v < bv)) { best = x; bs = s; bv = v; }
    }
    for (uint64_t x = q; x < e; ++x)
        if (x != best) dup[vals[x]] = 1;
}

// ---- windowed groups: markDuplicateFragments / markDuplicatePairs without a global sort ----
// Items (records, or pairs ordered by their first record) are in anchor order; each has a group
// coordinate C (5' coordinate of the fragment / of read1) with D1 >= A - C and D2 >= C - A (exact
// maxima reduced by k_cand_frag / k_pair_build).  Tile t (items [tT, tT+T)) owns the groups whose C
// lies in [A(tT), A(tT+T)) (first tile from -inf, last to +inf): every group has one owner, and all
// its members lie in the window of items whose anchors are in [A(tT) - D2, A(tT+T) + D1).  The
// owner builds the groups in an LDS hash table (best = max score, then smallest read1 / record
// index: the reference's first strict max in index order) and marks the duplicates.  A window
// larger than the tile's table (a pile of reads at one position) sends the whole stage to the
// sort-based kernels above.
constexpr uint32_t kWinTile = 512;   // items per tile
// window items per tile, powers of two (a window of m items uses the smallest power of two >= 2m
// table slots).  LDS: fragments 16 B x 2 cap = 32 KiB (4 blocks per CU), pairs 42 B x cap = 42 KiB;
// C2 windows hold ~560 items.
constexpr uint32_t kFragCap = 1024;
constexpr uint32_t kPairCap = 1024;
static_assert((kFragCap & (kFragCap - 1)) == 0 && (kPairCap & (kPairCap - 1)) == 0, "caps must be powers of two");

__device__ __forceinline__ int64_t win_anchor(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ ax, uint64_t i) {
    return skeys ? anchor_of_key(skeys[i]) : ax[i];
}
// first i in [lo, hi) with anchor(i) >= v (hi if none)
__device__ uint64_t win_lower_bound(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ ax, uint64_t lo,
                                    uint64_t hi, int64_t v) {
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (win_anchor(skeys, ax, mid) < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
struct WinTile {
    int64_t lo, hi;  // owned group coordinates [lo, hi)
    bool first, last;
};
__device__ __forceinline__ WinTile win_tile(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ ax, uint64_t n,
                                            uint64_t t) {
    WinTile w;
    const uint64_t b0 = t * kWinTile, b1 = b0 + kWinTile;
    w.first = t == 0;
    w.last = b1 >= n;
    w.lo = w.first ? INT64_MIN : win_anchor(skeys, ax, b0);
    w.hi = w.last ? INT64_MAX : win_anchor(skeys, ax, b1);
    return w;
}
// one thread per tile: its window [s, e) of items (empty when it owns nothing); *ovf when a window
// exceeds cap
// amax: no item's group coordinate reaches it, and items from the first anchor >= amax on (the
// unmapped tail of the sorted records) never join a window.
__global__ __launch_bounds__(kT) void k_win_bounds(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ ax, uint64_t n,
                                                    uint32_t ntiles, uint32_t cap, const unsigned long long *__restrict__ dev,
                                                    int64_t amax, uint2 *__restrict__ bounds, uint32_t *__restrict__ ovl,
                                                    unsigned int *__restrict__ novf, unsigned long long *__restrict__ ovf_items) {
    const uint32_t t = blockIdx.x * kT + threadIdx.x;
    uint64_t s = 0, e = 0;
    if (t < ntiles) {
        const int64_t D1 = max((int64_t)dev[0] - kDevBias, (int64_t)0), D2 = max((int64_t)dev[1] - kDevBias, (int64_t)0);
        const WinTile w = win_tile(skeys, ax, n, t);
        const uint64_t b0 = (uint64_t)t * kWinTile;
        if ((w.first || w.last || w.lo < w.hi) && w.lo < amax) {
            s = w.first ? 0 : win_lower_bound(skeys, ax, 0, b0 + 1, w.lo - D2);
            e = win_lower_bound(skeys, ax, b0, n, w.last ? amax : min(w.hi + D1, amax));
        }
        bounds[t] = make_uint2((uint32_t)s, (uint32_t)e);
    }
    // tiles whose window exceeds cap (a pile of reads at one position): listed for the sort path
    const bool over = e - s > cap;
    const uint32_t slot = oge_wave_append(over, novf);
    if (over) {
        ovl[slot] = t;
        atomicAdd(ovf_items, (unsigned long long)(e - s));
    }
}

// items owned by the overflowing tiles ovl[] -> (key, value) lists for the sort-based stages
// (fragments: fk / fv; pairs: hk / pair index).  One block per listed tile.
template <bool PAIRS>
__global__ __launch_bounds__(kT) void k_win_collect(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                                     const uint64_t *__restrict__ hi, const uint64_t *__restrict__ lo,
                                                     const uint64_t *__restrict__ skeys, const int64_t *__restrict__ ax,
                                                     uint64_t n, KeyLayout L, const uint2 *__restrict__ bounds,
                                                     const uint32_t *__restrict__ ovl, uint64_t *__restrict__ ok,
                                                     uint32_t *__restrict__ ov, unsigned int *__restrict__ cnt) {
    const uint32_t t = ovl[blockIdx.x];
    const uint2 b = bounds[t];
    const WinTile w = win_tile(skeys, ax, n, t);
    const uint64_t smask = (1ull << L.sb) - 1;
    for (uint64_t base = b.x; base < b.y; base += kT) {  // uniform trip count: oge_wave_append is convergent
        const uint64_t i = base + threadIdx.x;
        bool own = false;
        if (i < b.y) {
            if (PAIRS) {
                const uint64_t h = hi[i];
                const int64_t c = win_x((uint32_t)((h >> 32) & smask), (int64_t)(int32_t)((uint32_t)h ^ 0x80000000u) + 1);
                own = !(lo[i] >> 63) && c >= w.lo && c < w.hi;
            } else {
                const uint64_t k = keys[i];
                const int64_t c = win_x((uint32_t)((k >> 33) & smask), (int64_t)(int32_t)((uint32_t)(k >> 1) ^ 0x80000000u) + 1);
                own = !(k & (1ull << 46)) && c >= w.lo && c < w.hi;
            }
        }
        const uint32_t slot = oge_wave_append(own, cnt);
        if (own) {
            ok[slot] = keys[i];
            ov[slot] = PAIRS ? (uint32_t)i : vals[i];
        }
    }
}

__device__ __forceinline__ uint32_t win_hash(uint64_t k) { return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 32); }
__device__ __forceinline__ uint32_t win_slots(uint32_t m) {  // power of two >= 2m, >= 64
    uint32_t h = 64;
    while (h < 2 * m) h <<= 1;
    return h;
}

// fragments: items = records (fk / fv from k_cand_frag), anchors = the sorted coordinate keys.
// Table slot: group key (47 bits; bit 63 = the group holds a paired end) + packed best of the
// unpaired ends ((score + 2^15) << 32 | ~record index).
__global__ __launch_bounds__(kT) void k_frag_win(const uint64_t *__restrict__ fk, const uint32_t *__restrict__ fv,
                                                  const uint64_t *__restrict__ skeys, uint64_t n, KeyLayout L,
                                                  const uint2 *__restrict__ bounds, uint32_t cap, uint8_t *__restrict__ dup) {
    __shared__ unsigned long long skey[2 * kFragCap], sbest[2 * kFragCap];
    const uint2 b = bounds[blockIdx.x];
    if (b.x >= b.y || b.y - b.x > cap) return;  // owns nothing / overflow (cap <= kFragCap): k_win_collect's list
    const WinTile w = win_tile(skeys, nullptr, n, blockIdx.x);
    const uint32_t H = win_slots(b.y - b.x);
    constexpr unsigned long long kEmpty = ~0ull, kPaired = 1ull << 63;
    const uint64_t gmask = (1ull << 47) - 1, smask = (1ull << L.sb) - 1;
    for (uint32_t j = threadIdx.x; j < H; j += kT) { skey[j] = kEmpty; sbest[j] = 0; }
    __syncthreads();
    for (uint32_t i = b.x + threadIdx.x; i < b.y; i += kT) {
        const uint64_t k = fk[i];
        if (k & (1ull << 46)) continue;  // not a fragment
        const int64_t c = win_x((uint32_t)((k >> 33) & smask), (int64_t)(int32_t)((uint32_t)(k >> 1) ^ 0x80000000u) + 1);
        if (c < w.lo || c >= w.hi) continue;
        const uint64_t g = k & gmask;
        uint32_t h = win_hash(g) & (H - 1);
        for (;;) {
            const unsigned long long cur = atomicCAS(&skey[h], kEmpty, (unsigned long long)g);
            if (cur == kEmpty || (cur & ~kPaired) == g) break;
            h = (h + 1) & (H - 1);
        }
        if (k >> 63) atomicOr(&skey[h], kPaired);
        else atomicMax(&sbest[h], ((unsigned long long)(((k >> 47) & 0xFFFF) ^ 0x8000) << 32) | (0xFFFFFFFFu - fv[i]));
    }
    __syncthreads();
    for (uint32_t i = b.x + threadIdx.x; i < b.y; i += kT) {
        const uint64_t k = fk[i];
        if (k & ((1ull << 46) | (1ull << 63))) continue;  // not a fragment / a paired end: never marked here
        const int64_t c = win_x((uint32_t)((k >> 33) & smask), (int64_t)(int32_t)((uint32_t)(k >> 1) ^ 0x80000000u) + 1);
        if (c < w.lo || c >= w.hi) continue;
        const uint64_t g = k & gmask;
        uint32_t h = win_hash(g) & (H - 1);
        while ((skey[h] & ~kPaired) != g) h = (h + 1) & (H - 1);
        const uint32_t v = fv[i];
        const unsigned long long mine = ((unsigned long long)(((k >> 47) & 0xFFFF) ^ 0x8000) << 32) | (0xFFFFFFFFu - v);
        if ((skey[h] & kPaired) || sbest[h] != mine) dup[v] = 1;
    }
}

// pairs: items = pair ReadEnds in first-record order (k_pair_build), anchors pax.  The window's
// owned keys are staged in LDS; a slot holds the window index of its group's first inserted pair
// and the packed best ((score + 2^15) << 32 | ~read1 index).
__global__ __launch_bounds__(kT) void k_pair_win(const uint64_t *__restrict__ hi, const uint64_t *__restrict__ lo,
                                                  const uint2 *__restrict__ idx, const int64_t *__restrict__ pax, uint64_t np,
                                                  KeyLayout L, const uint2 *__restrict__ bounds, uint32_t cap,
                                                  uint8_t *__restrict__ dup) {
    __shared__ unsigned long long ikh[kPairCap], ikl[kPairCap], sbest[2 * kPairCap];
    __shared__ uint32_t srep[2 * kPairCap];
    __shared__ uint16_t islot[kPairCap];
    const uint2 b = bounds[blockIdx.x];
    if (b.x >= b.y || b.y - b.x > cap) return;  // owns nothing / overflow (cap <= kPairCap): k_win_collect's list
    const WinTile w = win_tile(nullptr, pax, np, blockIdx.x);
    const uint32_t m = b.y - b.x, H = win_slots(m);
    const uint64_t kmask = (1ull << 48) - 1, smask = (1ull << L.sb) - 1;
    constexpr unsigned long long kNone = ~0ull;
    for (uint32_t j = threadIdx.x; j < H; j += kT) { srep[j] = 0xFFFFFFFFu; sbest[j] = 0; }
    for (uint32_t x = threadIdx.x; x < m; x += kT) {
        const uint64_t h = hi[b.x + x], l = lo[b.x + x];
        const int64_t c = win_x((uint32_t)((h >> 32) & smask), (int64_t)(int32_t)((uint32_t)h ^ 0x80000000u) + 1);
        const bool own = !(l >> 63) && c >= w.lo && c < w.hi;  // bit 63 of lo: unconfirmed, not a pair
        ikh[x] = h & kmask;
        ikl[x] = own ? l : kNone;
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < m; x += kT) {
        const unsigned long long kl = ikl[x];
        if (kl == kNone) continue;
        const unsigned long long kh = ikh[x];
        uint32_t h = win_hash(kh ^ (kl * 0xff51afd7ed558ccdull)) & (H - 1);
        for (;;) {
            const uint32_t cur = atomicCAS(&srep[h], 0xFFFFFFFFu, x);
            if (cur == 0xFFFFFFFFu || (ikh[cur] == kh && ikl[cur] == kl)) break;
            h = (h + 1) & (H - 1);
        }
        islot[x] = (uint16_t)h;
        atomicMax(&sbest[h], ((unsigned long long)((hi[b.x + x] >> 48) ^ 0x8000) << 32) | (0xFFFFFFFFu - idx[b.x + x].x));
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < m; x += kT) {
        if (ikl[x] == kNone) continue;
        const uint2 ii = idx[b.x + x];
        const unsigned long long mine = ((unsigned long long)((hi[b.x + x] >> 48) ^ 0x8000) << 32) | (0xFFFFFFFFu - ii.x);
        if (sbest[islot[x]] != mine) {
            dup[ii.x] = 1;
            dup[ii.y] = 1;
        }
    }
}

__global__ __launch_bounds__(kT) void k_any(const uint8_t *__restrict__ dup, uint64_t n, unsigned int *__restrict__ any) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (__ballot(i < n && dup[i]) && (threadIdx.x & 63) == 0) atomicOr(any, 1u);
}

__global__ __launch_bounds__(kT) void k_apply(uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                                               const RecMeta *__restrict__ meta, uint8_t *__restrict__ dup, int apply,
                                               int compat, const unsigned int *__restrict__ any,
                                               unsigned long long *__restrict__ ndup) {
    __shared__ uint32_t wsum[kT / 64];
    uint32_t mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kT) {
        const uint64_t m = meta[i].m;
        const uint8_t d = compat ? (uint8_t)(i == 0 && *any) : dup[i];
        const uint8_t hi = (uint8_t)(m >> 40);
        uint8_t nh = hi;
        if (!(m & OGE_M_PRIMARY)) {
            dup[i] = 2;
        } else {
            dup[i] = d;
            mine += d;
            // FLAG bit 0x400 is bit 2 of the flag's high byte (record byte 19)
            nh = d ? (uint8_t)(hi | 0x04) : (uint8_t)(hi & ~0x04);
            if (apply && nh != hi) recs[off[i] + OGE_OFF_FLAG + 1] = nh;
        }
    }
    // one atomic per block: per-thread counts -> wave sums -> block sum
    const uint32_t ws = oge_wave_sum(mine);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = ws;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int q = 0; q < kT / 64; ++q) t += wsum[q];
        if (t) atomicAdd(ndup, (unsigned long long)t);
    }
}

// k_apply for the fused pipeline from the 8-byte desc0 words (k_cand_frag): dup[] as k_apply leaves
// it (apply = 0) and the gather descriptor with the final FLAG high byte.
__global__ __launch_bounds__(kT) void k_apply_desc(const uint64_t *__restrict__ desc0, uint64_t n, uint8_t *__restrict__ dup,
                                                    int compat, const unsigned int *__restrict__ any,
                                                    unsigned long long *__restrict__ ndup, uint64_t *__restrict__ desc) {
    __shared__ uint32_t wsum[kT / 64];
    uint32_t mine = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kT) {
        const uint64_t D = desc0[i];
        const uint8_t d = compat ? (uint8_t)(i == 0 && *any) : dup[i];
        const uint8_t hi = (uint8_t)(D >> 56);
        uint8_t nh = hi;
        if (!((D >> 39) & 1)) {
            dup[i] = 2;
        } else {
            dup[i] = d;
            mine += d;
            nh = d ? (uint8_t)(hi | 0x04) : (uint8_t)(hi & ~0x04);
        }
        desc[i] = (D & ((1ull << 39) - 1)) | (D & (0xffffull << 40)) | ((uint64_t)nh << 56);
    }
    const uint32_t ws = oge_wave_sum(mine);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = ws;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int q = 0; q < kT / 64; ++q) t += wsum[q];
        if (t) atomicAdd(ndup, (unsigned long long)t);
    }
}

// ---- windowed mate join (records in coordinate order, one GPU) ----
// Mates of a proper pair sit within ~ insert size / read spacing records of each other in coordinate
// order, so most of the ReadEndsMap's pairs are found in a window, without the global hash sort:
//   k_mate_win    tile of kMjT records + kMjW on each side in an LDS table of candidate fingerprints
//                 (count, first and last window slot): a tile record whose fingerprint occurs exactly
//                 twice in its window gets the other occurrence as partner; a partner in the same tile
//                 decides at once (window pair owned by the smaller index, or both leftovers)
//   k_mate_agree  a partner in another tile: i and j = partner[i] agree (partner[j] == i, equal hash bits)
//                 or i is a leftover.  Every leftover's hash bits go into a global set (a bitmap filter in
//                 front of an open-addressing table)
//   k_mate_check  a window pair whose hash is in that set gives both ends to the leftovers: its key has
//                 other occurrences (first-seen / second-seen pairing must see them all)
// The leftovers take the sort-based join; every hash bit pattern then occurs exactly twice among the
// window pairs' records (the same provisional pair the sort path forms from a run of two), or its
// records all went the sort path.  A window pair whose names differ (a 48-bit collision) makes the caller
// redo the join by sort (k_pair_build counts them).
constexpr uint32_t kMjT = 1024, kMjW = 512, kMjSlots = 4096;
static_assert(kMjT + 2 * kMjW <= kMjSlots / 2, "window table at most half full");
constexpr uint32_t kNone = 0xffffffffu, kSortPair = 0x80000000u;

__device__ __forceinline__ bool is_cand(const uint32_t *__restrict__ cflag, uint64_t i) { return cflag[i] != 0; }
__device__ __forceinline__ uint32_t mj_fp(uint64_t h) {
    const uint32_t x = (uint32_t)h ^ (uint32_t)(h >> 32) * 0x9E3779B1u;
    return x ? x : 1u;
}

__device__ __forceinline__ uint32_t mj_slot(uint64_t key, uint32_t mask) { return (uint32_t)(mix64(key) & mask); }
__device__ __forceinline__ uint32_t mj_bit(uint64_t key, uint32_t bmask) { return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32) & bmask; }
constexpr int kMjProbes = 64;
constexpr uint32_t kPending = 2;  // k_mate_win's decision: the partner lies in another tile, k_mate_agree decides
constexpr uint32_t kPendBit = 0x80000000u;  // partner[i] of a pending record (record indices < 2^31)

// Leftovers (records the sort-based join pairs) appended to lk as their candidate keys (hash bits << ib |
// index).  One counter would serialise the appends at its L2 channel (~88 atomics/us: at 300M reads ~2M wave
// appends took 20 ms), so the list is striped: record r goes to stripe (r >> 10) % kMjStripes, each stripe
// with its own counter (128 bytes apart) and a region of lcap slots -- every record is appended at most once
// and a stripe's records number at most lcap, so no region overflows.  k_left_pack then concatenates them.
constexpr uint32_t kMjStripes = 64, kMjCntStride = 32;
__device__ __forceinline__ uint32_t mj_stripe(uint64_t r) { return (uint32_t)(r >> 10) & (kMjStripes - 1); }
// the lanes of a wave hold 64 consecutive records of one 1024-record tile: one stripe, one atomic per wave
__device__ __forceinline__ void mj_left(bool pred, uint64_t key, uint64_t rec, uint64_t *__restrict__ lk,
                                        unsigned int *__restrict__ lcnt, uint32_t lcap) {
    const uint64_t m = __ballot(pred);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)(__ffsll((long long)m) - 1);
    const uint32_t st = mj_stripe(rec);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lcnt + st * kMjCntStride, (unsigned int)__popcll(m));
    base = __shfl(base, (int)leader, 64) + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    if (pred) lk[(uint64_t)st * lcap + base] = key;
}
// one record of any tile (the partner end of a conflicting window pair: rare)
__device__ __forceinline__ void mj_left1(uint64_t key, uint64_t rec, uint64_t *__restrict__ lk, unsigned int *__restrict__ lcnt,
                                         uint32_t lcap) {
    const uint32_t st = mj_stripe(rec);
    lk[(uint64_t)st * lcap + atomicAdd(lcnt + st * kMjCntStride, 1u)] = key;
}

// a leftover's hash bits into the conflict set (bitmap filter + open-addressing table)
__device__ __forceinline__ void mj_conflict(uint64_t h, unsigned long long *__restrict__ tab, uint32_t mask,
                                            uint32_t *__restrict__ bits, uint32_t bmask, unsigned int *__restrict__ ovf) {
    const unsigned long long key = h + 1;
    const uint32_t b = mj_bit(key, bmask);
    atomicOr(&bits[b >> 5], 1u << (b & 31));
    uint32_t s = mj_slot(key, mask);
    for (int p = 0; p < kMjProbes; ++p) {
        const unsigned long long o = atomicCAS(&tab[s], 0ull, key);
        if (o == 0ull || o == key) return;
        s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
}

// Per tile: the window's fingerprint table, then every tile record's decision.  A partner inside the tile
// saw the same table (agreement is given; the full hash bits are compared from the staged window): a window
// pair (mate[] of the smaller index) or two leftovers.  A partner in another tile: partner[i] | kPendBit.
__global__ __launch_bounds__(kMjT) void k_mate_win(const uint32_t *__restrict__ cflag, const uint64_t *__restrict__ cval, uint64_t n,
                                                   uint32_t ib, uint32_t *__restrict__ partner, uint32_t *__restrict__ mate,
                                                   unsigned long long *__restrict__ tab, uint32_t mask,
                                                   uint32_t *__restrict__ bits, uint32_t bmask, unsigned int *__restrict__ ovf,
                                                   uint64_t *__restrict__ lk, unsigned int *__restrict__ lcnt, uint32_t lcap) {
    __shared__ uint32_t key[kMjSlots], lo[kMjSlots], hi[kMjSlots], cnt[kMjSlots];
    __shared__ uint64_t hv[kMjT + 2 * kMjW];  // the window's hash bits (0: not a candidate)
    const uint32_t t = threadIdx.x;
    for (uint32_t s = t; s < kMjSlots; s += kMjT) key[s] = 0, lo[s] = kNone, hi[s] = 0, cnt[s] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kMjT, w0 = t0 - (int64_t)kMjW;
    for (uint32_t w = t; w < kMjT + 2 * kMjW; w += kMjT) {
        const int64_t i = w0 + (int64_t)w;
        hv[w] = 0;
        if (i < 0 || (uint64_t)i >= n || !is_cand(cflag, (uint64_t)i)) continue;
        const uint64_t h = cval[i] >> ib;
        hv[w] = h + 1;
        const uint32_t f = mj_fp(h);
        uint32_t s = (f * 2654435761u) >> 20;  // 12 bits: kMjSlots
        for (;;) {
            const uint32_t o = atomicCAS(&key[s], 0u, f);
            if (o == 0u || o == f) break;
            s = (s + 1) & (kMjSlots - 1);
        }
        atomicAdd(&cnt[s], 1u);
        atomicMin(&lo[s], w);
        atomicMax(&hi[s], w);
    }
    __syncthreads();
    const uint64_t i = (uint64_t)t0 + t;
    if (i >= n) return;
    const uint32_t w = t + kMjW;
    uint32_t r = kNone, m = kNone, lf = 0;
    uint64_t h = 0;
    if (hv[w]) {
        h = hv[w] - 1;
        const uint32_t f = mj_fp(h);
        uint32_t s = (f * 2654435761u) >> 20;
        while (key[s] != f) s = (s + 1) & (kMjSlots - 1);
        if (cnt[s] == 2) {
            const uint32_t pw = lo[s] == w ? hi[s] : lo[s];
            r = (uint32_t)(w0 + (int64_t)pw);
            if (pw >= kMjW && pw < kMjW + kMjT) {  // the partner is a record of this tile
                if (hv[pw] == hv[w]) {
                    if ((uint64_t)r > i) m = r;
                } else {
                    lf = 1;  // a fingerprint collision: two different keys
                }
            } else {
                lf = kPending;
            }
        } else {
            lf = 1;
        }
        if (lf == 1) {
            r = kNone;
            mj_conflict(h, tab, mask, bits, bmask, ovf);
        }
    }
    mj_left(lf == 1, (h << ib) | i, i, lk, lcnt, lcap);
    partner[i] = lf == kPending ? r | kPendBit : r;  // (kNone: no partner)
    mate[i] = m;
}

// the pending records (a partner in another tile): i and j = partner[i] agree (partner[j] == i, equal hash
// bits) -- a window pair owned by the smaller index -- or i is a leftover
__global__ __launch_bounds__(kT) void k_mate_agree(const uint64_t *__restrict__ cval, uint64_t n, uint32_t ib,
                                                   const uint32_t *__restrict__ partner, uint32_t *__restrict__ mate,
                                                   unsigned long long *__restrict__ tab, uint32_t mask,
                                                   uint32_t *__restrict__ bits, uint32_t bmask, unsigned int *__restrict__ ovf,
                                                   uint64_t *__restrict__ lk, unsigned int *__restrict__ lcnt, uint32_t lcap) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const uint32_t pi = partner[i];
    if (pi == kNone || !(pi & kPendBit)) return;
    const uint32_t j = pi & ~kPendBit;
    const uint64_t ci = cval[i], h = ci >> ib;
    const bool agree = partner[j] == ((uint32_t)i | kPendBit) && (cval[j] >> ib) == h;
    if (agree) {
        if (i < j) mate[i] = j;
    } else {
        mj_conflict(h, tab, mask, bits, bmask, ovf);
    }
    mj_left(!agree, ci, i, lk, lcnt, lcap);
}

// also counts the pairs each 256-record block owns (bcnt[blockIdx]: mate[i] != kNone afterwards; k_mate_scatter
// adds the sort path's) for k_mate_compact (r06: per-record owner flags and their full scan before)
__global__ __launch_bounds__(kT) void k_mate_check(const uint64_t *__restrict__ cval, uint64_t n, uint32_t ib,
                                                   const unsigned long long *__restrict__ tab, uint32_t mask,
                                                   const uint32_t *__restrict__ bits, uint32_t bmask, uint32_t *__restrict__ mate,
                                                   uint32_t *__restrict__ bcnt, uint64_t *__restrict__ lk,
                                                   unsigned int *__restrict__ lcnt, uint32_t lcap) {
    __shared__ uint32_t ws[kT / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t m = i < n ? mate[i] : kNone;
    const uint64_t cv = i < n ? cval[i] : 0;  // loaded beside mate[i], not after it (the bitmap read waits on both)
    uint32_t own = 0;
    bool hit = false;
    uint64_t h = 0;
    if (m != kNone) {
        own = 1;
        h = cv >> ib;
        const unsigned long long key = h + 1;
        const uint32_t b = mj_bit(key, bmask);
        uint32_t s = mj_slot(key, mask);
        hit = ((bits[b >> 5] >> (b & 31)) & 1u) != 0;  // a probe run longer than the insert bound: only after an overflow
        for (int p = 0; hit && p < kMjProbes; ++p) {
            const unsigned long long o = tab[s];
            if (o == key) break;
            if (o == 0ull) { hit = false; break; }
            s = (s + 1) & mask;
        }
        if (hit) {  // both ends to the leftovers (a window pair's ends have equal hash bits)
            mate[i] = kNone;
            own = 0;
        }
    }
    mj_left(hit, (h << ib) | i, i, lk, lcnt, lcap);
    if (hit) mj_left1((h << ib) | m, m, lk, lcnt, lcap);
    const uint32_t wsum = oge_wave_sum(own);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = wsum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int q = 0; q < kT / 64; ++q) t += ws[q];
        bcnt[blockIdx.x] = t;
    }
}

// the sort path's pairs of leftovers (a << 32 | b, a < b) -> mate[a] = b | kSortPair, counted in a's block
__global__ __launch_bounds__(kT) void k_mate_scatter(const uint64_t *__restrict__ pairs, uint32_t np, uint32_t *__restrict__ mate,
                                                     uint32_t *__restrict__ bcnt) {
    const uint32_t p = blockIdx.x * kT + threadIdx.x;
    if (p >= np) return;
    uint32_t a = (uint32_t)(pairs[p] >> 32), b = (uint32_t)pairs[p];
    if (a > b) { const uint32_t x = a; a = b; b = x; }
    mate[a] = b | kSortPair;
    atomicAdd(&bcnt[a / kT], 1u);
}

// pairs in first-record order: block b's owners (mate[i] != kNone) take slots boff[b], ... in record order
// (ranks by ballot inside each wave, wave offsets through LDS), and each owner builds its pair's ReadEnds
// there at once (r06: the pairs were first written out as words, then read back by k_pair_build)
__global__ __launch_bounds__(kT) void k_mate_compact(const uint32_t *__restrict__ boff, const uint32_t *__restrict__ mate, uint64_t n,
                                                     const uint8_t *__restrict__ recs, const RecMeta *__restrict__ meta, KeyLayout L,
                                                     uint64_t *__restrict__ hi, uint64_t *__restrict__ lo, uint2 *__restrict__ idx,
                                                     const uint64_t *__restrict__ skeys, int64_t *__restrict__ pax,
                                                     unsigned long long *__restrict__ dev, unsigned int *__restrict__ win_bad) {
    __shared__ uint32_t ws[kT / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    const uint32_t m = i < n ? mate[i] : kNone, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool own = m != kNone;
    const uint64_t b = __ballot(own);
    if (lane == 0) ws[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t r = boff[blockIdx.x] + (uint32_t)__popcll(b & ((1ull << lane) - 1));
    for (uint32_t q = 0; q < w; ++q) r += ws[q];
    bool has = false;
    int64_t ax = 0, cx = 0;
    if (own) pair_entry(r, (uint32_t)i, m, recs, meta, L, hi, lo, idx, nullptr, nullptr, skeys, pax, win_bad, has, ax, cx);
    if (skeys) win_dev_update(has, ax, cx, dev);
}

// the stripes of lk concatenated into out (stripe s from the sum of the counts before it): blockIdx.y = stripe
__global__ __launch_bounds__(kT) void k_left_pack(const uint64_t *__restrict__ lk, const unsigned int *__restrict__ lcnt, uint32_t lcap,
                                                  uint64_t *__restrict__ out) {
    const uint32_t st = blockIdx.y, c = lcnt[st * kMjCntStride];
    uint32_t off = 0;
    for (uint32_t q = 0; q < st; ++q) off += lcnt[q * kMjCntStride];
    for (uint32_t j = blockIdx.x * kT + threadIdx.x; j < c; j += gridDim.x * kT) out[off + j] = lk[(uint64_t)st * lcap + j];
}

uint32_t bits_for(uint64_t v) {  // bits to hold values 0..v
    uint32_t b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b ? b : 1;
}

// high-32-bit mask covering record indices 0..n-1 (only the bits that can vary)
uint64_t bits_mask_hi32(uint64_t n) {
    const uint32_t b = bits_for(n ? n - 1 : 0);
    return (b >= 32 ? 0xFFFFFFFFull : ((1ull << b) - 1)) << 32;
}

}  // namespace

// Allocate the per-record ReadEnds summaries (`name` selects the buffer) and upload the RG table.
int oge_markdup_prepare(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, const char *name, RecMeta **meta,
                        OgeRgTable *rg) {
    if (!opts) return oge_fail(ctx, OGE_ERR_ARG, "markdup: opts is NULL");
    if (opts->split_chains < 0 || opts->split_chains > 4096)
        return oge_fail(ctx, OGE_ERR_ARG, "markdup: split_chains out of [0, 4096]");
    if (opts->split_chains > 1 && opts->compat_nonverbose_index)
        return oge_fail(ctx, OGE_ERR_ARG, "markdup: split_chains > 1 with compat_nonverbose_index is not supported");
    if (n > 0xFFFFFFFEull) return oge_fail(ctx, OGE_ERR_LIMIT, "markdup: more than 2^32-2 records");
    if (opts->n_rg < 0 || (opts->n_rg && (!opts->rg_ids || !opts->rg_lib)))
        return oge_fail(ctx, OGE_ERR_ARG, "markdup: bad read-group table");
    if (opts->n_rg > OGE_MAX_RG) return oge_fail(ctx, OGE_ERR_LIMIT, "markdup: more than 32767 read groups");
    *meta = (RecMeta *)(strcmp(name, "md_meta_in") ? ctx->ws(name, (n + 1) * sizeof(RecMeta))
                                                   : ctx->scratch(name, (n + 1) * sizeof(RecMeta)));
    std::vector<uint32_t> offs(opts->n_rg + 1, 0);
    const char *p = opts->rg_ids;
    for (int32_t g = 0; g < opts->n_rg; ++g) {
        size_t L = strnlen(p, opts->rg_ids_bytes - (size_t)(p - opts->rg_ids));
        offs[g + 1] = offs[g] + (uint32_t)L + 1;
        p += L + 1;
    }
    std::vector<uint8_t> w16((size_t)opts->n_rg * 16, 0);  // idw: ids of <= 15 bytes, zero-padded
    for (int32_t g = 0; g < opts->n_rg; ++g)
        if (offs[g + 1] - offs[g] - 1 <= 15) memcpy(&w16[(size_t)g * 16], opts->rg_ids + offs[g], offs[g + 1] - offs[g] - 1);
    uint8_t *ids = (uint8_t *)ctx->ws("md_rgids", offs.back() + 16);
    uint4 *idw = (uint4 *)ctx->ws("md_rgidw", w16.size() + 16);
    uint32_t *doff = (uint32_t *)ctx->ws("md_rgoff", offs.size() * 4);
    int16_t *lib = (int16_t *)ctx->ws("md_rglib", (size_t)(opts->n_rg + 1) * 2);
    if (!*meta || !ids || !idw || !doff || !lib) return OGE_ERR_HIP;
    if (offs.back()) OGE_HIP_TRY(ctx, hipMemcpyAsync(ids, opts->rg_ids, offs.back(), hipMemcpyHostToDevice, ctx->stream));
    if (!w16.empty()) OGE_HIP_TRY(ctx, hipMemcpyAsync(idw, w16.data(), w16.size(), hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(doff, offs.data(), offs.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    if (opts->n_rg) OGE_HIP_TRY(ctx, hipMemcpyAsync(lib, opts->rg_lib, (size_t)opts->n_rg * 2, hipMemcpyHostToDevice, ctx->stream));
    rg->ids = ids;
    rg->idw = idw;
    rg->off = doff;
    rg->lib = lib;
    rg->n_rg = opts->n_rg;
    rg->unknown_lib = opts->unknown_lib;
    rg->split_k = opts->split_chains;
    // the host copies above read pageable memory; make sure they are done before returning
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

namespace {
__global__ __launch_bounds__(kT) void k_pair_rehash(const uint64_t *__restrict__ hi, const uint64_t *__restrict__ lo, uint32_t np,
                                                     uint64_t *__restrict__ hk, uint32_t *__restrict__ val) {
    const uint32_t p = blockIdx.x * kT + threadIdx.x;
    if (p >= np) return;
    hk[p] = mix64(mix64(hi[p] & ((1ull << 48) - 1)) ^ lo[p]);
    val[p] = p;
}
}  // namespace

int oge_md_pairs_rehash(oge_ctx *ctx, OgeMdPairs *P) {
    if (!P->np) return OGE_OK;
    P->hk = (uint64_t *)ctx->scratch("md_hi2", (uint64_t)P->np * 8);
    P->val = (uint32_t *)ctx->scratch("md_pv", (uint64_t)P->np * 4);
    if (!P->hk || !P->val) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_pair_rehash, dim3(oge_ceil_div(P->np, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)P->hi,
                       (const uint64_t *)P->lo, P->np, P->hk, P->val);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

// ------------------------------------------------------------------------------------ stages
// oge_markdup_finish is the sequence cand_frag -> join_build -> pair_groups -> frag_groups -> apply;
// the multi-GPU path (dist.hip) runs the same stages on ReadEnds exchanged between ranks.

static int md_layout(oge_ctx *ctx, const oge_markdup_opts *opts, KeyLayout *L) {
    int16_t maxlib = opts->unknown_lib;
    for (int32_t g = 0; g < opts->n_rg; ++g) maxlib = std::max(maxlib, opts->rg_lib[g]);
    if (opts->unknown_lib < 0) return oge_fail(ctx, OGE_ERR_ARG, "markdup: negative library id");
    for (int32_t g = 0; g < opts->n_rg; ++g)
        if (opts->rg_lib[g] < 0) return oge_fail(ctx, OGE_ERR_ARG, "markdup: negative library id");
    *L = KeyLayout{bits_for((uint64_t)std::max(opts->n_ref, 1)), bits_for((uint64_t)maxlib), opts->split_chains};
    if (L->sb + L->lb + 34 > 47 || L->sb + L->lb > 16)
        return oge_fail(ctx, OGE_ERR_LIMIT, "markdup: too many references x libraries for the packed group key");
    return OGE_OK;
}

static CandKey md_candkey(const oge_markdup_opts *opts, uint64_t n) {
    CandKey ckl;
    ckl.ib = bits_for(n ? n - 1 : 0);
    ckl.hb = std::min<uint32_t>(48, 64 - ckl.ib);
    ckl.split_k = opts->split_chains;
    if (opts->debug_hash_bits > 0 && (uint32_t)opts->debug_hash_bits < ckl.hb) ckl.hb = (uint32_t)opts->debug_hash_bits;
    return ckl;
}

static bool mate_win_enabled() {
    const char *e = getenv("OGE_MD_MATEWIN");  // "0": the sort-based join only (A/B, tests); read per call
    return !(e && e[0] == '0');
}
// the windowed mate join applies: records in coordinate order (skeys) on one GPU, the default key hash, one chain
static bool mate_window_ok(const oge_markdup_opts *opts, uint64_t n, const uint64_t *skeys) {
    return skeys && n && n < (1ull << 31) && opts->split_chains <= 1 && opts->debug_hash_bits <= 0 && mate_win_enabled();
}

// gin / perm (the fused gather): meta[i] = gin[perm[i]] is written here too, by k_meta_gather_cf
// the products' buffers (and, with want_dev, the zeroed deviation slots); *L / *ck the layouts they use
static int cand_frag_alloc(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, bool want_desc, bool want_dev, OgeMdFrags *f,
                           KeyLayout *L, CandKey *ck, uint64_t *desc0_buf = nullptr) {
    int rc = md_layout(ctx, opts, L);
    if (rc) return rc;
    *f = OgeMdFrags{};
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    if (!cnt) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
    f->cpos = (uint32_t *)ctx->scratch("md_cpos", (n + 1) * 4);
    f->fk = (uint64_t *)ctx->scratch("md_fk", (n + 1) * 8);
    f->fv = (uint32_t *)ctx->scratch("md_fv", (n + 1) * 4);
    f->cval = (uint64_t *)ctx->scratch("md_cval", (n + 1) * 8);
    f->desc0 = !want_desc ? nullptr : desc0_buf ? desc0_buf : (uint64_t *)ctx->scratch("md_desc0", (n + 1) * 8);
    if (!f->cpos || !f->fk || !f->fv || !f->cval || (want_desc && !f->desc0)) return OGE_ERR_HIP;
    *ck = md_candkey(opts, n);
    if (want_dev) {
        // per-block deviation maxima: kDevSlots word pairs for the fragments, as many for the pairs
        f->dev = (unsigned long long *)ctx->ws("md_devslots", 4 * kDevSlots * sizeof(unsigned long long));
        if (!f->dev) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(f->dev, 0, 4 * kDevSlots * sizeof(unsigned long long), ctx->stream));
    }
    return OGE_OK;
}

static int cand_frag_launch(oge_ctx *ctx, const oge_markdup_opts *opts, const RecMeta *meta, uint64_t n, bool want_desc,
                            OgeMdFrags *f, const uint64_t *skeys, const RecMeta *gin, const uint32_t *perm,
                            uint64_t *desc0_buf = nullptr) {
    KeyLayout L;
    CandKey ckl;
    int rc = cand_frag_alloc(ctx, opts, n, want_desc, skeys != nullptr, f, &L, &ckl, desc0_buf);
    if (rc) return rc;
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    f->skeys = skeys;
    if (perm)
        hipLaunchKernelGGL(k_meta_gather_cf, dim3(oge_ceil_div(4 * (n + 1), kT)), dim3(kT), 0, ctx->stream, gin, perm, n,
                           (RecMeta *)meta, L, ckl, f->cpos, f->fk, f->fv, f->cval, f->desc0, cnt + 3, skeys, f->dev);
    else
        hipLaunchKernelGGL(k_cand_frag, dim3(oge_ceil_div(n + 1, kT)), dim3(kT), 0, ctx->stream, meta, n, L, ckl, f->cpos, f->fk,
                           f->fv, f->cval, f->desc0, cnt + 3, skeys, f->dev);
    OGE_LAUNCH_CHECK(ctx);
    f->fused = perm != nullptr;
    return OGE_OK;
}

// after the launch: the candidate scan (unless the windowed join takes the flags) and the overflow word
static int cand_frag_post(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t n, OgeMdFrags *f) {
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    if (!cnt) return OGE_ERR_HIP;
    const uint64_t *skeys = f->skeys;
    int rc;
    uint32_t nc = 0, ovf = 0;
    f->cpos_scanned = !mate_window_ok(opts, n, skeys);  // the windowed join reads the flags as they are
    if (f->cpos_scanned) {
        rc = oge_exclusive_scan_u32(ctx, f->cpos, f->cpos, n + 1);
        if (rc) return rc;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&nc, f->cpos + n, 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&ovf, cnt + 3, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    f->nc = nc;
    f->desc_ovf = ovf != 0;
    return OGE_OK;
}

int oge_md_cand_frag(oge_ctx *ctx, const oge_markdup_opts *opts, const RecMeta *meta, uint64_t n, bool want_desc,
                     OgeMdFrags *f, const uint64_t *skeys) {
    int rc = cand_frag_launch(ctx, opts, meta, n, want_desc, f, skeys, nullptr, nullptr);
    return rc ? rc : cand_frag_post(ctx, opts, n, f);
}

int oge_md_cand_frag_gather(oge_ctx *ctx, const oge_markdup_opts *opts, const RecMeta *in, const uint32_t *perm, uint64_t n,
                            RecMeta *out, bool want_desc, const uint64_t *skeys, OgeMdFrags *f, uint64_t *desc0_buf) {
    return cand_frag_launch(ctx, opts, out, n, want_desc, f, skeys, in, perm, desc0_buf);
}

// The sort-based ReadEndsMap pairing (mark_duplicates.cpp:210-245) of the candidates flagged by cpos
// (exclusive scan of the flags, nc of them) -> pairs a << 32 | b (a first seen), *np of them, in
// candidate-hash order, in ws "md_pairs"; "md_pairs2" is the spare of the same size.
// packed (optional): the nc candidate keys already in an array of at least nc + 1 (in any order; cpos unused):
// sorted on hash AND index bits, which puts each hash run in record order as the stable hash-only sort does
// for keys packed in record order.
static int join_sorted(oge_ctx *ctx, const CandKey &ckl, const uint8_t *recs, const RecMeta *meta, uint64_t n, const uint32_t *cpos,
                       const uint64_t *cval, uint32_t nc, uint64_t **pairs_out, uint64_t **spare_out, uint32_t *np_out,
                       uint64_t *packed = nullptr) {
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    const uint64_t nc1 = (uint64_t)nc + 1;
    uint64_t *ck = packed ? packed : (uint64_t *)ctx->scratch("md_ck", nc1 * 8);
    uint64_t *ck2 = (uint64_t *)ctx->scratch("md_ck2", nc1 * 8);
    uint8_t *used = (uint8_t *)ctx->scratch("md_used", nc1);
    uint32_t *pflag = (uint32_t *)ctx->scratch("md_pflag", nc1 * 4);
    uint64_t *sparse = (uint64_t *)ctx->scratch("md_sparse", nc1 * 8);
    uint64_t *pairs = (uint64_t *)ctx->scratch("md_pairs", (nc1 / 2 + 1) * 8);
    uint64_t *pairs2 = (uint64_t *)ctx->scratch("md_pairs2", (nc1 / 2 + 1) * 8);
    uint32_t *slow = (uint32_t *)ctx->scratch("md_slow", nc1 * 4);
    if (!cnt || !ck || !ck2 || !used || !pflag || !sparse || !pairs || !pairs2 || !slow) return OGE_ERR_HIP;
    if (n && !packed) {
        hipLaunchKernelGGL(k_cand_pack, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, cpos, cval, n, ck);
        OGE_LAUNCH_CHECK(ctx);
    }
    uint64_t *sk;
    const uint64_t smask = ((1ull << ckl.hb) - 1) << ckl.ib | (packed ? ckl.idx_mask() : 0ull);
    int rc = oge_radix_sort_pairs(ctx, ck, nullptr, ck2, nullptr, nc, smask, &sk, nullptr);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt + 2, 0, 4, ctx->stream));
    hipLaunchKernelGGL(k_pair_runs, dim3(oge_ceil_div(nc1, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)sk, (uint64_t)nc, ckl,
                       pflag, sparse, slow, cnt + 2);
    OGE_LAUNCH_CHECK(ctx);
    uint32_t nslow = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&nslow, cnt + 2, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (nslow) {
        OGE_HIP_TRY(ctx, hipMemsetAsync(used, 0, nc1, ctx->stream));
        hipLaunchKernelGGL(k_pair_runs_slow, dim3(oge_ceil_div(nslow, kT)), dim3(kT), 0, ctx->stream, recs, meta,
                           (const uint64_t *)sk, (uint64_t)nc, ckl, (const uint32_t *)slow, nslow, used, pflag, sparse);
        OGE_LAUNCH_CHECK(ctx);
    }
    rc = oge_exclusive_scan_u32(ctx, pflag, pflag, nc1);
    if (rc) return rc;
    uint32_t np = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&np, pflag + nc, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    // flags were overwritten by the scan: compact by comparing neighbouring prefix sums
    hipLaunchKernelGGL(k_pair_compact_scan, dim3(oge_ceil_div(nc1, kT)), dim3(kT), 0, ctx->stream, (const uint32_t *)pflag,
                       (const uint64_t *)sparse, (uint64_t)nc, pairs);
    OGE_LAUNCH_CHECK(ctx);
    *pairs_out = pairs;
    *spare_out = pairs2;
    *np_out = np;
    return OGE_OK;
}

// The pair ReadEnds of np pairs in first-record order (k_pair_build).  win_bad (optional): counts the
// windowed join's pairs whose names differ.
// lazy_hk (the windowed join, whose pair groups are windowed too): hk / val are not written here, only by
// pairs_hk when a fallback path sorts by them.
static int pair_build(oge_ctx *ctx, const KeyLayout &L, const uint8_t *recs, const RecMeta *meta, const OgeMdFrags &f,
                      const uint64_t *spairs, uint32_t np, OgeMdPairs *P, unsigned int *win_bad, bool lazy_hk = false) {
    P->np = np;
    if (!np) return OGE_OK;
    P->hi = (uint64_t *)ctx->scratch("md_hi", (uint64_t)np * 8);
    P->lo = (uint64_t *)ctx->scratch("md_lo", (uint64_t)np * 8);
    P->idx = (uint2 *)ctx->scratch("md_pidx", (uint64_t)np * sizeof(uint2));
    if (!lazy_hk) {
        P->hk = (uint64_t *)ctx->scratch("md_hi2", (uint64_t)np * 8);
        P->val = (uint32_t *)ctx->scratch("md_pv", (uint64_t)np * 4);
        if (!P->hk || !P->val) return OGE_ERR_HIP;
    }
    if (!P->hi || !P->lo || !P->idx) return OGE_ERR_HIP;
    if (f.skeys) {
        P->pax = (int64_t *)ctx->scratch("md_pax", (uint64_t)np * 8);
        P->dev = f.dev + 2 * kDevSlots;
        if (!P->pax) return OGE_ERR_HIP;
        // the pair half of the deviation slots: a redone join starts them again
        OGE_HIP_TRY(ctx, hipMemsetAsync(P->dev, 0, 2 * kDevSlots * sizeof(unsigned long long), ctx->stream));
    }
    if (!spairs) return OGE_OK;  // (the windowed join builds them in k_mate_compact)
    hipLaunchKernelGGL(k_pair_build, dim3(oge_ceil_div(np, kT)), dim3(kT), 0, ctx->stream, spairs, np, recs, meta, L, P->hi, P->lo,
                       P->idx, P->val, P->hk, f.skeys, P->pax, P->dev, win_bad);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

// The windowed join (see k_mate_win) for records in coordinate order; *done = false when it cannot
// decide (the conflict set overflowed, or a window pair's names differ): the caller runs the sort path.
static int join_window(oge_ctx *ctx, const KeyLayout &L, const CandKey &ckl, const uint8_t *recs, const RecMeta *meta, uint64_t n,
                       const OgeMdFrags &f, OgeMdPairs *P, bool *done) {
    *done = false;
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    unsigned int *lcnt = (unsigned int *)ctx->ws("md_lcnt", kMjStripes * kMjCntStride * 4);
    const uint32_t nb = (uint32_t)oge_ceil_div(n, kT);
    uint32_t *partner = (uint32_t *)ctx->scratch("md_mpart", (n + 1) * 4);
    uint32_t *mate = (uint32_t *)ctx->scratch("md_mate", (n + 1) * 4);
    uint32_t *bcnt = (uint32_t *)ctx->scratch("md_bcnt", ((uint64_t)nb + 1) * 4);
    // the leftovers' candidate keys, appended by the three kernels below into kMjStripes regions of lcap
    // slots (the records of a stripe's 1024-record tiles: see mj_left), then packed (r06: flags, a scan over all
    // records and a packing pass before)
    const uint32_t lcap = (uint32_t)(oge_ceil_div(oge_ceil_div(n, 1024), kMjStripes) * 1024ull);
    uint64_t *lk = (uint64_t *)ctx->scratch("md_lk", (uint64_t)kMjStripes * lcap * 8);
    if (!cnt || !lcnt || !partner || !mate || !bcnt || !lk) return OGE_ERR_HIP;
    // the conflict set: a table of >= n/16 slots behind a bitmap of >= n/2 bits, at most 4 MiB so it stays in
    // an XCD's L2 for k_mate_check's random reads (a probe run past kMjProbes means too many leftovers for the
    // window path: the sort path decides)
    uint32_t slots = 1024, nbits = 1u << 15;
    while (slots < n / 16 && slots < (1u << 30)) slots <<= 1;
    while (nbits < n / 2 && nbits < (1u << 25)) nbits <<= 1;
    unsigned long long *tab = (unsigned long long *)ctx->scratch("md_mconf", (uint64_t)slots * 8);
    uint32_t *bits = (uint32_t *)ctx->scratch("md_mbits", nbits / 8);
    if (!tab || !bits) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(lcnt, 0, kMjStripes * kMjCntStride * 4, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(tab, 0, (uint64_t)slots * 8, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(bits, 0, nbits / 8, ctx->stream));
    hipLaunchKernelGGL(k_mate_win, dim3(oge_ceil_div(n, kMjT)), dim3(kMjT), 0, ctx->stream, (const uint32_t *)f.cpos,
                       (const uint64_t *)f.cval, n, ckl.ib, partner, mate, tab, slots - 1, bits, nbits - 1, cnt + 1, lk, lcnt,
                       lcap);
    OGE_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(k_mate_agree, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)f.cval, n, ckl.ib,
                       (const uint32_t *)partner, mate, tab, slots - 1, bits, nbits - 1, cnt + 1, lk, lcnt, lcap);
    OGE_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(k_mate_check, dim3(nb), dim3(kT), 0, ctx->stream, (const uint64_t *)f.cval, n, ckl.ib,
                       (const unsigned long long *)tab, slots - 1, (const uint32_t *)bits, nbits - 1, mate, bcnt, lk, lcnt, lcap);
    OGE_LAUNCH_CHECK(ctx);
    uint32_t lc[kMjStripes * kMjCntStride], ovf = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(lc, lcnt, sizeof(lc), hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&ovf, cnt + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t left = 0;
    uint32_t lmax = 0;
    for (uint32_t q = 0; q < kMjStripes; ++q) left += lc[q * kMjCntStride], lmax = std::max(lmax, lc[q * kMjCntStride]);
    ctx->counters["md_mate_left"] = left;
    if (ovf || lmax > lcap) {
        ctx->counters["md_mate_ovf"] = 1;
        return OGE_OK;
    }
    int rc;
    if (left) {  // the leftovers through the sort-based join, their pairs into mate[] / the block counts
        uint64_t *lkc = (uint64_t *)ctx->scratch("md_ck", (left + 1) * 8);
        if (!lkc) return OGE_ERR_HIP;
        hipLaunchKernelGGL(k_left_pack, dim3(std::max<uint32_t>(1, oge_ceil_div(lmax, 4 * kT)), kMjStripes), dim3(kT), 0, ctx->stream,
                           (const uint64_t *)lk, (const unsigned int *)lcnt, lcap, lkc);
        OGE_LAUNCH_CHECK(ctx);
        uint64_t *lp, *spare;
        uint32_t lnp = 0;
        if ((rc = join_sorted(ctx, ckl, recs, meta, n, nullptr, f.cval, (uint32_t)left, &lp, &spare, &lnp, lkc))) return rc;
        if (lnp) {
            hipLaunchKernelGGL(k_mate_scatter, dim3(oge_ceil_div(lnp, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)lp, lnp, mate, bcnt);
            OGE_LAUNCH_CHECK(ctx);
        }
    }
    // all pairs in first-record order: the blocks' counts scanned, each block's owners written from its offset
    OGE_HIP_TRY(ctx, hipMemsetAsync(bcnt + nb, 0, 4, ctx->stream));
    if ((rc = oge_exclusive_scan_u32(ctx, bcnt, bcnt, (uint64_t)nb + 1))) return rc;
    uint32_t np = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&np, bcnt + nb, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt + 2, 0, 4, ctx->stream));
    if ((rc = pair_build(ctx, L, recs, meta, f, nullptr, np, P, cnt + 2, true))) return rc;  // buffers only
    if (np) {
        hipLaunchKernelGGL(k_mate_compact, dim3(nb), dim3(kT), 0, ctx->stream, (const uint32_t *)bcnt, (const uint32_t *)mate, n,
                           recs, meta, L, P->hi, P->lo, P->idx, f.skeys, P->pax, P->dev, cnt + 2);
        OGE_LAUNCH_CHECK(ctx);
    }
    uint32_t bad = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&bad, cnt + 2, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->counters["md_mate_pairs"] = np;
    if (bad) {
        ctx->counters["md_mate_redo"] = bad;
        *P = OgeMdPairs{};
        return OGE_OK;
    }
    *done = true;
    return OGE_OK;
}

int oge_md_join_build(oge_ctx *ctx, const oge_markdup_opts *opts, const uint8_t *recs, const RecMeta *meta, uint64_t n,
                      const OgeMdFrags &f, OgeMdPairs *P) {
    KeyLayout L;
    int rc = md_layout(ctx, opts, &L);
    if (rc) return rc;
    *P = OgeMdPairs{};
    const CandKey ckl = md_candkey(opts, n);
    uint32_t nc = f.nc;
    if (!f.cpos_scanned) {  // oge_md_cand_frag left the candidate flags for the windowed join
        bool done = false;
        if ((rc = join_window(ctx, L, ckl, recs, meta, n, f, P, &done))) return rc;
        if (done) return OGE_OK;
        // the sort path after all: the flags' exclusive scan (the window path left them untouched)
        if ((rc = oge_exclusive_scan_u32(ctx, f.cpos, f.cpos, n + 1))) return rc;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&nc, f.cpos + n, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    uint64_t *pairs, *pairs2;
    uint32_t np = 0;
    if ((rc = join_sorted(ctx, ckl, recs, meta, n, f.cpos, f.cval, nc, &pairs, &pairs2, &np))) return rc;
    // order the pairs by first-mate position: k_pair_build then reads both summaries from nearby rows
    uint64_t *spairs = pairs;
    rc = oge_radix_sort_pairs(ctx, pairs, nullptr, pairs2, nullptr, np, bits_mask_hi32(n), &spairs, nullptr);
    if (rc) return rc;
    return pair_build(ctx, L, recs, meta, f, spairs, np, P, nullptr);
}

// hk / val of pairs built without them (pair_build's lazy_hk), for the paths that sort by them
static int pairs_hk(oge_ctx *ctx, OgeMdPairs &P) {
    if (P.hk || !P.np) return OGE_OK;
    P.hk = (uint64_t *)ctx->scratch("md_hi2", (uint64_t)P.np * 8);
    P.val = (uint32_t *)ctx->scratch("md_pv", (uint64_t)P.np * 4);
    if (!P.hk || !P.val) return OGE_ERR_HIP;
    hipLaunchKernelGGL(k_pair_rehash, dim3(oge_ceil_div(P.np, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)P.hi,
                       (const uint64_t *)P.lo, P.np, P.hk, P.val);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

static int pair_groups_sorted(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t *hk, uint32_t *val, uint32_t m,
                              const OgeMdPairs &P, uint8_t *dup);
int oge_md_pair_groups(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdPairs &P0, uint8_t *dup) {
    OgeMdPairs P = P0;
    if (int rc = pairs_hk(ctx, P)) return rc;
    return pair_groups_sorted(ctx, opts, P.hk, P.val, P.np, P, dup);
}

int oge_md_frag_groups(oge_ctx *ctx, uint64_t *fk, uint32_t *fv, uint64_t n, uint8_t *dup) {
    if (!n) return OGE_OK;
    uint64_t *fk2 = (uint64_t *)ctx->scratch("md_fk2", (n + 1) * 8);
    uint32_t *fv2 = (uint32_t *)ctx->scratch("md_fv2", (n + 1) * 4);
    if (!fk2 || !fv2) return OGE_ERR_HIP;
    uint64_t o = 0, a = 0;
    int rc = oge_reduce_or_and_u64(ctx, fk, n, (1ull << 47) - 1, &o, &a);
    if (rc) return rc;
    uint64_t *k;
    uint32_t *v;
    rc = oge_radix_sort_pairs(ctx, fk, fv, fk2, fv2, n, (o ^ a) & ((1ull << 47) - 1), &k, &v);
    if (rc) return rc;
    hipLaunchKernelGGL(k_frag_groups, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)k, (const uint32_t *)v, n,
                       dup);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

// window bounds of every tile into scratch, and the list of tiles whose window exceeds cap
struct WinPlan {
    uint2 *bounds = nullptr;
    uint32_t ntiles = 0;
    uint32_t *ovl = nullptr;  // overflowing tiles (device)
    uint32_t novf = 0;
    uint64_t ovf_items = 0;   // window items of the overflowing tiles (bounds the owned items)
};
static int md_win_bounds(oge_ctx *ctx, const uint64_t *skeys, const int64_t *ax, uint64_t n, uint32_t cap,
                         const unsigned long long *dev_slots, int64_t amax, WinPlan *W) {
    W->ntiles = oge_ceil_div(n, kWinTile);
    W->bounds = (uint2 *)ctx->scratch("md_winb", (uint64_t)W->ntiles * sizeof(uint2));
    W->ovl = (uint32_t *)ctx->scratch("md_winovl", (uint64_t)W->ntiles * 4);
    // cnt[0] = overflowing tiles, cnt[1..2] = their window items (u64)
    unsigned int *cnt = (unsigned int *)ctx->ws("md_winovf", 16);
    unsigned long long *dev = (unsigned long long *)ctx->ws("md_windev", 2 * sizeof(unsigned long long));
    if (!W->bounds || !W->ovl || !cnt || !dev) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
    hipLaunchKernelGGL(k_dev_fold, dim3(1), dim3(kDevSlots), 0, ctx->stream, dev_slots, dev);
    OGE_LAUNCH_CHECK(ctx);
    hipLaunchKernelGGL(k_win_bounds, dim3(oge_ceil_div(W->ntiles, kT)), dim3(kT), 0, ctx->stream, skeys, ax, n, W->ntiles, cap,
                       (const unsigned long long *)dev, amax, W->bounds, W->ovl, cnt, (unsigned long long *)(cnt + 2));
    OGE_LAUNCH_CHECK(ctx);
    uint32_t h[4] = {0, 0, 0, 0};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(h, cnt, 16, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    W->novf = h[0];
    W->ovf_items = (uint64_t)h[2] | ((uint64_t)h[3] << 32);
    return OGE_OK;
}

// OGE_MD_WINCAP=k (tests) lowers the window caps so that most tiles overflow and take the collect + sort
// path.  Read per call.
static uint32_t md_win_cap(uint32_t cap) {
    const char *e = getenv("OGE_MD_WINCAP");
    const long v = e && *e ? atol(e) : 0;
    return v > 0 && (uint64_t)v < cap ? (uint32_t)v : cap;
}

// sort-based pair groups over (hk, val) lists of m pairs: hk's top rb bits group equal chunk keys,
// k_pair_groups_h splits the runs into exact keys and picks each chunk's best explicitly
static int pair_groups_sorted(oge_ctx *ctx, const oge_markdup_opts *opts, uint64_t *hk, uint32_t *val, uint32_t m,
                              const OgeMdPairs &P, uint8_t *dup) {
    if (!m) return OGE_OK;
    uint64_t *lo2 = (uint64_t *)ctx->scratch("md_lo2", (uint64_t)m * 8);
    uint32_t *pv2 = (uint32_t *)ctx->scratch("md_pv2", (uint64_t)m * 4);
    if (!lo2 || !pv2) return OGE_ERR_HIP;
    // 32 bits of a hash of the whole chunk key (hk) group equal keys (k_pair_groups_h splits runs);
    // debug_hash_bits (tests) also narrows these bits, so runs holding several keys are exercised
    uint64_t *k2;
    uint32_t *v2;
    const int rb = opts->debug_hash_bits > 0 ? std::min(32, opts->debug_hash_bits) : 32;
    const uint64_t rmask = ~0ull << (64 - rb);
    int rc = oge_radix_sort_pairs(ctx, hk, val, lo2, pv2, m, rmask, &k2, &v2);
    if (rc) return rc;
    hipLaunchKernelGGL(k_pair_groups_h, dim3(oge_ceil_div(m, kT)), dim3(kT), 0, ctx->stream, (const uint64_t *)k2,
                       (const uint32_t *)v2, (const uint64_t *)P.hi, (const uint64_t *)P.lo, (const uint2 *)P.idx, m, rmask, dup);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

int oge_md_frag_groups_win(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdFrags &f, uint64_t n, uint8_t *dup,
                           bool *done) {
    *done = false;
    if (!f.skeys || !f.dev || opts->debug_sort_groups) return OGE_OK;
    if (!n) { *done = true; return OGE_OK; }
    KeyLayout L;
    int rc = md_layout(ctx, opts, &L);
    if (rc) return rc;
    OgeStageTimer *t = ctx->begin_stage("md_frag_win");  // nested in md_frags: shows which path ran
    // the unmapped tail (refID' = n_ref) holds no fragment
    const int64_t amax = ((int64_t)opts->n_ref << 34) + (1ll << 32);
    WinPlan W;
    const uint32_t cap = md_win_cap(kFragCap);
    if ((rc = md_win_bounds(ctx, f.skeys, nullptr, n, cap, f.dev, amax, &W))) return rc;
    hipLaunchKernelGGL(k_frag_win, dim3(W.ntiles), dim3(kT), 0, ctx->stream, (const uint64_t *)f.fk, (const uint32_t *)f.fv,
                       f.skeys, n, L, (const uint2 *)W.bounds, cap, dup);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    if (W.novf) {  // the overflowing tiles' fragments through the sort-based stage
        t = ctx->begin_stage("md_frag_ovf");
        uint64_t *ok = (uint64_t *)ctx->scratch("md_ofk", W.ovf_items * 8 + 8);
        uint32_t *ov = (uint32_t *)ctx->scratch("md_ofv", W.ovf_items * 4 + 4);
        unsigned int *cnt = (unsigned int *)ctx->ws("md_ocnt", 4);
        if (!ok || !ov || !cnt) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 4, ctx->stream));
        hipLaunchKernelGGL(k_win_collect<false>, dim3(W.novf), dim3(kT), 0, ctx->stream, (const uint64_t *)f.fk,
                           (const uint32_t *)f.fv, (const uint64_t *)nullptr, (const uint64_t *)nullptr, f.skeys,
                           (const int64_t *)nullptr, n, L, (const uint2 *)W.bounds, (const uint32_t *)W.ovl, ok, ov, cnt);
        OGE_LAUNCH_CHECK(ctx);
        unsigned int m = 0;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&m, cnt, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if ((rc = oge_md_frag_groups(ctx, ok, ov, m, dup))) return rc;
        ctx->end_stage(t);
    }
    *done = true;
    return OGE_OK;
}

int oge_md_pair_groups_win(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdPairs &P, uint8_t *dup, bool *done) {
    *done = false;
    if (!P.pax || !P.dev || opts->debug_sort_groups) return OGE_OK;
    if (!P.np) { *done = true; return OGE_OK; }
    // debug_hash_bits narrows the sort-based path's hash to exercise its collision handling: keep it
    if (opts->debug_hash_bits > 0) return OGE_OK;
    KeyLayout L;
    int rc = md_layout(ctx, opts, &L);
    if (rc) return rc;
    OgeStageTimer *t = ctx->begin_stage("md_pair_win");  // nested in md_pairs
    WinPlan W;
    const uint32_t cap = md_win_cap(kPairCap);
    if ((rc = md_win_bounds(ctx, nullptr, P.pax, P.np, cap, P.dev, INT64_MAX, &W))) return rc;
    hipLaunchKernelGGL(k_pair_win, dim3(W.ntiles), dim3(kT), 0, ctx->stream, (const uint64_t *)P.hi, (const uint64_t *)P.lo,
                       (const uint2 *)P.idx, (const int64_t *)P.pax, (uint64_t)P.np, L, (const uint2 *)W.bounds, cap, dup);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    if (W.novf) {  // the overflowing tiles' pairs through the sort-based stage
        t = ctx->begin_stage("md_pair_ovf");
        OgeMdPairs Q = P;
        if ((rc = pairs_hk(ctx, Q))) return rc;
        uint64_t *ok = (uint64_t *)ctx->scratch("md_ohk", W.ovf_items * 8 + 8);
        uint32_t *ov = (uint32_t *)ctx->scratch("md_opv", W.ovf_items * 4 + 4);
        unsigned int *cnt = (unsigned int *)ctx->ws("md_ocnt", 4);
        if (!ok || !ov || !cnt) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 4, ctx->stream));
        hipLaunchKernelGGL(k_win_collect<true>, dim3(W.novf), dim3(kT), 0, ctx->stream, (const uint64_t *)Q.hk,
                           (const uint32_t *)nullptr, (const uint64_t *)P.hi, (const uint64_t *)P.lo,
                           (const uint64_t *)nullptr, (const int64_t *)P.pax, (uint64_t)P.np, L, (const uint2 *)W.bounds,
                           (const uint32_t *)W.ovl, ok, ov, cnt);
        OGE_LAUNCH_CHECK(ctx);
        unsigned int m = 0;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&m, cnt, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if ((rc = pair_groups_sorted(ctx, opts, ok, ov, m, P, dup))) return rc;
        ctx->end_stage(t);
    }
    *done = true;
    return OGE_OK;
}

int oge_md_apply_desc(oge_ctx *ctx, const uint64_t *desc0, uint64_t n, uint8_t *dup, uint64_t *desc, uint64_t *n_dup_out) {
    unsigned long long *ndup = (unsigned long long *)ctx->ws("md_ndup", 8);
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    if (!ndup || !cnt) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(ndup, 0, 8, ctx->stream));
    if (n) {
        hipLaunchKernelGGL(k_apply_desc, dim3(std::min<uint32_t>(oge_ceil_div(n, kT), 2048u)), dim3(kT), 0, ctx->stream, desc0, n, dup, 0,
                           (const unsigned int *)(cnt + 1), ndup, desc);
        OGE_LAUNCH_CHECK(ctx);
    }
    unsigned long long h = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&h, ndup, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_dup_out = h;
    return OGE_OK;
}

// 0x400 set / cleared in place on the primaries of n records (record k at recs + off[k], summary
// meta[k], mark dup[k]); dup[k] becomes 1/0/2 as in oge_markdup.  *n_dup_out: records flagged.
int oge_md_apply_inplace(oge_ctx *ctx, uint8_t *recs, const uint64_t *off, uint64_t n, const RecMeta *meta, uint8_t *dup,
                         uint64_t *n_dup_out) {
    unsigned long long *ndup = (unsigned long long *)ctx->ws("md_ndup", 8);
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    if (!ndup || !cnt) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(ndup, 0, 8, ctx->stream));
    if (n) {
        hipLaunchKernelGGL(k_apply, dim3(std::min<uint32_t>(oge_ceil_div(n, kT), 2048u)), dim3(kT), 0, ctx->stream, recs, off, n, meta,
                           dup, 1, 0, (const unsigned int *)(cnt + 1), ndup);
        OGE_LAUNCH_CHECK(ctx);
    }
    unsigned long long h = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&h, ndup, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_dup_out = h;
    return OGE_OK;
}

// Everything after the per-record ReadEnds pass.  meta[i] describes record i of the stream
// (record index = i); its bytes are at recs + meta[i].src (only read to confirm pair keys).
// dup[i] receives 1/0/2 (see oge_markdup); with apply, FLAG 0x400 is rewritten in place at
// recs + off[i].
int oge_markdup_finish_pre(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                           const RecMeta *meta, uint8_t *d_dup, int apply, uint64_t *n_dup_out, uint64_t *d_desc, bool *desc_ok,
                           const uint64_t *skeys, const OgeMdFrags *pre);
int oge_markdup_finish(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                       const oge_markdup_opts *opts, const RecMeta *meta, uint8_t *d_dup, int apply, uint64_t *n_dup_out,
                       uint64_t *d_desc, bool *desc_ok, const uint64_t *skeys) {
    return oge_markdup_finish_pre(ctx, d_recs, d_off, n, opts, meta, d_dup, apply, n_dup_out, d_desc, desc_ok, skeys, nullptr);
}
// pre: the products of oge_md_cand_frag_gather (the fused gather already wrote them for these n records)
int oge_markdup_finish_pre(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                           const RecMeta *meta, uint8_t *d_dup, int apply, uint64_t *n_dup_out, uint64_t *d_desc, bool *desc_ok,
                           const uint64_t *skeys, const OgeMdFrags *pre) {
    if (desc_ok) *desc_ok = false;
    KeyLayout L;
    int rc = md_layout(ctx, opts, &L);
    if (rc) return rc;
    unsigned int *cnt = (unsigned int *)ctx->ws("md_counts", 16);
    unsigned long long *ndup = (unsigned long long *)ctx->ws("md_ndup", 8);
    if (!cnt || !ndup) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(d_dup, 0, n ? n : 1, ctx->stream));
    if (!n) { *n_dup_out = 0; return OGE_OK; }
    const uint32_t nb = oge_ceil_div(n, kT);

    // ---- mate join ----
    OgeStageTimer *t = ctx->begin_stage("md_matejoin");
    OgeMdFrags F;
    if (pre) {  // the fused gather's products: only the scan / overflow read-back is left
        if (!pre->fused || pre->skeys != skeys || (d_desc && !pre->desc0))
            return oge_fail(ctx, OGE_ERR_ARG, "markdup: precomputed summaries do not match this call");
        F = *pre;
        rc = cand_frag_post(ctx, opts, n, &F);
    } else {
        rc = oge_md_cand_frag(ctx, opts, meta, n, d_desc != nullptr, &F, skeys);
    }
    if (rc) return rc;
    const bool use_desc = d_desc && !F.desc_ovf;
    OgeMdPairs P;
    rc = oge_md_join_build(ctx, opts, d_recs, meta, n, F, &P);
    if (rc) return rc;
    ctx->end_stage(t);

    // ---- pair groups ----
    t = ctx->begin_stage("md_pairs");
    bool done = false;
    rc = oge_md_pair_groups_win(ctx, opts, P, d_dup, &done);
    if (!rc && !done) rc = oge_md_pair_groups(ctx, opts, P, d_dup);
    if (rc) return rc;
    ctx->end_stage(t);

    // ---- fragment groups ----
    t = ctx->begin_stage("md_frags");
    rc = oge_md_frag_groups_win(ctx, opts, F, n, d_dup, &done);
    if (!rc && !done) rc = oge_md_frag_groups(ctx, F.fk, F.fv, n, d_dup);  // fk / fv were written by k_cand_frag
    if (rc) return rc;
    ctx->end_stage(t);

    // ---- apply ----
    if (pre && pre->defer_apply && use_desc && !apply && !opts->compat_nonverbose_index) {
        // the record gather finishes the descriptors (desc0 + dup) and counts the duplicates itself
        if (desc_ok) *desc_ok = true;
        *n_dup_out = ~0ull;
        return OGE_OK;
    }
    t = ctx->begin_stage("md_apply");
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt, 0, 16, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(ndup, 0, 8, ctx->stream));
    if (opts->compat_nonverbose_index) {
        hipLaunchKernelGGL(k_any, dim3(nb), dim3(kT), 0, ctx->stream, (const uint8_t *)d_dup, n, cnt + 1);
        OGE_LAUNCH_CHECK(ctx);
    }
    if (use_desc && !apply)
        hipLaunchKernelGGL(k_apply_desc, dim3(std::min<uint32_t>(nb, 2048u)), dim3(kT), 0, ctx->stream, (const uint64_t *)F.desc0,
                           n, d_dup, opts->compat_nonverbose_index, (const unsigned int *)(cnt + 1), ndup, d_desc);
    else
        hipLaunchKernelGGL(k_apply, dim3(std::min<uint32_t>(nb, 2048u)), dim3(kT), 0, ctx->stream, d_recs, d_off, n, meta, d_dup,
                           apply, opts->compat_nonverbose_index, (const unsigned int *)(cnt + 1), ndup);
    OGE_LAUNCH_CHECK(ctx);
    ctx->end_stage(t);
    unsigned long long h = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&h, ndup, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *n_dup_out = h;
    if (desc_ok) *desc_ok = use_desc && !apply;
    return OGE_OK;
}

namespace {
// bad[2] |= 1 when some record's anchor (refID', pos + 1) is smaller than its predecessor's
__global__ __launch_bounds__(kT) void k_anchors_sorted(const uint64_t *__restrict__ keys, uint64_t n, unsigned int *__restrict__ bad) {
    bool down = false;
    for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * kT)
        down |= anchor_of_key(keys[i]) < anchor_of_key(keys[i - 1]);
    if (__ballot(down) && (threadIdx.x & 63) == __builtin_ctzll(__ballot(down))) atomicOr(bad + 2, 1u);
}
}  // namespace

// Standalone duplicate marking of records in stream order (record index = position): `openge dedup`
// (commands/command_dedup.cpp:48-69 -> MarkDuplicates over the file's records as they come).
// r06: the input pass also writes each record's coordinate key, and when the keys'
// anchors (refID', pos + 1) never decrease -- a coordinate-sorted file, which is what `openge dedup` is
// run on -- the keys go to the windowed mate join and groups exactly as in the fused chain (whose exactness
// needs only that the record index order has non-decreasing anchors, not the sort itself).  Anything else
// (unsorted input, refIDs outside the dictionary, OGE_MD_INPLACE_WINDOW=0) keeps the sort-based paths.
int oge_markdup_run(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                    uint8_t *d_dup, int apply, uint64_t *n_dup_out) {
    RecMeta *meta;
    OgeRgTable rg;
    int rc = oge_markdup_prepare(ctx, opts, n, "md_meta", &meta, &rg);
    if (rc) return rc;
    const char *we = getenv("OGE_MD_INPLACE_WINDOW");
    const bool try_win = n > 1 && n < (1ull << 31) && !(we && we[0] == '0');
    uint64_t *keys = nullptr;
    uint32_t *vals = nullptr;
    unsigned int *bad = nullptr;
    if (try_win) {
        keys = (uint64_t *)ctx->scratch("mdi_keys", (n + 1) * 8);
        vals = (uint32_t *)ctx->scratch("mdi_vals", (n + 1) * 4);
        bad = (unsigned int *)ctx->ws("mdi_bad", 16);
        if (!keys || !vals || !bad) return OGE_ERR_HIP;
        OGE_HIP_TRY(ctx, hipMemsetAsync(bad, 0, 16, ctx->stream));
    }
    OgeStageTimer *t = ctx->begin_stage("md_readends");
    OgePassArgs a = {};
    a.recs = d_recs;
    a.off = d_off;
    a.n = n;
    a.meta = meta;
    a.rg = rg;
    a.keys = keys;
    a.vals = vals;
    a.n_ref = opts->n_ref;
    a.bad = bad;
    // with the keys (try_win) the input pass also writes k_cand_frag's words from the summaries it builds
    // (r06): the rows are not streamed a second time
    OgeMdFrags F;
    if (try_win) {
        KeyLayout L;
        CandKey ck;
        if ((rc = cand_frag_alloc(ctx, opts, n, false, true, &F, &L, &ck))) return rc;
        OGE_HIP_TRY(ctx, hipMemsetAsync(F.cpos + n, 0, 4, ctx->stream));
        a.cf_f = F.cpos, a.cf_fk = F.fk, a.cf_fv = F.fv, a.cf_cval = F.cval, a.cf_dev = F.dev;
        a.cf_sb = L.sb, a.cf_lb = L.lb, a.cf_split = L.split_k, a.cf_ib = ck.ib, a.cf_hb = ck.hb;
        F.fused = true;
    }
    rc = oge_input_pass(ctx, a);
    if (rc) return rc;
    const uint64_t *skeys = nullptr;
    if (try_win) {
        hipLaunchKernelGGL(k_anchors_sorted, dim3((uint32_t)std::min<uint64_t>(oge_ceil_div(n, kT), 4096)), dim3(kT), 0, ctx->stream,
                           (const uint64_t *)keys, n, bad);
        OGE_LAUNCH_CHECK(ctx);
        unsigned int hb[3] = {0, 0, 0};
        OGE_HIP_TRY(ctx, hipMemcpyAsync(hb, bad, 12, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        const bool sorted = !(hb[0] & 1) && !hb[2];
        ctx->counters["md_inplace_window"] = sorted;
        if (sorted) skeys = keys;
        F.skeys = skeys;  // unsorted: the words stand, the deviation slots go unused (no windowed stage)
        if (!sorted) F.dev = nullptr;
    }
    ctx->end_stage(t);
    return oge_markdup_finish_pre(ctx, d_recs, d_off, n, opts, meta, d_dup, apply, n_dup_out, nullptr, nullptr, skeys,
                                  try_win ? &F : nullptr);
}

namespace {
// four lanes per 64-byte summary, 16 bytes each: a wave moves 16 rows with one load and one store
// instruction (r04: one lane per row, four of each)
__global__ __launch_bounds__(kT) void k_meta_gather(const RecMeta *__restrict__ in, const uint32_t *__restrict__ perm, uint64_t n,
                                                     RecMeta *__restrict__ out) {
    static_assert(sizeof(RecMeta) == 64, "four 16-byte pieces per summary");
    const uint64_t g = (uint64_t)blockIdx.x * kT + threadIdx.x, k = g >> 2;
    const uint32_t part = (uint32_t)g & 3;
    if (k < n) ((uint4 *)(out + k))[part] = ((const uint4 *)(in + perm[k]))[part];
}
}  // namespace

// out[k] = in[perm[k]]: ReadEnds summaries into sorted order (one random 64-byte read per record).
int oge_meta_gather(oge_ctx *ctx, const RecMeta *in, const uint32_t *perm, uint64_t n, RecMeta *out) {
    if (!n) return OGE_OK;
    hipLaunchKernelGGL(k_meta_gather, dim3(oge_ceil_div(4 * n, kT)), dim3(kT), 0, ctx->stream, in, perm, n, out);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}
