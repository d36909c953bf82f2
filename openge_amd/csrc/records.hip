// records.hip -- the two streaming passes over BAM records of the sort+dedup pipeline.
//
// k_input_pass (input order, records read once): a 256-thread block stages a tile of 256
//   consecutive records (~73 KB for 150 bp reads) into LDS with 16-byte LDS-DMA loads
//   (global_load_lds_dwordx4: the whole tile in flight at once), then each
//   thread parses one record from LDS and emits
//     KEYS: the coordinate sort key (sort.hip) and its index
//     META: a 32-byte summary -- the fragment ReadEnds fields of buildReadEnds
//           (algorithms/mark_duplicates.cpp:147-164: getUnclippedStart/End :88-129, getScore :135-144,
//           getLibraryId :282-318), the RG ":" name pair-key hash (:210-213), the bin the writer must
//           store (util/bam_serializer.h:112-116), the flag byte and the record's source offset.
//   Records outside the staged window (non-contiguous offsets, >76 KB tiles) are parsed straight
//   from global memory by the same code.
//
// k_gather16 (output order, records read once and written once): a wave owns 64 consecutive
//   output records, whose output bytes are one contiguous range.  Lanes write that range as
//   aligned 16-byte chunks; a chunk is one unaligned 16-byte load of the source record (gfx950 serves
//   unaligned dwordx4 at stream rate, tools/probes/unaligned.hip).  Where a record boundary falls
//   inside the chunk it is the tail 16 bytes of one record and the head 16 bytes of the next,
//   funnel-shifted together -- every load stays inside its record, so no cache line outside the
//   records is fetched.  Bin and FLAG 0x400 are patched in registers.  Only the two chunks at the
//   ends of a batch, shared with neighbouring waves, fall back to byte stores.
#include <algorithm>
#include <cstdlib>

#include "oge_ctx.h"
#include "bam_layout.h"
#include "dev_util.h"
#include "records.h"
#include "md_keys.h"

namespace {

constexpr int kT = 256;

// --- byte readers over the LDS tile or global memory (x = absolute byte index) ---
struct LdsRd {
    const uint8_t *b;  // LDS tile base (16-byte aligned)
    __device__ __forceinline__ uint32_t u8(uint64_t x) const { return b[x]; }
    __device__ __forceinline__ uint32_t a32(uint64_t x) const { return *(const uint32_t *)(b + x); }
    __device__ __forceinline__ uint4 a128(uint64_t x) const { return *(const uint4 *)(b + x); }
    __device__ __forceinline__ uint32_t u32(uint64_t x) const {
        const uint32_t sh = (uint32_t)(x & 3) * 8;
        const uint32_t lo = a32(x & ~3ull);
        return sh ? (lo >> sh) | (a32((x & ~3ull) + 4) << (32 - sh)) : lo;
    }
};
struct GlbRd {
    const uint8_t *b;  // arena base
    __device__ __forceinline__ uint32_t u8(uint64_t x) const { return b[x]; }
    __device__ __forceinline__ uint32_t a32(uint64_t x) const { return *(const uint32_t *)(b + x); }
    __device__ __forceinline__ uint4 a128(uint64_t x) const { return *(const uint4 *)(b + x); }
    __device__ __forceinline__ uint32_t u32(uint64_t x) const { return oge_ldu32(b + x); }
};

// getScore's per-byte term (b >= 15 ? b : 0) summed over the 4 bytes of w, plus acc: a SWAR
// ">= 15" mask (no carries cross bytes: low 7 bits + 0x71 <= 0xf0; bytes >= 128 pass by their top
// bit) and one v_sad_u8 against zero.
__device__ __forceinline__ uint32_t qsum4(uint32_t w, uint32_t acc) {
    const uint32_t ge = (((w & 0x7f7f7f7fu) + 0x71717171u) | w) & 0x80808080u;
    return __builtin_amdgcn_sad_u8(w & ((ge >> 7) * 0xffu), 0u, acc);
}

// The pair-key hash (split chain, RG string, read name) folded 4 bytes at a time -- each segment's length,
// then its little-endian words, the tail zero-padded; a 64-bit multiply per word -- and finished with the
// MurmurHash3 fmix64 avalanche so every bit of the 48 kept is usable as a radix digit (the mate join sorts
// by as many bits as fit).  Any function of the key bytes serves: the mate join and the pair groups
// confirm the exact key (test_gpu_parity forces collisions).  r05: words instead of a byte-wise FNV-1a
// chain, whose one dependent LDS byte read per step sat on the parse's critical path.
__device__ __forceinline__ uint64_t h_word(uint64_t h, uint32_t w) { return (h ^ w) * 0x9e3779b97f4a7c15ull; }
__device__ __forceinline__ uint64_t h_fmix(uint64_t h) {
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; return h ^ (h >> 33);
}
template <class Rd>
__device__ __forceinline__ uint64_t h_bytes(const Rd &rd, uint64_t h, uint64_t p, uint32_t len) {
    h = h_word(h, len);
    uint32_t y = 0;
    for (; y + 4 <= len; y += 4) h = h_word(h, rd.u32(p + y));
    if (y < len) {
        uint32_t w = 0;
        for (uint32_t k = 0; y + k < len; ++k) w |= rd.u8(p + y + k) << (8 * k);
        h = h_word(h, w);
    }
    return h;
}

// Record at absolute index r of reader `rd`; i = record index, src = its offset in the arena.
template <bool META, bool KEYS, class Rd>
__device__ __forceinline__ void parse_input(const Rd &rd, uint64_t r, uint64_t i, uint64_t src, const OgePassArgs &a, uint64_t &kor,
                                            uint64_t &knot, uint64_t &dv0, uint64_t &dv1) {
    uint64_t kk = 0;  // the coordinate key (KEYS)
    const uint32_t bs = rd.u32(r);
    const int32_t ref = (int32_t)rd.u32(r + OGE_OFF_REFID);
    const int32_t pos = (int32_t)rd.u32(r + OGE_OFF_POS);
    const uint32_t w12 = rd.u32(r + OGE_OFF_LNAME);
    const uint32_t w16 = rd.u32(r + OGE_OFF_NCIGAR);
    const uint32_t lname = w12 & 0xFF, nc = w16 & 0xFFFF, flag = w16 >> 16;
    const uint32_t lseq = rd.u32(r + OGE_OFF_LSEQ);
    if (KEYS) {
        uint64_t k;
        if (ref == -1) {
            k = (uint64_t)(uint32_t)a.n_ref << 33;
        } else {
            if (ref < -1 || ref >= a.n_ref || pos < -1) atomicOr(a.bad, 1u);
            k = ((uint64_t)(uint32_t)ref << 33) | ((uint64_t)(uint32_t)(pos + 1) << 1) | ((flag >> 4) & 1u);
        }
        if (bs < 32 || bs > 10000) atomicOr(a.bad, 2u);
        a.keys[i] = k | ((uint64_t)(bs + 4) << 50);
        kk = k;
        kor |= k;
        knot |= ~k & OGE_SORT_KEY_MASK;
        a.vals[i] = (uint32_t)(a.ibase + i);
    }
    if (!META) return;
    const uint64_t c = r + OGE_OFF_NAME + lname;
    int32_t rl = 0, lead = 0, trail = 0;
    bool in_lead = true;
    for (uint32_t k = 0; k < nc; ++k) {
        const uint32_t op = rd.u32(c + 4 * k), t = op & 0xF, len = op >> 4;
        if (t == OGE_CIG_M || t == OGE_CIG_D || t == OGE_CIG_N || t == OGE_CIG_EQ || t == OGE_CIG_X) rl += (int32_t)len;
        const bool clip = (t == OGE_CIG_S || t == OGE_CIG_H);
        if (in_lead && clip) lead += (int32_t)len; else in_lead = false;
        trail = clip ? trail + (int32_t)len : 0;
    }
    RecMeta M;
    M.src = src;
    M.seq = -1;
    M.coord = 0;
    M.rgi = OGE_RGI_NONE;
    M.hash_hi = 0;
    M.hash = 0;
    uint64_t m = ((uint64_t)oge_reg2bin(pos, pos + rl) << 48) | ((uint64_t)(flag >> 8) << 40);
    if (!(flag & OGE_F_SECONDARY)) m |= OGE_M_PRIMARY;
    // name slot, every record: l_read_name bytes (with the NUL) when they fit, zero-padded -- the sort's
    // tie order compares these instead of the records' bytes (r05: only mate-join candidates had it, and
    // ties between any other records read their names byte by byte from global memory)
    if (lname <= OGE_NAME_SLOT) {
        m |= OGE_M_NAMEFIT;
        uint32_t *ns = (uint32_t *)M.name;
#pragma unroll
        for (uint32_t q = 0; q < OGE_NAME_SLOT / 4; ++q) {
            uint32_t v = 0;
            if (4 * q < lname) {
                v = rd.u32(r + OGE_OFF_NAME + 4 * q);
                const uint32_t rem = lname - 4 * q;
                if (rem < 4) v &= (1u << (8 * rem)) - 1u;
            }
            ns[q] = v;
        }
    }
    if (!((flag & OGE_F_UNMAP) || ref == -1 || (flag & OGE_F_SECONDARY))) {
        m |= OGE_M_FRAG;
        const bool rev = (flag & OGE_F_REVERSE) != 0;
        if (rev) m |= OGE_M_REV;
        M.coord = rev ? pos + rl - 1 + trail : pos - lead;  // getUnclippedEnd / getUnclippedStart
        M.seq = ref;
        // getScore: int16 accumulator over raw quality bytes >= 15
        const uint64_t q0 = c + 4 * nc + (lseq + 1) / 2, q1 = q0 + lseq;
        uint32_t sc = 0;
        uint64_t x = q0;
        for (; x < q1 && (x & 15); ++x) { const uint32_t b = rd.u8(x); sc += b >= 15 ? b : 0; }
        for (; x + 16 <= q1; x += 16) {  // 16-byte aligned reads (LDS tile and arena are 16-aligned)
            const uint4 v = rd.a128(x);
            sc = qsum4(v.w, qsum4(v.z, qsum4(v.y, qsum4(v.x, sc))));
        }
        for (; x < q1; ++x) { const uint32_t b = rd.u8(x); sc += b >= 15 ? b : 0; }
        m |= (uint64_t)(uint16_t)sc;
        // RG tag (GetTag<string> / FindTag semantics, util/bamtools/BamAlignment.cpp:270-294,699-780)
        const uint64_t tend = r + 4 + bs;
        uint64_t p = q1, rgv = 0;
        uint32_t rgl = 0;
        bool has = false;
        while (p + 3 <= tend) {
            const uint32_t w = rd.u32(p);
            const uint32_t t0 = w & 0xff, t1 = (w >> 8) & 0xff, type = (w >> 16) & 0xff;
            p += 3;
            if (t0 == 'R' && t1 == 'G') {
                // the value's NUL: four bytes per read (the first zero byte of a word by the borrow trick)
                uint64_t s = p;
                for (;;) {
                    if (s + 4 <= tend) {
                        const uint32_t v = rd.u32(s);
                        const uint32_t z = (v - 0x01010101u) & ~v & 0x80808080u;
                        if (z) {
                            s += (uint32_t)__builtin_ctz(z) >> 3;
                            break;
                        }
                        s += 4;
                    } else {
                        while (s < tend && rd.u8(s)) ++s;
                        break;
                    }
                }
                rgv = p;
                rgl = (uint32_t)(s - p);
                has = true;
                break;
            }
            if (type == 0) break;
            bool ok = true;
            switch (type) {
            case 'A': case 'c': case 'C': p += 1; break;
            case 's': case 'S': p += 2; break;
            case 'f': case 'i': case 'I': p += 4; break;
            case 'Z': case 'H':
                while (p < tend && rd.u8(p)) ++p;
                ++p;
                break;
            case 'B': {
                if (p + 5 > tend) { ok = false; break; }
                const uint32_t at = rd.u8(p);
                const int32_t cnt = (int32_t)rd.u32(p + 1);
                p += 5;
                const int sz = (at == 'c' || at == 'C') ? 1 : (at == 's' || at == 'S') ? 2 : (at == 'f' || at == 'i' || at == 'I') ? 4 : 0;
                if (!sz) { ok = false; break; }
                p += (int64_t)cnt * sz;
                break;
            }
            default: ok = false;
            }
            if (!ok || p >= tend || rd.u8(p) == 0) break;
        }
        // an RG value of <= 15 bytes as four zero-padded words (compared with the table's idw and hashed)
        uint32_t rv[4] = {0u, 0u, 0u, 0u};
        if (rgl <= 15) {
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                if (4 * q >= rgl) continue;
                uint32_t v = 0;
                if (rgv + 4 * q + 4 <= tend) {
                    v = rd.u32(rgv + 4 * q);
                } else {
                    for (uint32_t k = 0; 4 * q + k < rgl; ++k) v |= rd.u8(rgv + 4 * q + k) << (8 * k);
                }
                const uint32_t rem = rgl - 4 * q;
                rv[q] = rem < 4 ? v & ((1u << (8 * rem)) - 1u) : v;
            }
        }
        int16_t lib = a.rg.unknown_lib;
        M.rgi = OGE_RGI_NONE;
        if (has && rgl) {
            M.rgi = OGE_RGI_UNLISTED;
            for (int32_t g = 0; g < a.rg.n_rg; ++g) {
                const uint32_t o = a.rg.off[g], Lg = a.rg.off[g + 1] - o - 1;
                if (Lg != rgl) continue;
                bool eq = true;
                if (Lg <= 15) {
                    const uint4 w = a.rg.idw[g];
                    eq = w.x == rv[0] && w.y == rv[1] && w.z == rv[2] && w.w == rv[3];
                } else {
                    for (uint32_t y = 0; y < Lg && eq; ++y) eq = a.rg.ids[o + y] == rd.u8(rgv + y);
                }
                if (eq) { lib = a.rg.lib[g]; M.rgi = (int16_t)g; break; }
            }
        }
        m |= (uint64_t)(uint16_t)lib << 16;
        const bool paired_mm = (flag & OGE_F_PAIRED) && !(flag & OGE_F_MUNMAP);
        // isPaired(): read2Sequence = mate refID (buildReadEnds :156-158), -1 otherwise
        if (paired_mm && (int32_t)rd.u32(r + OGE_OFF_MREFID) != -1) m |= OGE_M_PAIRED;
        if (paired_mm) {
            m |= OGE_M_CAND;
            uint64_t h = 0xcbf29ce484222325ull;
            if (a.rg.split_k > 1) h = h_word(h, 0x100u + (uint32_t)(ref % a.rg.split_k));  // the chain
            if (rgl <= 15) {  // the words read for the lookup (equal keys: equal lengths, the same branch)
                h = h_word(h, rgl);
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    if (4 * q < rgl) h = h_word(h, rv[q]);
            } else {
                h = h_bytes(rd, h, rgv, rgl);
            }
            // the name slot's words (filled above when the name fits) also feed the hash (equal keys have
            // equal lengths, so both take the same branch)
            if (lname <= OGE_NAME_SLOT) {
                const uint32_t *ns = (const uint32_t *)M.name;
                h = h_word(h, lname);
#pragma unroll
                for (uint32_t q = 0; q < OGE_NAME_SLOT / 4; ++q)
                    if (4 * q < lname) h = h_word(h, ns[q]);
            } else {
                h = h_bytes(rd, h, r + OGE_OFF_NAME, lname - 1u);
            }
            h = h_fmix(h);
            M.hash = (uint32_t)h;
            M.hash_hi = (uint16_t)(h >> 32);
        }
    }
    M.m = m;
    a.meta[i] = M;
    if (KEYS && a.cf_f) {  // the in-place dedup's key words (k_cand_frag's, without the descriptors)
        bool has = false;
        int64_t ax = 0, cx = 0;
        cand_frag_one(M, i, KeyLayout{a.cf_sb, a.cf_lb, a.cf_split}, CandKey{a.cf_ib, a.cf_hb, a.cf_split}, a.cf_f, a.cf_fk,
                      a.cf_fv, a.cf_cval, nullptr, nullptr, nullptr, has, ax, cx);
        if (m & OGE_M_FRAG) {
            ax = anchor_of_key(kk);
            cx = win_x((uint32_t)M.seq, (int64_t)M.coord + 1);
            dv0 = max(dv0, (uint64_t)(ax - cx + kDevBias));
            dv1 = max(dv1, (uint64_t)(cx - ax + kDevBias));
        }
    }
}

// NT records per tile and NT threads per block; the tile window is NT x 304 bytes of LDS (76 KB at
// NT = 256: 2 blocks per CU; 38 KB at 128: 4 blocks of 2 waves, so staging and parsing of different
// blocks overlap more finely).
template <bool META, bool KEYS, int NT>
__global__ __launch_bounds__(NT) void k_input_pass(OgePassArgs a) {
    constexpr uint32_t kTileRecs = NT;
    constexpr uint32_t kLdsCap = NT * 304;
    __shared__ uint4 tile[kLdsCap / 16];
    __shared__ uint64_t tb[2];
    const uint8_t *lds = (const uint8_t *)tile;
    // Tile window = [first record, next tile's first record); only a cache: every record is checked
    // against it and parsed from global memory when it is not inside.  The window bounds (thread 0)
    // and each thread's record offset for tile t+1 are loaded while tile t's LDS-DMA is in flight,
    // so no tile starts with a dependent global-load round trip.
    auto window = [&](uint64_t r0, uint64_t &wb0, uint64_t &wb1) {
        const uint64_t r1 = (a.n - r0) < kTileRecs ? a.n : r0 + kTileRecs;
        wb0 = a.off[r0] & ~15ull;
        uint64_t e;
        if (r1 < a.n) {
            e = a.off[r1];
        } else {
            const uint64_t last = a.off[r1 - 1];
            e = last + 4 + oge_ldu32(a.recs + last);
        }
        wb1 = (e > wb0 && e - wb0 <= kLdsCap) ? e : wb0;  // empty window: parse from global
    };
    const uint64_t stride = (uint64_t)gridDim.x * kTileRecs;
    uint64_t r0 = (uint64_t)blockIdx.x * kTileRecs;
    uint64_t wb0 = 0, wb1 = 0, my_off = 0;
    uint64_t kor = 0, knot = 0;  // this thread's keys' OR and OR of complements (a.keyred)
    uint64_t dv0 = 0, dv1 = 0;   // this thread's fragment deviation maxima (a.cf_dev)
    if (r0 < a.n) {
        if (threadIdx.x == 0) window(r0, wb0, wb1);
        if (r0 + threadIdx.x < a.n) my_off = a.off[r0 + threadIdx.x];
    }
    for (; r0 < a.n; r0 += stride) {
        const uint64_t r1 = (a.n - r0) < kTileRecs ? a.n : r0 + kTileRecs;
        if (threadIdx.x == 0) {
            tb[0] = wb0;
            tb[1] = wb1;
        }
        __syncthreads();
        const uint64_t b0 = tb[0], b1 = tb[1];
        const uint64_t nch = (b1 - b0 + 15) >> 4;
        const uint4 *g = (const uint4 *)(a.recs + b0);
        // LDS-DMA: every chunk load of the tile in flight at once, no VGPR round trip
        const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        for (uint64_t c0 = (uint64_t)wv * 64; c0 < nch; c0 += NT)
            if (c0 + ln < nch)
                __builtin_amdgcn_global_load_lds((const void *)(g + c0 + ln),
                                                 (__attribute__((address_space(3))) void *)(tile + c0), 16, 0, 0);
        const uint64_t o = my_off;
        const uint64_t n0 = r0 + stride;
        if (n0 < a.n) {  // next tile's window and offsets, overlapping this tile's loads
            if (threadIdx.x == 0) window(n0, wb0, wb1);
            if (n0 + threadIdx.x < a.n) my_off = a.off[n0 + threadIdx.x];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint64_t i = r0 + threadIdx.x;
        if (i < r1) {
            const uint32_t bs = (o >= b0 && o + 4 <= b1) ? LdsRd{lds}.u32(o - b0) : 0u;
            if (bs && o + 4 + bs <= b1) parse_input<META, KEYS>(LdsRd{lds}, o - b0, i, o, a, kor, knot, dv0, dv1);
            else parse_input<META, KEYS>(GlbRd{a.recs}, o, i, o, a, kor, knot, dv0, dv1);
        }
        __syncthreads();
    }
    if (META && KEYS && a.cf_dev) md_dev_slots(dv0, dv1, a.cf_dev);
    if (KEYS && a.keyred) {  // a wave's OR, then one atomic per wave and word
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) kor |= __shfl_xor(kor, d, 64), knot |= __shfl_xor(knot, d, 64);
        if ((threadIdx.x & 63) == 0) {
            if (kor) atomicOr(&a.keyred[0], (unsigned long long)kor);
            if (knot) atomicOr(&a.keyred[1], (unsigned long long)knot);
            if (blockIdx.x == 0 && threadIdx.x == 0) a.bad[1] = 1u;
        }
    }
}

// ---------------------------------------------------------------- gather
__device__ __forceinline__ uint4 ldu128(const uint8_t *p) { return *(const uint4 *)p; }

// bytes [o, o + 16) of the 32-byte string t ++ h (1 <= o <= 15)
__device__ __forceinline__ uint4 funnel16(uint4 t, uint4 h, int o) {
    const uint64_t W0 = ((uint64_t)t.y << 32) | t.x, W1 = ((uint64_t)t.w << 32) | t.z;
    const uint64_t W2 = ((uint64_t)h.y << 32) | h.x, W3 = ((uint64_t)h.w << 32) | h.z;
    const uint32_t sh = 8u * (uint32_t)o;  // 8..120
    const bool hi = sh >= 64;
    const uint32_t r = sh & 63;
    const uint64_t a0 = hi ? W1 : W0, a1 = hi ? W2 : W1, a2 = hi ? W3 : W2;
    const uint64_t q0 = r ? (a0 >> r) | (a1 << (64 - r)) : a0;
    const uint64_t q1 = r ? (a1 >> r) | (a2 << (64 - r)) : a1;
    return make_uint4((uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32));
}

__device__ __forceinline__ void set_byte(uint4 &v, int pos, uint32_t byte) {
    const uint32_t sh = 8 * (pos & 3), mk = ~(0xffu << sh), bv = byte << sh;
    switch (pos >> 2) {
    case 0: v.x = (v.x & mk) | bv; break;
    case 1: v.y = (v.y & mk) | bv; break;
    case 2: v.z = (v.z & mk) | bv; break;
    default: v.w = (v.w & mk) | bv; break;
    }
}

// bytes 14,15 (bin) and 19 (FLAG high byte) of a record starting at `rs` (relative), chunk at `rel`
__device__ __forceinline__ void patch_chunk(uint4 &v, int64_t rel, int64_t rs, uint32_t bf) {
    const int64_t p14 = rs + 14 - rel, p19 = rs + 19 - rel;
    if (p14 >= 0 && p14 < 16) set_byte(v, (int)p14, bf & 0xff);
    if (p14 + 1 >= 0 && p14 + 1 < 16) set_byte(v, (int)(p14 + 1), (bf >> 8) & 0xff);
    if (p19 >= 0 && p19 < 16) set_byte(v, (int)p19, (bf >> 16) & 0xff);
}

__device__ __forceinline__ uint32_t patch_byte(uint64_t ro, uint32_t byte, uint32_t bf) {
    if (ro == 14) return bf & 0xff;
    if (ro == 15) return (bf >> 8) & 0xff;
    if (ro == 19) return (bf >> 16) & 0xff;
    return byte;
}

// Where output chunk A (16-byte aligned, relative position rel = A - D0 in the wave's batch) reads
// from: record k of the batch at byte src of its source, or -- when a record boundary falls inside
// the chunk (two) -- the last 16 bytes of record k (src = its length - 16) and the first 16 of k+1.
struct GChunk {
    int k;
    bool full, two;
    int64_t rel, rs;
    uint64_t src;
};
__device__ __forceinline__ GChunk gchunk_plan(const uint32_t *sdw, uint32_t cnt, uint64_t A, uint64_t D0, uint64_t Dend) {
    GChunk g;
    g.rel = (int64_t)A - (int64_t)D0;
    const int64_t x0 = g.rel < 0 ? 0 : g.rel;
    int lo = 0, hi = (int)cnt - 1;  // record holding byte x0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int64_t)sdw[mid] <= x0) lo = mid; else hi = mid - 1;
    }
    g.k = lo;
    g.rs = sdw[lo];
    g.full = g.rel >= 0 && A + 16 <= Dend;
    g.two = (lo + 1 < (int)cnt) && (int64_t)sdw[lo + 1] < g.rel + 16;
    g.src = g.two ? (uint64_t)((int64_t)sdw[lo + 1] - g.rs) - 16 : (uint64_t)(g.rel - g.rs);
    return g;
}

// MODE 0: source = off[perm[k]], bin/flags parsed from the record; 1: from the output-order summaries
// (smeta) and dup[]; 2: from the 8-byte descriptors (desc); 3: from k_cand_frag's descriptors and dup[]
// (r06: the dedup's apply pass folded in here), the primaries flagged counted into a.ndup.
template <int MODE>
__global__ __launch_bounds__(kT) void k_gather16(OgePassArgs a) {
    uint32_t nd = 0;  // MODE 3: flagged primaries of this lane's records
    __shared__ uint32_t sd[kT / 64][65];   // per wave: output start of record j relative to the batch
    __shared__ uint64_t ss[kT / 64][64];   // source offset of record j
    __shared__ uint32_t sbf[kT / 64][64];  // bin | FLAG-high-byte << 16 to write
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t wave = ((uint64_t)blockIdx.x * kT + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * kT) >> 6;
    for (uint64_t R = wave * 64; R < a.n; R += nwaves * 64) {
        const uint32_t cnt = (uint32_t)((a.n - R) < 64 ? (a.n - R) : 64);
        const uint64_t D0 = a.out_off[R];
        if (lane < cnt) {
            const uint64_t rec = R + lane;
            const uint64_t d = a.out_off[rec];
            if (lane == cnt - 1) sd[w][cnt] = (uint32_t)(a.out_off[rec + 1] - D0);
            uint64_t s;
            uint32_t bin, fhi;
            bool primary;
            if (MODE == 2) {
                const uint64_t D = a.desc[rec];
                s = D & ((1ull << 40) - 1);
                bin = (uint32_t)(D >> 40) & 0xffff;
                fhi = (uint32_t)(D >> 56);
                primary = false;  // 0x400 already applied in the descriptor
            } else if (MODE == 3) {
                const uint64_t D = a.desc[rec];
                s = D & ((1ull << 39) - 1);
                bin = (uint32_t)(D >> 40) & 0xffff;
                fhi = (uint32_t)(D >> 56);
                primary = false;  // applied here, not below
                if ((D >> 39) & 1) {
                    const bool d = a.dup[rec] == 1;
                    fhi = d ? (fhi | 0x04u) : (fhi & ~0x04u);
                    nd += d;
                }
            } else if (MODE == 1) {
                const RecMeta M = a.smeta[rec];
                s = M.src;
                bin = (uint32_t)(M.m >> 48);
                fhi = (uint32_t)(M.m >> 40) & 0xff;
                primary = (M.m & OGE_M_PRIMARY) != 0;
            } else {
                s = a.off[a.perm ? a.perm[rec] : rec];
                const uint8_t *r = a.recs + s;
                const int32_t pos = (int32_t)oge_ldu32(r + OGE_OFF_POS);
                const uint32_t w16 = oge_ldu32(r + OGE_OFF_NCIGAR);
                const uint32_t nc = w16 & 0xFFFF, flag = w16 >> 16;
                const uint8_t *cg = r + OGE_OFF_NAME + r[OGE_OFF_LNAME];
                int32_t rl = 0;
                for (uint32_t k = 0; k < nc; ++k) {
                    const uint32_t op = oge_ldu32(cg + 4 * k), t = op & 0xF;
                    if (t == OGE_CIG_M || t == OGE_CIG_D || t == OGE_CIG_N || t == OGE_CIG_EQ || t == OGE_CIG_X) rl += (int32_t)(op >> 4);
                }
                bin = oge_reg2bin(pos, pos + rl);
                fhi = flag >> 8;
                primary = !(flag & OGE_F_SECONDARY);
            }
            if (a.dup && primary) fhi = a.dup[rec] == 1 ? (fhi | 0x04u) : (fhi & ~0x04u);
            sd[w][lane] = (uint32_t)(d - D0);
            ss[w][lane] = s;
            sbf[w][lane] = (bin & 0xffff) | (fhi << 16);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t Dend = D0 + sd[w][cnt];
        for (uint64_t A = (D0 & ~15ull) + 16ull * lane; A < Dend; A += 1024) {
            const GChunk g = gchunk_plan(sd[w], cnt, A, D0, Dend);
            if (g.full) {
                uint4 v = ldu128(a.recs + ss[w][g.k] + g.src);
                if (g.two) {
                    // the last `keep` bytes of record k and the head of record k+1, each loaded from
                    // inside its own record (no bytes of source neighbours, which would pull in cache
                    // lines no record here needs), funnelled together
                    const int64_t rs2 = sd[w][g.k + 1];
                    const uint4 h = ldu128(a.recs + ss[w][g.k + 1]);
                    v = funnel16(v, h, 16 - (int)(rs2 - g.rel));
                    patch_chunk(v, g.rel, rs2, sbf[w][g.k + 1]);
                }
                patch_chunk(v, g.rel, g.rs, sbf[w][g.k]);
                *(uint4 *)(a.out + A) = v;
            } else {
                // batch edge: bytes shared with neighbouring waves
                const uint64_t xe = (A + 16 < Dend ? A + 16 : Dend) - D0;
                int kk = g.k;
                for (uint64_t x = (uint64_t)(g.rel < 0 ? 0 : g.rel); x < xe; ++x) {
                    while (kk + 1 < (int)cnt && sd[w][kk + 1] <= x) ++kk;
                    const uint64_t ro = x - sd[w][kk];
                    a.out[D0 + x] = (uint8_t)patch_byte(ro, a.recs[ss[w][kk] + ro], sbf[w][kk]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (MODE == 3) {  // a wave's count, one atomic per wave on one of 64 counters
        const uint32_t ws = oge_wave_sum(nd);
        if ((threadIdx.x & 63) == 0 && ws) atomicAdd(a.ndup + (blockIdx.x & 63) * 32, ws);
    }
}

}  // namespace

template <int NT>
static void launch_input_pass(oge_ctx *ctx, const OgePassArgs &a, uint64_t cap) {
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(oge_ceil_div(a.n, NT), cap);
    if (a.meta && a.keys)
        hipLaunchKernelGGL((k_input_pass<true, true, NT>), dim3(blocks), dim3(NT), 0, ctx->stream, a);
    else if (a.meta)
        hipLaunchKernelGGL((k_input_pass<true, false, NT>), dim3(blocks), dim3(NT), 0, ctx->stream, a);
    else
        hipLaunchKernelGGL((k_input_pass<false, true, NT>), dim3(blocks), dim3(NT), 0, ctx->stream, a);
}

int oge_input_pass(oge_ctx *ctx, const OgePassArgs &a) {
    if (!a.n || (!a.meta && !a.keys)) return OGE_OK;
    // 256 records (= threads) per block, the grid capped at 2048 blocks (r01: 128 / 64-record tiles,
    // more blocks per CU, measured 34.1 / 28.3 ms against 26.6 ms)
    launch_input_pass<256>(ctx, a, 2048);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

int oge_gather_pass(oge_ctx *ctx, const OgePassArgs &a) {
    if (!a.n) return OGE_OK;
    constexpr uint64_t cap = 131072;  // blocks in flight enough to cover the gather's latency (48 -> 41 ms, r01)
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(oge_ceil_div(a.n, 64 * (kT / 64)), cap);
    if (a.desc && a.ndup)
        hipLaunchKernelGGL(k_gather16<3>, dim3(blocks), dim3(kT), 0, ctx->stream, a);
    else if (a.desc)
        hipLaunchKernelGGL(k_gather16<2>, dim3(blocks), dim3(kT), 0, ctx->stream, a);
    else if (a.smeta)
        hipLaunchKernelGGL(k_gather16<1>, dim3(blocks), dim3(kT), 0, ctx->stream, a);
    else
        hipLaunchKernelGGL(k_gather16<0>, dim3(blocks), dim3(kT), 0, ctx->stream, a);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}
