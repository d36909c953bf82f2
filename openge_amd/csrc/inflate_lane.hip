// inflate_lane.hip -- BGZF inflate with one LANE per block: Huffman decode in phase 1, LZ77 resolved in
// phase 2.  Replaces BgzfInputStream::decompress (openge/src/util/bgzf_input_stream.cpp:65-142: one
// zlib inflate per BGZF block on the pool) -- the same RFC 1951 decode, laid out for wave64.
//
// Why this shape.  A BGZF block is an independent deflate stream of <= 64 KiB whose Huffman decode is
// one long serial chain.  The grouped decoder (inflate.hip, k_inflate_g) runs one chain per 32 lanes,
// so a wave64 instruction advances two blocks.  Here every lane is its own decoder: one wave
// instruction advances 64 blocks, and the per-lane state (64-bit bit buffer, a 32-byte input
// double-buffer in VGPRs, output accumulator) needs no cross-lane traffic.
//
// Phase 1 (k_infl_huff, persistent, 64-lane workgroups, 640 B of LDS per lane = 4 workgroups/CU):
//   each lane decodes symbols of its block.  Literals are written at their output position (8-byte
//   aligned chunks assembled in a register); a match (length L >= 3, distance D) leaves a hole of L
//   bytes whose first three bytes receive the descriptor (L-3, D-1 in 23 bits) and sets the hole's
//   start bit in the block's 65536-bit bitmap.  Decode tables live in the lane's LDS region: a 6-bit
//   direct litlen table and 5-bit direct distance table, plus the canonical-code limits and the
//   sorted symbol lists for longer codes.  Tables are built by the whole wave for one lane at a time
//   (ballot counting, as the lanes reach a new dynamic block), so a lane's table build costs the
//   wave ~hundreds of instructions, not thousands of serial ones.
// Phase 2 (k_infl_lz, one 512-thread workgroup per block): refs[p] = p for every position, then
//   refs[p + j] = p - D + j for every hole; pointer jumping (refs[q] = refs[refs[q]]) in LDS until
//   every position points at a literal (log2 of the copy-chain depth rounds; BAM data: 5-7); the
//   final bytes are gathered from the literal positions, staged in LDS, CRC-32 checked, written out.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bgzf_dev.h"
#include "oge_ctx.h"

namespace {

using namespace oge_bgzf;

enum { E_STORED = 1, E_CODE = 2, E_OVERRUN = 3, E_LEN = 4, E_DIST = 5, E_FAR = 6, E_TYPE = 7, E_PAST = 8, E_SIZE = 9,
       E_TABLE = 10, E_CRC = 11 };

__device__ __forceinline__ void report(uint32_t *err, uint32_t code, uint64_t blk) {
    atomicOr(err, 1u << code);
    atomicMin(err + 1, (uint32_t)min<uint64_t>(blk, 0xffffffffull));
}

// ---------------------------------------------------------------------------- per-lane LDS region
constexpr uint32_t kRegion = 640;
constexpr uint32_t R_LT = 0;      // u16[64]  litlen direct table (6 bits): sym | L << 9, 0 = longer code
                                  // u8[128]  during code-length decoding: CL table (7 bits), sym | L << 5
constexpr uint32_t R_DT = 128;    // u8[32]   distance direct table (5 bits): sym | L << 5
constexpr uint32_t R_LLIM = 160;  // u16[8]   litlen left-justified 15-bit limits, lengths 7..14
constexpr uint32_t R_LLIM15 = 176;  // u16    limit of length 15
constexpr uint32_t R_LIE = 180;   // u32[9]   lengths 7..15: (list index - first code) | end-of-literals << 16
constexpr uint32_t R_DLIM = 224;  // u16[8]   distance limits, lengths 6..13; +16: u16 L=14, +18: u16 L=15
constexpr uint32_t R_DIDX = 244;  // u16[10]  distance lengths 6..15: list index - first code
constexpr uint32_t R_DS = 264;    // u8[32]   distance symbols with codes longer than 5 bits, canonical order
constexpr uint32_t R_LS = 296;    // u8[288]  litlen symbols longer than 6 bits, canonical order (low 8 bits)
constexpr uint32_t R_LENS = 128;  // u8[318]  code lengths while a dynamic header is decoded
constexpr int TBL = 6, TBD = 5;

__constant__ uint8_t kClOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { ST_HDR = 0, ST_CL = 1, ST_SYM = 2, ST_STORED = 3, ST_BCL = 4, ST_BLD = 5, ST_NEXT = 6, ST_DONE = 7 };

// ---------------------------------------------------------------------------- wave-cooperative builds
// Canonical Huffman code (RFC 1951 3.2.2) of one alphabet for lane j's region R, the wave's 64
// lanes holding the lengths of symbols lane, lane+64, ... in len[0..NR).  Direct table of TB bits for
// codes <= TB; codes longer than TB: left-justified limits + list index per length, symbols in
// canonical order.  Returns false for an over-subscribed code.
template <int NR, int TB, bool LIT>
__device__ bool wbuild(uint8_t *R, const uint32_t (&len)[NR], uint32_t n) {
    const uint32_t lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t cnt[16], lo[16];
#pragma unroll
    for (int L = 0; L < 16; ++L) cnt[L] = lo[L] = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int L = 1; L < 16; ++L) {
            const uint32_t c = (uint32_t)__popcll(__ballot(len[r] == (uint32_t)L));
            cnt[L] += c;
            if (r < 4) lo[L] += c;  // litlen symbols < 256
        }
    }
    int left = 1;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
        left = 2 * left - (int)cnt[L];
        if (left < 0) return false;
    }
    uint32_t first[16], offl[16];  // canonical first code; index of the first symbol of length L in the long list
    uint32_t code = 0, ol = 0;
    first[0] = offl[0] = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {
        code = (code + cnt[L - 1]) << 1;
        first[L] = code;
        offl[L] = ol;
        if (L > TB) ol += cnt[L];
    }
    // zero the direct table
    constexpr uint32_t tbytes = LIT ? (2u << TB) : (1u << TB);
    uint32_t *tw = (uint32_t *)(R + (LIT ? R_LT : R_DT));
    if (lane < tbytes / 4) tw[lane] = 0;
    uint32_t run[16];
#pragma unroll
    for (int L = 0; L < 16; ++L) run[L] = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint32_t myL = len[r], s = r * 64 + lane;
        uint32_t rank = 0, fc = 0, ofl = 0;
#pragma unroll
        for (int L = 1; L < 16; ++L) {
            const uint64_t m = __ballot(myL == (uint32_t)L);
            if (myL == (uint32_t)L) rank = run[L] + (uint32_t)__popcll(m & lt), fc = first[L], ofl = offl[L];
            run[L] += (uint32_t)__popcll(m);
        }
        if (myL && s < n) {
            if (myL <= (uint32_t)TB) {
                const uint32_t rev = __builtin_bitreverse32(fc + rank) >> (32 - myL);
                for (uint32_t k = 0; k < (1u << (TB - myL)); ++k) {
                    const uint32_t ix = rev | (k << myL);
                    if (LIT) ((uint16_t *)(R + R_LT))[ix] = (uint16_t)(s | (myL << 9));
                    else R[R_DT + ix] = (uint8_t)(s | (myL << 5));
                }
            } else {
                R[(LIT ? R_LS : R_DS) + ofl + rank] = (uint8_t)s;
            }
        }
    }
    if (lane == 0) {
        if (LIT) {
            uint16_t *lim = (uint16_t *)(R + R_LLIM);
            uint32_t *lie = (uint32_t *)(R + R_LIE);
#pragma unroll
            for (int L = 7; L < 16; ++L) {
                const uint32_t v = (first[L] + cnt[L]) << (15 - L);
                if (L < 15) lim[L - 7] = (uint16_t)v;
                else *(uint16_t *)(R + R_LLIM15) = (uint16_t)min(v, 65535u);
                lie[L - 7] = ((offl[L] - first[L]) & 0xffff) | ((offl[L] + lo[L]) << 16);
            }
        } else {
            uint16_t *lim = (uint16_t *)(R + R_DLIM);
            uint16_t *idx = (uint16_t *)(R + R_DIDX);
#pragma unroll
            for (int L = 6; L < 16; ++L) {
                lim[L - 6] = (uint16_t)min((first[L] + cnt[L]) << (15 - L), 65535u);
                idx[L - 6] = (uint16_t)((offl[L] - first[L]) & 0xffff);
            }
        }
    }
    return true;
}

// code-length code: 19 symbols, lengths 3 bits each packed in clp (symbol s at bits 3s), 7-bit table
__device__ bool wbuild_cl(uint8_t *R, uint64_t clp) {
    const uint32_t lane = threadIdx.x;
    const uint32_t myL = lane < 19 ? (uint32_t)((clp >> (3 * lane)) & 7) : 0;
    uint32_t cnt[8];
#pragma unroll
    for (int L = 0; L < 8; ++L) cnt[L] = L ? (uint32_t)__popcll(__ballot(myL == (uint32_t)L)) : 0;
    int left = 1;
#pragma unroll
    for (int L = 1; L < 8; ++L) {
        left = 2 * left - (int)cnt[L];
        if (left < 0) return false;
    }
    uint32_t code = 0, fc = 0, rank = 0;
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int L = 1; L < 8; ++L) {
        code = (code + cnt[L - 1]) << 1;
        const uint64_t m = __ballot(myL == (uint32_t)L);
        if (myL == (uint32_t)L) fc = code, rank = (uint32_t)__popcll(m & lt);
    }
    uint32_t *tw = (uint32_t *)(R + R_LT);
    if (lane < 32) tw[lane] = 0;
    if (myL) {
        const uint32_t rev = __builtin_bitreverse32(fc + rank) >> (32 - myL);
        for (uint32_t k = 0; k < (1u << (7 - myL)); ++k) R[R_LT + (rev | (k << myL))] = (uint8_t)(lane | (myL << 5));
    }
    return true;
}

// litlen + distance tables of lane j's dynamic (or fixed) block
__device__ bool wbuild_ld(uint8_t *R, uint32_t hlit, uint32_t hdist, bool fixed) {
    const uint32_t lane = threadIdx.x;
    uint32_t ll[5], dl[1];
    // every length is read before anything is written (the lengths share the region with the tables)
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const uint32_t s = r * 64 + lane;
        ll[r] = 0;
        if (s < hlit) ll[r] = fixed ? (s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8) : R[R_LENS + s];
    }
    dl[0] = lane < hdist ? (fixed ? 5u : (uint32_t)R[R_LENS + hlit + lane]) : 0u;
    __builtin_amdgcn_wave_barrier();
    if (!wbuild<5, TBL, true>(R, ll, hlit)) return false;
    return wbuild<1, TBD, false>(R, dl, hdist);
}

// ---------------------------------------------------------------------------- phase 1
__global__ void __launch_bounds__(64) k_infl_huff(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0a,
                                                  const uint64_t *__restrict__ d1a, const uint64_t *__restrict__ uoff, uint64_t b0,
                                                  uint64_t nb, uint8_t *__restrict__ out, uint64_t *__restrict__ bitmap,
                                                  uint32_t *__restrict__ err, uint32_t *__restrict__ trace) {
    extern __shared__ __align__(16) uint8_t smem[];
    const uint32_t lane = threadIdx.x;
    uint8_t *const myR = smem + lane * kRegion;
    const uint64_t stride = (uint64_t)gridDim.x * 64;
    const uintptr_t zend = (uintptr_t)z + zbytes;

    // input: 64-bit bit buffer + two 16-byte chunks (q being consumed, p loaded ahead)
    uint64_t buf = 0;
    uint32_t cnt = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0, p0 = 0, p1 = 0, p2 = 0, p3 = 0, qn = 0;
    uintptr_t cp = 0;
    auto load16 = [&](uintptr_t a, uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3) {
        if (a < zend) {  // a 16-byte aligned chunk holding at least one stream byte never leaves its page
            const uint4 v = *(const uint4 *)a;
            x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
        } else {
            x0 = x1 = x2 = x3 = 0;
        }
    };
    auto refill = [&]() {
        if (cnt <= 32) {
            buf |= (uint64_t)q0 << cnt;
            cnt += 32;
            q0 = q1, q1 = q2, q2 = q3;
            if (--qn == 0) {
                q0 = p0, q1 = p1, q2 = p2, q3 = p3, qn = 4;
                load16(cp, p0, p1, p2, p3);
                cp += 16;
            }
        }
    };
    auto skip = [&](uint32_t k) {
        buf >>= k;
        cnt -= k;
    };
    auto get = [&](uint32_t k) {
        const uint32_t v = (uint32_t)buf & ((1u << k) - 1);
        skip(k);
        return v;
    };
    auto bitpos = [&]() -> uint64_t { return (uint64_t)(cp - 16 - 4 * qn) * 8 - cnt; };
    auto seek = [&](uintptr_t a) {  // start reading at byte address a
        const uintptr_t al = a & ~(uintptr_t)15;
        load16(al, q0, q1, q2, q3);
        load16(al + 16, p0, p1, p2, p3);
        cp = al + 32;
        qn = 4;
        for (uint32_t k = 0; k < (uint32_t)((a - al) >> 2); ++k) q0 = q1, q1 = q2, q2 = q3, --qn;
        buf = 0;
        cnt = 0;
        refill();
        refill();
        skip((uint32_t)(a & 3) * 8);
    };

    // output: 8-byte chunk accumulator; the block's first/last chunk are written byte by byte
    uint8_t *obase = nullptr;
    uint32_t osz = 0, pos = 0;
    uint64_t oc = ~0ull, acc = 0;
    auto flush = [&]() {
        if (oc == ~0ull) return;
        uint8_t *c = (uint8_t *)(oc << 3);
        if (c >= obase && c + 8 <= obase + osz) {
            *(uint64_t *)c = acc;
        } else {
            for (uint32_t k = 0; k < 8; ++k)
                if (c + k >= obase && c + k < obase + osz) c[k] = (uint8_t)(acc >> (8 * k));
        }
    };
    auto put = [&](uint32_t p, uint32_t v) {
        const uintptr_t a = (uintptr_t)(obase + p);
        if ((a >> 3) != oc) {
            flush();
            oc = a >> 3;
            acc = 0;
        }
        acc |= (uint64_t)(v & 0xff) << ((a & 7) * 8);
    };
    // match-start bitmap of the block (1024 words per block of the chunk)
    uint64_t *bmp = nullptr, bm = 0;
    uint32_t bw = 0;
    auto mark = [&](uint32_t p) {
        const uint32_t w = p >> 6;
        if (w != bw) {
            bmp[bw] = bm;
            for (uint32_t k = bw + 1; k < w; ++k) bmp[k] = 0;
            bm = 0;
            bw = w;
        }
        bm |= 1ull << (p & 63);
    };

    uint32_t st = ST_NEXT, fin = 0, hlit = 0, hdist = 0, ci = 0, prev = 0, srem = 0, fixed = 0;
    uint64_t clp = 0, b = b0 + lane + (uint64_t)blockIdx.x * 64, d1bit = 0;
    bool first = true;

    auto fail = [&](uint32_t code) {
        report(err, code, b);
        st = ST_NEXT;
    };
    auto block_end = [&]() {  // last deflate block of the BGZF block consumed
        if (pos != osz) return fail(E_SIZE);
        if (bitpos() > d1bit) return fail(E_PAST);
        flush();
        bmp[bw] = bm;
        for (uint32_t k = bw + 1; k < (osz + 63) >> 6; ++k) bmp[k] = 0;
        st = ST_NEXT;
    };

    for (;;) {
        // ---- table builds, the whole wave for one lane at a time
        uint64_t need = __ballot(st == ST_BCL || st == ST_BLD);
        while (need) {
            const uint32_t j = (uint32_t)__builtin_ctzll(need);
            need &= need - 1;
            uint8_t *Rj = smem + j * kRegion;
            const uint32_t sj = __builtin_amdgcn_readlane(st, j);
            bool ok;
            if (sj == ST_BCL) {
                // readlane returns int: go through uint32_t so the low word is not sign-extended
                const uint64_t c = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)clp, j) |
                                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(clp >> 32), j) << 32);
                ok = wbuild_cl(Rj, c);
                if (trace && lane == j && b == 0) {  // debug: the CL table and lengths of block 0
                    uint32_t *d = trace + 1 + 4 * 200000;
                    d[0] = (uint32_t)c, d[1] = (uint32_t)(c >> 32), d[2] = ok;
                    for (int k = 0; k < 32; ++k) d[3 + k] = ((const uint32_t *)Rj)[k];
                }
                if (lane == j) {
                    if (ok) st = ST_CL, ci = 0, prev = 0;
                    else fail(E_TABLE);
                }
            } else {
                ok = wbuild_ld(Rj, __builtin_amdgcn_readlane(hlit, j), __builtin_amdgcn_readlane(hdist, j),
                               __builtin_amdgcn_readlane(fixed, j) != 0);
                if (lane == j) {
                    if (ok) st = ST_SYM;
                    else fail(E_TABLE);
                }
            }
        }
        // ---- next block for lanes that finished theirs
        if (st == ST_NEXT) {
            if (!first) b += stride;
            first = false;
            if (b >= b0 + nb) {
                st = ST_DONE;
            } else {
                obase = out + uoff[b];
                osz = (uint32_t)(uoff[b + 1] - uoff[b]);
                pos = 0;
                oc = ~0ull;
                acc = 0;
                bmp = bitmap + (b - b0) * 1024;
                bm = 0;
                bw = 0;
                d1bit = ((uint64_t)(uintptr_t)z + d1a[b]) * 8;
                seek((uintptr_t)z + d0a[b]);
                st = ST_HDR;
            }
        }
        if (__ballot(st != ST_DONE) == 0) break;

        if (st == ST_SYM) {
            refill();
            const uint32_t v = (uint32_t)buf;
            uint32_t e = ((const uint16_t *)(myR + R_LT))[v & ((1u << TBL) - 1)];
            uint32_t sym, L;
            if (e) {
                sym = e & 511, L = e >> 9;
            } else {  // code longer than TBL bits: canonical limits
                const uint32_t c15 = __builtin_bitreverse32(v) >> 17;
                const uint4 lm = *(const uint4 *)(myR + R_LLIM);
                L = 7 + (c15 >= (lm.x & 0xffff)) + (c15 >= (lm.x >> 16)) + (c15 >= (lm.y & 0xffff)) + (c15 >= (lm.y >> 16)) +
                    (c15 >= (lm.z & 0xffff)) + (c15 >= (lm.z >> 16)) + (c15 >= (lm.w & 0xffff)) + (c15 >= (lm.w >> 16));
                const uint32_t lie = ((const uint32_t *)(myR + R_LIE))[L - 7];
                const uint32_t k = ((lie & 0xffff) + (c15 >> (15 - L))) & 0xffff;
                sym = myR[R_LS + min(k, 287u)] + (k >= (lie >> 16) ? 256u : 0u);
                if (L == 15 && c15 >= *(const uint16_t *)(myR + R_LLIM15)) sym = 512;  // no such code
            }
            skip(L);
            if (trace && b == 0 && trace[0] < 200000) {  // debug: symbol trace of block 0
                const uint32_t k = trace[0]++;
                trace[1 + 4 * k] = pos, trace[2 + 4 * k] = sym, trace[3 + 4 * k] = L, trace[4 + 4 * k] = (uint32_t)(bitpos() - ((uint64_t)(uintptr_t)z + d0a[0]) * 8);
            }
            if (sym < 256) {
                if (pos >= osz) {
                    fail(E_OVERRUN);
                } else {
                    put(pos, sym);
                    ++pos;
                }
            } else if (sym == 256) {
                if (fin) block_end();
                else st = ST_HDR;
            } else if (sym > 285) {
                fail(sym == 512 ? E_CODE : E_LEN);
            } else {
                const uint32_t c = sym - 257;
                const uint32_t ext = c < 8 ? 0u : c < 28 ? (c - 4) >> 2 : 0u;
                const uint32_t base = c < 8 ? c + 3 : c < 28 ? ((4 + (c & 3)) << ext) + 3 : 258u;
                const uint32_t len = base + get(ext);
                refill();
                const uint32_t w = (uint32_t)buf;
                const uint32_t de = myR[R_DT + (w & ((1u << TBD) - 1))];
                uint32_t ds, DL;
                if (de) {
                    ds = de & 31, DL = de >> 5;
                } else {
                    const uint32_t c15 = __builtin_bitreverse32(w) >> 17;
                    const uint4 lm = *(const uint4 *)(myR + R_DLIM);
                    const uint32_t l1415 = *(const uint32_t *)(myR + R_DLIM + 16);
                    DL = 6 + (c15 >= (lm.x & 0xffff)) + (c15 >= (lm.x >> 16)) + (c15 >= (lm.y & 0xffff)) + (c15 >= (lm.y >> 16)) +
                         (c15 >= (lm.z & 0xffff)) + (c15 >= (lm.z >> 16)) + (c15 >= (lm.w & 0xffff)) + (c15 >= (lm.w >> 16)) +
                         (c15 >= (l1415 & 0xffff));
                    const uint32_t k = (((const uint16_t *)(myR + R_DIDX))[DL - 6] + (c15 >> (15 - DL))) & 0xffff;
                    ds = myR[R_DS + min(k, 31u)];
                    if (DL == 15 && c15 >= (l1415 >> 16)) ds = 31;  // no such code
                }
                skip(DL);
                if (ds >= 30) {
                    fail(E_DIST);
                } else {
                    const uint32_t dext = ds < 4 ? 0u : (ds - 2) >> 1;
                    const uint32_t dist = (ds < 4 ? ds + 1 : ((2 + (ds & 1)) << dext) + 1) + get(dext);
                    if (dist > pos || pos + len > osz) {
                        fail(E_FAR);
                    } else {
                        const uint32_t d = (len - 3) | ((dist - 1) << 8);  // descriptor in the hole's first bytes
                        put(pos, d);
                        put(pos + 1, d >> 8);
                        put(pos + 2, d >> 16);
                        mark(pos);
                        pos += len;
                    }
                }
            }
        } else if (st == ST_CL) {
            refill();
            const uint32_t e = myR[R_LT + ((uint32_t)buf & 127)];
            const uint32_t s = e & 31, L = e >> 5;
            skip(L);
            const uint32_t total = hlit + hdist;
            if (trace && b == 0 && trace[0] < 200000) {
                const uint32_t k = trace[0]++;
                trace[1 + 4 * k] = 0x80000000u | ci, trace[2 + 4 * k] = e, trace[3 + 4 * k] = (uint32_t)buf, trace[4 + 4 * k] = total;
            }
            uint32_t rep = 1, val = s;
            if (!e) {
                fail(E_CODE);
            } else {
                if (s == 16) rep = 3 + get(2), val = prev;
                else if (s == 17) rep = 3 + get(3), val = 0;
                else if (s == 18) rep = 11 + get(7), val = 0;
                if ((s == 16 && ci == 0) || ci + rep > total) {
                    fail(E_TABLE);
                } else {
                    for (uint32_t k = 0; k < rep; ++k) myR[R_LENS + ci + k] = (uint8_t)val;
                    prev = val;
                    ci += rep;
                    if (ci == total) {
                        if (myR[R_LENS + 256] == 0) fail(E_TABLE);
                        else st = ST_BLD;
                    }
                }
            }
        } else if (st == ST_HDR) {
            refill();
            const uint32_t h = get(3);
            fin = h & 1;
            const uint32_t type = h >> 1;
            if (type == 0) {
                skip((8 - (uint32_t)(bitpos() & 7)) & 7);
                refill();
                const uint32_t len = get(16), nlen = get(16);
                if ((len ^ 0xffffu) != nlen) fail(E_STORED);
                else if (pos + len > osz) fail(E_OVERRUN);
                else srem = len, st = ST_STORED;
            } else if (type == 1) {
                fixed = 1, hlit = 288, hdist = 30, st = ST_BLD;
            } else if (type == 2) {
                hlit = get(5) + 257;
                hdist = get(5) + 1;
                const uint32_t hclen = get(4) + 4;
                if (hlit > 286 || hdist > 30) {
                    fail(E_TABLE);
                } else {
                    clp = 0;
#pragma unroll
                    for (int i = 0; i < 19; ++i) {
                        if ((uint32_t)i < hclen) {
                            refill();
                            clp |= (uint64_t)get(3) << (3 * kClOrd[i]);
                        }
                    }
                    fixed = 0;
                    st = ST_BCL;
                }
            } else {
                fail(E_TYPE);
            }
        } else if (st == ST_STORED) {
            refill();
            const uint32_t k = min(srem, 4u);
            for (uint32_t i = 0; i < k; ++i) put(pos + i, get(8));
            pos += k;
            srem -= k;
            if (!srem) {
                if (fin) block_end();
                else st = ST_HDR;
            }
        }
    }
}

// ---------------------------------------------------------------------------- phase 2
constexpr uint32_t kT2 = 512;

__global__ void __launch_bounds__(kT2) k_infl_lz(uint8_t *__restrict__ out, const uint64_t *__restrict__ uoff,
                                                 const uint32_t *__restrict__ crc, const uint64_t *__restrict__ bitmap,
                                                 uint64_t b0, const uint32_t *__restrict__ zpow, uint32_t *__restrict__ err) {
    __shared__ __align__(16) uint16_t refs[kSlot + 16];  // after resolution: the block's bytes, right-aligned
    __shared__ uint32_t crctab[4][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t crcs[kT2];
    const uint32_t t = threadIdx.x;
    const uint64_t b = b0 + blockIdx.x;
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint8_t *const O = out + uoff[b];
    if (osz > kSlot) {
        if (t == 0) report(err, E_SIZE, b);
        return;
    }
    if (crc) crc_setup<kT2>(crctab, zp, zpow, t);
    // 1. every position its own source
    const uint32_t q0 = 128 * t;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t p = q0 + 8 * k;
        uint4 v;
        v.x = p | ((p + 1) << 16), v.y = (p + 2) | ((p + 3) << 16), v.z = (p + 4) | ((p + 5) << 16), v.w = (p + 6) | ((p + 7) << 16);
        *(uint4 *)(refs + p) = v;
    }
    __syncthreads();
    // 2. holes: refs[p + j] = p - D + j
    const uint64_t *bmp = bitmap + (b - b0) * 1024;
    const uint32_t nw = (osz + 63) >> 6;
    for (uint32_t w = 2 * t; w < 2 * t + 2 && w < nw; ++w) {
        uint64_t m = bmp[w];
        while (m) {
            const uint32_t p = 64 * w + (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t d = O[p] | ((uint32_t)O[p + 1] << 8) | ((uint32_t)O[p + 2] << 16);
            const uint32_t len = (d & 0xff) + 3, dist = (d >> 8) + 1;
            const uint32_t e = min(p + len, osz);  // phase 1 checked it; a failed block must not write past the array
            for (uint32_t j = p; j < e; ++j) refs[j] = (uint16_t)(j - dist);
        }
    }
    __syncthreads();
    // 3. pointer jumping until every position names a literal
    const uint32_t qe = min(q0 + 128, osz);
    for (int round = 0; round < 20; ++round) {
        int changed = 0;
        for (uint32_t q = q0; q < qe; q += 8) {
            const uint4 v = *(const uint4 *)(refs + q);
            const uint32_t r8[8] = {v.x & 0xffff, v.x >> 16, v.y & 0xffff, v.y >> 16, v.z & 0xffff, v.z >> 16, v.w & 0xffff, v.w >> 16};
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                if (q + i < qe && r8[i] != q + i) {
                    const uint32_t rr = refs[r8[i]];
                    if (rr != r8[i]) refs[q + i] = (uint16_t)rr, changed = 1;
                }
            }
        }
        if (!__syncthreads_or(changed)) break;
    }
    // 4. final bytes of [q0, q0 + 128): literal-filled bytes (aligned dword loads, funnel-shifted),
    //    holes gathered from their literal sources
    uint32_t wv[32];
    {
        const uintptr_t a = (uintptr_t)(O + q0);
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t *W = (const uint32_t *)(a & ~(uintptr_t)3);
        const uintptr_t lim = (uintptr_t)(O + osz);  // a dword starting below lim holds a block byte: readable
        uint32_t raw[33];
#pragma unroll
        for (int k = 0; k < 33; ++k) raw[k] = (uintptr_t)(W + k) < lim ? W[k] : 0u;
#pragma unroll
        for (int k = 0; k < 32; ++k) wv[k] = sh ? __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh) : raw[k];
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t q = q0 + 4 * k;
        if (q >= qe) break;
        const uint2 rv = *(const uint2 *)(refs + q);
        const uint32_t r4[4] = {rv.x & 0xffff, rv.x >> 16, rv.y & 0xffff, rv.y >> 16};
        uint32_t x = wv[k];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (q + i < qe && r4[i] != q + i) x = (x & ~(0xffu << (8 * i))) | ((uint32_t)O[min(r4[i], osz - 1)] << (8 * i));
        wv[k] = x;
    }
    __syncthreads();  // refs no longer read: the region becomes the byte image
    // 5. stage the bytes in LDS (crc_window512's layout: byte q at img + q), CRC, write out
    uint8_t *img = (uint8_t *)refs;
#pragma unroll
    for (int k = 0; k < 32; ++k)
        if (q0 + 4 * k < osz) *(uint32_t *)(img + q0 + 4 * k) = wv[k];
    __syncthreads();
    if (crc) {
        const uint32_t c = crc_window512((const uint32_t *)img, osz, crctab, zp, crcs, t);
        if (t == 0 && c != crc[b]) report(err, E_CRC, b);
    }
    const uint32_t sh = (uint32_t)((uintptr_t)O & 3);
    uint32_t *A = (uint32_t *)((uintptr_t)O & ~(uintptr_t)3);
    const uint32_t nwords = (osz + sh + 3) / 4;
    for (uint32_t g = t; g < nwords; g += kT2) {
        const int32_t r0 = (int32_t)(4 * g) - (int32_t)sh;  // relative position of the word's first byte
        if (r0 >= 0 && r0 + 4 <= (int32_t)osz) {
            A[g] = ld32((const uint32_t *)img, (uint32_t)r0);
        } else {
            for (int i = 0; i < 4; ++i) {
                const int32_t r = r0 + i;
                if (r >= 0 && r < (int32_t)osz) ((uint8_t *)(A + g))[i] = img[r];
            }
        }
    }
}

}  // namespace

// Inflate indexed blocks [0, nblk) with the lane decoder; err as in oge_bgzf_inflate_dev (err[0] bits,
// err[1] first failing block).  zpow: the CRC zero operators (device).
int oge_inflate_lanes(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                      const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                      const uint32_t *zpow) {
    static int ncu = [] {
        int d = 0, n = 0;
        hipGetDevice(&d);
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
        return n > 0 ? n : 256;
    }();
    const uint64_t chunk = std::min<uint64_t>(nblk, 262144);
    uint64_t *bitmap = (uint64_t *)ctx->ws("infl_bitmap", chunk * 1024 * 8);
    if (!bitmap) return OGE_ERR_HIP;
    static const bool tr = getenv("OGE_INFLATE_TRACE") != nullptr;
    uint32_t *trace = nullptr;
    if (tr) {
        trace = (uint32_t *)ctx->ws("infl_trace", 4 * (1 + 4 * 200000 + 64));
        hipMemsetAsync(trace, 0, 4, ctx->stream);
    }
    for (uint64_t b0 = 0; b0 < nblk; b0 += chunk) {
        const uint64_t nb = std::min(chunk, nblk - b0);
        const uint32_t g1 = (uint32_t)std::min<uint64_t>((nb + 63) / 64, (uint64_t)ncu * 4);
        k_infl_huff<<<g1, 64, 64 * kRegion, ctx->stream>>>(d_z, zbytes, d0, d1, uoff, b0, nb, out, bitmap, err, b0 ? nullptr : trace);
        OGE_LAUNCH_CHECK(ctx);
        k_infl_lz<<<(uint32_t)nb, kT2, 0, ctx->stream>>>(out, uoff, crc, bitmap, b0, zpow, err);
        OGE_LAUNCH_CHECK(ctx);
    }
    if (tr) {
        hipStreamSynchronize(ctx->stream);
        uint32_t n = 0;
        hipMemcpy(&n, trace, 4, hipMemcpyDeviceToHost);
        std::vector<uint32_t> h(1 + 4 * 200000 + 64);
        hipMemcpy(h.data(), trace, h.size() * 4, hipMemcpyDeviceToHost);
        if (FILE *f = fopen(getenv("OGE_INFLATE_TRACE"), "wb")) fwrite(h.data(), 4, h.size(), f), fclose(f);
    }
    return OGE_OK;
}
