// inflate_lane.hip -- BGZF inflate with one LANE per block: Huffman decode in phase 1, LZ77 resolved in
// phase 2.  Replaces BgzfInputStream::decompress (openge/src/util/bgzf_input_stream.cpp:65-142: one
// zlib inflate per BGZF block on the pool) -- the same RFC 1951 decode, laid out for wave64.
//
// Why this shape.  A BGZF block is an independent deflate stream of <= 64 KiB whose Huffman decode is
// one long serial chain.  Every lane is its own decoder: one wave instruction advances 64 blocks.  A
// lane's decode step is a dependent chain (table lookup -> shift -> next lookup), and a wave executes
// the UNION of its 64 lanes' paths every step (some lane is nearly always on each rare path: a long
// code, a match, a long distance code), so the rare paths must be cheap and must not wait on memory:
//
//   * Only LDS and registers in the chain.  The hot 6-bit literal/length and 4-bit distance direct
//     tables, the long LENGTH codes' symbols and the long DISTANCE codes' symbols live in LDS
//     (lane-interleaved [entry][lane]: a wave's 64 lookups hit 64 banks); the canonical limits of the
//     longer codes in VGPRs.  A long LITERAL code (7..15 bits: ~7% of BAM literals) needs no symbol to
//     continue the bit stream -- its length comes from the limits and the literal/length split from
//     the code's canonical index -- so phase 1 writes the index (< 256) in place of the byte, marks the
//     position in a second bitmap, and phase 2 translates it through the table's list (written once
//     per table to a per-block area).  r03 looked the symbol up in a per-lane global scratch in the
//     chain: a global load per step that also waited (vmcnt counts stores too) for every output store
//     in flight.
//   * Wave-wide work (table builds, the block queue, the exit test) every kInner steps instead of every
//     step; a lane waiting for it idles at most kInner steps (a few per BGZF block).
//
// Phase 1 (k_infl_huff, persistent 64-lane workgroups): each lane decodes the symbols of its blocks.
//   Literals are written at their output position (8-byte chunks assembled in a register); a match
//   (length L >= 3, distance D) leaves a hole of L bytes whose first three bytes receive the
//   descriptor (L-3, D-1 in 23 bits) and sets the hole's start bit in the block's bitmap.
// Phase 2 (k_infl_lz, persistent 1024-thread workgroups, one block at a time, the next block's bytes loaded
//   under this block's CRC): deferred literals translated; refs[p] = p for
//   every position, then refs[p + j] = p - D + j for every hole; pointer jumping (three hops per round,
//   refs[q] = refs[refs[refs[refs[q]]]], chunks retired by a root test) in LDS until every position points
//   at a literal; the block's bytes are then staged in LDS, every
//   byte gathered from its root, CRC-32 checked and written out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

#include "bgzf_dev.h"
#include "oge_ctx.h"

namespace {

using namespace oge_bgzf;

__device__ __forceinline__ void report(uint32_t *err, uint32_t code, uint64_t blk) {
    atomicOr(err, 1u << code);
    atomicMin(err + 1, (uint32_t)min<uint64_t>(blk, 0xffffffffull));
}

constexpr int TL = 6, TD = 4;  // direct-table bits: literal/length, distance
constexpr int kWps = 3;        // waves per SIMD (VGPR budget 512 / 3)
#ifndef OGE_INFL_STREAMS
#define OGE_INFL_STREAMS 1
#endif
#ifndef OGE_INFL_CHUNK
#define OGE_INFL_CHUNK 4
#endif
constexpr int kStreams = OGE_INFL_STREAMS;     // chunk pipelines (see oge_inflate_lanes)
constexpr uint64_t kChunkLanes = OGE_INFL_CHUNK;  // blocks per lane per chunk, at most
#ifndef OGE_INFL_LB
#define OGE_INFL_LB 6
#endif
constexpr int LB = OGE_INFL_LB;  // literals per batch (see the ST_SYM path; 20M reads, LB 3 / 4 / 5 / 6:
                                 // 48.1 / 45.1 / 43.5 / 43.2 ms)
#ifndef OGE_INFL_ITER  // iteration shape (build knob): 0 batch + symbol + batch, 1 symbol + 2 batches, 2 batch +
#define OGE_INFL_ITER 0  // symbol + 2 batches; 20M reads (LB 6): 43.8 / 43.6 / 45.6 ms
#endif
#ifndef OGE_INFL_INNER
#define OGE_INFL_INNER 16
#endif
constexpr int kInner = OGE_INFL_INNER;  // decode steps between the wave-wide phases
constexpr int kNT = 4;         // tables per BGZF block whose long literals phase 2 translates
constexpr uint32_t kXList = 288;                 // a table's canonical list of long codes (bytes)
constexpr uint32_t kXTab = 1280;                 // per block: kNT lists, then kNT u32 start positions
constexpr uint32_t kXStart = kNT * kXList;       // offset of the start positions
constexpr uint32_t kDefer = 0x1000;              // sym: a long literal whose byte phase 2 looks up

// per-wave LDS, lane-interleaved ([entry][lane]): element e of lane l at e * 64 + l.  13,312 bytes: 12
// waves per CU fit the 160 KiB.
struct P1Lds {
    uint16_t lt[1 << TL][64];  // sym | L << 9, 0x100 = longer code (bit 8 set: not a literal, L = 0); while
                                // code lengths are decoded a lane's
                                // column holds its 7-bit code-length table (cl_at): sym | L << 5
    uint8_t dt[1 << TD][64];   // sym | L << 5, 0 = longer code
    uint8_t ll[32][64];        // long length codes (and end of block): symbol - 256, by long-length index
                               // (32: the fixed code's 286 / 287 have codes too)
    uint8_t dl[30][64];        // long distance codes: symbol, by long-distance index
    uint32_t cnt[16], lo[16];  // a build's per-length counts (all / literal symbols)
};
// per-lane global scratch
constexpr uint32_t kScr = 640;
constexpr uint32_t S_LENS = 0;   // u8[320] code lengths of the block being set up (zeroed by the CL build)
constexpr uint32_t S_LS = 320;   // u8[288] the long-code list of a table whose literals are not deferred
constexpr uint32_t S_CLP = 608;  // u64: the code-length code's lengths between a header and its build

__constant__ uint8_t kClOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// entry i (7-bit code) of lane l's code-length table: byte i & 1 of lane l's literal/length entry i >> 1,
// so building one lane's table never touches another lane's column
__device__ __forceinline__ uint32_t cl_at(uint32_t i, uint32_t l) { return ((i >> 1) * 64 + l) * 2 + (i & 1); }

enum { ST_HDR = 0, ST_CL = 1, ST_SYM = 2, ST_STORED = 3, ST_BCL = 4, ST_BLD = 5, ST_NEXT = 6, ST_DONE = 7, ST_LOAD = 8 };

// the slow-path parameters of one lane, in VGPRs (u16 pairs)
struct Slow {
    uint32_t ll[4];   // litlen left-justified 15-bit limits, lengths 7..14
    uint32_t l15;     // limit of length 15
    uint32_t pk[9];   // lengths 7..15: (list index - first code) & 0xffff | end of literals << 16 | long
                      // length codes before this length << 25
    uint32_t dl[6];   // distance limits, lengths 5..15 (slot 11 unused)
    uint32_t di[6];   // distance lengths 5..15: list index - first code
};

// Compile-time loop: f(integral_constant<K>) for K < N.  Register arrays (Slow) must only ever be indexed
// by constants -- a '#pragma unroll' loop still indexes them by a variable when SROA runs, which sends
// the whole array to scratch memory and turns pick() into a scratch load (a global-memory round trip
// per long code).
template <class F, int... K>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, K...>) {
    (f(std::integral_constant<int, K>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
    sfor_(f, std::make_integer_sequence<int, N>{});
}
template <int N>
__device__ __forceinline__ uint32_t pick(const uint32_t (&a)[N], uint32_t i) {  // a[i], i < N, in VGPRs
    uint32_t v = a[0];
    sfor<N>([&](auto k) { v = i == (uint32_t)k() ? a[k()] : v; });
    return v;
}
__device__ __forceinline__ uint32_t u16of(const uint32_t (&a)[6], uint32_t i) {
    return (pick(a, i >> 1) >> ((i & 1) * 16)) & 0xffff;
}
// Slow's fields by flat index (the pre-pass record's order): ll[4] l15 pk[9] dl[6] di[6]
template <int I>
__device__ __forceinline__ void tset(Slow &T, uint32_t v) {
    if constexpr (I < 4) T.ll[I] = v;
    else if constexpr (I == 4) T.l15 = v;
    else if constexpr (I < 14) T.pk[I - 5] = v;
    else if constexpr (I < 20) T.dl[I - 14] = v;
    else T.di[I - 20] = v;
}

// ---------------------------------------------------------------------------- wave-cooperative builds
// Canonical Huffman code (RFC 1951 3.2.2) of one alphabet for lane j, the wave's 64 lanes holding the
// lengths of symbols lane, lane+64, ... in len[0..NR).  Codes <= TB bits go to lane j's column of the
// direct table.  Longer codes, in canonical order (length, then symbol): LIT -- the literal/length
// alphabet -- all of them to `list` (the lane's scratch) and, when `xl` is given and there are at most
// 256 of them (a list index then fits the byte phase 1 writes), to xl (phase 2's translation list); the
// length codes among them also to lane j's column of S.ll.  !LIT (distances): to lane j's column of S.dl.
// Returns lane L's (L < 16) left-justified 15-bit limit in *lim and its list parameters in *pk (see
// Slow), the number of long codes in *nlong; false = over-subscribed code.
template <int NR, int TB, bool LIT>
__device__ bool wbuild(P1Lds &S, uint32_t j, OGE_G uint8_t *list, OGE_G uint8_t *xl, const uint32_t (&len)[NR], uint32_t n,
                       uint32_t *lim, uint32_t *pk, uint32_t *nlong) {
    const uint32_t lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1;
    if (lane < 16) S.cnt[lane] = S.lo[lane] = 0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint32_t L = len[r];
        if (L && r * 64 + lane < n) {
            atomicAdd(&S.cnt[L], 1u);
            if (LIT && r < 4) atomicAdd(&S.lo[L], 1u);  // literal symbols < 256
        }
    }
    __builtin_amdgcn_wave_barrier();
    // lane L: first code, long-list offset, long literals before it, Kraft term of length L
    uint32_t fst = 0, ofl = 0, litb = 0, kraft = 0, c = 0, lo = 0;
    if (lane >= 1 && lane < 16) {
        for (uint32_t l = 1; l < lane; ++l) {
            const uint32_t cl = S.cnt[l];
            fst += cl << (lane - l);
            if (l > (uint32_t)TB) ofl += cl, litb += S.lo[l];
        }
        c = S.cnt[lane];
        lo = S.lo[lane];
        kraft = c << (15 - lane);
    }
    *lim = min((fst + c) << (15 - (lane & 15)), 65535u);
    *pk = ((ofl - fst) & 0xffff) | ((ofl + lo) << 16) | ((ofl - litb) << 25);
    // over-subscribed iff the Kraft sum exceeds 2^15 (every prefix check of RFC 1951 follows from it)
    uint32_t ks = kraft, nl = lane > (uint32_t)TB && lane < 16 ? c : 0u;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) ks += __shfl_xor(ks, d, 64), nl += __shfl_xor(nl, d, 64);
    ks = __builtin_amdgcn_readfirstlane(ks);
    *nlong = __builtin_amdgcn_readfirstlane(nl);
    if (ks > 32768u) return false;
    const bool wx = xl != nullptr && *nlong <= 256;
    for (uint32_t r = lane; r < (1u << TB); r += 64) {  // clear lane j's column of the direct table
        if (LIT) S.lt[r][j] = 0x100;
        else S.dt[r][j] = 0;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t run = 0;  // lane L: symbols of length L placed so far
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint32_t myL = len[r], s = r * 64 + lane;
        const bool mine = myL && s < n;
        const uint32_t src = mine ? myL : 0u;
        const uint32_t base = __shfl(run, src, 64), fc = __shfl(fst, src, 64), ol = __shfl(ofl, src, 64);
        const uint32_t lob = LIT ? __shfl(lo, src, 64) : 0u, lenb = LIT ? __shfl(ofl - litb, src, 64) : 0u;
        uint32_t rank = 0, add = 0;
#pragma unroll
        for (int L = 1; L < 16; ++L) {
            const uint64_t m = __ballot(mine && myL == (uint32_t)L);
            if (myL == (uint32_t)L) rank = (uint32_t)__popcll(m & lt);
            if (lane == (uint32_t)L) add = (uint32_t)__popcll(m);
        }
        run += add;
        if (mine) {
            rank += base;
            if (myL <= (uint32_t)TB) {
                const uint32_t rev = __builtin_bitreverse32(fc + rank) >> (32 - myL);
                for (uint32_t k = 0; k < (1u << (TB - myL)); ++k) {
                    const uint32_t ix = rev | (k << myL);
                    if (LIT) S.lt[ix][j] = (uint16_t)(s | (myL << 9));
                    else S.dt[ix][j] = (uint8_t)(s | (myL << 5));
                }
            } else if (LIT) {
                list[ol + rank] = (uint8_t)s;
                if (wx) xl[ol + rank] = (uint8_t)s;
                if (s >= 256) S.ll[min(lenb + rank - lob, 31u)][j] = (uint8_t)(s - 256);
            } else {
                S.dl[min(ol + rank, 29u)][j] = (uint8_t)s;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// ---------------------------------------------------------------------------- header pre-pass
// k_infl_prep (r06): the FIRST deflate header of every BGZF block starts at a known byte
// (d0), so it is parsed -- block type, code-length code, the code lengths -- and its two tables built by one
// lane per block in a kernel of their own, before phase 1.  Phase 1 then copies a block's ready tables
// into its lane's LDS column (one wave-wide load per lane) instead of running the header, the code-length
// decode (a few hundred decode-loop iterations per block) and two wave-wide builds inside its decode loop.
// Measured before (profiles/r06a/r06b, OGE_EXP=3, 100M reads): the builds were 2.3 % and the iterations
// carrying a code-length lane 4.2 % of a phase-1 wave's cycles -- the lanes of a wave stay in lockstep
// (equal-size BGZF payloads), so those phases mostly coincide.
// Output per block (kPrep bytes, the layout phase 1's copy reads with one 8-byte load per lane): lt image
// (64 u16) | dt (16 B) | ll (32 B) | dl (32 B) | the Slow parameters (26 u32); the long-literal translation
// list into the block's xtab slot 0; pmeta[bi] = prepared (bit 31) | deferred long literals (29) | BFINAL
// (28) | bits from d0 to the first symbol (< 2^24).  Anything unusual -- a stored or invalid first block,
// an over-subscribed code, more than 256 long literal/length codes, a header past the block's end -- leaves
// pmeta = 0 and phase 1 parses that block itself, as before (same results, same error codes).
constexpr uint32_t kPrep = 336;
constexpr uint32_t P_SLOW = 208;  // byte offset of the Slow parameters: ll[4] l15 pk[9] dl[6] di[6]

template <int N>
__device__ __forceinline__ void sadd(uint32_t (&a)[N], uint32_t i, uint32_t v) {  // a[i] += v, a in VGPRs
    sfor<N>([&](auto k) { a[k()] += i == (uint32_t)k() ? v : 0u; });
}

__global__ void __launch_bounds__(64) k_infl_prep(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0a,
                                                  const uint64_t *__restrict__ d1a, uint64_t b0, uint64_t nb,
                                                  uint8_t *__restrict__ prep, uint32_t *__restrict__ pmeta,
                                                  uint8_t *__restrict__ xtab) {
    // per-lane LDS columns ([entry][lane]: a wave's accesses at one entry index hit 64 banks)
    __shared__ uint16_t img[64][64];          // the code-length code's table (bytes, cl_at), then the lt image
    __shared__ uint32_t lens8[40][64];        // code lengths, eight per word: symbol s in nibble s & 7 of word s >> 3
    __shared__ uint8_t sm[16 + 32 + 30][64];  // dt | ll | dl images
    // per length (LDS atomics): count | literal count << 16, then rank (bits 0-8) | the length's code /
    // list base (9-31)
    __shared__ uint32_t cnt[16][64];
    const uint32_t lane = threadIdx.x;
    const uint64_t bi = (uint64_t)blockIdx.x * 64 + lane;
    if (bi >= nb) return;  // no wave-wide operation below
    const uint64_t b = b0 + bi;
    pmeta[bi] = 0;
    const uint64_t a0 = d0a[b], a1 = d1a[b];
    if (a1 <= a0 || a1 > zbytes) return;
    auto len_of = [&](uint32_t s) { return (lens8[s >> 3][lane] >> (4 * (s & 7))) & 15; };
    // bit reader over the block's bytes: 64-bit buffer fed from 16-byte chunks loaded two ahead (a header
    // is ~100-300 bytes: a global round trip per refill was most of this kernel's time)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uintptr_t zend = (uintptr_t)z + zbytes, zlast = (zend - 1) & ~(uintptr_t)15;
    auto load16 = [&](uintptr_t a) { return *(const OGE_G u32x4 *)(a < zend ? a : zlast); };
    const uintptr_t al16 = ((uintptr_t)z + a0) & ~(uintptr_t)15;
    u32x4 q = load16(al16), p1 = load16(al16 + 16), p2 = load16(al16 + 32);
    uintptr_t cp = al16 + 48;
    uint32_t qn = 4;
    for (uint32_t k = 0; k < (uint32_t)((a0 & 15) >> 2); ++k) q.x = q.y, q.y = q.z, q.z = q.w, --qn;
    uint64_t buf = 0;
    uint32_t cn = 0, used = 0;  // used: bits consumed from d0
    auto refill = [&]() {
        while (cn <= 32) {
            buf |= (uint64_t)q.x << cn;
            cn += 32;
            q.x = q.y, q.y = q.z, q.z = q.w;
            if (--qn == 0) {
                q = p1, p1 = p2, qn = 4;
                p2 = load16(cp);
                cp += 16;
            }
        }
    };
    auto get = [&](uint32_t k) {
        const uint32_t v = (uint32_t)buf & ((1u << k) - 1);
        buf >>= k;
        cn -= k;
        used += k;
        return v;
    };
    refill();
    {
        const uint32_t sk = (uint32_t)(a0 & 3) * 8;
        buf >>= sk;
        cn -= sk;
    }
    refill();
    const uint32_t h = get(3), type = h >> 1;
    uint32_t hl, hd;
    if (type == 1) {
        hl = 288, hd = 30;
        for (uint32_t w = 0; w < 40; ++w)
            lens8[w][lane] = w < 18 ? 0x88888888u : w < 32 ? 0x99999999u : w < 35 ? 0x77777777u : w < 36 ? 0x88888888u : 0x55555555u;
    } else if (type == 2) {
        hl = get(5) + 257;
        hd = get(5) + 1;
        const uint32_t hclen = get(4) + 4;
        if (hl > 286 || hd > 30) return;
        uint64_t c = 0;
        for (uint32_t i = 0; i < hclen; ++i) {
            refill();
            c |= (uint64_t)get(3) << (3 * kClOrd[i]);
        }
        // the code-length code: counts, Kraft, canonical codes in symbol order, 7-bit direct table
        uint32_t cl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t s = 0; s < 19; ++s) sadd(cl, (uint32_t)(c >> (3 * s)) & 7, 1);
        int left = 1;
        bool ok = true;
        uint32_t nx[8];
        uint32_t code = 0;
        nx[0] = 0;
        sfor<7>([&](auto k) {
            constexpr int L = decltype(k)::value + 1;
            left = 2 * left - (int)cl[L];
            ok = ok && left >= 0;
            code = (code + (L > 1 ? cl[L - 1] : 0u)) << 1;
            nx[L] = code;
        });
        if (!ok) return;
        uint8_t *clt = (uint8_t *)&img[0][0];
        for (uint32_t i = 0; i < 64; ++i) img[i][lane] = 0;
        for (uint32_t s = 0; s < 19; ++s) {
            const uint32_t L = (uint32_t)(c >> (3 * s)) & 7;
            if (!L) continue;
            const uint32_t cd = pick(nx, L);
            sadd(nx, L, 1);
            const uint32_t rev = __builtin_bitreverse32(cd) >> (32 - L);
            for (uint32_t k = 0; k < (1u << (7 - L)); ++k) clt[cl_at(rev | (k << L), lane)] = (uint8_t)(s | (L << 5));
        }
        // the code lengths (RFC 1951 3.2.7), OR-ed into cleared words (zero runs write nothing)
        for (uint32_t w = 0; w < 40; ++w) lens8[w][lane] = 0;
        const uint32_t total = hl + hd;
        uint32_t ci = 0, prev = 0;
        while (ci < total) {
            refill();
            const uint32_t e = clt[cl_at((uint32_t)buf & 127, lane)];
            if (!e) return;
            get(e >> 5);
            const uint32_t s = e & 31;
            uint32_t rep = 1, val = s;
            if (s == 16) {
                if (ci == 0) return;
                rep = 3 + get(2), val = prev;
            } else if (s == 17) {
                rep = 3 + get(3), val = 0;
            } else if (s == 18) {
                rep = 11 + get(7), val = 0;
            }
            if (ci + rep > total) return;
            if (val)
                for (uint32_t k = 0; k < rep; ++k) {
                    const uint32_t t = ci + k, s2 = t < hl ? t : t - hl + 288;  // distance lengths at 288.. (the fixed layout)
                    atomicOr(&lens8[s2 >> 3][lane], val << (4 * (s2 & 7)));
                }
            prev = val;
            ci += rep;
        }
        if (!len_of(256)) return;  // no end-of-block code
    } else {
        return;  // stored (or invalid) first block: phase 1 handles it
    }
    if ((uint64_t)a0 * 8 + used > (uint64_t)a1 * 8 || used >= (1u << 24)) return;

    // ---- literal/length table (TL-bit direct, long codes by canonical limits): what wbuild<5, TL, true> makes
    uint32_t Slow[26];
    {
        for (uint32_t i = 0; i < 16; ++i) cnt[i][lane] = 0;
        for (uint32_t w = 0; w < (hl + 7) / 8; ++w) {
            const uint32_t x = lens8[w][lane];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                const uint32_t s = 8 * w + i, L = (x >> (4 * i)) & 15;
                if (s < hl && L) atomicAdd(&cnt[L][lane], s < 256 ? 0x10001u : 1u);  // literal symbols counted high
            }
        }
        uint32_t c[16], lo[16];
        sfor<16>([&](auto k) {
            constexpr int L = decltype(k)::value;
            const uint32_t v = L ? cnt[L][lane] : 0u;
            c[L] = v & 0xffff;
            lo[L] = v >> 16;
        });
        uint32_t kraft = 0, nlong = 0;
        sfor<15>([&](auto k) {
            constexpr int L = decltype(k)::value + 1;
            kraft += c[L] << (15 - L);
            if (L > TL) nlong += c[L];
        });
        if (kraft > 32768u || nlong > 256) return;
        uint32_t fst[16], ofl[16], litb[16];
        sfor<16>([&](auto k) {
            constexpr int L = decltype(k)::value;
            uint32_t f = 0, o = 0, lbb = 0;
            sfor<L>([&](auto m) {
                constexpr int l = decltype(m)::value;
                if (l >= 1) {
                    f += c[l] << (L - l);
                    if (l > TL) o += c[l], lbb += lo[l];
                }
            });
            fst[L] = f, ofl[L] = o, litb[L] = lbb;
            // per length: the first code (direct codes) or the list base and the length-code base + 320 (long
            // codes) above a cleared rank
            cnt[L][lane] = (L <= TL ? f : o | ((o - lbb - lo[L] + 320) << 9)) << 9;
        });
        sfor<4>([&](auto k) {
            constexpr int L0 = 7 + 2 * decltype(k)::value, L1 = L0 + 1;
            Slow[decltype(k)::value] = min((fst[L0] + c[L0]) << (15 - L0), 65535u) | (min((fst[L1] + c[L1]) << (15 - L1), 65535u) << 16);
        });
        Slow[4] = min(fst[15] + c[15], 65535u);
        sfor<9>([&](auto k) {
            constexpr int L = 7 + decltype(k)::value;
            Slow[5 + decltype(k)::value] = ((ofl[L] - fst[L]) & 0xffff) | ((ofl[L] + lo[L]) << 16) | ((ofl[L] - litb[L]) << 25);
        });
        for (uint32_t i = 0; i < 64; ++i) img[i][lane] = 0x100;
        for (uint32_t i = 16; i < 78; ++i) sm[i][lane] = 0;  // entries no valid code reaches: deterministic bytes
        OGE_G uint8_t *xl = (OGE_G uint8_t *)(xtab + bi * kXTab);  // table slot 0's translation list
        for (uint32_t w = 0; w < (hl + 7) / 8; ++w) {
            const uint32_t x = lens8[w][lane];
            for (uint32_t i = 0; i < 8; ++i) {
                const uint32_t s = 8 * w + i, L = (x >> (4 * i)) & 15;
                if (s >= hl || !L) continue;
                const uint32_t r = atomicAdd(&cnt[L][lane], 1u), rank = r & 511, inf = r >> 9;
                if (L <= (uint32_t)TL) {
                    const uint32_t rev = __builtin_bitreverse32(inf + rank) >> (32 - L);
                    for (uint32_t k = 0; k < (1u << (TL - L)); ++k) img[rev | (k << L)][lane] = (uint16_t)(s | (L << 9));
                } else {
                    xl[(inf & 511) + rank] = (uint8_t)s;
                    if (s >= 256) sm[16 + min((inf >> 9) + rank - 320, 31u)][lane] = (uint8_t)(s - 256);
                }
            }
        }
    }
    // ---- distance table (TD-bit direct): what wbuild<1, TD, false> makes
    {
        for (uint32_t i = 0; i < 16; ++i) cnt[i][lane] = 0;
        for (uint32_t w = 36; w < 36 + (hd + 7) / 8; ++w) {
            const uint32_t x = lens8[w][lane];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                const uint32_t s = 8 * (w - 36) + i, L = (x >> (4 * i)) & 15;
                if (s < hd && L) atomicAdd(&cnt[L][lane], 1u);
            }
        }
        uint32_t c[16];
        sfor<16>([&](auto k) {
            constexpr int L = decltype(k)::value;
            c[L] = L ? cnt[L][lane] : 0u;
        });
        uint32_t kraft = 0;
        sfor<15>([&](auto k) {
            constexpr int L = decltype(k)::value + 1;
            kraft += c[L] << (15 - L);
        });
        if (kraft > 32768u) return;
        uint32_t lim[16], pk[16];
        sfor<16>([&](auto k) {
            constexpr int L = decltype(k)::value;
            uint32_t f = 0, o = 0;
            sfor<L>([&](auto m) {
                constexpr int l = decltype(m)::value;
                if (l >= 1) {
                    f += c[l] << (L - l);
                    if (l > TD) o += c[l];
                }
            });
            lim[L] = L ? min((f + c[L]) << (15 - L), 65535u) : 0u;
            pk[L] = ((o - f) & 0xffff) | (o << 16) | (o << 25);
            cnt[L][lane] = (L <= TD ? f : o) << 9;
        });
        sfor<6>([&](auto k) {
            constexpr int K = decltype(k)::value;
            Slow[14 + K] = lim[5 + 2 * K] | (K < 5 ? lim[(6 + 2 * K) & 15] << 16 : 0u);
            Slow[20 + K] = (pk[5 + 2 * K] & 0xffff) | (K < 5 ? pk[(6 + 2 * K) & 15] << 16 : 0u);
        });
        for (uint32_t i = 0; i < 16; ++i) sm[i][lane] = 0;
        for (uint32_t s = 0; s < hd; ++s) {
            const uint32_t L = len_of(288 + s);
            if (!L) continue;
            const uint32_t r = atomicAdd(&cnt[L][lane], 1u), rank = r & 511, inf = r >> 9;
            if (L <= (uint32_t)TD) {
                const uint32_t rev = __builtin_bitreverse32(inf + rank) >> (32 - L);
                for (uint32_t k = 0; k < (1u << (TD - L)); ++k) sm[rev | (k << L)][lane] = (uint8_t)(s | (L << 5));
            } else {
                sm[48 + min(inf + rank, 29u)][lane] = (uint8_t)s;
            }
        }
    }
    // ---- the record: lt | dt ll dl | Slow
    OGE_G uint32_t *R = (OGE_G uint32_t *)(prep + bi * kPrep);
    for (uint32_t i = 0; i < 32; ++i) R[i] = (uint32_t)img[2 * i][lane] | ((uint32_t)img[2 * i + 1][lane] << 16);
    for (uint32_t i = 0; i < 20; ++i)
        R[32 + i] = (uint32_t)sm[4 * i][lane] | ((uint32_t)sm[4 * i + 1][lane] << 8) | (4 * i + 2 < 78 ? (uint32_t)sm[4 * i + 2][lane] << 16 : 0u) |
                    (4 * i + 3 < 78 ? (uint32_t)sm[4 * i + 3][lane] << 24 : 0u);
    sfor<26>([&](auto k) { R[P_SLOW / 4 + decltype(k)::value] = Slow[decltype(k)::value]; });
    pmeta[bi] = 0x80000000u | 0x20000000u | ((h & 1) << 28) | used;
}

// ---------------------------------------------------------------------------- phase 1
// An iteration (ST_SYM) decodes up to LB literals from the direct table, then one symbol of any kind (a
// long-code literal, end of block, or a match with its length and distance codes), then up to LB direct
// literals again; every part starts with a refill, which leaves >= 33 bits in the buffer: five direct codes
// take <= 30 bits (a sixth is taken only when its length fits the bits left), a literal/length code + its
// extra bits <= 20, a distance code + its extra bits <= 28.  (r02 commit 3941758 let a batch follow a long code without a refill -- 15 + 3 * 6 = 33 > 32 --
// and corrupted a block at 300M reads; tests/test_gpu_inflate.py::test_long_codes_before_direct_literal_runs
// pins it.)  A wave's iteration count is the maximum over its 64 blocks, and it runs the union of their
// paths, so a lane makes as much progress per iteration as the union costs: C2 BGZF blocks take 11.5k
// iterations of this shape instead of 19.8k one-symbol-or-literal-batch steps (r03).
// Bit-budget guard (always on): every skip of more bits than the buffer holds sets `under`, and the
// block fails with E_BITS instead of decoding from zero bits.
// Output: bytes go through a 64-bit shift register (the newest byte enters at the top) that is stored
// when it holds a whole 8-byte chunk of the output; the block's first and last chunk (shared with the
// neighbouring blocks) are stored byte by byte.  Bitmap words (holes, deferred literals) per 64
// positions, zeroed before the launch, stored when a lane leaves a word that has bits.
// a block's hole / deferred-literal bitmap pairs (1024 x 16 B) at this stride in u64 words (r06: a skew of
// 64 or 512 B per block measured equal, profiles/r06dd)
constexpr uint64_t kBmStride = 2048;

__global__ void __launch_bounds__(64, kWps) k_infl_huff(const uint8_t *__restrict__ z, uint64_t zbytes,
                                                      const uint64_t *__restrict__ d0a, const uint64_t *__restrict__ d1a,
                                                      const uint64_t *__restrict__ uoff, uint64_t b0, uint64_t nb,
                                                      uint8_t *__restrict__ out, uint64_t *__restrict__ bitmap,
                                                      uint8_t *__restrict__ xtab, uint8_t *__restrict__ scratch,
                                                      uint32_t *__restrict__ err, unsigned long long *__restrict__ next,
                                                      const uint8_t *__restrict__ prep, const uint32_t *__restrict__ pmeta) {
    static_assert(LB + 1 < 8, "a batch and the pending literal: fewer bytes than the 8-byte register (put_n shifts < 64)");
    static_assert(sizeof(P1Lds) <= 13312, "12 waves per CU");
    __shared__ P1Lds S;
    const uint32_t lane = threadIdx.x;
    auto scr = [&]() { return (OGE_G uint8_t *)(scratch + ((uint64_t)blockIdx.x * 64 + threadIdx.x) * kScr); };  // lens / list
    const uintptr_t zend = (uintptr_t)z + zbytes;
    const uintptr_t zlast = (zend - 1) & ~(uintptr_t)15;  // the stream's last 16-byte chunk

    // input: 64-bit bit buffer + two 16-byte chunks (q being consumed, p loaded ahead)
    uint64_t buf = 0;
    uint32_t under = 0;  // a skip past the buffered bits happened in this block (the guard)
    // q: the chunk being consumed (q.x next), p: the next chunk, loaded ahead.  Both are 4-register tuples:
    // a load lands in p's own registers (four scalar u32s made the compiler load into a temporary tuple
    // and copy it out at once -- a wait for the load right where it was issued)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 q = {0, 0, 0, 0}, p = {0, 0, 0, 0};
    uint32_t cnt = 0, qn = 0;
    uintptr_t cp = 0;
    // A 16-byte aligned chunk holding at least one stream byte never leaves its page; past the end the
    // last chunk is loaded again (only a corrupt stream reads those bits, and it fails E_PAST / E_BITS).
    // No branch around the load: a value merged after a branch is waited for on the spot, and the
    // prefetch one chunk ahead would wait for its HBM round trip -- and, vmcnt counting stores too, for
    // every output store in flight -- at every fourth refill.
    auto load16 = [&](uintptr_t a) { return *(const OGE_G u32x4 *)(a < zend ? a : zlast); };
#if OGE_EXP == 2  // timing experiment: cycles spent taking the prefetched chunk (its wait) vs the decode loop
    uint64_t x_wait = 0, x_loop = 0, x_steps = 0;
#endif
#if OGE_EXP == 3  // timing experiment: a wave's cycles in the table builds / block taking / decode loop, and
                  // how many of its decode iterations run each state's path (some lane in that state)
    uint64_t y_bld = 0, y_nxt = 0, y_loop = 0, y_clc = 0, y_oc = 0;
    uint32_t y_it = 0, y_cl = 0, y_hdr = 0, y_sto = 0, y_sym = 0, y_nbcl = 0, y_nbld = 0, y_blk = 0;
#endif
    auto refill = [&]() {
        if (cnt <= 32) {
            buf |= (uint64_t)q.x << cnt;
            cnt += 32;
            q.x = q.y, q.y = q.z, q.z = q.w;
            if (--qn == 0) {
#if OGE_EXP == 2
                const uint64_t c0 = __builtin_readcyclecounter();
                q = p, qn = 4;
                __asm__ volatile("" ::"v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w));
                x_wait += __builtin_readcyclecounter() - c0;
#else
                q = p, qn = 4;
                // q takes p's values before the next load is issued, so the load can land in p's registers
                __asm__ volatile("" : "+v"(q.x), "+v"(q.y), "+v"(q.z), "+v"(q.w)::"memory");
#endif
                p = load16(cp);
                cp += 16;
            }
        }
    };
    auto skip = [&](uint32_t k) {
        under |= k > cnt;
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
        q = load16(al);
        p = load16(al + 16);
        cp = al + 32;
        qn = 4;
        for (uint32_t k = 0; k < (uint32_t)((a - al) >> 2); ++k) q.x = q.y, q.y = q.z, q.z = q.w, --qn;
        buf = 0;
        cnt = 0;
        refill();
        refill();
        skip((uint32_t)(a & 3) * 8);
    };

    // output: position q = pos + al from the 8-aligned base ob8; the shift register acc holds the last
    // 8 bytes put (oldest in the low byte), so at a chunk boundary it IS the chunk
    OGE_G uint8_t *ob8 = nullptr;
    uint32_t al = 0, osz = 0, pos = 0, clast = 0;
    uint64_t acc = 0;
    auto store_chunk = [&](uint32_t c, uint64_t v) {  // chunk c (8 bytes at ob8 + 8c) = v
        OGE_G uint64_t *A = (OGE_G uint64_t *)ob8 + c;
        if ((c == 0 && al) || (c == clast && ((al + osz) & 7))) {  // shared with a neighbouring block
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t q = 8 * c + k;
                if (q >= al && q < al + osz) ((OGE_G uint8_t *)A)[k] = (uint8_t)(v >> (8 * k));
            }
        } else {
            *A = v;
        }
    };
    auto put = [&](uint32_t v) {  // one byte at pos
        acc = (acc >> 8) | ((uint64_t)(v & 0xff) << 56);
        const uint32_t q = pos + al + 1;
        ++pos;
        if (!(q & 7)) store_chunk((q >> 3) - 1, acc);
    };
    // n (<= LB + 1) bytes at pos, the first in the low byte of v: one shift-or into the register and at most
    // one chunk store (the batch completes the current chunk when it brings its m missing bytes)
    auto put_n = [&](uint64_t v, uint32_t n) {
        const uint32_t q0 = pos + al, m = 8 - (q0 & 7);
        const uint32_t mm = min(m, (uint32_t)LB + 1), nn = max(n, 1u);  // shifts stay below 64 on the paths not taken
        if (n >= m) store_chunk(q0 >> 3, (acc >> (8 * mm)) | (v << (64 - 8 * mm)));
        if (n) acc = (acc >> (8 * nn)) | (v << (64 - 8 * nn));
        pos += n;
    };
    auto flush_partial = [&]() {  // the chunk holding the last byte put, when it is not complete
        const uint32_t q = pos + al;
        if (q & 7) store_chunk(q >> 3, acc >> (8 * (8 - (q & 7))));
    };
    // Up to LB literals whose codes sit in the direct table (sym < 256: bit 8 of the entry clear).  After
    // the refill >= 33 bits are buffered: five direct codes (<= 30 bits) need no budget check, a sixth or
    // seventh stops the batch when its length exceeds the bits left.
    // Branch-free: the lookup chain (entry -> shift -> next entry) carries only selects, and the batch's
    // bytes go out in one put_n (r04: a put per literal, whose chunk-store branch sat in that chain).
    // np (0 or 1) pending bytes in pb -- the literal of the iteration's main symbol -- go out with the batch
    // r06: go is monotone, so while it holds the k-th literal of the batch is byte k: constant 32-bit shifts
    // into two words instead of a variable 64-bit shift and two selects per literal, the output-room test a
    // compare with the constant k, and the pending byte joined once per batch (100M reads: infl_huff 105.5 ->
    // 98.0 ms)
    auto lit_batch = [&](uint32_t pb, uint32_t np) {
        refill();
        const int32_t room = (int32_t)(osz - pos - np);  // >= 0: pos + np <= osz here
        uint32_t lo = 0, hi = 0, n = 0;
        bool go = true;
#pragma unroll
        for (int k = 0; k < LB; ++k) {
            const uint32_t e2 = S.lt[(uint32_t)buf & ((1u << TL) - 1)][lane];
            go = go && !(e2 & 0x100) && k < room;  // bit 8: a length code, end of block or a longer code
            // a refill guarantees 33 bits: TL * 5 of them; longer batches stop where the buffered bits end
            if (TL * (k + 1) > 32) go = go && (e2 >> 9) <= cnt;  // folded at compile time (k unrolled)
            const uint32_t L = go ? e2 >> 9 : 0u;
            buf >>= L;
            cnt -= L;
            const uint32_t b = go ? (e2 & 0xff) : 0u;
            if (k < 4) lo |= b << (8 * k);
            else hi |= b << (8 * (k - 4));
            n += go;
        }
        const uint64_t batch = (uint64_t)lo | ((uint64_t)hi << 32);
        put_n(np ? (uint64_t)pb | (batch << 8) : batch, n + np);
    };
    // hole and deferred-literal bitmaps of the block (1024 word pairs per block of the chunk)
    uint64_t bm = 0, lm = 0;
    uint32_t bw = 0, bi = 0;  // word, block index in the chunk
    auto word = [&](uint32_t p) {
        const uint32_t w = p >> 6;
        if (w != bw) {
            if (bm | lm) {
                typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
                u64x2 v;
                v.x = bm, v.y = lm;
                *(OGE_G u64x2 *)(bitmap + (uint64_t)bi * kBmStride + 2 * bw) = v;
            }
            bm = lm = 0;
            bw = w;
        }
    };
    // tables built in this block << 1 | the current table's long literals are deferred to phase 2
    uint32_t tabs = 0;

    Slow T;
    sfor<4>([&](auto k) { T.ll[k()] = 0; });
    sfor<9>([&](auto k) { T.pk[k()] = 0; });
    sfor<6>([&](auto k) { T.dl[k()] = T.di[k()] = 0; });
    T.l15 = 0;
    // hl: hlit | hdist << 16; aux: the code-length walk (ci | prev << 16 | l256 << 24) or a stored block's
    // bytes left; flg: the block header's BFINAL (1) and fixed-codes (2) bits
    uint32_t st = ST_NEXT, hl = 0, aux = 0, flg = 0;
    uint32_t b = 0;  // block index (a chunk of a launch holds < 2^32 blocks)

    // a failing block: the lane stops decoding it at once, the error is reported (atomics on err) in the
    // next wave-wide phase, before the lane takes another block -- no atomics inlined into the decode
    // loop at each of its error sites
    uint32_t ferr = 0;
    auto fail = [&](uint32_t code) {
        ferr = code;
        st = ST_NEXT;
    };
    auto block_end = [&]() {  // last deflate block of the BGZF block consumed
        if (under) return fail(E_BITS);
        if (pos != osz) return fail(E_SIZE);
        if (bitpos() > ((uint64_t)(uintptr_t)z + d1a[b]) * 8) return fail(E_PAST);
        flush_partial();
        word(0xffffffffu);
        st = ST_NEXT;
    };

    for (;;) {
        if (ferr) {
            report(err, ferr, b);
            ferr = 0;
        }
        // ---- table builds, the whole wave for one lane at a time
#if OGE_EXP == 3
        const uint64_t y0 = __builtin_readcyclecounter();
        y_nbcl += (uint32_t)__popcll(__ballot(st == ST_BCL));
        y_nbld += (uint32_t)__popcll(__ballot(st == ST_BLD));
#endif
        uint64_t need = __ballot(st == ST_BCL || st == ST_BLD);
        if (need) __threadfence_block();  // lanes' code-length stores before the wave reads them
        while (need) {
            const uint32_t j = (uint32_t)__builtin_ctzll(need);
            need &= need - 1;
            OGE_G uint8_t *sj = (OGE_G uint8_t *)(scratch + ((uint64_t)blockIdx.x * 64 + j) * kScr);
            if (__builtin_amdgcn_readlane(st, j) == ST_BCL) {
                // code-length code: 19 symbols, lengths 3 bits each (symbol s at bits 3s of lane j's clp)
                const uint64_t c = *(const OGE_G uint64_t *)(sj + S_CLP);  // lane j's, stored at its header
                const uint32_t myL = lane < 19 ? (uint32_t)((c >> (3 * lane)) & 7) : 0;
                uint32_t cntl[8];
#pragma unroll
                for (int L = 0; L < 8; ++L) cntl[L] = L ? (uint32_t)__popcll(__ballot(myL == (uint32_t)L)) : 0;
                int left = 1;
                bool ok = true;
#pragma unroll
                for (int L = 1; L < 8; ++L) {
                    left = 2 * left - (int)cntl[L];
                    ok = ok && left >= 0;
                }
                uint32_t code = 0, fc = 0, rank = 0;
                const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
                for (int L = 1; L < 8; ++L) {
                    code = (code + cntl[L - 1]) << 1;
                    const uint64_t m = __ballot(myL == (uint32_t)L);
                    if (myL == (uint32_t)L) fc = code, rank = (uint32_t)__popcll(m & lt);
                }
                uint8_t *cl = (uint8_t *)&S.lt[0][0];
                S.lt[lane][j] = 0;
                __builtin_amdgcn_wave_barrier();
                if (ok && myL) {
                    const uint32_t rev = __builtin_bitreverse32(fc + rank) >> (32 - myL);
                    for (uint32_t k = 0; k < (1u << (7 - myL)); ++k) cl[cl_at(rev | (k << myL), j)] = (uint8_t)(lane | (myL << 5));
                }
                ((OGE_G uint32_t *)(sj + S_LENS))[lane] = 0;  // all 320 bytes: 17/18 runs then need no stores
                if (lane < 16) ((OGE_G uint32_t *)(sj + S_LENS))[64 + lane] = 0;
                if (lane == j) {
                    if (ok) st = ST_CL, aux = 0;
                    else fail(E_TABLE);
                }
            } else {
                const uint32_t hlj = __builtin_amdgcn_readlane(hl, j), hd = hlj >> 16, hl = hlj & 0xffff;
                const bool fx = (__builtin_amdgcn_readlane(flg, j) & 2) != 0;
                const uint32_t nt = __builtin_amdgcn_readlane(tabs, j) >> 1;
                uint32_t ll[5], dl[1];
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    const uint32_t s = r * 64 + lane;
                    ll[r] = 0;
                    if (s < hl) ll[r] = fx ? (s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8) : sj[S_LENS + s];
                }
                dl[0] = lane < hd ? (fx ? 5u : (uint32_t)sj[S_LENS + hl + lane]) : 0u;
                // the long-code list: the lane's scratch, and the block's translation area while it has a
                // free table slot (else the table's long literals are looked up in the chain, as r03 did)
                OGE_G uint8_t *xj = (OGE_G uint8_t *)(xtab + (uint64_t)__builtin_amdgcn_readlane(bi, j) * kXTab);
                uint32_t lim, pk, nlong;
                bool ok = wbuild<5, TL, true>(S, j, sj + S_LS, nt < kNT ? xj + nt * kXList : nullptr, ll, hl, &lim, &pk, &nlong);
                const uint32_t dfr = ok && nt < kNT && nlong <= 256;
                sfor<4>([&](auto k) {
                    const uint32_t v = (uint32_t)__shfl(lim, 7 + 2 * k(), 64) | ((uint32_t)__shfl(lim, 8 + 2 * k(), 64) << 16);
                    if (lane == j) T.ll[k()] = v;
                });
                {
                    const uint32_t v = (uint32_t)__shfl(lim, 15, 64);
                    if (lane == j) T.l15 = v;
                }
                sfor<9>([&](auto k) {
                    const uint32_t v = (uint32_t)__shfl(pk, 7 + k(), 64);
                    if (lane == j) T.pk[k()] = v;
                });
                ok = ok && wbuild<1, TD, false>(S, j, nullptr, nullptr, dl, hd, &lim, &pk, &nlong);
                sfor<6>([&](auto k) {
                    const uint32_t a = (uint32_t)__shfl(lim, 5 + 2 * k(), 64), c2 = (uint32_t)__shfl(lim, 6 + 2 * k(), 64);
                    const uint32_t pa = (uint32_t)__shfl(pk, 5 + 2 * k(), 64), pc = (uint32_t)__shfl(pk, 6 + 2 * k(), 64);
                    if (lane == j) {
                        T.dl[k()] = a | (k() < 5 ? c2 << 16 : 0u);
                        T.di[k()] = (pa & 0xffff) | (k() < 5 ? pc << 16 : 0u);
                    }
                });
                if (lane == j) {
                    if (!ok) {
                        fail(E_TABLE);
                    } else {
                        if (dfr) ((OGE_G uint32_t *)(xj + kXStart))[nt] = pos;  // the table's first position
                        tabs = ((nt + 1) << 1) | dfr;
                        st = ST_SYM;
                    }
                }
            }
        }
        // ---- next block for lanes that finished theirs: taken from the launch's queue (one atomic per
        // wave), so a lane never idles while blocks are left -- the launch ends when the queue drains,
        // not when the slowest of a fixed block-per-lane assignment does
#if OGE_EXP == 3
        const uint64_t y1 = __builtin_readcyclecounter();
        y_bld += y1 - y0;
#endif
        const uint64_t want = __ballot(st == ST_NEXT);
        if (want) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(want);
            unsigned long long q = 0;
            if (lane == leader) q = atomicAdd(next, (unsigned long long)__popcll(want));
            q = ((unsigned long long)__shfl((unsigned)(q >> 32), (int)leader, 64) << 32) | (unsigned)__shfl((unsigned)q, (int)leader, 64);
            if (st == ST_NEXT) b = (uint32_t)(b0 + q) + (uint32_t)__popcll(want & ((1ull << lane) - 1));
        }
        if (st == ST_NEXT) {
            if ((uint64_t)b >= b0 + nb) {
                st = ST_DONE;
            } else {
                const uintptr_t ob = (uintptr_t)(out + uoff[b]);
                osz = (uint32_t)(uoff[b + 1] - uoff[b]);
                al = (uint32_t)(ob & 7);
                ob8 = (OGE_G uint8_t *)(ob - al);
                clast = (al + osz + 7) / 8 - 1;
                pos = 0;
                acc = 0;
                bi = (uint32_t)(b - b0);
                bm = lm = 0;
                bw = 0;
                // the pre-pass's verdict: prepared (tables ready, the first symbol's bit offset) or not
                const uint32_t pm = pmeta ? pmeta[bi] : 0u;
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                *(OGE_G u32x4 *)(xtab + (uint64_t)bi * kXTab + kXStart) =
                    u32x4{(pm >> 29) & 1 ? 0u : 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
                tabs = 0;
                const uint32_t u = pm & 0xffffff;
                seek((uintptr_t)z + d0a[b] + (u >> 3));
                skip(u & 7);
                under = 0;
                flg = (pm >> 28) & 1;
                st = (pm >> 31) ? ST_LOAD : ST_HDR;
            }
        }
#if OGE_EXP == 3
        y_blk += (uint32_t)__popcll(__ballot(st == ST_HDR));
        y_nxt += __builtin_readcyclecounter() - y1;
#endif
        // ---- prepared first tables (k_infl_prep): lane j's record copied into its LDS column and Slow
        // registers by the whole wave, one 8-byte load per lane; the next lane's record is loaded while
        // this one is written
        if (uint64_t ld = __ballot(st == ST_LOAD)) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            auto rec = [&](uint32_t j) {
                const uint32_t bj = __builtin_amdgcn_readlane(bi, j);
                const OGE_G u32x2 *R = (const OGE_G u32x2 *)(prep + (uint64_t)bj * kPrep);
                return lane < kPrep / 8 ? R[lane] : u32x2{0u, 0u};
            };
            uint32_t j = (uint32_t)__builtin_ctzll(ld);
            ld &= ld - 1;
            u32x2 v = rec(j);
            for (;;) {
                const uint32_t jn = ld ? (uint32_t)__builtin_ctzll(ld) : j;
                u32x2 vn = {0u, 0u};
                if (ld) vn = rec(jn);
                if (lane < 16) {
                    S.lt[4 * lane][j] = (uint16_t)v.x, S.lt[4 * lane + 1][j] = (uint16_t)(v.x >> 16);
                    S.lt[4 * lane + 2][j] = (uint16_t)v.y, S.lt[4 * lane + 3][j] = (uint16_t)(v.y >> 16);
                } else if (lane < 26) {  // dt | ll | dl rows (contiguous in P1Lds): 8 per lane
                    const uint32_t r0 = 8 * (lane - 16);
                    uint8_t *row = &S.dt[0][0] + r0 * 64 + j;
#pragma unroll
                    for (uint32_t i = 0; i < 8; ++i)
                        if (r0 + i < 16 + 32 + 30) row[i * 64] = (uint8_t)((i < 4 ? v.x : v.y) >> (8 * (i & 3)));
                }
                sfor<13>([&](auto k) {
                    constexpr int K = decltype(k)::value;
                    const uint32_t a = __builtin_amdgcn_readlane(v.x, P_SLOW / 8 + K), c = __builtin_amdgcn_readlane(v.y, P_SLOW / 8 + K);
                    if (lane == j) {
                        tset<2 * K>(T, a);
                        tset<2 * K + 1>(T, c);
                    }
                });
                if (lane == j) tabs = 3, st = ST_SYM;  // table 0, long literals deferred
                if (!ld) break;
                ld &= ld - 1;
                j = jn;
                v = vn;
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (__ballot(st != ST_DONE) == 0) {
#if OGE_EXP == 3
            if (lane == 0 && blockIdx.x < 16)
                printf("infl-exp3 wave %u: cycles build %llu next %llu loop %llu | iters %u: with CL %u HDR %u STORED %u SYM %u | "
                       "blocks %u builds cl %u tab %u | cycles in iters with CL %llu without %llu\n",
                       blockIdx.x, (unsigned long long)y_bld, (unsigned long long)y_nxt, (unsigned long long)y_loop, y_it, y_cl,
                       y_hdr, y_sto, y_sym, y_blk, y_nbcl, y_nbld, (unsigned long long)y_clc, (unsigned long long)y_oc);
#endif
#if OGE_EXP == 2
            uint64_t w = x_wait;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) w = max(w, (uint64_t)__shfl_xor((unsigned long long)w, d, 64));
            if (lane == 0 && blockIdx.x < 8)
                printf("infl-exp wave %u: loop cycles %llu, steps %llu, max lane wait cycles %llu\n", blockIdx.x,
                       (unsigned long long)x_loop, (unsigned long long)x_steps, (unsigned long long)w);
#endif
            break;
        }

        // ---- kInner decode steps; a lane that reaches a wave-wide state (build, next block) idles
#if OGE_EXP == 2
        const uint64_t l0 = __builtin_readcyclecounter();
        x_steps += kInner;
#endif
#if OGE_EXP == 3
        const uint64_t y2 = __builtin_readcyclecounter();
#endif
        for (int it = 0; it < kInner; ++it) {
#if OGE_EXP == 3
            ++y_it;
            const uint64_t yi = __builtin_readcyclecounter();
            const bool ycl = __ballot(st == ST_CL) != 0;
            y_cl += ycl;
            y_hdr += __ballot(st == ST_HDR) != 0;
            y_sto += __ballot(st == ST_STORED) != 0;
            y_sym += __ballot(st == ST_SYM) != 0;
#endif
            if (st == ST_SYM) {
                // an iteration: up to LB direct literals, one symbol of any kind, up to LB direct literals.
                // A wave runs the union of its lanes' paths, so a lane should make as much progress per
                // iteration as the union costs: a match and the literals around it in one pass (C2 blocks:
                // 11.5k iterations per BGZF block instead of 19.8k one-symbol steps; tools/ana policy)
#if OGE_INFL_ITER != 1
                lit_batch(0, 0);
#endif
                refill();
                uint32_t pb = 0, np = 0;  // a literal main symbol: put with the second batch
                const uint32_t v = (uint32_t)buf;
                const uint32_t e = S.lt[v & ((1u << TL) - 1)][lane];
                uint32_t sym, L;
                if (e >> 9) {
                    sym = e & 511, L = e >> 9;
                } else {  // code longer than TL bits: canonical limits (VGPRs)
                    const uint32_t c15 = __builtin_bitreverse32(v) >> 17;
                    // L = 7 + the limits <= c15 (limits never decrease with the length); the same tests pick
                    // the length's list parameters
                    L = 7;
                    uint32_t pk = T.pk[0];
                    sfor<4>([&](auto k) {
                        const bool g0 = c15 >= (T.ll[k()] & 0xffff), g1 = c15 >= (T.ll[k()] >> 16);
                        L += g0 + g1;
                        pk = g0 ? T.pk[2 * k() + 1] : pk;
                        pk = g1 ? T.pk[2 * k() + 2] : pk;
                    });
                    const uint32_t k = ((pk & 0xffff) + (c15 >> (15 - L))) & 0xffff;
                    const uint32_t litend = (pk >> 16) & 511;
                    if (k < litend) {  // a literal: its byte later (phase 2), or now from the lane's scratch
                        sym = (tabs & 1) ? kDefer | k : (uint32_t)scr()[S_LS + min(k, 287u)];
                    } else {  // a length code or end of block: LDS
                        sym = 256u + S.ll[min(k - litend + (pk >> 25), 31u)][lane];
                    }
                    if (L == 15 && c15 >= T.l15) sym = 512;  // no such code
                }
                skip(L);
                if (sym < 256 || sym >= kDefer) {
                    if (pos >= osz) {
                        fail(E_OVERRUN);
                    } else {
                        if (sym >= kDefer) {
                            word(pos);
                            lm |= 1ull << (pos & 63);
                        }
                        pb = sym & 0xff, np = 1;
                    }
                } else if (sym == 256) {
                    if (flg & 1) block_end();
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
                    const uint32_t de = S.dt[w & ((1u << TD) - 1)][lane];
                    uint32_t ds, DL;
                    if (de) {
                        ds = de & 31, DL = de >> 5;
                    } else {
                        const uint32_t c15 = __builtin_bitreverse32(w) >> 17;
                        DL = 5;
                        uint32_t di = T.di[0] & 0xffff;
                        sfor<5>([&](auto k) {
                            const bool g0 = c15 >= (T.dl[k()] & 0xffff), g1 = c15 >= (T.dl[k()] >> 16);
                            DL += g0 + g1;
                            di = g0 ? T.di[k()] >> 16 : di;
                            di = g1 ? T.di[k() + 1] & 0xffff : di;
                        });
                        const uint32_t k = (di + (c15 >> (15 - DL))) & 0xffff;
                        ds = S.dl[min(k, 29u)][lane];
                        if (DL == 15 && c15 >= (T.dl[5] & 0xffff)) ds = 31;  // no such code
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
                            word(pos);
                            bm |= 1ull << (pos & 63);
                            const uint32_t dsc = (len - 3) | ((dist - 1) << 8);  // descriptor in the hole's first bytes
                            put_n(dsc, 3);
                            // the rest of the hole: the shift register moves on with it (a chunk it leaves
                            // half-written is stored now; hole bytes are don't-care)
                            const uint32_t q = pos + al, qe = q + len - 3;
                            if ((qe >> 3) == (q >> 3)) {
                                acc >>= 8 * (qe - q);
                            } else {
                                flush_partial();
                            }
                            pos += len - 3;
                        }
                    }
                }
                if (st == ST_SYM) lit_batch(pb, np);  // a failed block drops its pending byte
#if OGE_INFL_ITER >= 1
                if (st == ST_SYM) lit_batch(0, 0);
#endif
            } else if (st == ST_CL) {
                refill();
                const uint32_t e = ((const uint8_t *)&S.lt[0][0])[cl_at((uint32_t)buf & 127, lane)];
                const uint32_t s = e & 31, L = e >> 5;
                skip(L);
                const uint32_t total = (hl & 0xffff) + (hl >> 16);
                uint32_t ci = aux & 0xffff, prev = (aux >> 16) & 0xff, l256 = aux >> 24;
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
                        if (val)  // zero runs need no stores: the buffer was zeroed by the CL build
                            for (uint32_t k = 0; k < rep; ++k) scr()[S_LENS + ci + k] = (uint8_t)val;
                        if (ci <= 256 && 256 < ci + rep) l256 = val;
                        prev = val;
                        ci += rep;
                        aux = ci | (prev << 16) | (l256 << 24);
                        if (ci == total) {
                            if (!l256) fail(E_TABLE);  // no end-of-block code
                            else st = ST_BLD;
                        }
                    }
                }
            } else if (st == ST_HDR) {
                refill();
                const uint32_t h = get(3);
                flg = h & 1;
                const uint32_t type = h >> 1;
                if (type == 0) {
                    skip((8 - (uint32_t)(bitpos() & 7)) & 7);
                    refill();
                    const uint32_t len = get(16), nlen = get(16);
                    if ((len ^ 0xffffu) != nlen) fail(E_STORED);
                    else if (pos + len > osz) fail(E_OVERRUN);
                    else aux = len, st = ST_STORED;
                } else if (type == 1) {
                    flg |= 2, hl = 288 | (30 << 16), st = ST_BLD;
                } else if (type == 2) {
                    const uint32_t hlit = get(5) + 257;
                    const uint32_t hdist = get(5) + 1;
                    hl = hlit | (hdist << 16);
                    const uint32_t hclen = get(4) + 4;
                    if (hlit > 286 || hdist > 30) {
                        fail(E_TABLE);
                    } else {
                        uint64_t c = 0;
#pragma unroll
                        for (int i = 0; i < 19; ++i) {
                            if ((uint32_t)i < hclen) {
                                refill();
                                c |= (uint64_t)get(3) << (3 * kClOrd[i]);
                            }
                        }
                        *(OGE_G uint64_t *)(scr() + S_CLP) = c;
                        st = ST_BCL;
                    }
                } else {
                    fail(E_TYPE);
                }
            } else if (st == ST_STORED) {
                refill();
                const uint32_t k = min(aux, 4u);
                for (uint32_t i = 0; i < k; ++i) put(get(8));
                aux -= k;
                if (!aux) {
                    if (flg & 1) block_end();
                    else st = ST_HDR;
                }
            }
#if OGE_EXP == 3
            {
                const uint64_t yc = __builtin_readcyclecounter() - yi;
                if (ycl) y_clc += yc;
                else y_oc += yc;
            }
#endif
        }
#if OGE_EXP == 2
        x_loop += __builtin_readcyclecounter() - l0;
#endif
#if OGE_EXP == 3
        y_loop += __builtin_readcyclecounter() - y2;
#endif
    }
}

// ---------------------------------------------------------------------------- phase 2
// 1024-thread workgroups (r02: 512 threads; the refs array keeps it to one workgroup per CU, so sixteen
// waves instead of eight hide the LDS and barrier latency of the pointer-jumping rounds), persistent since
// r04 (see the block loop).  Tried in r04 and not kept: hole refs filled chunk by chunk by every thread
// (owners mark their holes' positions in an LDS bitmap and write the start refs only; each 8-position chunk
// then finds its covering hole's start) instead of by the window's owner: 20M reads 46.5 -> 47.9 ms.
// Thread t owns the block's bytes [64t, 64t + 64) for the hole descriptors and the CRC, and the
// 8-position chunks c = 1024 k + t (k < 8) for the refs / image passes (a wave's 64 lanes touch 64
// consecutive chunks: conflict-free LDS).
constexpr uint32_t kT2 = 1024;
#ifndef OGE_LZ_HOPS
#define OGE_LZ_HOPS 3  // refs hops per pointer-jumping round (step 4); >= 2
#endif

__global__ void __launch_bounds__(kT2) k_infl_lz(uint8_t *__restrict__ out, const uint64_t *__restrict__ uoff,
                                                 const uint32_t *__restrict__ crc, uint64_t *__restrict__ bitmap,
                                                 const uint8_t *__restrict__ xtab, uint64_t b0, uint64_t nb,
                                                 const uint32_t *__restrict__ zpow, uint32_t *__restrict__ err) {
    __shared__ __align__(16) uint16_t refs[kSlot + 16];  // later the block's bytes (img)
    __shared__ uint32_t crctab[4][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t crcs[kT2 / 64];
    __shared__ __align__(16) uint8_t xl[kXTab];
    __shared__ uint32_t zl[32][64];  // the CRC's per-lane combine operators (crc_combine1024l)
    const uint32_t t = threadIdx.x;
    if (crc) {  // once per workgroup (r04: once per block)
        crc_setup<kT2>(crctab, zp, zpow, t);
        for (uint32_t i = t; i < 32 * 64; i += kT2) zl[i >> 6][i & 63] = zpow[17 * 32 + i];
    }
    const uint32_t q0 = 64 * t;
    // A persistent workgroup walks blocks i = blockIdx.x, + gridDim.x, ... (its 139 KiB of LDS make it the
    // CU's only one).  Block i + gridDim.x's global inputs are loaded into registers while block i's CRC is
    // computed, so a block starts with its bytes at hand (r04: one workgroup per block, whose loads -- and
    // the refs-init barrier waiting on them -- were ~14k of its ~117k cycles with the CU otherwise idle).
    //  hv: this window's hole / deferred-literal bitmap pair; xv: the block's long-literal translation
    //  lists (1,280 B, staged in LDS: the deferred literals of step 5 look their bytes up without a global
    //  round trip each); raw: this thread's 64 literal-filled bytes [q0, q0 + 64) and the next word
    //  (descriptors may straddle), aligned dwords, funnel-shifted at use.
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u64x2 hv = {0, 0};
    u32x4 xv = {0, 0, 0, 0};
    uint32_t raw[18];
    auto fetch = [&](uint64_t i) {
        const uint64_t b = b0 + i;
        const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
        const uint8_t *O = out + uoff[b];
        hv = u64x2{0, 0};
        if (t < ((osz + 63) >> 6)) {
            OGE_G u64x2 *bp = (OGE_G u64x2 *)((OGE_G uint64_t *)(bitmap + i * kBmStride) + 2 * t);
            hv = *bp;
            *bp = u64x2{0, 0};  // cleared behind the read: the next chunk's phase 1 needs no memset (r05)
        }
        xv = u32x4{0, 0, 0, 0};
        if (t < kXTab / 16) xv = *(const OGE_G u32x4 *)(xtab + i * kXTab + 16 * t);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)((uintptr_t)(O + q0) & ~(uintptr_t)3);
        const uintptr_t lim = (uintptr_t)(O + osz);  // a dword starting below lim holds a block byte: readable
#pragma unroll
        for (int k = 0; k < 18; ++k) raw[k] = (uintptr_t)(W + k) < lim ? W[k] : 0u;
    };
    // past the last block: registers defined without a load (else the compiler keeps the consumed values
    // of the previous block alive across the loop for that path, and spills)
    auto fetch_or_clear = [&](uint64_t i) {
        if (i < nb) {
            fetch(i);
        } else {
            hv = u64x2{0, 0}, xv = u32x4{0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 18; ++k) raw[k] = 0;
        }
    };
    fetch_or_clear(blockIdx.x);
    const uint32_t t_ = t;
    for (uint64_t i = blockIdx.x; i < nb; i += gridDim.x) {
    // the thread index laundered per block: the per-block index math below (the refs-init values alone
    // are 32 registers) must not be hoisted out of the loop -- hoisted, it spilled 14 VGPRs
    uint32_t t = t_;
    __asm__ volatile("" : "+v"(t));
    const uint32_t q0 = 64 * t;
    const uint64_t b = b0 + i;
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint8_t *const O = out + uoff[b];
    const uint32_t want = crc ? crc[b] : 0u;  // loaded now, compared after step 7's CRC (no round trip there)
    if (osz > kSlot) {  // uniform: no LDS touched for this block
        if (t == 0) report(err, E_SIZE, b);
        fetch_or_clear(i + gridDim.x);
        continue;
    }
#if OGE_EXP == 7  // timing experiment: phase clocks of a phase-2 workgroup (thread 0) and its rounds
    uint64_t zc[12];
    int zn = 0, zr = 0;
#define ZCLK() (zc[zn++] = __builtin_readcyclecounter())
#else
#define ZCLK()
#endif
    ZCLK();
    // 1. the prefetched window bytes
    uint32_t wv[17];
    {
        const uint32_t sh = (uint32_t)((uintptr_t)(O + q0) & 3);
#pragma unroll
        for (int k = 0; k < 17; ++k) wv[k] = sh ? __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh) : raw[k];
    }
    ZCLK();
    if (t < kXTab / 16) *(u32x4 *)(xl + 16 * t) = xv;
    // 2. every position its own source
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t p = 8 * (kT2 * k + t);
        uint4 v;
        v.x = p | ((p + 1) << 16), v.y = (p + 2) | ((p + 3) << 16), v.z = (p + 4) | ((p + 5) << 16), v.w = (p + 6) | ((p + 7) << 16);
        *(uint4 *)(refs + p) = v;
    }
    __syncthreads();
    ZCLK();
    uint64_t dm = hv.y;  // this window's deferred literals
    // 3. holes: refs[p + j] = p - D + j, descriptors read from this thread's window registers
    {
        uint64_t m = hv.x;
        while (m) {
            const uint32_t jb = (uint32_t)__builtin_ctzll(m);  // byte in the window
            m &= m - 1;
            const uint32_t d = jb >> 2, sh = (jb & 3) * 8;
            uint32_t lo = wv[0], hi = wv[1];
#pragma unroll
            for (uint32_t k = 1; k < 16; ++k) lo = d == k ? wv[k] : lo, hi = d == k ? wv[k + 1] : hi;
            const uint32_t x = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
            const uint32_t p = q0 + jb, len = (x & 0xff) + 3, dist = ((x >> 8) & 0x7fff) + 1;
            const uint32_t e = min(p + len, osz);  // phase 1 checked it; a failed block must not write past the array
            // refs over [p, e) in stores as wide as the alignment allows: 1 / 2 / 4 entries up to the next
            // 8-aligned position, 8 per 16-byte store, then 4 / 2 / 1 (at most 3 + 3 narrow stores per copy,
            // was up to 7 + 7 single entries: a wave waits for its lane with the most; 100M reads: k_infl_lz 66.4 -> 64.9 ms,
            // profiles/r06cy).  An overlapping copy (dist < len) repeats its first dist bytes: refs[p + j] =
            // p - dist + j mod dist, always before p (r03 chained q -> q - dist inside the copy: len / dist levels
            // of pointer jumping for a run)
            const uint32_t r0 = p - dist;
            uint32_t k = 0;
            auto fill = [&](auto &&nx) {
                uint32_t q = p;
                if ((q & 1) && q < e) refs[q++] = (uint16_t)nx();
                if ((q & 2) && q + 2 <= e) {
                    uint32_t a = nx();
                    a |= nx() << 16;
                    *(uint32_t *)(refs + q) = a;
                    q += 2;
                }
                if ((q & 4) && q + 4 <= e) {
                    uint2 v;
                    v.x = nx(), v.x |= nx() << 16;
                    v.y = nx(), v.y |= nx() << 16;
                    *(uint2 *)(refs + q) = v;
                    q += 4;
                }
                for (; q + 8 <= e; q += 8) {
                    uint4 v;
                    v.x = nx(), v.x |= nx() << 16;
                    v.y = nx(), v.y |= nx() << 16;
                    v.z = nx(), v.z |= nx() << 16;
                    v.w = nx(), v.w |= nx() << 16;
                    *(uint4 *)(refs + q) = v;
                }
                if (q + 4 <= e) {
                    uint2 v;
                    v.x = nx(), v.x |= nx() << 16;
                    v.y = nx(), v.y |= nx() << 16;
                    *(uint2 *)(refs + q) = v;
                    q += 4;
                }
                if (q + 2 <= e) {
                    uint32_t a = nx();
                    a |= nx() << 16;
                    *(uint32_t *)(refs + q) = a;
                    q += 2;
                }
                if (q < e) refs[q] = (uint16_t)nx();
            };
            if (dist >= len) {  // refs[q] = q - dist: the source lies before the copy
                fill([&]() { return (r0 + k++) & 0xffffu; });
            } else {
                fill([&]() {
                    const uint32_t r = r0 + k;
                    k = k + 1 == dist ? 0u : k + 1;
                    return r & 0xffffu;
                });
            }
        }
    }
    __syncthreads();
    ZCLK();
    // 4. pointer jumping until every position names a literal.  A chunk of literals only (every ref its
    //    own position) or one whose refs all name roots never changes again: `act` drops it, so later
    //    rounds only touch the chunks still inside unresolved copies.
    auto ident = [](uint4 v, uint32_t q) {
        return v.x == (q | ((q + 1) << 16)) && v.y == ((q + 2) | ((q + 3) << 16)) && v.z == ((q + 4) | ((q + 5) << 16)) &&
               v.w == ((q + 6) | ((q + 7) << 16));
    };
    uint32_t act = 0;
    for (uint32_t k = 0; k < 8; ++k)
        if (8 * (kT2 * k + t) < osz) act |= 1u << k;
    for (int round = 0; round < 20; ++round) {
        int changed = 0;
        uint32_t m = act;
        while (m) {
            const uint32_t k = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t q = 8 * (kT2 * k + t);
            const uint4 v = *(const uint4 *)(refs + q);
            if (ident(v, q)) {
                act &= ~(1u << k);
                continue;
            }
            const uint32_t r8[8] = {v.x & 0xffff, v.x >> 16, v.y & 0xffff, v.y >> 16, v.z & 0xffff, v.z >> 16, v.w & 0xffff, v.w >> 16};
            uint32_t r1[8], rr[8];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) r1[i] = refs[r8[i]];  // all issued before any is used
            // a second hop in the same round (r06): every value any thread reads or writes is an ancestor of
            // its position on the copy chain, so reading refs while other chunks are rewritten is race-free;
            // a round advances 3x instead of 2x (more when a source was already rewritten this round).
            // 100M reads: k_infl_lz 72.2 -> 70.4 ms; a third hop 71.7 (profiles/r06cq, r06cr)
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) rr[i] = refs[r1[i]];
            // with the root test below, a third hop pays (67.8 -> 66.7 ms; without the test it did not)
#pragma unroll
            for (int h = 2; h < OGE_LZ_HOPS; ++h) {
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) r1[i] = rr[i], rr[i] = refs[rr[i]];
            }
            bool ch = false, fin = true;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) ch |= rr[i] != r8[i], fin &= rr[i] == r1[i];
            if (ch) {  // positions past the end point at themselves: never changed
                uint4 o;
                o.x = rr[0] | (rr[1] << 16), o.y = rr[2] | (rr[3] << 16), o.z = rr[4] | (rr[5] << 16), o.w = rr[6] | (rr[7] << 16);
                *(uint4 *)(refs + q) = o;
            }
            // refs[r1] == r1 names a root (a non-root's ref is always below it), so a chunk whose last hops
            // all returned the previous hop's value now holds roots only: it leaves `act` at once and does not
            // keep the workgroup in the loop for a round that would only confirm it (100M reads: k_infl_lz
            // 70.3 -> 67.8 ms, profiles/r06cu)
            if (!ch || fin) act &= ~(1u << k);
            else changed = 1;
        }
#if OGE_EXP == 7
        zr = round + 1;
#endif
        if (!__syncthreads_or(changed)) break;
    }
    ZCLK();
    // 5. this thread's chunks' roots into registers, then the region becomes the byte image of the block
    //    (the literal-filled bytes, from the registers of step 1: no second global read)
    uint32_t rf[32];
    uint32_t cp = 0;  // chunks holding copied bytes (a ref other than its own position)
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t q = 8 * (kT2 * k + t);
        const uint4 v = *(const uint4 *)(refs + q);
        rf[4 * k] = v.x, rf[4 * k + 1] = v.y, rf[4 * k + 2] = v.z, rf[4 * k + 3] = v.w;
        if (!ident(v, q)) cp |= 1u << k;
    }
    __syncthreads();
    // the image is padded (bgzf_dev.h pw<4>: a spare word per 64 bytes) so the CRC's 64-byte pieces,
    // one per thread, start in distinct banks; byte q lives at ib(q)
    constexpr int PS = 4;
    uint8_t *img = (uint8_t *)refs;
    uint32_t *img32 = (uint32_t *)refs;
    auto ib = [](uint32_t q) { return q + ((q >> 6) << 2); };
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) img32[17 * t + k] = wv[k];
    // deferred literals of this window: the byte phase 1 wrote is the code's index in its table's
    // canonical long-code list; the table is the last one whose first position is <= the literal's
    if (dm) {
        const u32x4 xs = *(const u32x4 *)(xl + kXStart);
        while (dm) {
            const uint32_t p = q0 + (uint32_t)__builtin_ctzll(dm);
            dm &= dm - 1;
            const uint32_t tb = (p >= xs.w ? 3u : p >= xs.z ? 2u : p >= xs.y ? 1u : 0u);
            img[ib(p)] = xl[tb * kXList + img[ib(p)]];
        }
    }
    __syncthreads();
    ZCLK();
    // 6. every copied byte from its root (a literal position of the image); literal-only chunks are
    //    already in place
    const uint32_t last = osz ? osz - 1 : 0;
    uint32_t cw[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        cw[2 * k] = cw[2 * k + 1] = 0;
        if (!((cp >> k) & 1)) continue;
        uint32_t r[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) r[2 * i] = min(rf[4 * k + i] & 0xffff, last), r[2 * i + 1] = min(rf[4 * k + i] >> 16, last);
        cw[2 * k] = (uint32_t)img[ib(r[0])] | ((uint32_t)img[ib(r[1])] << 8) | ((uint32_t)img[ib(r[2])] << 16) |
                    ((uint32_t)img[ib(r[3])] << 24);
        cw[2 * k + 1] = (uint32_t)img[ib(r[4])] | ((uint32_t)img[ib(r[5])] << 8) | ((uint32_t)img[ib(r[6])] << 16) |
                        ((uint32_t)img[ib(r[7])] << 24);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (!((cp >> k) & 1)) continue;
        const uint32_t w = 2 * (kT2 * k + t);  // w, w + 1: same 16-word group
        img32[pw<PS>(w)] = cw[2 * k];
        img32[pw<PS>(w) + 1] = cw[2 * k + 1];
    }
    __syncthreads();
    ZCLK();
    // 7. the next block's inputs (registers free again: hv, xv and raw were consumed by steps 1-5), then
    //    the CRC and the write-out at the block's alignment
    fetch_or_clear(i + gridDim.x);
    ZCLK();
    if (crc) {
        const uint32_t c = crc_window1024l<PS>(img32, osz, crctab, zl, zp, crcs, t);
        if (t == 0 && c != want) report(err, E_CRC, b);
    }
    ZCLK();
    const uint32_t sh = (uint32_t)((uintptr_t)O & 3);
    OGE_G uint32_t *A = (OGE_G uint32_t *)((uintptr_t)O & ~(uintptr_t)3);
    const uint32_t nwords = (osz + sh + 3) / 4;
    for (uint32_t g = t; g < nwords; g += kT2) {
        const int32_t r0 = (int32_t)(4 * g) - (int32_t)sh;  // relative position of the word's first byte
        if (r0 >= 0 && r0 + 4 <= (int32_t)osz) {
            A[g] = ld32p<PS>(img32, (uint32_t)r0);
        } else {
            for (int i = 0; i < 4; ++i) {
                const int32_t r = r0 + i;
                if (r >= 0 && r < (int32_t)osz) ((OGE_G uint8_t *)(A + g))[i] = img[ib((uint32_t)r)];
            }
        }
    }
#if OGE_EXP == 7
    ZCLK();
    if (t == 0 && blockIdx.x == 7 && (i / gridDim.x) % 64 == 3)
        printf("lz-exp blk %u: load %llu init %llu holes %llu jump %llu (%d rounds) roots+defer %llu gather %llu crc+out %llu\n",
               blockIdx.x, (unsigned long long)(zc[1] - zc[0]), (unsigned long long)(zc[2] - zc[1]),
               (unsigned long long)(zc[3] - zc[2]), (unsigned long long)(zc[4] - zc[3]), zr, (unsigned long long)(zc[5] - zc[4]),
               (unsigned long long)(zc[6] - zc[5]), (unsigned long long)(zc[9] - zc[6]));
    if (t == 0 && blockIdx.x == 7 && (i / gridDim.x) % 64 == 3)
        printf("lz-exp blk %u: fetch %llu crc %llu out %llu\n", blockIdx.x, (unsigned long long)(zc[7] - zc[6]),
               (unsigned long long)(zc[8] - zc[7]), (unsigned long long)(zc[9] - zc[8]));
#endif
#undef ZCLK
    __syncthreads();  // the write-out's LDS reads before the next block's refs
    }
}

}  // namespace

// Inflate indexed blocks [0, nblk) with the lane decoder; err as in oge_bgzf_inflate_dev (err[0] bits,
// err[1] first failing block).  zpow: the CRC zero operators (device).
int oge_inflate_lanes(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                      const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                      const uint32_t *zpow) {
    const int ncu = ctx->cu_count();
    // persistent lanes (the 12 resident waves per CU) take blocks from a queue; a chunk is at most
    // kChunkLanes blocks per lane, and no more than a quarter of the free device memory holds bitmaps and
    // lists for (17.3 KiB per block), at least one block per lane.  With kStreams > 1, chunks alternate
    // over that many streams with a buffer set each, so one chunk's phase-1 drain and phase 2 can overlap
    // the next chunk.  Measured (r04): standalone at 100M reads (435k blocks) three chunks of one block
    // per lane on two streams beat one chunk on one stream (209-218 vs 225 ms) and at 200M two chunks of
    // four on two streams did (400 vs 434 ms); but inside the 300M chain -- the number that counts --
    // one stream with chunks of four blocks per lane is fastest: 649 ms against 695 (two streams, one
    // per lane), 715 (two, two) and 728 (two, four): concurrent phase-1 launches on two streams share the
    // CUs and the L2 and both finish late.  So one stream by default (a 14 GB workspace at 300M).
    const uint64_t lanes = (uint64_t)ncu * 4 * kWps * 64;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
    constexpr uint64_t kPerBlk = kBmStride * 8 + kXTab + kPrep + 4;  // bitmaps + translation lists + prepared tables
    constexpr int S = kStreams;
    const uint64_t budget =
        std::max<uint64_t>(lanes, std::min<uint64_t>(kChunkLanes * lanes, (uint64_t)(fr / 4) / (S * kPerBlk)));
    const uint64_t nchunks = std::max<uint64_t>(1, (nblk + budget - 1) / budget);
    const uint64_t chunk = std::max<uint64_t>(1, (nblk + nchunks - 1) / nchunks);
    const uint64_t wgs = std::min<uint64_t>((chunk + 63) / 64, lanes / 64);
    struct Set {
        uint64_t *bitmap;
        uint8_t *xtab, *scr, *prep;
        uint32_t *pmeta;
        unsigned long long *next;
        hipStream_t st;
    } B[S];
    // OGE_INFL_PREP=0: no header pre-pass (phase 1 parses every header itself; the A/B switch)
    const char *pe = getenv("OGE_INFL_PREP");
    const bool use_prep = !(pe && *pe == '0');
    for (int k = 0; k < S; ++k) {
        const std::string x = std::to_string(k);
        B[k].bitmap = (uint64_t *)ctx->ws(("infl_bitmap" + x).c_str(), chunk * kBmStride * 8);
        B[k].xtab = (uint8_t *)ctx->ws(("infl_xtab" + x).c_str(), chunk * kXTab);
        B[k].scr = (uint8_t *)ctx->ws(("infl_scratch" + x).c_str(), wgs * 64 * kScr);
        B[k].next = (unsigned long long *)ctx->ws(("infl_next" + x).c_str(), 8);
        B[k].prep = use_prep ? (uint8_t *)ctx->ws(("infl_prep" + x).c_str(), chunk * kPrep) : nullptr;
        B[k].pmeta = use_prep ? (uint32_t *)ctx->ws(("infl_pmeta" + x).c_str(), chunk * 4) : nullptr;
        if (use_prep && (!B[k].prep || !B[k].pmeta)) return OGE_ERR_HIP;
        B[k].st = S == 1 ? ctx->stream : ctx->side_stream(k);
        if (!B[k].bitmap || !B[k].xtab || !B[k].scr || !B[k].next || !B[k].st) return OGE_ERR_HIP;
    }
    hipEvent_t ev[S + 1];
    int nev = 0;
    struct Evs {
        hipEvent_t *e;
        int &n;
        ~Evs() {
            for (int i = 0; i < n; ++i) (void)hipEventDestroy(e[i]);
        }
    } evs{ev, nev};
    for (; nev < S + 1; ++nev) OGE_HIP_TRY(ctx, hipEventCreateWithFlags(&ev[nev], hipEventDisableTiming));
    if (S > 1) {  // inputs ready for the side streams
        OGE_HIP_TRY(ctx, hipEventRecord(ev[S], ctx->stream));
        for (int k = 0; k < S; ++k) OGE_HIP_TRY(ctx, hipStreamWaitEvent(B[k].st, ev[S], 0));
    }
    uint64_t k = 0;
    for (uint64_t b0 = 0; b0 < nblk; b0 += chunk, ++k) {
        const uint64_t nb = std::min(chunk, nblk - b0);
        const uint32_t g1 = (uint32_t)std::min<uint64_t>((nb + 63) / 64, wgs);
        const Set &u = B[k % S];
        OGE_HIP_TRY(ctx, hipMemsetAsync(u.next, 0, 8, u.st));
        // phase 1 stores only words with bits, so the bitmaps must start clear: phase 2 clears every word it
        // read, which leaves the buffer clear for the next chunk and the next call (ctx->infl_clean: the
        // buffer and how many of its bytes are known clear; a failed launch forgets it).  Fresh or grown
        // buffers, and the two-stream layout, are cleared here (a 21 GB memset per 300M-read step before).
        const uint64_t bbytes = nb * kBmStride * 8;
        const bool clean = S == 1 && ctx->infl_clean_ptr == u.bitmap && ctx->infl_clean_bytes >= bbytes;
        if (!clean) OGE_HIP_TRY(ctx, hipMemsetAsync(u.bitmap, 0, bbytes, u.st));
        if (S == 1) {
            const uint64_t known = clean ? ctx->infl_clean_bytes : bbytes;
            ctx->infl_clean_ptr = nullptr, ctx->infl_clean_bytes = 0;  // until phase 2 is launched
            ctx->infl_clean_next = known;
        }
        // each phase's own time (stages "infl_huff" / "infl_lz", summed over the chunks) on the one stream
        if (use_prep) {
            OgeStageTimer *t0 = S == 1 ? ctx->begin_stage("infl_prep") : nullptr;
            k_infl_prep<<<(uint32_t)((nb + 63) / 64), 64, 0, u.st>>>(d_z, zbytes, d0, d1, b0, nb, u.prep, u.pmeta, u.xtab);
            OGE_LAUNCH_CHECK(ctx);
            ctx->end_stage(t0);
        }
        OgeStageTimer *t1 = S == 1 ? ctx->begin_stage("infl_huff") : nullptr;
        k_infl_huff<<<g1, 64, 0, u.st>>>(d_z, zbytes, d0, d1, uoff, b0, nb, out, u.bitmap, u.xtab, u.scr, err, u.next, u.prep,
                                         u.pmeta);
        OGE_LAUNCH_CHECK(ctx);
        ctx->end_stage(t1);
        OgeStageTimer *t2 = S == 1 ? ctx->begin_stage("infl_lz") : nullptr;
        k_infl_lz<<<(uint32_t)std::min<uint64_t>(nb, (uint64_t)ncu), kT2, 0, u.st>>>(out, uoff, crc, u.bitmap, u.xtab, b0, nb,
                                                                                   zpow, err);
        OGE_LAUNCH_CHECK(ctx);
        ctx->end_stage(t2);
        if (S == 1) ctx->infl_clean_ptr = u.bitmap, ctx->infl_clean_bytes = ctx->infl_clean_next;
    }
    if (S > 1) {  // the context stream waits for every chunk
        for (int j = 0; j < S; ++j) {
            OGE_HIP_TRY(ctx, hipEventRecord(ev[j], B[j].st));
            OGE_HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev[j], 0));
        }
    }
    return OGE_OK;
}
