// inflate_lane.hip -- BGZF inflate with one LANE per block: Huffman decode in phase 1, LZ77 resolved in
// phase 2.  Replaces BgzfInputStream::decompress (openge/src/util/bgzf_input_stream.cpp:65-142: one
// zlib inflate per BGZF block on the pool) -- the same RFC 1951 decode, laid out for wave64.
//
// Why this shape.  A BGZF block is an independent deflate stream of <= 64 KiB whose Huffman decode is
// one long serial chain.  The r01 grouped decoder (one chain per 32 lanes: 19.7 GB/s at 20M reads,
// removed in r03) let a wave64 instruction advance two blocks.  Here every lane is its own decoder:
// one wave instruction advances 64 blocks (46.5 GB/s at 20M reads, profiles/r02_inflate_20m*).  A lane's decode step is a dependent chain (table lookup -> shift
// -> next lookup), so throughput comes from waves in flight: phase 1 keeps only the hot 6-bit
// literal/length and 4-bit distance tables in LDS (144 B per lane, lane-interleaved so a wave's 64
// lookups hit 64 different banks), holds the canonical limits of the longer codes in VGPRs and their
// symbol lists in a per-lane global scratch (MALL-resident): 12 waves per CU (VGPR-bound).
//
// Phase 1 (k_infl_huff, persistent 64-lane workgroups): each lane decodes the symbols of its blocks.
//   Literals are written at their output position (8-byte chunks assembled in a register); a match
//   (length L >= 3, distance D) leaves a hole of L bytes whose first three bytes receive the
//   descriptor (L-3, D-1 in 23 bits) and sets the hole's start bit in the block's 65536-bit bitmap.
//   Code tables are built by the whole wave for one lane at a time (ballot counting, when a lane
//   reaches a new dynamic block).
// Phase 2 (k_infl_lz, one 1024-thread workgroup per block): refs[p] = p for every position, then
//   refs[p + j] = p - D + j for every hole; pointer jumping (refs[q] = refs[refs[q]]) in LDS until
//   every position points at a literal (log2 of the copy-chain depth rounds; BAM data: 5-7); the
//   block's literal-filled bytes are then staged in LDS, every byte gathered from its root, CRC-32
//   checked and written out.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
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
constexpr int LB = 4;          // literals per decode step (see the ST_SYM path)
// Codes longer than the direct tables take their symbol from the lane's canonical list in its global
// scratch (MALL-resident); list heads in LDS (r02 cfg 1-3) measured slower in the 300M chain: 1615 vs
// 1157 ms (profiles/r02s3_infl_cfg.json).
// per-wave LDS, lane-interleaved ([entry][lane]): element e of lane l at e * 64 + l
struct P1Lds {
    uint16_t lt[1 << TL][64];  // sym | L << 9, 0 = longer code; while code lengths are decoded a lane's
                                // column holds its 7-bit code-length table (cl_at): sym | L << 5
    uint8_t dt[1 << TD][64];    // sym | L << 5, 0 = longer code
    uint32_t cnt[16], lo[16], first[16], offl[16], run[16], lim[16], lie[16];  // the build's per-length values
    uint64_t clp[64];           // a lane's code-length-code lengths between its header and its CL build
};
// per-lane global scratch
constexpr uint32_t kScr = 640;
constexpr uint32_t S_LENS = 0;   // u8[320] code lengths of the block being set up (zeroed by the CL build)
constexpr uint32_t S_LS = 320;   // u8[288] literal/length symbols with codes longer than TBL, canonical order
constexpr uint32_t S_DS = 608;   // u8[32]  distance symbols with codes longer than TBD

__constant__ uint8_t kClOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// entry i (7-bit code) of lane l's code-length table: byte i & 1 of lane l's literal/length entry i >> 1,
// so building one lane's table never touches another lane's column
__device__ __forceinline__ uint32_t cl_at(uint32_t i, uint32_t l) { return ((i >> 1) * 64 + l) * 2 + (i & 1); }

enum { ST_HDR = 0, ST_CL = 1, ST_SYM = 2, ST_STORED = 3, ST_BCL = 4, ST_BLD = 5, ST_NEXT = 6, ST_DONE = 7 };

// the slow-path parameters of one lane, in VGPRs (u16 pairs)
struct Slow {
    uint32_t ll[4];   // litlen left-justified 15-bit limits, lengths 7..14
    uint32_t l15;     // limit of length 15
    uint32_t lie[9];  // lengths 7..15: (list index - first code) & 0xffff | end-of-literals << 16
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

// ---------------------------------------------------------------------------- wave-cooperative builds
// Canonical Huffman code (RFC 1951 3.2.2) of one alphabet for lane j, the wave's 64 lanes holding the
// lengths of symbols lane, lane+64, ... in len[0..NR).  Codes <= TB bits go to lane j's column of the
// direct table; longer codes to lane j's symbol list (global scratch).  Per length L (lane L of the
// wave): left-justified 15-bit limit in S.lim[L], (list index - first code) | end-of-literals << 16 in
// S.lie[L].  The per-length values pass through LDS so the build holds few scalars.
// false = over-subscribed code.
template <int NR, int TB, bool LIT, class Lds>
__device__ bool wbuild(Lds &S, uint32_t j, OGE_G uint8_t *list, const uint32_t (&len)[NR], uint32_t n) {
    const uint32_t lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1;
    if (lane < 16) S.cnt[lane] = S.lo[lane] = S.run[lane] = 0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint32_t L = len[r];
        if (L && r * 64 + lane < n) {
            atomicAdd(&S.cnt[L], 1u);
            if (r < 4) atomicAdd(&S.lo[L], 1u);  // literal/length symbols < 256
        }
    }
    __builtin_amdgcn_wave_barrier();
    // lane L: first code, long-list offset, Kraft term of length L
    uint32_t fst = 0, ofl = 0, kraft = 0;
    if (lane >= 1 && lane < 16) {
        for (uint32_t l = 1; l < lane; ++l) {
            const uint32_t c = S.cnt[l];
            fst += c << (lane - l);
            if (l > (uint32_t)TB) ofl += c;
        }
        const uint32_t c = S.cnt[lane];
        kraft = c << (15 - lane);
        S.first[lane] = fst;
        S.offl[lane] = ofl;
        S.lim[lane] = min((fst + c) << (15 - lane), 65535u);
        S.lie[lane] = ((ofl - fst) & 0xffff) | ((ofl + S.lo[lane]) << 16);
    }
    // over-subscribed iff the Kraft sum exceeds 2^15 (every prefix check of RFC 1951 follows from it)
    uint32_t ks = kraft;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) ks += __shfl_xor(ks, d, 64);
    ks = __builtin_amdgcn_readfirstlane(ks);
    if (ks > 32768u) return false;
    for (uint32_t r = lane; r < (1u << TB); r += 64) {  // zero lane j's column of the direct table
        if (LIT) S.lt[r][j] = 0;
        else S.dt[r][j] = 0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const uint32_t myL = len[r], s = r * 64 + lane;
        const bool mine = myL && s < n;
        const uint32_t base = mine ? S.run[myL] : 0u, fc = mine ? S.first[myL] : 0u, ol = mine ? S.offl[myL] : 0u;
        uint32_t rank = 0, add = 0;
#pragma unroll
        for (int L = 1; L < 16; ++L) {
            const uint64_t m = __ballot(mine && myL == (uint32_t)L);
            if (myL == (uint32_t)L) rank = (uint32_t)__popcll(m & lt);
            if (lane == (uint32_t)L) add = (uint32_t)__popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        if (lane >= 1 && lane < 16) S.run[lane] += add;
        __builtin_amdgcn_wave_barrier();
        if (mine) {
            rank += base;
            if (myL <= (uint32_t)TB) {
                const uint32_t rev = __builtin_bitreverse32(fc + rank) >> (32 - myL);
                for (uint32_t k = 0; k < (1u << (TB - myL)); ++k) {
                    const uint32_t ix = rev | (k << myL);
                    if (LIT) S.lt[ix][j] = (uint16_t)(s | (myL << 9));
                    else S.dt[ix][j] = (uint8_t)(s | (myL << 5));
                }
            } else {
                list[ol + rank] = (uint8_t)s;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// ---------------------------------------------------------------------------- phase 1
// A step decodes one whole symbol (a match's length and distance codes in the same step).  A literal
// decoded from the direct table may be followed, in the same step, by up to LB - 1 more literals whose
// codes also sit in the direct table: a step starts with >= 32 bits in the buffer (refill tops up to
// 32..64), a direct code takes <= TL = 6 bits, so 4 direct codes (<= 24 bits) always fit.  Not after a
// long (7..15-bit) code: 15 + 3 * 6 = 33 > 32 (r02 commit 3941758 allowed it and corrupted a block at
// 300M reads; tests/test_gpu_inflate.py::test_long_codes_before_direct_literal_runs pins it).  A wave's
// step count is the maximum over its 64 blocks' symbol counts, so literal runs (BAM qualities, bases)
// take fewer steps: 300M reads in the chain, LB = 1 / 2 / 4 -> 1152 / 941 / 792 ms
// (profiles/r02s3_infl_litb.json).
// Bit-budget guard (always on): every skip of more bits than the buffer holds sets `under`, and the
// block fails with E_BITS instead of decoding from zero bits.
__global__ void __launch_bounds__(64, kWps) k_infl_huff(const uint8_t *__restrict__ z, uint64_t zbytes,
                                                      const uint64_t *__restrict__ d0a, const uint64_t *__restrict__ d1a,
                                                      const uint64_t *__restrict__ uoff, uint64_t b0, uint64_t nb,
                                                      uint8_t *__restrict__ out, uint64_t *__restrict__ bitmap,
                                                      uint8_t *__restrict__ scratch, uint32_t *__restrict__ err,
                                                      unsigned long long *__restrict__ next) {
    static_assert(LB <= 4 && TL * LB <= 32, "a step's literal batch must fit the 32 bits a refill guarantees");
    __shared__ P1Lds S;
    const uint32_t lane = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * 64 + lane;
    OGE_G uint8_t *const scr = (OGE_G uint8_t *)(scratch + gid * kScr);  // this lane's lens / long-code symbol lists
    const uintptr_t zend = (uintptr_t)z + zbytes;

    // input: 64-bit bit buffer + two 16-byte chunks (q being consumed, p loaded ahead)
    uint64_t buf = 0;
    uint32_t under = 0;  // a skip past the buffered bits happened in this block (the guard)
    uint32_t cnt = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0, p0 = 0, p1 = 0, p2 = 0, p3 = 0, qn = 0;
    uintptr_t cp = 0;
    auto load16 = [&](uintptr_t a, uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3) {
        if (a < zend) {  // a 16-byte aligned chunk holding at least one stream byte never leaves its page
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = *(const OGE_G u32x4 *)a;
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
        const uintptr_t c = oc << 3, ob = (uintptr_t)obase;
        if (c >= ob && c + 8 <= ob + osz) {
            *(OGE_G uint64_t *)c = acc;
        } else {
            for (uint32_t k = 0; k < 8; ++k)
                if (c + k >= ob && c + k < ob + osz) ((OGE_G uint8_t *)c)[k] = (uint8_t)(acc >> (8 * k));
        }
    };
    auto put = [&](uint32_t p, uint32_t v, uint32_t nbytes) {  // nbytes (1..3) little-endian bytes of v at p
        const uintptr_t a = (uintptr_t)(obase + p);
        const uint32_t sh = (uint32_t)(a & 7);
        if ((a >> 3) == oc && sh + nbytes <= 8) {
            acc |= (uint64_t)(v & ((1u << (8 * nbytes)) - 1)) << (8 * sh);
            return;
        }
        for (uint32_t k = 0; k < nbytes; ++k) {
            const uintptr_t ak = a + k;
            if ((ak >> 3) != oc) {
                flush();
                oc = ak >> 3;
                acc = 0;
            }
            acc |= (uint64_t)((v >> (8 * k)) & 0xff) << ((ak & 7) * 8);
        }
    };
    // match-start bitmap of the block (1024 words per block of the chunk)
    OGE_G uint64_t *bmp = nullptr;
    uint64_t bm = 0;
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

    Slow T;
    sfor<4>([&](auto k) { T.ll[k()] = 0; });
    sfor<9>([&](auto k) { T.lie[k()] = 0; });
    sfor<6>([&](auto k) { T.dl[k()] = T.di[k()] = 0; });
    T.l15 = 0;
    uint32_t st = ST_NEXT, fin = 0, hlit = 0, hdist = 0, ci = 0, prev = 0, srem = 0, fixed = 0, l256 = 0;
    uint64_t b = 0, d1bit = 0;

    auto fail = [&](uint32_t code) {
        report(err, code, b);
        st = ST_NEXT;
    };
    auto block_end = [&]() {  // last deflate block of the BGZF block consumed
        if (under) return fail(E_BITS);
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
        if (need) __threadfence_block();  // lanes' code-length stores before the wave reads them
        while (need) {
            const uint32_t j = (uint32_t)__builtin_ctzll(need);
            need &= need - 1;
            OGE_G uint8_t *sj = (OGE_G uint8_t *)(scratch + ((uint64_t)blockIdx.x * 64 + j) * kScr);
            if (__builtin_amdgcn_readlane(st, j) == ST_BCL) {
                // code-length code: 19 symbols, lengths 3 bits each (symbol s at bits 3s of S.clp[j])
                const uint64_t c = S.clp[j];
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
                    if (ok) st = ST_CL, ci = 0, prev = 0, l256 = 0;
                    else fail(E_TABLE);
                }
            } else {
                const uint32_t hl = __builtin_amdgcn_readlane(hlit, j), hd = __builtin_amdgcn_readlane(hdist, j);
                const bool fx = __builtin_amdgcn_readlane(fixed, j) != 0;
                uint32_t ll[5], dl[1];
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    const uint32_t s = r * 64 + lane;
                    ll[r] = 0;
                    if (s < hl) ll[r] = fx ? (s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8) : sj[S_LENS + s];
                }
                dl[0] = lane < hd ? (fx ? 5u : (uint32_t)sj[S_LENS + hl + lane]) : 0u;
                bool ok = wbuild<5, TL, true>(S, j, sj + S_LS, ll, hl);
                if (ok && lane == j) {
                    sfor<4>([&](auto k) { T.ll[k()] = S.lim[7 + 2 * k()] | (S.lim[8 + 2 * k()] << 16); });
                    T.l15 = S.lim[15];
                    sfor<9>([&](auto k) { T.lie[k()] = S.lie[7 + k()]; });
                }
                ok = ok && wbuild<1, TD, false>(S, j, sj + S_DS, dl, hd);
                if (lane == j) {
                    if (!ok) {
                        fail(E_TABLE);
                    } else {
                        sfor<6>([&](auto k) {
                            T.dl[k()] = S.lim[5 + 2 * k()] | (k() < 5 ? S.lim[6 + 2 * k()] << 16 : 0u);
                            T.di[k()] = (S.lie[5 + 2 * k()] & 0xffff) | (k() < 5 ? S.lie[6 + 2 * k()] << 16 : 0u);
                        });
                        st = ST_SYM;
                    }
                }
            }
        }
        // ---- next block for lanes that finished theirs: taken from the launch's queue (one atomic per
        // wave), so a lane never idles while blocks are left -- the launch ends when the queue drains,
        // not when the slowest of a fixed block-per-lane assignment does
        const uint64_t want = __ballot(st == ST_NEXT);
        if (want) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(want);
            unsigned long long q = 0;
            if (lane == leader) q = atomicAdd(next, (unsigned long long)__popcll(want));
            q = ((unsigned long long)__shfl((unsigned)(q >> 32), (int)leader, 64) << 32) | (unsigned)__shfl((unsigned)q, (int)leader, 64);
            b = b0 + q + (uint64_t)__popcll(want & ((1ull << lane) - 1));
        }
        if (st == ST_NEXT) {
            if (b >= b0 + nb) {
                st = ST_DONE;
            } else {
                obase = out + uoff[b];
                osz = (uint32_t)(uoff[b + 1] - uoff[b]);
                pos = 0;
                oc = ~0ull;
                acc = 0;
                bmp = (OGE_G uint64_t *)(bitmap + (b - b0) * 1024);
                bm = 0;
                bw = 0;
                d1bit = ((uint64_t)(uintptr_t)z + d1a[b]) * 8;
                seek((uintptr_t)z + d0a[b]);
                under = 0;
                st = ST_HDR;
            }
        }
        if (__ballot(st != ST_DONE) == 0) break;

        if (st == ST_SYM) {
            refill();
            const uint32_t v = (uint32_t)buf;
            const uint32_t e = S.lt[v & ((1u << TL) - 1)][lane];
            uint32_t sym, L;
            if (e) {
                sym = e & 511, L = e >> 9;
            } else {  // code longer than TBL bits: canonical limits (VGPRs), symbol from the lane's list
                const uint32_t c15 = __builtin_bitreverse32(v) >> 17;
                L = 7;
                sfor<4>([&](auto k) { L += (c15 >= (T.ll[k()] & 0xffff)) + (c15 >= (T.ll[k()] >> 16)); });
                const uint32_t lie = pick(T.lie, L - 7);
                const uint32_t k = ((lie & 0xffff) + (c15 >> (15 - L))) & 0xffff;
#if OGE_EXP == 1  // timing experiment: a long literal's byte is not looked up (wrong output, same bit stream)
                if (k < (lie >> 16)) sym = k & 255;
                else sym = scr[S_LS + min(k, 287u)] + 256u;
#else
                sym = scr[S_LS + min(k, 287u)] + (k >= (lie >> 16) ? 256u : 0u);
#endif
                if (L == 15 && c15 >= T.l15) sym = 512;  // no such code
            }
            skip(L);
            if (sym < 256) {
                if (pos >= osz) {
                    fail(E_OVERRUN);
                } else {
                    put(pos, sym, 1);
                    ++pos;
                    if (e) {  // more direct-table literals in this step (>= 26 bits left: three more)
#pragma unroll
                        for (int q = 1; q < LB; ++q) {
                            const uint32_t e2 = S.lt[(uint32_t)buf & ((1u << TL) - 1)][lane];
                            if (!e2 || (e2 & 511) >= 256 || pos >= osz) break;
                            skip(e2 >> 9);
                            put(pos, e2 & 511, 1);
                            ++pos;
                        }
                    }
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
                const uint32_t de = S.dt[w & ((1u << TD) - 1)][lane];
                uint32_t ds, DL;
                if (de) {
                    ds = de & 31, DL = de >> 5;
                } else {
                    const uint32_t c15 = __builtin_bitreverse32(w) >> 17;
                    DL = 5;
                    sfor<5>([&](auto k) { DL += (c15 >= (T.dl[k()] & 0xffff)) + (c15 >= (T.dl[k()] >> 16)); });
                    const uint32_t k = (u16of(T.di, DL - 5) + (c15 >> (15 - DL))) & 0xffff;
                    ds = scr[S_DS + min(k, 31u)];
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
                        put(pos, (len - 3) | ((dist - 1) << 8), 3);  // descriptor in the hole's first bytes
                        mark(pos);
                        pos += len;
                    }
                }
            }
        } else if (st == ST_CL) {
            refill();
            const uint32_t e = ((const uint8_t *)&S.lt[0][0])[cl_at((uint32_t)buf & 127, lane)];
            const uint32_t s = e & 31, L = e >> 5;
            skip(L);
            const uint32_t total = hlit + hdist;
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
                        for (uint32_t k = 0; k < rep; ++k) scr[S_LENS + ci + k] = (uint8_t)val;
                    if (ci <= 256 && 256 < ci + rep) l256 = val;
                    prev = val;
                    ci += rep;
                    if (ci == total) {
                        if (!l256) fail(E_TABLE);  // no end-of-block code
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
                    uint64_t clp = 0;
#pragma unroll
                    for (int i = 0; i < 19; ++i) {
                        if ((uint32_t)i < hclen) {
                            refill();
                            clp |= (uint64_t)get(3) << (3 * kClOrd[i]);
                        }
                    }
                    S.clp[lane] = clp;
                    fixed = 0;
                    st = ST_BCL;
                }
            } else {
                fail(E_TYPE);
            }
        } else if (st == ST_STORED) {
            refill();
            const uint32_t k = min(srem, 4u);
            for (uint32_t i = 0; i < k; ++i) put(pos + i, get(8), 1);
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
// One 1024-thread workgroup per block (r02: 512 threads; the refs array keeps it to one workgroup per
// CU, so sixteen waves instead of eight hide the LDS and barrier latency of the pointer-jumping rounds).
// Thread t owns the block's bytes [64t, 64t + 64) for the hole descriptors and the CRC, and the
// 8-position chunks c = 1024 k + t (k < 8) for the refs / image passes (a wave's 64 lanes touch 64
// consecutive chunks: conflict-free LDS).
constexpr uint32_t kT2 = 1024;

__global__ void __launch_bounds__(kT2) k_infl_lz(uint8_t *__restrict__ out, const uint64_t *__restrict__ uoff,
                                                 const uint32_t *__restrict__ crc, const uint64_t *__restrict__ bitmap,
                                                 uint64_t b0, const uint32_t *__restrict__ zpow, uint32_t *__restrict__ err) {
    __shared__ __align__(16) uint16_t refs[kSlot + 16];  // later the block's bytes (img)
    __shared__ uint32_t crctab[4][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t crcs[kT2 / 64];
    const uint32_t t = threadIdx.x;
    const uint64_t b = b0 + blockIdx.x;
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint8_t *const O = out + uoff[b];
    if (osz > kSlot) {
        if (t == 0) report(err, E_SIZE, b);
        return;
    }
    if (crc) crc_setup<kT2>(crctab, zp, zpow, t);
    const uint32_t q0 = 64 * t;
    // 1. this thread's 64 literal-filled bytes [q0, q0 + 64) and the next word (descriptors may
    //    straddle): aligned dword loads, funnel-shifted
    uint32_t wv[17];
    {
        const uintptr_t a = (uintptr_t)(O + q0);
        const uint32_t sh = (uint32_t)(a & 3);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)(a & ~(uintptr_t)3);
        const uintptr_t lim = (uintptr_t)(O + osz);  // a dword starting below lim holds a block byte: readable
        uint32_t raw[18];
#pragma unroll
        for (int k = 0; k < 18; ++k) raw[k] = (uintptr_t)(W + k) < lim ? W[k] : 0u;
#pragma unroll
        for (int k = 0; k < 17; ++k) wv[k] = sh ? __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh) : raw[k];
    }
    // 2. every position its own source
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t p = 8 * (kT2 * k + t);
        uint4 v;
        v.x = p | ((p + 1) << 16), v.y = (p + 2) | ((p + 3) << 16), v.z = (p + 4) | ((p + 5) << 16), v.w = (p + 6) | ((p + 7) << 16);
        *(uint4 *)(refs + p) = v;
    }
    __syncthreads();
    // 3. holes: refs[p + j] = p - D + j, descriptors read from this thread's window registers
    const OGE_G uint64_t *bmp = (const OGE_G uint64_t *)(bitmap + (b - b0) * 1024);
    const uint32_t nw = (osz + 63) >> 6;
    {
        uint64_t m = t < nw ? bmp[t] : 0;
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
            // refs[q] = q - dist over [p, e): single entries up to the next 8-aligned position, then
            // 8 entries per 16-byte store, then the tail
            uint32_t q = p;
            const uint32_t a8 = min((p + 7) & ~7u, e);
            for (; q < a8; ++q) refs[q] = (uint16_t)(q - dist);
            for (; q + 8 <= e; q += 8) {
                const uint32_t r = q - dist;
                uint4 v;
                v.x = (r & 0xffff) | (((r + 1) & 0xffff) << 16), v.y = ((r + 2) & 0xffff) | (((r + 3) & 0xffff) << 16);
                v.z = ((r + 4) & 0xffff) | (((r + 5) & 0xffff) << 16), v.w = ((r + 6) & 0xffff) | (((r + 7) & 0xffff) << 16);
                *(uint4 *)(refs + q) = v;
            }
            for (; q < e; ++q) refs[q] = (uint16_t)(q - dist);
        }
    }
    __syncthreads();
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
            uint32_t rr[8];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) rr[i] = refs[r8[i]];  // all issued before any is used
            bool ch = false;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) ch |= rr[i] != r8[i];
            if (ch) {  // positions past the end point at themselves: never changed
                uint4 o;
                o.x = rr[0] | (rr[1] << 16), o.y = rr[2] | (rr[3] << 16), o.z = rr[4] | (rr[5] << 16), o.w = rr[6] | (rr[7] << 16);
                *(uint4 *)(refs + q) = o;
                changed = 1;
            } else {
                act &= ~(1u << k);
            }
        }
        if (!__syncthreads_or(changed)) break;
    }
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
    __syncthreads();
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
    // 7. CRC and the write-out at the block's alignment
    if (crc) {
        const uint32_t c = crc_window1024<PS>(img32, osz, crctab, zp, crcs, t);
        if (t == 0 && c != crc[b]) report(err, E_CRC, b);
    }
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
}

}  // namespace

// Inflate indexed blocks [0, nblk) with the lane decoder; err as in oge_bgzf_inflate_dev (err[0] bits,
// err[1] first failing block).  zpow: the CRC zero operators (device).
int oge_inflate_lanes(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                      const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                      const uint32_t *zpow) {
    static int ncu = [] {
        int d = 0, n = 0;
        (void)hipGetDevice(&d);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
        return n > 0 ? n : 256;
    }();
    // persistent lanes (the 12 resident waves per CU) take blocks from a queue; a chunk is at most 4
    // blocks per lane (the queue keeps the lanes busy, so a larger chunk gains nothing: 300M reads = 2
    // launches, a 6.4 GB bitmap workspace that lives as long as the context), and no more than a
    // quarter of the free device memory holds bitmaps for (8 KiB per block), at least one block per lane
    const uint64_t lanes = (uint64_t)ncu * 4 * kWps * 64;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
    const uint64_t budget = std::max<uint64_t>(lanes, std::min<uint64_t>(4 * lanes, (uint64_t)(fr / 4) / (1024 * 8)));
    const uint64_t nchunks = std::max<uint64_t>(1, (nblk + budget - 1) / budget);
    const uint64_t chunk = std::max<uint64_t>(1, (nblk + nchunks - 1) / nchunks);
    const uint64_t wgs = std::min<uint64_t>((chunk + 63) / 64, lanes / 64);
    uint64_t *bitmap = (uint64_t *)ctx->ws("infl_bitmap", chunk * 1024 * 8);
    uint8_t *scr = (uint8_t *)ctx->ws("infl_scratch", wgs * 64 * kScr);
    unsigned long long *next = (unsigned long long *)ctx->ws("infl_next", 8);
    if (!bitmap || !scr || !next) return OGE_ERR_HIP;
    for (uint64_t b0 = 0; b0 < nblk; b0 += chunk) {
        const uint64_t nb = std::min(chunk, nblk - b0);
        const uint32_t g1 = (uint32_t)std::min<uint64_t>((nb + 63) / 64, wgs);
        OGE_HIP_TRY(ctx, hipMemsetAsync(next, 0, 8, ctx->stream));
        k_infl_huff<<<g1, 64, 0, ctx->stream>>>(d_z, zbytes, d0, d1, uoff, b0, nb, out, bitmap, scr, err, next);
        OGE_LAUNCH_CHECK(ctx);
        k_infl_lz<<<(uint32_t)nb, kT2, 0, ctx->stream>>>(out, uoff, crc, bitmap, b0, zpow, err);
        OGE_LAUNCH_CHECK(ctx);
    }
    return OGE_OK;
}
