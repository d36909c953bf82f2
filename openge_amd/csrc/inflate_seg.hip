// inflate_seg.hip -- BGZF inflate with one 1024-thread WORKGROUP per block: the block's deflate bit
// stream is cut into 1024 segments that the threads Huffman-decode in parallel (speculatively, then
// synchronised), and the LZ77 copies are resolved in LDS by pointer jumping.  Replaces
// BgzfInputStream::decompress (openge/src/util/bgzf_input_stream.cpp:65-142: one zlib inflate per
// BGZF block on the host pool) -- the same RFC 1951 decode, laid out for a CDNA4 CU.
//
// Why this shape (r03).  The lane decoder (inflate_lane.hip, one lane per block) gives every lane its own
// Huffman table, so the tables are tiny (6-bit direct), long codes go to a global symbol list, the
// wave runs the union of 64 different paths, and the output is 64 scattered 8-byte streams (4.7x write
// amplification).  Here the whole workgroup shares ONE table per deflate block: 10-bit literal/length
// and 8-bit distance direct tables (entries carry the base length / distance and extra-bit counts),
// long codes through per-length canonical limits, all in LDS.
//
// Per BGZF block (one deflate stream of <= 64 KiB output, any number of deflate blocks):
//   header   thread 0 parses the deflate block header (code-length code, run-length coded lengths);
//            all threads build the tables (fixed codes: the same build).  Stored blocks are copied.
//   pass A   the data bits [h, end) are cut into nseg <= 1024 segments of >= 64 bits; thread t decodes
//            from its segment start s_t as if a symbol started there, until the first symbol start
//            >= s_{t+1} (its exit x_t), counting output bytes, and remembers in a 128-bit mask which
//            positions of [s_t, s_t + 128) it started a symbol at.  Huffman codes resynchronise: a
//            decode started at a wrong bit soon lands on a true symbol start, and from there on it IS
//            the true decode.
//   pass B   the true entry of segment t is x_{t-1} (thread 0's is h).  Thread t decodes from it until
//            it reaches a position its pass-A decode also started a symbol at (synchronised: the rest
//            of pass A stands, and the output count is corrected by re-counting pass A's path up to
//            there), or until its segment end (its exit and count change; the neighbour re-checks in
//            the next round).  Rounds until no exit changes.
//   scan     the first segment whose true decode ends the deflate block (end-of-block code, or an
//            invalid code = corrupt data) closes it; exclusive scan of the counts = output offsets.
//   pass D   every thread decodes its true range again and writes the LDS refs array: a literal
//            byte b at position p as refs[p] = 0xFF00 | b, a match (L, D) as refs[p + j] =
//            p - D + (j mod D) (an overlapping copy points straight at the source period).
//   LZ       pointer jumping refs[q] = refs[refs[q]] until every entry holds a byte (>= 0xFF00):
//            log2 of the copy-chain depth rounds; then the bytes become an image in the same LDS,
//            CRC-32 is checked and the block is written out with coalesced dword stores.
// The next deflate block of the same BGZF block (zlib splits at 16K symbols) starts at the exit of
// the segment that held the end-of-block code; its output continues the refs array.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <utility>

#include "bgzf_dev.h"
#include "oge_ctx.h"

namespace {

using namespace oge_bgzf;

constexpr uint32_t kT = 512;   // threads per workgroup = max segments per deflate block
constexpr uint32_t kNCh = kSlot / 8 / kT;  // 8-position refs chunks per thread
constexpr int TLB = 10;        // literal/length direct-table bits
constexpr int TDB = 8;         // distance direct-table bits
constexpr uint32_t kMinSeg = 64;  // bits per segment at least (a symbol is <= 48 bits: exits stay in the next segment)
constexpr uint32_t kWin = 128;    // bits after a segment start whose pass-A symbol starts are remembered
constexpr uint32_t kHdrWin = 1024;  // stream bytes staged in LDS for the header parse

// table entries: L (code length, 4 bits; 0 = not in the direct table) | kind << 4 | payload << 8
enum { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3 };
// literal: payload = byte; length: payload = base (9 bits) | extra bits << 9
// distance entries: L | bad << 4 | base << 8 (15 bits) | extra bits << 24

__constant__ uint8_t kClOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct SegLds {
    uint16_t refs[kSlot + 64];  // refs / the block's byte image (padded 64-byte rows) at the end
    uint32_t lt[1 << TLB];
    uint32_t dt[1 << TDB];
    uint32_t llong[288];  // literal/length codes longer than TLB, canonical order (entries with their real L)
    uint32_t dlong[32];
    uint32_t llim[16], lbase[16], dlim[16], dbase[16];  // per length: left-justified 15-bit limit, list index - first code
    uint32_t cnt[2][16];
    uint32_t crctab[4][256];
    uint32_t zp[17][32];
    uint32_t crcs[kT / 64];
    uint32_t wsum[kT / 64];
    uint32_t exits[kT];
    uint8_t lens[320];
    uint8_t clt[128];  // code-length code direct table: sym | L << 5
    uint32_t hcl[19], hcnt[8], hnxt[8];  // thread 0's header parse (LDS, not scratch memory)
    // header result (thread 0 -> all): type, final, next bit, hlit, hdist, stored bytes / error
    uint32_t h_type, h_final, h_pos, h_nl, h_nd, h_err, h_slen, h_sbyte;
    uint4 hwin[kHdrWin / 16];  // the stream bytes at the header, for the serial parse
    uint32_t tstar, berr;
    // payloads over 65280 bytes: a position >= 0xFF00 cannot be named by a ref (those values are bytes),
    // so the copied bytes there keep their source here and are filled in order after the jumping
    uint16_t side[kSlot - 0xFF00];
};

__device__ __forceinline__ void report(uint32_t *err, uint32_t code, uint64_t blk) {
    atomicOr(err, 1u << code);
    atomicMin(err + 1, (uint32_t)min<uint64_t>(blk, 0xffffffffull));
}

// ---------------------------------------------------------------------------- bit reader
// 64-bit buffer fed from two 16-byte chunks (q being consumed, p loaded ahead); after refill() the
// buffer holds >= 32 bits: a literal/length code + its extra bits (<= 20) or a distance code + its
// extra bits (<= 28) always fit.
// WIN: the 16-byte chunks of [win, win + kHdrWin) come from a copy in LDS (the header parse: one
// parallel load instead of a serial chain of global round trips)
template <bool WIN>
struct RdT {
    uint64_t buf;
    uint32_t cnt, q0, q1, q2, q3, p0, p1, p2, p3, qn;
    uintptr_t cp, zlast;  // zlast: the last 16-byte aligned chunk holding a stream byte
    uintptr_t win;
    const uint4 *wl;
    __device__ __forceinline__ void load16(uintptr_t a, uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3) {
        if (WIN && a - win < kHdrWin) {
            const uint4 v = wl[(a - win) >> 4];
            x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
        } else {
            // always a load (no branch around it: a conditional load would be waited for on the spot, and
            // the reader's one-chunk prefetch would become a memory round trip per 16 bytes); past the end
            // of the stream the last chunk is read again (those bits are never part of a true decode)
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = *(const OGE_G u32x4 *)min(a, zlast);
            x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
        }
    }
    __device__ __forceinline__ void refill() {
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
    }
    __device__ __forceinline__ void skip(uint32_t k) { buf >>= k, cnt -= k; }
    __device__ __forceinline__ uint32_t peek() const { return (uint32_t)buf; }
    __device__ __forceinline__ uint32_t get(uint32_t k) {
        const uint32_t v = (uint32_t)buf & ((1u << k) - 1);
        skip(k);
        return v;
    }
    // start reading at bit `bit` of the stream at byte address zb
    __device__ __forceinline__ void seek(uintptr_t zb, uint32_t bit) {
        const uintptr_t a = zb + (bit >> 3);
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
        skip((uint32_t)(a & 3) * 8 + (bit & 7));
    }
};
using Rd = RdT<false>;

// ---------------------------------------------------------------------------- symbol decode
// codes longer than the direct tables: canonical limits of lengths TB+1..15
__device__ __forceinline__ uint32_t lit_long(const SegLds &S, uint32_t v) {
    const uint32_t *lim = S.llim;
    const uint32_t c15 = __builtin_bitreverse32(v) >> 17;
    uint32_t L = TLB + 1;
#pragma unroll
    for (int k = TLB + 1; k < 15; ++k) L += c15 >= lim[k];
    if (c15 >= lim[15]) return (K_BAD << 4) | 15;
    return S.llong[min((S.lbase[L] + (c15 >> (15 - L))) & 0xffffu, 287u)];
}
__device__ __forceinline__ uint32_t dist_long(const SegLds &S, uint32_t v) {
    const uint32_t *lim = S.dlim;
    const uint32_t c15 = __builtin_bitreverse32(v) >> 17;
    uint32_t L = TDB + 1;
#pragma unroll
    for (int k = TDB + 1; k < 15; ++k) L += c15 >= lim[k];
    if (c15 >= lim[15]) return 16 | 15;
    return S.dlong[min((S.dbase[L] + (c15 >> (15 - L))) & 0xffffu, 31u)];
}
__device__ __forceinline__ uint32_t lit_entry(const SegLds &S, uint32_t v) {
    const uint32_t e = S.lt[v & ((1u << TLB) - 1)];
    return (e & 15) ? e : lit_long(S, v);
}
__device__ __forceinline__ uint32_t dist_entry(const SegLds &S, uint32_t v) {
    const uint32_t e = S.dt[v & ((1u << TDB) - 1)];
    return (e & 15) ? e : dist_long(S, v);
}

struct Sym {
    uint32_t kind, len, val, bits;  // val: literal byte / match distance
};
// one symbol (a match = length + distance) at the reader; a bad symbol consumes nothing
__device__ __forceinline__ void dsym(Rd &r, const SegLds &S, Sym &y) {
    r.refill();
    const uint32_t v = r.peek();
    const uint32_t e = lit_entry(S, v);
    const uint32_t L = e & 15;
    y.kind = L ? (e >> 4) & 3 : (uint32_t)K_BAD;  // (a zero-length entry never comes out of a good table)
    y.bits = L;
    y.len = 0;
    y.val = (e >> 8) & 255;
    if (y.kind == K_LIT) {
        r.skip(L);
        y.len = 1;
    } else if (y.kind == K_LEN) {
        const uint32_t ext = (e >> 17) & 7;
        const uint32_t len = ((e >> 8) & 511) + ((v >> L) & ((1u << ext) - 1));
        r.skip(L + ext);
        r.refill();
        const uint32_t w = r.peek();
        const uint32_t de = dist_entry(S, w);
        if ((de & 16) || !(de & 15)) {
            y.kind = K_BAD;
            y.bits = 0;
            return;
        }
        const uint32_t DL = de & 15, dext = (de >> 24) & 15;
        y.val = ((de >> 8) & 0x7fff) + ((w >> DL) & ((1u << dext) - 1));
        r.skip(DL + dext);
        y.len = len;
        y.bits = L + ext + DL + dext;
    } else if (y.kind == K_EOB) {
        r.skip(L);
    } else {
        y.bits = 0;
    }
}

__device__ __forceinline__ uint32_t len_base(uint32_t c) {  // length symbol - 257 (0..28)
    if (c < 8) return c + 3;
    if (c == 28) return 258;
    const uint32_t x = (c - 4) >> 2;
    return ((4 + (c & 3)) << x) + 3;
}
__device__ __forceinline__ uint32_t len_ext(uint32_t c) { return c < 8 || c == 28 ? 0u : (c - 4) >> 2; }
__device__ __forceinline__ uint32_t dist_base(uint32_t d) { return d < 4 ? d + 1 : ((2 + (d & 1)) << ((d - 2) >> 1)) + 1; }
__device__ __forceinline__ uint32_t dist_ext(uint32_t d) { return d < 4 ? 0u : (d - 2) >> 1; }

// ---------------------------------------------------------------------------- table build (all threads)
// lens[0, nl) literal/length lengths, lens[nl, nl + nd) distance lengths.  false (S.berr) = over-subscribed.
__device__ void build_tables(SegLds &S, uint32_t nl, uint32_t nd, uint32_t t) {
    for (uint32_t i = t; i < (1u << TLB); i += kT) S.lt[i] = 0;
    if (t < (1u << TDB)) S.dt[t] = 0;
    if (t < 32) S.cnt[t >> 4][t & 15] = 0;
    __syncthreads();
    if (t < nl + nd) {
        const uint32_t L = S.lens[t];
        if (L) atomicAdd(&S.cnt[t < nl ? 0 : 1][L], 1u);
    }
    __syncthreads();
    // thread a * 16 + L: first code, list offset, limit of length L in alphabet a
    uint32_t fst = 0, ofl = 0;
    if (t < 32) {
        const uint32_t a = t >> 4, L = t & 15, TB = a ? TDB : TLB;
        uint32_t kraft = 0;
        for (uint32_t l = 1; l < 16; ++l) {
            const uint32_t c = S.cnt[a][l];
            if (l < L) {
                fst += c << (L - l);
                if (l > TB) ofl += c;
            }
            kraft += c << (15 - l);
        }
        if (L == 1 && kraft > 32768u) S.berr = 1;  // over-subscribed
        if (L >= 1) {
            const uint32_t lim = min((fst + S.cnt[a][L]) << (15 - L), 65535u);
            const uint32_t base = (ofl - fst) & 0xffff;
            if (a) S.dlim[L] = lim, S.dbase[L] = base;
            else S.llim[L] = lim, S.lbase[L] = base;
        }
    }
    __syncthreads();
    if (t < nl + nd) {
        const bool dist = t >= nl;
        const uint32_t a0 = dist ? nl : 0, sym = t - a0, L = S.lens[t];
        if (L) {
            const uint32_t TB = dist ? TDB : TLB;
            // rank among the alphabet's earlier symbols of the same length
            uint32_t rank = 0;
            for (uint32_t j = a0; j < t; ++j) rank += S.lens[j] == L;
            // first code of length L and the list offset (same sums as above)
            uint32_t f = 0, o = 0;
            for (uint32_t l = 1; l < L; ++l) {
                const uint32_t c = S.cnt[dist][l];
                f += c << (L - l);
                if (l > TB) o += c;
            }
            uint32_t e;
            if (!dist) {
                if (sym < 256) e = L | (K_LIT << 4) | (sym << 8);
                else if (sym == 256) e = L | (K_EOB << 4);
                else if (sym < 286) e = L | (K_LEN << 4) | (len_base(sym - 257) << 8) | (len_ext(sym - 257) << 17);
                else e = L | (K_BAD << 4);
            } else {
                e = sym < 30 ? L | (dist_base(sym) << 8) | (dist_ext(sym) << 24) : (L | 16);
            }
            const uint32_t code = f + rank;
            if (L <= TB) {
                const uint32_t rev = __builtin_bitreverse32(code) >> (32 - L);
                for (uint32_t k = 0; k < (1u << (TB - L)); ++k) {
                    if (dist) S.dt[rev | (k << L)] = e;
                    else S.lt[rev | (k << L)] = e;
                }
            } else {
                if (dist) S.dlong[min(o + rank, 31u)] = e;
                else S.llong[min(o + rank, 287u)] = e;
            }
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------- header (thread 0)
// Parses the deflate block header at bit pos: S.h_type (0 stored, 1 fixed, 2 dynamic), S.h_final, S.h_pos
// (first data bit; stored: first payload byte * 8), lens[] + h_nl / h_nd for dynamic codes, h_slen
// (stored length), h_err (error code or 0).
__device__ void parse_header(SegLds &S, uintptr_t zb, uint32_t pos, uint32_t end_bits, uintptr_t zend) {
    S.h_err = 0;
    if (pos + 3 > end_bits) { S.h_err = E_PAST; return; }
    RdT<true> r;
    r.zlast = (zend - 1) & ~(uintptr_t)15;
    r.win = (zb + (pos >> 3)) & ~(uintptr_t)15;
    r.wl = S.hwin;
    r.seek(zb, pos);
    const uint32_t h = r.get(3);
    pos += 3;
    S.h_final = h & 1;
    const uint32_t type = h >> 1;
    S.h_type = type;
    if (type == 0) {
        const uint32_t al = (pos + 7) & ~7u;
        r.refill();
        r.skip(al - pos);
        r.refill();
        const uint32_t len = r.get(16), nlen = r.get(16);
        if ((len ^ 0xffffu) != nlen) { S.h_err = E_STORED; return; }
        S.h_slen = len;
        S.h_pos = al + 32;
        if (S.h_pos + 8 * len > end_bits) S.h_err = E_PAST;
        return;
    }
    if (type == 1) {
        S.h_nl = 288, S.h_nd = 30;  // lens filled by all threads (fixed codes; 286/287 and 30/31 decode as bad)
        S.h_pos = pos;
        return;
    }
    if (type != 2) { S.h_err = E_TYPE; return; }
    r.refill();
    const uint32_t hlit = r.get(5) + 257, hdist = r.get(5) + 1, hclen = r.get(4) + 4;
    pos += 14;
    if (hlit > 286 || hdist > 30) { S.h_err = E_TABLE; return; }
    uint32_t *cl = S.hcl, *cntl = S.hcnt, *nxt = S.hnxt;
    for (int i = 0; i < 19; ++i) cl[i] = 0;
    for (uint32_t i = 0; i < hclen; ++i) {
        r.refill();
        cl[kClOrd[i]] = r.get(3);
    }
    pos += 3 * hclen;
    // code-length code: canonical, 7-bit direct table
    for (int L = 0; L < 8; ++L) cntl[L] = 0;
    for (int i = 0; i < 19; ++i) cntl[cl[i]]++;
    cntl[0] = 0;
    int left = 1;
    for (int L = 1; L < 8; ++L) {
        left = 2 * left - (int)cntl[L];
        if (left < 0) { S.h_err = E_TABLE; return; }
    }
    uint32_t code = 0;
    nxt[0] = 0;
    for (int L = 1; L < 8; ++L) {
        code = (code + cntl[L - 1]) << 1;
        nxt[L] = code;
    }
    for (int i = 0; i < 128; ++i) S.clt[i] = 0;
    for (int s = 0; s < 19; ++s) {
        const uint32_t L = cl[s];
        if (!L) continue;
        const uint32_t rev = __builtin_bitreverse32(nxt[L]++) >> (32 - L);
        for (uint32_t k = 0; k < (1u << (7 - L)); ++k) S.clt[rev | (k << L)] = (uint8_t)(s | (L << 5));
    }
    const uint32_t total = hlit + hdist;
    uint32_t ci = 0, prev = 0;
    while (ci < total) {
        r.refill();
        const uint32_t e = S.clt[r.peek() & 127];
        if (!e) { S.h_err = E_CODE; return; }
        const uint32_t s = e & 31, L = e >> 5;
        r.skip(L);
        pos += L;
        uint32_t rep = 1, val = s;
        if (s == 16) {
            if (ci == 0) { S.h_err = E_TABLE; return; }
            rep = 3 + r.get(2), val = prev, pos += 2;
        } else if (s == 17) {
            rep = 3 + r.get(3), val = 0, pos += 3;
        } else if (s == 18) {
            rep = 11 + r.get(7), val = 0, pos += 7;
        }
        if (ci + rep > total) { S.h_err = E_TABLE; return; }
        if (val)  // zero runs need no stores (lens was zeroed)
            for (uint32_t k = 0; k < rep; ++k) {
                const uint32_t i = ci + k;
                S.lens[i < hlit ? i : 288 + (i - hlit)] = (uint8_t)val;  // distance lengths at 288
            }
        prev = val;
        ci += rep;
        if (pos > end_bits) { S.h_err = E_PAST; return; }
    }
    if (!S.lens[256]) { S.h_err = E_TABLE; return; }  // no end-of-block code
    S.h_nl = 288, S.h_nd = hdist;  // the build reads lit lengths at [0, 288), distance lengths at [288, 288 + nd)
    S.h_pos = pos;
}

// exclusive scan over the workgroup (u32)
__device__ __forceinline__ uint32_t block_scan(SegLds &S, uint32_t v, uint32_t t, uint32_t *total) {
    const uint32_t lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) S.wsum[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t k = 0; k < kT / 64; ++k) {
        const uint32_t s = S.wsum[k];
        before += k < w ? s : 0u;
        all += s;
    }
    *total = all;
    __syncthreads();
    return before + x - v;
}

enum { ST_RUN = 0, ST_EOB = 1, ST_BAD = 2 };

// One BGZF block b by the whole workgroup.  bnext (or ~0): the block this workgroup takes next; its
// compressed bytes are touched once during this block's decode so they come from L2 when it starts
// (warm keeps those loads alive: the workgroup's decode is a chain of dependent memory round trips).
__device__ __forceinline__ void infl_block(SegLds &S, const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0a,
                                           const uint64_t *__restrict__ d1a, const uint64_t *__restrict__ uoff,
                                           const uint32_t *__restrict__ crc, uint8_t *__restrict__ out, uint32_t *__restrict__ err,
                                           uint32_t *__restrict__ dbg, uint64_t dbg_blk, uint64_t b, uint64_t bnext,
                                           uint32_t &warm) {
    const uint32_t t = threadIdx.x;
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint8_t *const O = out + uoff[b];
    uintptr_t zn = 0;
    uint32_t zn_bytes = 0;
    if (bnext != ~0ull) zn = (uintptr_t)z + d0a[bnext], zn_bytes = (uint32_t)(d1a[bnext] - d0a[bnext]);
    if (osz > kSlot) {
        if (t == 0) report(err, E_SIZE, b);
        return;
    }
    const uintptr_t zb = (uintptr_t)z + d0a[b];
    const uintptr_t zend = (uintptr_t)z + zbytes;
    const uint32_t end_bits = (uint32_t)(d1a[b] - d0a[b]) * 8u;
    if (t < 8) S.refs[min(osz + t, (uint32_t)kSlot + 63)] = 0xFF00;  // the last chunk's tail reads as resolved
    if (osz > 0xFF00 && t < kSlot - 0xFF00) S.side[t] = 0xFFFF;

    const bool tdbg = dbg && b == dbg_blk && t == 0;  // TEMP phase clocks
#define TMARK(i) if (tdbg) dbg[16 * kT + (i)] = (uint32_t)clock64()
    TMARK(0);
    uint32_t pos = 0, base = 0;  // next deflate block header (bit), output produced so far
    uint32_t fail = 0;
    for (;;) {
        for (uint32_t i = t; i < 320; i += kT) S.lens[i] = 0;  // the header parse then stores non-zero lengths only
        if (t < kHdrWin / 16) {  // the header's bytes into LDS, all chunks in flight at once
            const uintptr_t a = ((zb + (pos >> 3)) & ~(uintptr_t)15) + 16 * t;
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 v = {0, 0, 0, 0};
            if (a < zend) v = *(const OGE_G u32x4 *)a;
            S.hwin[t] = make_uint4(v.x, v.y, v.z, v.w);
        }
        __syncthreads();  // every thread has read the previous deflate block's header / error words
        if (t == 0) {
            S.berr = 0;
            TMARK(1);
            parse_header(S, zb, pos, end_bits, zend);
            TMARK(2);
        }
        __syncthreads();
        const uint32_t type = S.h_type, fin = S.h_final;
        if (S.h_err) { fail = S.h_err; break; }
        const uint32_t h = S.h_pos;
        if (type == 0) {  // stored: copy LEN bytes
            const uint32_t len = S.h_slen;
            if (base + len > osz) { fail = E_OVERRUN; break; }
            const OGE_G uint8_t *src = (const OGE_G uint8_t *)(zb + (h >> 3));
            for (uint32_t i = t; i < len; i += kT) S.refs[base + i] = (uint16_t)(0xFF00u | src[i]);
            base += len;
            pos = h + 8 * len;
            __syncthreads();
            if (fin) break;
            continue;
        }
        if (type == 1) {  // fixed codes
            if (t < 288) S.lens[t] = t < 144 ? 8 : t < 256 ? 9 : t < 280 ? 7 : 8;
            else if (t < 318) S.lens[t] = 5;
            __syncthreads();
        }
        // dynamic and fixed: literal/length lengths at [0, 288), distance lengths at [288, 288 + nd)
        build_tables(S, 288, S.h_nd, t);
        if (S.berr) { fail = E_TABLE; break; }

        TMARK(3);
        // ---- pass A: speculative decode of segment t
        const uint32_t span = end_bits > h ? end_bits - h : 0u;
        const uint32_t nseg = max(1u, min(kT, span / kMinSeg));
        const uint32_t seg = (span + nseg - 1) / nseg;
        const bool act = t < nseg;
        const uint32_t s = h + t * seg, e = min(s + seg, end_bits);
        uint32_t bm0 = 0, bm1 = 0, bm2 = 0, bm3 = 0;
        uint32_t xA = s, nA = 0, stA = ST_RUN;
        Rd r;
        r.zlast = (zend - 1) & ~(uintptr_t)15;
        if (act) {
            r.seek(zb, s);
            for (uint32_t o = 128 * t; o < zn_bytes; o += 128 * kT) warm ^= *(const OGE_G uint32_t *)(zn + o);  // next block -> L2
            zn_bytes = 0;
            uint32_t p = s, n = 0;
            while (p < e) {
                const uint32_t rel = p - s;
                if (rel < kWin) {
                    const uint32_t bit = 1u << (rel & 31), wsel = rel >> 5;
                    bm0 |= wsel == 0 ? bit : 0u;
                    bm1 |= wsel == 1 ? bit : 0u;
                    bm2 |= wsel == 2 ? bit : 0u;
                    bm3 |= wsel == 3 ? bit : 0u;
                }
                Sym y;
                dsym(r, S, y);
                if (y.kind == K_BAD) { stA = ST_BAD; break; }
                p += y.bits;
                n += y.len;
                if (y.kind == K_EOB) { stA = ST_EOB; break; }
            }
            xA = p;
            nA = n;
            S.exits[t] = p;
        }
        // ---- pass B: synchronise with the true entry x_{t-1}
        uint32_t vE = s, x = xA, n = nA, st = stA;
        __syncthreads();
        TMARK(4);
        uint32_t nrounds = 0;
        for (;;) {
            ++nrounds;
            __syncthreads();
            const uint32_t E = t == 0 ? h : (act ? S.exits[t - 1] : 0u);
            __syncthreads();
            int ch = 0;
            if (act && t > 0 && E != vE) {
                vE = E;
                uint32_t nx, nn = 0, ns = ST_RUN;
                bool synced = false;
                r.seek(zb, E);
                uint32_t p = E;
                for (;;) {
                    {  // did pass A start a symbol at p?
                        const uint32_t rel = p - s, wsel = rel >> 5;
                        const uint32_t w = wsel == 0 ? bm0 : wsel == 1 ? bm1 : wsel == 2 ? bm2 : bm3;
                        if (p >= s && rel < kWin && ((w >> (rel & 31)) & 1)) { synced = true; break; }
                    }
                    if (p >= e) break;
                    Sym y;
                    dsym(r, S, y);
                    if (y.kind == K_BAD) { ns = ST_BAD; break; }
                    p += y.bits;
                    nn += y.len;
                    if (y.kind == K_EOB) { ns = ST_EOB; break; }
                }
                if (synced) {  // pass A's path from p on is the true one: its count minus its count up to p
                    uint32_t c = 0, q = s;
                    r.seek(zb, s);
                    while (q < p) {
                        Sym y;
                        dsym(r, S, y);
                        if (y.kind == K_BAD) break;
                        q += y.bits;
                        c += y.len;
                    }
                    nx = xA;
                    nn = nn + nA - c;
                    ns = stA;
                } else {
                    nx = p;
                }
                ch = nx != x;
                x = nx, n = nn, st = ns;
                S.exits[t] = x;
            }
            if (!__syncthreads_or(ch)) break;
        }
        TMARK(5);
        if (tdbg) dbg[16 * kT + 20] = nrounds;
        // ---- the segment that ends this deflate block, output offsets
        if (t == 0) S.tstar = kT;
        __syncthreads();
        if (act && st != ST_RUN) atomicMin(&S.tstar, t);
        __syncthreads();
        const uint32_t ts = S.tstar;
        uint32_t total = 0;
        const uint32_t off = block_scan(S, act && t <= ts ? n : 0u, t, &total);
        if (ts == kT) { fail = E_PAST; break; }  // no end-of-block code before the data ends
        if (base + total > osz) { fail = E_OVERRUN; break; }
        if (dbg && b == dbg_blk && base == 0) {  // TEMP debug
            uint32_t *D = dbg + 16 * t;
            D[0] = s, D[1] = e, D[2] = xA, D[3] = nA, D[4] = stA, D[5] = vE, D[6] = x, D[7] = n, D[8] = st, D[9] = off;
            D[10] = h, D[11] = ts, D[12] = nseg, D[13] = seg, D[14] = act, D[15] = total;
        }
        __syncthreads();
        TMARK(11);
        TMARK(6);
        // ---- pass D: decode again and write the refs
        if (act && t <= ts) {
            r.seek(zb, vE);
            uint32_t p = vE, o = base + off;
            while (p < x) {
                Sym y;
                dsym(r, S, y);
                if (y.kind == K_BAD) break;
                p += y.bits;
                if (y.kind == K_LIT) {
                    if (o >= osz) {
                        S.berr = E_OVERRUN;
                        break;
                    }
                    S.refs[o++] = (uint16_t)(0xFF00u | y.val);
                } else if (y.kind == K_LEN) {
                    const uint32_t D = y.val, L = y.len;
                    if (D > o || o + L > osz) {
                        S.berr = D > o ? E_FAR : E_OVERRUN;
                        break;
                    }
                    uint32_t src = o - D;
                    const uint32_t s0 = src, stop = o;
                    if (o + L <= 0xFF00) {
                        for (uint32_t j = 0; j < L; ++j) {
                            S.refs[o + j] = (uint16_t)src;
                            if (++src == stop) src = s0;
                        }
                    } else {  // the end of a payload over 65280 bytes
                        for (uint32_t j = 0; j < L; ++j) {
                            const uint32_t q = o + j;
                            if (q >= 0xFF00) S.side[q - 0xFF00] = (uint16_t)src, S.refs[q] = 0xFF00;
                            else S.refs[q] = (uint16_t)src;
                            if (++src == stop) src = s0;
                        }
                    }
                    o += L;
                } else {
                    break;  // end of block
                }
            }
            if (!S.berr && o != base + off + n) S.berr = E_SEG;  // pass D wrote what passes A/B counted
        }
        // the closing segment: end of block (next header at its exit) or a bad code
        __syncthreads();
        if (t == ts) {
            S.h_err = st == ST_BAD ? (uint32_t)E_CODE : 0u;
            S.h_pos = x;
        }
        __syncthreads();
        if (S.berr) { fail = S.berr; break; }
        if (S.h_err) { fail = S.h_err; break; }
        base += total;
        pos = S.h_pos;
        if (fin) break;
    }
    if (!fail && base != osz) fail = E_SIZE;
    if (!fail && pos > end_bits) fail = E_PAST;
    if (fail) {
        if (t == 0) report(err, fail, b);
        return;  // uniform: every thread saw the same LDS flags
    }
    __syncthreads();

    TMARK(7);
    // ---- LZ: pointer jumping until every position holds a byte (chunks c = 1024 k + t of 8 positions)
    uint32_t actc = 0;
    for (uint32_t k = 0; k < kNCh; ++k)
        if (8 * (kT * k + t) < osz) actc |= 1u << k;
    for (int round = 0;; ++round) {
        int changed = 0;
        uint32_t m = actc;
        while (m) {
            const uint32_t k = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t q = 8 * (kT * k + t);
            const uint4 v = *(const uint4 *)(S.refs + q);
            const uint32_t r8[8] = {v.x & 0xffff, v.x >> 16, v.y & 0xffff, v.y >> 16, v.z & 0xffff, v.z >> 16, v.w & 0xffff, v.w >> 16};
            bool open = false;
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) open |= r8[i] < 0xFF00u;
            if (!open) {
                actc &= ~(1u << k);
                continue;
            }
            uint32_t rr[8];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) rr[i] = r8[i] < 0xFF00u ? S.refs[r8[i]] : r8[i];
            uint4 o;
            o.x = rr[0] | (rr[1] << 16), o.y = rr[2] | (rr[3] << 16), o.z = rr[4] | (rr[5] << 16), o.w = rr[6] | (rr[7] << 16);
            *(uint4 *)(S.refs + q) = o;
            changed = 1;
        }
        if (!__syncthreads_or(changed)) {
            if (tdbg) dbg[16 * kT + 21] = round;
            break;
        }
        if (round == 17) {  // depth <= 65536 needs at most 17 rounds
            if (t == 0) report(err, E_LZ, b);
            return;
        }
    }
    TMARK(8);
    // ---- bytes into the image (same LDS; padded rows: byte q at q + (q >> 6) * 4), CRC, write-out
    uint32_t cw[2 * kNCh];
#pragma unroll
    for (uint32_t k = 0; k < kNCh; ++k) {
        const uint4 v = *(const uint4 *)(S.refs + 8 * (kT * k + t));
        cw[2 * k] = (v.x & 0xff) | ((v.x >> 8) & 0xff00) | ((v.y & 0xff) << 16) | ((v.y >> 16) << 24);
        cw[2 * k + 1] = (v.z & 0xff) | ((v.z >> 8) & 0xff00) | ((v.w & 0xff) << 16) | ((v.w >> 16) << 24);
    }
    __syncthreads();
    constexpr int PS = 4;
    uint32_t *img32 = (uint32_t *)S.refs;
    uint8_t *img = (uint8_t *)S.refs;
#pragma unroll
    for (uint32_t k = 0; k < kNCh; ++k) {
        const uint32_t w = 2 * (kT * k + t);
        img32[pw<PS>(w)] = cw[2 * k];
        img32[pw<PS>(w) + 1] = cw[2 * k + 1];
    }
    auto ib = [](uint32_t q) { return q + ((q >> 6) << 2); };
    if (osz > 0xFF00) {  // copied bytes past position 0xFF00, in order (each source is final by then)
        __syncthreads();
        if (t == 0)
            for (uint32_t q = 0xFF00; q < osz; ++q)
                if (S.side[q - 0xFF00] != 0xFFFF) img[ib(q)] = img[ib(S.side[q - 0xFF00])];
    }
    __syncthreads();
    TMARK(9);
    if (crc) {
        const uint32_t c = kT == 1024 ? crc_window1024<PS>(img32, osz, S.crctab, S.zp, S.crcs, t)
                                      : crc_window512<PS>(img32, osz, S.crctab, S.zp, S.crcs, t);
        if (t == 0 && c != crc[b]) report(err, E_CRC, b);
    }
    TMARK(10);
    const uint32_t sh = (uint32_t)((uintptr_t)O & 3);
    OGE_G uint32_t *A = (OGE_G uint32_t *)((uintptr_t)O & ~(uintptr_t)3);
    const uint32_t nwords = (osz + sh + 3) / 4;
    for (uint32_t g = t; g < nwords; g += kT) {
        const int32_t r0 = (int32_t)(4 * g) - (int32_t)sh;
        if (r0 >= 0 && r0 + 4 <= (int32_t)osz) {
            A[g] = ld32p<PS>(img32, (uint32_t)r0);
        } else {
            for (int i = 0; i < 4; ++i) {
                const int32_t rq = r0 + i;
                if (rq >= 0 && rq < (int32_t)osz) ((OGE_G uint8_t *)(A + g))[i] = img[ib((uint32_t)rq)];
            }
        }
    }
    __syncthreads();
    TMARK(12);
#undef TMARK
}

// persistent workgroups (one per CU: the LDS allows no more), blocks b0 + i for i = blockIdx.x, + gridDim.x, ...
__global__ void __launch_bounds__(kT) k_infl_seg(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0a,
                                                  const uint64_t *__restrict__ d1a, const uint64_t *__restrict__ uoff,
                                                  const uint32_t *__restrict__ crc, uint64_t b0, uint64_t nb,
                                                  uint8_t *__restrict__ out, const uint32_t *__restrict__ zpow,
                                                  uint32_t *__restrict__ err, uint32_t *__restrict__ dbg, uint64_t dbg_blk) {
    __shared__ SegLds S;
    if (crc) crc_setup<kT>(S.crctab, S.zp, zpow, threadIdx.x);
    uint32_t warm = 0;
    for (uint64_t i = blockIdx.x; i < nb; i += gridDim.x) {
        const uint64_t nx = i + gridDim.x < nb ? b0 + i + gridDim.x : ~0ull;
        infl_block(S, z, zbytes, d0a, d1a, uoff, crc, out, err, dbg, dbg_blk, b0 + i, nx, warm);
        __syncthreads();  // the LDS is the next block's
    }
    if (warm == 0x9e3779b9u && threadIdx.x == kT - 1) err[3] = warm;  // (keeps the warm-up loads; err[3] is unused)
}

}  // namespace

// Inflate indexed blocks [0, nblk) with the segment decoder; err as in oge_bgzf_inflate_dev (err[0] bits,
// err[1] first failing block).  zpow: the CRC zero operators (device).
int oge_inflate_seg(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                    const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                    const uint32_t *zpow) {
    constexpr uint64_t kLaunch = 1u << 20;  // blocks per launch
    static int ncu = [] {
        int d = 0, n = 0;
        (void)hipGetDevice(&d);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
        return n > 0 ? n : 256;
    }();
    for (uint64_t b0 = 0; b0 < nblk; b0 += kLaunch) {
        const uint64_t nb = std::min(kLaunch, nblk - b0);
        static const char *dbe = getenv("OGE_INFL_DEBUG_BLOCK");  // TEMP debug
        uint32_t *dbg = dbe ? (uint32_t *)ctx->ws("infl_dbg", 17 * kT * 4) : nullptr;
        k_infl_seg<<<(uint32_t)std::min<uint64_t>(nb, ncu), kT, 0, ctx->stream>>>(d_z, zbytes, d0, d1, uoff, crc, b0, nb, out, zpow,
                                                                                 err, dbg, dbe ? (uint64_t)atoll(dbe) : ~0ull);
        if (dbg) {
            static uint32_t hb[17 * kT];
            (void)hipMemcpyAsync(hb, dbg, sizeof hb, hipMemcpyDeviceToHost, ctx->stream);
            (void)hipStreamSynchronize(ctx->stream);
            FILE *f = fopen(getenv("OGE_INFL_DEBUG_OUT"), "wb");
            if (f) fwrite(hb, 1, sizeof hb, f), fclose(f);
        }
        OGE_LAUNCH_CHECK(ctx);
    }
    return OGE_OK;
}
