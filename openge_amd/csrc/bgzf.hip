// bgzf.hip -- BGZF (blocked gzip) compression on the GPU, plus the device-side writer helpers
// (bin recompute, duplicate-record removal) that let FileWriter compress records where they sit.
//
// Replaces the host deflate of `BgzfOutputStream` (openge/src/util/bgzf_output_stream.cpp:59-250;
// deflateInit2(level,-15,8,Z_DEFAULT_STRATEGY) at :74-79, crc32 at :139) and the bin recompute of
// `BamSerializer::write` (util/bam_serializer.h:112-116).  Compressed bytes are not part of parity
// (only the decompressed stream is); every block is a complete RFC 1952 member with the
// BGZF `BC` extra field, so any gzip/BGZF reader inflates it.
//
// Layout: the input is cut into 65,280-byte payloads (htslib's framing, as the host writer uses).
// Each payload becomes one BGZF block holding one final deflate block with dynamic Huffman codes
// (or a stored block when that is smaller).  Three launches per chunk of blocks:
//
//   k_defl_tokens  one 512-thread workgroup per payload.  The payload is staged in LDS.  Match
//                  candidates come from a 4096-bucket hash of 4-byte prefixes, filled in rounds of
//                  512 consecutive positions (a position sees every earlier round, so the result is
//                  deterministic); each thread then greedily parses its own 64-byte segment into
//                  literal / (length, distance) tokens (matches end at the segment edge) and counts
//                  symbol frequencies.  Tokens go to global scratch, interleaved so every store of a
//                  wave is one contiguous line.  (152 KiB of LDS: one per CU, with room beside it for an
//                  emit or Huffman workgroup of the chunk another stream is on.)
//   k_defl_huff    one wave per payload: length-limited Huffman code lengths for the literal/length
//                  (15 bits), distance (15) and code-length (7) alphabets, canonical bit-reversed
//                  codes, and the block header bit string.
//   k_defl_emit    one 512-thread workgroup per payload: per-segment bit counts, a block scan for
//                  the bit offsets, then every thread writes its own bits (interior words with plain
//                  stores, the two edge words with atomicOr); the payload's CRC-32 from 128-byte pieces
//                  read from global memory, combined with zero-run operators; BGZF header and footer.
//   k_defl_compact copies the variable-size blocks from their 64 KiB slots to their final offsets.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bam_layout.h"
#include "oge_ctx.h"
#include "records.h"
#include "bgzf_dev.h"

namespace {

using namespace oge_bgzf;
constexpr int kT = 512;                   // threads per workgroup (tokens / emit)
constexpr int kSeg = 64;                  // bytes per thread segment
constexpr int kSub = kT * kSeg;           // 32768 positions per sub-block
constexpr int kNSub = 2;                  // sub-blocks per payload
constexpr int kNSeg = kT * kNSub;         // 1024 segments per payload
constexpr int kHashBits = 12;
constexpr int kLit = 286, kDist = 30, kCl = 19;
constexpr int kFreq = kLit + kDist;       // 316
constexpr int kHdrWords = 144;            // >= 4498 header bits

struct DeflTab {
    uint32_t lit[kLit];    // bit-reversed code | length << 16
    uint32_t dist[kDist];
    uint32_t hdr_bits;
    uint32_t hdr[kHdrWords];
};


__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashBits); }

// length 3..258 -> symbol 257..285, extra bits, extra value
__device__ __forceinline__ void len_code(uint32_t L, uint32_t &sym, uint32_t &nb, uint32_t &ev) {
    const uint32_t l = L - 3;
    if (l < 8) {
        sym = 257 + l, nb = 0, ev = 0;
    } else if (l == 255) {
        sym = 285, nb = 0, ev = 0;
    } else {
        const uint32_t lg = 31 - __builtin_clz(l);
        sym = 257 + 4 * (lg - 1) + ((l >> (lg - 2)) & 3);
        nb = lg - 2;
        ev = l & ((1u << nb) - 1);
    }
}

// distance 1..32768 -> code 0..29, extra bits, extra value
__device__ __forceinline__ void dist_code(uint32_t D, uint32_t &sym, uint32_t &nb, uint32_t &ev) {
    const uint32_t d = D - 1;
    if (d < 4) {
        sym = d, nb = 0, ev = 0;
    } else {
        const uint32_t lg = 31 - __builtin_clz(d);
        sym = 2 * lg + ((d >> (lg - 1)) & 1);
        nb = lg - 1;
        ev = d & ((1u << nb) - 1);
    }
}


// ------------------------------------------------------------------------------------ tokens
// tok layout: [(blk * kNSub + sub) * kSeg + k] * kT + t  (u32: literal byte, or a match at symbol
// level: 0x80000000 | (length symbol - 257) << 26 | length extra value << 21 | distance symbol << 16 |
// distance extra value, so k_defl_emit only looks codes up); ntok[(blk * kNSub + sub) * kT + t].
// zpow[k][32]: operator of feeding 2^k zero bytes through the (reflected) CRC-32 register.
// PS: padded layouts (bgzf_dev.h pw) -- every thread's 64-byte segment of `in` starts in its own bank
// for the greedy parse (PS = 4), or none (PS = 31).  The payload CRC is computed by k_defl_emit, so this
// kernel's LDS (one workgroup per CU) leaves room for an emit or Huffman workgroup of another chunk.
// R: positions per thread per candidate round (rounds of R * 512 consecutive positions; a position
// sees the hash table as the earlier rounds left it).  Fewer, fuller rounds cut the barriers per
// payload (128 at R = 1) at the price of not seeing the rest of its own round.
// LB: literals per parse step.  A position without a candidate is a literal, and so are the
// candidate-free positions right after it: a lane emits up to LB of them in one step, so a wave's
// step count (the maximum over its 64 segments) drops for literal-heavy payload (BAM qualities)
// while the tokens stay those of the one-symbol parse.
template <int PS, int R, int LB>
__global__ void __launch_bounds__(kT) k_defl_tokens(const uint8_t *__restrict__ src, uint64_t n, uint64_t blk0,
                                                    uint32_t *__restrict__ tok, uint8_t *__restrict__ ntok,
                                                    uint32_t *__restrict__ freq_out) {
    constexpr uint32_t kInW = kPay / 4 + 4 + (PS < 31 ? (kPay / 4 + 4) / (1u << PS) + 1 : 0);
    __shared__ uint32_t in[kInW];
    __shared__ uint32_t htab[1 << kHashBits];
    __shared__ uint16_t cand[kSub + 2 * (kSub / 64)];
    __shared__ uint32_t freq[kFreq];
    const int t = threadIdx.x;
    const uint64_t blk = blk0 + blockIdx.x;
    const uint64_t start = blk * kPay;
    const uint32_t len = (uint32_t)min<uint64_t>(kPay, n - start);
    const uint8_t *s = src + start;

    stage_words<kT, PS>(in, s, len, t);
    auto cix = [](uint32_t q) { return q + 2 * (q >> 6); };  // candidate q of the sub-block
    for (int i = t; i < (1 << kHashBits); i += kT) htab[i] = 0;
    for (int i = t; i < kFreq; i += kT) freq[i] = 0;
    __syncthreads();

    for (int sub = 0; sub < kNSub; ++sub) {
        const uint32_t base = sub * kSub;
        if (base >= len) {
            ntok[((uint64_t)blockIdx.x * kNSub + sub) * kT + t] = 0;
            continue;
        }
        const uint32_t end = min(len, base + kSub);
        // candidates, one round of R * kT consecutive positions at a time
        for (uint32_t r = base; r < end; r += R * kT) {
            uint32_t hh[R];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const uint32_t p = r + k * kT + t;
                uint32_t h = 0, c = 0;
                if (p + 4 <= len) {
                    const uint32_t w = ld32p<PS>(in, p);
                    h = hash4(w);
                    const uint32_t j1 = htab[h];
                    if (j1 && p - (j1 - 1) <= 32768 && ld32p<PS>(in, j1 - 1) == w) c = j1;
                }
                hh[k] = h;
                if (p < end) cand[cix(p - base)] = (uint16_t)c;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const uint32_t p = r + k * kT + t;
                if (p + 4 <= len && p < end) atomicMax(&htab[hh[k]], p + 1);
            }
            __syncthreads();
        }
        // greedy parse of this thread's segment
        const uint32_t s0 = base + t * kSeg, s1 = min(end, s0 + kSeg);
        uint32_t k = 0;
        uint32_t *tp = tok + ((uint64_t)blockIdx.x * kNSub + sub) * kSeg * kT + t;
        for (uint32_t p = s0; p < s1;) {
            const uint32_t c = p < s1 ? cand[cix(p - base)] : 0;
            if (LB > 1 && !c) {
#pragma unroll
                for (int q = 0; q < LB; ++q) {
                    if (q > 0 && (p >= s1 || cand[cix(p - base)] != 0)) break;
                    const uint32_t b = byte_at<PS>(in, p);
                    atomicAdd(&freq[b], 1u);
                    tp[(uint64_t)k * kT] = b;
                    ++k;
                    ++p;
                }
                continue;
            }
            uint32_t L = 0;
            if (c) {
                const uint32_t j = c - 1;
                const uint32_t maxL = min(258u, s1 - p);
                L = min(4u, maxL);
                if (LB > 1) {  // 8 bytes per step
                    while (L < maxL) {
                        const uint32_t x0 = ld32p<PS>(in, p + L) ^ ld32p<PS>(in, j + L);
                        const uint32_t x1 = ld32p<PS>(in, p + L + 4) ^ ld32p<PS>(in, j + L + 4);
                        if (x0) {
                            L += __builtin_ctz(x0) >> 3;
                            break;
                        }
                        if (x1) {
                            L += 4 + (__builtin_ctz(x1) >> 3);
                            break;
                        }
                        L += 8;
                    }
                } else {
                    while (L < maxL) {
                        const uint32_t x = ld32p<PS>(in, p + L) ^ ld32p<PS>(in, j + L);
                        if (x == 0) {
                            L += 4;
                        } else {
                            L += __builtin_ctz(x) >> 3;
                            break;
                        }
                    }
                }
                L = min(L, maxL);
            }
            uint32_t tokv;
            if (L >= 3) {
                const uint32_t d = p - (c - 1);
                uint32_t sym, nb, ev, dsym, dnb, dev;
                len_code(L, sym, nb, ev);
                atomicAdd(&freq[sym], 1u);
                dist_code(d, dsym, dnb, dev);
                atomicAdd(&freq[kLit + dsym], 1u);
                tokv = 0x80000000u | ((sym - 257) << 26) | (ev << 21) | (dsym << 16) | dev;
                p += L;
            } else {
                const uint32_t b = byte_at<PS>(in, p);
                tokv = b;
                atomicAdd(&freq[b], 1u);
                p += 1;
            }
            tp[(uint64_t)k * kT] = tokv;
            ++k;
        }
        ntok[((uint64_t)blockIdx.x * kNSub + sub) * kT + t] = (uint8_t)k;
        __syncthreads();  // cand is reused by the next sub-block
    }
    for (int i = t; i < kFreq; i += kT) freq_out[(uint64_t)blockIdx.x * kFreq + i] = freq[i];
}

// ------------------------------------------------------------------------------------ Huffman
// Code lengths for n symbols with frequencies f (LDS), limited to M bits.  Called by one whole wave.
// Huffman tree by the two-queue method over the symbols sorted by (freq, symbol); depths beyond M are
// clamped and the length counts repaired to an exactly complete code (Kraft sum 1); lengths are then
// handed out longest-first to the least frequent symbols.
struct HuffScratch {
    uint16_t sorted[kLit];
    uint32_t w[2 * kLit];
    uint16_t parent[2 * kLit];
    uint32_t cnt[16];
    uint32_t m;
};

__device__ void huff_lengths(const uint32_t *f, int n, int M, uint8_t *len, HuffScratch &hs) {
    const int lane = threadIdx.x;
    uint32_t m = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const uint32_t fi = i < n ? f[i] : 0;
        if (i < n) len[i] = 0;
        if (fi) {
            uint32_t r = 0;
            for (int j = 0; j < n; ++j) {
                const uint32_t fj = f[j];
                r += fj && (fj < fi || (fj == fi && j < i));
            }
            hs.sorted[r] = (uint16_t)i;
        }
        m += __popcll(__ballot(fi != 0));
    }
    __syncthreads();
    if (lane == 0) {
        if (m == 1) {
            len[hs.sorted[0]] = 1;
        } else if (m > 1) {
            for (uint32_t k = 0; k < m; ++k) hs.w[k] = f[hs.sorted[k]];
            uint32_t i = 0, j = m, nx = m;
            for (uint32_t c = 0; c + 1 < m; ++c) {
                uint32_t a, b;
                if (i < m && (j >= nx || hs.w[i] <= hs.w[j])) a = i++; else a = j++;
                if (i < m && (j >= nx || hs.w[i] <= hs.w[j])) b = i++; else b = j++;
                hs.w[nx] = hs.w[a] + hs.w[b];
                hs.parent[a] = (uint16_t)nx;
                hs.parent[b] = (uint16_t)nx;
                ++nx;
            }
            // depths, root first (w is reused for the depth)
            const uint32_t root = 2 * m - 2;
            hs.w[root] = 0;
            for (int x = (int)root - 1; x >= 0; --x) hs.w[x] = hs.w[hs.parent[x]] + 1;
            for (int b = 0; b < 16; ++b) hs.cnt[b] = 0;
            for (uint32_t k = 0; k < m; ++k) hs.cnt[min(hs.w[k], (uint32_t)M)]++;
            const uint32_t one = 1u << M;
            uint32_t K = 0;
            for (int b = 1; b <= M; ++b) K += hs.cnt[b] << (M - b);
            while (K > one) {  // over-subscribed after clamping: lengthen the longest code < M
                int b = M - 1;
                while (hs.cnt[b] == 0) --b;
                hs.cnt[b]--;
                hs.cnt[b + 1]++;
                K -= 1u << (M - b - 1);
            }
            while (K < one) {  // under-subscribed: shorten the longest code that still fits
                int b = M;
                while (hs.cnt[b] == 0 || K + (1u << (M - b)) > one) --b;
                hs.cnt[b]--;
                hs.cnt[b - 1]++;
                K += 1u << (M - b);
            }
            uint32_t k = 0;
            for (int b = M; b >= 1; --b)
                for (uint32_t c = 0; c < hs.cnt[b]; ++c) len[hs.sorted[k++]] = (uint8_t)b;
        }
    }
    __syncthreads();
}

// canonical codes, bit-reversed for LSB-first emission: out[i] = rcode | len << 16
__device__ void huff_codes(const uint8_t *len, int n, uint32_t *out) {
    const int lane = threadIdx.x;
    __shared__ uint32_t first[16];
    if (lane == 0) {
        uint32_t cnt[16] = {0};
        for (int i = 0; i < n; ++i) cnt[len[i]]++;
        cnt[0] = 0;
        uint32_t code = 0;
        for (int b = 1; b < 16; ++b) {
            code = (code + cnt[b - 1]) << 1;
            first[b] = code;
        }
    }
    __syncthreads();
    for (int i = lane; i < n; i += 64) {
        const uint32_t L = len[i];
        uint32_t v = 0;
        if (L) {
            uint32_t r = 0;
            for (int j = 0; j < i; ++j) r += len[j] == L;
            const uint32_t code = first[L] + r;
            v = (__builtin_bitreverse32(code) >> (32 - L)) | (L << 16);
        }
        out[i] = v;
    }
    __syncthreads();
}

__constant__ uint8_t kClOrder[kCl] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__global__ void __launch_bounds__(64) k_defl_huff(const uint32_t *__restrict__ freq_in, DeflTab *__restrict__ tabs) {
    __shared__ uint32_t f[kFreq];
    __shared__ uint8_t lens[kFreq];
    __shared__ uint32_t fcl[kCl];
    __shared__ uint8_t lcl[kCl];
    __shared__ uint32_t ccl[kCl];
    __shared__ uint8_t cl_sym[kFreq], cl_ext[kFreq];
    __shared__ uint32_t ncl;
    __shared__ HuffScratch hs;
    const int lane = threadIdx.x;
    DeflTab &T = tabs[blockIdx.x];
    for (int i = lane; i < kFreq; i += 64) f[i] = freq_in[(uint64_t)blockIdx.x * kFreq + i];
    __syncthreads();
    if (lane == 0) {
        f[256] = 1;  // end of block
        // at least two used codes per tree (a one-code tree would be incomplete)
        uint32_t nz = 0;
        for (int i = 0; i < kLit; ++i) nz += f[i] != 0;
        for (int i = 0; nz < 2 && i < kLit; ++i)
            if (!f[i]) f[i] = 1, ++nz;
        nz = 0;
        for (int i = 0; i < kDist; ++i) nz += f[kLit + i] != 0;
        for (int i = 0; nz < 2 && i < kDist; ++i)
            if (!f[kLit + i]) f[kLit + i] = 1, ++nz;
    }
    __syncthreads();
    huff_lengths(f, kLit, 15, lens, hs);
    huff_lengths(f + kLit, kDist, 15, lens + kLit, hs);
    huff_codes(lens, kLit, T.lit);
    huff_codes(lens + kLit, kDist, T.dist);

    // run-length code the two length sequences separately (RFC 1951 3.2.7)
    __shared__ uint32_t hlit, hdist;
    if (lane == 0) {
        int a = kLit;
        while (a > 257 && lens[a - 1] == 0) --a;
        int b = kDist;
        while (b > 1 && lens[kLit + b - 1] == 0) --b;
        hlit = a;
        hdist = b;
        for (int i = 0; i < kCl; ++i) fcl[i] = 0;
        uint32_t q = 0;
        for (int part = 0; part < 2; ++part) {
            const uint8_t *L = part ? lens + kLit : lens;
            const int N = part ? b : a;
            for (int i = 0; i < N;) {
                const uint8_t v = L[i];
                int run = 1;
                while (i + run < N && L[i + run] == v) ++run;
                if (v == 0 && run >= 3) {
                    const int r = min(run, 138);
                    if (r >= 11) cl_sym[q] = 18, cl_ext[q] = (uint8_t)(r - 11);
                    else cl_sym[q] = 17, cl_ext[q] = (uint8_t)(r - 3);
                    fcl[cl_sym[q]]++;
                    ++q;
                    i += r;
                    continue;
                }
                cl_sym[q] = v, cl_ext[q] = 0, fcl[v]++, ++q;
                ++i;
                int rest = run - 1;
                if (v != 0) {
                    while (rest >= 3) {
                        const int r = min(rest, 6);
                        cl_sym[q] = 16, cl_ext[q] = (uint8_t)(r - 3), fcl[16]++, ++q;
                        rest -= r;
                        i += r;
                    }
                }
                // the (< 3) remaining equal values go round the loop as plain lengths
            }
        }
        ncl = q;
        uint32_t nz = 0;
        for (int i = 0; i < kCl; ++i) nz += fcl[i] != 0;
        for (int i = 0; nz < 2 && i < kCl; ++i)
            if (!fcl[i]) fcl[i] = 1, ++nz;
    }
    __syncthreads();
    huff_lengths(fcl, kCl, 7, lcl, hs);
    huff_codes(lcl, kCl, ccl);
    if (lane == 0) {
        int hclen = kCl;
        while (hclen > 4 && lcl[kClOrder[hclen - 1]] == 0) --hclen;
        uint64_t acc = 0;
        uint32_t nacc = 0, wi = 0, total = 0;
        auto put = [&](uint32_t v, uint32_t nb) {
            acc |= (uint64_t)v << nacc;
            nacc += nb;
            total += nb;
            if (nacc >= 32) {
                T.hdr[wi++] = (uint32_t)acc;
                acc >>= 32;
                nacc -= 32;
            }
        };
        put(1, 1);  // BFINAL
        put(2, 2);  // BTYPE = dynamic
        put(hlit - 257, 5);
        put(hdist - 1, 5);
        put(hclen - 4, 4);
        for (int i = 0; i < hclen; ++i) put(lcl[kClOrder[i]], 3);
        for (uint32_t i = 0; i < ncl; ++i) {
            const uint32_t s = cl_sym[i], c = ccl[s];
            put(c & 0xffff, c >> 16);
            if (s == 16) put(cl_ext[i], 2);
            else if (s == 17) put(cl_ext[i], 3);
            else if (s == 18) put(cl_ext[i], 7);
        }
        if (nacc) T.hdr[wi++] = (uint32_t)acc;
        T.hdr_bits = total;
    }
}

// ------------------------------------------------------------------------------------ emit
struct BitW {
    uint32_t *base;
    uint64_t acc;
    uint32_t nacc;
    uint32_t wpos;
    bool first;
    __device__ void init(uint32_t *b, uint32_t bit) {
        base = b, acc = 0, nacc = bit & 31, wpos = bit >> 5, first = true;
    }
    __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {
        acc |= (uint64_t)v << nacc;
        nacc += nb;
        if (nacc >= 32) {
            const uint32_t w = (uint32_t)acc;
            if (first) atomicOr(base + wpos, w), first = false;
            else base[wpos] = w;
            ++wpos;
            acc >>= 32;
            nacc -= 32;
        }
    }
    __device__ void finish() {
        if (nacc && (uint32_t)acc) atomicOr(base + wpos, (uint32_t)acc);
    }
};

// extra-bit counts of a length symbol - 257 (0..28) and of a distance symbol (0..29)
__device__ __forceinline__ uint32_t len_extra(uint32_t ls) { return ls < 8 ? 0u : ls < 28 ? (ls - 4) >> 2 : 0u; }
__device__ __forceinline__ uint32_t dist_extra(uint32_t ds) { return ds < 4 ? 0u : (ds - 2) >> 1; }

__device__ __forceinline__ uint32_t tok_bits(uint32_t v, const uint32_t *lit, const uint32_t *dist) {
    if (!(v >> 31)) return lit[v] >> 16;
    const uint32_t ls = (v >> 26) & 31, ds = (v >> 16) & 31;
    return (lit[257 + ls] >> 16) + len_extra(ls) + (dist[ds] >> 16) + dist_extra(ds);
}


// zpow[k][32]: operator of feeding 2^k zero bytes through the (reflected) CRC-32 register
__global__ void __launch_bounds__(kT) k_defl_emit(const uint8_t *__restrict__ src, uint64_t n, uint64_t blk0, int level,
                                                  const uint32_t *__restrict__ tok, const uint8_t *__restrict__ ntok,
                                                  const DeflTab *__restrict__ tabs, const uint32_t *__restrict__ zpow,
                                                  uint8_t *__restrict__ slots, uint32_t *__restrict__ sizes) {
    __shared__ uint32_t lit[kLit], dist[kDist];
    __shared__ uint32_t scan[kNSeg];
    __shared__ uint32_t wsum[kT / 64];
    __shared__ uint32_t sh_total, sh_stored, sh_crc;
    __shared__ uint32_t crctab[1][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t crcs[kT / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t blk = blk0 + blockIdx.x;
    const uint64_t start = blk * kPay;
    const uint32_t len = (uint32_t)min<uint64_t>(kPay, n - start);
    const uint8_t *s = src + start;
    const DeflTab &T = tabs[blockIdx.x];
    for (int i = t; i < kLit; i += kT) lit[i] = T.lit[i];
    for (int i = t; i < kDist; i += kT) dist[i] = T.dist[i];
    crc_setup<kT, 1>(crctab, zp, zpow, t);
    __syncthreads();
    {  // payload CRC-32 from global memory (the tokens kernel keeps its LDS for the match search)
        const uint32_t c = crc_global512(s, len, crctab, zp, crcs, t);
        if (t == 0) sh_crc = c;
    }

    // bit counts per segment, in stream order (sub-block 0 segments then sub-block 1)
    uint32_t cnt[kNSub];
    for (int sub = 0; sub < kNSub; ++sub) {
        const uint32_t nt = ntok[((uint64_t)blockIdx.x * kNSub + sub) * kT + t];
        const uint32_t *tp = tok + ((uint64_t)blockIdx.x * kNSub + sub) * kSeg * kT + t;
        uint32_t b = 0;
        for (uint32_t k0 = 0; k0 < nt; k0 += 8) {  // every segment owns kSeg token slots: batch the loads
            uint32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = tp[(uint64_t)min(k0 + j, (uint32_t)kSeg - 1) * kT];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (k0 + j < nt) b += tok_bits(v[j], lit, dist);
        }
        cnt[sub] = b;
        scan[sub * kT + t] = b;
    }
    __syncthreads();
    // exclusive scan of scan[0..kNSeg): thread t owns entries 2t, 2t + 1
    {
        const uint32_t a = scan[2 * t], b = scan[2 * t + 1];
        uint32_t x = a + b, inc = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wv; ++w) pre += wsum[w];
        const uint32_t ex = pre + inc - x;
        __syncthreads();
        scan[2 * t] = ex;
        scan[2 * t + 1] = ex + a;
        if (t == kT - 1) {
            const uint32_t body = ex + x;
            const uint32_t bits = T.hdr_bits + body + (lit[256] >> 16);
            const uint32_t dbytes = (bits + 7) / 8;
            sh_stored = level == 0 || dbytes > len + 5;
            sh_total = sh_stored ? 18 + 5 + len + 8 : 18 + dbytes + 8;
        }
    }
    __syncthreads();
    const uint32_t total = sh_total;
    const bool stored = sh_stored;
    uint8_t *out = slots + (uint64_t)blockIdx.x * kSlot;
    uint32_t *ow = (uint32_t *)out;
    // zero what the block will occupy (atomicOr targets included)
    for (uint32_t i = t; i < (total + 15) / 16; i += kT) ((uint4 *)out)[i] = make_uint4(0, 0, 0, 0);
    // workgroup-scope release/acquire (in __syncthreads) orders these stores before the atomics of
    // other waves; a device-scope __threadfence would write back the XCD's L2 on gfx950
    __syncthreads();
    if (t == 0) {
        ow[0] = 0x04088b1fu;  // ID1 ID2 CM=8 FLG=FEXTRA
        ow[1] = 0;            // MTIME
        ow[2] = 0x0006ff00u;  // XFL=0 OS=255 XLEN=6
        ow[3] = 0x00024342u;  // 'B' 'C' SLEN=2
    }
    const uint32_t bsize = total - 1;
    if (stored) {
        if (t == 0) {
            out[16] = (uint8_t)bsize, out[17] = (uint8_t)(bsize >> 8);
            out[18] = 1;
            out[19] = (uint8_t)len, out[20] = (uint8_t)(len >> 8);
            out[21] = (uint8_t)~len, out[22] = (uint8_t)(~len >> 8);
        }
        for (uint32_t i = t; i < len; i += kT) out[23 + i] = s[i];
        if (t == 0) {
            const uint32_t q = 23 + len;
            const uint32_t c = sh_crc;
            for (int b = 0; b < 4; ++b) out[q + b] = (uint8_t)(c >> (8 * b)), out[q + 4 + b] = (uint8_t)(len >> (8 * b));
        }
    } else {
        uint32_t *bw = ow + 4;  // stream bit 0 = bit 16 of word 4 (byte 18)
        if (t == 0) atomicOr(ow + 4, bsize & 0xffff);
        // header bits
        const uint32_t hb = T.hdr_bits;
        for (uint32_t i = t; i < (hb + 31) / 32; i += kT) {
            const uint32_t v = T.hdr[i];
            atomicOr(bw + i, v << 16);
            if (v >> 16) atomicOr(bw + i + 1, v >> 16);
        }
        for (int sub = 0; sub < kNSub; ++sub) {
            if (!cnt[sub]) continue;
            const uint32_t nt = ntok[((uint64_t)blockIdx.x * kNSub + sub) * kT + t];
            const uint32_t *tp = tok + ((uint64_t)blockIdx.x * kNSub + sub) * kSeg * kT + t;
            BitW w;
            w.init(bw, 16 + hb + scan[sub * kT + t]);
            for (uint32_t k0 = 0; k0 < nt; k0 += 8) {
              uint32_t vv[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) vv[j] = tp[(uint64_t)min(k0 + j, (uint32_t)kSeg - 1) * kT];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                if (k0 + j >= nt) break;
                const uint32_t v = vv[j];
                if (!(v >> 31)) {
                    const uint32_t c = lit[v];
                    w.put(c & 0xffff, c >> 16);
                } else {
                    const uint32_t ls = (v >> 26) & 31, ds = (v >> 16) & 31;
                    const uint32_t c = lit[257 + ls];
                    w.put((c & 0xffff) | (((v >> 21) & 31) << (c >> 16)), (c >> 16) + len_extra(ls));
                    const uint32_t d = dist[ds];
                    w.put((d & 0xffff) | ((v & 0x1fff) << (d >> 16)), (d >> 16) + dist_extra(ds));
                }
              }
            }
            w.finish();
        }
        if (t == kT - 1) {
            const uint32_t body_end = 16 + hb + scan[kNSeg - 1] + cnt[kNSub - 1];
            BitW w;
            w.init(bw, body_end);
            const uint32_t c = lit[256];
            w.put(c & 0xffff, c >> 16);  // first flush of a BitW is an atomicOr, as is finish()
            w.finish();
            // footer: CRC32, ISIZE right after the last (zero-padded) deflate byte
            const uint32_t q = 18 + (body_end - 16 + (c >> 16) + 7) / 8;
            const uint64_t v = (uint64_t)sh_crc | ((uint64_t)len << 32);
            const uint32_t wi = q >> 2, shb = (q & 3) * 8;
            const uint64_t sv = v << shb;
            atomicOr(ow + wi, (uint32_t)sv);
            atomicOr(ow + wi + 1, (uint32_t)(sv >> 32));
            if (shb) atomicOr(ow + wi + 2, (uint32_t)(v >> (64 - shb)));
        }
    }
    if (t == 0) sizes[blockIdx.x] = total;
}

__global__ void __launch_bounds__(256) k_defl_compact(const uint8_t *__restrict__ slots, const uint32_t *__restrict__ sizes,
                                                      const uint32_t *__restrict__ offs, const uint64_t *__restrict__ base,
                                                      uint8_t *__restrict__ dst) {
    const uint8_t *s = slots + (uint64_t)blockIdx.x * kSlot;
    uint8_t *d = dst + *base + offs[blockIdx.x];
    const uint32_t sz = sizes[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < sz; i += blockDim.x) d[i] = s[i];
}

// exclusive scan of n <= 8192 block sizes, one 1024-thread workgroup, 8 consecutive entries per thread
// (the per-chunk offsets; runs on the chunk's own stream)
constexpr uint32_t kMaxChunk = 8192;
__global__ void __launch_bounds__(1024) k_scan_chunk(const uint32_t *__restrict__ in, uint32_t n, uint32_t *__restrict__ out) {
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t a[8], v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = 8 * t + i < n ? in[8 * t + i] : 0u;
        v += a[i];
    }
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    if (t < 16) {
        uint32_t s = ws[t], z = s;
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t y = __shfl_up(z, d, 16);
            if ((t & 15) >= (uint32_t)d) z += y;
        }
        ws[t] = z - s;
    }
    __syncthreads();
    uint32_t excl = ws[w] + x - v;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (8 * t + i < n) out[8 * t + i] = excl;
        excl += a[i];
    }
}

__global__ void k_defl_advance(uint64_t *base, const uint32_t *offs, const uint32_t *sizes, uint32_t nb) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *base += (uint64_t)offs[nb - 1] + sizes[nb - 1];
}

// ------------------------------------------------------------------------------------ records
__global__ void k_fix_bins(uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *r = recs + off[i];
    oge_wr_u16(r + OGE_OFF_BIN, oge_rec_bin(r));
}

}  // namespace


extern "C" uint64_t oge_bgzf_bound(uint64_t n) { return ((n + kPay - 1) / kPay) * (uint64_t)kSlot; }

extern "C" int oge_bgzf_deflate_dev(oge_ctx *ctx, const uint8_t *d_src, uint64_t n, int level, uint8_t *d_dst,
                                    uint64_t dst_cap, uint64_t *out_bytes) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!out_bytes || (n && (!d_src || !d_dst))) return oge_fail(ctx, OGE_ERR_ARG, "null buffer");
    if (level < 0 || level > 9) return oge_fail(ctx, OGE_ERR_ARG, "level must be 0..9");
    if (dst_cap < oge_bgzf_bound(n)) return oge_fail(ctx, OGE_ERR_ARG, "dst_cap < oge_bgzf_bound(n)");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    *out_bytes = 0;
    if (!n) return OGE_OK;
    const uint64_t nblk = (n + kPay - 1) / kPay;
    // payloads per chunk: one launch of each kernel.  The Huffman kernel is one serial chain per payload
    // (latency-bound, little LDS): more payloads per launch amortise that latency.  OGE_DEFL_CHUNK
    // overrides (256..8192).
    static const uint64_t chunk_max = [] {
        const char *e = getenv("OGE_DEFL_CHUNK");
        const long v = e ? atol(e) : 4096;
        return (uint64_t)std::min<long>(std::max<long>(v, 256), kMaxChunk);
    }();
    const uint64_t chunk = std::min<uint64_t>(nblk, chunk_max);
    // OGE_DEFL_CAND_R = 1 | 2 | 4: positions per thread per candidate round.  20M C2 reads: 70.0 / 72.2 /
    // 72.5 GB/s at ratio 0.6991 / 0.7007 / 0.7030 (profiles/r02s3_defl_r.json): 2 by default
    static const int cand_r = [] {
        const char *e = getenv("OGE_DEFL_CAND_R");
        return e && *e ? atoi(e) : 2;
    }();
    // OGE_DEFL_LITB = 1 | 2 | 4 | 8 | 16: literals per parse step (with R = 2; > 1 also extends matches 8
    // bytes per step).  The tokens are the same for every setting.  20M reads: 72.6 / 75.3 / 79.8 / 78.5 /
    // 72.6 GB/s for 1 / 2 / 4 / 8 / 16 (profiles/r02s3_defl_litb.json): 4 by default
    static const int lit_batch = [] {
        const char *e = getenv("OGE_DEFL_LITB");
        return e && *e ? atoi(e) : 4;
    }();
    static const bool pad = [] {  // OGE_DEFL_PAD=0: unpadded tokens LDS layout (A/B)
        const char *e = getenv("OGE_DEFL_PAD");
        return !(e && atoi(e) == 0);
    }();
    // Chunks go round-robin over S streams: one chunk's Huffman and emit kernels (small LDS) run on
    // the CUs beside another chunk's tokens workgroups (153 KiB of LDS, one per CU); only the
    // compaction, which advances the running output offset, is ordered chunk after chunk (events).
    const int S = nblk > chunk ? 3 : 1;
    struct Bufs {
        uint32_t *tok, *freq, *sizes, *offs;
        uint8_t *ntok, *slots;
        DeflTab *tabs;
        hipStream_t st;
    } B[3];
    for (int s = 0; s < S; ++s) {
        const std::string x = std::to_string(s);
        B[s].tok = (uint32_t *)ctx->ws(("defl_tok" + x).c_str(), chunk * kNSub * kSeg * kT * 4);
        B[s].ntok = (uint8_t *)ctx->ws(("defl_ntok" + x).c_str(), chunk * kNSeg);
        B[s].freq = (uint32_t *)ctx->ws(("defl_freq" + x).c_str(), chunk * kFreq * 4);
        B[s].tabs = (DeflTab *)ctx->ws(("defl_tabs" + x).c_str(), chunk * sizeof(DeflTab));
        B[s].slots = (uint8_t *)ctx->ws(("defl_slots" + x).c_str(), chunk * kSlot);
        B[s].sizes = (uint32_t *)ctx->ws(("defl_sizes" + x).c_str(), chunk * 4 + 16);
        B[s].offs = (uint32_t *)ctx->ws(("defl_offs" + x).c_str(), chunk * 4 + 16);
        B[s].st = S == 1 ? ctx->stream : ctx->side_stream(s);
        if (!B[s].tok || !B[s].ntok || !B[s].freq || !B[s].tabs || !B[s].slots || !B[s].sizes || !B[s].offs ||
            !B[s].st)
            return OGE_ERR_HIP;
    }
    uint32_t *zpow = (uint32_t *)ctx->ws("defl_zpow", 17 * 32 * 4);
    uint64_t *base = (uint64_t *)ctx->ws("defl_base", 16);
    if (!zpow || !base) return OGE_ERR_HIP;
    static uint32_t z[17][32];
    static bool zinit = false;
    if (!zinit) crc_zpow(z), zinit = true;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(zpow, z, sizeof(z), hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(base, 0, 8, ctx->stream));
    OgeStageTimer *tm = ctx->begin_stage("bgzf_deflate");
    hipEvent_t ev[4];
    for (auto &e : ev) OGE_HIP_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct Evs {
        hipEvent_t *e;
        ~Evs() {
            for (int i = 0; i < 4; ++i) hipEventDestroy(e[i]);
        }
    } evs{ev};
    OGE_HIP_TRY(ctx, hipEventRecord(ev[3], ctx->stream));  // inputs ready for the side streams
    for (int s = 0; s < S; ++s)
        if (B[s].st != ctx->stream) OGE_HIP_TRY(ctx, hipStreamWaitEvent(B[s].st, ev[3], 0));
    uint64_t k = 0;
    for (uint64_t b0 = 0; b0 < nblk; b0 += chunk, ++k) {
        const uint32_t nb = (uint32_t)std::min(chunk, nblk - b0);
        Bufs &u = B[k % S];
        if (!pad) k_defl_tokens<31, 1, 1><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (lit_batch >= 16) k_defl_tokens<4, 2, 16><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (lit_batch >= 8) k_defl_tokens<4, 2, 8><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (lit_batch >= 4 && cand_r >= 4) k_defl_tokens<4, 4, 4><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (lit_batch >= 4) k_defl_tokens<4, 2, 4><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (lit_batch == 2) k_defl_tokens<4, 2, 2><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (cand_r >= 4) k_defl_tokens<4, 4, 1><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else if (cand_r == 2) k_defl_tokens<4, 2, 1><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        else k_defl_tokens<4, 1, 1><<<nb, kT, 0, u.st>>>(d_src, n, b0, u.tok, u.ntok, u.freq);
        OGE_LAUNCH_CHECK(ctx);
        k_defl_huff<<<nb, 64, 0, u.st>>>(u.freq, u.tabs);
        OGE_LAUNCH_CHECK(ctx);
        k_defl_emit<<<nb, kT, 0, u.st>>>(d_src, n, b0, level, u.tok, u.ntok, u.tabs, zpow, u.slots, u.sizes);
        OGE_LAUNCH_CHECK(ctx);
        k_scan_chunk<<<1, 1024, 0, u.st>>>(u.sizes, nb, u.offs);
        OGE_LAUNCH_CHECK(ctx);
        if (k) OGE_HIP_TRY(ctx, hipStreamWaitEvent(u.st, ev[(k - 1) % S], 0));  // previous chunk's offset advance
        k_defl_compact<<<nb, 256, 0, u.st>>>(u.slots, u.sizes, u.offs, base, d_dst);
        OGE_LAUNCH_CHECK(ctx);
        k_defl_advance<<<1, 64, 0, u.st>>>(base, u.offs, u.sizes, nb);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipEventRecord(ev[k % S], u.st));
    }
    // the last chunk's advance follows every earlier compaction: the context stream waits for it
    if (S > 1) OGE_HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev[(k - 1) % S], 0));
    ctx->end_stage(tm);
    uint64_t total = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&total, base, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *out_bytes = total;
    return OGE_OK;
}

extern "C" int oge_bgzf_deflate(oge_ctx *ctx, const uint8_t *src, uint64_t n, int level, uint8_t *dst, uint64_t dst_cap,
                                uint64_t *out_bytes) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!out_bytes || (n && (!src || !dst))) return oge_fail(ctx, OGE_ERR_ARG, "null buffer");
    hipSetDevice(ctx->device);
    *out_bytes = 0;
    if (!n) return OGE_OK;
    const uint64_t bound = oge_bgzf_bound(n);
    uint8_t *ds = (uint8_t *)ctx->ws("defl_hsrc", n + 16);
    uint8_t *dd = (uint8_t *)ctx->ws("defl_hdst", bound);
    if (!ds || !dd) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(ds, src, n, hipMemcpyHostToDevice, ctx->stream));
    uint64_t got = 0;
    int rc = oge_bgzf_deflate_dev(ctx, ds, n, level, dd, bound, &got);
    if (rc) return rc;
    if (got > dst_cap) return oge_fail(ctx, OGE_ERR_ARG, "dst_cap too small for the compressed stream");
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dst, dd, got, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *out_bytes = got;
    return OGE_OK;
}

extern "C" int oge_fix_bins_dev(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    hipSetDevice(ctx->device);
    if (!n) return OGE_OK;
    k_fix_bins<<<oge_ceil_div(n, 256), 256, 0, ctx->stream>>>(d_recs, d_off, n);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}

