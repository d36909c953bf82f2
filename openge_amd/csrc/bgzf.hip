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
// (or a stored block when that is smaller).  Per chunk of 16384 payloads:
//
//   k_defl_parse   one 512-thread workgroup per payload, the payload in LDS: hash-table match candidates
//                  in rounds, a greedy parse of every 64-byte segment by its thread (literal runs
//                  skipped by mask), symbol frequencies; out: per segment a literal mask + its matches.
//   k_defl_huff    one wave per payload: length-limited Huffman code lengths for the literal/length
//                  (15 bits), distance (15) and code-length (7) alphabets, canonical bit-reversed
//                  codes, the block header bit string, and the exact block size (stored or dynamic).
//   k_scan_chunk / k_defl_advance   the blocks' offsets in the output stream.
//   k_defl_emit    one 512-thread workgroup per payload: segment bit counts, block scan, bits written
//                  into an LDS image of the whole BGZF block, CRC-32, then the block out at its final
//                  offset with coalesced stores.
// Deterministic: the same input gives the same bytes (the candidate rounds fix what each position sees).
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
constexpr int kT = 512;                   // threads per workgroup (parse / emit)
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
    uint32_t stored;       // 1: the block is written as one stored block
    uint32_t total;        // bytes of the whole BGZF block (header, deflate data, footer)
    uint32_t hdr[kHdrWords];
};



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


// ------------------------------------------------------------------------------------ parse
// One 512-thread workgroup per payload, the payload staged in LDS (unpadded).  Per sub-block of 32768
// positions (two per payload):
//   candidates  rounds of R * 512 consecutive positions: position p looks up the 4096-bucket hash of its
//               4-byte prefix (the table as the earlier rounds left it: deterministic), keeps the
//               candidate only if its 15-bit tag matches within 32 KiB (r06; the 4 bytes themselves are
//               compared where the parse visits it), then the round's positions enter the table
//               (atomicMax: the latest position wins).  A wave's 64 lanes hold 64 consecutive
//               positions = one 64-byte segment, so one ballot gives the segment's candidate mask.
//   parse       each thread greedily parses its own segment: literal runs are skipped with the mask
//               (ctz to the next candidate: no per-literal work in the serial chain); at a candidate the
//               match is extended 8 bytes per step and taken when >= 3 bytes (matches end at the segment
//               edge).  The same tokens as a one-symbol-at-a-time greedy parse.
//   counts      literal frequencies from the segment's literal mask (16-byte LDS reads, unrolled), length
//               and distance symbol frequencies at each match.
// Output per segment s (stream order: sub-block 0's 512 segments, then sub-block 1's): lmask[s] (bit i =
// byte i of the segment is a literal), nmatch[s], and the matches mlist[k][s] (k < nmatch[s]):
// offset in the segment << 23 | (length - 3) << 15 | (distance - 1).  About 8 B per payload byte less
// than a token per symbol (r02: 4-byte tokens written here and read twice by the emitter).
// Literal counts (levels 1-7) spread over kLC interleaved copies from word kLitCopies of the spare table, copy
// = thread & (kLC - 1), folded into the counts after the sub-block (r06): lanes counting the same byte value
// in one instruction hit the same LDS word, and the copies cut that serialisation (20M reads: deflate 26.3 ->
// 25.8 ms with 4 copies, 26.0 with 2, 26.1 with 8; the chained levels measured slower with them: 87.3 -> 90.5 ms)
constexpr int kLitCopies = 1024, kLC = 4;
constexpr int kMaxM = 21;   // matches per 64-byte segment (each >= 3 bytes)
#ifndef OGE_DEFL_TP
#define OGE_DEFL_TP 1024
#endif
// parse workgroup: 1024 threads (r04: 16 waves per CU instead of 8 hide the candidate rounds' chains of
// dependent LDS reads and their barriers; the same rounds of 1024 positions, so the same bytes: 20M reads
// 42.6 -> 37.8 ms); threads >= kT only take part in the staging and the candidate rounds
constexpr int kTP = OGE_DEFL_TP;  // a candidate round is kR * kTP = 1024 positions
constexpr int kR = 1024 / kTP;    // positions per thread per candidate round (r02: rounds of 512 / 1024 / 2048
                                  // positions -> ratio 0.6991 / 0.7007 / 0.7030)
static_assert(kR * kTP == 1024 && kTP >= kT, "round size and segment threads");

__device__ __forceinline__ uint64_t bits_below(uint32_t q) { return q >= 64 ? ~0ull : ((1ull << q) - 1); }

// Persistent (r04): workgroup blockIdx.x parses payloads i = blockIdx.x, + gridDim.x, ... < nb of the chunk,
// and loads payload i + gridDim.x's words into registers while payload i's last sub-block is parsed, so
// a payload's staging is a register -> LDS copy (r04: one workgroup per payload, ~8k of its ~112k cycles
// staging from HBM with the CU otherwise idle).
constexpr uint32_t kPre = kPay / 4 / kTP + 1;  // prefetched words per thread (16 for a full payload)

// depth > 1 (levels 8-9): at a candidate the parse also walks the chain of earlier positions with the same
// 4-byte prefix that the candidate array holds implicitly (cand[c] of a candidate c is c's own verified
// predecessor, so the chain never leaves the prefix; it ends at the sub-block's start) and takes the longest
// match of up to `depth` of them; with lazy, a match shorter than 32 bytes gives way to a literal when the
// next position's best match is longer (zlib's lazy evaluation).  depth 1 without lazy: the greedy parse.
template <bool CHAIN>  // depth > 1 (levels 8-9): exact candidates for the chain walks
__global__ void __launch_bounds__(kTP) k_defl_parse(const uint8_t *__restrict__ src, uint64_t n, uint64_t blk0, uint64_t nb,
                                                   uint64_t *__restrict__ lmask, uint8_t *__restrict__ nmatch,
                                                   uint32_t *__restrict__ mlist, uint32_t *__restrict__ freq_out, int depth,
                                                   int lazy) {
    // 163,600 B of LDS: the payload, two hash tables, the sub-block's candidates (the symbol counts live
    // in the table not in use while a sub-block is parsed; the candidate masks are read back from cand)
    __shared__ __align__(16) uint32_t in[kPay / 4 + 4];
    __shared__ uint32_t htab[2][1 << kHashBits];
    __shared__ __align__(16) uint16_t cand[kSub];
    const int t_ = threadIdx.x;
    // the payload's whole words when it starts 4-byte aligned (every payload does when src does: kPay is a
    // multiple of 4); otherwise stage_words reads them at the payload's start
    const bool al4 = ((uintptr_t)src & 3) == 0;
    uint32_t pre[kPre];
    auto fetch = [&](uint64_t i) {
        const uint64_t st0 = (blk0 + i) * kPay;
        const uint32_t ln = (uint32_t)min<uint64_t>(kPay, n - st0);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)(src + st0);
#pragma unroll
        for (uint32_t j = 0; j < kPre; ++j) {
            const uint32_t k = t_ + j * kTP;
            pre[j] = al4 && k < ln / 4 ? W[k] : 0u;
        }
    };
    auto fetch_or_clear = [&](uint64_t i) {  // registers defined on every path (see k_infl_lz)
        if (i < nb) {
            fetch(i);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < kPre; ++j) pre[j] = 0;
        }
    };
    fetch_or_clear(blockIdx.x);
    for (uint64_t pi = blockIdx.x; pi < nb; pi += gridDim.x) {
    int t = t_;
    __asm__ volatile("" : "+v"(t));  // per-payload index math stays in the loop (see k_infl_lz)
    const uint64_t blk = blk0 + pi;
    const uint64_t start = blk * kPay;
    const uint32_t len = (uint32_t)min<uint64_t>(kPay, n - start);

#if OGE_EXP == 4  // timing experiment: phase clocks of a parse workgroup (thread 0)
    uint64_t pc[12];
    int pn = 0;
#define PCLK() (pc[pn++] = __builtin_readcyclecounter())
#else
#define PCLK()
#endif
    PCLK();
    if (al4) {  // the prefetched words, then the zero-padded tail (as stage_words leaves it)
        const uint32_t safe = len / 4, nw = (len + 3) / 4;
#pragma unroll
        for (uint32_t j = 0; j < kPre; ++j) {
            const uint32_t k = t + j * kTP;
            if (k < safe) in[k] = pre[j];
        }
        for (uint32_t k = safe + t; k < nw + 4; k += kTP) {
            uint32_t v = 0;
            if (k < nw)
                for (int b = 0; b < 4; ++b)
                    if (4 * k + b < len) v |= (uint32_t)src[start + 4 * k + b] << (8 * b);
            in[k] = v;
        }
    } else {
        stage_words<kTP>(in, src + start, len, t);
    }
    for (int i = t; i < 2 << kHashBits; i += kTP) (&htab[0][0])[i] = 0;
    __syncthreads();
    PCLK();

    // Candidate rounds with one barrier each (r04; r03 had two: lookups, barrier, inserts, barrier).  Round
    // g looks up in htab[g & 1] and inserts into htab[(g + 1) & 1] both its own positions and round g - 1's:
    // at the start of round g, htab[g & 1] holds every position of the rounds before g (what r03's single
    // table held) and htab[(g + 1) & 1] those before g - 1, so the lookups see exactly r03's table -- the
    // same candidates, the same bytes -- while the inserts go to the other table.  20M reads: 32.24 ->
    // 32.09 ms only: a round is bound by its chain of dependent LDS reads and the bank conflicts of the
    // random bucket / candidate reads and atomics, not by its barriers.
    uint32_t g = 0;
    uint32_t hp[kR], vp[kR];  // the previous round's buckets and positions + 1 (0: nothing to insert)
#pragma unroll
    for (int k = 0; k < kR; ++k) hp[k] = 0, vp[k] = 0;
    static_assert(kNSub == 2, "f0 holds sub-block 0's counts while sub-block 1 reuses their table: two sub-blocks only");
    uint32_t f0 = 0;  // symbol t's count in sub-block 0 (kept while sub-block 1 reuses the table it was in)
    const uint64_t seg_base = pi * kNSeg;
    for (int sub = 0; sub < kNSub; ++sub) {
        const uint32_t base = sub * kSub;
        const uint64_t sg = seg_base + (uint64_t)sub * kT + t;  // this thread's segment, stream order
        if (base >= len) {
            if (t < kT) lmask[sg] = 0, nmatch[sg] = 0;
            continue;
        }
        const uint32_t end = min(len, base + kSub);
        if (sub > 0) {  // the spare table held sub-block 0's counts: keep them, then make it a copy of the full one
            uint32_t *F = htab[(g + 1) & 1];
            if (t < kFreq) f0 = F[t];
            __syncthreads();
            for (int i = t; i < (1 << kHashBits); i += kTP) F[i] = htab[g & 1][i];
            __syncthreads();
        }
        for (uint32_t r = base; r < end; r += kR * kTP, ++g) {
            const uint32_t *A = htab[g & 1];
            uint32_t *B = htab[(g + 1) & 1];
            // the kR lookup chains (prefix word -> bucket -> candidate's word) of a thread run side by side
            uint32_t hh[kR], cc[kR];
#pragma unroll
            for (int k = 0; k < kR; ++k) {
                const uint32_t p = r + k * kTP + t;
                uint32_t h = 0, c = 0;
                if (p + 4 <= len) {
                    const uint32_t w = ld32(in, p);
                    // bucket = the top 12 bits of the multiplicative hash.  Levels 1-7 (r06): entries are
                    // position + 1 << 15 | tag, the tag the hash's next 15 bits, so a bucket entry of another
                    // prefix is rejected in registers instead of by reading the candidate's bytes inside this
                    // chain of dependent LDS reads (20M reads: 27.15 -> 26.32 ms, the same bytes); the rare tag
                    // collisions are caught where the parse visits a candidate.  The chained levels keep
                    // entries of position + 1 and verify the 4 bytes here: every cand entry they walk is exact.
                    const uint32_t x = w * 2654435761u, tg = CHAIN ? 0u : (x >> 5) & 0x7fffu;
                    h = x >> (32 - kHashBits);
                    const uint32_t e = A[h], j1 = CHAIN ? e : e >> 15;
                    if (j1 && p - (j1 - 1) <= 32768 && (CHAIN ? ld32(in, j1 - 1) == w : (e & 0x7fffu) == tg)) c = j1;
                    h |= tg << 16;
                }
                hh[k] = h;
                cc[k] = c;
            }
#pragma unroll
            for (int k = 0; k < kR; ++k) {
                const uint32_t p = r + k * kTP + t;
                if (p < end) cand[p - base] = (uint16_t)cc[k];
                if (vp[k]) atomicMax(&B[hp[k]], vp[k]);
                const bool ins = p + 4 <= len && p < end;
                const uint32_t iv = CHAIN ? p + 1 : ((p + 1) << 15) | (hh[k] >> 16), hb = hh[k] & 0xffffu;
                if (ins) atomicMax(&B[hb], iv);
                hp[k] = hb;
                vp[k] = ins ? iv : 0u;
            }
            __syncthreads();
        }
        PCLK();
        if (sub == kNSub - 1 || base + kSub >= len) fetch_or_clear(pi + gridDim.x);  // under the last parse
        // the symbol counts of this sub-block go to the spare table (it is rebuilt before it is read again)
        uint32_t *freq = htab[(g + 1) & 1];
        for (int i = t; i < kFreq; i += kTP) freq[i] = 0;
        if (!CHAIN)
            for (int i = t; i < 256 * kLC; i += kTP) freq[kLitCopies + i] = 0;
        __syncthreads();
        // greedy parse of this thread's segment
        const uint32_t s0 = base + t * kSeg, s1 = min(end, s0 + kSeg);
        uint64_t lit = 0;
        uint32_t nm = 0;
        if (t < kT && s0 < s1) {
            const uint32_t sl = s1 - s0;
            uint64_t cm = 0;  // the segment's candidate mask, from its 64 cand entries (eight 16-byte reads)
            {
                const uint4 *cv = (const uint4 *)(cand + (s0 - base));
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint4 v = cv[q];
                    const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        cm |= (uint64_t)(((ww[i >> 1] >> (16 * (i & 1))) & 0xffff) != 0) << (8 * q + i);
                }
                cm &= bits_below(sl);
            }
            uint32_t *mp = mlist + (pi * kMaxM) * kNSeg + (uint64_t)sub * kT + t;
            // match length of candidate j at payload position pq (their first 4 bytes are equal), <= maxL
            auto ext = [&](uint32_t pq, uint32_t j, uint32_t maxL) {
                uint32_t L = min(4u, maxL);
                while (L < maxL) {  // 8 bytes per step
                    const uint32_t x0 = ld32(in, pq + L) ^ ld32(in, j + L);
                    const uint32_t x1 = ld32(in, pq + L + 4) ^ ld32(in, j + L + 4);
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
                return min(L, maxL);
            };
            // the best match at segment offset q (a candidate position): its candidate, then (depth > 1) the
            // chain of earlier same-prefix positions through cand; *jo = the source of the longest (the
            // nearest of equal lengths)
            auto best = [&](uint32_t q, uint32_t *jo) {
                const uint32_t pq = s0 + q, maxL = min(258u, sl - q);
                uint32_t j = cand[pq - base] - 1;
                if (!CHAIN && ld32(in, pq) != ld32(in, j)) {  // a tag collision: no candidate (a literal)
                    *jo = j;
                    return 0u;
                }
                uint32_t L = ext(pq, j, maxL), bj = j;
                for (int d = 1; CHAIN && d < depth && L < maxL; ++d) {
                    if (j < base) break;
                    const uint32_t nx = cand[j - base];
                    if (!nx || pq - (nx - 1) > 32768) break;
                    j = nx - 1;
                    const uint32_t Lj = ext(pq, j, maxL);
                    if (Lj > L) L = Lj, bj = j;
                }
                *jo = bj;
                return L;
            };
            for (uint32_t p = 0; p < sl;) {
                const uint64_t m = cm & ~bits_below(p);
                const uint32_t q = m ? (uint32_t)__builtin_ctzll(m) : sl;
                lit |= bits_below(q) & ~bits_below(p);  // literals [p, q)
                if (q >= sl) break;
                const uint32_t pq = s0 + q;
                uint32_t j;
                const uint32_t L = best(q, &j);
                if (CHAIN && lazy && L >= 3 && L < 32 && q + 1 < sl && ((cm >> (q + 1)) & 1)) {
                    uint32_t j1;
                    if (best(q + 1, &j1) > L) {  // a literal here, the longer match from the next position
                        lit |= 1ull << q;
                        p = q + 1;
                        continue;
                    }
                }
                if (L >= 3) {
                    const uint32_t d = pq - j;
                    uint32_t sym, nb, ev, dsym, dnb, dev;
                    len_code(L, sym, nb, ev);
                    dist_code(d, dsym, dnb, dev);
                    atomicAdd(&freq[sym], 1u);
                    atomicAdd(&freq[kLit + dsym], 1u);
                    mp[(uint64_t)nm * kNSeg] = (q << 23) | ((L - 3) << 15) | (d - 1);
                    ++nm;
                    p = q + L;
                } else {
                    lit |= 1ull << q;
                    p = q + 1;
                }
            }
            // literal frequencies: the segment's 64 bytes in four 16-byte LDS reads
            const uint4 *v4 = (const uint4 *)(in + s0 / 4);
#pragma unroll
            for (int w4 = 0; w4 < 4; ++w4) {
                const uint4 v = v4[w4];
                const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if ((lit >> (16 * w4 + k)) & 1) {
                        const uint32_t b = (ww[k >> 2] >> (8 * (k & 3))) & 0xff;
                        atomicAdd(&freq[CHAIN ? b : kLitCopies + b * kLC + (t & (kLC - 1))], 1u);
                    }
            }
        }
        if (t < kT) lmask[sg] = lit, nmatch[sg] = (uint8_t)nm;
        __syncthreads();  // cand and the counts are reused by the next sub-block
        if (!CHAIN) {  // the literal copies folded into the counts
            if (t < 256) {
                uint32_t c = 0;
#pragma unroll
                for (int q = 0; q < kLC; ++q) c += freq[kLitCopies + t * kLC + q];
                freq[t] += c;
            }
            __syncthreads();
        }
        PCLK();
    }
    // counts: sub-block 0's (kept in f0 when sub-block 1 ran) + those in the spare table
    static_assert(kFreq <= kTP, "one count per thread");
    if (t < kFreq) freq_out[pi * kFreq + t] = f0 + htab[(g + 1) & 1][t];
#if OGE_EXP == 4
    if (t == 0 && blockIdx.x < 4 && blk0 == 0)
        printf("parse-exp blk %u: stage %llu | sub0 rounds %llu parse+counts %llu | sub1 rounds %llu parse+counts %llu\n", blockIdx.x,
               (unsigned long long)(pc[1] - pc[0]), (unsigned long long)(pc[2] - pc[1]), (unsigned long long)(pc[3] - pc[2]),
               (unsigned long long)(pc[4] - pc[3]), (unsigned long long)(pc[5] - pc[4]));
#endif
#undef PCLK
    __syncthreads();  // the counts read out of htab before the next payload clears it
    }
}

// ------------------------------------------------------------------------------------ Huffman
// Code lengths for n symbols with frequencies f (LDS), limited to M bits.  Called by one whole wave.
// Huffman tree by the two-queue method over the symbols sorted by (freq, symbol); depths beyond M are
// clamped and the length counts repaired to an exactly complete code (Kraft sum 1); lengths are then
// handed out longest-first to the least frequent symbols.
struct HuffScratch {
    uint16_t sorted[kLit];
    uint32_t w[2 * kLit];      // the leaves' weights (+ 2 sentinels), later the node depths
    uint32_t nw[kLit + 2];     // the internal nodes' weights, in creation order (+ sentinels)
    uint64_t pick[(kLit + 31) / 32];  // the merge's picks, 2 bits per node: leaf first, leaf second
    uint16_t parent[2 * kLit]; // parent node, later the pointer-jumping ancestor
    uint32_t cnt[16];
    uint32_t m;
};
static_assert(2 * kLit >= 512, "the sort keys live in HuffScratch::w");

// One wave, everything but the two-queue merge lane-parallel (r03: the r02 version ran the depth walk,
// the depth counts and the length hand-out as serial lane-0 loops over LDS, one LDS round trip per step;
// the same lengths, so the same compressed bytes).
// Bitonic sort of S <= 512 keys held 8 per lane (key index = 8 lane + e), ascending: stages whose partner
// lies in the same lane compare registers, the others exchange through a lane shuffle -- no LDS, no barriers
// (r06; the r03-r05 network ran its 45 stages on LDS with a barrier each)
template <int S>
__device__ __forceinline__ void sort8(uint32_t (&key)[8], uint32_t lane) {
#pragma unroll
    for (uint32_t k = 2; k <= (uint32_t)S; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j >= 8) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const uint32_t idx = 8 * lane + (uint32_t)e;
                    const uint32_t y = (uint32_t)__shfl_xor((int)key[e], (int)(j >> 3), 64);
                    const bool up = (idx & k) == 0, lower = (idx & j) == 0;
                    const uint32_t mn = min(key[e], y), mx = max(key[e], y);
                    key[e] = (up == lower) ? mn : mx;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if ((uint32_t)e & j) continue;
                    const int e2 = e | (int)j;
                    const uint32_t idx = 8 * lane + (uint32_t)e;
                    const bool up = (idx & k) == 0;
                    const uint32_t x = key[e], y = key[e2];
                    if ((x > y) == up) key[e] = y, key[e2] = x;
                }
            }
        }
    }
}

#if OGE_EXP == 3
__device__ uint64_t g_hl_clk[8];  // timing experiment: huff_lengths' phase clocks of block 0, literal alphabet
#define HLCLK(k) do { if (n == kLit && blockIdx.x == 0 && threadIdx.x == 0) g_hl_clk[k] = __builtin_readcyclecounter(); } while (0)
#else
#define HLCLK(k) do { } while (0)
#endif
__device__ void huff_lengths(const uint32_t *f, int n, int M, uint8_t *len, HuffScratch &hs) {
    const int lane = threadIdx.x;
    HLCLK(0);
    // the used symbols ranked by (frequency, symbol): keys f << 9 | symbol (f <= 65281), unused slots
    // 0xffffffff, sorted in registers by the wave (8 keys per lane, 512 slots at most)
    uint32_t m = 0;
    const uint32_t S = n <= 32 ? 32u : n <= 64 ? 64u : n <= 128 ? 128u : n <= 256 ? 256u : 512u;  // sorted slots
    uint32_t key[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int i = 8 * lane + e;
        const uint32_t fi = i < n ? f[i] : 0;
        if (i < n) len[i] = 0;
        key[e] = fi ? (fi << 9) | (uint32_t)i : 0xffffffffu;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) m += __popcll(__ballot(key[e] != 0xffffffffu));  // every lane in every ballot
    HLCLK(1);
    switch (S) {
    case 32: sort8<32>(key, lane); break;
    case 64: sort8<64>(key, lane); break;
    case 128: sort8<128>(key, lane); break;
    case 256: sort8<256>(key, lane); break;
    default: sort8<512>(key, lane); break;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const uint32_t r = 8 * lane + (uint32_t)e;
        if (r < m) hs.sorted[r] = (uint16_t)(key[e] & 511), hs.w[r] = key[e] >> 9;  // rank r's symbol and weight
    }
    __syncthreads();
    HLCLK(2);
    if (m == 0) return;
    if (m == 1) {
        if (lane == 0) len[hs.sorted[0]] = 1;
        __syncthreads();
        return;
    }
    const uint32_t root = 2 * m - 2;
    // two-queue merge (lane 0) over the leaves w[0, m) and the nodes nw[] in creation order (tree index m + k).
    // r06: queues closed by +inf sentinels -- an exhausted leaf queue and a node not made yet read as +inf --
    // so a pick is one compare and two selects (the same picks as the guarded r05 merge: ties take the leaf);
    // the merge runs on the scalar unit, which the CU's 16 waves share, so its instruction count is its time
    if (lane < 2) hs.w[m + lane] = 0xffffffffu;
    for (uint32_t k = lane; k <= m; k += 64) hs.nw[k] = 0xffffffffu;
    __syncthreads();
    if (lane == 0) {  // weights and picks only: the parents follow from the picks below, lane-parallel
        uint32_t i = 0, j = 0;
        uint64_t bits = 0;
        for (uint32_t c = 0; c + 1 < m; ++c) {
            const uint32_t l0 = hs.w[i], l1 = hs.w[i + 1], n0 = hs.nw[j], n1 = hs.nw[j + 1];
            const bool p1 = l0 <= n0;  // first pick: the leaf unless the node is lighter
            const uint32_t wa = p1 ? l0 : n0;
            const uint32_t lh = p1 ? l1 : l0, nh = p1 ? n0 : n1;  // the queue heads after it
            const bool p2 = lh <= nh;
            const uint32_t wb = p2 ? lh : nh;
            i += (uint32_t)p1 + (uint32_t)p2;
            j += 2u - (uint32_t)p1 - (uint32_t)p2;
            hs.nw[c] = wa + wb;
            bits |= (uint64_t)((uint32_t)p1 | (uint32_t)p2 << 1) << (2 * (c & 31));
            if ((c & 31) == 31) hs.pick[c >> 5] = bits, bits = 0;
        }
        if ((m - 1) & 31) hs.pick[(m - 2) >> 5] = bits;
    }
    __syncthreads();
    // node c's children from the picks: the leaves taken before step c are a prefix sum of the picks (i_c),
    // the nodes 2c - i_c; a leaf pick takes the next leaf, a node pick the next node
    {
        uint32_t carry = 0;  // leaves taken by the steps of the chunks before
        for (uint32_t c0 = 0; c0 + 1 < m; c0 += 64) {
            const uint32_t c = c0 + lane;
            const bool live = c + 1 < m;
            const uint32_t pb = live ? (uint32_t)(hs.pick[c >> 5] >> (2 * (c & 31))) & 3u : 0u;
            const uint32_t p1 = pb & 1u, p2 = pb >> 1, nl = p1 + p2;
            uint32_t inc = nl;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += y;
            }
            const uint32_t ic = carry + inc - nl, jc = 2 * c - ic;  // queue heads at step c
            carry += __shfl(inc, 63, 64);
            if (live) {
                const uint32_t a = p1 ? ic : m + jc;
                const uint32_t b = p2 ? (p1 ? ic + 1 : ic) : m + (p1 ? jc : jc + 1);
                hs.parent[a] = (uint16_t)(m + c);
                hs.parent[b] = (uint16_t)(m + c);
            }
        }
        if (lane == 0) hs.parent[root] = (uint16_t)root;
    }
    __syncthreads();
    HLCLK(3);
    // depths by pointer jumping over the parent tree: d[x] = edges to the root (<= 10 doublings)
    for (uint32_t x = lane; x <= root; x += 64) hs.w[x] = x == root ? 0u : 1u;
    __syncthreads();
    for (int round = 0; round < 10; ++round) {
        uint32_t nd[9], na[9];
        bool open = false;  // some ancestor is not the root yet
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const uint32_t x = lane + 64 * q;
            nd[q] = 0, na[q] = 0;
            if (x <= root) {
                const uint32_t a = hs.parent[x];
                open |= a != root;
                nd[q] = hs.w[x] + (a != root ? hs.w[a] : 0u);
                na[q] = hs.parent[a];
            }
        }
        if (!__syncthreads_or(open)) break;  // every depth final (r06: typical trees need 4-5 of the 10 rounds)
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const uint32_t x = lane + 64 * q;
            if (x <= root) hs.w[x] = nd[q], hs.parent[x] = (uint16_t)na[q];
        }
        __syncthreads();
    }
    HLCLK(4);
    // leaves per clamped depth (LDS atomics), Kraft repair (lane 0, <= 15 entries, only when the clamp made the
    // code incomplete), lengths handed out longest-first to the least frequent symbols: rank k gets the b whose
    // range holds k (r06: per-depth ballots and per-rank walks over the counts before)
    if (lane < 16) hs.cnt[lane] = 0;
    __syncthreads();
    for (uint32_t k = lane; k < m; k += 64) atomicAdd(&hs.cnt[min(hs.w[k], (uint32_t)M)], 1u);
    __syncthreads();
    {
        const uint32_t c = lane >= 1 && lane <= M ? hs.cnt[lane] : 0u;
        uint32_t K = c << ((M - lane) & 31);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) K += __shfl_xor(K, o, 64);
        if (lane == 0 && K != (1u << M)) {
            const uint32_t one = 1u << M;
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
        }
    }
    __syncthreads();
    {
        // suf[b] = codes of length >= b; rank k gets the number of b in 1..M with suf[b] > k
        uint32_t suf = lane >= 1 && lane <= M ? hs.cnt[lane] : 0u;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = __shfl_down(suf, o, 64);
            if (lane + o < 16) suf += y;
        }
        uint32_t sb[15];
#pragma unroll
        for (int b = 0; b < 15; ++b) sb[b] = (uint32_t)__shfl((int)suf, b + 1, 64);
        for (uint32_t k = lane; k < m; k += 64) {
            uint32_t b = 0;
#pragma unroll
            for (int q = 0; q < 15; ++q) b += (q < M && k < sb[q]) ? 1u : 0u;
            len[hs.sorted[k]] = (uint8_t)b;
        }
    }
    __syncthreads();
    HLCLK(5);
#if OGE_EXP == 3
    if (n == kLit && blockIdx.x == 0 && threadIdx.x == 0)
        printf("huff_lengths lit: keys %llu sort %llu merge %llu depths %llu counts+lengths %llu (m %u)\n",
               (unsigned long long)(g_hl_clk[1] - g_hl_clk[0]), (unsigned long long)(g_hl_clk[2] - g_hl_clk[1]),
               (unsigned long long)(g_hl_clk[3] - g_hl_clk[2]), (unsigned long long)(g_hl_clk[4] - g_hl_clk[3]),
               (unsigned long long)(g_hl_clk[5] - g_hl_clk[4]), m);
#endif
}

// canonical codes, bit-reversed for LSB-first emission: out[i] = rcode | len << 16
// (lengths counted and symbols ranked inside their length by ballots: r03 counted on lane 0 and ranked each
// symbol by a walk over the symbols before it)
__device__ void huff_codes(const uint8_t *len, int n, uint32_t *out) {
    const int lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t cnt = 0;  // lane L: codes of length L
    for (int i0 = 0; i0 < n; i0 += 64) {
        const uint32_t L = i0 + lane < n ? len[i0 + lane] : 0u;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const uint32_t c = (uint32_t)__popcll(__ballot(L == (uint32_t)b));
            if (lane == b) cnt += c;
        }
    }
    uint32_t first = 0, code = 0;  // lane L: the first code of length L
#pragma unroll
    for (int b = 1; b < 16; ++b) {
        code = (code + (b > 1 ? (uint32_t)__shfl(cnt, b - 1, 64) : 0u)) << 1;
        if (lane == b) first = code;
    }
    uint32_t run = 0;  // lane L: codes of length L handed out so far
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const uint32_t L = i < n ? len[i] : 0u;
        const uint32_t base = (uint32_t)__shfl(run, (int)L, 64) + (uint32_t)__shfl(first, (int)L, 64);
        uint32_t r = 0, add = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const uint64_t mk = __ballot(L == (uint32_t)b);
            if (L == (uint32_t)b) r = (uint32_t)__popcll(mk & lt);
            if (lane == b) add = (uint32_t)__popcll(mk);
        }
        run += add;
        if (i < n) out[i] = L ? (__builtin_bitreverse32(base + r) >> (32 - L)) | (L << 16) : 0u;
    }
    __syncthreads();
}

__constant__ uint8_t kClOrder[kCl] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// extra-bit counts of a length symbol - 257 (0..28) and of a distance symbol (0..29)
__device__ __forceinline__ uint32_t len_extra(uint32_t ls) { return ls < 8 ? 0u : ls < 28 ? (ls - 4) >> 2 : 0u; }
__device__ __forceinline__ uint32_t dist_extra(uint32_t ds) { return ds < 4 ? 0u : (ds - 2) >> 1; }

// Also the exact size of the block (sizes[]): header bits + sum over symbols of frequency x (code length +
// extra bits), so the compressed blocks get their final offsets before they are emitted.
__global__ void __launch_bounds__(64) k_defl_huff(const uint32_t *__restrict__ freq_in, DeflTab *__restrict__ tabs, uint64_t n,
                                                 uint64_t blk0, int level, uint32_t *__restrict__ sizes) {
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
#if OGE_EXP == 3  // timing experiment: phase clocks of one wave
    uint64_t xc[10];
    int xn = 0;
#define XCLK() (xc[xn++] = __builtin_readcyclecounter())
#else
#define XCLK()
#endif
    XCLK();
    uint32_t nzl = 0, nzd = 0;  // used literal/length and distance codes (ballots: r05 counted on lane 0)
    for (int i = lane, r = 0; r < (kFreq + 63) / 64; i += 64, ++r) {
        const uint32_t v = i < kFreq ? freq_in[(uint64_t)blockIdx.x * kFreq + i] + (i == 256) : 0u;  // + end of block
        if (i < kFreq) f[i] = v;
        nzl += (uint32_t)__popcll(__ballot(i < kLit && v != 0));
        nzd += (uint32_t)__popcll(__ballot(i >= kLit && i < kFreq && v != 0));
    }
    __syncthreads();
    if (lane == 0 && (nzl < 2 || nzd < 2)) {  // at least two used codes per tree (a one-code tree would be incomplete)
        for (int i = 0; nzl < 2 && i < kLit; ++i)
            if (!f[i]) f[i] = 1, ++nzl;
        for (int i = 0; nzd < 2 && i < kDist; ++i)
            if (!f[kLit + i]) f[kLit + i] = 1, ++nzd;
    }
    __syncthreads();
    XCLK();
    huff_lengths(f, kLit, 15, lens, hs);
    XCLK();
    huff_lengths(f + kLit, kDist, 15, lens + kLit, hs);
    XCLK();
    huff_codes(lens, kLit, T.lit);
    huff_codes(lens + kLit, kDist, T.dist);
    XCLK();

    // run-length code the two length sequences separately (RFC 1951 3.2.7), the whole wave at once (r03 walked
    // them on lane 0: ~150k cycles of dependent LDS reads per block, then ~100k for the header bit string).
    // A run of v of length R (maximal, inside one sequence) always becomes the same tokens:
    //   v = 0: floor(R / 138) x 18(138), then the rest r = R % 138 as one 17 / 18 if r >= 3, else r zeros;
    //   v > 0: v, floor((R - 1) / 6) x 16(6), then the rest r = (R - 1) % 6 as one 16(r) if r >= 3, else r x v
    // (tests/deflate_parse.py restates the sequential walk; tests/test_gpu_bgzf.py pins the headers to it).
    __shared__ uint32_t hlit, hdist;
    __shared__ uint32_t hw[kHdrWords];
    {
        // one past the last used code: at least 257 / 1
        uint32_t la = 0, lb = 0;
        for (int r = 0; r < 5; ++r) {
            const int i = 64 * r + lane;
            const uint64_t mk = __ballot(i < kLit && lens[i] != 0);
            if (mk) la = 64 * r + 64 - __builtin_clzll(mk);
        }
        const uint64_t mkd = __ballot(lane < kDist && lens[kLit + lane] != 0);
        if (mkd) lb = 64 - __builtin_clzll(mkd);
        const uint32_t a = max(la, 257u), b = max(lb, 1u), N = a + b;
        auto val = [&](uint32_t p) -> uint32_t { return p < a ? lens[p] : lens[kLit + p - a]; };
        // run starts, as five wave masks over positions 64 r + lane
        uint64_t st[5];
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const uint32_t p = 64 * r + lane;
            st[r] = __ballot(p < N && (p == 0 || p == a || val(p) != val(p - 1)));
        }
        if (lane < kCl) fcl[lane] = 0;
        if (lane == 0) hlit = a, hdist = b;
        __syncthreads();
        // tokens per run, their exclusive prefix in position order, then each run writes its tokens
        uint32_t base = 0;
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const uint32_t p = 64 * r + lane;
            const bool start = (st[r] >> lane) & 1;
            uint32_t R = 0, v = 0, ntok = 0;
            if (start) {
                uint32_t nx = N;  // the next run start after p
                const uint64_t rest = lane < 63 ? st[r] & (~0ull << (lane + 1)) : 0ull;
                if (rest) {
                    nx = 64 * r + __builtin_ctzll(rest);
                } else {
#pragma unroll
                    for (int r2 = 4; r2 > r; --r2)
                        if (st[r2]) nx = 64 * r2 + __builtin_ctzll(st[r2]);
                }
                R = min(nx, N) - p;
                v = val(p);
                if (v == 0) {
                    const uint32_t rm = R % 138;
                    ntok = R / 138 + (rm >= 3 ? 1 : rm);
                } else {
                    const uint32_t rm = (R - 1) % 6;
                    ntok = 1 + (R - 1) / 6 + (rm >= 3 ? 1 : rm);
                }
            }
            uint32_t inc = ntok;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += y;
            }
            uint32_t k = base + inc - ntok;
            base += __shfl(inc, 63, 64);
            if (start) {
                auto tok = [&](uint32_t sym, uint32_t ext) {
                    cl_sym[k] = (uint8_t)sym;
                    cl_ext[k] = (uint8_t)ext;
                    atomicAdd(&fcl[sym], 1u);
                    ++k;
                };
                if (v == 0) {
                    for (uint32_t q = 0; q < R / 138; ++q) tok(18, 127);
                    const uint32_t rm = R % 138;
                    if (rm >= 11) tok(18, rm - 11);
                    else if (rm >= 3) tok(17, rm - 3);
                    else
                        for (uint32_t q = 0; q < rm; ++q) tok(0, 0);
                } else {
                    tok(v, 0);
                    for (uint32_t q = 0; q < (R - 1) / 6; ++q) tok(16, 3);
                    const uint32_t rm = (R - 1) % 6;
                    if (rm >= 3) tok(16, rm - 3);
                    else
                        for (uint32_t q = 0; q < rm; ++q) tok(v, 0);
                }
            }
        }
        __syncthreads();
        if (lane == 0) {
            ncl = base;
            uint32_t nz = 0;
            for (int i = 0; i < kCl; ++i) nz += fcl[i] != 0;
            for (int i = 0; nz < 2 && i < kCl; ++i)
                if (!fcl[i]) fcl[i] = 1, ++nz;
        }
    }
    __syncthreads();
    XCLK();
    huff_lengths(fcl, kCl, 7, lcl, hs);
    huff_codes(lcl, kCl, ccl);
    XCLK();
    {
        // the header bit string: 17 fixed bits, HCLEN x 3 bits, then every token's code and extra bits at the
        // prefix sum of the token lengths, OR-ed into LDS words (a token spans at most two)
        for (int i = lane; i < kHdrWords; i += 64) hw[i] = 0;
        const uint64_t mh = __ballot(lane >= 4 && lane < kCl && lcl[kClOrder[lane]] != 0);
        const uint32_t hclen = mh ? 64 - __builtin_clzll(mh) : 4u;
        __syncthreads();
        auto orbits = [&](uint32_t at, uint32_t v, uint32_t nb) {  // nb <= 32
            if (!nb) return;
            const uint32_t w = at >> 5, sh = at & 31;
            atomicOr(&hw[w], v << sh);
            if (sh + nb > 32) atomicOr(&hw[w + 1], v >> (32 - sh));
        };
        if (lane == 0) orbits(0, 1u | (2u << 1) | ((hlit - 257) << 3) | ((hdist - 1) << 8) | ((hclen - 4) << 13), 17);
        if ((uint32_t)lane < hclen) orbits(17 + 3 * lane, lcl[kClOrder[lane]], 3);
        const uint32_t n = ncl;
        uint32_t at = 17 + 3 * hclen;
        for (uint32_t t0 = 0; t0 < n; t0 += 64) {
            const uint32_t t = t0 + lane;
            uint32_t nb = 0, v = 0;
            if (t < n) {
                const uint32_t sym = cl_sym[t], c = ccl[sym], cb = c >> 16;
                const uint32_t eb = sym == 16 ? 2u : sym == 17 ? 3u : sym == 18 ? 7u : 0u;
                nb = cb + eb;
                v = (c & 0xffff) | ((uint32_t)cl_ext[t] << cb);
            }
            uint32_t inc = nb;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += y;
            }
            orbits(at + inc - nb, v, nb);
            at += __shfl(inc, 63, 64);
        }
        __syncthreads();
        for (uint32_t i = lane; i < (at + 31) / 32; i += 64) T.hdr[i] = hw[i];
        if (lane == 0) {
            T.hdr_bits = at;
            ncl = at;  // the header's bit count, for the size below
        }
    }
    __syncthreads();
    uint32_t bits = 0;
    for (int i = lane; i < kFreq; i += 64) {
        const uint32_t fr = freq_in[(uint64_t)blockIdx.x * kFreq + i] + (i == 256);  // the real counts + end of block
        const uint32_t ex = i < 257 ? 0u : i < kLit ? len_extra(i - 257) : dist_extra(i - kLit);
        bits += fr * (lens[i] + ex);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) bits += __shfl_xor(bits, o, 64);
    if (lane == 0) {
        const uint64_t start = (blk0 + blockIdx.x) * kPay;
        const uint32_t len = (uint32_t)min<uint64_t>(kPay, n - start);
        const uint32_t dbytes = (ncl + bits + 7) / 8;
        const uint32_t stored = level == 0 || dbytes > len + 5;
        const uint32_t total = stored ? 18 + 5 + len + 8 : 18 + dbytes + 8;
        T.stored = stored;
        T.total = total;
        sizes[blockIdx.x] = total;
    }
#if OGE_EXP == 3
    XCLK();
    if (lane == 0 && blockIdx.x < 4 && blk0 == 0)
        printf("huff-exp blk %u: load %llu lit-lengths %llu dist-lengths %llu codes %llu rle %llu cl %llu header+size %llu\n",
               blockIdx.x, (unsigned long long)(xc[1] - xc[0]), (unsigned long long)(xc[2] - xc[1]), (unsigned long long)(xc[3] - xc[2]),
               (unsigned long long)(xc[4] - xc[3]), (unsigned long long)(xc[5] - xc[4]), (unsigned long long)(xc[6] - xc[5]),
               (unsigned long long)(xc[7] - xc[6]));
#endif
}

// ------------------------------------------------------------------------------------ emit
// One 512-thread workgroup per payload (two per CU: 74 KiB of LDS).  The whole BGZF block is assembled in
// LDS -- header, deflate bits, footer -- and written once, with coalesced dword stores, straight to its
// final place in the output stream (offset = the chunk's base + the scan of the block sizes k_defl_huff
// computed): no 64 KiB slot per block and no compaction copy (r02: each lane stored 4-byte words into its
// own segment's bit range in global memory, 64 lines per wave store, then k_defl_compact copied the block).
//   1. per segment (the thread's two: sub-block 0 and 1): its 64 payload bytes in registers, the literal
//      mask and the match list from k_defl_parse; bit count = code lengths of its literals + its matches
//   2. block scan of the 1024 counts -> every segment's bit offset
//   3. every thread writes its segments' bits into the LDS image (plain stores inside its range, LDS
//      atomicOr on the two edge words shared with its neighbours); header bits, end-of-block code,
//      CRC-32 (from the payload in global memory, slice-by-1 per 128-byte piece, pieces combined) and
//      ISIZE likewise
//   4. the image [0, total) goes out at the block's byte offset: aligned dwords inside it, single bytes
//      at the two ends (the neighbouring blocks own the other bytes of those dwords)
struct LdsBits {  // LSB-first bit writer into LDS words; its first and last words are shared
    uint32_t *base;
    uint64_t acc;
    uint32_t nacc, wpos;
    __device__ __forceinline__ void init(uint32_t *b, uint32_t bit) { base = b, acc = 0, nacc = bit & 31, wpos = bit >> 5; }
    __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {  // nb <= 32, nacc < 32 on entry
        acc |= (uint64_t)v << nacc;
        nacc += nb;
        if (nacc >= 32) {
            const uint32_t w = (uint32_t)acc;
            // every word by LDS OR: the image is zeroed, so an OR into an interior word is its store, and the
            // first word (shared with the previous segment) needs no flag and no branch of its own (r06: the
            // first-word flag's nested branch at every store, 20M deflate 25.65 -> 25.21 ms, same bytes)
            atomicOr(base + wpos, w);
            ++wpos;
            acc >>= 32;
            nacc -= 32;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc && (uint32_t)acc) atomicOr(base + wpos, (uint32_t)acc);
    }
};

// The emitter's symbol table ct[512] (LDS, built per payload): ct[b] (b < 256) = literal b, ct[256 + L - 3]
// = match length L with its extra bits -- bit-reversed code | extra << code length in the low 24 bits,
// total bit count << 24: one lookup for either, no length-symbol arithmetic per match (r03 looked the
// length symbol up through len_code, branches the whole wave ran at every match position).
__device__ __forceinline__ uint32_t ct_entry(uint32_t i, const uint32_t *tlit) {
    if (i < 256) {
        const uint32_t c = tlit[i];
        return (c & 0xffff) | (c >> 16) << 24;
    }
    uint32_t sym, nb, ev;
    len_code(i - 256 + 3, sym, nb, ev);
    const uint32_t c = tlit[sym];
    return ((c & 0xffff) | (ev << (c >> 16))) | ((c >> 16) + nb) << 24;
}
// distance 1..32768 -> code | extra << code length, bit count (branch-free; dist_code's cases as selects)
__device__ __forceinline__ void dist_bits(uint32_t D, const uint32_t *dist, uint32_t &v, uint32_t &n) {
    const uint32_t d = D - 1, lg = 31 - __builtin_clz(d | 1);
    const bool small = d < 4;
    const uint32_t dnb = small ? 0u : lg - 1;
    const uint32_t dsym = small ? d : 2 * lg + ((d >> ((lg - 1) & 31)) & 1);
    const uint32_t dev = d & ((1u << dnb) - 1);
    const uint32_t c = dist[dsym];
    v = (c & 0xffff) | (dev << (c >> 16));
    n = (c >> 16) + dnb;
}
__device__ __forceinline__ uint32_t match_bits(uint32_t m, const uint32_t *ct, const uint32_t *dist) {
    uint32_t dv, dn;
    dist_bits((m & 0x7fff) + 1, dist, dv, dn);
    return (ct[256 + ((m >> 15) & 255)] >> 24) + dn;
}

// a segment's 64 payload bytes (zero past len) into registers
__device__ __forceinline__ void seg_load(const uint8_t *s, uint32_t s0, uint32_t len, uint32_t (&w)[16]) {
    if (s0 + kSeg <= len && !((uintptr_t)(s + s0) & 15)) {
        const uint4 *g = (const uint4 *)(s + s0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = g[k];
            w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (s0 + 4 * k + b < len) v |= (uint32_t)s[s0 + 4 * k + b] << (8 * b);
            w[k] = v;
        }
    }
}

// (r04: a wave-per-segment emitter -- lane i = byte i, the segment's match tokens gathered to their start
// lanes by rank, a DPP prefix sum of the bit counts, LDS atomicOr into the image -- measured slower: 13.3k
// vs 10.3k VALU per wave (it does ~80 VALU per segment per wave, this one ~16 per position per lane with
// 64 segments side by side), 20M deflate 36.5-37.6 vs 32.8 ms; same bytes)
// Latency, not work, bounds these two: a code lookup or a match-token load inside a data-dependent branch
// is waited for on the spot.  So the segment's literal codes are looked up 16 at a time without branches
// (independent LDS reads in flight together) and its first kMPre match tokens are loaded at once.
#ifndef OGE_EMIT_MPRE  // (20M deflate with 2 / 4 / 8 / 12 / 16: 30.6 / 29.6 / 28.8 / 29.0 / 29.2 ms)
#define OGE_EMIT_MPRE 8
#endif
constexpr int kMPre = OGE_EMIT_MPRE;
__device__ __forceinline__ void seg_tokens(const uint32_t *mp, uint32_t nm, uint32_t (&m)[kMPre]) {
    const uint32_t last = nm ? nm - 1 : 0;  // (clamped: every load is a real address, no branch around it)
#pragma unroll
    for (int k = 0; k < kMPre; ++k) m[k] = mp[(uint64_t)min((uint32_t)k, last) * kNSeg];
}

__device__ __forceinline__ uint32_t seg_bits(const uint32_t (&w)[16], uint64_t lm, uint32_t nm, const uint32_t *mp,
                                             const uint32_t (&m)[kMPre], const uint32_t *ct, const uint32_t *dist) {
    uint32_t bits = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        uint32_t c[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = ct[(w[4 * g + (i >> 2)] >> (8 * (i & 3))) & 0xff];
#pragma unroll
        for (int i = 0; i < 16; ++i) bits += (lm >> (16 * g + i)) & 1 ? c[i] >> 24 : 0u;
    }
#pragma unroll
    for (int k = 0; k < kMPre; ++k)
        if ((uint32_t)k < nm) bits += match_bits(m[k], ct, dist);
    for (uint32_t k = kMPre; k < nm; ++k) bits += match_bits(mp[(uint64_t)k * kNSeg], ct, dist);
    return bits;
}

__device__ __forceinline__ void seg_emit(const uint32_t (&w)[16], uint64_t lm, uint32_t nm, const uint32_t *mp,
                                         uint32_t (&m)[kMPre], const uint32_t *ct, const uint32_t *dist, uint32_t *img,
                                         uint32_t bit) {
    // the next match's length / distance codes are looked up one match ahead (software pipelined): at a
    // match start the codes are already in registers, and the lookups for the following match overlap
    // the literals in between
    uint32_t k = 0, cur = m[0], moff = nm ? (cur >> 23) : 64u;
    uint32_t lc, dv, dn;
    auto look = [&](uint32_t tok) {
        lc = ct[256 + ((tok >> 15) & 255)];
        dist_bits((tok & 0x7fff) + 1, dist, dv, dn);
    };
    look(cur);
    LdsBits bw;
    bw.init(img, bit);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        uint32_t c[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = ct[(w[4 * g + (i >> 2)] >> (8 * (i & 3))) & 0xff];
        // positions in pairs: the pair's literal codes (<= 30 bits) go out in one put; a match can start at
        // only one of the two (it covers >= 3 positions), after the literal that may precede it.  (Tried:
        // the first 8 matches deferred -- bits skipped here, written afterwards into their gaps with LDS
        // atomicOr: the same bytes, 29.27 vs 28.93 ms at 20M reads; the bookkeeping costs what it saves.)
#pragma unroll
        for (int i0 = 0; i0 < 16; i0 += 2) {
            const int i = 16 * g + i0;
            const uint32_t a = (lm >> i) & 1 ? c[i0] : 0u, b = (lm >> (i + 1)) & 1 ? c[i0 + 1] : 0u;
            bw.put((a & 0xffffff) | ((b & 0xffffff) << (a >> 24)), (a >> 24) + (b >> 24));
            if (((uint32_t)i | 1u) == (moff | 1u)) {  // a match starts at i or i + 1
#if OGE_EXP == 8  // timing experiment: matches not emitted (wrong bytes)
                ++k;
#pragma unroll
                for (int q = 0; q + 1 < kMPre; ++q) m[q] = m[q + 1];
                moff = k < nm && k < (uint32_t)kMPre ? m[0] >> 23 : 64u;
#else
                bw.put(lc & 0xffffff, lc >> 24);
                bw.put(dv, dn);
                ++k;
#pragma unroll
                for (int q = 0; q + 1 < kMPre; ++q) m[q] = m[q + 1];  // the next token to the front
                if (k < nm) {
                    cur = k < (uint32_t)kMPre ? m[0] : mp[(uint64_t)k * kNSeg];
                    moff = cur >> 23;
                    look(cur);
                } else {
                    moff = 64;
                }
#endif
            }
        }
    }
    bw.finish();
}

__global__ void __launch_bounds__(kT, 4) k_defl_emit(const uint8_t *__restrict__ src, uint64_t n, uint64_t blk0,
                                                     const uint64_t *__restrict__ lmask, const uint8_t *__restrict__ nmatch,
                                                     const uint32_t *__restrict__ mlist, const DeflTab *__restrict__ tabs,
                                                     const uint32_t *__restrict__ zpow, const uint32_t *__restrict__ offs,
                                                     const uint64_t *__restrict__ cbase, uint8_t *__restrict__ dst) {
    __shared__ __align__(16) uint32_t img[kSlot / 4 + 4];
    __shared__ uint32_t ct[512], dist[kDist];
    __shared__ uint32_t scan[kNSeg];
    __shared__ uint32_t wsum[kT / 64];
    __shared__ uint32_t crctab[4][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t zl[32][16];  // the CRC's per-lane combine operators (crc_combine512l)
    __shared__ uint32_t crcs[kT / 64];
    __shared__ uint32_t sh_crc;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t blk = blk0 + blockIdx.x;
    const uint64_t start = blk * kPay;
    const uint32_t len = (uint32_t)min<uint64_t>(kPay, n - start);
    const uint8_t *s = src + start;
    const DeflTab &T = tabs[blockIdx.x];
    const uint32_t total = T.total, stored = T.stored, hb = T.hdr_bits;
    for (int i = t; i < 512; i += kT) ct[i] = ct_entry(i, T.lit);
    for (int i = t; i < kDist; i += kT) dist[i] = T.dist[i];
    crc_setup<kT>(crctab, zp, zpow, t);
    for (int i = t; i < 32 * 16; i += kT) zl[i >> 4][i & 15] = zpow[17 * 32 + i];
    for (uint32_t i = t; i < (total + 15) / 16; i += kT) ((uint4 *)img)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    {
        const uint32_t c = crc_global512x4l(s, len, crctab, zl, zp, crcs, t);
        if (t == 0) sh_crc = c;
    }
    const uint32_t bsize = total - 1;
    if (stored) {
        for (uint32_t i = t; i < len; i += kT) ((uint8_t *)img)[23 + i] = s[i];
    } else {
        // 1. the thread's two segments (sub-block 0 and 1): bytes, literal masks, bit counts
        const uint32_t s0a = t * kSeg, s0b = kSub + t * kSeg;
        const uint64_t sga = (uint64_t)blockIdx.x * kNSeg + t, sgb = sga + kT;
        const uint64_t lma = s0a < len ? lmask[sga] : 0, lmb = s0b < len ? lmask[sgb] : 0;
        const uint32_t nma = s0a < len ? nmatch[sga] : 0, nmb = s0b < len ? nmatch[sgb] : 0;
        const uint32_t *mpa = mlist + ((uint64_t)blockIdx.x * kMaxM) * kNSeg + t, *mpb = mpa + kT;
        // (the bytes and tokens are loaded again for the emit below -- L2 hits -- rather than held in
        // registers across the scan)
        uint32_t ca, cb;
        {
            uint32_t w[16], m[kMPre];
            seg_load(s, s0a, len, w);
            seg_tokens(mpa, nma, m);
            ca = seg_bits(w, lma, nma, mpa, m, ct, dist);
            seg_load(s, s0b, len, w);
            seg_tokens(mpb, nmb, m);
            cb = seg_bits(w, lmb, nmb, mpb, m, ct, dist);
        }
        scan[t] = ca;
        scan[kT + t] = cb;
        __syncthreads();
        // 2. exclusive scan of scan[0..kNSeg): thread t owns entries 2t, 2t + 1
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
            for (int q = 0; q < wv; ++q) pre += wsum[q];
            const uint32_t ex = pre + inc - x;
            __syncthreads();
            scan[2 * t] = ex;
            scan[2 * t + 1] = ex + a;
        }
        __syncthreads();
        // 3. bits into the image: stream bit 0 = byte 18 = bit 144
        for (uint32_t i = t; i < (hb + 31) / 32; i += kT) {  // the header bit string
            const uint32_t v = T.hdr[i];
            atomicOr(img + 4 + i, v << 16);
            if (v >> 16) atomicOr(img + 5 + i, v >> 16);
        }
        {
            uint32_t w[16], m[kMPre];
            if (ca) {
                seg_load(s, s0a, len, w);
                seg_tokens(mpa, nma, m);
                seg_emit(w, lma, nma, mpa, m, ct, dist, img, 144 + hb + scan[t]);
            }
            if (cb) {
                seg_load(s, s0b, len, w);
                seg_tokens(mpb, nmb, m);
                seg_emit(w, lmb, nmb, mpb, m, ct, dist, img, 144 + hb + scan[kT + t]);
            }
        }
        if (t == kT - 1) {  // end of block after the last segment
            const uint32_t body_end = 144 + hb + scan[kNSeg - 1] + cb;
            LdsBits bw;
            bw.init(img, body_end);
            const uint32_t c = T.lit[256];
            bw.put(c & 0xffff, c >> 16);
            bw.finish();
        }
    }
    __syncthreads();
    uint8_t *ib = (uint8_t *)img;
    if (t == 0) {  // BGZF header (the stream's first bits are already in bytes 18, 19) and footer
        img[0] = 0x04088b1fu;  // ID1 ID2 CM=8 FLG=FEXTRA
        img[1] = 0;            // MTIME
        img[2] = 0x0006ff00u;  // XFL=0 OS=255 XLEN=6
        img[3] = 0x00024342u;  // 'B' 'C' SLEN=2
        ib[16] = (uint8_t)bsize, ib[17] = (uint8_t)(bsize >> 8);
        if (stored) {
            ib[18] = 1;
            ib[19] = (uint8_t)len, ib[20] = (uint8_t)(len >> 8);
            ib[21] = (uint8_t)~len, ib[22] = (uint8_t)(~len >> 8);
        }
        const uint32_t q = total - 8;
        for (int b = 0; b < 4; ++b) ib[q + b] = (uint8_t)(sh_crc >> (8 * b)), ib[q + 4 + b] = (uint8_t)(len >> (8 * b));
    }
    __syncthreads();
    // 4. out at the block's final offset
    uint8_t *D = dst + *cbase + offs[blockIdx.x];
    const uint32_t sh = (uint32_t)((uintptr_t)D & 3);
    OGE_G uint32_t *A = (OGE_G uint32_t *)((uintptr_t)D & ~(uintptr_t)3);
    const uint32_t nwords = (total + sh + 3) / 4;
    for (uint32_t g = t; g < nwords; g += kT) {
        const int32_t r0 = (int32_t)(4 * g) - (int32_t)sh;  // block byte of the dword's first byte
        if (r0 >= 0 && r0 + 4 <= (int32_t)total) {
            A[g] = ld32(img, (uint32_t)r0);
        } else {
            for (int i = 0; i < 4; ++i) {
                const int32_t r = r0 + i;
                if (r >= 0 && r < (int32_t)total) ((OGE_G uint8_t *)(A + g))[i] = ib[r];
            }
        }
    }
}

// exclusive scan of n <= kMaxChunk block sizes, one 1024-thread workgroup, kPer consecutive entries per
// thread (the per-chunk offsets; runs on the chunk's own stream)
constexpr uint32_t kMaxChunk = 16384, kPer = kMaxChunk / 1024;
__global__ void __launch_bounds__(1024) k_scan_chunk(const uint32_t *__restrict__ in, uint32_t n, uint32_t *__restrict__ out) {
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t a[kPer], v = 0;
#pragma unroll
    for (uint32_t i = 0; i < kPer; ++i) {
        a[i] = kPer * t + i < n ? in[kPer * t + i] : 0;
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
    for (uint32_t i = 0; i < kPer; ++i) {
        if (kPer * t + i < n) out[kPer * t + i] = excl;
        excl += a[i];
    }
}

// the chunk's base in the output stream (*cbase) and the running end for the next chunk (*base)
__global__ void k_defl_advance(uint64_t *base, uint64_t *cbase, const uint32_t *offs, const uint32_t *sizes, uint32_t nb) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const uint64_t b = *base;
        *cbase = b;
        *base = b + (uint64_t)offs[nb - 1] + sizes[nb - 1];
    }
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
    // levels 1-7: the greedy one-candidate parse; 8 / 9: same-prefix chains 8 / 32 deep and lazy matching
    const int depth = level >= 9 ? 32 : level == 8 ? 8 : 1, lazy = level >= 8 ? 1 : 0;
    if (dst_cap < oge_bgzf_bound(n)) return oge_fail(ctx, OGE_ERR_ARG, "dst_cap < oge_bgzf_bound(n)");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    *out_bytes = 0;
    if (!n) return OGE_OK;
    const uint64_t nblk = (n + kPay - 1) / kPay;
    const int ncu = ctx->cu_count();  // persistent parse workgroups: one per CU of this context's device
    // payloads per chunk: one launch of each kernel.  r02 measured 4096 best (2048 / 4096 / 8192,
    // profiles/r02_ab/codec_k*.json); on the r06 kernels larger chunks win (fewer persistent-parse tails):
    // 100M reads 126.7 / 124.0 / 122.4 ms for 4096 / 8192 / 16384, 40M reads (11 chunks) 50.5 / 48.8 ms for
    // 4096 / 16384, the same bytes (profiles/r06dg-di).  Buffers: ~97 KB per payload and stream set.
    // The chunk halves (down to 4096) until the S buffer sets fit in a quarter of the device memory that is free
    // or already held by them (a caller that keeps most of HBM, like the 300M chain test, gets 4096).
#ifndef OGE_DEFL_STREAMS
#define OGE_DEFL_STREAMS 3
#endif
#ifndef OGE_DEFL_CHUNK  // experiment builds: another largest chunk
#define OGE_DEFL_CHUNK kMaxChunk
#endif
    static_assert(OGE_DEFL_CHUNK <= kMaxChunk, "k_scan_chunk bound");
    constexpr uint64_t kPerPay = (uint64_t)kNSeg * 8 + kNSeg + (uint64_t)kMaxM * kNSeg * 4 + kFreq * 4 + sizeof(DeflTab) + 8;
    const int S0 = nblk > 4096 ? OGE_DEFL_STREAMS : 1;
    uint64_t chunk = std::min<uint64_t>(nblk, OGE_DEFL_CHUNK);
    if (chunk > 4096) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
        uint64_t held = 0;
        for (int s = 0; s < 3; ++s) {
            const auto it = ctx->bufs.find("defl_mlist" + std::to_string(s));
            if (it != ctx->bufs.end()) held += it->second.cap / ((uint64_t)kMaxM * kNSeg * 4) * kPerPay;
        }
        while (chunk > 4096 && (uint64_t)S0 * chunk * kPerPay > (fr + held) / 4) chunk = std::max<uint64_t>(4096, chunk / 2);
    }
    // Chunks go round-robin over S streams: one chunk's Huffman and emit kernels run on the CUs beside
    // another chunk's parse workgroups (150 KiB of LDS, one per CU); only the offset advance, which
    // gives each chunk its base in the output stream, is ordered chunk after chunk (events).
    // B[] below holds three buffer sets; 300M chain: 2 streams 423.6 ms, 3 streams 417.4 ms (r04)
    static_assert(OGE_DEFL_STREAMS >= 1 && OGE_DEFL_STREAMS <= 3, "deflate: 1-3 streams");
    const int S = nblk > chunk ? OGE_DEFL_STREAMS : 1;
    struct Bufs {
        uint64_t *lmask, *cbase;
        uint32_t *mlist, *freq, *sizes, *offs;
        uint8_t *nmatch;
        DeflTab *tabs;
        hipStream_t st;
    } B[3];
    for (int s = 0; s < S; ++s) {
        const std::string x = std::to_string(s);
        B[s].lmask = (uint64_t *)ctx->ws(("defl_lmask" + x).c_str(), chunk * kNSeg * 8);
        B[s].nmatch = (uint8_t *)ctx->ws(("defl_nmatch" + x).c_str(), chunk * kNSeg);
        B[s].mlist = (uint32_t *)ctx->ws(("defl_mlist" + x).c_str(), chunk * kMaxM * kNSeg * 4);
        B[s].freq = (uint32_t *)ctx->ws(("defl_freq" + x).c_str(), chunk * kFreq * 4);
        B[s].tabs = (DeflTab *)ctx->ws(("defl_tabs" + x).c_str(), chunk * sizeof(DeflTab));
        B[s].sizes = (uint32_t *)ctx->ws(("defl_sizes" + x).c_str(), chunk * 4 + 16);
        B[s].offs = (uint32_t *)ctx->ws(("defl_offs" + x).c_str(), chunk * 4 + 16);
        B[s].cbase = (uint64_t *)ctx->ws(("defl_cbase" + x).c_str(), 16);
        B[s].st = S == 1 ? ctx->stream : ctx->side_stream(s);
        if (!B[s].lmask || !B[s].nmatch || !B[s].mlist || !B[s].freq || !B[s].tabs || !B[s].sizes || !B[s].offs ||
            !B[s].cbase || !B[s].st)
            return OGE_ERR_HIP;
    }
    // the 2^k zero-byte operators, then the emit's 16-lane combine operators (crc_zlane, 128-byte pieces)
    uint32_t *zpow = (uint32_t *)ctx->ws("defl_zpow", (17 * 32 + 32 * 16) * 4);
    uint64_t *base = (uint64_t *)ctx->ws("defl_base", 16);
    if (!zpow || !base) return OGE_ERR_HIP;
    static struct {
        uint32_t z[17][32], zl[32][16];
    } zh = [] {
        decltype(zh) v;
        crc_zpow(v.z);
        crc_zlane<16>(v.z, 128, &v.zl[0][0]);
        return v;
    }();
    OGE_HIP_TRY(ctx, hipMemcpyAsync(zpow, &zh, sizeof(zh), hipMemcpyHostToDevice, ctx->stream));
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
        if (depth > 1)
            k_defl_parse<true><<<(uint32_t)std::min<uint64_t>(nb, (uint64_t)ncu), kTP, 0, u.st>>>(d_src, n, b0, nb, u.lmask, u.nmatch,
                                                                                            u.mlist, u.freq, depth, lazy);
        else
            k_defl_parse<false><<<(uint32_t)std::min<uint64_t>(nb, (uint64_t)ncu), kTP, 0, u.st>>>(d_src, n, b0, nb, u.lmask, u.nmatch,
                                                                                             u.mlist, u.freq, 1, 0);
        OGE_LAUNCH_CHECK(ctx);
        k_defl_huff<<<nb, 64, 0, u.st>>>(u.freq, u.tabs, n, b0, level, u.sizes);
        OGE_LAUNCH_CHECK(ctx);
        k_scan_chunk<<<1, 1024, 0, u.st>>>(u.sizes, nb, u.offs);
        OGE_LAUNCH_CHECK(ctx);
        if (k) OGE_HIP_TRY(ctx, hipStreamWaitEvent(u.st, ev[(k - 1) % S], 0));  // previous chunk's offset advance
        k_defl_advance<<<1, 64, 0, u.st>>>(base, u.cbase, u.offs, u.sizes, nb);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipEventRecord(ev[k % S], u.st));
        k_defl_emit<<<nb, kT, 0, u.st>>>(d_src, n, b0, u.lmask, u.nmatch, u.mlist, u.tabs, zpow, u.offs, u.cbase, d_dst);
        OGE_LAUNCH_CHECK(ctx);
    }
    // every chunk's emit: the context stream waits for all side streams
    if (S > 1) {
        for (int s = 0; s < S; ++s) {
            OGE_HIP_TRY(ctx, hipEventRecord(ev[s], B[s].st));
            OGE_HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev[s], 0));
        }
    }
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

