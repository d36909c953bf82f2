// inflate.hip -- BGZF decompression on the GPU, and the device-side BAM record boundary parse.
//
// Replaces `BgzfInputStream::decompress` (openge/src/util/bgzf_input_stream.cpp:65-142,208-240:
// inflateInit2(-15) per block at :116-123) and the record walk of `BamDeserializer::read`
// (util/bam_deserializer.h:143-193, block_size bounds at :160-163).  SURVEY §8f rows 1-2.
//
//   oge_bgzf_index (host)  walks the BGZF framing: per block the deflate byte range, the payload
//                          offset (prefix sum of ISIZE) and the stored CRC-32.
//   inflate itself          inflate_lane.hip: one lane per BGZF block (Huffman decode), then one
//                          workgroup per block (LZ77 resolution, CRC-32 check, write-out).
//   k_rec_walk             BAM record boundaries: one thread per 64 KiB chunk walks the block_size
//                          chain from its chunk's first record start (found by an 8-record
//                          plausibility chain); the host verifies that every chunk's walk ends where
//                          the next one starts and re-walks from the true end when it does not, so
//                          the result equals the sequential walk.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "bam_layout.h"
#include "bgzf_dev.h"
#include "oge_ctx.h"

namespace {

using namespace oge_bgzf;

// ------------------------------------------------------------------------------ record boundaries
__device__ __forceinline__ uint32_t rd32u(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// the reader's plausibility test for a record start (bamio.cpp plausible_record)
__device__ bool plausible(const uint8_t *d, uint64_t s, uint64_t n, int32_t n_ref) {
    if (s + 36 > n) return false;
    const uint32_t bs = rd32u(d + s);
    if (bs < 32 || bs > 10000 || s + 4 + bs > n) return false;
    const int32_t ref = (int32_t)rd32u(d + s + 4), mref = (int32_t)rd32u(d + s + 24);
    if (ref < -1 || ref >= n_ref || mref < -1 || mref >= n_ref) return false;
    const uint32_t lname = d[s + 12], nc = d[s + 16] | (d[s + 17] << 8), lseq = rd32u(d + s + 20);
    if (lname == 0 || d[s + 36 + lname - 1] != 0) return false;
    return 32ull + lname + 4ull * nc + (lseq + 1ull) / 2 + lseq <= bs;
}

constexpr uint64_t kNone = ~0ull;

// a kChain-record plausibility chain starts at s (or the chain reaches the stream's end, at_end: n is it).
// Only a guess: every chunk start is verified by the join of the walks, a wrong one costs a second walk.
// 8 (r05; 16 before): the guess pass 5.6 -> 3.6 ms at 300M reads, the same walks (a false 8-record chain
// needs eight consecutive plausible headers -- sizes, refIDs, NUL-terminated names -- at a wrong offset)
#ifndef OGE_REC_CHAIN
#define OGE_REC_CHAIN 8
#endif
constexpr int kChain = OGE_REC_CHAIN;
__device__ bool chain_at(const uint8_t *d, uint64_t s, uint64_t n, bool at_end, int32_t n_ref) {
    uint64_t q = s;
    int k = 0;
    for (; k < kChain && q < n && plausible(d, q, n, n_ref); ++k) q += 4 + rd32u(d + q);
    return k == kChain || (at_end && q == n && k > 0);
}

// chunk c covers [p + c*CH, min(lim, p + (c+1)*CH)) (bytes readable up to n); guess its first record start.
// A thread per chunk: the plausibility chain is the cost, and a wave runs 64 of them side by side (r05: a
// wave per chunk, its lanes testing 64 positions at once, measured 6.4 vs 5.7 ms at 300M reads)
__global__ void k_rec_guess(const uint8_t *__restrict__ d, uint64_t p, uint64_t lim, uint64_t n, bool at_end, int32_t n_ref,
                            uint64_t CH, uint64_t C, uint64_t *__restrict__ start) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (c == 0) {
        start[0] = p;
        return;
    }
    const uint64_t cut = p + c * CH, ls = min(n, cut + 20016);
    for (uint64_t s = cut; s < ls; ++s)
        if (chain_at(d, s, n, at_end, n_ref)) {
            start[c] = s;
            return;
        }
    start[c] = kNone;
}

// the first plausible record start in [0, lim): one workgroup, thread t tries t, t + 256, ...
__global__ void __launch_bounds__(256) k_rec_guess_first(const uint8_t *__restrict__ d, uint64_t lim, uint64_t n, bool at_end,
                                                         int32_t n_ref, unsigned long long *__restrict__ out) {
    __shared__ unsigned long long best;
    if (threadIdx.x == 0) best = kNone;
    __syncthreads();
    for (uint64_t base = 0; base < lim; base += 256) {
        const uint64_t s = base + threadIdx.x;
        if (s < lim && s < best && chain_at(d, s, n, at_end, n_ref)) atomicMin(&best, (unsigned long long)s);
        __syncthreads();
        if (best != kNone) break;
    }
    if (threadIdx.x == 0) *out = best;
}

// the block_size chain from q while it starts before end: k records, *q the first start at or past end
// (or the invalid record's); with out != NULL the offsets from out[o0], never at or past out[cap]
__device__ __forceinline__ uint64_t walk_chunk(const uint8_t *__restrict__ d, uint64_t &q, uint64_t end, uint64_t n,
                                               uint64_t *__restrict__ out, uint64_t o0, uint64_t cap, uint16_t *__restrict__ rel,
                                               uint64_t cut, uint32_t SC) {
    uint64_t k = 0, acc = 0;  // rel: four slots per 8-byte store (SC is a multiple of 4)
    while (q < end) {
        if (q + 4 > n) break;
        const uint32_t bs = rd32u(d + q);
        if (bs < 32 || bs > 10000 || q + 4 + bs > n) break;
        if (out && o0 + k < cap) out[o0 + k] = q;
        if (rel && k < SC) {
            acc |= (q - cut) << (16 * (k & 3));
            if ((k & 3) == 3) *(uint64_t *)(rel + (k & ~3ull)) = acc, acc = 0;
        }
        ++k;
        q += 4 + bs;
    }
    if (rel && (k & 3) && k < SC) *(uint64_t *)(rel + (k & ~3ull)) = acc;
    return k;
}

// walk chunk c from start[c] to the first record start at or past the chunk end; with out != NULL
// also write the (absolute) offsets from pos[c], never at or past out[cap] (a stream that changed since
// the counts in pos were made may hold more records: the caller then detects it and walks again); with
// rel != NULL the first SC record starts relative to the chunk's first byte (< 64 KiB: u16) go to
// rel[c * SC ...] for k_rec_fill
__global__ void k_rec_walk(const uint8_t *__restrict__ d, uint64_t p, uint64_t lim, uint64_t n, uint64_t CH, uint64_t C,
                           const uint64_t *__restrict__ start, uint64_t *__restrict__ stop, uint64_t *__restrict__ count,
                           const uint64_t *__restrict__ pos, uint64_t *__restrict__ out, uint64_t cap, uint16_t *__restrict__ rel,
                           uint32_t SC) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t cut = p + c * CH, end = min(lim, cut + CH);
    uint64_t q = start[c];
    if (q == kNone) {
        stop[c] = kNone;
        count[c] = 0;
        return;
    }
    const uint64_t k = walk_chunk(d, q, end, n, out, out ? pos[c] : 0, cap, rel ? rel + c * SC : nullptr, cut, SC);
    stop[c] = q < end ? kNone - 1 : q;  // kNone - 1: invalid record inside the chunk
    count[c] = k;
}

// the offsets from the converged count walk's slots: one wave per chunk, 64 offsets per store; a chunk
// with more records than slots (under 128 bytes a record on average) is walked again by its lane 0
__global__ void __launch_bounds__(256) k_rec_fill(const uint8_t *__restrict__ d, uint64_t p, uint64_t lim, uint64_t n, uint64_t CH,
                                                  uint64_t C, const uint64_t *__restrict__ start, const uint64_t *__restrict__ count,
                                                  const uint64_t *__restrict__ pos, const uint16_t *__restrict__ rel, uint32_t SC,
                                                  uint64_t *__restrict__ out, uint64_t cap) {
    const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (c >= C) return;
    const uint64_t k_n = count[c], o0 = pos[c], cut = p + c * CH;
    if (k_n <= SC) {
        const uint16_t *r = rel + c * SC;
        for (uint64_t k = lane; k < k_n; k += 64)
            if (o0 + k < cap) out[o0 + k] = cut + r[k];
    } else if (lane == 0) {
        uint64_t q = start[c];
        (void)walk_chunk(d, q, min(lim, cut + CH), n, out, o0, cap, nullptr, cut, 0);
    }
}

// chunk c + 1 starts where chunk c's walk stopped; *st bit 0: a start moved, bit 1: a stop that is
// invalid (or the last chunk's short of the window's end)
__global__ void k_rec_join(const uint64_t *__restrict__ stop, uint64_t *__restrict__ start, uint64_t C, uint64_t lim,
                           unsigned int *__restrict__ st) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t e = stop[c];
    if (e >= kNone - 1) {
        atomicOr(st, 2u);
        return;
    }
    if (c + 1 < C) {
        if (start[c + 1] != e) {
            start[c + 1] = e;
            atomicOr(st, 1u);
        }
    } else if (e < lim) {
        atomicOr(st, 2u);
    }
}


// ------------------------------------------------------------------------------ BGZF framing index
// The framing walk of oge_bgzf_index done in parallel: every byte position is tested for a BGZF
// member header (gzip magic, FLG = FEXTRA, a BC subfield; the same acceptance as the host walk),
// candidates are compacted in stream order, and the candidate list is accepted only when it is the
// exact chain 0 -> p + BSIZE -> ... -> end (a false candidate inside deflate data, or a corrupt
// stream, fails the check and the caller falls back to the host walk, which reports errors).
__device__ __forceinline__ uint32_t bgzf_head(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t p) {
    if (p + 18 > zbytes || z[p] != 31 || z[p + 1] != 139 || z[p + 2] != 8 || z[p + 3] != 4) return 0;
    const uint32_t xlen = z[p + 10] | ((uint32_t)z[p + 11] << 8);
    const uint64_t xend = p + 12 + xlen;
    if (xend > zbytes) return 0;
    uint32_t bsize = 0;
    for (uint64_t x = p + 12; x + 4 <= xend;) {
        const uint32_t slen = z[x + 2] | ((uint32_t)z[x + 3] << 8);
        if (z[x] == 'B' && z[x + 1] == 'C' && slen == 2 && x + 6 <= xend) bsize = (z[x + 4] | ((uint32_t)z[x + 5] << 8)) + 1;
        x += 4 + slen;
    }
    if (!bsize || p + bsize > zbytes || bsize < 12 + xlen + 8) return 0;
    return bsize;
}

constexpr int kIdxPos = 64;  // byte positions per thread (300M reads, 60 GB file: 16 -> 18.6 ms, 64 -> 15.1 ms,
                             // 128 / 256 -> 41 / 48 ms: the 4-slot stash per workgroup overflows and the
                             // second scan runs)

constexpr uint32_t kStash = 4;  // candidate slots per 256 * kIdxPos-position block in the counting pass

template <bool EMIT>
__global__ void __launch_bounds__(256) k_bgzf_cand(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t plim,
                                                   uint32_t *__restrict__ cnt,
                                                   const uint32_t *__restrict__ base, uint64_t *__restrict__ cpos,
                                                   uint32_t *__restrict__ cbs, uint64_t *__restrict__ stash_pos = nullptr,
                                                   uint32_t *__restrict__ stash_bs = nullptr,
                                                   unsigned int *__restrict__ ovf = nullptr) {
    __shared__ uint32_t wsum[4];
    const uint32_t t = threadIdx.x;
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256 + t) * kIdxPos;
    uint32_t mine = 0;
    if (p0 < plim) {
        // the thread's kIdxPos positions + 4 bytes of look-ahead in registers (16-byte loads + one dword):
        // only a position whose 4 bytes are the gzip/deflate/FEXTRA signature 1f 8b 08 04 goes on to
        // bgzf_head's global loads (a bare 0x1f byte every 256 stalled the wave on dependent loads)
        const uint32_t *w = (const uint32_t *)(z + p0);
        uint32_t v[kIdxPos / 4 + 1];
        if (p0 + kIdxPos <= zbytes) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int k = 0; k < kIdxPos / 16; ++k) {
                const u32x4 q = ((const u32x4 *)w)[k];
                v[4 * k] = q.x, v[4 * k + 1] = q.y, v[4 * k + 2] = q.z, v[4 * k + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kIdxPos / 4; ++k) v[k] = p0 + 4 * k + 4 <= zbytes ? w[k] : 0;
        }
        v[kIdxPos / 4] = p0 + kIdxPos + 4 <= zbytes ? w[kIdxPos / 4] : 0;
#pragma unroll
        for (int k = 0; k < kIdxPos; ++k) {
            const uint32_t sig = (k & 3) ? __builtin_amdgcn_alignbyte(v[(k >> 2) + 1], v[k >> 2], k & 3) : v[k >> 2];
            if (sig == 0x04088b1fu && p0 + k < plim && bgzf_head(z, zbytes, p0 + k)) ++mine;
        }
    }
    // block-wide exclusive prefix of the per-thread counts
    const uint32_t lane = t & 63, wv = t >> 6;
    uint32_t incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        if (k < wv) before += wsum[k];
        tot += wsum[k];
    }
    if (!EMIT) {
        if (t == 0) cnt[blockIdx.x] = tot;
        // stash: a block's candidates (nearly always 0 or 1 per 16 KiB) in its kStash slots, so the
        // compaction needs no second scan of the file; a fuller block raises the overflow word
        if (stash_pos) {
            if (tot > kStash) {
                if (t == 0) atomicOr(ovf, 1u);
                return;
            }
            if (!mine) return;
            uint64_t o = (uint64_t)blockIdx.x * kStash + before + incl - mine;
            for (int k = 0; k < kIdxPos; ++k) {
                const uint64_t p = p0 + k;
                if (p >= plim || z[p] != 31) continue;
                const uint32_t bs = bgzf_head(z, zbytes, p);
                if (bs) stash_pos[o] = p, stash_bs[o] = bs, ++o;
            }
        }
        return;
    }
    if (!mine) return;
    uint64_t o = base[blockIdx.x] + before + incl - mine;
    for (int k = 0; k < kIdxPos; ++k) {
        const uint64_t p = p0 + k;
        if (p >= plim || z[p] != 31) continue;
        const uint32_t bs = bgzf_head(z, zbytes, p);
        if (bs) cpos[o] = p, cbs[o] = bs, ++o;
    }
}

// chain check + per-block fields over the candidates at or past s (positions below s get isz 0 and
// are left out): the first is s itself, every later one starts where its predecessor ends, and the
// last ends at or past `own` (the end of the range whose block starts are indexed; for a whole file
// own = zbytes, so the chain ends exactly at the end).  *xend = that end.
__global__ void k_bgzf_chain(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t s, uint64_t own,
                             const uint64_t *__restrict__ cpos, const uint32_t *__restrict__ cbs, uint64_t m,
                             uint32_t *__restrict__ bad, uint32_t *__restrict__ isz, unsigned long long *__restrict__ xend) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t p = cpos[i], e = p + cbs[i];
    if (p < s) {
        isz[i] = 0;
        return;
    }
    const bool ok = (p == s || (i > 0 && cpos[i - 1] >= s && cpos[i - 1] + cbs[i - 1] == p)) && (i + 1 == m ? e >= own : true);
    if (i + 1 == m) atomicMax(xend, (unsigned long long)e);
    const uint32_t sz = z[e - 4] | ((uint32_t)z[e - 3] << 8) | ((uint32_t)z[e - 2] << 16) | ((uint32_t)z[e - 1] << 24);
    if (!ok || sz > kSlot) atomicAdd(bad, 1u);
    isz[i] = sz;
}

__global__ void k_bgzf_fill(const uint8_t *__restrict__ z, const uint64_t *__restrict__ cpos, const uint32_t *__restrict__ cbs,
                            const uint32_t *__restrict__ isz, const uint32_t *__restrict__ slot, uint64_t m,
                            uint64_t *__restrict__ d0, uint64_t *__restrict__ d1, uint64_t *__restrict__ usz,
                            uint32_t *__restrict__ crc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || !isz[i]) return;
    const uint64_t p = cpos[i], e = p + cbs[i], k = slot[i];
    d0[k] = p + 12 + (z[p + 10] | ((uint32_t)z[p + 11] << 8));
    d1[k] = e - 8;
    usz[k] = isz[i];
    crc[k] = z[e - 8] | ((uint32_t)z[e - 7] << 8) | ((uint32_t)z[e - 6] << 16) | ((uint32_t)z[e - 5] << 24);
}

__global__ void k_nonzero_u32(const uint32_t *__restrict__ a, uint64_t n, uint32_t *__restrict__ f) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = a[i] != 0;
    else if (i == n) f[i] = 0;
}

// ---- segment walk (r06): the framing chain followed from known starts instead of a scan of every byte.
// [s, own) is cut into segments of kSegBytes (more than the largest block, 64 KiB, so every segment but a
// short last one holds a block start).  Segment 0 starts at s; segment k > 0 guesses its first block start
// -- the first position of its first kSegScan bytes where three headers chain (or a chain reaches the end of
// the buffer) -- and one thread per segment walks BSIZE links while the block starts lie in the segment.  A
// segment is right when its start is where its predecessor's walk left off; a wrong guess (a false chain
// inside deflate data) is walked again from there, so the result is the sequential walk from s.  Reads:
// the headers plus ~half a block per segment for the guesses, not the whole file.
constexpr uint64_t kSegBytes = 1ull << 20;
constexpr uint64_t kSegScan = 256ull << 10;
constexpr uint64_t kSegNone = ~0ull, kSegBad = ~0ull - 1;

__device__ bool chain3(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t p) {
    for (int k = 0; k < 3; ++k) {
        const uint32_t bs = bgzf_head(z, zbytes, p);
        if (!bs) return false;
        p += bs;
        if (p == zbytes) return true;
    }
    return true;
}

// one wave per segment k >= 1: start[k] = the guess (kSegNone: none within kSegScan); 64 lanes test 16
// positions each per 1 KiB step, the lowest valid position wins
__global__ void __launch_bounds__(256) k_seg_guess(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t s, uint64_t own,
                                                   uint64_t nseg, uint64_t *__restrict__ start) {
    const uint64_t k = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (k >= nseg) return;
    if (k == 0) {
        if (lane == 0) start[0] = s;
        return;
    }
    const uint64_t a = s + k * kSegBytes, lim = min(min(a + kSegScan, own), zbytes);
    uint64_t found = kSegNone;
    for (uint64_t c = a; c < lim && found == kSegNone; c += 64 * 16) {
        uint64_t mine = kSegNone;
        const uint64_t p0 = c + 16ull * lane;
        // the lane's 16 positions + 3 bytes of look-ahead in registers; only the gzip/deflate/FEXTRA
        // signature 1f 8b 08 04 goes on to the header chain's loads
        uint32_t v[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t pb = p0 + 4 * q + b;
                if (pb < zbytes) x |= (uint32_t)z[pb] << (8 * b);
            }
            v[q] = x;
        }
        for (uint32_t j = 0; j < 16 && mine == kSegNone; ++j) {
            const uint64_t p = p0 + j;
            if (p >= lim) break;
            const uint32_t sig = (j & 3) ? __builtin_amdgcn_alignbyte(v[(j >> 2) + 1], v[j >> 2], j & 3) : v[j >> 2];
            if (sig == 0x04088b1fu && chain3(z, zbytes, p)) mine = p;
        }
        // the lowest lane with a hit
        const uint64_t m = __ballot(mine != kSegNone);
        if (m) found = __shfl(mine, __ffsll((long long)m) - 1, 64);
    }
    if (lane == 0) start[k] = found;
}

// one thread per segment: walk from start[k] while block starts lie below the segment's end b (the last
// segment: below own); ex[k] = where the walk left off (kSegBad: an invalid header on the way), cnt[k] =
// blocks.  EMIT: the starts and sizes go to cpos / cbs from base[k].  only: walk only the segments whose
// flag is set (the re-walks), prev_ex: their start is the predecessor's exit.
template <bool EMIT>
__global__ void __launch_bounds__(256) k_seg_walk(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t s, uint64_t own,
                                                  uint64_t nseg, const uint64_t *__restrict__ start, uint64_t *__restrict__ ex,
                                                  uint32_t *__restrict__ cnt, const uint32_t *__restrict__ base,
                                                  uint64_t *__restrict__ cpos, uint32_t *__restrict__ cbs) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= nseg) return;
    const uint64_t b = k + 1 == nseg ? own : s + (k + 1) * kSegBytes;
    uint64_t p = start[k];
    uint32_t c = 0;
    uint64_t o = EMIT ? base[k] : 0;
    if (p == kSegNone) {
        if (!EMIT) ex[k] = kSegNone, cnt[k] = 0;
        return;
    }
    while (p < b) {
        const uint32_t bs = bgzf_head(z, zbytes, p);
        if (!bs) {
            p = kSegBad;
            break;
        }
        if (EMIT) cpos[o] = p, cbs[o] = bs, ++o;
        ++c;
        p += bs;
    }
    if (!EMIT) ex[k] = p, cnt[k] = c;
}

// segments whose start is not their predecessor's exit take that exit as their start (ex_prev: the exits of
// the last walk); *chg counts them
__global__ void k_seg_join(uint64_t nseg, const uint64_t *__restrict__ ex, uint64_t *__restrict__ start, unsigned int *__restrict__ chg) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k == 0 || k >= nseg) return;
    const uint64_t want = ex[k - 1];
    if (start[k] != want) {
        start[k] = want;
        atomicAdd(chg, 1u);
    }
}

// the first header candidate of [0, lim) (the kIndexFirst guess): atomicMin over positions
__global__ void __launch_bounds__(256) k_first_cand(const uint8_t *__restrict__ z, uint64_t zbytes, uint64_t lim,
                                                    unsigned long long *__restrict__ first) {
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    for (uint32_t j = 0; j < 16; ++j) {
        const uint64_t p = p0 + j;
        if (p >= lim) return;
        if (z[p] == 31 && bgzf_head(z, zbytes, p)) {
            atomicMin(first, (unsigned long long)p);
            return;
        }
    }
}
}  // namespace

// ------------------------------------------------------------------------------------ host side
static inline uint16_t rd16h(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t rd32h(const uint8_t *p) { return (uint32_t)p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

extern "C" int oge_bgzf_index(const uint8_t *z, uint64_t zbytes, uint64_t *d0, uint64_t *d1, uint64_t *uoff, uint32_t *crc,
                              uint64_t cap, uint64_t *nblk) {
    if (!nblk || (zbytes && !z)) return oge_fail(nullptr, OGE_ERR_ARG, "null argument");
    uint64_t p = 0, k = 0, total = 0;
    while (p < zbytes) {
        if (zbytes - p < 18 || z[p] != 31 || z[p + 1] != 139 || z[p + 2] != 8 || !(z[p + 3] & 4))
            return oge_fail(nullptr, OGE_ERR_IO, "not a BGZF stream or truncated block header");
        if (z[p + 3] & ~4u) return oge_fail(nullptr, OGE_ERR_IO, "unsupported gzip header flags in a BGZF block");
        const uint16_t xlen = rd16h(z + p + 10);
        uint64_t x = p + 12, xend = x + xlen, bsize = 0;
        if (xend > zbytes) return oge_fail(nullptr, OGE_ERR_IO, "truncated BGZF extra field");
        while (x + 4 <= xend) {
            const uint16_t slen = rd16h(z + x + 2);
            if (z[x] == 'B' && z[x + 1] == 'C' && slen == 2) bsize = (uint64_t)rd16h(z + x + 4) + 1;
            x += 4 + slen;
        }
        if (!bsize) return oge_fail(nullptr, OGE_ERR_IO, "BGZF block without BC field");
        if (p + bsize > zbytes || bsize < xend - p + 8) return oge_fail(nullptr, OGE_ERR_IO, "truncated BGZF block");
        const uint32_t isize = rd32h(z + p + bsize - 4);
        if (isize > kSlot) return oge_fail(nullptr, OGE_ERR_IO, "BGZF block payload larger than 64 KiB");
        if (isize) {
            if (k < cap) {
                if (d0) d0[k] = xend;
                if (d1) d1[k] = p + bsize - 8;
                if (uoff) uoff[k] = total;
                if (crc) crc[k] = rd32h(z + p + bsize - 8);
            }
            ++k;
            total += isize;
        }
        p += bsize;
    }
    if (k <= cap && uoff) uoff[k] = total;
    *nblk = k;
    return k <= cap ? OGE_OK : oge_fail(nullptr, OGE_ERR_ARG, "index capacity too small");
}


// The same framing walk on the host with T threads (oge_mergesort_bgzf_host indexes a host file while its
// first chunks upload): thread t walks the blocks that start in [zbytes t / T, zbytes (t + 1) / T) from the
// first position there that begins a chain of valid headers (three blocks, or to the end of the stream);
// each walk must start where its predecessor's ended (a wrong guess is walked again from that exit).  The
// output equals oge_bgzf_index's (nonempty blocks only); returns false on anything it cannot walk (the
// caller then takes the sequential walk, which reports the error).
static uint32_t host_bgzf_head(const uint8_t *z, uint64_t zbytes, uint64_t p) {
    if (zbytes - p < 18 || z[p] != 31 || z[p + 1] != 139 || z[p + 2] != 8 || z[p + 3] != 4) return 0;
    const uint64_t xend = p + 12 + rd16h(z + p + 10);
    if (xend > zbytes) return 0;
    uint32_t bs = 0;
    for (uint64_t x = p + 12; x + 4 <= xend;) {
        const uint32_t sl = rd16h(z + x + 2);
        if (z[x] == 'B' && z[x + 1] == 'C' && sl == 2) bs = (uint32_t)rd16h(z + x + 4) + 1;
        x += 4 + sl;
    }
    if (!bs || p + bs > zbytes || bs < xend - p + 8) return 0;
    if (rd32h(z + p + bs - 4) > kSlot) return 0;
    return bs;
}

bool oge_bgzf_index_host_mt(const uint8_t *z, uint64_t zbytes, int T, std::vector<uint64_t> &d0, std::vector<uint64_t> &d1,
                            std::vector<uint64_t> &uoff, std::vector<uint32_t> &crc) {
    T = std::max(1, std::min(T, 64));
    if (zbytes < (uint64_t)T * (1u << 20)) T = 1;
    struct Part {
        uint64_t s = 0, x = 0;
        bool ok = false;
        std::vector<uint64_t> pos;  // block starts (every block, empty ones included)
    };
    std::vector<Part> P(T);
    auto walk = [&](Part &w, uint64_t s, uint64_t lim) {
        w.s = s, w.pos.clear(), w.ok = false;
        uint64_t p = s;
        while (p < lim) {
            const uint32_t bs = host_bgzf_head(z, zbytes, p);
            if (!bs) return;
            w.pos.push_back(p);
            p += bs;
        }
        w.x = p;
        w.ok = true;
    };
    auto guess = [&](uint64_t a, uint64_t lim) -> uint64_t {  // first position in [a, lim) starting a valid chain
        for (uint64_t p = a; p < lim; ++p) {
            if (z[p] != 31) continue;
            uint64_t q = p;
            int k = 0;
            for (; k < 3 && q < zbytes; ++k) {
                const uint32_t bs = host_bgzf_head(z, zbytes, q);
                if (!bs) break;
                q += bs;
            }
            if (k == 3 || q == zbytes) return p;
        }
        return lim;
    };
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t)
        ts.emplace_back([&, t]() {
            const uint64_t a = zbytes * (uint64_t)t / (uint64_t)T, b = zbytes * (uint64_t)(t + 1) / (uint64_t)T;
            walk(P[t], t ? guess(a, std::min(zbytes, a + (1u << 20))) : 0, b);
        });
    for (auto &t : ts) t.join();
    for (int t = 0; t < T; ++t) {  // the join: every part starts where the previous one ended
        const uint64_t b = zbytes * (uint64_t)(t + 1) / (uint64_t)T;
        const uint64_t want = t ? P[t - 1].x : 0;
        if (!P[t].ok || P[t].s != want) {
            if (want >= b) {  // no block starts in this part
                P[t].s = P[t].x = want, P[t].pos.clear(), P[t].ok = true;
                continue;
            }
            walk(P[t], want, b);
            if (!P[t].ok) return false;
        }
    }
    if (P[T - 1].x != zbytes) return false;
    d0.clear(), d1.clear(), uoff.clear(), crc.clear();
    uint64_t total = 0;
    for (auto &w : P)
        for (uint64_t p : w.pos) {
            const uint32_t bs = host_bgzf_head(z, zbytes, p), isize = rd32h(z + p + bs - 4);
            if (!isize) continue;
            d0.push_back(p + 12 + rd16h(z + p + 10));
            d1.push_back(p + bs - 8);
            uoff.push_back(total);
            crc.push_back(rd32h(z + p + bs - 8));
            total += isize;
        }
    uoff.push_back(total);
    return true;
}

// Device framing index into the context's workspace (pointers valid until the next call that uses
// it).  Returns 1 (no error recorded) when the candidate chain is not exact: the caller then uses
// the host walk, which also produces the reference-like error messages.
// the stashed candidates of every block into stream order
__global__ void k_bgzf_unstash(const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ base, uint64_t G,
                               const uint64_t *__restrict__ stash_pos, const uint32_t *__restrict__ stash_bs,
                               uint64_t *__restrict__ cpos, uint32_t *__restrict__ cbs) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= G) return;
    const uint32_t c = cnt[b], o = base[b];
    for (uint32_t j = 0; j < c; ++j) cpos[o + j] = stash_pos[b * kStash + j], cbs[o + j] = stash_bs[b * kStash + j];
}

// candidates by a scan of every byte position of [0, own) (the r02-r05 path; now the fallback of the
// segment walk): 0 with *cpos / *cbs / *m set (the chain check follows), 1 = no candidate at s, 2 = none in
// the range
static int scan_candidates(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t *s_io, uint64_t own, uint32_t *bad,
                           uint64_t **cpos_o, uint32_t **cbs_o, uint64_t *m_o) {
    uint64_t s = *s_io;
    const uint64_t per_blk = 256ull * kIdxPos;
    const uint64_t G = (own + per_blk - 1) / per_blk;
    if (!G) return 2;
    if (G > 0xffffffffull) return 1;
    uint32_t *cnt = (uint32_t *)ctx->ws("bix_cnt", (G + 1) * 4);
    uint32_t *base = (uint32_t *)ctx->ws("bix_base", (G + 1) * 4);
    uint64_t *stash_pos = (uint64_t *)ctx->ws("bix_stash_pos", G * kStash * 8);
    uint32_t *stash_bs = (uint32_t *)ctx->ws("bix_stash_bs", G * kStash * 4);
    if (!cnt || !base || !stash_pos || !stash_bs) return OGE_ERR_HIP;
    k_bgzf_cand<false><<<(uint32_t)G, 256, 0, ctx->stream>>>(d_z, zbytes, own, cnt, nullptr, nullptr, nullptr, stash_pos, stash_bs,
                                                              bad + 1);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt + G, 0, 4, ctx->stream));
    int rc = oge_exclusive_scan_u32(ctx, cnt, base, G + 1);
    if (rc) return rc;
    uint32_t m32 = 0, stash_ovf = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&m32, base + G, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&stash_ovf, bad + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t m = m32;
    if (!m) return s == kIndexFirst ? 2 : 1;
    uint64_t *cpos = (uint64_t *)ctx->ws("bix_cpos", m * 8);
    uint32_t *cbs = (uint32_t *)ctx->ws("bix_cbs", m * 4);
    if (!cpos || !cbs) return OGE_ERR_HIP;
    if (stash_ovf)  // a block with more than kStash candidates: the second scan places them
        k_bgzf_cand<true><<<(uint32_t)G, 256, 0, ctx->stream>>>(d_z, zbytes, own, cnt, base, cpos, cbs);
    else
        k_bgzf_unstash<<<oge_ceil_div(G, 256), 256, 0, ctx->stream>>>(cnt, base, G, stash_pos, stash_bs, cpos, cbs);
    OGE_LAUNCH_CHECK(ctx);
    if (s == kIndexFirst) {  // the range's first candidate
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&s, cpos, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    *s_io = s, *cpos_o = cpos, *cbs_o = cbs, *m_o = m;
    return OGE_OK;
}

// the block chain from s by the segment walk (see k_seg_walk): 0 with the exact chain's starts and sizes in
// *cpos / *cbs (*m blocks), 1 = an invalid header on the chain (the host walk reports it), 3 = undecided
// (no candidate near the start of a kIndexFirst range, or wrong guesses that keep moving): the scan decides
static int seg_candidates(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t *s_io, uint64_t own, uint64_t **cpos_o,
                          uint32_t **cbs_o, uint64_t *m_o) {
    uint64_t s = *s_io;
    unsigned long long *w = (unsigned long long *)ctx->ws("bix_seg_w", 16);
    if (!w) return OGE_ERR_HIP;
    unsigned int *chg = (unsigned int *)(w + 1);
    if (s == kIndexFirst) {
        const uint64_t lim = std::min<uint64_t>(own, kSegScan);
        unsigned long long first = ~0ull;
        OGE_HIP_TRY(ctx, hipMemsetAsync(w, 0xff, 8, ctx->stream));
        if (lim) k_first_cand<<<(uint32_t)oge_ceil_div(oge_ceil_div(lim, 16), 256), 256, 0, ctx->stream>>>(d_z, zbytes, lim, w);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&first, w, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (first == ~0ull) return 3;
        s = first;
    }
    if (s >= own) return 3;
    const uint64_t nseg = (own - s + kSegBytes - 1) / kSegBytes;
    if (nseg > 0xffffffffull) return 3;
    uint64_t *start = (uint64_t *)ctx->ws("bix_seg_start", (nseg + 1) * 8);
    uint64_t *ex = (uint64_t *)ctx->ws("bix_seg_ex", (nseg + 1) * 8);
    uint32_t *cnt = (uint32_t *)ctx->ws("bix_seg_cnt", (nseg + 1) * 4);
    uint32_t *base = (uint32_t *)ctx->ws("bix_seg_base", (nseg + 1) * 4);
    if (!start || !ex || !cnt || !base) return OGE_ERR_HIP;
    k_seg_guess<<<(uint32_t)oge_ceil_div(nseg * 64, 256), 256, 0, ctx->stream>>>(d_z, zbytes, s, own, nseg, start);
    OGE_LAUNCH_CHECK(ctx);
    const uint32_t gw = (uint32_t)oge_ceil_div(nseg, 256);
    for (int it = 0;; ++it) {
        k_seg_walk<false><<<gw, 256, 0, ctx->stream>>>(d_z, zbytes, s, own, nseg, start, ex, cnt, nullptr, nullptr, nullptr);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipMemsetAsync(chg, 0, 4, ctx->stream));
        k_seg_join<<<gw, 256, 0, ctx->stream>>>(nseg, ex, start, chg);
        OGE_LAUNCH_CHECK(ctx);
        unsigned int hc = 0;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(&hc, chg, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        if (!hc) break;
        if (it == 32) return 3;
    }
    uint64_t xl = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&xl, ex + nseg - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemsetAsync(cnt + nseg, 0, 4, ctx->stream));
    int rc = oge_exclusive_scan_u32(ctx, cnt, base, nseg + 1);
    if (rc) return rc;
    uint32_t m32 = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&m32, base + nseg, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (xl == kSegBad || xl == kSegNone || xl < own || !m32) return 1;  // every bad or missing exit reaches the last
    uint64_t *cpos = (uint64_t *)ctx->ws("bix_cpos", (uint64_t)m32 * 8);
    uint32_t *cbs = (uint32_t *)ctx->ws("bix_cbs", (uint64_t)m32 * 4);
    if (!cpos || !cbs) return OGE_ERR_HIP;
    k_seg_walk<true><<<gw, 256, 0, ctx->stream>>>(d_z, zbytes, s, own, nseg, start, ex, cnt, base, cpos, cbs);
    OGE_LAUNCH_CHECK(ctx);
    *s_io = s, *cpos_o = cpos, *cbs_o = cbs, *m_o = m32;
    return OGE_OK;
}

int oge_bgzf_index_range_ws(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t s, uint64_t own, OgeBgzfIndex *ix,
                            uint64_t *s_used, uint64_t *xend) {
    hipSetDevice(ctx->device);
    ix->nblk = 0;
    ix->total = 0;
    if (own > zbytes || (s != kIndexFirst && s >= own)) return 2;
    if ((uintptr_t)d_z & 3) return 1;
    uint32_t *bad = (uint32_t *)ctx->ws("bix_bad", 32);
    if (!bad) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(bad, 0, 32, ctx->stream));
    uint64_t *cpos = nullptr, m = 0;
    uint32_t *cbs = nullptr;
    // the segment walk (r06), the byte scan when it cannot decide (or with OGE_BGZF_INDEX=scan)
    const char *mode = getenv("OGE_BGZF_INDEX");
    int rc = mode && !strcmp(mode, "scan") ? 3 : seg_candidates(ctx, d_z, zbytes, &s, own, &cpos, &cbs, &m);
    if (rc == 3) rc = scan_candidates(ctx, d_z, zbytes, &s, own, bad, &cpos, &cbs, &m);
    if (rc) return rc;
    uint32_t *isz = (uint32_t *)ctx->ws("bix_isz", (m + 1) * 4);
    uint32_t *slot = (uint32_t *)ctx->ws("bix_slot", (m + 1) * 4);
    if (!isz || !slot) return OGE_ERR_HIP;
    if (s_used) *s_used = s;
    unsigned long long *dx = (unsigned long long *)(bad + 4);
    k_bgzf_chain<<<oge_ceil_div(m, 256), 256, 0, ctx->stream>>>(d_z, zbytes, s, own, cpos, cbs, m, bad, isz, dx);
    OGE_LAUNCH_CHECK(ctx);
    k_nonzero_u32<<<oge_ceil_div(m + 1, 256), 256, 0, ctx->stream>>>(isz, m, slot);
    OGE_LAUNCH_CHECK(ctx);
    rc = oge_exclusive_scan_u32(ctx, slot, slot, m + 1);
    if (rc) return rc;
    uint32_t hb[2] = {0, 0};
    unsigned long long xe = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&hb[0], bad, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&hb[1], slot + m, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&xe, dx, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (hb[0]) return 1;
    if (xend) *xend = xe;
    const uint64_t nb = hb[1];
    uint64_t *ix64 = (uint64_t *)ctx->ws("bix_out", (3 * nb + 2) * 8);
    uint32_t *crc = (uint32_t *)ctx->ws("bix_crc", (nb + 1) * 4);
    if (!ix64 || !crc) return OGE_ERR_HIP;
    uint64_t *d0 = ix64, *d1 = ix64 + nb, *uoff = ix64 + 2 * nb;
    k_bgzf_fill<<<oge_ceil_div(m, 256), 256, 0, ctx->stream>>>(d_z, cpos, cbs, isz, slot, m, d0, d1, uoff, crc);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemsetAsync(uoff + nb, 0, 8, ctx->stream));
    rc = oge_exclusive_scan_u64(ctx, uoff, uoff, nb + 1);
    if (rc) return rc;
    uint64_t total = 0;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&total, uoff + nb, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ix->d0 = d0;
    ix->d1 = d1;
    ix->uoff = uoff;
    ix->crc = crc;
    ix->nblk = nb;
    ix->total = total;
    return OGE_OK;
}

int oge_bgzf_index_ws(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, OgeBgzfIndex *ix) {
    ix->nblk = 0;
    ix->total = 0;
    if (!zbytes) return OGE_OK;
    const int rc = oge_bgzf_index_range_ws(ctx, d_z, zbytes, 0, zbytes, ix, nullptr, nullptr);
    return rc == 2 ? 1 : rc;  // no candidate at all: the host walk reports it
}

extern "C" int oge_bgzf_index_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t *d_d0, uint64_t *d_d1,
                                  uint64_t *d_uoff, uint32_t *d_crc, uint64_t cap, uint64_t *nblk) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!nblk || (zbytes && !d_z)) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    OgeStageTimer *tm = ctx->begin_stage("bgzf_index");
    OgeBgzfIndex ix;
    int rc = oge_bgzf_index_ws(ctx, d_z, zbytes, &ix);
    ctx->end_stage(tm);
    if (rc == 1) {  // not an exact chain: the host walk (and its error messages)
        std::vector<uint8_t> h(zbytes);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h.data(), d_z, zbytes, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        uint64_t nb = 0;
        rc = oge_bgzf_index(h.data(), zbytes, nullptr, nullptr, nullptr, nullptr, 0, &nb);
        if (rc != OGE_OK && rc != OGE_ERR_ARG) return oge_fail(ctx, rc, oge_last_error(nullptr));
        std::vector<uint64_t> a(3 * nb + 1);
        std::vector<uint32_t> c(nb + 1);
        rc = oge_bgzf_index(h.data(), zbytes, a.data(), a.data() + nb, a.data() + 2 * nb, c.data(), nb, &nb);
        if (rc) return oge_fail(ctx, rc, oge_last_error(nullptr));
        *nblk = nb;
        if (!d_d0 && !d_d1 && !d_uoff && !d_crc) return OGE_OK;  // count only
        if (nb > cap) return oge_fail(ctx, OGE_ERR_ARG, "index capacity too small");
        if (d_d0) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_d0, a.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
        if (d_d1) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_d1, a.data() + nb, nb * 8, hipMemcpyHostToDevice, ctx->stream));
        if (d_uoff) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_uoff, a.data() + 2 * nb, (nb + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        if (d_crc) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_crc, c.data(), nb * 4, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    }
    if (rc) return rc;
    *nblk = ix.nblk;
    if (!d_d0 && !d_d1 && !d_uoff && !d_crc) return OGE_OK;  // count only
    if (ix.nblk > cap) return oge_fail(ctx, OGE_ERR_ARG, "index capacity too small");
    const uint64_t nb = ix.nblk;
    if (d_d0 && nb) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_d0, ix.d0, nb * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (d_d1 && nb) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_d1, ix.d1, nb * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (d_uoff) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_uoff, ix.uoff, (nb + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (d_crc && nb) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_crc, ix.crc, nb * 4, hipMemcpyDeviceToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

extern "C" int oge_bgzf_inflate_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d_d0,
                                    const uint64_t *d_d1, const uint64_t *d_uoff, const uint32_t *d_crc, uint64_t nblk,
                                    uint8_t *d_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (nblk && (!d_z || !d_d0 || !d_d1 || !d_uoff || !d_out)) return oge_fail(ctx, OGE_ERR_ARG, "null buffer");
    if ((uintptr_t)d_z & 3) return oge_fail(ctx, OGE_ERR_ARG, "d_z must be 4-byte aligned");
    hipSetDevice(ctx->device);
    ctx->reset_timing();
    if (!nblk) return OGE_OK;
    uint32_t *err = (uint32_t *)ctx->ws("infl_err", 16);
    // the 2^k zero-byte operators, then phase 2's per-lane combine operators (crc_zlane, 64-byte pieces)
    uint32_t *zpow = (uint32_t *)ctx->ws("infl_zpow", (17 * 32 + 32 * 64) * 4);
    if (!err || !zpow) return OGE_ERR_HIP;
    static struct {
        uint32_t z[17][32], zl[32][64];
    } zh = [] {
        decltype(zh) v;
        crc_zpow(v.z);
        crc_zlane<64>(v.z, 64, &v.zl[0][0]);
        return v;
    }();
    const uint32_t init[2] = {0, 0xffffffffu};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(err, init, 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(zpow, &zh, sizeof(zh), hipMemcpyHostToDevice, ctx->stream));
    // the lane decoder (inflate_lane.hip), CRC fused into its phase 2
    OgeStageTimer *tm = ctx->begin_stage("bgzf_inflate");
    const int rc = oge_inflate_lanes(ctx, d_z, zbytes, d_d0, d_d1, d_uoff, d_crc, nblk, d_out, err, zpow);
    ctx->end_stage(tm);
    if (rc) return rc;
    uint32_t got[2];
    OGE_HIP_TRY(ctx, hipMemcpyAsync(got, err, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (got[0]) {
        ctx->infl_clean_ptr = nullptr;  // a failed block may have left bits phase 2 did not clear
        char msg[160];
        snprintf(msg, sizeof msg, "BGZF block %u failed to inflate (%s; error bits 0x%x)", got[1],
                 (got[0] >> E_CRC) & 1 ? "CRC mismatch" : "corrupt deflate data", got[0]);
        return oge_fail(ctx, OGE_ERR_IO, msg);
    }
    return OGE_OK;
}

extern "C" int oge_bgzf_inflate(oge_ctx *ctx, const uint8_t *z, uint64_t zbytes, uint8_t *out, uint64_t out_cap,
                                uint64_t *out_bytes) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!out_bytes) return oge_fail(ctx, OGE_ERR_ARG, "null out_bytes");
    hipSetDevice(ctx->device);
    *out_bytes = 0;
    uint64_t nb = 0;
    int rc = oge_bgzf_index(z, zbytes, nullptr, nullptr, nullptr, nullptr, 0, &nb);
    if (rc != OGE_OK && rc != OGE_ERR_ARG) return oge_fail(ctx, rc, oge_last_error(nullptr));
    std::vector<uint64_t> d0(nb), d1(nb), uo(nb + 1);
    std::vector<uint32_t> crc(nb);
    rc = oge_bgzf_index(z, zbytes, d0.data(), d1.data(), uo.data(), crc.data(), nb, &nb);
    if (rc) return oge_fail(ctx, rc, oge_last_error(nullptr));
    const uint64_t total = uo[nb];
    if (total > out_cap) return oge_fail(ctx, OGE_ERR_ARG, "out_cap too small for the decompressed stream");
    if (!nb) return OGE_OK;
    uint8_t *dz = (uint8_t *)ctx->ws("infl_hz", zbytes + 16);
    uint64_t *dd = (uint64_t *)ctx->ws("infl_hidx", (3 * nb + 1) * 8);
    uint32_t *dc = (uint32_t *)ctx->ws("infl_hcrc", nb * 4);
    uint8_t *dout = (uint8_t *)ctx->ws("infl_hout", total + 16);
    if (!dz || !dd || !dc || !dout) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dz, z, zbytes, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dd, d0.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dd + nb, d1.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dd + 2 * nb, uo.data(), (nb + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(dc, crc.data(), nb * 4, hipMemcpyHostToDevice, ctx->stream));
    rc = oge_bgzf_inflate_dev(ctx, dz, zbytes, dd, dd + nb, dd + 2 * nb, dc, nb, dout);
    if (rc) return rc;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *out_bytes = total;
    return OGE_OK;
}

int oge_record_guess(oge_ctx *ctx, const uint8_t *d, uint64_t lim, uint64_t bufend, bool at_end, int32_t n_ref, uint64_t *out) {
    *out = kNone;
    if (!lim) return OGE_OK;
    unsigned long long *w = (unsigned long long *)ctx->ws("rec_guess", 16);
    if (!w) return OGE_ERR_HIP;
    k_rec_guess_first<<<1, 256, 0, ctx->stream>>>(d, std::min<uint64_t>(lim, 20016), bufend, at_end, n_ref, w);
    OGE_LAUNCH_CHECK(ctx);
    unsigned long long h = kNone;
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&h, w, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *out = h;
    return OGE_OK;
}

int oge_record_walk(oge_ctx *ctx, const uint8_t *d_stream, uint64_t rec_base, uint64_t limit, uint64_t end, bool at_end,
                    int32_t n_ref, uint64_t *d_off, uint64_t cap, uint64_t *n_out, uint64_t *exit, bool keep, void *rel_buf,
                    uint64_t rel_cap) {
    if (!n_out || rec_base > limit || limit > end || (end > rec_base && !d_stream)) return oge_fail(ctx, OGE_ERR_ARG, "bad argument");
    hipSetDevice(ctx->device);
    *n_out = 0;
    *exit = rec_base;
    const uint64_t CH = 1ull << 16;
    const uint64_t C = std::max<uint64_t>(1, (limit - rec_base + CH - 1) / CH);
    uint64_t *ws = (uint64_t *)ctx->ws("rec_walk", (5 * C + 4) * 8 + 64);
    if (!ws) return OGE_ERR_HIP;
    // start[C], stop[C], count[C + 1], pos[C + 1], pos2[C + 1], st
    uint64_t *start = ws, *stop = ws + C, *count = ws + 2 * C, *pos = ws + 3 * C + 1, *pos2 = ws + 4 * C + 2;
    unsigned int *st = (unsigned int *)(ws + 5 * C + 3);
    if (limit == rec_base) {
        if (d_off && cap >= 1) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off, &rec_base, 8, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    }
    const uint32_t TB = 128, G = oge_ceil_div(C, TB), G4 = oge_ceil_div(C, 4);
    uint16_t *rel = nullptr;
    uint32_t SC = 0;
    // one walk + join pass: *st bit 0 = a start moved, bit 1 = an invalid or unjoined stop
    auto walk_join = [&](uint64_t *pos_arg, uint64_t *out, unsigned int *h) -> int {
        OGE_HIP_TRY(ctx, hipMemsetAsync(st, 0, 4, ctx->stream));
        k_rec_walk<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, limit, end, CH, C, start, stop, count, pos_arg, out, cap, rel, SC);
        OGE_LAUNCH_CHECK(ctx);
        k_rec_join<<<G, TB, 0, ctx->stream>>>(stop, start, C, limit, st);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h, st, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    };
    // n = the sum of the chunk counts, pos = their exclusive scan; *x = the last chunk's stop
    auto scan_counts = [&](uint64_t *dst, uint64_t *n, uint64_t *x) -> int {
        OGE_HIP_TRY(ctx, hipMemsetAsync(count + C, 0, 8, ctx->stream));  // count[C] = 0 (pos[C] = total)
        int rc = oge_exclusive_scan_u64(ctx, count, dst, C + 1);
        if (rc) return rc;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(n, dst + C, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipMemcpyAsync(x, stop + C - 1, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    };
    auto &RW = ctx->recwalk;
    if (d_off && RW.stream == d_stream && RW.base == rec_base && RW.limit == limit && RW.end == end && RW.n_ref == n_ref &&
        RW.C == C) {
        const uint64_t n = RW.n, x = RW.x;
        RW.stream = nullptr;
        if (cap < n + 1) return oge_fail(ctx, OGE_ERR_ARG, "offset capacity too small (need n + 1)");
        if (RW.rel && keep) {
            // a trusted caller's count and fill calls (keep: the stream is unchanged between them): expand the
            // count walk's slots
            k_rec_fill<<<G4, 256, 0, ctx->stream>>>(d_stream, rec_base, limit, end, CH, C, start, count, pos, RW.rel, RW.sc, d_off, cap);
            OGE_LAUNCH_CHECK(ctx);
            OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off + n, &x, 8, hipMemcpyHostToDevice, ctx->stream));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            *n_out = n;
            *exit = x;
            return OGE_OK;
        }
        // the count-only call on this stream converged just before: fill from its chunk starts and
        // offsets (still in the workspace), then check the walk joined and counted the same
        unsigned int h = 0;
        uint64_t n2 = 0, x2 = 0;
        int rc = walk_join(pos, d_off, &h);
        if (rc) return rc;
        if (!h && !(rc = scan_counts(pos2, &n2, &x2)) && n2 == n) {
            OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off + n, &x2, 8, hipMemcpyHostToDevice, ctx->stream));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            *n_out = n;
            *exit = x2;
            return OGE_OK;
        }
        if (rc) return rc;
        // the stream changed between the calls: the full walk below
    }
    RW.stream = nullptr;
    if (keep && !d_off) {
        // record slots for the fill call, a multiple of 4 (OGE_RECWALK_SLOTS: a test forces the overflow walk
        // with few)
        const char *e = getenv("OGE_RECWALK_SLOTS");
        SC = e ? (uint32_t)std::min<unsigned long>((std::max<unsigned long>(strtoul(e, nullptr, 10), 1ul) + 3) & ~3ul, 2048ul) : 512u;
        const uint64_t need = C * SC * 2;
        rel = rel_buf && rel_cap >= need ? (uint16_t *)rel_buf : (uint16_t *)ctx->ws("rec_rel", need);
        if (!rel) return OGE_ERR_HIP;
    }
    k_rec_guess<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, limit, end, at_end, n_ref, CH, C, start);
    OGE_LAUNCH_CHECK(ctx);
    // walk, then every chunk starts where its predecessor's walk stopped (k_rec_join), until no start
    // moves: the chain from chunk 0 then equals the sequential walk (and the slots of the last walk,
    // whose starts all held, are its records)
    unsigned int h = 0;
    for (int it = 0;; ++it) {
        int rc = walk_join(nullptr, nullptr, &h);
        if (rc) return rc;
        if (!(h & 1)) break;
        if (it > 64) return oge_fail(ctx, OGE_ERR_IO, "BAM record walk did not converge (corrupt stream?)");
    }
    if (h) return oge_fail(ctx, OGE_ERR_IO, "Invalid BAM record (block size out of range or record past the end of the stream)");
    uint64_t n = 0, x = 0;
    int rc = scan_counts(pos, &n, &x);
    if (rc) return rc;
    *n_out = n;
    *exit = x;
    if (!d_off) {
        RW.stream = d_stream, RW.base = rec_base, RW.limit = limit, RW.end = end, RW.n_ref = n_ref, RW.n = n, RW.C = C, RW.x = x;
        RW.rel = rel, RW.sc = SC;
        return OGE_OK;
    }
    if (cap < n + 1) return oge_fail(ctx, OGE_ERR_ARG, "offset capacity too small (need n + 1)");
    rel = nullptr;
    k_rec_walk<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, limit, end, CH, C, start, stop, count, pos, d_off, cap, nullptr, 0);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off + n, &x, 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}

extern "C" int oge_bam_record_offsets_dev(oge_ctx *ctx, const uint8_t *d_stream, uint64_t rec_base, uint64_t end, int32_t n_ref,
                                          uint64_t *d_off, uint64_t cap, uint64_t *n_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!n_out || rec_base > end || (end > rec_base && !d_stream)) return oge_fail(ctx, OGE_ERR_ARG, "bad argument");
    uint64_t x = 0;
    return oge_record_walk(ctx, d_stream, rec_base, end, end, true, n_ref, d_off, cap, n_out, &x);
}
