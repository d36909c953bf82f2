// inflate.hip -- BGZF decompression on the GPU, and the device-side BAM record boundary parse.
//
// Replaces `BgzfInputStream::decompress` (openge/src/util/bgzf_input_stream.cpp:65-142,208-240:
// inflateInit2(-15) per block at :116-123) and the record walk of `BamDeserializer::read`
// (util/bam_deserializer.h:143-193, block_size bounds at :160-163).  SURVEY §8f rows 1-2.
//
//   oge_bgzf_index (host)  walks the BGZF framing: per block the deflate byte range, the payload
//                          offset (prefix sum of ISIZE) and the stored CRC-32.
//   k_inflate              one wave per block.  The whole decoder runs wave-uniform (every lane
//                          computes the same symbol), so its state lives in scalar registers; the
//                          compressed bits stream through two VGPRs (256 bytes each, lane l holding
//                          word l) read with v_readlane, decode tables (10-bit direct lookup + the
//                          canonical count/offset walk for longer codes) sit in LDS.  Output goes
//                          through a 4 KiB LDS ring (literals written by lane 0, back-references
//                          copied by all 64 lanes at once) flushed to HBM 256 bytes at a time;
//                          only references further back than the ring read HBM.
//   k_crc_check            one 512-thread workgroup per block: the payload staged in LDS, slice-by-4
//                          CRC-32 combined across threads; any mismatch fails the call.
//   k_rec_walk             BAM record boundaries: one thread per 64 KiB chunk walks the block_size
//                          chain from its chunk's first record start (found by a 16-record
//                          plausibility chain); the host verifies that every chunk's walk ends where
//                          the next one starts and re-walks from the true end when it does not, so
//                          the result equals the sequential walk.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bam_layout.h"
#include "bgzf_dev.h"
#include "oge_ctx.h"

namespace {

using namespace oge_bgzf;

__constant__ uint16_t kLBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                    31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Wave-uniform LSB-first bit reader over the compressed bytes: a 64-bit scalar bit buffer refilled
// 32 bits at a time (v_readlane) from two 256-byte chunks held one word per lane.  All state is
// wave-uniform and kept in SGPRs (table entries are readfirstlane'd), which keeps the per-symbol path
// to a few scalar instructions.
struct Bits {
    const uint32_t *zw;
    uint64_t zwords;
    uint64_t wbase;  // absolute word index of relative word 0
    uint32_t widx;   // next relative word to enter the buffer
    uint32_t cbase;  // relative word held by lane 0 of `cur`
    uint32_t cur, nxt;
    uint64_t buf;    // low `cnt` bits are the next bits of the stream
    uint32_t cnt;
    __device__ __forceinline__ uint32_t ldw(uint32_t rel) const {
        const uint64_t w = wbase + rel;
        return w < zwords ? zw[w] : 0u;
    }
    __device__ __forceinline__ void refill() {
        while (cnt <= 32) {
            const uint32_t r = widx - cbase;
            const uint32_t w = __builtin_amdgcn_readlane(r < 64 ? cur : nxt, r & 63);
            buf |= (uint64_t)w << cnt;
            cnt += 32;
            ++widx;
            if (widx - cbase >= 64) {
                cur = nxt;
                cbase += 64;
                nxt = ldw(cbase + 64 + (threadIdx.x & 63));
            }
        }
    }
    __device__ void seek(uint64_t bit) {
        wbase = bit >> 5;
        widx = cbase = 0;
        const uint32_t l = threadIdx.x & 63;
        cur = ldw(l);
        nxt = ldw(64 + l);
        buf = 0;
        cnt = 0;
        refill();
        skip((uint32_t)(bit & 31));
    }
    __device__ __forceinline__ uint64_t bitpos() const { return (wbase + widx) * 32 - cnt; }
    __device__ __forceinline__ uint32_t peek() const { return (uint32_t)buf; }
    __device__ __forceinline__ void skip(uint32_t n) {  // n <= 32
        buf >>= n;
        cnt -= n;
        if (cnt <= 32) refill();
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) {  // n <= 31
        const uint32_t v = (uint32_t)buf & ((1u << n) - 1);
        skip(n);
        return v;
    }
};

// Canonical Huffman decode tables for one alphabet (RFC 1951 3.2.2): tab = 2^TB direct entries
// (symbol | length << 9, 0 = longer code or unused), cnt[len] and sym[] (symbols ordered by (length,
// value)) for the bit-by-bit walk.  Returns false for an over-subscribed code.
template <int TB>
__device__ bool build_table(const uint8_t *lens, int n, uint16_t *tab, uint32_t *cnt, uint16_t *sym, uint32_t *first,
                            uint32_t *offs) {
    const int lane = threadIdx.x;
    for (int i = lane; i < (1 << TB); i += 64) tab[i] = 0;
    uint32_t tot[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) tot[b] = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int s = c0 + lane;
        const uint32_t L = s < n ? lens[s] : 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) tot[b] += __popcll(__ballot(L == (uint32_t)b));
    }
    int left = 1;
#pragma unroll
    for (int b = 1; b < 16; ++b) {
        left = 2 * left - (int)tot[b];
        if (left < 0) return false;
    }
    if (lane == 0) {
        uint32_t code = 0, off = 0;
        cnt[0] = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            code = (code + (b > 1 ? tot[b - 1] : 0)) << (b > 1 ? 1 : 0);
            first[b] = code;
            offs[b] = off;
            off += tot[b];
            cnt[b] = tot[b];
        }
    }
    __syncthreads();
    uint32_t run[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) run[b] = 0;
    const uint64_t lt = (1ull << lane) - 1;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int s = c0 + lane;
        const uint32_t L = s < n ? lens[s] : 0;
        uint32_t rank = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const uint64_t m = __ballot(L == (uint32_t)b);
            if (L == (uint32_t)b) rank = run[b] + __popcll(m & lt);
            run[b] += __popcll(m);
        }
        if (L) {
            const uint32_t code = first[L] + rank;
            sym[offs[L] + rank] = (uint16_t)s;
            if (L <= (uint32_t)TB) {
                const uint32_t r = __builtin_bitreverse32(code) >> (32 - L);
                const uint16_t e = (uint16_t)(s | (L << 9));
                for (uint32_t k = 0; k < (1u << (TB - L)); ++k) tab[r | (k << L)] = e;
            }
        }
    }
    __syncthreads();
    return true;
}

template <int TB>
__device__ __forceinline__ int decode_sym(Bits &br, const uint16_t *tab, const uint32_t *cnt, const uint16_t *sym) {
    const uint32_t v = br.peek();
    const uint32_t e = __builtin_amdgcn_readfirstlane(tab[v & ((1u << TB) - 1)]);
    if (e) {
        br.skip(e >> 9);
        return (int)(e & 511);
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; ++len) {
        code |= (int)((v >> (len - 1)) & 1);
        const int count = (int)__builtin_amdgcn_readfirstlane(cnt[len]);
        if (code - count < first) {
            br.skip(len);
            return (int)__builtin_amdgcn_readfirstlane(sym[index + (code - first)]);
        }
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

constexpr uint32_t kRing = 4096;

enum { E_STORED = 1, E_CODE = 2, E_OVERRUN = 3, E_LEN = 4, E_DIST = 5, E_FAR = 6, E_TYPE = 7, E_PAST = 8, E_SIZE = 9,
       E_TABLE = 10, E_CRC = 11 };

__device__ __forceinline__ void report(uint32_t *err, uint32_t code, uint64_t blk) {
    atomicOr(err, 1u << code);
    atomicMin(err + 1, (uint32_t)min<uint64_t>(blk, 0xffffffffull));
}

__global__ void __launch_bounds__(64) k_inflate(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0,
                                                const uint64_t *__restrict__ d1, const uint64_t *__restrict__ uoff,
                                                uint8_t *__restrict__ out, uint32_t *__restrict__ err) {
    __shared__ uint16_t ltab[1024], dtab[1024], ctab[128];
    __shared__ uint32_t lcnt[16], dcnt[16], ccnt[16], tfirst[16], toffs[16];
    __shared__ uint16_t lsym[288], dsym[32], csym[19];
    __shared__ uint8_t lens[320], cl[19];
    // the most recent kRing output bytes; whole 256-byte chunks are flushed to `o` by the wave
    __shared__ uint8_t ring[kRing];
    const int lane = threadIdx.x;
    const uint64_t b = blockIdx.x;
    Bits br;
    br.zw = (const uint32_t *)z;
    br.zwords = (zbytes + 3) / 4;
    br.seek(d0[b] * 8);
    const uint64_t end_bit = d1[b] * 8;
    uint8_t *o = out + uoff[b];
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint32_t pos = 0, flushed = 0;
    int e = 0;
    auto flush = [&](uint32_t upto) {  // ring bytes [flushed, upto) -> o (byte stores, 64 lanes)
        for (uint32_t q0 = flushed; q0 < upto; q0 += 64) {  // uniform trip count keeps pos/flushed scalar
            const uint32_t q = q0 + lane;
            if (q < upto) o[q] = ring[q & (kRing - 1)];
        }
        flushed = upto;
    };
    for (;;) {
        const uint32_t h = br.get(3);
        const uint32_t type = h >> 1;
        if (type == 0) {
            br.skip((8 - (uint32_t)(br.bitpos() & 7)) & 7);
            const uint32_t len = br.get(16), nlen = br.get(16);
            const uint64_t src = br.bitpos() >> 3;
            if ((len ^ 0xffffu) != nlen || pos + len > osz || src + len > d1[b]) {
                e = E_STORED;
                break;
            }
            for (uint32_t i = 0; i < len; i += 64) {
                const uint32_t m = min(64u, len - i);
                if ((uint32_t)lane < m) ring[(pos + lane) & (kRing - 1)] = z[src + i + lane];
                pos += m;
                if (pos - flushed >= 256) flush(pos & ~255u);
            }
            br.seek(br.bitpos() + (uint64_t)len * 8);
        } else if (type == 1 || type == 2) {
            int hlit = 288, hdist = 30;
            if (type == 1) {
                for (int s = lane; s < 318; s += 64)
                    lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
                __syncthreads();
            } else {
                hlit = (int)br.get(5) + 257;
                hdist = (int)br.get(5) + 1;
                const int hclen = (int)br.get(4) + 4;
                if (hlit > 286 || hdist > 30) {
                    e = E_TABLE;
                    break;
                }
                if (lane < 19) cl[lane] = 0;
                __syncthreads();
                for (int i = 0; i < hclen; ++i) {
                    const uint32_t v = br.get(3);
                    if (lane == 0) cl[kClOrd[i]] = (uint8_t)v;
                }
                __syncthreads();
                if (!build_table<7>(cl, 19, ctab, ccnt, csym, tfirst, toffs)) {
                    e = E_TABLE;
                    break;
                }
                const int total = hlit + hdist;
                int i = 0;
                uint32_t prev = 0;
                while (i < total) {
                    const int s = decode_sym<7>(br, ctab, ccnt, csym);
                    if (s < 0) {
                        e = E_CODE;
                        break;
                    }
                    if (s < 16) {
                        if (lane == 0) lens[i] = (uint8_t)s;
                        prev = (uint32_t)s;
                        ++i;
                        continue;
                    }
                    uint32_t val = 0, rep;
                    if (s == 16) {
                        if (i == 0) {
                            e = E_TABLE;
                            break;
                        }
                        val = prev;
                        rep = 3 + br.get(2);
                    } else if (s == 17) {
                        rep = 3 + br.get(3);
                    } else {
                        rep = 11 + br.get(7);
                    }
                    if (i + (int)rep > total) {
                        e = E_TABLE;
                        break;
                    }
                    if ((uint32_t)lane < rep) lens[i + lane] = (uint8_t)val;
                    if (rep > 64 && (uint32_t)lane + 64 < rep) lens[i + 64 + lane] = (uint8_t)val;
                    if (rep > 128 && (uint32_t)lane + 128 < rep) lens[i + 128 + lane] = (uint8_t)val;
                    prev = val;
                    i += (int)rep;
                }
                if (e) break;
                __syncthreads();
                if (lens[256] == 0) {
                    e = E_TABLE;
                    break;
                }
            }
            // fixed codes: literal/length lens[0..288), distance lens[288..318)
            const uint8_t *dl = type == 1 ? lens + 288 : lens + hlit;
            if (!build_table<10>(lens, hlit, ltab, lcnt, lsym, tfirst, toffs) ||
                !build_table<10>(dl, hdist, dtab, dcnt, dsym, tfirst, toffs)) {
                e = E_TABLE;
                break;
            }
            for (;;) {
                pos = __builtin_amdgcn_readfirstlane(pos);
                flushed = __builtin_amdgcn_readfirstlane(flushed);
                int s = decode_sym<10>(br, ltab, lcnt, lsym);
                if (s < 0) {
                    e = E_CODE;
                    break;
                }
                if (s < 256) {
                    if (pos >= osz) {
                        e = E_OVERRUN;
                        break;
                    }
                    ring[pos & (kRing - 1)] = (uint8_t)s;  // every lane stores the same byte
                    ++pos;
                    if (pos - flushed >= 256) flush(pos & ~255u);
                    continue;
                }
                if (s == 256) break;
                s -= 257;
                if (s >= 29) {
                    e = E_LEN;
                    break;
                }
                const uint32_t L = kLBase[s] + br.get(kLExt[s]);
                const int ds = decode_sym<10>(br, dtab, dcnt, dsym);
                if (ds < 0 || ds >= 30) {
                    e = E_DIST;
                    break;
                }
                const uint32_t D = kDBase[ds] + br.get(kDExt[ds]);
                if (D > pos || pos + L > osz) {
                    e = E_FAR;
                    break;
                }
                if (D + 259 <= kRing) {  // the match cannot overwrite its own source slots
                    for (uint32_t i = 0; i < L; i += 64) {
                        const uint32_t j = i + lane;
                        uint8_t v = 0;
                        if (j < L) v = ring[(pos - D + (D >= L ? j : j % D)) & (kRing - 1)];
                        if (j < L) ring[(pos + j) & (kRing - 1)] = v;
                    }
                } else {  // far source: flush everything so far, then make the stores visible
                    flush(pos);
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                    for (uint32_t i = 0; i < L; i += 64) {
                        const uint32_t j = i + lane;
                        if (j < L) ring[(pos + j) & (kRing - 1)] = o[pos - D + j];
                    }
                }
                pos += L;
                if (pos - flushed >= 256) flush(pos & ~255u);
            }
            if (e) break;
        } else {
            e = E_TYPE;
            break;
        }
        if (br.bitpos() > end_bit) {
            e = E_PAST;
            break;
        }
        if (h & 1) break;
    }
    if (!e && pos != osz) e = E_SIZE;
    if (!e) flush(pos);
    if (e && lane == 0) report(err, e, b);
}

// ---------------------------------------------------------------- grouped (VALU) decoder
// G lanes decode one block; a wave runs 64 / G blocks at once.  The decoder state is per lane
// (uniform within the group), so it executes on the SIMD's vector ALU, four of which share the
// CU's single scalar unit that bounds k_inflate.  Each group owns its decode tables and an R-byte
// output ring in LDS; no workgroup barriers are used (one wave per workgroup, LDS is in order).
template <int G, int R, int LTB, int DTB>
struct GLds {
    uint16_t ltab[1 << LTB];
    uint16_t dtab[1 << DTB];
    uint16_t ctab[128];
    uint32_t lcnt[16], dcnt[16], ccnt[16];
    uint16_t lsym[288], dsym[32], csym[20];
    uint32_t aux[48];
    uint8_t lens[320], cl[32];
    uint8_t ring[R];
};

template <int G>
struct GBits {
    const uint32_t *zw;
    uint64_t zwords;
    uint64_t wbase;
    uint32_t widx, cbase;
    uint32_t cur, nxt;  // lane gl of the group holds words cbase + gl and cbase + G + gl
    uint64_t buf;
    uint32_t cnt;
    uint32_t gl;
    __device__ __forceinline__ uint32_t ldw(uint32_t rel) const {
        const uint64_t w = wbase + rel;
        return w < zwords ? zw[w] : 0u;
    }
    __device__ __forceinline__ void refill() {
        while (cnt <= 32) {
            const uint32_t r = widx - cbase;
            const uint32_t w = (uint32_t)__shfl((int)(r < (uint32_t)G ? cur : nxt), (int)(r & (G - 1)), G);
            buf |= (uint64_t)w << cnt;
            cnt += 32;
            ++widx;
            if (widx - cbase >= (uint32_t)G) {
                cur = nxt;
                cbase += G;
                nxt = ldw(cbase + G + gl);
            }
        }
    }
    __device__ void seek(uint64_t bit) {
        wbase = bit >> 5;
        widx = cbase = 0;
        cur = ldw(gl);
        nxt = ldw(G + gl);
        buf = 0;
        cnt = 0;
        refill();
        skip((uint32_t)(bit & 31));
    }
    __device__ __forceinline__ uint64_t bitpos() const { return (wbase + widx) * 32 - cnt; }
    __device__ __forceinline__ void skip(uint32_t n) {
        buf >>= n;
        cnt -= n;
        if (cnt <= 32) refill();
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) {
        const uint32_t v = (uint32_t)buf & ((1u << n) - 1);
        skip(n);
        return v;
    }
};

template <int G>
__device__ __forceinline__ uint64_t gballot(bool p, uint32_t gbase) {
    const uint64_t m = __ballot(p) >> gbase;
    return G == 64 ? m : (m & ((1ull << G) - 1));
}

template <int G, int TB>
__device__ bool gbuild(const uint8_t *lens, int n, uint16_t *tab, uint32_t *cnt, uint16_t *sym, uint32_t *aux, uint32_t gl,
                       uint32_t gbase) {
    // aux: 48 words of group scratch: first code [0,16), symbol offset [16,32), running rank [32,48).
    // Per-length values live in LDS (lane gl holds length gl's count) to keep VGPR pressure low.
    for (int i = gl; i < (1 << TB); i += G) tab[i] = 0;
    uint32_t mine = 0;  // lane b (1..15): number of codes of length b
    for (int c0 = 0; c0 < n; c0 += G) {
        const int s = c0 + (int)gl;
        const uint32_t L = s < n ? lens[s] : 0;
        for (int b = 1; b < 16; ++b) {
            const uint32_t c = __popcll(gballot<G>(L == (uint32_t)b, gbase));
            if ((int)gl == b) mine += c;
        }
    }
    for (uint32_t i = gl; i < 16; i += G) cnt[i] = 0;
    __builtin_amdgcn_wave_barrier();
    if (gl >= 1 && gl < 16) cnt[gl] = mine;
    __builtin_amdgcn_wave_barrier();
    int left = 1;
    uint32_t code = 0, off = 0;
    for (int b = 1; b < 16; ++b) {
        const uint32_t t = cnt[b];
        left = 2 * left - (int)t;
        code = (code + (b > 1 ? cnt[b - 1] : 0)) << (b > 1 ? 1 : 0);
        if ((int)gl == b) aux[b] = code, aux[16 + b] = off, aux[32 + b] = 0;
        off += t;
    }
    if (left < 0) return false;
    __builtin_amdgcn_wave_barrier();
    const uint64_t lt = (1ull << gl) - 1;
    for (int c0 = 0; c0 < n; c0 += G) {
        const int s = c0 + (int)gl;
        const uint32_t L = s < n ? lens[s] : 0;
        uint64_t my = 0;
        uint32_t mc = 0;
        for (int b = 1; b < 16; ++b) {
            const uint64_t m = gballot<G>(L == (uint32_t)b, gbase);
            if (L == (uint32_t)b) my = m;
            if ((int)gl == b) mc = __popcll(m);
        }
        if (L) {
            const uint32_t rank = aux[32 + L] + __popcll(my & lt);
            sym[aux[16 + L] + rank] = (uint16_t)s;
            if (L <= (uint32_t)TB) {
                const uint32_t r = __builtin_bitreverse32(aux[L] + rank) >> (32 - L);
                const uint16_t e = (uint16_t)(s | (L << 9));
                for (uint32_t k = 0; k < (1u << (TB - L)); ++k) tab[r | (k << L)] = e;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (gl >= 1 && gl < 16) aux[32 + gl] += mc;
        __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

template <int G, int TB>
__device__ __forceinline__ int gdecode(GBits<G> &br, const uint16_t *tab, const uint32_t *cnt, const uint16_t *sym) {
    const uint32_t v = (uint32_t)br.buf;
    const uint32_t e = tab[v & ((1u << TB) - 1)];
    if (e) {
        br.skip(e >> 9);
        return (int)(e & 511);
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; ++len) {
        code |= (int)((v >> (len - 1)) & 1);
        const int count = (int)cnt[len];
        if (code - count < first) {
            br.skip(len);
            return sym[index + (code - first)];
        }
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

template <int G, int R, int LTB, int DTB>
__global__ void __launch_bounds__(64) k_inflate_g(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ d0,
                                                  const uint64_t *__restrict__ d1, const uint64_t *__restrict__ uoff, uint64_t nblk,
                                                  uint8_t *__restrict__ out, uint32_t *__restrict__ err) {
    constexpr int NG = 64 / G;
    __shared__ GLds<G, R, LTB, DTB> gs[NG];
    const uint32_t lane = threadIdx.x, g = lane / G, gl = lane % G, gbase = g * G;
    const uint64_t b = (uint64_t)blockIdx.x * NG + g;
    if (b >= nblk) return;
    GLds<G, R, LTB, DTB> &S = gs[g];
    GBits<G> br;
    br.gl = gl;
    br.zw = (const uint32_t *)z;
    br.zwords = (zbytes + 3) / 4;
    br.seek(d0[b] * 8);
    const uint64_t end_bit = d1[b] * 8;
    uint8_t *o = out + uoff[b];
    const uint32_t osz = (uint32_t)(uoff[b + 1] - uoff[b]);
    uint32_t pos = 0, flushed = 0;
    int e = 0;
    auto flush = [&](uint32_t upto) {
        for (uint32_t q0 = flushed; q0 < upto; q0 += G) {
            const uint32_t q = q0 + gl;
            if (q < upto) o[q] = S.ring[q & (R - 1)];
        }
        flushed = upto;
    };
    for (;;) {
        const uint32_t h = br.get(3);
        const uint32_t type = h >> 1;
        if (type == 0) {
            br.skip((8 - (uint32_t)(br.bitpos() & 7)) & 7);
            const uint32_t len = br.get(16), nlen = br.get(16);
            const uint64_t src = br.bitpos() >> 3;
            if ((len ^ 0xffffu) != nlen || pos + len > osz || src + len > d1[b]) {
                e = E_STORED;
                break;
            }
            for (uint32_t i = 0; i < len; i += G) {
                const uint32_t m = min((uint32_t)G, len - i);
                if (gl < m) S.ring[(pos + gl) & (R - 1)] = z[src + i + gl];
                pos += m;
                if (pos - flushed >= 256) flush(pos & ~255u);
            }
            br.seek(br.bitpos() + (uint64_t)len * 8);
        } else if (type == 1 || type == 2) {
            int hlit = 288, hdist = 30;
            if (type == 1) {
                for (int s = gl; s < 318; s += G) S.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
                __builtin_amdgcn_wave_barrier();
            } else {
                hlit = (int)br.get(5) + 257;
                hdist = (int)br.get(5) + 1;
                const int hclen = (int)br.get(4) + 4;
                if (hlit > 286 || hdist > 30) {
                    e = E_TABLE;
                    break;
                }
                for (int i = gl; i < 19; i += G) S.cl[i] = 0;
                __builtin_amdgcn_wave_barrier();
                for (int i = 0; i < hclen; ++i) {
                    const uint32_t v = br.get(3);
                    S.cl[kClOrd[i]] = (uint8_t)v;  // every lane of the group stores the same byte
                }
                __builtin_amdgcn_wave_barrier();
                if (!gbuild<G, 7>(S.cl, 19, S.ctab, S.ccnt, S.csym, S.aux, gl, gbase)) {
                    e = E_TABLE;
                    break;
                }
                const int total = hlit + hdist;
                int i = 0;
                uint32_t prev = 0;
                while (i < total) {
                    const int sy = gdecode<G, 7>(br, S.ctab, S.ccnt, S.csym);
                    if (sy < 0) {
                        e = E_CODE;
                        break;
                    }
                    if (sy < 16) {
                        S.lens[i] = (uint8_t)sy;
                        prev = (uint32_t)sy;
                        ++i;
                        continue;
                    }
                    uint32_t val = 0, rep;
                    if (sy == 16) {
                        if (i == 0) {
                            e = E_TABLE;
                            break;
                        }
                        val = prev;
                        rep = 3 + br.get(2);
                    } else if (sy == 17) {
                        rep = 3 + br.get(3);
                    } else {
                        rep = 11 + br.get(7);
                    }
                    if (i + (int)rep > total) {
                        e = E_TABLE;
                        break;
                    }
                    for (uint32_t k = gl; k < rep; k += G) S.lens[i + k] = (uint8_t)val;
                    prev = val;
                    i += (int)rep;
                }
                if (e) break;
                __builtin_amdgcn_wave_barrier();
                if (S.lens[256] == 0) {
                    e = E_TABLE;
                    break;
                }
            }
            const uint8_t *dl = type == 1 ? S.lens + 288 : S.lens + hlit;
            if (!gbuild<G, LTB>(S.lens, hlit, S.ltab, S.lcnt, S.lsym, S.aux, gl, gbase) ||
                !gbuild<G, DTB>(dl, hdist, S.dtab, S.dcnt, S.dsym, S.aux, gl, gbase)) {
                e = E_TABLE;
                break;
            }
            for (;;) {
                int sy = gdecode<G, LTB>(br, S.ltab, S.lcnt, S.lsym);
                if (sy < 0) {
                    e = E_CODE;
                    break;
                }
                if (sy < 256) {
                    if (pos >= osz) {
                        e = E_OVERRUN;
                        break;
                    }
                    S.ring[pos & (R - 1)] = (uint8_t)sy;
                    ++pos;
                    if (pos - flushed >= 256) flush(pos & ~255u);
                    continue;
                }
                if (sy == 256) break;
                sy -= 257;
                if (sy >= 29) {
                    e = E_LEN;
                    break;
                }
                const uint32_t L = kLBase[sy] + br.get(kLExt[sy]);
                const int ds = gdecode<G, DTB>(br, S.dtab, S.dcnt, S.dsym);
                if (ds < 0 || ds >= 30) {
                    e = E_DIST;
                    break;
                }
                const uint32_t D = kDBase[ds] + br.get(kDExt[ds]);
                if (D > pos || pos + L > osz) {
                    e = E_FAR;
                    break;
                }
                // ring path iff the match cannot overwrite its own source slots (D + L <= R); a far
                // source is read back from HBM after flushing everything written so far
                if (D + 259 <= (uint32_t)R) {
                    for (uint32_t i = 0; i < L; i += G) {
                        const uint32_t j = i + gl;
                        uint8_t v = 0;
                        if (j < L) v = S.ring[(pos - D + (D >= L ? j : j % D)) & (R - 1)];
                        __builtin_amdgcn_wave_barrier();
                        if (j < L) S.ring[(pos + j) & (R - 1)] = v;
                        __builtin_amdgcn_wave_barrier();
                    }
                } else {
                    flush(pos);
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                    for (uint32_t i = 0; i < L; i += G) {
                        const uint32_t j = i + gl;
                        if (j < L) S.ring[(pos + j) & (R - 1)] = o[pos - D + j];
                    }
                }
                pos += L;
                if (pos - flushed >= 256) flush(pos & ~255u);
            }
            if (e) break;
        } else {
            e = E_TYPE;
            break;
        }
        if (br.bitpos() > end_bit) {
            e = E_PAST;
            break;
        }
        if (h & 1) break;
    }
    if (!e && pos != osz) e = E_SIZE;
    if (!e) flush(pos);
    if (e && gl == 0) report(err, e, b);
}

__global__ void __launch_bounds__(512) k_crc_check(const uint8_t *__restrict__ out, const uint64_t *__restrict__ uoff,
                                                   const uint32_t *__restrict__ crc, const uint32_t *__restrict__ zpow,
                                                   uint32_t *__restrict__ err) {
    __shared__ uint32_t in[kSlot / 4 + 4];
    __shared__ uint32_t crctab[4][256];
    __shared__ uint32_t zp[17][32];
    __shared__ uint32_t crcs[512];
    const int t = threadIdx.x;
    const uint64_t b = blockIdx.x;
    const uint32_t len = (uint32_t)(uoff[b + 1] - uoff[b]);
    if (len > kSlot) {
        if (t == 0) report(err, E_SIZE, b);
        return;
    }
    stage_words<512>(in, out + uoff[b], len, t);
    crc_setup<512>(crctab, zp, zpow, t);
    __syncthreads();
    const uint32_t c = crc_window512(in, len, crctab, zp, crcs, t);
    if (t == 0 && c != crc[b]) report(err, E_CRC, b);
}

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

// chunk c covers [p + c*CH, min(n, p + (c+1)*CH)); guess its first record start
__global__ void k_rec_guess(const uint8_t *__restrict__ d, uint64_t p, uint64_t n, int32_t n_ref, uint64_t CH, uint64_t C,
                            uint64_t *__restrict__ start) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (c == 0) {
        start[0] = p;
        return;
    }
    const uint64_t cut = p + c * CH, lim = min(n, cut + 20016);
    for (uint64_t s = cut; s < lim; ++s) {
        uint64_t q = s;
        int k = 0;
        for (; k < 16 && q < n && plausible(d, q, n, n_ref); ++k) q += 4 + rd32u(d + q);
        if (k == 16 || (q == n && k > 0)) {
            start[c] = s;
            return;
        }
    }
    start[c] = kNone;
}

// walk chunk c from start[c] to the first record start at or past the chunk end; with out != NULL
// also write the (absolute) offsets from pos[c]
__global__ void k_rec_walk(const uint8_t *__restrict__ d, uint64_t p, uint64_t n, uint64_t CH, uint64_t C,
                           const uint64_t *__restrict__ start, uint64_t *__restrict__ stop, uint64_t *__restrict__ count,
                           const uint64_t *__restrict__ pos, uint64_t *__restrict__ out) {
    const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t end = min(n, p + (c + 1) * CH);
    uint64_t q = start[c], k = 0;
    if (q == kNone) {
        stop[c] = kNone;
        count[c] = 0;
        return;
    }
    uint64_t *o = out ? out + pos[c] : nullptr;
    while (q < end) {
        if (q + 4 > n) break;
        const uint32_t bs = rd32u(d + q);
        if (bs < 32 || bs > 10000 || q + 4 + bs > n) break;
        if (o) o[k] = q;
        ++k;
        q += 4 + bs;
    }
    stop[c] = q < end ? kNone - 1 : q;  // kNone - 1: invalid record inside the chunk
    count[c] = k;
}

// chunk c + 1 starts where chunk c's walk stopped; *st bit 0: a start moved, bit 1: a stop that is
// invalid (or the last chunk's not at the end)
__global__ void k_rec_join(const uint64_t *__restrict__ stop, uint64_t *__restrict__ start, uint64_t C, uint64_t n,
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
    } else if (e != n) {
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

constexpr int kIdxPos = 16;  // byte positions per thread

constexpr uint32_t kStash = 4;  // candidate slots per 4096-position block in the counting pass

template <bool EMIT>
__global__ void __launch_bounds__(256) k_bgzf_cand(const uint8_t *__restrict__ z, uint64_t zbytes, uint32_t *__restrict__ cnt,
                                                   const uint32_t *__restrict__ base, uint64_t *__restrict__ cpos,
                                                   uint32_t *__restrict__ cbs, uint64_t *__restrict__ stash_pos = nullptr,
                                                   uint32_t *__restrict__ stash_bs = nullptr,
                                                   unsigned int *__restrict__ ovf = nullptr) {
    __shared__ uint32_t wsum[4];
    const uint32_t t = threadIdx.x;
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256 + t) * kIdxPos;
    uint32_t mine = 0;
    if (p0 < zbytes) {
        // the thread's 16 positions + 4 bytes of look-ahead in registers (one 16-byte load + one dword):
        // only a position whose 4 bytes are the gzip/deflate/FEXTRA signature 1f 8b 08 04 goes on to
        // bgzf_head's global loads (a bare 0x1f byte every 256 stalled the wave on dependent loads)
        const uint32_t *w = (const uint32_t *)(z + p0);
        uint32_t v[kIdxPos / 4 + 1];
        if (p0 + kIdxPos <= zbytes) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 q = *(const u32x4 *)w;
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
#pragma unroll
            for (int k = 0; k < kIdxPos / 4; ++k) v[k] = p0 + 4 * k + 4 <= zbytes ? w[k] : 0;
        }
        v[kIdxPos / 4] = p0 + kIdxPos + 4 <= zbytes ? w[kIdxPos / 4] : 0;
#pragma unroll
        for (int k = 0; k < kIdxPos; ++k) {
            const uint32_t sig = (k & 3) ? __builtin_amdgcn_alignbyte(v[(k >> 2) + 1], v[k >> 2], k & 3) : v[k >> 2];
            if (sig == 0x04088b1fu && p0 + k < zbytes && bgzf_head(z, zbytes, p0 + k)) ++mine;
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
        // stash: a block's candidates (nearly always 0 or 1 per 4096 bytes) in its kStash slots, so the
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
                if (p >= zbytes || z[p] != 31) continue;
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
        if (p >= zbytes || z[p] != 31) continue;
        const uint32_t bs = bgzf_head(z, zbytes, p);
        if (bs) cpos[o] = p, cbs[o] = bs, ++o;
    }
}

// chain check + per-block fields; nonempty[i] = payload size > 0
__global__ void k_bgzf_chain(const uint8_t *__restrict__ z, uint64_t zbytes, const uint64_t *__restrict__ cpos,
                             const uint32_t *__restrict__ cbs, uint64_t m, uint32_t *__restrict__ bad,
                             uint32_t *__restrict__ isz) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t p = cpos[i], e = p + cbs[i];
    const bool ok = (i == 0 ? p == 0 : cpos[i - 1] + cbs[i - 1] == p) && (i + 1 == m ? e == zbytes : true);
    const uint32_t s = z[e - 4] | ((uint32_t)z[e - 3] << 8) | ((uint32_t)z[e - 2] << 16) | ((uint32_t)z[e - 1] << 24);
    if (!ok || s > kSlot) atomicAdd(bad, 1u);
    isz[i] = s;
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

int oge_bgzf_index_ws(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, OgeBgzfIndex *ix) {
    hipSetDevice(ctx->device);
    ix->nblk = 0;
    ix->total = 0;
    if (!zbytes) return OGE_OK;
    if ((uintptr_t)d_z & 3) return 1;
    const uint64_t per_blk = 256ull * kIdxPos;
    const uint64_t G = (zbytes + per_blk - 1) / per_blk;
    if (G > 0xffffffffull) return 1;
    uint32_t *cnt = (uint32_t *)ctx->ws("bix_cnt", (G + 1) * 4);
    uint32_t *base = (uint32_t *)ctx->ws("bix_base", (G + 1) * 4);
    uint32_t *bad = (uint32_t *)ctx->ws("bix_bad", 16);
    uint64_t *stash_pos = (uint64_t *)ctx->ws("bix_stash_pos", G * kStash * 8);
    uint32_t *stash_bs = (uint32_t *)ctx->ws("bix_stash_bs", G * kStash * 4);
    if (!cnt || !base || !bad || !stash_pos || !stash_bs) return OGE_ERR_HIP;
    OGE_HIP_TRY(ctx, hipMemsetAsync(bad + 1, 0, 4, ctx->stream));
    k_bgzf_cand<false><<<(uint32_t)G, 256, 0, ctx->stream>>>(d_z, zbytes, cnt, nullptr, nullptr, nullptr, stash_pos, stash_bs,
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
    if (!m) return 1;
    uint64_t *cpos = (uint64_t *)ctx->ws("bix_cpos", m * 8);
    uint32_t *cbs = (uint32_t *)ctx->ws("bix_cbs", m * 4);
    uint32_t *isz = (uint32_t *)ctx->ws("bix_isz", (m + 1) * 4);
    uint32_t *slot = (uint32_t *)ctx->ws("bix_slot", (m + 1) * 4);
    if (!cpos || !cbs || !isz || !slot) return OGE_ERR_HIP;
    if (stash_ovf)  // a block with more than kStash candidates: the second scan places them
        k_bgzf_cand<true><<<(uint32_t)G, 256, 0, ctx->stream>>>(d_z, zbytes, cnt, base, cpos, cbs);
    else
        k_bgzf_unstash<<<oge_ceil_div(G, 256), 256, 0, ctx->stream>>>(cnt, base, G, stash_pos, stash_bs, cpos, cbs);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemsetAsync(bad, 0, 4, ctx->stream));
    k_bgzf_chain<<<oge_ceil_div(m, 256), 256, 0, ctx->stream>>>(d_z, zbytes, cpos, cbs, m, bad, isz);
    OGE_LAUNCH_CHECK(ctx);
    k_nonzero_u32<<<oge_ceil_div(m + 1, 256), 256, 0, ctx->stream>>>(isz, m, slot);
    OGE_LAUNCH_CHECK(ctx);
    rc = oge_exclusive_scan_u32(ctx, slot, slot, m + 1);
    if (rc) return rc;
    uint32_t hb[2] = {0, 0};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&hb[0], bad, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(&hb[1], slot + m, 4, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (hb[0]) return 1;
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
    uint32_t *zpow = (uint32_t *)ctx->ws("infl_zpow", 17 * 32 * 4);
    if (!err || !zpow) return OGE_ERR_HIP;
    static uint32_t zh[17][32];
    static bool zinit = false;
    if (!zinit) crc_zpow(zh), zinit = true;
    const uint32_t init[2] = {0, 0xffffffffu};
    OGE_HIP_TRY(ctx, hipMemcpyAsync(err, init, 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipMemcpyAsync(zpow, zh, sizeof(zh), hipMemcpyHostToDevice, ctx->stream));
    // decoder: OGE_INFLATE_GROUP unset = one lane per block (inflate_lane.hip); else lanes per block of the
    // grouped decoder -- 32, 16, or 0 = the wave-uniform scalar decoder k_inflate.
    // Measured on 20M C2 reads (5.68 GB): scalar 437 ms (bound by the CU's one scalar ALU), 32 lanes
    // with a 1 KiB ring 254 ms, 16 lanes 268-296 ms (divergence between the wave's groups); larger
    // rings or tables cost occupancy and were slower (2 KiB 327 ms, 8 KiB 591 ms).
    static const int inflate_group = [] {
        const char *v = getenv("OGE_INFLATE_GROUP");
        return v && *v ? atoi(v) : -1;
    }();
    if (inflate_group < 0) {  // default: the lane decoder (inflate_lane.hip), CRC fused into its phase 2
        OgeStageTimer *tm = ctx->begin_stage("bgzf_inflate");
        int rc = oge_inflate_lanes(ctx, d_z, zbytes, d_d0, d_d1, d_uoff, d_crc, nblk, d_out, err, zpow);
        ctx->end_stage(tm);
        if (rc) return rc;
    } else {
    OgeStageTimer *tm = ctx->begin_stage("bgzf_inflate");
    for (uint64_t b0 = 0; b0 < nblk; b0 += (1u << 30)) {
        const uint32_t nb = (uint32_t)std::min<uint64_t>(nblk - b0, 1u << 30);
        const uint64_t *a0 = d_d0 + b0, *a1 = d_d1 + b0, *au = d_uoff + b0;
        switch (inflate_group) {
        case 0: k_inflate<<<nb, 64, 0, ctx->stream>>>(d_z, zbytes, a0, a1, au, d_out, err); break;
        case 16: k_inflate_g<16, 1024, 9, 8><<<oge_ceil_div(nb, 4), 64, 0, ctx->stream>>>(d_z, zbytes, a0, a1, au, nb, d_out, err); break;
        default: k_inflate_g<32, 1024, 10, 8><<<oge_ceil_div(nb, 2), 64, 0, ctx->stream>>>(d_z, zbytes, a0, a1, au, nb, d_out, err); break;
        }
        OGE_LAUNCH_CHECK(ctx);
    }
    ctx->end_stage(tm);
    if (d_crc) {
        OgeStageTimer *tc = ctx->begin_stage("bgzf_crc");
        for (uint64_t b0 = 0; b0 < nblk; b0 += (1u << 30)) {
            const uint32_t nb = (uint32_t)std::min<uint64_t>(nblk - b0, 1u << 30);
            k_crc_check<<<nb, 512, 0, ctx->stream>>>(d_out, d_uoff + b0, d_crc + b0, zpow, err);
            OGE_LAUNCH_CHECK(ctx);
        }
        ctx->end_stage(tc);
    }
    }
    uint32_t got[2];
    OGE_HIP_TRY(ctx, hipMemcpyAsync(got, err, 8, hipMemcpyDeviceToHost, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (got[0]) {
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

extern "C" int oge_bam_record_offsets_dev(oge_ctx *ctx, const uint8_t *d_stream, uint64_t rec_base, uint64_t end, int32_t n_ref,
                                          uint64_t *d_off, uint64_t cap, uint64_t *n_out) {
    if (!ctx) return oge_fail(nullptr, OGE_ERR_ARG, "null ctx");
    if (!n_out || rec_base > end || (end > rec_base && !d_stream)) return oge_fail(ctx, OGE_ERR_ARG, "bad argument");
    hipSetDevice(ctx->device);
    *n_out = 0;
    const uint64_t CH = 1ull << 16;
    const uint64_t C = std::max<uint64_t>(1, (end - rec_base + CH - 1) / CH);
    uint64_t *ws = (uint64_t *)ctx->ws("rec_walk", (5 * C + 4) * 8 + 64);
    if (!ws) return OGE_ERR_HIP;
    // start[C], stop[C], count[C + 1], pos[C + 1], pos2[C + 1], st
    uint64_t *start = ws, *stop = ws + C, *count = ws + 2 * C, *pos = ws + 3 * C + 1, *pos2 = ws + 4 * C + 2;
    unsigned int *st = (unsigned int *)(ws + 5 * C + 3);
    if (end == rec_base) {
        if (d_off && cap >= 1) OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off, &end, 8, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    }
    const uint32_t TB = 128, G = oge_ceil_div(C, TB);
    // one walk + join pass: *st bit 0 = a start moved, bit 1 = an invalid or unjoined stop
    auto walk_join = [&](uint64_t *pos_arg, uint64_t *out, unsigned int *h) -> int {
        OGE_HIP_TRY(ctx, hipMemsetAsync(st, 0, 4, ctx->stream));
        k_rec_walk<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, end, CH, C, start, stop, count, pos_arg, out);
        OGE_LAUNCH_CHECK(ctx);
        k_rec_join<<<G, TB, 0, ctx->stream>>>(stop, start, C, end, st);
        OGE_LAUNCH_CHECK(ctx);
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h, st, 4, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    };
    // n = the sum of the chunk counts, pos = their exclusive scan
    auto scan_counts = [&](uint64_t *dst, uint64_t *n) -> int {
        OGE_HIP_TRY(ctx, hipMemsetAsync(count + C, 0, 8, ctx->stream));  // count[C] = 0 (pos[C] = total)
        int rc = oge_exclusive_scan_u64(ctx, count, dst, C + 1);
        if (rc) return rc;
        OGE_HIP_TRY(ctx, hipMemcpyAsync(n, dst + C, 8, hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OGE_OK;
    };
    auto &RW = ctx->recwalk;
    if (d_off && RW.stream == d_stream && RW.base == rec_base && RW.end == end && RW.n_ref == n_ref && RW.C == C) {
        // the count-only call on this stream converged just before: fill from its chunk starts and
        // offsets (still in the workspace), then check the walk joined and counted the same
        const uint64_t n = RW.n;
        RW.stream = nullptr;
        if (cap < n + 1) return oge_fail(ctx, OGE_ERR_ARG, "offset capacity too small (need n + 1)");
        unsigned int h = 0;
        uint64_t n2 = 0;
        int rc = walk_join(pos, d_off, &h);
        if (rc) return rc;
        if (!h && !(rc = scan_counts(pos2, &n2)) && n2 == n) {
            OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off + n, &end, 8, hipMemcpyHostToDevice, ctx->stream));
            OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            *n_out = n;
            return OGE_OK;
        }
        if (rc) return rc;
        // the stream changed between the calls: the full walk below
    }
    RW.stream = nullptr;
    k_rec_guess<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, end, n_ref, CH, C, start);
    OGE_LAUNCH_CHECK(ctx);
    // walk, then every chunk starts where its predecessor's walk stopped (k_rec_join), until no start
    // moves: the chain from chunk 0 then equals the sequential walk
    unsigned int h = 0;
    for (int it = 0;; ++it) {
        int rc = walk_join(nullptr, nullptr, &h);
        if (rc) return rc;
        if (!(h & 1)) break;
        if (it > 64) return oge_fail(ctx, OGE_ERR_IO, "BAM record walk did not converge (corrupt stream?)");
    }
    if (h) return oge_fail(ctx, OGE_ERR_IO, "Invalid BAM record (block size out of range or record past the end of the stream)");
    uint64_t n = 0;
    int rc = scan_counts(pos, &n);
    if (rc) return rc;
    *n_out = n;
    if (!d_off) {
        RW.stream = d_stream, RW.base = rec_base, RW.end = end, RW.n_ref = n_ref, RW.n = n, RW.C = C;
        return OGE_OK;
    }
    if (cap < n + 1) return oge_fail(ctx, OGE_ERR_ARG, "offset capacity too small (need n + 1)");
    k_rec_walk<<<G, TB, 0, ctx->stream>>>(d_stream, rec_base, end, CH, C, start, stop, count, pos, d_off);
    OGE_LAUNCH_CHECK(ctx);
    OGE_HIP_TRY(ctx, hipMemcpyAsync(d_off + n, &end, 8, hipMemcpyHostToDevice, ctx->stream));
    OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return OGE_OK;
}
