// bgzf_dev.h -- device helpers shared by the BGZF deflate (bgzf.hip) and inflate (inflate.hip)
// kernels: LDS payload staging, slice-by-4 CRC-32 with zero-operator combining.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// Global-address-space pointers.  A pointer rebuilt from an integer is a generic (flat) pointer, and on
// gfx9 a flat load or store also counts in lgkmcnt: every later wait for an LDS read then waits for
// that HBM access too.  Kernels that mix LDS table lookups with in-flight global traffic cast to this.
#define OGE_G __attribute__((address_space(1)))

namespace oge_bgzf {

constexpr uint32_t kPay = 65280;   // BGZF payload per block written here
constexpr uint32_t kSlot = 65536;  // max BGZF block size (and max payload accepted on input)

// inflate error bits (err[0] |= 1 << code; err[1] = the first failing block)
enum InflErr { E_STORED = 1, E_CODE = 2, E_OVERRUN = 3, E_LEN = 4, E_DIST = 5, E_FAR = 6, E_TYPE = 7, E_PAST = 8, E_SIZE = 9,
               E_TABLE = 10, E_CRC = 11, E_BITS = 12 };

__device__ __forceinline__ uint32_t ld32(const uint32_t *w, uint32_t p) {  // unaligned LDS read
    const uint32_t a = w[p >> 2], b = w[(p >> 2) + 1];
    return __builtin_amdgcn_alignbyte(b, a, p & 3);
}

// Padded LDS byte layouts: one spare word after every 2^PS words, so word w lives at w + (w >> PS).
// Threads that each walk their own 2^PS-word (or 2^(PS+1)-word) piece then start in different banks
// (a 64- or 128-byte stride otherwise puts a wave's 64 lanes on 2-4 banks).  PS = 31: no padding.
template <int PS>
__device__ __forceinline__ uint32_t pw(uint32_t w) { return PS >= 31 ? w : w + (w >> PS); }
template <int PS>
__device__ __forceinline__ uint32_t ld32p(const uint32_t *in, uint32_t p) {
    const uint32_t w = p >> 2, a = in[pw<PS>(w)];
    if (!(p & 3)) return a;
    return __builtin_amdgcn_alignbyte(in[pw<PS>(w + 1)], a, p & 3);
}
template <int PS>
__device__ __forceinline__ uint32_t byte_at(const uint32_t *in, uint32_t p) {
    return (in[pw<PS>(p >> 2)] >> (8 * (p & 3))) & 0xff;
}

__device__ __forceinline__ uint32_t crc_mat(const uint32_t *M, uint32_t c) {  // GF(2) matrix x vector
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) r ^= (uint32_t)(-(int32_t)((c >> b) & 1)) & M[b];
    return r;
}

// Stage len bytes at s (any alignment) into LDS words in[0 .. (len+3)/4 + 4), zero padded.
// Aligned dword loads, funnel-shifted, U loads in flight per thread.
template <int NT, int PS = 31>
__device__ void stage_words(uint32_t *in, const uint8_t *s, uint32_t len, int t) {
    const uintptr_t a = (uintptr_t)s & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
    const OGE_G uint32_t *W = (const OGE_G uint32_t *)a;
    const uint32_t nw = (len + 3) / 4;
    const uint32_t safe = len / 4;  // words wholly inside the payload
    constexpr int U = 8;
    for (uint32_t k0 = t; k0 < safe; k0 += U * NT) {
        uint32_t lo[U], hi[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = min(k0 + j * NT, safe - 1);
            lo[j] = W[k];
            hi[j] = sh ? W[k + 1] : 0;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t k = k0 + j * NT;
            if (k < safe) in[pw<PS>(k)] = sh ? __builtin_amdgcn_alignbyte(hi[j], lo[j], sh) : lo[j];
        }
    }
    for (uint32_t k = safe + t; k < nw + 4; k += NT) {
        uint32_t v = 0;
        if (k < nw)
            for (int b = 0; b < 4; ++b)
                if (4 * k + b < len) v |= (uint32_t)((const OGE_G uint8_t *)s)[4 * k + b] << (8 * b);
        in[pw<PS>(k)] = v;
    }
}

// Slice-by-NSL tables (NSL = 4, or 1 for the byte table only) and the 2^k-zero-byte operators (zpow
// from the host, 17 x 32 words, k = 0..16).
template <int NT, int NSL = 4>
__device__ void crc_setup(uint32_t (*crctab)[256], uint32_t (*zp)[32], const uint32_t *zpow, int t) {
    if (t < 256) {
        auto byte_step = [](uint32_t c) {
            for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (uint32_t)(-(int32_t)(c & 1)));
            return c;
        };
        uint32_t c = byte_step(t);
        crctab[0][t] = c;
        for (int k = 1; k < NSL; ++k) c = (c >> 8) ^ byte_step(c & 0xff), crctab[k][t] = c;
    }
    for (int i = t; i < 17 * 32; i += NT) zp[i >> 5][i & 31] = zpow[i];
}

// The 0xffffffff preset carried over len zero bytes: Z_len(0xffffffff) from the 2^k operators, one GF(2)
// matrix-vector product per set bit of len (each 32 dependent LDS reads) -- except for the 65,280-byte
// payload of every full BGZF block, whose value is a constant (python: 32-bit CRC register 0xffffffff
// stepped over 65,280 zero bytes, reflected polynomial 0xEDB88320).
constexpr uint32_t kPresetFull = 0x012c2d38u;
__device__ __forceinline__ uint32_t crc_preset(uint32_t len, const uint32_t (*zp)[32]) {
    if (len == kPay) return kPresetFull;
    uint32_t r = 0xffffffffu;
    for (int k = 0; k < 17; ++k)
        if ((len >> k) & 1) r = crc_mat(zp[k], r);
    return r;
}

// CRC-32 of a payload of len (<= 65536) bytes with 512 threads; the result is valid in thread 0.
// The data is right-aligned in a 65536-byte window (leading zeros leave a zero register unchanged);
// thread t owns window bytes [128t, 128t + 128) and passes the CRC of its piece (zero register start) to
// crc_combine512, which combines pieces pairwise with crc(A || B) = Z_|B|(crc A) ^ crc B -- six levels
// inside each wave by shuffles, the last three over the eight wave results (one barrier) -- and the
// whole with the 0xffffffff preset.
__device__ __forceinline__ uint32_t crc_word(const uint32_t (*crctab)[256], uint32_t c) {
    return crctab[3][c & 0xff] ^ crctab[2][(c >> 8) & 0xff] ^ crctab[1][(c >> 16) & 0xff] ^ crctab[0][c >> 24];
}

__device__ inline uint32_t crc_combine512(uint32_t c, uint32_t len, const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lane = t & 63;
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {  // pieces of 128 << lv bytes, pairs inside the wave
        const uint32_t o = __shfl_down(c, 1u << lv, 64);
        if (!(lane & ((2u << lv) - 1))) c = crc_mat(zp[7 + lv], c) ^ o;
    }
    if (lane == 0) crcs[t >> 6] = c;
    __syncthreads();
    uint32_t r = 0xffffffffu;
    if (t < 64) {
        c = t < 8 ? crcs[t] : 0u;
#pragma unroll
        for (int lv = 0; lv < 3; ++lv) {  // 8192-byte wave pieces
            const uint32_t o = __shfl_down(c, 1u << lv, 64);
            if (!(t & ((2u << lv) - 1))) c = crc_mat(zp[13 + lv], c) ^ o;
        }
        if (t == 0) r = crc_preset(len, zp);
    }
    return ~(r ^ c);
}

// 512 threads with per-lane operators of 16 lanes (2 KiB of LDS: the deflate emit's two workgroups per CU
// leave no room for 64): lane l carries its 128-byte piece's register over 128 (15 - l % 16) bytes with
// zl[.][l % 16], the 16-lane groups XOR, two levels join the four 2048-byte group pieces of a wave, three
// the eight wave pieces -- three matrix-vector products per lane instead of six before the barrier
__device__ inline uint32_t crc_combine512l(uint32_t c, uint32_t len, const uint32_t (*zl)[16], const uint32_t (*zp)[32],
                                           uint32_t *crcs, int t) {
    const uint32_t lane = t & 63;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) v ^= (uint32_t)(-(int32_t)((c >> b) & 1)) & zl[b][lane & 15];
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) v ^= __shfl_xor(v, d, 64);
#pragma unroll
    for (int lv = 0; lv < 2; ++lv) {  // 2048-byte group pieces
        const uint32_t o = __shfl_down(v, 16u << lv, 64);
        if (!(lane & ((32u << lv) - 1))) v = crc_mat(zp[11 + lv], v) ^ o;
    }
    if (lane == 0) crcs[t >> 6] = v;
    __syncthreads();
    uint32_t r = 0xffffffffu;
    if (t < 64) {
        c = t < 8 ? crcs[t] : 0u;
#pragma unroll
        for (int lv = 0; lv < 3; ++lv) {  // 8192-byte wave pieces
            const uint32_t o = __shfl_down(c, 1u << lv, 64);
            if (!(t & ((2u << lv) - 1))) c = crc_mat(zp[13 + lv], c) ^ o;
        }
        if (t == 0) r = crc_preset(len, zp);
    }
    return ~(r ^ c);
}

// The same for NT = 1024 threads (pieces of 64 bytes, sixteen waves): six in-wave levels, four over
// the wave results.
__device__ inline uint32_t crc_combine1024(uint32_t c, uint32_t len, const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lane = t & 63;
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {  // pieces of 64 << lv bytes, pairs inside the wave
        const uint32_t o = __shfl_down(c, 1u << lv, 64);
        if (!(lane & ((2u << lv) - 1))) c = crc_mat(zp[6 + lv], c) ^ o;
    }
    if (lane == 0) crcs[t >> 6] = c;
    __syncthreads();
    uint32_t r = 0xffffffffu;
    if (t < 64) {
        c = t < 16 ? crcs[t] : 0u;
#pragma unroll
        for (int lv = 0; lv < 4; ++lv) {  // 4096-byte wave pieces
            const uint32_t o = __shfl_down(c, 1u << lv, 64);
            if (!(t & ((2u << lv) - 1))) c = crc_mat(zp[12 + lv], c) ^ o;
        }
        if (t == 0) r = crc_preset(len, zp);
    }
    return ~(r ^ c);
}

// The same with per-lane operators (r04): lane l's register is carried over the 64 (63 - l) bytes that
// follow its piece inside the wave's 4096 bytes by its own matrix zl[.][l] (zl = [bit][lane], a wave's 64
// reads hit 64 banks) and the wave XORs the results -- one matrix-vector product per lane instead of six
// shuffle levels of them (crc_zlane builds zl on the host)
__device__ inline uint32_t crc_combine1024l(uint32_t c, uint32_t len, const uint32_t (*zl)[64], const uint32_t (*zp)[32],
                                            uint32_t *crcs, int t) {
    const uint32_t lane = t & 63;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) v ^= (uint32_t)(-(int32_t)((c >> b) & 1)) & zl[b][lane];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) v ^= __shfl_xor(v, d, 64);
    if (lane == 0) crcs[t >> 6] = v;
    __syncthreads();
    uint32_t r = 0xffffffffu;
    if (t < 64) {
        c = t < 16 ? crcs[t] : 0u;
#pragma unroll
        for (int lv = 0; lv < 4; ++lv) {  // 4096-byte wave pieces
            const uint32_t o = __shfl_down(c, 1u << lv, 64);
            if (!(t & ((2u << lv) - 1))) c = crc_mat(zp[12 + lv], c) ^ o;
        }
        if (t == 0) r = crc_preset(len, zp);
    }
    return ~(r ^ c);
}

// 1024 threads over the payload staged in LDS (padded layout PS): thread t owns window bytes
// [64t, 64t + 64) of the right-aligned 65536-byte window
template <int PS = 31>
__device__ uint32_t crc_window1024(const uint32_t *in, uint32_t len, const uint32_t (*crctab)[256], const uint32_t (*zp)[32],
                                   uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 64u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;
#pragma unroll 4
        for (int i = 0; i < 16; ++i) c = crc_word(crctab, c ^ ld32p<PS>(in, d0 + 4 * i));
    } else if (w0 + 64 > lead) {
        for (uint32_t d = 0; d < w0 + 64 - lead; ++d) c = crctab[0][(c ^ byte_at<PS>(in, d)) & 0xff] ^ (c >> 8);
    }
    return crc_combine1024(c, len, zp, crcs, t);
}
template <int PS = 31>
__device__ uint32_t crc_window1024l(const uint32_t *in, uint32_t len, const uint32_t (*crctab)[256], const uint32_t (*zl)[64],
                                    const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 64u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;
#pragma unroll 4
        for (int i = 0; i < 16; ++i) c = crc_word(crctab, c ^ ld32p<PS>(in, d0 + 4 * i));
    } else if (w0 + 64 > lead) {
        for (uint32_t d = 0; d < w0 + 64 - lead; ++d) c = crctab[0][(c ^ byte_at<PS>(in, d)) & 0xff] ^ (c >> 8);
    }
    return crc_combine1024l(c, len, zl, zp, crcs, t);
}

// the payload staged in LDS (padded layout PS)
template <int PS = 31>
__device__ uint32_t crc_window512(const uint32_t *in, uint32_t len, const uint32_t (*crctab)[256], const uint32_t (*zp)[32],
                                  uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 128u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;
#pragma unroll 4
        for (int i = 0; i < 32; ++i) c = crc_word(crctab, c ^ ld32p<PS>(in, d0 + 4 * i));
    } else if (w0 + 128 > lead) {
        for (uint32_t d = 0; d < w0 + 128 - lead; ++d) c = crctab[0][(c ^ byte_at<PS>(in, d)) & 0xff] ^ (c >> 8);
    }
    return crc_combine512(c, len, zp, crcs, t);
}

// the payload read from global memory at s (any alignment): aligned dword loads, funnel-shifted;
// the byte table only (crctab[0]), so a caller needs 1 KiB of LDS for it
__device__ inline uint32_t crc_global512(const uint8_t *s, uint32_t len, const uint32_t (*crctab)[256],
                                         const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 128u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;  // the piece is payload bytes [d0, d0 + 128)
        const uintptr_t a = (uintptr_t)(s + d0);
        const uint32_t sh = (uint32_t)(a & 3);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)(a & ~(uintptr_t)3);
        uint32_t raw[33];
#pragma unroll
        for (int k = 0; k < 33; ++k) raw[k] = (k < 32 || sh) ? W[k] : 0u;  // a 33rd word only when unaligned
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            c ^= sh ? __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh) : raw[i];
#pragma unroll
            for (int b = 0; b < 4; ++b) c = crctab[0][c & 0xff] ^ (c >> 8);
        }
    } else if (w0 + 128 > lead) {
        const OGE_G uint8_t *b = (const OGE_G uint8_t *)s;
        for (uint32_t d = 0; d < w0 + 128 - lead; ++d) c = crctab[0][(c ^ b[d]) & 0xff] ^ (c >> 8);
    }
    return crc_combine512(c, len, zp, crcs, t);
}

// the same with the slice-by-4 tables (crctab[0..3]): four independent lookups per word, so a thread's
// 32-word chain is 32 table round trips instead of 128
__device__ inline uint32_t crc_global512x4(const uint8_t *s, uint32_t len, const uint32_t (*crctab)[256],
                                           const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 128u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;
        const uintptr_t a = (uintptr_t)(s + d0);
        const uint32_t sh = (uint32_t)(a & 3);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)(a & ~(uintptr_t)3);
        uint32_t raw[33];
#pragma unroll
        for (int k = 0; k < 33; ++k) raw[k] = (k < 32 || sh) ? W[k] : 0u;
#pragma unroll
        for (int i = 0; i < 32; ++i) c = crc_word(crctab, c ^ (sh ? __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh) : raw[i]));
    } else if (w0 + 128 > lead) {
        const OGE_G uint8_t *b = (const OGE_G uint8_t *)s;
        for (uint32_t d = 0; d < w0 + 128 - lead; ++d) c = crctab[0][(c ^ b[d]) & 0xff] ^ (c >> 8);
    }
    return crc_combine512(c, len, zp, crcs, t);
}
__device__ inline uint32_t crc_global512x4l(const uint8_t *s, uint32_t len, const uint32_t (*crctab)[256], const uint32_t (*zl)[16],
                                            const uint32_t (*zp)[32], uint32_t *crcs, int t) {
    const uint32_t lead = kSlot - len, w0 = t * 128u;
    uint32_t c = 0;
    if (w0 >= lead) {
        const uint32_t d0 = w0 - lead;
        const uintptr_t a = (uintptr_t)(s + d0);
        const uint32_t sh = (uint32_t)(a & 3);
        const OGE_G uint32_t *W = (const OGE_G uint32_t *)(a & ~(uintptr_t)3);
        uint32_t raw[33];
#pragma unroll
        for (int k = 0; k < 33; ++k) raw[k] = (k < 32 || sh) ? W[k] : 0u;
#pragma unroll
        for (int i = 0; i < 32; ++i) c = crc_word(crctab, c ^ (sh ? __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh) : raw[i]));
    } else if (w0 + 128 > lead) {
        const OGE_G uint8_t *b = (const OGE_G uint8_t *)s;
        for (uint32_t d = 0; d < w0 + 128 - lead; ++d) c = crctab[0][(c ^ b[d]) & 0xff] ^ (c >> 8);
    }
    return crc_combine512l(c, len, zl, zp, crcs, t);
}

// host: zero-byte operators Z_{2^k}, k = 0..16 (columns = images of the 32 basis bits)
inline void crc_zpow(uint32_t z[17][32]) {
    for (int b = 0; b < 32; ++b) {  // one zero byte
        uint32_t c = 1u << b;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (uint32_t)(-(int32_t)(c & 1)));
        z[0][b] = c;
    }
    for (int k = 1; k < 17; ++k)
        for (int b = 0; b < 32; ++b) {
            uint32_t v = z[k - 1][b], r = 0;
            for (int j = 0; j < 32; ++j)
                if ((v >> j) & 1) r ^= z[k - 1][j];
            z[k][b] = r;
        }
}

// host: the per-lane operators of crc_combine1024l (W = 64) / crc_combine512l (W = 16) for pieces of P = 2^k
// bytes: zl[b * W + l] = column b of Z_{P (W - 1 - l)}
template <int W>
inline void crc_zlane(const uint32_t z[17][32], uint32_t P, uint32_t *zl) {
    int k = 0;
    while ((1u << k) < P) ++k;
    uint32_t M[32];
    for (int b = 0; b < 32; ++b) M[b] = 1u << b;  // Z_0
    for (int j = 0; j < W; ++j) {               // M = Z_{P j}
        for (int b = 0; b < 32; ++b) zl[b * W + W - 1 - j] = M[b];
        for (int b = 0; b < 32; ++b) {
            uint32_t r = 0;
            for (int i = 0; i < 32; ++i)
                if ((M[b] >> i) & 1) r ^= z[k][i];
            M[b] = r;
        }
    }
}

}  // namespace oge_bgzf
