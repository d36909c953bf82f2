// dev_util.h -- small gfx950 device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Append one slot per lane whose `pred` is set, with ONE atomic per wave (ballot + popcount).
// Per-thread atomics on a single counter serialise at the L2 (~88 ops/us per word on MI355X,
// MI355X_MICROARCH.md "dequeue" row); this keeps it to one per wave.  Must be reached by every
// lane of the wave (convergent).  Returns the lane's slot (meaningless where !pred).
__device__ __forceinline__ uint32_t oge_wave_append(bool pred, unsigned int *counter) {
    const uint64_t m = __ballot(pred);
    if (m == 0) return 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned int)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// Unaligned little-endian 32-bit load from a byte address: two aligned dword loads + shift.
// May read up to 3 bytes past p+4 (arenas carry >= 16 bytes of tail slack).
__device__ __forceinline__ uint32_t oge_ldu32(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t lo = q[0];
    if (!sh) return lo;
    const uint32_t hi = q[1];
    return (lo >> sh) | (hi << (32 - sh));
}
__device__ __forceinline__ uint16_t oge_ldu16(const uint8_t *p) { return (uint16_t)(oge_ldu32(p) & 0xFFFF); }

__device__ __forceinline__ uint32_t oge_wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
