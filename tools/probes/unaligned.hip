// Probe: do unaligned 16-byte global loads/stores (global_load/store_dwordx4 at byte offsets) give
// correct data on gfx950?  And how fast are they vs aligned?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>

__global__ void copy16(const uint8_t *src, uint8_t *dst, size_t nchunks, int soff, int doff) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < nchunks; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = *(const uint4 *)(src + soff + 16 * i);
        *(uint4 *)(dst + doff + 16 * i) = v;
    }
}

int main() {
    const size_t N = 1ull << 30;  // 1 GiB
    uint8_t *s, *d;
    hipMalloc(&s, N + 64);
    hipMalloc(&d, N + 64);
    std::vector<uint8_t> h(N + 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + 7);
    hipMemcpy(s, h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cases[][2] = {{0, 0}, {1, 0}, {3, 5}, {7, 13}, {0, 9}};
    for (auto &c : cases) {
        hipMemset(d, 0, N + 64);
        size_t nch = N / 16;
        copy16<<<4096, 256>>>(s, d, nch, c[0], c[1]);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) copy16<<<4096, 256>>>(s, d, nch, c[0], c[1]);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        hipError_t e = hipGetLastError();
        std::vector<uint8_t> o(N + 64);
        hipMemcpy(o.data(), d, o.size(), hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t i = 0; i < N; i += 4097) if (o[c[1] + i] != h[c[0] + i]) ++bad;
        printf("soff=%d doff=%d err=%s bad=%zu  %.1f GB/s (read+write)\n", c[0], c[1], hipGetErrorString(e), bad,
               2.0 * N * 5 / (ms / 1e3) / 1e9);
    }
    return 0;
}
