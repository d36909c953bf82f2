"""Experiment: host<->device copy bandwidth from page-locked memory, one stream vs several, chunk sizes,
both directions at once (profiling aid for the PCIe-inclusive leg, not a test)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
N = 16 << 30
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(N, dtype=torch.uint8, pin_memory=True)
d = torch.empty(N, dtype=torch.uint8, device="cuda")
d2 = torch.empty(N, dtype=torch.uint8, device="cuda")
h.fill_(1)
torch.cuda.synchronize()
streams = []
for _ in range(8):
    s = ctypes.c_void_p()
    hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    streams.append(s)


def copy(dst, src, kind, nstreams, chunk):
    t = time.perf_counter()
    k = 0
    for o in range(0, N, chunk):
        hip.hipMemcpyAsync(ctypes.c_void_p(dst + o), ctypes.c_void_p(src + o), ctypes.c_size_t(min(chunk, N - o)), kind,
                           streams[k % nstreams])
        k += 1
    for s in streams[:nstreams]:
        hip.hipStreamSynchronize(s)
    return N / (time.perf_counter() - t) / 1e9


for ns, ch in ((1, N), (1, 256 << 20), (2, 256 << 20), (4, 256 << 20), (2, 2 << 30), (4, 1 << 30)):
    up = max(copy(d.data_ptr(), h.data_ptr(), 1, ns, ch) for _ in range(2))
    dn = max(copy(h2.data_ptr(), d.data_ptr(), 2, ns, ch) for _ in range(2))
    print(f"streams {ns} chunk {ch >> 20} MiB: H2D {up:.1f} GB/s, D2H {dn:.1f} GB/s", flush=True)
# both directions at once
t = time.perf_counter()
for o in range(0, N, 1 << 30):
    hip.hipMemcpyAsync(ctypes.c_void_p(d2.data_ptr() + o), ctypes.c_void_p(h.data_ptr() + o), ctypes.c_size_t(1 << 30), 1, streams[0])
    hip.hipMemcpyAsync(ctypes.c_void_p(h2.data_ptr() + o), ctypes.c_void_p(d.data_ptr() + o), ctypes.c_size_t(1 << 30), 2, streams[1])
hip.hipStreamSynchronize(streams[0])
hip.hipStreamSynchronize(streams[1])
print(f"both directions: {2 * N / (time.perf_counter() - t) / 1e9:.1f} GB/s total", flush=True)
