"""Experiment: why the host pipeline's output copies run at ~45 GB/s (57 GB/s in tools/exp_pcie.py):
a 57 GB page-locked destination vs a 16 GB one, copies of 1.4 GB pieces, with and without kernels
running beside them, and the page-locked buffer placed on the GPU's NUMA node (profiling aid)."""
import ctypes
import os
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
bus = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(bus, 64, 0)
bdf = bus.value.decode().lower()
node = None
try:
    node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
except OSError:
    pass
print(f"GPU {bdf} numa node {node}; process cpus {len(os.sched_getaffinity(0))}", flush=True)
S = ctypes.c_void_p()
hip.hipStreamCreateWithFlags(ctypes.byref(S), 1)
PIECE = 1400 << 20
d = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
d.fill_(7)
torch.cuda.synchronize()


def d2h(hptr, total, busy=False):
    x = torch.empty(4 << 30, dtype=torch.uint8, device="cuda") if busy else None
    t = time.perf_counter()
    o = 0
    while o < total:
        n = min(PIECE, total - o)
        hip.hipMemcpyAsync(ctypes.c_void_p(hptr + o), ctypes.c_void_p(d.data_ptr() + (o % (15 << 30))), ctypes.c_size_t(n), 2, S)
        if busy:
            for _ in range(4):
                x.add_(1)  # kernels on torch's stream beside the copies
        o += n
    hip.hipStreamSynchronize(S)
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return total / dt / 1e9


big = torch.empty(57 << 30, dtype=torch.uint8, pin_memory=True)
small = torch.empty(16 << 30, dtype=torch.uint8, pin_memory=True)
print(f"D2H into 16 GB pinned: {d2h(small.data_ptr(), 16 << 30):.1f} GB/s", flush=True)
print(f"D2H into 57 GB pinned (first 16 GB): {d2h(big.data_ptr(), 16 << 30):.1f} GB/s", flush=True)
print(f"D2H into 57 GB pinned (all): {d2h(big.data_ptr(), 56 << 30):.1f} GB/s", flush=True)
print(f"D2H into 57 GB pinned, kernels beside: {d2h(big.data_ptr(), 56 << 30, busy=True):.1f} GB/s", flush=True)
del big, small
if node is not None and node >= 0:
    rng = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    cs = set()
    for part in rng.split(","):
        a, _, b = part.partition("-")
        cs.update(range(int(a), int(b or a) + 1))
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, cs & old or cs)
    loc = torch.empty(57 << 30, dtype=torch.uint8, pin_memory=True)
    os.sched_setaffinity(0, old)
    print(f"D2H into 57 GB pinned on node {node}: {d2h(loc.data_ptr(), 56 << 30):.1f} GB/s", flush=True)
    print(f"D2H into 57 GB pinned on node {node}, kernels beside: {d2h(loc.data_ptr(), 56 << 30, busy=True):.1f} GB/s", flush=True)
