"""Experiment: does a device-to-host copy slow the GPU deflate running beside it (the host pipeline's
segments take 31 ms instead of ~10 ms while their copies run)?  Deflate alone, copies alone, both at once
(profiling aid; run under rocprofv3 --kernel-trace to see whether the copies are kernels)."""
import ctypes
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from openge_amd import lib as L  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
ctx = L.Context(0)
p = L.synth_params(15_000_000, preset="c2", seed=3)
n = 2 * p.n_pairs
d_offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), None)
ctx.sync()
B = int(d_offs[-1].item())
src = torch.empty(B + 64, dtype=torch.uint8, device="cuda")
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), src.data_ptr())
ctx.sync()
bound = int(L.lib().oge_bgzf_bound(B))
dst = torch.empty(bound + 64, dtype=torch.uint8, device="cuda")
H = 16 << 30
h = torch.empty(H, dtype=torch.uint8, pin_memory=True)
dsrc = torch.empty(H, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
S = ctypes.c_void_p()
hip.hipStreamCreateWithFlags(ctypes.byref(S), 1)


def deflate():
    t = time.perf_counter()
    z = ctx.bgzf_deflate_dev(src.data_ptr(), B, 6, dst.data_ptr(), bound)
    return time.perf_counter() - t, z


def copies():
    for o in range(0, H, 1400 << 20):
        hip.hipMemcpyAsync(ctypes.c_void_p(h.data_ptr() + o), ctypes.c_void_p(dsrc.data_ptr() + o),
                           ctypes.c_size_t(min(1400 << 20, H - o)), 2, S)


deflate()
td, z = deflate()
print(f"deflate alone: {B / 1e9:.2f} GB in {td * 1e3:.1f} ms", flush=True)
t = time.perf_counter()
copies()
hip.hipStreamSynchronize(S)
tc = time.perf_counter() - t
print(f"D2H alone: {H / 1e9:.1f} GB in {tc * 1e3:.1f} ms = {H / tc / 1e9:.1f} GB/s", flush=True)
t = time.perf_counter()
copies()
td2, _ = deflate()
hip.hipStreamSynchronize(S)
tb = time.perf_counter() - t
print(f"both: deflate {td2 * 1e3:.1f} ms, all done {tb * 1e3:.1f} ms", flush=True)
