"""Probe: hipMalloc / hipFree cost for large buffers (device pipeline first-call overhead)."""
import ctypes as C
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from openge_amd import lib as L  # noqa: E402

ctx = L.Context(0)
lib = L.lib()
for gb in (1, 10, 40, 40):
    p = C.c_void_p()
    t = time.perf_counter()
    L.check(lib.oge_dev_alloc(ctx.h, gb << 30, C.byref(p)))
    ta = time.perf_counter() - t
    t = time.perf_counter()
    L.check(lib.oge_dev_free(ctx.h, p))
    tf = time.perf_counter() - t
    print(f"{gb:3d} GiB: alloc {ta * 1e3:8.1f} ms  free {tf * 1e3:8.1f} ms", flush=True)

# first touch vs second touch of a fresh allocation (torch for the memset; same HIP runtime)
import torch  # noqa: E402
for gb in (10, 40):
    p = C.c_void_p()
    L.check(lib.oge_dev_alloc(ctx.h, gb << 30, C.byref(p)))
    hip = C.CDLL("libamdhip64.so.7")
    for k in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        assert hip.hipMemset(p, 0, C.c_size_t(gb << 30)) == 0
        assert hip.hipDeviceSynchronize() == 0
        print(f"{gb:3d} GiB memset #{k}: {(time.perf_counter() - t) * 1e3:8.1f} ms", flush=True)
    L.check(lib.oge_dev_free(ctx.h, p))
