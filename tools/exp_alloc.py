"""Experiment: where the first (cold) e2e step's extra seconds go -- hipMalloc of fresh HBM vs the first
touch of it vs later touches (profiling aid, not a test)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
torch.cuda.init()
torch.zeros(1, device=dev)
torch.cuda.synchronize()
for gb in (8, 40, 80):
    n = gb << 30
    p = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n))
    t1 = time.perf_counter()
    hip.hipMemsetAsync(p, ctypes.c_int(1), ctypes.c_size_t(n), None)
    hip.hipDeviceSynchronize()
    t2 = time.perf_counter()
    hip.hipMemsetAsync(p, ctypes.c_int(2), ctypes.c_size_t(n), None)
    hip.hipDeviceSynchronize()
    t3 = time.perf_counter()
    hip.hipFree(p)
    t4 = time.perf_counter()
    # stream-ordered pool: allocate, free, allocate again
    s = ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(s))
    q = ctypes.c_void_p()
    t5 = time.perf_counter()
    hip.hipMallocAsync(ctypes.byref(q), ctypes.c_size_t(n), s)
    hip.hipMemsetAsync(q, ctypes.c_int(1), ctypes.c_size_t(n), s)
    hip.hipStreamSynchronize(s)
    t6 = time.perf_counter()
    hip.hipFreeAsync(q, s)
    hip.hipStreamSynchronize(s)
    hip.hipMallocAsync(ctypes.byref(q), ctypes.c_size_t(n), s)
    hip.hipMemsetAsync(q, ctypes.c_int(1), ctypes.c_size_t(n), s)
    hip.hipStreamSynchronize(s)
    t7 = time.perf_counter()
    hip.hipFreeAsync(q, s)
    hip.hipStreamSynchronize(s)
    print(f"{gb} GB: hipMalloc {t1 - t0:.3f} s, first memset {t2 - t1:.3f} s, second memset {t3 - t2:.3f} s, "
          f"hipFree {t4 - t3:.3f} s; pool malloc+memset {t6 - t5:.3f} s, again after free {t7 - t6:.3f} s", flush=True)
