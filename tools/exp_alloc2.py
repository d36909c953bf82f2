"""Experiment: is re-acquiring HBM that this process just returned to the driver the slow part of the
first e2e step (the bench frees its 172 GB of setup buffers, then the chain's workspace takes them)?
Fresh hipMalloc vs hipMalloc after a hipFree of the same bytes vs a stream-ordered pool that keeps
freed memory (profiling aid, not a test)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
GB = 1 << 30


def malloc(n):
    p = ctypes.c_void_p()
    t = time.perf_counter()
    rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n))
    assert rc == 0, rc
    return p, time.perf_counter() - t


def touch(p, n, s=None):
    hip.hipMemsetAsync(p, ctypes.c_int(1), ctypes.c_size_t(n), s)
    hip.hipDeviceSynchronize()


# 1. fresh: two 85 GB buffers
a, ta = malloc(85 * GB)
b, tb = malloc(85 * GB)
touch(a, 85 * GB), touch(b, 85 * GB)
print(f"fresh hipMalloc 85 GB x2: {ta:.3f} s, {tb:.3f} s", flush=True)
t = time.perf_counter()
hip.hipFree(a), hip.hipFree(b)
print(f"hipFree x2: {time.perf_counter() - t:.3f} s", flush=True)
# 2. the same bytes again right after the free
a, ta = malloc(85 * GB)
t = time.perf_counter()
touch(a, 85 * GB)
print(f"re-acquired hipMalloc 85 GB: {ta:.3f} s (+ touch {time.perf_counter() - t:.3f} s)", flush=True)
time.sleep(3.0)
b, tb = malloc(85 * GB)
print(f"re-acquired hipMalloc 85 GB after 3 s idle: {tb:.3f} s", flush=True)
hip.hipFree(a), hip.hipFree(b)
# 3. stream-ordered pool, release threshold unlimited: freed bytes stay in the process
s = ctypes.c_void_p()
hip.hipStreamCreate(ctypes.byref(s))
pool = ctypes.c_void_p()
hip.hipDeviceGetDefaultMemPool(ctypes.byref(pool), 0)
thr = ctypes.c_uint64(2**64 - 1)
hip.hipMemPoolSetAttribute(pool, 4, ctypes.byref(thr))  # hipMemPoolAttrReleaseThreshold
for k in range(3):
    q = [ctypes.c_void_p(), ctypes.c_void_p()]
    t = time.perf_counter()
    for x in q:
        assert hip.hipMallocAsync(ctypes.byref(x), ctypes.c_size_t(85 * GB), s) == 0
    hip.hipStreamSynchronize(s)
    t1 = time.perf_counter()
    for x in q:
        touch(x, 85 * GB, s)
    t2 = time.perf_counter()
    for x in q:
        hip.hipFreeAsync(x, s)
    hip.hipStreamSynchronize(s)
    print(f"pool pass {k}: 2 x 85 GB malloc {t1 - t:.3f} s, touch {t2 - t1:.3f} s", flush=True)
# 4. a torch allocation freed with empty_cache, then hipMalloc (the bench's order)
hip.hipMemPoolTrimTo(pool, ctypes.c_size_t(0))
x = torch.empty(85 * GB, dtype=torch.uint8, device="cuda")
x.fill_(3)
torch.cuda.synchronize()
del x
torch.cuda.empty_cache()
a, ta = malloc(85 * GB)
print(f"hipMalloc 85 GB after torch empty_cache of 85 GB: {ta:.3f} s", flush=True)
hip.hipFree(a)
