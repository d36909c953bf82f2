"""Debug aid: symbol trace of the lane inflate's block 0 on a zlib level-6 stream of 2-bit ACGT data."""
import os, struct, sys, zlib
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from openge_amd import lib as L
rng = np.random.default_rng(1)
data = bytes(rng.integers(0, 4, 300_000, dtype=np.uint8) + ord("A"))[:65280]
c = zlib.compressobj(6, zlib.DEFLATED, -15)
body = c.compress(data) + c.flush()
z = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", 18 + len(body) + 7) + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))
os.makedirs("gpurun_out/dbg", exist_ok=True)
open("gpurun_out/dbg/block.bin", "wb").write(body)
ctx = L.Context(0)
try:
    out = ctx.bgzf_inflate(z)
    print("ok", out == data)
except Exception as e:
    print("err", e)
