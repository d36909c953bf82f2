"""Device BGZF compression throughput on C2-shaped records already resident in HBM.

    python tools/bgzf_bench.py [reads=20000000] [reps=3]

Prints one JSON line: payload GB/s (HIP-event time of the `bgzf_deflate` stage), compressed ratio,
the inflate of the same stream back (lane decoder), and the ratio of host zlib level 6 on a 64 MB sample of the same bytes for comparison."""
import json
import sys
import time
import zlib
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from openge_amd import lib as L  # noqa: E402


def main():
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    ctx = L.Context(0)
    p = L.synth_params(reads // 2, preset="c2", seed=1234)
    n = 2 * (reads // 2)
    d_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), None)
    ctx.sync()
    B = int(d_offs[-1].item())
    d_recs = torch.empty(B + 64, dtype=torch.uint8, device=dev)
    ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), d_recs.data_ptr())
    ctx.sync()
    cap = int(L.lib().oge_bgzf_bound(B))
    d_z = torch.empty(cap, dtype=torch.uint8, device=dev)
    ms, wall = [], []
    zb = 0
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, 6, d_z.data_ptr(), cap)
        wall.append(time.perf_counter() - t0)
        ms.append(ctx.timing("bgzf_deflate"))
    ms, wall = ms[1:], wall[1:]
    # inflate the same stream back on the device (index on the host, as the reader does)
    import ctypes as C
    zh = d_z[:zb].cpu().numpy()
    nb = C.c_uint64()
    L.lib().oge_bgzf_index(zh.ctypes.data, zb, None, None, None, None, 0, C.byref(nb))
    idx = np.zeros(3 * nb.value + 1, dtype=np.uint64)
    crc = np.zeros(nb.value, dtype=np.uint32)
    i0 = idx.ctypes.data
    L.check(L.lib().oge_bgzf_index(zh.ctypes.data, zb, i0, i0 + 8 * nb.value, i0 + 16 * nb.value, crc.ctypes.data,
                                   nb.value, C.byref(nb)))
    d_idx = torch.from_numpy(idx.view(np.int64)).to(dev)
    d_crc = torch.from_numpy(crc.view(np.int32)).to(dev)
    d_back = torch.empty(B + 64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    k = nb.value
    inf_ms = []
    d_back.zero_()
    torch.cuda.synchronize()  # (the zeroing runs on torch's stream, the inflate on the context's)
    for _ in range(reps + 1):
        p0 = d_idx.data_ptr()
        L.check(L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k,
                                             d_back.data_ptr()), ctx.h)
        inf_ms.append(ctx.timing("bgzf_inflate"))  # CRC fused into inflate phase 2
    inf_ms = inf_ms[1:]
    assert torch.equal(d_back[:B], d_recs[:B])
    sample = d_recs[: min(B, 64 << 20)].cpu().numpy().tobytes()
    host = sum(len(zlib.compress(sample[i:i + 65280], 6)) + 26 for i in range(0, len(sample), 65280))
    print(json.dumps({
        "reads": n, "payload_bytes": B, "compressed_bytes": zb, "ratio": round(zb / B, 4),
        "zlib6_ratio_sample": round(host / len(sample), 4),
        "ms": [round(x, 2) for x in ms], "wall_s": [round(x, 3) for x in wall],
        "GBps": round(B / (min(ms) * 1e-3) / 1e9, 1),
        "inflate_ms": [round(x, 2) for x in inf_ms],
        "inflate_GBps": round(B / (min(inf_ms) * 1e-3) / 1e9, 1),
    }), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
