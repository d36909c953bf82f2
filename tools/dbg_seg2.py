"""TEMP: deflate the 20M C2 stream once per round, inflate it repeatedly with both implementations,
count failures (separates a deflate fault from an inflate race)."""
import ctypes as C, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np, torch
from openge_amd import lib as L
reads = int(sys.argv[1]); rounds = int(sys.argv[2]); reps = int(sys.argv[3]); impls = [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else '0,1').split(',')]
concurrent = len(sys.argv) > 5 and sys.argv[5] == 'conc'
dev = torch.device("cuda", 0)
ctx = L.Context(0)
p = L.synth_params(reads // 2, preset="c2", seed=1234)
n = 2 * (reads // 2)
d_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), None); ctx.sync()
B = int(d_offs[-1].item())
d_recs = torch.empty(B + 64, dtype=torch.uint8, device=dev)
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), d_recs.data_ptr()); ctx.sync()
cap = int(L.lib().oge_bgzf_bound(B))
d_z = torch.empty(cap, dtype=torch.uint8, device=dev)
d_back = torch.zeros(B + 64, dtype=torch.uint8, device=dev)
ref = None
for rnd in range(rounds):
    zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, 6, d_z.data_ptr(), cap)
    zs = d_z[:zb].clone()
    same = ref is None or (ref.numel() == zs.numel() and torch.equal(ref, zs))
    if ref is None: ref = zs
    zh = d_z[:zb].cpu().numpy()
    nb = C.c_uint64()
    L.lib().oge_bgzf_index(zh.ctypes.data, zb, None, None, None, None, 0, C.byref(nb))
    k = nb.value
    idx = np.zeros(3 * k + 1, dtype=np.uint64); crc = np.zeros(k, dtype=np.uint32)
    i0 = idx.ctypes.data
    L.check(L.lib().oge_bgzf_index(zh.ctypes.data, zb, i0, i0 + 8 * k, i0 + 16 * k, crc.ctypes.data, k, C.byref(nb)))
    d_idx = torch.from_numpy(idx.view(np.int64)).to(dev); d_crc = torch.from_numpy(crc.view(np.int32)).to(dev)
    res = {}
    for impl in impls:
        ctx.set_inflate(impl)
        fails = []
        for _ in range(reps):
            if concurrent:
                d_back.zero_()  # on torch's stream, NOT ordered with the inflate (a concurrent kernel)
            p0 = d_idx.data_ptr()
            rc = L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k, d_back.data_ptr())
            if rc:
                fails.append(L.lib().oge_last_error(ctx.h).decode())
            elif not concurrent and not torch.equal(d_back[:B], d_recs[:B]):
                fails.append("bytes differ without error")
        res[impl] = fails
    print(f"round {rnd}: deflate same as round 0: {same}; fails {[(i, len(res[i]), res[i][:2]) for i in impls]}", flush=True)
