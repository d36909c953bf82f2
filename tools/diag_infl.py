"""Diagnostic: inflate stage time of the 20M codec stream (DIAG_READS overrides the read count) with an
alternative library build (argv[1] = .so path; errors are reported, not raised: diagnostic builds may drop
work); the last run's output is compared with the records."""
import ctypes as C, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np, torch
from openge_amd import lib as L
if len(sys.argv) > 1:
    L.LIB_PATH = Path(sys.argv[1])
reads = int(os.environ.get("DIAG_READS", 20_000_000))
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
zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, 6, d_z.data_ptr(), cap)
zh = d_z[:zb].cpu().numpy()
nb = C.c_uint64()
L.lib().oge_bgzf_index(zh.ctypes.data, zb, None, None, None, None, 0, C.byref(nb))
k = nb.value
idx = np.zeros(3 * k + 1, dtype=np.uint64); crc = np.zeros(k, dtype=np.uint32)
i0 = idx.ctypes.data
L.check(L.lib().oge_bgzf_index(zh.ctypes.data, zb, i0, i0 + 8 * k, i0 + 16 * k, crc.ctypes.data, k, C.byref(nb)))
d_idx = torch.from_numpy(idx.view(np.int64)).to(dev); d_crc = torch.from_numpy(crc.view(np.int32)).to(dev)
d_back = torch.zeros(B + 64, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
ab = os.environ.get("DIAG_AB")  # NAME: alternate NAME=0 / NAME=1 call by call in this process (A/B on one box)
if ab:
    res = {"0": [], "1": []}
    stg = {"0": [], "1": []}
    for it in range(12):
        v = "01"[it % 2]
        os.environ[ab] = v
        p0 = d_idx.data_ptr()
        rc = L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k, d_back.data_ptr())
        if it >= 2:
            res[v].append(round(ctx.timing("bgzf_inflate"), 2))
            stg[v].append({x: round(ctx.timing(x), 2) for x in ("infl_prep", "infl_huff", "infl_lz")})
    same = bool(torch.equal(d_back[:B], d_recs[:B]))
    for v in "01":
        print(f"{ab}={v} reads {reads} blocks {k} inflate ms {res[v]} median {sorted(res[v])[len(res[v]) // 2]} stages {stg[v][-1]}", flush=True)
    print("rc", rc, "same", same, flush=True)
    sys.exit(0)
ms = []
for _ in range(4):
    p0 = d_idx.data_ptr()
    rc = L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k, d_back.data_ptr())
    ms.append(round(ctx.timing("bgzf_inflate"), 2))
    st = {k: round(ctx.timing(k), 2) for k in ("infl_prep", "infl_huff", "infl_lz")}
same = bool(torch.equal(d_back[:B], d_recs[:B]))
print(sys.argv[1:] or ["default"], "reads", reads, "blocks", k, "inflate ms", ms[1:], "rc", rc, "same", same, "stages", st, flush=True)
