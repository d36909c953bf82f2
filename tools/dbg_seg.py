"""TEMP: dump block N of the 20M codec stream (compressed bytes, GPU per-thread pass state, both outputs)."""
import ctypes as C, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np, torch
from openge_amd import lib as L
blk = int(sys.argv[1]); reads = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
out = Path("gpurun_out/dbg"); out.mkdir(parents=True, exist_ok=True)
os.environ["OGE_INFL_DEBUG_OUT"] = str(out / "state.bin")
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
d0, d1, uo = idx[:k], idx[k:2 * k], idx[2 * k:]
np.save(out / "zblock.npy", zh[int(d0[blk]):int(d1[blk])])
payload = d_recs[int(uo[blk]):int(uo[blk + 1])].cpu().numpy()
np.save(out / "payload.npy", payload)
d_idx = torch.from_numpy(idx.view(np.int64)).to(dev); d_crc = torch.from_numpy(crc.view(np.int32)).to(dev)
d_back = torch.zeros(B + 64, dtype=torch.uint8, device=dev)
os.environ["OGE_INFL_DEBUG_BLOCK"] = str(blk)
p0 = d_idx.data_ptr()
rc = L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k, d_back.data_ptr())
print("rc", rc, L.lib().oge_last_error(ctx.h))
got = d_back[int(uo[blk]):int(uo[blk + 1])].cpu().numpy()
np.save(out / "got.npy", got)
bad = np.nonzero(got != payload)[0]
print("diff bytes", len(bad), bad[:20])
