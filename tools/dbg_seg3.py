"""TEMP: phase clocks of a few blocks of the 20M codec stream (segment inflate)."""
import ctypes as C, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np, torch
from openge_amd import lib as L
reads = int(sys.argv[1]); blocks = [int(x) for x in sys.argv[2].split(',')]
out = Path("gpurun_out/dbg"); out.mkdir(parents=True, exist_ok=True)
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
names = ["start", "hdr0", "hdr1", "built", "passA", "passB", "scan", "passD", "LZ", "image", "crc", "write"]
for blk in blocks:
    f = out / f"state_{blk}.bin"
    os.environ["OGE_INFL_DEBUG_OUT"] = str(f)
    os.environ["OGE_INFL_DEBUG_BLOCK"] = str(blk)
    p0 = d_idx.data_ptr()
    L.check(L.lib().oge_bgzf_inflate_dev(ctx.h, d_z.data_ptr(), zb, p0, p0 + 8 * k, p0 + 16 * k, d_crc.data_ptr(), k, d_back.data_ptr()), ctx.h)
    st = np.fromfile(f, dtype=np.uint32)
    kT = len(st) // 17
    T = st[16 * kT:]
    marks = [int(T[i]) for i in (0, 1, 2, 3, 4, 5, 6, 11, 7, 8, 9, 10, 12)]
    D = st[:16 * kT].reshape(kT, 16)
    d = np.diff(np.array(marks, dtype=np.int64) & 0xffffffff) % (1 << 32)
    labs = ["pre", "hdr", "build", "passA", "passB", "scan", "dbgdump", "passD+", "LZ", "image", "crc", "write"]
    rounds_b, rounds_lz = int(T[20]), int(T[21])
    nseg, seg = int(D[0, 12]), int(D[0, 13])
    resync = int(((D[:, 5] != D[:, 0]) & (D[:, 14] == 1)).sum())
    print(blk, dict(zip(labs, d.tolist())), "total", int(sum(d)), "passB rounds", rounds_b, "LZ rounds", rounds_lz, "nseg", nseg, "seg", seg, "reverified", resync, flush=True)
