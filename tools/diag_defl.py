"""Diagnostic: run the GPU deflate of a 2M-read C2 stream with an alternative library build (argv[1])."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from openge_amd import lib as L
if len(sys.argv) > 1:
    L.LIB_PATH = Path(sys.argv[1])
reads = 2_000_000
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
for _ in range(2):
    zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, 6, d_z.data_ptr(), cap)
    print("deflate ms", ctx.timing("bgzf_deflate"), "bytes", zb, flush=True)
