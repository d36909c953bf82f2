"""Diagnostic: GPU deflate stage time of the 20M-read C2 stream (the codec bench size) with the default
library or an alternative build (argv[1]); prints the stage times of 3 runs after a warm-up, the
compressed size and the sha256 of the output (same bytes = same sha)."""
import hashlib
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch
from openge_amd import lib as L
if len(sys.argv) > 1:
    L.LIB_PATH = Path(sys.argv[1])
import os
reads = int(os.environ.get("DIAG_READS", 20_000_000))
level = int(os.environ.get("DIAG_LEVEL", 6))
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
ms = []
for _ in range(4):
    zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, level, d_z.data_ptr(), cap)
    ms.append(round(ctx.timing("bgzf_deflate"), 2))
sha = hashlib.sha256(d_z[:zb].cpu().numpy().tobytes()).hexdigest()[:16]
print(sys.argv[1:] or ["default"], "level", level, "deflate ms", ms[1:], "bytes", zb, "ratio", round(zb / B, 4), "sha", sha, flush=True)
if os.environ.get("DIAG_ZLIB"):  # zlib level 6 per 65,280-byte payload over the first 32 MiB, for comparison
    import zlib
    h = d_recs[: 65280 * 514].cpu().numpy().tobytes()
    g = bytes(d_z[: 0].cpu().numpy())
    zs = sum(len(zlib.compress(h[i:i + 65280], 6)) - 6 + 26 for i in range(0, len(h), 65280))
    print("zlib-6 sample ratio", round(zs / len(h), 4), flush=True)
