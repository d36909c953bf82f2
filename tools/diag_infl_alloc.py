"""Diagnostic: the inflate stage with every buffer it touches (compressed file, output, the library's
own workspaces) allocated by the library, so OGE_ALLOC_CONTIG=1 (hipExtMallocWithFlags with
hipDeviceMallocContiguous) vs 0 (hipMalloc) tests whether phase 1's per-process spread (97-106 ms at
100M reads on one box, profiles/r06cq-cy) follows the buffers' page fragments.  DIAG_READS as diag_infl.py."""
import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from openge_amd import lib as L  # noqa: E402

if len(sys.argv) > 1:  # an experiment build (tools/build_variant.py)
    L.LIB_PATH = Path(sys.argv[1])

reads = int(os.environ.get("DIAG_READS", 100_000_000))
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


def dalloc(nbytes: int) -> int:
    ptr = C.c_void_p()
    L.check(L.lib().oge_dev_alloc(ctx.h, nbytes, C.byref(ptr)), ctx.h)
    return ptr.value


cap = int(L.lib().oge_bgzf_bound(B))
z = dalloc(cap)
out = dalloc(B + 64)
zb = ctx.bgzf_deflate_dev(d_recs.data_ptr(), B, 6, z, cap)
nb = ctx.bgzf_index_dev(z, zb)
idx = torch.empty(3 * nb + 1, dtype=torch.int64, device=dev)
d_crc = torch.empty(nb, dtype=torch.int32, device=dev)
p0 = idx.data_ptr()
ctx.bgzf_index_dev(z, zb, p0, p0 + 8 * nb, p0 + 16 * nb, d_crc.data_ptr(), nb)
ctx.sync()
st = []
for _ in range(4):
    L.check(L.lib().oge_bgzf_inflate_dev(ctx.h, z, zb, p0, p0 + 8 * nb, p0 + 16 * nb, d_crc.data_ptr(), nb, out), ctx.h)
    st.append({k: round(ctx.timing(k), 2) for k in ("bgzf_inflate", "infl_huff", "infl_lz")})
ctx.sync()
back = torch.empty(B, dtype=torch.uint8, device=dev)
L.check(L.lib().oge_memcpy(ctx.h, back.data_ptr(), out, B, 3), ctx.h)
ctx.sync()
same = bool(torch.equal(back, d_recs[:B]))
print(f"{Path(sys.argv[1]).stem if len(sys.argv) > 1 else 'default'} contig={os.environ.get('OGE_ALLOC_CONTIG', '0')} reads {reads} blocks {nb} same {same} runs {st[1:]}", flush=True)
