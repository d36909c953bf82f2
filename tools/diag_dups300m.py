"""Diagnostic (not a test): the 300M bench workload sorted + marked on the device, compared record by record
with tests/dupcheck.py's restated MarkDuplicates; for the records whose 0x400 differs prints the restated pair
(partner, chunk key, chunk members and scores) and the product's marks of every member."""
import ctypes as C
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from openge_amd import lib as L  # noqa: E402
import dupcheck  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 150_000_000
ctx = L.Context(0)
p = L.synth_params(pairs, preset="c2", seed=1234)
n = 2 * pairs
d_offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), None)
ctx.sync()
B = int(d_offs[-1].item())
d_recs = torch.empty(B + 64, dtype=torch.uint8, device="cuda")
ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), d_recs.data_ptr())
buf = C.create_string_buffer(1 << 16)
L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
hdr_text = buf.value.decode()
opts, keep = L.markdup_opts_from_header(hdr_text, p.n_ref)
d_out = torch.empty(B + 64, dtype=torch.uint8, device="cuda")
d_out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(), d_out_off.data_ptr())
ctx.sync()
del d_recs, d_offs
torch.cuda.empty_cache()
off = d_out_off[:n]
flag = d_out[off + 18].to(torch.int64) | (d_out[off + 19].to(torch.int64) << 8)
got = ((flag >> 10) & 1).bool()
dbg = {}
t0 = time.time()
primary, want = dupcheck.expected_dups(d_out, off, hdr_text, debug=dbg)
print(f"restated in {time.time() - t0:.1f} s; product {nd} dups, restated {int(want.sum())}", flush=True)
bad = torch.nonzero(want != got).squeeze(1)
print(f"{bad.numel()} mismatches; product-only {int((got & ~want).sum())}, restated-only {int((want & ~got).sum())}", flush=True)
r1, r2, k1, k2, psc, gid = (dbg[k] for k in ("pr1", "pr2", "pk1", "pk2", "psc", "pgid"))
ref = dupcheck._i32(d_out, off + 4)
pos = dupcheck._i32(d_out, off + 8)
lname = d_out[off + 12].to(torch.int64)


def name_of(i):
    o = int(off[i].item())
    return bytes(d_out[o + 36:o + 36 + int(lname[i].item()) - 1].cpu().numpy()).decode()


def desc(i):
    return (f"#{i} {name_of(i)} ref {int(ref[i])} pos {int(pos[i])} flag {hex(int(flag[i]))} coord {int(dbg['coord'][i])} "
            f"score {int(dbg['score'][i])} lib {int(dbg['lib'][i])} got {int(got[i])} want {int(want[i])}")


# which pair (restated) each mismatched record is in
pair_of = torch.full((n,), -1, dtype=torch.int64, device="cuda")
ar = torch.arange(r1.numel(), device="cuda")
pair_of[r1] = ar
pair_of[r2] = ar
nopair = 0
for i in bad[:12].tolist():
    print("----", desc(i), flush=True)
    q = int(pair_of[i])
    if q < 0:
        nopair += 1
        print("   restated: in no pair", flush=True)
        continue
    g = int(gid[q])
    mem = torch.nonzero(gid == g).squeeze(1)
    print(f"   restated pair chunk {g}: k1 {hex(int(k1[q]))} k2 {hex(int(k2[q]))}, {mem.numel()} pairs", flush=True)
    for m in mem[:8].tolist():
        print(f"     pair score {int(psc[m])}: r1 {desc(int(r1[m]))}\n                       r2 {desc(int(r2[m]))}", flush=True)
print("mismatches in no restated pair:", int((pair_of[bad] < 0).sum()), flush=True)
ctx.close()
