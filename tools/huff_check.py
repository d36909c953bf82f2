"""Debug (r04): GPU deflate of the c2_records case of test_deflate_header_equals_restated_builder with a
given library build; prints, for the first dynamic block, which symbols' lengths differ from the CPU
restatement of the Huffman builder."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent)); sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import numpy as np
from openge_amd import lib as L
if len(sys.argv) > 1:
    L.LIB_PATH = Path(sys.argv[1])
import deflate_parse as DP
import test_gpu_bgzf as T
ctx = L.Context(0)
data = T._bam_bytes(6000)
z = ctx.bgzf_deflate(data, 6)
bad = 0
for bi, (payload, body) in enumerate(T.split_blocks(z)):
    for b in DP.parse_block(body):
        if b["type"] != 2:
            continue
        lit, dist, cl = DP.header_lengths(b["lit_count"], b["dist_count"])
        if b["lit"] != lit or b["dist"] != dist or b["cl"] != cl:
            bad += 1
            if bad <= 2:
                dif = [(s, b["lit_count"][s], b["lit"][s], lit[s]) for s in range(min(len(lit), len(b["lit"]))) if b["lit"][s] != lit[s]]
                print("block", bi, "lit diffs (sym, count, gpu, cpu):", dif[:12], "dist eq", b["dist"] == dist, "cl eq", b["cl"] == cl)
print(sys.argv[1:] or ["default"], "blocks with differing headers:", bad)
