"""Print the golden of tests/test_gpu_bgzf.py::test_deflate_bytes_pinned (run on the GPU box): the GPU deflate
of the C2 generator's 20,000 pairs (seed 99) at level 6."""
import hashlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from openge_amd import lib as L  # noqa: E402

ctx = L.Context(0)
p = L.synth_params(20_000, preset="c2", seed=99)
recs, offs, _ = L.synth_host(p)
data = recs[:int(offs[-1])].tobytes()
z = ctx.bgzf_deflate(data, 6)
print(json.dumps({"what": "GPU deflate (oge_bgzf_deflate, level 6) of synth_params(20000, c2, seed 99) records",
                  "input_bytes": len(data), "output_bytes": len(z), "sha256": hashlib.sha256(z).hexdigest()}))
ctx.close()
