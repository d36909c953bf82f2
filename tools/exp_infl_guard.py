"""One-off check (r03): the crafted long/short-code streams (tests/deflate_craft.py) must break the
r02 3941758 literal-batch logic, built into openge_amd/_exp/libopenge_hip_badbatch.so from a patched
copy of inflate_lane.hip.  Prints whether the bad build fails (corruption or the E_BITS guard)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from openge_amd import lib as L  # noqa: E402

L.LIB_PATH = ROOT / "openge_amd" / "_exp" / "libopenge_hip_badbatch.so"
import deflate_craft as D  # noqa: E402

ctx = L.Context(0)
for seed in (7, 8):
    data, z = D.long_short_stream(130, seed=seed)
    try:
        out = ctx.bgzf_inflate(z)
        print(f"seed {seed}: bad build returned {'EQUAL' if out == data else 'DIFFERENT'} bytes", flush=True)
    except L.OgeError as e:
        print(f"seed {seed}: bad build failed loudly: {e}", flush=True)
ctx.close()
