"""Experiment builds (not product): openge_amd/_var/lib_<name>.so = the normal library with ONE source file
recompiled with extra defines, e.g.

    python tools/build_variant.py nolonglit inflate_lane.hip -DOGE_EXP=1
    python tools/build_variant.py r03 inflate_lane.hip=openge_amd/_var/inflate_lane_r03.hip

tools/diag_infl.py <path to .so> then times the inflate stage with it.  The _var directory is git-ignored
and deleted when the experiment is recorded."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from openge_amd import build as B  # noqa: E402

name, src, *defs = sys.argv[1:]
# src: a file in openge_amd/csrc (recompiled with defs), or SRC=PATH:a replacement for that file
repl = None
if "=" in src:
    src, repl = src.split("=", 1)
B.build()
var = ROOT / "openge_amd" / "_var"
var.mkdir(exist_ok=True)
obj = var / f"{Path(src).stem}_{name}.o"
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-x", "hip", *B.COMMON, *defs, f"-I{B.CSRC}", "-c", repl or str(B.CSRC / src),
                "-o", str(obj)], check=True)
objs = [str(B.BUILD / (s + ".o")) for s in B.HIP_SRCS if s != src]
objs += [str(B.BUILD / (s + ".o")) for s in B.HOST_SRCS]
out = var / f"lib_{name}.so"
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-o", str(out), str(obj), *objs, "-L/opt/rocm/lib", "-lrccl",
                "-lz", "-lpthread", "-ldl"], check=True)
print("built", out)
