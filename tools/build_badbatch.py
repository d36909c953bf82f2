"""One-off (r03): build openge_amd/_exp/libopenge_hip_badbatch.so, the library with the r02 commit 3941758
literal-batch rule put back into a copy of inflate_lane.hip (the batch follows every literal, long codes
included: 15 + 3 x 6 bits can exceed the 32 a refill guarantees).  tools/exp_infl_guard.py then checks that the crafted streams of
tests/deflate_craft.py make that build fail.  Uses the objects of the normal build for everything else."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from openge_amd import build as B  # noqa: E402

B.build()
exp = ROOT / "openge_amd" / "_exp"
exp.mkdir(exist_ok=True)
src = (B.CSRC / "inflate_lane.hip").read_text()
good = "if (e) {  // more direct-table literals"
assert src.count(good) == 1, "batch condition not found"
(exp / "inflate_lane_bad.hip").write_text(src.replace(good, "if (true) {  // r02 3941758: after a long code too"))
obj = exp / "inflate_lane_bad.o"
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-x", "hip", *B.COMMON, f"-I{B.CSRC}", "-c",
                str(exp / "inflate_lane_bad.hip"), "-o", str(obj)], check=True)
objs = [str(B.BUILD / (s + ".o")) for s in B.HIP_SRCS if s != "inflate_lane.hip"]
objs += [str(B.BUILD / (s + ".o")) for s in B.HOST_SRCS]
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-o", str(exp / "libopenge_hip_badbatch.so"), str(obj),
                *objs, "-L/opt/rocm/lib", "-lrccl", "-lz", "-lpthread", "-ldl"], check=True)
print("built", exp / "libopenge_hip_badbatch.so")
