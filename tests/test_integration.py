"""CPU: the INTEGRATION.md modules (integration/gpu_modules.{h,cpp}: GpuReadSorter / GpuMarkDuplicates as
AlgorithmModule subclasses over the C ABI) compile against the reference's own headers in its own
C++98 dialect and link with its FileReader / AlgorithmModule / BamSerializer objects (built in place
by oracle/Makefile.ref) and libopenge_hip.so -- the drop-in claim for the reference side, checked
(VERDICT r01).  Running the linked chain needs a GPU: tests/test_gpu_integration.py."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference/openge/src")


@pytest.mark.skipif(not REF.exists(), reason="the reference tree exists only in the build container")
def test_gpu_modules_build_against_reference_headers(built):
    import oracle
    assert oracle.build_ref(), "reference objects (oracle/_ref) could not be built"
    r = subprocess.run(["make", "-f", str(ROOT / "integration" / "Makefile")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    exe = ROOT / "oracle" / "_ref" / "integration" / "gpu_chain"
    assert exe.exists()
    syms = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    for s in ("oge_ctx_create", "oge_sort_coord", "oge_markdup", "oge_localrealign", "oge_last_error"):
        assert s in syms
    # the reference's own modules are in the binary (not stand-ins)
    defined = subprocess.run(["nm", "-C", str(exe)], capture_output=True, text=True).stdout
    assert "FileReader::runInternal" in defined and "AlgorithmModule::runChain" in defined
