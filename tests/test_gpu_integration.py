"""GPU: the reference's own module chain (FileReader -> sorter -> marker -> BamSerializer sink,
cmd/command_mergesort.cpp:68-117) with the INTEGRATION.md GPU modules in place of ReadSorter and
MarkDuplicates (oracle/_ref/integration/gpu_chain, linked in the build container by
tests/test_integration.py) gives the reference's `mergesort -M` output on the golden cases."""
from pathlib import Path
import subprocess

import pytest

from goldens import load_case
from test_gpu_cli import case_input, digests

pytestmark = pytest.mark.gpu
EXE = Path(__file__).resolve().parent.parent / "oracle" / "_ref" / "integration" / "gpu_chain"


@pytest.mark.skipif(not EXE.exists(), reason="oracle/_ref/integration/gpu_chain is built in the build container")
@pytest.mark.parametrize("name", ["simple", "yhet208", "mix3k", "c2_20k"])
def test_reference_chain_with_gpu_modules(name, tmp_path, built):
    case = load_case(name)
    src = case_input(case, tmp_path)
    r = subprocess.run([str(EXE), str(src), str(tmp_path / "o.bam")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    assert f"Marked {g['n_dup']} records" in r.stderr
