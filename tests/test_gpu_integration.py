"""GPU: the reference's own module chain (FileReader -> sorter -> marker -> BamSerializer sink,
cmd/command_mergesort.cpp:68-117) with the INTEGRATION.md GPU modules in place of ReadSorter and
MarkDuplicates (oracle/_ref/integration/gpu_chain, linked in the build container by
tests/test_integration.py) gives the reference's `mergesort -M` output on the golden cases."""
from pathlib import Path
import subprocess

import pytest

from goldens import load_case
from test_gpu_cli import _refs, case_input, digests

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


REF_DRIVER = Path(__file__).resolve().parent.parent / "oracle" / "_ref" / "ref_driver"


@pytest.mark.skipif(not (EXE.exists() and REF_DRIVER.exists()), reason="reference-built binaries come from the build container")
def test_reference_chain_remove_dups_drops_preflagged_secondaries(tmp_path, built):
    """-R drops every record whose FLAG carries 0x400 after the apply step (alg/mark_duplicates.cpp:456),
    including non-primary records that arrive with 0x400 already set (their bit is never touched).
    The expected output is the reference's own sortdedup -v chain with removeDuplicates (ref_driver -D)
    run on the same input here."""
    import struct
    import bamutil
    case = load_case("mix3k")
    recs = case.recs.copy()
    n_sec = 0
    for k, o in enumerate(case.offs[:-1]):
        if k % 37 == 5:  # primary -> secondary with the duplicate bit already set
            (fl,) = struct.unpack_from("<H", recs, int(o) + 18)
            struct.pack_into("<H", recs, int(o) + 18, fl | 0x100 | 0x400)
            n_sec += 1
    src = tmp_path / "in.bam"
    bamutil.write_bam_py(src, case.header, _refs(case.header),
                         [bamutil.rec_bytes(recs, o) for o in case.offs[:-1]])
    r = subprocess.run([str(EXE), str(src), str(tmp_path / "o.bam"), "-R"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rr = subprocess.run([str(REF_DRIVER), "sortdedup", "-v", "-D", "-t", "4", "-T", str(tmp_path), str(src),
                         str(tmp_path / "ref.bam")], capture_output=True, text=True, timeout=300)
    assert rr.returncode == 0, rr.stderr
    got, want = digests(tmp_path / "o.bam"), digests(tmp_path / "ref.bam")
    assert got == want
    # the pre-flagged secondaries are gone from both
    _, _, orecs, ooffs = bamutil.read_bam(tmp_path / "o.bam")
    assert len(ooffs) < case.n - n_sec
    assert not any(struct.unpack_from("<H", orecs, int(o) + 18)[0] & 0x400 for o in ooffs)


@pytest.mark.skipif(not EXE.exists(), reason="oracle/_ref/integration/gpu_chain is built in the build container")
@pytest.mark.parametrize("name", ["rl_small", "rl_edge", "rl_qual", "rl_c5_2k"])
def test_reference_chain_with_gpu_localrealign(name, tmp_path, built):
    """`openge localrealign` as cmd/command_localrealign.cpp:37-75 wires it -- the reference's FileReader
    -> GpuLocalRealignment (the INTEGRATION.md drop-in for LocalRealignment, alg/local_realignment.h:
    67-527, with its setReferenceFilename / setIntervalsFilename) -> the reference's BamSerializer --
    writes exactly the REFERENCE's own realigned records (tests/golden/rl_*)."""
    import bamutil
    import realign_util as R
    from test_realign import load_rl_case
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    src = tmp_path / "reads.bam"
    out = tmp_path / "realigned.bam"
    r = subprocess.run([str(EXE), "realign", str(fa), str(iv), str(src), str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _, _, orecs, ooffs = bamutil.read_bam(out)
    assert len(ooffs) == meta["n_out"]
    assert R.digest(orecs, ooffs)["stream_sha256"] == meta["stream_sha256"]
