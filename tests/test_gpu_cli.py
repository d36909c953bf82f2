"""GPU: the `openge` command-line drop-in (openge_amd/openge) end to end, BAM in -> BAM out, against
the REFERENCE's own outputs (tests/golden; made by oracle/_ref from the reference's modules).  These
read like the reference's CTest smoke tests (openge/test/CMakeLists.txt:32,44-45) with the outputs
pinned byte for byte (decompressed records + header text; compressed bytes are not part of parity)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import bamutil
import realign_util as R
from goldens import CASE_NAMES, GOLDEN, load_case
from openge_amd import lib as L
from test_realign import RL_CASES, check_output, load_rl_case

pytestmark = pytest.mark.gpu
OPENGE = str(L.PKG / "openge")


def run(*args):
    r = subprocess.run([OPENGE, *map(str, args)], capture_output=True, text=True, timeout=300, env=dict(os.environ))
    assert r.returncode == 0, r.stderr
    return r


def case_input(case, tmp_path):
    if case.meta["spec"]["kind"] == "file":
        return GOLDEN / "inputs" / case.meta["spec"]["file"]
    path = tmp_path / "in.bam"
    bamutil.write_bam_py(path, case.header, _refs(case.header), [bamutil.rec_bytes(case.recs, o) for o in case.offs[:-1]])
    return path


def _refs(header):
    out = []
    for line in header.splitlines():
        if line.startswith("@SQ"):
            f = dict(x.split(":", 1) for x in line.split("\t")[1:])
            out.append((f["SN"], int(f["LN"])))
    return out


def digests(path):
    h, _, recs, offs = bamutil.read_bam(path)
    hm, tail = hashlib.sha256(), []
    for o in offs:
        rb = bamutil.rec_bytes(recs, o)
        (tail.append(rb) if int.from_bytes(rb[4:8], "little", signed=True) == -1 else hm.update(rb))
    return h, hm.hexdigest(), hashlib.sha256(b"".join(sorted(tail))).hexdigest()


@pytest.fixture(scope="module", params=CASE_NAMES)
def case(request, built):
    return load_case(request.param)


def test_cli_mergesort_M_matches_reference(case, tmp_path):
    src = case_input(case, tmp_path)
    run("mergesort", "-M", "--nopg", src, "-o", tmp_path / "o.bam")
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]


def test_cli_sort_alias_then_dedup_matches_reference(case, tmp_path):
    src = case_input(case, tmp_path)
    run("sort", "--nopg", src, "-o", tmp_path / "s.bam")
    h, m, t = digests(tmp_path / "s.bam")
    assert h == case.meta["sorted_header"] and m == case.meta["sort"]["mapped_sha256"]
    run("dedup", "--nopg", tmp_path / "s.bam", "-o", tmp_path / "d.bam")
    h, m, t = digests(tmp_path / "d.bam")
    g = case.meta["dedup_sorted_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]


def test_cli_split_chains_match_reference(case, tmp_path):
    """the reference's split-by-chromosome chains, explicitly (--split-chains K) and by
    the reference's own rule (--compat-split: K = min(12, -t / 2))."""
    src = case_input(case, tmp_path)
    run("mergesort", "-M", "--nopg", "--split-chains", 3, src, "-o", tmp_path / "m3.bam")
    h, m, t = digests(tmp_path / "m3.bam")
    g = case.meta["sortdedup_v_k3"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    run("sort", "--nopg", src, "-o", tmp_path / "s.bam")
    run("dedup", "--nopg", "--compat-split", "-t", 24, tmp_path / "s.bam", "-o", tmp_path / "d12.bam")
    h, m, t = digests(tmp_path / "d12.bam")
    g = case.meta["dedup_sorted_v_k12"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    run("dedup", "--nopg", "--compat-split", "--nosplit", "-t", 24, tmp_path / "s.bam", "-o", tmp_path / "dn.bam")
    h, m, t = digests(tmp_path / "dn.bam")
    assert m == case.meta["dedup_sorted_v"]["mapped_sha256"]


def test_cli_dedup_remove_drops_flagged_records(case, tmp_path):
    src = case_input(case, tmp_path)
    run("mergesort", "-R", "--nopg", src, "-o", tmp_path / "r.bam")
    _, _, recs, offs = bamutil.read_bam(tmp_path / "r.bam")
    assert len(offs) == case.n - case.meta["sortdedup_v"]["n_dup"]
    assert not (bamutil.flags_of(recs, offs) & 0x400).any()


def test_cli_program_record(tmp_path):
    src = tmp_path / "mix.bam"
    p = L.synth_params(200, preset="mix", seed=3)
    recs, offs, hdr = L.synth_host(p)
    L.write_bam(src, hdr, recs, offs, 400)
    run("mergesort", src, "-o", tmp_path / "p.bam", "-c", "1")
    h = bamutil.read_bam(tmp_path / "p.bam")[0]
    pg = [l for l in h.splitlines() if l.startswith("@PG")]
    # FileWriter::runInternal (algorithms/file_writer.cpp:76-89) + BamProgramRecord::toString
    assert pg == [f"@PG\tID:openge\tCL:openge mergesort {src} -o {tmp_path / 'p.bam'} -c 1 \tVN:0.3-dev"]
    run("mergesort", tmp_path / "p.bam", "-o", tmp_path / "p2.bam")
    ids = [l.split("\t")[1] for l in bamutil.read_bam(tmp_path / "p2.bam")[0].splitlines() if l.startswith("@PG")]
    assert ids == ["ID:openge", "ID:openge-2"]


@pytest.mark.parametrize("device_write", ["0", "1"])
@pytest.mark.parametrize("name", ["rl_small", "rl_edge"])
def test_cli_localrealign_matches_reference(name, device_write, tmp_path, monkeypatch):
    """Default: the realigned records are written by the host codec; OGE_WRITE_DEVICE=1: they go up to the
    device and out through the GPU deflate.  The same records either way."""
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    monkeypatch.setenv("OGE_WRITE_DEVICE", device_write)
    r = run("localrealign", "-v", "--nopg", "-R", fa, "-L", iv, tmp_path / "reads.bam", "-o", tmp_path / "rl.bam")
    assert ("(gpu, segmented)" in r.stderr) == (device_write == "1"), r.stderr
    oh, _, orecs, ooffs = bamutil.read_bam(tmp_path / "rl.bam")
    assert oh == meta["output_header"]
    check_output(meta, arrays, orecs, np.append(ooffs, np.uint64(len(orecs))))


def test_cli_errors_are_loud(tmp_path):
    r = subprocess.run([OPENGE, "localrealign", str(GOLDEN / "inputs" / "simple.bam")], capture_output=True, text=True)
    assert r.returncode != 0 and "FASTA reference" in r.stderr
    r = subprocess.run([OPENGE, "mergesort", str(GOLDEN / "inputs" / "208.truncated.bam"), "-o", str(tmp_path / "t.bam")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "truncated" in r.stderr
    # --gpus: the sharded reader rejects the file on every rank and the whole-file reader reports it
    r = subprocess.run([OPENGE, "mergesort", "--gpus", "2", str(GOLDEN / "inputs" / "208.truncated.bam"), "-o",
                        str(tmp_path / "t2.bam")], capture_output=True, text=True)
    assert r.returncode != 0 and "truncated" in r.stderr


@pytest.mark.parametrize("cmd", [("mergesort", "-M"), ("dedup", "-r")])
def test_cli_gpu_bgzf_equals_host_codec(tmp_path, cmd):
    """The writer compresses device-resident records on the GPU by default; the decompressed file
    must equal the host codec's (OGE_BGZF_CODEC=libdeflate) byte for byte, incl. -r (dups dropped
    on the device) and the bins recomputed there."""
    import gzip
    import os
    p = L.synth_params(60_000, preset="c2", seed=77)
    recs, offs, hdr = L.synth_host(p)
    src = tmp_path / "in.bam"
    L.write_bam(str(src), hdr, recs, offs, len(offs) - 1, level=1)
    out = {}
    for codec in ("gpu", "libdeflate"):
        env = dict(os.environ)
        env.pop("OGE_BGZF_CODEC", None)
        if codec != "gpu":
            env["OGE_BGZF_CODEC"] = codec
        dst = tmp_path / f"{codec}.bam"
        r = subprocess.run([OPENGE, *cmd, "--nopg", "-v", str(src), "-o", str(dst)],
                           capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        assert ("(gpu," in r.stderr) == (codec == "gpu"), r.stderr
        out[codec] = gzip.decompress(dst.read_bytes())
    assert out["gpu"] == out["libdeflate"]
    assert len(out["gpu"]) > 1_000_000


def test_cli_write_failures_exit_nonzero(tmp_path):
    """a failed device write must leave the writer inert (no write into the closed FILE),
    and a failed fwrite / fflush / fclose (full disk) must give a non-zero exit, not a truncated BAM
    with status 0."""
    import os
    src = GOLDEN / "inputs" / "208.yhet.bam"
    env = dict(os.environ, OGE_TEST_FAIL="write_device")
    r = subprocess.run([OPENGE, "mergesort", "-M", str(src), "-o", str(tmp_path / "f.bam")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode > 0 and "injected failure" in r.stderr, (r.returncode, r.stderr)
    r = subprocess.run([OPENGE, "mergesort", "-M", str(src), "-o", "/dev/full"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode > 0 and "error writing" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.parametrize("G", [2, 3, 8])
def test_cli_gpus_matches_reference(case, tmp_path, G):
    """`--gpus G` (replacing SplitByChromosome/SortedMerge, cmd/command_mergesort.cpp:118-179,
    cmd/command_dedup.cpp:70-113): the same reference outputs as one GPU -- mergesort -M, sort, and
    dedup of the sorted file, with -R dropping the flagged records.  The one input file is read by the
    G ranks from their own byte ranges (FileReader::read_sharded, oge_bgzf_decode_shard).  On a one-GPU
    box the G ranks share the GPU through the host-staged transport."""
    src = case_input(case, tmp_path)
    r = run("mergesort", "-M", "--nopg", "-v", "--gpus", G, src, "-o", tmp_path / "o.bam")
    assert f"{G} ranks" in r.stderr
    assert f"FileReader (sharded over {G} ranks)" in r.stderr
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    run("sort", "--nopg", "--gpus", G, src, "-o", tmp_path / "s.bam")
    h, m, t = digests(tmp_path / "s.bam")
    assert h == case.meta["sorted_header"] and m == case.meta["sort"]["mapped_sha256"]
    run("dedup", "--nopg", "--gpus", G, tmp_path / "s.bam", "-o", tmp_path / "d.bam")
    h, m, t = digests(tmp_path / "d.bam")
    g = case.meta["dedup_sorted_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    run("mergesort", "-R", "--nopg", "--gpus", G, src, "-o", tmp_path / "r.bam")
    _, _, recs, offs = bamutil.read_bam(tmp_path / "r.bam")
    assert len(offs) == case.n - case.meta["sortdedup_v"]["n_dup"]


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("name", ["rl_short", "rl_small", "rl_c5_2k"])
def test_cli_localrealign_gpus_matches_reference(name, G, tmp_path):
    """localrealign --gpus G: the device work sharded over G ranks by interval
    ranges (oge_localrealign_multi) -- rl_short is ONE contig, so the cuts fall inside it -- equals the
    reference's output; every rank gets a share of the intervals, within 10 % of the mean on the C5-shaped
    set (ranges balanced by reads)."""
    import json
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    r = run("localrealign", "-v", "--nopg", "--gpus", G, "-R", fa, "-L", iv, tmp_path / "reads.bam", "-o", tmp_path / "rl.bam")
    oh, _, orecs, ooffs = bamutil.read_bam(tmp_path / "rl.bam")
    assert oh == meta["output_header"]
    check_output(meta, arrays, orecs, np.append(ooffs, np.uint64(len(orecs))))
    line = [l for l in r.stderr.splitlines() if f"LocalRealignment over {G} devices" in l]
    assert line, r.stderr
    st = json.loads(line[0].split(": ", 1)[1])
    iv_per = [st[f"prep_rank{g}_intervals"] for g in range(G)]
    assert sum(iv_per) == st["prep_device_intervals"] and st["prep_host_intervals"] == 0 and min(iv_per) > 0
    if name == "rl_c5_2k":
        mean = sum(iv_per) / G
        assert max(iv_per) <= 1.1 * mean and min(iv_per) >= 0.9 * mean, iv_per


def test_cli_chunked_matches_reference(case, tmp_path):
    """Inputs larger than HBM take the chunked path (sorted runs spilled into host memory, key ranges
    sorted and written one by one); OGE_CHUNK_BYTES forces it with tiny chunks: the reference's
    mergesort -M / sort / -R outputs."""
    import os
    src = case_input(case, tmp_path)
    env = dict(os.environ, OGE_CHUNK_BYTES="200000")
    r = subprocess.run([OPENGE, "mergesort", "-M", "--nopg", "-v", str(src), "-o", str(tmp_path / "o.bam")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert "sorted runs" in r.stderr
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    r = subprocess.run([OPENGE, "sort", "--nopg", str(src), "-o", str(tmp_path / "s.bam")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    h, m, t = digests(tmp_path / "s.bam")
    assert h == case.meta["sorted_header"] and m == case.meta["sort"]["mapped_sha256"]
    r = subprocess.run([OPENGE, "mergesort", "-R", "--nopg", str(src), "-o", str(tmp_path / "r.bam")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    _, _, recs, offs = bamutil.read_bam(tmp_path / "r.bam")
    assert len(offs) == case.n - case.meta["sortdedup_v"]["n_dup"]


@pytest.mark.parametrize("prefetch", [False, True])
def test_cli_streamed_reader_matches_reference(case, tmp_path, prefetch):
    """Files are streamed into HBM through page-locked buffers and indexed on the device
    (OGE_STREAM_MIN lowers the size threshold and the chunk to 64 KiB, so the golden inputs take that
    path in many chunks): the reference's mergesort -M outputs.  prefetch: the CLI reads the file on
    helper threads while HIP comes up and the reader copies those bytes up (OGE_PREFETCH_MIN lowers its
    64 MiB threshold)."""
    import os
    src = case_input(case, tmp_path)
    env = dict(os.environ, OGE_STREAM_MIN="1")
    env.update({"OGE_PREFETCH_MIN": "1"} if prefetch else {"OGE_PREFETCH": "0"})
    r = subprocess.run([OPENGE, "mergesort", "-M", "--nopg", "-v", str(src), "-o", str(tmp_path / "o.bam")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert ("prefetched + device index" if prefetch else "streamed + device index") in r.stderr
    h, m, t = digests(tmp_path / "o.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
