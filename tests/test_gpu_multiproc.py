"""GPU, several PROCESSES on the one GPU: bench.py --gpus N's own bootstrap and call sequence, launched
the way the driver launches it (torch.distributed.run, one process per rank, gloo for the id broadcast
and timing): oge_comm_unique_id on rank 0 -> broadcast -> oge_comm_init_rank -> oge_mergesort_bgzf_dist.
The ranks share the GPU, so oge_comm_init_rank picks the host-staged transport (RCCL refuses two ranks
on one device); on an 8-GPU node the same calls take RCCL.  bench.py --seed 99 --pairs 20000 generates
exactly the c2_20k golden input, so the concatenated rank slices must decompress to the REFERENCE's
own `mergesort -M --nosplit -v` output (tests/golden/c2_20k) and byte for byte to the one-GPU
oge_mergesort_bgzf_dev output of the same reads.  Replaces SplitByChromosome / SortedMerge
(alg/split_by_chromosome.cpp:30-58, alg/sorted_merge.cpp:66-101; cmd/command_mergesort.cpp:118-179)."""
import gzip
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from goldens import load_case
from test_gpu_cli import case_input, digests

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _header_bytes(stream: bytes) -> int:
    """bytes of the BAM header block at the start of a decompressed BAM stream (magic, text, refs)"""
    import struct
    (lt,) = struct.unpack_from("<i", stream, 4)
    q = 8 + lt
    (nref,) = struct.unpack_from("<i", stream, q)
    q += 4
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", stream, q)
        q += 4 + ln + 4
    return q


@pytest.fixture(scope="module")
def one_gpu_c2_20k(built, tmp_path_factory):
    """The one-GPU chain on the golden input: decompressed output bytes."""
    import torch
    from openge_amd import lib as L
    case = load_case("c2_20k")
    src = case_input(case, tmp_path_factory.mktemp("one"))
    z = Path(src).read_bytes()
    ctx = L.Context(0)
    try:
        dz = torch.from_numpy(np.frombuffer(z + b"\0" * 8, np.uint8).copy()).cuda()
        d, nb, nr, nd = ctx.mergesort_bgzf_dev(dz.data_ptr(), len(z), L.mergesort_opts(mark_duplicates=1))
        h = np.empty(nb, np.uint8)
        L.check(L.lib().oge_memcpy(ctx.h, h.ctypes.data, d, nb, 2), ctx.h)
    finally:
        ctx.close()
    return case, gzip.decompress(h.tobytes()), nr, nd


RL_INTERVALS = 1500  # C5 generator, small enough for 8 ranks that each generate the whole set


@pytest.fixture(scope="module")
def one_gpu_realign(built, tmp_path_factory):
    """bench.py's realign leg in one process (world 1) on the small C5 set: its realigned records."""
    d = tmp_path_factory.mktemp("rl1")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--realign-only", "--realign-intervals", str(RL_INTERVALS),
           "--no-cpu-baseline", "--dump-dir", str(d)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    return (d / "realign_0.bin").read_bytes()


@pytest.mark.parametrize("world,realign,records", [(2, False, "overlap"), (3, False, "overlap"), (4, True, "overlap"),
                                                  (8, False, "overlap"), (2, False, "blocking")])
def test_bench_multiprocess_bootstrap_matches_reference(world, realign, records, tmp_path, one_gpu_c2_20k, request):
    """ONE input file (the c2_20k golden input's records behind its header), every rank decoding the BGZF
    blocks of its byte range (oge_mergesort_bgzf_shard).  world 4 and 8 are the rank counts of the 8-GPU
    node's scaling run (config 4), here as processes sharing the one GPU; world 4 also runs the realign
    leg (contig-range shards, no exchange), whose concatenated rank outputs must equal the one-process
    realign output byte for byte.  records=blocking: the record exchange before the input pass
    (OGE_DIST_RECORDS=blocking, the fallback of the side-stream overlap), same output."""
    case, want, nr1, nd1 = one_gpu_c2_20k
    env = dict(os.environ, OGE_COMM_DIR=str(tmp_path), OGE_COMM_TIMEOUT="120", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="2")
    if records == "blocking":
        env["OGE_DIST_RECORDS"] = "blocking"
    # --standalone: the launcher binds its rendezvous port itself (port 0), so no other process can take it
    # between a probe and the bind (a probed free port was taken once on a shared box: EADDRINUSE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           f"--nproc-per-node={world}",
           str(ROOT / "bench.py"), "--gpus", str(world), "--pairs", "20000", "--seed", "99", "--steps", "1",
           "--warmup", "1", "--dump-dir", str(tmp_path)]
    cmd += ["--realign-intervals", str(RL_INTERVALS)] if realign else ["--no-realign"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world
    assert line["config"]["transport"] == "host"
    # the diagnosable breakdown: every rank's exchanges (bytes and times) and stage times
    ex = line["exchanges"]
    assert len(ex["per_rank"]) == world and len(line["stages_ms_per_rank"]) == world
    by = ex["by_tag"]
    for tag in ("records", "record_sizes", "fragments", "matejoin_candidates", "matejoin_minirecs", "pair_ends",
                "dup_marks", "plans", "status", "shard_framing", "shard_edges", "shard_records"):
        assert tag in by, tag
    # the codec is split: every rank inflated the blocks of its own byte range (~1/G of the file), the
    # parts add up to the whole file and stream
    sh = line["config"]["shard_per_rank"]
    assert len(sh) == world
    nblk = sum(s["shard_blocks"] for s in sh)
    assert sum(s["shard_zbytes"] for s in sh) == line["config"]["input_file_bytes"]
    assert max(s["shard_blocks"] for s in sh) <= nblk // world + 2
    assert sum(s["shard_records"] for s in sh) == nr1
    # every record moves to its range owner or stays: sent + kept = the record bytes of the input
    rec_bytes = by["records"]["bytes_between_ranks"] + by["records"]["bytes_kept"]
    assert rec_bytes == int(np.frombuffer(want, np.uint8).size) - _header_bytes(want)
    assert by["record_sizes"]["bytes_between_ranks"] + by["record_sizes"]["bytes_kept"] == 4 * nr1
    # the record exchange ran on a side stream beside the own records' input pass
    assert by["records"]["mode"] == ("side_stream" if records == "overlap" else "blocking")
    assert by["record_sizes"]["mode"] == "blocking"
    if realign:
        rl = line["realign"]
        assert rl["n_gpus"] == world and rl["value"] > 0
        got = b"".join((tmp_path / f"realign_{g}.bin").read_bytes() for g in range(world))
        assert got == request.getfixturevalue("one_gpu_realign")
    assert line["config"]["duplicates_flagged"] == case.meta["sortdedup_v"]["n_dup"] == nd1
    out = b"".join((tmp_path / f"slice_{g}.bam").read_bytes() for g in range(world))
    assert out[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    (tmp_path / "all.bam").write_bytes(out)
    h, m, t = digests(tmp_path / "all.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    assert gzip.decompress(out) == want
    assert not list(tmp_path.glob("oge_comm_*")), "meeting file left behind"
