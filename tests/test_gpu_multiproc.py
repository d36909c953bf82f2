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
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from goldens import load_case
from test_gpu_cli import case_input, digests

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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


@pytest.mark.parametrize("world", [2, 3])
def test_bench_multiprocess_bootstrap_matches_reference(world, tmp_path, one_gpu_c2_20k):
    case, want, nr1, nd1 = one_gpu_c2_20k
    env = dict(os.environ, OGE_COMM_DIR=str(tmp_path), OGE_COMM_TIMEOUT="120", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "bench.py"), "--gpus", str(world), "--pairs", "20000", "--seed", "99", "--steps", "1",
           "--warmup", "1", "--no-realign", "--dump-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world
    assert line["config"]["transport"] == "host"
    assert line["config"]["duplicates_flagged"] == case.meta["sortdedup_v"]["n_dup"] == nd1
    out = b"".join((tmp_path / f"slice_{g}.bam").read_bytes() for g in range(world))
    assert out[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    (tmp_path / "all.bam").write_bytes(out)
    h, m, t = digests(tmp_path / "all.bam")
    g = case.meta["sortdedup_v"]
    assert h == g["header"] and m == g["mapped_sha256"] and t == g["tail_multiset_sha256"]
    assert gzip.decompress(out) == want
    assert not list(tmp_path.glob("oge_comm_*")), "meeting file left behind"
