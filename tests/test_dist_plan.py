"""CPU: the multi-GPU partition code (openge_amd/csrc/dist_plan.h + dist_local.h) run by G threads over
the in-process hub with memcpy as the transport (tests/native/dist_selftest.cpp): range splitters on
C2 ByPosition keys, routing, the all-to-all plan and exchange, the max reduce-scatter.  The rank
slices must concatenate into the global sorted order with no key straddling two ranks, and the
load must stay within max/mean <= 1.05 up to 8 ranks (contig ownership gave 1.20).
The same binary is also built with ThreadSanitizer and run on a smaller key set."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "dist_selftest.cpp"
CSRC = ROOT / "openge_amd" / "csrc"


def _build(out: Path, extra=()):
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", f"-I{CSRC}", *extra, str(SRC), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def _c2_keys(pairs: int, seed: int) -> np.ndarray:
    from openge_amd import lib as L
    p = L.synth_params(pairs, preset="c2", seed=seed)
    recs, offs, _ = L.synth_host(p)
    o = offs[:-1].astype(np.int64)
    ref = recs[o[:, None] + np.arange(4, 8)].copy().view("<i4").reshape(-1).astype(np.int64)
    pos = recs[o[:, None] + np.arange(8, 12)].copy().view("<i4").reshape(-1).astype(np.int64)
    flag = recs[o[:, None] + np.arange(18, 20)].copy().view("<u2").reshape(-1).astype(np.int64)
    ref = np.where(ref < 0, p.n_ref, ref)
    k = (ref << 33) | ((pos + 1) << 1) | ((flag >> 4) & 1)
    return k.astype(np.uint64)


@pytest.fixture(scope="module")
def keys_file(tmp_path_factory, built):
    d = tmp_path_factory.mktemp("dist")
    f = d / "c2_keys.bin"
    _c2_keys(200_000, 7).tofile(f)
    return f


def test_range_split_exchange_and_balance(keys_file, tmp_path):
    exe = _build(tmp_path / "dist_selftest")
    r = subprocess.run([str(exe), str(keys_file), "1", "2", "3", "4", "5", "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    bal = json.loads(r.stdout)
    assert bal["1"] == 1.0
    for g, b in bal.items():
        assert b <= 1.05, (g, b)


def test_partition_code_is_race_free_under_tsan(keys_file, tmp_path):
    exe = _build(tmp_path / "dist_selftest_tsan", ("-fsanitize=thread", "-g"))
    small = tmp_path / "small.bin"
    np.fromfile(keys_file, dtype=np.uint64)[:60_000].tofile(small)
    r = subprocess.run([str(exe), str(small), "2", "3", "4"], capture_output=True, text=True, timeout=300,
                       env={"TSAN_OPTIONS": "halt_on_error=1", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_skewed_keys_still_exact(tmp_path):
    """A pile of identical keys bigger than 1/G of the input: it stays on one rank (balance is then
    bounded by the pile, not by the splitters), the output is still the global order."""
    exe = _build(tmp_path / "dist_selftest")
    rng = np.random.default_rng(3)
    k = np.concatenate([rng.integers(0, 1 << 40, 30_000), np.full(20_000, 12345 << 20)]).astype(np.uint64)
    rng.shuffle(k)
    f = tmp_path / "skew.bin"
    k.tofile(f)
    r = subprocess.run([str(exe), str(f), "2", "4", "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr


def test_host_staged_transport_across_processes(keys_file, tmp_path):
    """The host-staged transport (openge_amd/csrc/dist_shm.h: device -> shared host segment -> device,
    what oge_comm_init_rank picks when ranks share a GPU) run by G forked processes with memcpy ops and
    a 1 MB staging area, so every exchange takes many rounds: the same global order and balance."""
    import os
    exe = _build(tmp_path / "dist_selftest")
    env = dict(os.environ, OGE_COMM_STAGE_MB="1", OGE_COMM_TIMEOUT="60", OGE_COMM_DIR=str(tmp_path))
    r = subprocess.run([str(exe), "--shm", str(keys_file), "1", "2", "3", "5", "8"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    bal = json.loads(r.stdout)
    for g, b in bal.items():
        assert b <= 1.05, (g, b)
    assert not list(tmp_path.glob("oge_comm_*")), "the meeting file must be unlinked once every rank joined"


def test_failing_rank_returns_on_every_rank(tmp_path):
    """One rank's copy operations fail inside the collectives: over the in-process hub and
    over the host-staged transport, every rank still returns (no rank waits in a collective the failing
    one left), and the failing rank reports the failure."""
    import os
    exe = _build(tmp_path / "dist_selftest")
    env = dict(os.environ, OGE_COMM_TIMEOUT="60", OGE_COMM_DIR=str(tmp_path))
    r = subprocess.run([str(exe), "--fail-copy", "2", "3", "5"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr


def test_dead_peer_ends_the_wait(tmp_path):
    """A rank's process exits after joining the host-staged meeting (time out on a dead peer,
    not a slow one): the other ranks see its posted pid gone and return with an error within seconds,
    although the wall-clock backstop (OGE_COMM_TIMEOUT) is ten minutes."""
    import os
    import time
    exe = _build(tmp_path / "dist_selftest")
    env = dict(os.environ, OGE_COMM_TIMEOUT="600", OGE_COMM_DIR=str(tmp_path))
    t0 = time.time()
    r = subprocess.run([str(exe), "--dead-rank", "2", "4"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert time.time() - t0 < 60


def test_foreign_pid_namespace_peer_is_not_dead(tmp_path):
    """a rank whose posted pid means nothing in this pid namespace (a container sharing the
    segment) is alive while its heartbeat moves -- the schedule completes and verifies; when such a rank
    exits, its stopped heartbeat ends the others' waits (OGE_COMM_STALE_S) long before the backstop."""
    import os
    import time
    exe = _build(tmp_path / "dist_selftest")
    env = dict(os.environ, OGE_COMM_TIMEOUT="600", OGE_COMM_DIR=str(tmp_path), OGE_COMM_STALE_S="3")
    r = subprocess.run([str(exe), "--foreign-pid", "2", "4"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    t0 = time.time()
    r = subprocess.run([str(exe), "--foreign-dead", "3"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert time.time() - t0 < 60
