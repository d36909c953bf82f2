"""CPU (gloo, world_size 2 and 3): the contig-sharded sort + dedup protocol of openge_amd.shard --
ownership, ghost mates, all-to-all exchange, authority messages -- reproduces the single-process
`mergesort -M --nosplit` result byte for byte.  Each rank's local compute is the oracle
(tests/shard_util.OracleBackend); the GPU form of the same test is in test_gpu_shard.py."""
import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from shard_util import OracleBackend, free_port, init_gloo


def _data(preset, pairs, seed):
    from openge_amd import lib as L
    p = L.synth_params(pairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    return recs, offs, hdr, p.n_ref, [int(p.ref_len[i]) for i in range(p.n_ref)]


def _reference(recs, offs, hdr):
    n = len(offs) - 1
    be = OracleBackend(hdr)
    out, off, _ = be.sort_markdup(torch.from_numpy(recs), torch.from_numpy(offs.astype(np.int64)), n, None)
    return out.numpy()[:int(off[-1])].tobytes()


def _worker(rank, world, port, preset, pairs, seed, q):
    import torch.distributed as dist
    from openge_amd import shard
    init_gloo(rank, world, port)
    recs, offs, hdr, n_ref, lens = _data(preset, pairs, seed)
    n = len(offs) - 1
    # this rank's input shard: every world-th record (mates land on different ranks)
    idx = np.arange(rank, n, world)
    parts = [recs[int(offs[i]):int(offs[i + 1])] for i in idx]
    mine = np.concatenate(parts + [np.zeros(64, np.uint8)])
    moff = np.zeros(len(idx) + 1, np.int64)
    np.cumsum([len(x) for x in parts], out=moff[1:])
    owners = shard.contig_owners(lens, world)
    T = {}
    out, off, k = shard.sort_markdup_sharded(OracleBackend(hdr), torch.from_numpy(mine), torch.from_numpy(moff),
                                             len(idx), n_ref, owners, None, timings=T)
    got = [None] * world
    dist.all_gather_object(got, (out.numpy()[:int(off[k])].tobytes(), T["ghost_messages"]))
    if rank == 0:
        q.put((b"".join(g[0] for g in got), sum(g[1] for g in got)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,preset,pairs,seed", [(2, "mix", 1500, 5), (3, "c2", 2000, 11), (2, "c2", 2500, 3)])
def test_sharded_equals_single(built, world, preset, pairs, seed):
    recs, offs, hdr, n_ref, lens = _data(preset, pairs, seed)
    want = _reference(recs, offs, hdr)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, preset, pairs, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, msgs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert got == want
    if preset == "c2":
        assert msgs > 0  # inter-contig pairs exercised the authority messages


def test_contig_owners_monotone_and_balanced():
    from openge_amd import shard
    from openge_amd.lib import GRCH38_MB
    for w in (1, 2, 4, 8):
        o = shard.contig_owners(GRCH38_MB, w)
        assert o == sorted(o) and o[-1] == w - 1 and set(o) == set(range(w))
        load = [sum(l for l, x in zip(GRCH38_MB, o) if x == r) for r in range(w)]
        assert max(load) / (sum(GRCH38_MB) / w) < 1.35
