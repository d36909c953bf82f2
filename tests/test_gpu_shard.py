"""GPU: contig-sharded sort + dedup (openge_amd.shard with the HIP backend) run as 2 and 3 ranks
sharing the one GPU of the test box (gloo carries the exchange; RCCL needs one GPU per rank and is
exercised by bench.py --gpus N on a full node).  The concatenated rank outputs must equal the
single-GPU oge_sort_markdup_dev output byte for byte."""
import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from shard_util import free_port, init_gloo

pytestmark = pytest.mark.gpu


def _single(preset, pairs, seed):
    from openge_amd import lib as L
    p = L.synth_params(pairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    n = len(offs) - 1
    ctx = L.Context(0)
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(int(offs[-1]) + 64, dtype=torch.uint8, device="cuda")
    d_oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                         d_oo.data_ptr())
    ctx.sync()
    out = d_out[:int(d_oo[-1].item())].cpu().numpy().tobytes()
    ctx.close()
    return out


def _worker(rank, world, port, preset, pairs, seed, q):
    import torch.distributed as dist
    from openge_amd import lib as L, shard
    init_gloo(rank, world, port)
    torch.cuda.set_device(0)
    p = L.synth_params(pairs, preset=preset, seed=seed)
    n_all = 2 * pairs
    s0, s1 = n_all * rank // world, n_all * (rank + 1) // world
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    ctx = L.Context(0, stream=st.cuda_stream)
    d_offs = torch.empty(s1 - s0 + 1, dtype=torch.int64, device="cuda")
    ctx.synth_range_dev(p, s0, s1 - s0, d_offs.data_ptr(), None)
    ctx.sync()
    d_recs = torch.empty(int(d_offs[-1].item()) + 64, dtype=torch.uint8, device="cuda")
    ctx.synth_range_dev(p, s0, s1 - s0, d_offs.data_ptr(), d_recs.data_ptr())
    import ctypes as C
    buf = C.create_string_buffer(1 << 16)
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
    opts, keep = L.markdup_opts_from_header(buf.value.decode(), p.n_ref)
    owners = shard.contig_owners([int(p.ref_len[i]) for i in range(p.n_ref)], world)
    T = {}
    out, off, k = shard.sort_markdup_sharded(shard.HipBackend(ctx), d_recs, d_offs, s1 - s0, p.n_ref, owners, opts,
                                             timings=T)
    mine = out[:int(off[k].item())].cpu().numpy().tobytes()
    got = [None] * world
    dist.all_gather_object(got, (mine, T["ghost_messages"]))
    if rank == 0:
        q.put((b"".join(g[0] for g in got), sum(g[1] for g in got)))
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,preset,pairs,seed", [(2, "c2", 40000, 7), (3, "mix", 5000, 2)])
def test_gpu_sharded_equals_single_gpu(built, world, preset, pairs, seed):
    want = _single(preset, pairs, seed)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, preset, pairs, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, msgs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert got == want
    assert msgs > 0
