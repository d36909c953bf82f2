"""Multi-GPU sort + dedup: contig-sharded, one process per GPU, records exchanged with
torch.distributed all_to_all (RCCL over xGMI on MI355X; gloo in CPU tests).

Replaces the reference's split-by-chromosome parallelism (algorithms/split_by_chromosome.cpp:30-58
routes refID % K to K MarkDuplicates chains, algorithms/sorted_merge.cpp:66-101 re-merges them) with
a design whose result equals the single-GPU (`--nosplit`) result:

1. Ownership: rank r owns a contiguous refID range (``contig_owners``: balanced by contig length,
   non-decreasing in refID, refID -1 on the last rank), so rank outputs concatenate into the global
   coordinate order -- no k-way merge.
2. Exchange: every record goes to the owner of its refID.  A mate-join candidate whose mate's
   contig is owned elsewhere is also sent there as a read-only *ghost*.  Each rank then holds every
   pair whose read1 (the lower refID end, mark_duplicates.cpp:226-241) it owns, so its pair groups
   (keyed on read1) and fragment groups (keyed on the record itself) are complete, and the local
   sorted order of its records is the global order restricted to them.
3. Local pipeline: the single-GPU ``oge_sort_markdup_dev`` over owned + ghost records.
4. Authority: for a pair split across ranks only the rank owning read1 sees the whole pair group;
   it sends the 0x400 decision for its ghost read2 to read2's owner, which overrides its own.
5. Ghosts are dropped (``oge_gather_records_dev`` of the owned positions).

Collectives (per step): 2 tiny count exchanges, the record bytes, the record sizes and ids (8+8 B per
record), and the authority messages (ghost pairs only, ~1% of records).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from . import lib as L


def contig_owners(ref_lens: list[int], world: int) -> list[int]:
    """Owner rank of each refID (+ one trailing entry for refID -1, on the last rank).

    Contiguous refID ranges (so rank outputs concatenate in sorted order) minimising the largest
    range's total length: binary search on the capacity with a greedy fill (linear partition)."""
    lens = [float(x) for x in ref_lens]

    def fill(cap):
        owners, r, acc = [], 0, 0.0
        for ln in lens:
            if acc > 0 and acc + ln > cap:
                r, acc = r + 1, 0.0
            owners.append(r)
            acc += ln
        return owners

    lo, hi = max(lens, default=0.0), sum(lens)
    for _ in range(100):
        mid = (lo + hi) / 2
        if fill(mid)[-1:] and fill(mid)[-1] >= world:
            lo = mid
        else:
            hi = mid
    owners = fill(hi) if lens else []
    owners = [min(o, world - 1) for o in owners]
    return owners + [world - 1]


class HipBackend:
    """Device compute through the C ABI on torch CUDA(HIP) tensors."""

    def __init__(self, ctx: L.Context):
        # kernels and the torch ops between them must share one stream, or they race
        if ctx.stream != torch.cuda.current_stream().cuda_stream:
            raise ValueError("HipBackend: create the Context on torch's current stream "
                             "(torch.cuda.set_stream(s); L.Context(dev, stream=s.cuda_stream))")
        self.ctx = ctx

    def route(self, recs, offs, n, owner, n_ref, rank, dest=True, ghost=True, back=True):
        dev = recs.device
        d = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if dest else None
        g = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if ghost else None
        b = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if back else None
        p = lambda t: t.data_ptr() if t is not None else None
        L.check(L.lib().oge_shard_route_dev(self.ctx.h, recs.data_ptr(), offs.data_ptr(), n, owner.data_ptr(), n_ref,
                                            rank, p(d), p(g), p(b)), self.ctx.h)
        return tuple(t[:n] if t is not None else None for t in (d, g, b))

    def gather(self, recs, offs, perm):
        m = perm.numel()
        sizes = offs[1:] - offs[:-1]
        total = int(sizes[perm.long()].sum().item()) if m else 0
        out = torch.empty(total + 64, dtype=torch.uint8, device=recs.device)
        out_off = torch.empty(m + 1, dtype=torch.int64, device=recs.device)
        if m:
            self.ctx.gather_records_dev(recs.data_ptr(), offs.data_ptr(), perm.data_ptr(), m, out.data_ptr(),
                                        out_off.data_ptr())
        else:
            out_off.zero_()
        return out, out_off

    def sort_markdup(self, recs, offs, n, opts):
        total = int(offs[n].item())
        out = torch.empty(total + 64, dtype=torch.uint8, device=recs.device)
        out_off = torch.empty(n + 1, dtype=torch.int64, device=recs.device)
        perm = torch.empty(max(n, 1), dtype=torch.int32, device=recs.device)
        if n:
            self.ctx.sort_markdup_dev(recs.data_ptr(), offs.data_ptr(), n, opts, perm.data_ptr(), out.data_ptr(),
                                      out_off.data_ptr())
        else:
            out_off.zero_()
        return out, out_off, perm[:n]

    def sync(self):
        self.ctx.sync()


def _coll_device(group) -> bool:
    """True when the process group's backend moves device tensors (RCCL); gloo needs host tensors."""
    return dist.get_backend(group) != "gloo"


def _a2a(inp: torch.Tensor, in_splits: list[int], out_splits: list[int], group, out: torch.Tensor | None = None):
    """all_to_all_single with split sizes; receives into `out` when given (no staging copy on RCCL)."""
    dev = inp.device
    on_dev = _coll_device(group) or dev.type == "cpu"
    src = inp if on_dev else inp.cpu()
    dst = out if (out is not None and on_dev) else torch.empty(sum(out_splits), dtype=inp.dtype, device=src.device)
    dist.all_to_all_single(dst, src.contiguous(), out_splits, in_splits, group=group)
    if out is not None and dst is not out:
        out.copy_(dst)
        return out
    return dst.to(dev) if dst.device != dev else dst


def _counts(send: torch.Tensor, world: int, group) -> torch.Tensor:
    return _a2a(send.to(torch.int64), [1] * world, [1] * world, group)


def sort_markdup_sharded(backend, recs: torch.Tensor, offs: torch.Tensor, n: int, n_ref: int, owners: list[int],
                         opts, group=None, timings: dict | None = None):
    """One rank's part of contig-sharded sort + dedup.  `recs`/`offs` (n + 1) hold this rank's input
    shard (any subset of the sample).  Returns (out, out_off, n_owned): this rank's slice of the
    global `mergesort -M --nosplit` output, in order."""
    import time

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = recs.device
    T = timings if timings is not None else {}
    t0 = time.perf_counter()
    owner = torch.tensor(owners, dtype=torch.int32, device=dev)

    # ---- 1. route + pack (records ordered by destination; ghosts appended to their mate's owner)
    dest, ghost, _ = backend.route(recs, offs, n, owner, n_ref, rank, True, True, False)
    gi = torch.nonzero(ghost >= 0).squeeze(1)
    idx_all = torch.cat([torch.arange(n, device=dev, dtype=torch.int64), gi])
    dst_all = torch.cat([dest.long(), ghost[gi].long()])
    order = torch.argsort(dst_all, stable=True)
    send_idx = idx_all[order]
    send_cnt = torch.bincount(dst_all, minlength=world)
    send_recs, send_off = backend.gather(recs, offs, send_idx.to(torch.int32))
    cum = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(send_cnt, 0)])
    send_bytes = send_off[cum[1:]] - send_off[cum[:-1]]
    send_ids = (rank << 40) | send_idx
    send_sizes = send_off[1:] - send_off[:-1]
    del idx_all, dst_all, order, dest, ghost, gi
    T["route_pack_s"] = time.perf_counter() - t0

    # ---- 2. exchange
    t1 = time.perf_counter()
    recv_cnt = _counts(send_cnt, world, group)
    recv_bytes = _counts(send_bytes, world, group)
    sc, rc = send_cnt.tolist(), recv_cnt.tolist()
    sb, rb = send_bytes.tolist(), recv_bytes.tolist()
    n_recv = int(sum(rc))
    recv = torch.empty(int(sum(rb)) + 64, dtype=torch.uint8, device=dev)
    _a2a(send_recs[:sum(sb)], sb, rb, group, out=recv[:sum(rb)])
    recv_sizes = _a2a(send_sizes, sc, rc, group)
    recv_ids = _a2a(send_ids, sc, rc, group)
    del send_recs, send_off, send_sizes, send_ids
    recv_off = torch.zeros(n_recv + 1, dtype=torch.int64, device=dev)
    torch.cumsum(recv_sizes, 0, out=recv_off[1:])
    backend.sync()
    T["exchange_s"] = time.perf_counter() - t1
    T["exchanged_bytes"] = int(sum(sb))

    # ---- 3. local sort + dedup over owned + ghost records
    t2 = time.perf_counter()
    out, out_off, perm = backend.sort_markdup(recv, recv_off, n_recv, opts)
    ids_sorted = recv_ids[perm.long()]
    del recv, recv_off, recv_sizes, recv_ids, perm
    dest2, _, back = backend.route(out, out_off, n_recv, owner, n_ref, rank, True, False, True)
    backend.sync()
    T["local_s"] = time.perf_counter() - t2

    # ---- 4. authority messages: this rank's 0x400 decision for ghosts whose read1 it owns
    t3 = time.perf_counter()
    bi = torch.nonzero(back >= 0).squeeze(1)
    mdst = back[bi].long()
    o2 = torch.argsort(mdst, stable=True)
    bi, mdst = bi[o2], mdst[o2]
    msg_ids = ids_sorted[bi]
    msg_flag = ((out[out_off[bi] + 19] >> 2) & 1).to(torch.uint8)
    mcnt = torch.bincount(mdst, minlength=world)
    rmcnt = _counts(mcnt, world, group)
    ms, mr = mcnt.tolist(), rmcnt.tolist()
    r_ids = _a2a(msg_ids, ms, mr, group)
    r_flag = _a2a(msg_flag, ms, mr, group)

    # ---- 5. drop ghosts, apply the messages
    owned = torch.nonzero(dest2 == rank).squeeze(1)
    final, final_off = backend.gather(out, out_off, owned.to(torch.int32))
    final_ids = ids_sorted[owned]
    del out, out_off, ids_sorted, dest2, back
    if r_ids.numel():
        if final_ids.numel() == 0:
            raise RuntimeError("sharded dedup: an authority message names a record this rank does not own")
        sids, sorder = torch.sort(final_ids)
        pos = torch.searchsorted(sids, r_ids)
        pos = torch.clamp(pos, max=max(sids.numel() - 1, 0))
        if not torch.equal(sids[pos], r_ids):
            raise RuntimeError("sharded dedup: an authority message names a record this rank does not own")
        b = final_off[sorder[pos]] + 19
        final[b] = (final[b] & 0xFB) | (r_flag << 2)
    backend.sync()
    T["authority_s"] = time.perf_counter() - t3
    T["ghost_messages"] = int(r_ids.numel())
    return final, final_off, int(owned.numel())
