"""Multi-GPU local realignment: contig-range shards, one process per GPU, no data exchange.

SURVEY §8e: realignment shards naturally.  Everything LocalRealignment keeps between reads is per
contig: a read bin never spans contigs (ReadBin::add, algorithms/local_realignment.cpp:263-275),
intervals are walked in order (map_func :455-553), and the mate-fixing writer flushes and forgets
its mate map whenever a read of another contig arrives (ConstrainedMateFixingManager::
addReadInternal, util/gatk/ConstrainedMateFixingManager.cpp:312-330).  So rank r realigns the
records of its contig range (contiguous refID ranges, ``contig_owners``)
with the whole interval list, and the rank outputs concatenate into the single-process output.

The one coupling the writer has across a contig boundary -- a flush that finds
maxRecordsInMemory (150,000) reads still waiting keeps its modified mate entries -- is detected
(``tail_waiting`` in the stats) and reported as an error rather than silently diverging.
"""
from __future__ import annotations

import numpy as np

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


def record_refids(recs: np.ndarray, offs: np.ndarray, n: int) -> np.ndarray:
    """refID (int32 at byte 4) of records 0..n-1."""
    o = np.asarray(offs[:n], dtype=np.int64)
    b = recs[o[:, None] + np.arange(4, 8)]
    return np.ascontiguousarray(b).view("<i4").reshape(-1)


def contig_slices(recs: np.ndarray, offs: np.ndarray, n: int, ref_lens: list[int], world: int) -> list[tuple[int, int]]:
    """[lo, hi) record range of each rank in coordinate-sorted input."""
    owners = np.asarray(contig_owners(ref_lens, world), dtype=np.int64)
    ref = record_refids(recs, offs, n).astype(np.int64)
    own = owners[np.where(ref < 0, len(owners) - 1, ref)]
    if n and np.any(np.diff(own) < 0):
        raise ValueError("localrealign shards need coordinate-sorted input")
    cuts = np.searchsorted(own, np.arange(world + 1), side="left")
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def localrealign_slice(ctx: L.Context, header_text: str, recs: np.ndarray, offs: np.ndarray, lo: int, hi: int,
                       fasta: str, intervals: str, opts: L.RealignOpts | None, last: bool):
    """This rank's part: (out records, out offsets, stats)."""
    if hi <= lo:
        return np.zeros(0, np.uint8), np.zeros(1, np.uint64), {"tail_waiting": 0}
    o = np.ascontiguousarray(offs[lo:hi + 1], dtype=np.uint64)
    out, oo, st = ctx.localrealign(header_text, recs, o, hi - lo, fasta, intervals, opts)
    limit = opts.max_records_in_memory if opts is not None else 150000
    if not last and st.get("tail_waiting", 0) >= limit:
        raise RuntimeError("localrealign shards: the mate-fixing writer held >= maxRecordsInMemory reads at a "
                           "shard boundary; run this input on one GPU")
    return out, oo, st
