"""Multi-rank helpers for the sharded sort+dedup tests.

OracleBackend is TEST INFRASTRUCTURE: it lets the CPU suite run openge_amd.shard's partition /
exchange / authority protocol over gloo with the oracle (oracle/oge_oracle.c) as each rank's local
sort + dedup, to check the protocol reproduces the single-process result.  The product path binds
HipBackend (the HIP kernels) only."""
from __future__ import annotations

import os
import struct

import numpy as np
import torch

import oracle


class OracleBackend:
    def __init__(self, header: str):
        self.header = header

    @staticmethod
    def _fields(recs, offs, n):
        r = recs.numpy()
        o = offs.numpy()[:n].astype(np.int64)
        ref = np.array([struct.unpack_from("<i", r, x + 4)[0] for x in o], np.int64)
        mref = np.array([struct.unpack_from("<i", r, x + 24)[0] for x in o], np.int64)
        flag = np.array([struct.unpack_from("<H", r, x + 18)[0] for x in o], np.int64)
        return ref, mref, flag

    def route(self, recs, offs, n, owner, n_ref, rank, dest=True, ghost=True, back=True):
        ref, mref, flag = self._fields(recs, offs, n)
        own = owner.numpy().astype(np.int64)
        d = own[np.where((ref >= 0) & (ref < n_ref), ref, n_ref)]
        cand = ((flag & 1) != 0) & ((flag & 8) == 0) & (mref >= 0) & (mref < n_ref) & (ref >= 0)
        mo = own[np.where(cand, mref, n_ref)]
        g = np.where(cand & (mo != d), mo, -1)
        b = np.where((d != rank) & cand & (mref < ref), d, -1)
        t = lambda a: torch.from_numpy(a.astype(np.int32))
        return (t(d) if dest else None, t(g) if ghost else None, t(b) if back else None)

    def gather(self, recs, offs, perm):
        r, o = recs.numpy(), offs.numpy()
        parts = [r[int(o[i]):int(o[i + 1])] for i in perm.numpy().astype(np.int64)]
        sizes = [len(x) for x in parts]
        out = np.concatenate(parts + [np.zeros(64, np.uint8)]) if parts else np.zeros(64, np.uint8)
        off = np.zeros(len(parts) + 1, np.int64)
        np.cumsum(sizes, out=off[1:])
        return torch.from_numpy(out), torch.from_numpy(off)

    def sort_markdup(self, recs, offs, n, opts):
        r, o = recs.numpy(), offs.numpy().astype(np.uint64)
        perm = oracle.sort_perm(r, o, n)
        out, off = self.gather(recs, offs, torch.from_numpy(perm.astype(np.int64)))
        dup, _ = oracle.markdup(out.numpy(), off.numpy().astype(np.uint64), n, self.header)
        ob = out.numpy()
        for k in range(n):
            b = int(off[k]) + 19
            if dup[k] == 1:
                ob[b] |= 4
            elif dup[k] == 0:
                ob[b] &= 0xFB
        return out, off, torch.from_numpy(perm.astype(np.int32))

    def sync(self):
        pass


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init_gloo(rank: int, world: int, port: int):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
