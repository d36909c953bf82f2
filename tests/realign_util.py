"""Realignment test helpers: the CPU harness (product host phases + oracle scan) and output
comparison against the reference's outputs."""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np

import bamutil
from native.build import build as build_native

_h = None


def harness():
    global _h
    if _h is None:
        L = C.CDLL(str(build_native()))
        L.realign_cpu.restype = C.c_void_p
        L.realign_cpu.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_char_p, C.c_char_p,
                                  C.c_int, C.c_int, C.c_int]
        L.realign_cpu_stats.restype = C.c_char_p
        L.realign_cpu_stats.argtypes = [C.c_void_p]
        L.realign_cpu_error.restype = C.c_char_p
        L.realign_cpu_error.argtypes = [C.c_void_p]
        L.realign_cpu_count.restype = C.c_uint64
        L.realign_cpu_count.argtypes = [C.c_void_p]
        L.realign_cpu_records.restype = C.c_void_p
        L.realign_cpu_records.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.realign_cpu_offsets.restype = C.c_void_p
        L.realign_cpu_offsets.argtypes = [C.c_void_p]
        L.realign_cpu_free.argtypes = [C.c_void_p]
        _h = L
    return _h


def realign_cpu(header: str, recs: np.ndarray, offs: np.ndarray, n: int, fasta: str, intervals: str, threads: int = 4,
                max_records: int = 0, mate_sequential: bool = False, stats: dict | None = None):
    """-> (out recs, out offsets[n+1]) from the product host phases with the oracle scan.
    max_records > 0 overrides MAX_RECORDS_IN_MEMORY; mate_sequential forces the one-writer path."""
    L = harness()
    hb = header.encode()
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    h = L.realign_cpu(hb, len(hb), recs.ctypes.data, offs.ctypes.data, n, fasta.encode(), intervals.encode(), threads,
                      max_records, int(mate_sequential))
    try:
        err = L.realign_cpu_error(h).decode()
        if err:
            raise RuntimeError(err)
        if stats is not None:
            import json
            stats.update(json.loads(L.realign_cpu_stats(h).decode()))
        cnt = int(L.realign_cpu_count(h))
        nb = C.c_uint64()
        rp = L.realign_cpu_records(h, C.byref(nb))
        out = np.ctypeslib.as_array((C.c_uint8 * nb.value).from_address(rp)).copy()
        oo = np.ctypeslib.as_array((C.c_uint64 * (cnt + 1)).from_address(L.realign_cpu_offsets(h))).copy()
    finally:
        L.realign_cpu_free(h)
    return out, oo


def record_key(rb: bytes) -> tuple[str, int]:
    """Identity of a read across realignment: name + first/second-of-pair bits."""
    f = bamutil.fields(rb)
    return f["name"], f["flag"] & 0xC0


def digest(recs: np.ndarray, offs) -> dict:
    h = hashlib.sha256()
    per = []
    for o in offs:
        rb = bamutil.rec_bytes(recs, o)
        h.update(rb)
        per.append(int.from_bytes(hashlib.blake2b(rb, digest_size=8).digest(), "little"))
    return {"stream_sha256": h.hexdigest(), "per_record": np.array(per, dtype=np.uint64)}


def first_difference(a_recs, a_offs, b_recs, b_offs) -> str:
    """Human-readable description of the first differing record (for assertion messages)."""
    n = min(len(a_offs), len(b_offs))
    for k in range(n):
        ra, rb = bamutil.rec_bytes(a_recs, a_offs[k]), bamutil.rec_bytes(b_recs, b_offs[k])
        if ra != rb:
            return f"record {k}: got {bamutil.fields(ra)} expected {bamutil.fields(rb)}"
    return f"record counts differ: {len(a_offs)} vs {len(b_offs)}"
