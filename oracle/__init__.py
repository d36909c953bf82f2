"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the openge_amd parity tests.

`oge_oracle.c` restates the reference's coordinate sort order (util/bamtools/Sort.h:116-133),
MarkDuplicates (algorithms/mark_duplicates.cpp:185-540) and the local-realignment offset scan
(findBestOffset, algorithms/local_realignment.cpp:641-679,1126-1164) in plain C.  Only tests/, the smoke check
in __graft_entry__ and bench.py's cpu_baseline leg may use this package, and only as the checker
or the timed CPU baseline -- never as the thing measured or shipped.

The restatement is pinned against the reference itself: oracle/_ref/ref_driver is built from the
reference's own sources (oracle/Makefile.ref) and its outputs are the committed goldens under
tests/golden/ (see tests/golden/make_goldens.py and tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SO = HERE / "liboge_oracle.so"
SRC = HERE / "oge_oracle.c"
REF_DRIVER = HERE / "_ref" / "ref_driver"


def build() -> Path:
    if not SO.exists() or SO.stat().st_mtime < SRC.stat().st_mtime:
        subprocess.run(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-o", str(SO), str(SRC)], check=True)
    return SO


def build_ref() -> Path | None:
    """Build oracle/_ref/ref_driver from /root/reference (only where the reference is present)."""
    if not Path("/root/reference/openge/src").exists():
        return None
    subprocess.run(["make", "-s", "-f", str(HERE / "Makefile.ref"), "-j8"], check=True, cwd=str(HERE.parent))
    return REF_DRIVER


_lib = None


def _L():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(SO))
        L.oracle_sort_perm.restype = C.c_int
        L.oracle_sort_perm.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.oracle_realign_scan.restype = C.c_int
        L.oracle_realign_scan.argtypes = [C.c_void_p] * 6 + [C.c_uint64, C.c_void_p, C.c_void_p]
        L.oracle_markdup_split.restype = C.c_int64
        L.oracle_markdup_split.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                           C.c_int32, C.c_int16, C.c_int, C.c_int, C.c_void_p]
        L.oracle_filter.restype = C.c_uint64
        L.oracle_filter.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int] + [C.c_int32] * 7 + [C.c_uint64,
                                                                                               C.c_void_p]
        L.oracle_sort_name.restype = C.c_int
        L.oracle_sort_name.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.oracle_markdup.restype = C.c_int64
        L.oracle_markdup.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                     C.c_int32, C.c_int16, C.c_int, C.c_void_p]
        _lib = L
    return _lib


def sort_perm(recs: np.ndarray, offs: np.ndarray, n: int) -> np.ndarray:
    """perm[k] = input index at sorted position k (Sort::ByPosition, input-index tie-break)."""
    perm = np.empty(max(n, 1), dtype=np.uint32)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    if _L().oracle_sort_perm(recs.ctypes.data, offs.ctypes.data, n, perm.ctypes.data) != 0:
        raise MemoryError("oracle_sort_perm")
    return perm[:n]


def markdup(recs: np.ndarray, offs: np.ndarray, n: int, header_text: str, compat_nonverbose: bool = False,
            split_chains: int = 0):
    """dup[i] in {0,1,2} (2 = non-primary, untouched) and the number of records flagged.
    split_chains > 1 restates the default split-by-chromosome chains."""
    ids, libs, names = [], [], {}
    for line in header_text.splitlines():
        if line.startswith("@RG\t"):
            f = dict(x.split(":", 1) for x in line.split("\t")[1:] if len(x) >= 3)
            lb = f.get("LB", "") or "Unknown Library"
            names.setdefault(lb, len(names) + 1)
            ids.append(f.get("ID", ""))
            libs.append(names[lb])
    unknown = names.get("Unknown Library", len(names) + 1)
    idbuf = b"".join(i.encode() + b"\0" for i in ids) + b"\0"
    ida = np.frombuffer(idbuf, dtype=np.uint8).copy()
    liba = np.array(libs + [0], dtype=np.int16)
    dup = np.empty(max(n, 1), dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    nd = _L().oracle_markdup_split(recs.ctypes.data, offs.ctypes.data, n, ida.ctypes.data, len(idbuf) - 1,
                                   liba.ctypes.data, len(ids), unknown, 1 if compat_nonverbose else 0, split_chains,
                                   dup.ctypes.data)
    return dup[:n], int(nd)


def realign_scan(cons, cons_off, bases, quals, read_off, pairs):
    """findBestOffset for every (consensus, read) pair, literal restatement -> (best_index, best_score)."""
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 4)
    n = len(pairs)
    bi, bs = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32)
    arrs = [np.ascontiguousarray(a) for a in (cons, np.asarray(cons_off, np.uint64), bases, quals,
                                              np.asarray(read_off, np.uint64))]
    _L().oracle_realign_scan(*[a.ctypes.data for a in arrs], pairs.ctypes.data, n, bi.ctypes.data, bs.ctypes.data)
    return bi[:n], bs[:n]


FILTER_DEFAULTS = dict(has_region=0, ref_id=-1, left_pos=0, right_pos=0, mapq_min=0, min_len=0, max_len=2**31 - 1,
                       trim_total=0, count_limit=2**31 - 1)


def filter_keep(recs: np.ndarray, offs: np.ndarray, n: int, **opts) -> np.ndarray:
    """Filter::runInternal's kept-record mask (algorithms/filter.cpp:205-249), input order."""
    o = dict(FILTER_DEFAULTS, **opts)
    recs = np.ascontiguousarray(recs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs[:n], dtype=np.uint64)
    keep = np.zeros(max(n, 1), dtype=np.uint8)
    _L().oracle_filter(recs.ctypes.data, offs.ctypes.data, n, o["has_region"], o["ref_id"], o["left_pos"],
                       o["right_pos"], o["mapq_min"], o["min_len"], o["max_len"], o["trim_total"], o["count_limit"],
                       keep.ctypes.data)
    return keep[:n].astype(bool)


def parse_region(region: str, refs: list[tuple[str, int]]) -> dict | None:
    """Filter::ParseRegionString (algorithms/filter.cpp:31-137) in Python; None where it fails."""
    if not region:
        return None
    c1 = region.find(":")

    def atoi(t: str) -> int:
        import re
        m = re.match(r"\s*[+-]?\d+", t)
        return int(m.group(0)) if m else 0

    if c1 < 0:
        chrom, start, stop = region, 0, -1
    else:
        chrom = region[:c1]
        dots = region.find("..", c1 + 1)
        if dots < 0:
            start = stop = atoi(region[c1 + 1:])
        else:
            start = atoi(region[c1 + 1:dots])
            if region.find(":", dots + 1) >= 0:
                return None
            stop = atoi(region[dots + 2:])
    ref = -1
    for i, (nm, _) in enumerate(refs):
        if nm == chrom:
            ref = i
    if ref < 0:
        return None
    ln = refs[ref][1]
    if start >= ln or stop > ln:
        return None
    if stop == -1:
        stop = ln
    return dict(has_region=1, ref_id=ref, left_pos=start, right_pos=stop)


def sort_name_perm(recs: np.ndarray, offs: np.ndarray, n: int) -> np.ndarray:
    """Sort::ByName order (util/bamtools/Sort.h:67-90), equal names in input order."""
    recs = np.ascontiguousarray(recs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs[:n], dtype=np.uint64)
    perm = np.zeros(max(n, 1), dtype=np.uint32)
    _L().oracle_sort_name(recs.ctypes.data, offs.ctypes.data, n, perm.ctypes.data)
    return perm[:n]


def _bypos_key(recs: np.ndarray, off: int):
    """Sort::ByPosition (util/bamtools/Sort.h:116-133) down to the flag; refID -1 -> one equivalence class."""
    o = int(off)
    ref = int.from_bytes(recs[o + 4:o + 8].tobytes(), "little", signed=True)
    if ref == -1:
        return (1,)
    pos = int.from_bytes(recs[o + 8:o + 12].tobytes(), "little", signed=True)
    flag = int(recs[o + 18]) | int(recs[o + 19]) << 8
    name = recs[o + 36:o + 36 + int(recs[o + 12]) - 1].tobytes()
    return (0, ref, pos, (flag >> 4) & 1, name, flag)


def multireader_order(recs: np.ndarray, offs_per_file: list[np.ndarray]) -> list[tuple[int, int]]:
    """MultiReader::open/read (util/read_stream_reader.h:24-61,132-153): the files' heads in a
    std::multiset ordered by ByPosition; equivalent heads leave in insertion order (the reference's
    address tie-break among full ties is replaced by insertion order).
    -> (file, record index in file) in output order.  Pure Python: small cases only."""
    import heapq
    heap, seq = [], 0
    for f, offs in enumerate(offs_per_file):
        if len(offs):
            heap.append((_bypos_key(recs, offs[0]), seq, f, 0))
            seq += 1
    heapq.heapify(heap)
    out = []
    while heap:
        _, _, f, i = heapq.heappop(heap)
        out.append((f, i))
        if i + 1 < len(offs_per_file[f]):
            heapq.heappush(heap, (_bypos_key(recs, offs_per_file[f][i + 1]), seq, f, i + 1))
            seq += 1
    return out
