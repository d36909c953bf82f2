"""ctypes binding of libopenge_hip.so (the C ABI declared in include/openge_hip.h).

Python is test/bench plumbing here: the product is the C ABI and the C++ `openge` CLI.  Device
buffers can be torch tensors (``tensor.data_ptr()``) so torch owns HBM allocation and RCCL, and
the library only runs kernels on the context's stream.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["OGE_LIB"]) if os.environ.get("OGE_LIB") else PKG / "libopenge_hip.so"  # OGE_LIB: an A/B build

MAX_REF = 64


class SynthParams(C.Structure):
    """Mirror of oge_synth_params (openge_amd/csrc/synth.h)."""

    _fields_ = [
        ("seed", C.c_uint64), ("n_pairs", C.c_uint64), ("n_ref", C.c_uint32), ("read_len", C.c_uint32),
        ("ins_min", C.c_uint32), ("ins_max", C.c_uint32), ("dup_ppm", C.c_uint32), ("inter_ppm", C.c_uint32),
        ("munmap_ppm", C.c_uint32), ("clip_ppm", C.c_uint32), ("n_rg", C.c_uint32), ("qual_min", C.c_uint32),
        ("qual_max", C.c_uint32), ("shuffle", C.c_uint32),
        ("ref_len", C.c_uint64 * MAX_REF), ("ref_cum", C.c_uint64 * (MAX_REF + 1)),
    ]


class MarkdupOpts(C.Structure):
    """Mirror of oge_markdup_opts (include/openge_hip.h)."""

    _fields_ = [
        ("n_ref", C.c_int32), ("rg_ids", C.c_void_p), ("rg_ids_bytes", C.c_uint64), ("rg_lib", C.c_void_p),
        ("n_rg", C.c_int32), ("unknown_lib", C.c_int16), ("debug_sort_groups", C.c_int16),
        ("compat_nonverbose_index", C.c_int32), ("remove_duplicates", C.c_int32), ("debug_hash_bits", C.c_int32),
        ("split_chains", C.c_int32),
    ]


class FilterOpts(C.Structure):
    """oge_filter_opts (include/openge_hip.h): Filter's settings (algorithms/filter.h:34-47)."""

    _fields_ = [(k, C.c_int32) for k in ("has_region", "ref_id", "left_pos", "right_pos", "mapq_min", "min_len",
                                         "max_len", "trim_total")] + [("count_limit", C.c_uint64)]


class MergesortOpts(C.Structure):
    """Mirror of oge_mergesort_opts (include/openge_hip.h)."""

    _fields_ = [(k, C.c_int32) for k in ("level", "mark_duplicates", "remove_duplicates", "compat_nonverbose_index",
                                         "split_chains", "pad0")] + [("program_line", C.c_char_p)]


def mergesort_opts(**over) -> MergesortOpts:
    o = MergesortOpts()
    lib().oge_mergesort_opts_init(C.byref(o))
    for k, v in over.items():
        setattr(o, k, v)
    return o


class RealignSynthParams(C.Structure):
    """Mirror of oge_realign_synth_params (include/openge_hip.h)."""

    _fields_ = [("seed", C.c_uint64)] + [(k, C.c_uint32) for k in (
        "n_ref", "n_intervals", "spacing", "read_len", "frags_per_interval", "qual_min", "qual_max", "ins_min", "ins_max",
        "err_ppm", "noindel_ppm", "gapped_ppm", "alt_indel_ppm", "dup_ppm", "mapq0_ppm", "clip_ppm", "lower_ppm", "n_ppm",
        "md_ppm", "uq_ppm")]


class RealignOpts(C.Structure):
    """Mirror of oge_realign_opts (include/openge_hip.h)."""

    _fields_ = [("lod_threshold", C.c_double), ("mismatch_threshold", C.c_double)] + [(k, C.c_int32) for k in (
        "max_records_in_memory", "max_isize_for_movement", "max_pos_move_allowed", "max_reads",
        "no_original_alignment_tags", "threads")]


class RealignScanBatch(C.Structure):
    """Mirror of oge_realign_scan_batch (include/openge_hip.h)."""

    _fields_ = [("cons", C.c_void_p), ("cons_bytes", C.c_uint64), ("cons_off", C.c_void_p), ("n_cons", C.c_uint32),
                ("n_reads", C.c_uint32), ("bases", C.c_void_p), ("quals", C.c_void_p), ("read_bytes", C.c_uint64),
                ("read_off", C.c_void_p), ("pairs", C.c_void_p), ("n_pairs", C.c_uint64)]


def realign_synth_params(**over) -> RealignSynthParams:
    """C5-shaped realignment data set parameters (defaults: 50k intervals on 24 contigs)."""
    p = RealignSynthParams()
    lib().oge_realign_synth_defaults(C.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


def synth_realign(p: RealignSynthParams, directory, level: int = 6, threads: int = 8) -> tuple[str, str, str]:
    """Write ref.fa (+ .fai), targets.intervals and reads.bam into `directory`; returns their paths."""
    d = Path(directory)
    fa, iv, bam = str(d / "ref.fa"), str(d / "targets.intervals"), str(d / "reads.bam")
    check(lib().oge_synth_realign(C.byref(p), fa.encode(), iv.encode(), bam.encode(), level, threads))
    return fa, iv, bam


def realign_opts(**over) -> RealignOpts:
    o = RealignOpts()
    lib().oge_realign_opts_init(C.byref(o))
    for k, v in over.items():
        setattr(o, k, v)
    return o


# GRCh38 primary-assembly lengths chr1..22, X, Y (Mbp, rounded) -- relative contig sizes of C2.
GRCH38_MB = [248.96, 242.19, 198.30, 190.21, 181.54, 170.81, 159.35, 145.14, 138.39, 133.80, 135.09, 133.28,
             114.36, 107.04, 101.99, 90.34, 83.26, 80.37, 58.62, 64.44, 46.71, 50.82, 156.04, 57.23]


def synth_params(n_pairs: int, *, preset: str = "c1", seed: int = 1234, **over) -> SynthParams:
    """Synthetic read-set parameters.

    preset "c1": SURVEY §8d C1 -- one 5 Mbp contig, 150 bp pairs, 10% duplicate pairs, 1 RG.
    preset "c2": SURVEY §8d C2 -- 24 contigs with GRCh38 relative lengths scaled to 1.5 Gbp, 8% dup
                 pairs, 1% inter-contig, 0.5% mate-unmapped, 2 read groups / libraries.
    preset "mix": small multi-contig set exercising clipping, inter-contig and unmapped mates.
    """
    p = SynthParams()
    p.seed, p.n_pairs, p.read_len = seed, n_pairs, 150
    p.ins_min, p.ins_max, p.qual_min, p.qual_max, p.shuffle = 250, 450, 2, 40, 1
    if preset == "c1":
        p.n_ref, p.n_rg = 1, 1
        p.ref_len[0] = 5_000_000
        p.dup_ppm, p.inter_ppm, p.munmap_ppm, p.clip_ppm = 100_000, 0, 0, 0
    elif preset == "c2":
        p.n_ref, p.n_rg = 24, 2
        tot = sum(GRCH38_MB)
        for i, mb in enumerate(GRCH38_MB):
            p.ref_len[i] = int(1.5e9 * mb / tot)
        p.dup_ppm, p.inter_ppm, p.munmap_ppm, p.clip_ppm = 80_000, 10_000, 5_000, 50_000
    elif preset == "mix":
        p.n_ref, p.n_rg = 5, 3
        for i in range(5):
            p.ref_len[i] = 20_000 + 7_000 * i
        p.dup_ppm, p.inter_ppm, p.munmap_ppm, p.clip_ppm = 150_000, 40_000, 20_000, 200_000
    else:
        raise ValueError(preset)
    for k, v in over.items():
        if k == "ref_len":
            for i, x in enumerate(v):
                p.ref_len[i] = x
        else:
            setattr(p, k, v)
    return p


class OgeError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libopenge_hip.so (fails loudly if it has not been built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise OgeError(f"{LIB_PATH} is missing: run `python -m openge_amd.build` (no CPU fallback exists)")
    # torch wheels bundle their own libamdhip64.so.7.  Load torch first so the dynamic loader
    # resolves our NEEDED libamdhip64.so.7 to that same, already-loaded runtime: two HIP runtimes
    # in one process make the second one see no GPUs.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(str(LIB_PATH))
    vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int32, C.c_uint32
    sig = {
        "oge_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "oge_ctx_set_stream": (C.c_int, [vp, vp]),
        "oge_ctx_stream": (vp, [vp]),
        "oge_ctx_sync": (C.c_int, [vp]),
        "oge_ctx_destroy": (None, [vp]),
        "oge_last_error": (C.c_char_p, [vp]),
        "oge_ctx_timing": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_double)]),
        "oge_ctx_counter": (C.c_int, [vp, C.c_char_p, C.POINTER(u64)]),
        "oge_mergesort_reserve": (C.c_int, [vp, u64, C.POINTER(vp), C.POINTER(vp), C.POINTER(u64)]),
        "oge_version": (C.c_char_p, []),
        "oge_sort_coord": (C.c_int, [vp, vp, u64, vp, u64, i32, vp]),
        "oge_sort_coord_dev": (C.c_int, [vp, vp, vp, u64, i32, vp]),
        "oge_gather_records_dev": (C.c_int, [vp, vp, vp, vp, u64, vp, vp]),
        "oge_radix_sort_pairs_dev": (C.c_int, [vp, vp, vp, vp, vp, u64, u64, C.POINTER(C.c_int)]),
        "oge_exclusive_scan_dev": (C.c_int, [vp, vp, vp, u64, C.c_int]),
        "oge_markdup": (C.c_int, [vp, vp, u64, vp, u64, vp, vp, C.POINTER(u64)]),
        "oge_markdup_dev": (C.c_int, [vp, vp, vp, u64, vp, vp, C.c_int, C.POINTER(u64)]),
        "oge_sort_markdup_dev": (C.c_int, [vp, vp, vp, u64, vp, vp, vp, vp, C.POINTER(u64)]),
        "oge_synth_finalize": (C.c_int, [vp]),
        "oge_synth_params_size": (u64, []),
        "oge_synth_offsets_host": (C.c_int, [vp, vp, C.c_int]),
        "oge_synth_records_host": (C.c_int, [vp, vp, vp, C.c_int]),
        "oge_synth_header_text": (C.c_int, [vp, vp, u64, C.POINTER(u64)]),
        "oge_synth_offsets_dev": (C.c_int, [vp, vp, vp]),
        "oge_synth_records_dev": (C.c_int, [vp, vp, vp, vp]),
        "oge_bam_read": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(vp)]),
        "oge_bam_free": (None, [vp]),
        "oge_bam_count": (u64, [vp]),
        "oge_bam_records": (vp, [vp, C.POINTER(u64)]),
        "oge_bam_offsets": (vp, [vp]),
        "oge_bam_n_ref": (i32, [vp]),
        "oge_bam_header_text": (C.c_int, [vp, vp, u64, C.POINTER(u64)]),
        "oge_bam_markdup_opts": (C.c_int, [vp, vp, C.POINTER(vp), C.POINTER(vp)]),
        "oge_bam_write": (C.c_int, [C.c_char_p, C.c_char_p, u64, C.c_int, vp, vp, u64, vp, vp, C.c_int, C.c_int]),
        "oge_realign_scan": (C.c_int, [vp, vp, vp, vp]),
        "oge_sort_markdup_chunked": (C.c_int, [vp, vp, vp, u64, i32, vp, u64, vp, vp, C.POINTER(u64), C.POINTER(u64),
                                               C.POINTER(u64)]),
        "oge_mem_info": (C.c_int, [vp, C.POINTER(u64), C.POINTER(u64)]),
        "oge_device_count": (C.c_int, []),
        "oge_comm_unique_id_bytes": (u64, []),
        "oge_comm_unique_id": (C.c_int, [vp, u64]),
        "oge_comm_init_rank": (C.c_int, [vp, C.c_int, C.c_int, vp, C.POINTER(vp)]),
        "oge_comm_init_rank_mode": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_char_p, C.POINTER(vp)]),
        "oge_comm_stats_json": (C.c_int64, [vp, C.c_char_p, u64]),
        "oge_comm_init": (C.c_int, [vp, C.c_int, vp]),
        "oge_comm_destroy": (None, [vp]),
        "oge_comm_rank": (C.c_int, [vp]),
        "oge_comm_size": (C.c_int, [vp]),
        "oge_comm_transport": (C.c_char_p, [vp]),
        "oge_mergesort_bgzf_host": (C.c_int, [vp, vp, u64, vp, vp, u64, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]),
        "oge_mergesort_bgzf_dist": (C.c_int, [vp, vp, u64, vp, C.POINTER(vp), C.POINTER(u64), C.POINTER(u64),
                                              C.POINTER(u64)]),
        "oge_sort_markdup_dist": (C.c_int, [vp, vp, vp, u64, i32, C.c_int, vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(u64),
                                            C.POINTER(u64)]),
        "oge_mergesort_bgzf_shard": (C.c_int, [vp, vp, u64, u64, vp, C.POINTER(vp), C.POINTER(u64), C.POINTER(u64),
                                               C.POINTER(u64)]),
        "oge_bgzf_decode_shard": (C.c_int, [vp, vp, u64, u64, C.POINTER(vp), C.POINTER(vp), C.POINTER(u64), vp, u64,
                                            C.POINTER(u64)]),
        "oge_synth_offsets_range_dev": (C.c_int, [vp, vp, u64, u64, vp]),
        "oge_synth_records_range_dev": (C.c_int, [vp, vp, u64, u64, vp, vp]),
        "oge_dev_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "oge_dev_free": (C.c_int, [vp, vp]),
        "oge_memcpy": (C.c_int, [vp, vp, vp, u64, C.c_int]),
        "oge_host_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "oge_ctx_set_pool": (C.c_int, [vp, C.c_int]),
        "oge_host_free": (C.c_int, [vp, vp]),
        "oge_realign_opts_init": (None, [vp]),
        "oge_localrealign": (C.c_int, [vp, C.c_char_p, u64, vp, vp, u64, C.c_char_p, C.c_char_p, vp, C.POINTER(vp)]),
        "oge_localrealign_multi": (C.c_int, [vp, C.c_int, C.c_char_p, u64, vp, vp, u64, C.c_char_p, C.c_char_p, vp,
                                             C.POINTER(vp)]),
        "oge_realign_result_count": (u64, [vp]),
        "oge_realign_result_records": (vp, [vp, C.POINTER(u64)]),
        "oge_realign_result_offsets": (vp, [vp]),
        "oge_realign_result_stats": (C.c_char_p, [vp]),
        "oge_realign_result_free": (None, [vp]),
        "oge_realign_synth_defaults": (None, [vp]),
        "oge_synth_realign": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int]),
        "oge_bgzf_bound": (u64, [u64]),
        "oge_bgzf_deflate_dev": (C.c_int, [vp, vp, u64, C.c_int, vp, u64, C.POINTER(u64)]),
        "oge_bgzf_deflate": (C.c_int, [vp, vp, u64, C.c_int, vp, u64, C.POINTER(u64)]),
        "oge_fix_bins_dev": (C.c_int, [vp, vp, vp, u64]),
        "oge_bgzf_index": (C.c_int, [vp, u64, vp, vp, vp, vp, u64, C.POINTER(u64)]),
        "oge_bgzf_inflate_dev": (C.c_int, [vp, vp, u64, vp, vp, vp, vp, u64, vp]),
        "oge_bgzf_inflate": (C.c_int, [vp, vp, u64, vp, u64, C.POINTER(u64)]),
        "oge_bam_record_offsets_dev": (C.c_int, [vp, vp, u64, u64, i32, vp, u64, C.POINTER(u64)]),
        "oge_drop_flagged_dev": (C.c_int, [vp, vp, vp, u64, C.c_uint16, vp, vp, C.POINTER(u64)]),
        "oge_filter_opts_init": (None, [vp]),
        "oge_parse_region": (C.c_int, [C.c_char_p, C.c_char_p, i32, vp, vp]),
        "oge_filter_records_dev": (C.c_int, [vp, vp, vp, u64, vp, vp, vp, C.POINTER(u64)]),
        "oge_sort_name_dev": (C.c_int, [vp, vp, vp, u64, vp]),
        "oge_sort_name": (C.c_int, [vp, vp, u64, vp, u64, vp]),
        "oge_bgzf_index_dev": (C.c_int, [vp, vp, u64, vp, vp, vp, vp, u64, C.POINTER(u64)]),
        "oge_mergesort_opts_init": (None, [vp]),
        "oge_mergesort_bgzf_dev": (C.c_int, [vp, vp, u64, vp, C.POINTER(vp), C.POINTER(u64), C.POINTER(u64),
                                             C.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None:
            continue
        f.restype, f.argtypes = res, args
    _lib = L
    return L


def filter_opts(**over) -> FilterOpts:
    """Filter::Filter() defaults (algorithms/filter.cpp:185-194) with overrides."""
    o = FilterOpts()
    lib().oge_filter_opts_init(C.byref(o))
    for k, v in over.items():
        setattr(o, k, v)
    return o


def parse_region(region: str, refs: list[tuple[str, int]], opts: FilterOpts | None = None) -> FilterOpts:
    """Filter::ParseRegionString through the C ABI; raises OgeError with the reference's message."""
    o = opts if opts is not None else filter_opts()
    names = b"".join(nm.encode() + b"\0" for nm, _ in refs)
    lens = np.array([ln for _, ln in refs] or [0], dtype=np.int64)
    check(lib().oge_parse_region(region.encode(), names, len(refs), _ptr(lens), C.byref(o)))
    return o


def exported_symbols() -> list[str]:
    """Symbols include/openge_hip.h declares (parsed from the header)."""
    import re

    text = (PKG.parent / "include" / "openge_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(oge_[a-z0-9_]+)\s*\(", text)))


def check(rc: int, ctx=None) -> None:
    if rc != 0:
        msg = lib().oge_last_error(ctx)
        raise OgeError(f"openge_hip error {rc}: {msg.decode() if msg else ''}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ------------------------------------------------------------------------- synthetic data (host)
def synth_host(p: SynthParams, threads: int = 0) -> tuple[np.ndarray, np.ndarray, str]:
    """Generate the records on the host: (recs u8, offs u64[n+1], header text)."""
    L = lib()
    check(L.oge_synth_finalize(C.byref(p)))
    n = 2 * p.n_pairs
    offs = np.empty(n + 1, dtype=np.uint64)
    check(L.oge_synth_offsets_host(C.byref(p), _ptr(offs), threads))
    recs = np.empty(int(offs[-1]) + 16, dtype=np.uint8)
    recs[-16:] = 0
    check(L.oge_synth_records_host(C.byref(p), _ptr(offs), _ptr(recs), threads))
    ln = C.c_uint64()
    check(L.oge_synth_header_text(C.byref(p), None, 0, C.byref(ln)))
    buf = C.create_string_buffer(ln.value + 1)
    check(L.oge_synth_header_text(C.byref(p), buf, ln.value + 1, None))
    return recs, offs, buf.value.decode()


# ------------------------------------------------------------------------- BAM files
class Bam:
    """A BAM file decoded into one record arena (records in file order)."""

    def __init__(self, path: str | os.PathLike, threads: int = 8):
        L = lib()
        h = C.c_void_p()
        check(L.oge_bam_read(str(path).encode(), threads, C.byref(h)))
        self._h = h
        n = L.oge_bam_count(h)
        nb = C.c_uint64()
        rp = L.oge_bam_records(h, C.byref(nb))
        self.n = int(n)
        self.recs = np.ctypeslib.as_array((C.c_uint8 * nb.value).from_address(rp)) if nb.value else np.zeros(0, np.uint8)
        op = L.oge_bam_offsets(h)
        self.offs = np.ctypeslib.as_array((C.c_uint64 * self.n).from_address(op)) if self.n else np.zeros(0, np.uint64)
        self.n_ref = int(L.oge_bam_n_ref(h))
        ln = C.c_uint64()
        check(L.oge_bam_header_text(h, None, 0, C.byref(ln)))
        buf = C.create_string_buffer(ln.value + 1)
        check(L.oge_bam_header_text(h, buf, ln.value + 1, None))
        self.header_text = buf.value.decode()

    def markdup_opts(self) -> tuple[MarkdupOpts, tuple]:
        o = MarkdupOpts()
        ids, libs = C.c_void_p(), C.c_void_p()
        check(lib().oge_bam_markdup_opts(self._h, C.byref(o), C.byref(ids), C.byref(libs)))
        return o, (ids, libs)

    def __del__(self):
        try:
            lib().oge_bam_free(self._h)
        except Exception:
            pass


def markdup_opts_from_header(header_text: str, n_ref: int, compat_nonverbose: bool = False,
                             split_chains: int = 0) -> tuple[MarkdupOpts, tuple]:
    """RG -> library table as MarkDuplicates::getLibraryName resolves it (mark_duplicates.cpp:301-318)."""
    ids, libs, names = [], [], {}
    for line in header_text.splitlines():
        if not line.startswith("@RG\t"):
            continue
        f = dict(x.split(":", 1) for x in line.split("\t")[1:] if len(x) >= 3)
        lb = f.get("LB", "") or "Unknown Library"
        names.setdefault(lb, len(names) + 1)
        ids.append(f.get("ID", ""))
        libs.append(names[lb])
    unknown = names.get("Unknown Library", len(names) + 1)
    idbuf = b"".join(i.encode() + b"\0" for i in ids)
    ida = np.frombuffer(idbuf + b"\0", dtype=np.uint8).copy()
    liba = np.array(libs + [0], dtype=np.int16)
    o = MarkdupOpts()
    o.n_ref, o.rg_ids, o.rg_ids_bytes = n_ref, _ptr(ida), len(idbuf)
    o.rg_lib, o.n_rg, o.unknown_lib = _ptr(liba), len(ids), unknown
    o.compat_nonverbose_index = 1 if compat_nonverbose else 0
    o.split_chains = split_chains
    return o, (ida, liba)


def write_bam(path, header_text: str, recs: np.ndarray, offs: np.ndarray, n: int, order=None, flags=None,
              sort_order: int = -1, level: int = 6, threads: int = 8) -> None:
    L = lib()
    hb = header_text.encode()
    check(L.oge_bam_write(str(path).encode(), hb, len(hb), sort_order, _ptr(recs), _ptr(offs), n,
                          _ptr(order) if order is not None else None, _ptr(flags) if flags is not None else None,
                          level, threads))


# ------------------------------------------------------------------------- device context
class _RealignResult:
    """Owns an oge_realign_result; the record/offset arrays returned by Context.localrealign are
    zero-copy views that keep it alive."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h:
            lib().oge_realign_result_free(self.h)
            self.h = None


class Context:
    """A HIP device context (one per process/GPU)."""

    def __init__(self, device: int = 0, stream: int | None = None):
        L = lib()
        h = C.c_void_p()
        check(L.oge_ctx_create(device, C.byref(h)))
        self.h = h
        if stream:
            check(L.oge_ctx_set_stream(h, C.c_void_p(stream)), h)

    def close(self):
        if self.h:
            lib().oge_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return lib().oge_ctx_stream(self.h) or 0

    def sync(self):
        check(lib().oge_ctx_sync(self.h), self.h)

    def counter(self, name: str) -> int | None:
        """A work count of the last pipeline call (oge_ctx_counter), None when it recorded none."""
        v = C.c_uint64()
        return v.value if lib().oge_ctx_counter(self.h, name.encode(), C.byref(v)) == 0 else None

    def timing(self, stage: str) -> float:
        ms = C.c_double()
        check(lib().oge_ctx_timing(self.h, stage.encode(), C.byref(ms)), self.h)
        return ms.value

    # host-buffer entry points
    def sort_coord(self, recs: np.ndarray, offs: np.ndarray, n: int, n_ref: int) -> np.ndarray:
        perm = np.empty(max(n, 1), dtype=np.uint32)
        check(lib().oge_sort_coord(self.h, _ptr(recs), recs.nbytes, _ptr(offs), n, n_ref, _ptr(perm)), self.h)
        return perm[:n]

    def markdup(self, recs: np.ndarray, offs: np.ndarray, n: int, opts: MarkdupOpts) -> tuple[np.ndarray, int]:
        dup = np.empty(max(n, 1), dtype=np.uint8)
        nd = C.c_uint64()
        check(lib().oge_markdup(self.h, _ptr(recs), recs.nbytes, _ptr(offs), n, C.byref(opts), _ptr(dup),
                                C.byref(nd)), self.h)
        return dup[:n], nd.value

    # device entry points (pointers are ints, e.g. torch tensor .data_ptr())
    def sort_coord_dev(self, d_recs: int, d_off: int, n: int, n_ref: int, d_perm: int) -> None:
        check(lib().oge_sort_coord_dev(self.h, d_recs, d_off, n, n_ref, d_perm), self.h)

    def gather_records_dev(self, d_recs, d_off, d_perm, n, d_out, d_out_off) -> None:
        check(lib().oge_gather_records_dev(self.h, d_recs, d_off, d_perm, n, d_out, d_out_off), self.h)

    def radix_sort_pairs_dev(self, d_keys, d_vals, d_ktmp, d_vtmp, n, bit_mask) -> bool:
        """Stable radix sort of device (u64 key, u32 value) pairs on the bits of bit_mask; returns True
        when the result sits in the tmp buffers."""
        t = C.c_int()
        check(lib().oge_radix_sort_pairs_dev(self.h, d_keys, d_vals, d_ktmp, d_vtmp, n, bit_mask, C.byref(t)), self.h)
        return bool(t.value)

    def exclusive_scan_dev(self, d_in, d_out, n: int, elem_bytes: int) -> None:
        """oge_exclusive_scan_dev: exclusive prefix sum of n u32 (elem_bytes 4) or u64 (8) device elements."""
        check(lib().oge_exclusive_scan_dev(self.h, d_in, d_out, n, elem_bytes), self.h)

    def bgzf_deflate(self, data: bytes | np.ndarray, level: int = 6) -> bytes:
        """BGZF-compress host bytes on the device (no EOF marker)."""
        a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, np.uint8)
        cap = int(lib().oge_bgzf_bound(len(a)))
        out = np.empty(max(cap, 1), dtype=np.uint8)
        got = C.c_uint64()
        check(lib().oge_bgzf_deflate(self.h, _ptr(a), len(a), level, _ptr(out), cap, C.byref(got)), self.h)
        return out[:got.value].tobytes()

    def bgzf_deflate_dev(self, d_src, n: int, level: int, d_dst, dst_cap: int) -> int:
        got = C.c_uint64()
        check(lib().oge_bgzf_deflate_dev(self.h, d_src, n, level, d_dst, dst_cap, C.byref(got)), self.h)
        return got.value

    def bgzf_inflate(self, z: bytes, out_cap: int | None = None) -> bytes:
        """Decompress a BGZF stream on the device (host buffers in and out)."""
        a = np.frombuffer(z, dtype=np.uint8)
        nb = C.c_uint64()
        lib().oge_bgzf_index(_ptr(a), len(a), None, None, None, None, 0, C.byref(nb))
        uo = np.zeros(nb.value + 1, dtype=np.uint64)
        if nb.value:
            check(lib().oge_bgzf_index(_ptr(a), len(a), None, None, _ptr(uo), None, nb.value, C.byref(nb)))
        cap = int(uo[-1]) if out_cap is None else out_cap
        out = np.empty(max(cap, 1), dtype=np.uint8)
        got = C.c_uint64()
        check(lib().oge_bgzf_inflate(self.h, _ptr(a), len(a), _ptr(out), cap, C.byref(got)), self.h)
        return out[:got.value].tobytes()

    def bgzf_index_dev(self, d_z, zbytes: int, d_d0=None, d_d1=None, d_uoff=None, d_crc=None, cap: int = 0) -> int:
        nb = C.c_uint64()
        check(lib().oge_bgzf_index_dev(self.h, d_z, zbytes, d_d0, d_d1, d_uoff, d_crc, cap, C.byref(nb)), self.h)
        return nb.value

    def mergesort_bgzf_dev(self, d_z, zbytes: int, opts: "MergesortOpts") -> tuple[int, int, int, int]:
        """The whole mergesort [-M] chain on a BAM file resident in HBM -> (d_out, out_bytes, n_reads,
        n_dup); d_out (device pointer) is valid until the next call on this context."""
        d = C.c_void_p()
        ob, nr, nd = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().oge_mergesort_bgzf_dev(self.h, d_z, zbytes, C.byref(opts), C.byref(d), C.byref(ob), C.byref(nr),
                                           C.byref(nd)), self.h)
        return d.value or 0, ob.value, nr.value, nd.value

    def mergesort_reserve(self, total: int) -> tuple[int, int, int]:
        """Allocate the chain's two record arenas for streams of up to `total` decompressed bytes ->
        (x, y, cap): device pointers the caller may stage data in between chain calls."""
        x, y, cap = C.c_void_p(), C.c_void_p(), C.c_uint64()
        check(lib().oge_mergesort_reserve(self.h, total, C.byref(x), C.byref(y), C.byref(cap)), self.h)
        return x.value, y.value, cap.value

    def mergesort_bgzf_host(self, h_z: int, zbytes: int, opts: "MergesortOpts", h_out: int, out_cap: int) -> tuple[int, int, int]:
        """The chain on a BAM file in host memory (page-locked for full speed), PCIe overlapped with the
        codec -> (out_bytes written to h_out, n_reads, n_dup)."""
        ob, nr, nd = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().oge_mergesort_bgzf_host(self.h, h_z, zbytes, C.byref(opts), h_out, out_cap, C.byref(ob), C.byref(nr),
                                            C.byref(nd)), self.h)
        return ob.value, nr.value, nd.value

    def record_offsets_dev(self, d_stream, rec_base: int, end: int, n_ref: int, d_off=None, cap: int = 0) -> int:
        n = C.c_uint64()
        check(lib().oge_bam_record_offsets_dev(self.h, d_stream, rec_base, end, n_ref, d_off, cap, C.byref(n)), self.h)
        return n.value

    def fix_bins_dev(self, d_recs, d_off, n: int) -> None:
        check(lib().oge_fix_bins_dev(self.h, d_recs, d_off, n), self.h)

    def drop_flagged_dev(self, d_recs, d_off, n: int, flag_mask: int, d_out, d_out_off) -> int:
        m = C.c_uint64()
        check(lib().oge_drop_flagged_dev(self.h, d_recs, d_off, n, flag_mask, d_out, d_out_off, C.byref(m)), self.h)
        return m.value

    def filter_records_dev(self, d_recs, d_off, n: int, opts: "FilterOpts", d_out, d_out_off) -> int:
        m = C.c_uint64()
        check(lib().oge_filter_records_dev(self.h, d_recs, d_off, n, C.byref(opts), d_out, d_out_off, C.byref(m)),
              self.h)
        return m.value

    def sort_name(self, recs: np.ndarray, offs: np.ndarray, n: int) -> np.ndarray:
        perm = np.zeros(max(n, 1), dtype=np.uint32)
        check(lib().oge_sort_name(self.h, _ptr(recs), recs.nbytes, _ptr(offs), n, _ptr(perm)), self.h)
        return perm[:n]

    def sort_name_dev(self, d_recs, d_off, n: int, d_perm) -> None:
        check(lib().oge_sort_name_dev(self.h, d_recs, d_off, n, d_perm), self.h)

    def markdup_dev(self, d_recs, d_off, n, opts: MarkdupOpts, d_dup, apply: bool = True) -> int:
        nd = C.c_uint64()
        check(lib().oge_markdup_dev(self.h, d_recs, d_off, n, C.byref(opts), d_dup, 1 if apply else 0, C.byref(nd)),
              self.h)
        return nd.value

    def sort_markdup_dev(self, d_recs, d_off, n, opts: MarkdupOpts, d_perm, d_out, d_out_off) -> int:
        nd = C.c_uint64()
        check(lib().oge_sort_markdup_dev(self.h, d_recs, d_off, n, C.byref(opts), d_perm, d_out, d_out_off,
                                         C.byref(nd)), self.h)
        return nd.value

    def realign_scan(self, cons: np.ndarray, cons_off: np.ndarray, bases: np.ndarray, quals: np.ndarray,
                     read_off: np.ndarray, pairs: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """findBestOffset for every (consensus, read) pair -> (best_index, best_score)."""
        pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 4)
        n = len(pairs)
        b = RealignScanBatch(_ptr(cons), cons.nbytes, _ptr(cons_off), len(cons_off) - 1, len(read_off) - 1, _ptr(bases),
                             _ptr(quals), bases.nbytes, _ptr(read_off), _ptr(pairs), n)
        bi, bs = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32)
        check(lib().oge_realign_scan(self.h, C.byref(b), _ptr(bi), _ptr(bs)), self.h)
        return bi[:n], bs[:n]

    def localrealign(self, header_text: str, recs: np.ndarray, offs: np.ndarray, n: int, fasta: str, intervals: str,
                     opts: RealignOpts | None = None, more: "list[Context] | None" = None) -> tuple[np.ndarray, np.ndarray, dict]:
        """LocalRealignment over coordinate-sorted records -> (out recs, out offsets[n+1], stats).
        The arrays are read-only-by-convention views of the library's result buffer (no copy).  more: further
        contexts -- the device work is then spread over [self] + more by interval ranges
        (oge_localrealign_multi)."""
        import json
        L = lib()
        hb = header_text.encode()
        res = C.c_void_p()
        if more:
            hs = (C.c_void_p * (1 + len(more)))(self.h.value, *[c.h.value for c in more])
            check(L.oge_localrealign_multi(hs, len(hs), hb, len(hb), _ptr(recs), _ptr(offs), n, fasta.encode(),
                                           intervals.encode(), C.byref(opts) if opts is not None else None, C.byref(res)),
                  self.h)
        else:
            check(L.oge_localrealign(self.h, hb, len(hb), _ptr(recs), _ptr(offs), n, fasta.encode(), intervals.encode(),
                                     C.byref(opts) if opts is not None else None, C.byref(res)), self.h)
        holder = _RealignResult(res)  # frees the result when the last view goes away
        cnt = int(L.oge_realign_result_count(res))
        nb = C.c_uint64()
        rp = L.oge_realign_result_records(res, C.byref(nb))
        stats = json.loads(L.oge_realign_result_stats(res).decode())
        if nb.value:
            ra = (C.c_uint8 * nb.value).from_address(rp)
            ra._holder = holder
            out = np.ctypeslib.as_array(ra)
        else:
            out = np.zeros(0, np.uint8)
        oa = (C.c_uint64 * (cnt + 1)).from_address(L.oge_realign_result_offsets(res))
        oa._holder = holder
        oo = np.ctypeslib.as_array(oa)
        return out, oo, stats

    def synth_range_dev(self, p: SynthParams, slot0: int, nslots: int, d_offs: int, d_out: int | None) -> None:
        """Slots [slot0, slot0 + nslots) of the data set (one rank's input shard)."""
        L = lib()
        check(L.oge_synth_finalize(C.byref(p)))
        if d_offs and not d_out:
            check(L.oge_synth_offsets_range_dev(self.h, C.byref(p), slot0, nslots, d_offs), self.h)
        if d_out:
            check(L.oge_synth_records_range_dev(self.h, C.byref(p), slot0, nslots, d_offs, d_out), self.h)

    def synth_dev(self, p: SynthParams, d_offs: int, d_out: int | None) -> None:
        L = lib()
        check(L.oge_synth_finalize(C.byref(p)))
        if d_offs:
            check(L.oge_synth_offsets_dev(self.h, C.byref(p), d_offs), self.h)
        if d_out:
            check(L.oge_synth_records_dev(self.h, C.byref(p), d_offs, d_out), self.h)


# ------------------------------------------------------------------------- multi-GPU (oge_comm)
class Comm:
    """One rank of a multi-GPU communicator (oge_comm_*): RCCL over xGMI, or the in-process
    transport when several contexts share a GPU.  Every method is collective."""

    def __init__(self, h: C.c_void_p, ctx: "Context"):
        self.h, self.ctx = h, ctx

    @property
    def rank(self) -> int:
        return lib().oge_comm_rank(self.h)

    @property
    def size(self) -> int:
        return lib().oge_comm_size(self.h)

    @property
    def transport(self) -> str:
        return lib().oge_comm_transport(self.h).decode()

    def sort_markdup_dist(self, d_recs: int, d_off: int, n: int, n_ref: int, opts: "MarkdupOpts | None", sort: bool = True):
        """This rank's shard -> its slice of the sorted (and, with opts, duplicate-marked) output, or
        with sort=False its shard marked in place order (dedup): (d_out pointer, d_out_off pointer,
        records in the slice, duplicates over all ranks).  The pointers are owned by the rank's
        context (valid until its next call)."""
        d, do = C.c_void_p(), C.c_void_p()
        no, nd = C.c_uint64(), C.c_uint64()
        check(lib().oge_sort_markdup_dist(self.h, d_recs, d_off, n, n_ref, 1 if sort else 0,
                                          C.byref(opts) if opts is not None else None,
                                          C.byref(d), C.byref(do), C.byref(no), C.byref(nd)), self.ctx.h)
        return d.value or 0, do.value or 0, no.value, nd.value

    def mergesort_bgzf_dist(self, d_z: int, zbytes: int, opts: "MergesortOpts"):
        """Rank's input BAM file in HBM -> (its slice of the output file: device pointer, bytes; records
        written by all ranks; duplicates flagged by all ranks)."""
        d = C.c_void_p()
        ob, nr, nd = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().oge_mergesort_bgzf_dist(self.h, d_z, zbytes, C.byref(opts), C.byref(d), C.byref(ob), C.byref(nr),
                                            C.byref(nd)), self.ctx.h)
        return d.value or 0, ob.value, nr.value, nd.value

    def mergesort_bgzf_shard(self, d_z: int, zbytes: int, own_bytes: int, opts: "MergesortOpts"):
        """ONE input file over the ranks: this rank holds the file's bytes from a_g on (a_g = the earlier
        ranks' own_bytes summed) and decodes the blocks that start in its own_bytes -> (its slice of the
        output file: device pointer, bytes; records written by all ranks; duplicates flagged by all)."""
        d = C.c_void_p()
        ob, nr, nd = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().oge_mergesort_bgzf_shard(self.h, d_z, zbytes, own_bytes, C.byref(opts), C.byref(d), C.byref(ob),
                                             C.byref(nr), C.byref(nd)), self.ctx.h)
        return d.value or 0, ob.value, nr.value, nd.value

    def decode_shard(self, d_z: int, zbytes: int, own_bytes: int, hdr_cap: int = 1 << 22):
        """oge_bgzf_decode_shard: this rank's records of one sharded BGZF file -> (d_recs pointer, d_off
        pointer (n + 1 offsets), n, raw BAM header bytes)."""
        dr, do = C.c_void_p(), C.c_void_p()
        n, hl = C.c_uint64(), C.c_uint64()
        hb = C.create_string_buffer(hdr_cap)
        check(lib().oge_bgzf_decode_shard(self.h, d_z, zbytes, own_bytes, C.byref(dr), C.byref(do), C.byref(n), hb, hdr_cap,
                                          C.byref(hl)), self.ctx.h)
        return dr.value or 0, do.value or 0, n.value, hb.raw[:hl.value]

    def exchange_stats(self) -> list:
        """This rank's per-exchange record of its last sort_markdup_dist / mergesort_bgzf_dist call:
        [{tag, calls, bytes_sent, bytes_recv, bytes_self, ms}] (bytes to / from other ranks, kept here;
        host wall time of the collectives, waiting for peers included)."""
        import json
        n = lib().oge_comm_stats_json(self.h, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().oge_comm_stats_json(self.h, buf, n + 1)
        return json.loads(buf.value.decode())

    def close(self):
        if self.h:
            lib().oge_comm_destroy(self.h)
            self.h = None


BGZF_MAX_BLOCK = 65536  # BSIZE - 1 is a u16 (SAM spec 4.1): no block is longer


def shard_ranges(file_bytes: int, world: int) -> list[tuple[int, int, int]]:
    """Byte ranges of ONE BGZF file for `world` ranks (oge_bgzf_decode_shard / Comm.mergesort_bgzf_shard):
    (a_g, own_g, end_g) -- rank g decodes the blocks that start in [a_g, a_g + own_g) and holds the file's
    bytes [a_g, end_g) (its last block may run up to 64 KiB past its range; the last rank's ends at the
    end of the file)."""
    out = []
    for g in range(world):
        a, b = file_bytes * g // world, file_bytes * (g + 1) // world
        out.append((a, b - a, min(file_bytes, b + BGZF_MAX_BLOCK)))
    return out


def comm_init(ctxs: list["Context"]) -> list[Comm]:
    """One process, one rank per context (call each rank's methods from its own thread)."""
    n = len(ctxs)
    arr = (C.c_void_p * n)(*[c.h for c in ctxs])
    out = (C.c_void_p * n)()
    check(lib().oge_comm_init(arr, n, out))
    return [Comm(C.c_void_p(out[i]), ctxs[i]) for i in range(n)]


def comm_unique_id() -> bytes:
    nb = lib().oge_comm_unique_id_bytes()
    buf = C.create_string_buffer(nb)
    check(lib().oge_comm_unique_id(buf, nb))
    return buf.raw


def comm_init_rank(ctx: "Context", nranks: int, rank: int, uid: bytes, mode: str | None = None) -> Comm:
    """One process per GPU (RCCL): uid from comm_unique_id() on one rank, shared by the caller.  mode:
    "auto" | "rccl" | "host" (None = OGE_COMM)."""
    h = C.c_void_p()
    if mode is None:
        check(lib().oge_comm_init_rank(ctx.h, nranks, rank, uid, C.byref(h)), ctx.h)
    else:
        check(lib().oge_comm_init_rank_mode(ctx.h, nranks, rank, uid, mode.encode(), C.byref(h)), ctx.h)
    return Comm(h, ctx)


RANGE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)


def sort_markdup_chunked(ctx: "Context", recs: np.ndarray, offs: np.ndarray, n: int, n_ref: int,
                         opts: "MarkdupOpts | None", chunk_bytes: int = 0):
    """Out-of-core mergesort [-M] of host records (oge_sort_markdup_chunked).  `recs` is used as the
    spill space (it holds the sorted runs afterwards).  Returns (output record stream bytes,
    duplicates, runs, ranges)."""
    parts = []

    def on_range(user, d_recs, d_off, m):
        try:
            oo = np.empty(m + 1, np.uint64)
            check(lib().oge_memcpy(ctx.h, oo.ctypes.data, d_off, 8 * (m + 1), 2), ctx.h)
            b = np.empty(int(oo[m] - oo[0]), np.uint8)
            if b.size:
                check(lib().oge_memcpy(ctx.h, b.ctypes.data, d_recs + int(oo[0]), b.size, 2), ctx.h)
            parts.append(b.tobytes())
            return 0
        except Exception:  # noqa: BLE001
            return -1

    cb = RANGE_CB(on_range)
    nd, nr, ng = C.c_uint64(), C.c_uint64(), C.c_uint64()
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    check(lib().oge_sort_markdup_chunked(ctx.h, recs.ctypes.data, offs.ctypes.data, n, n_ref,
                                         C.byref(opts) if opts is not None else None, chunk_bytes, cb, None,
                                         C.byref(nd), C.byref(nr), C.byref(ng)), ctx.h)
    return b"".join(parts), nd.value, nr.value, ng.value
