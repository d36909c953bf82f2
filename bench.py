#!/usr/bin/env python
"""bench.py -- OpenGE post-alignment hot path on MI355X.

Metric (BASELINE.json): Mreads/s of sort+dedup (`openge mergesort -M --nosplit` semantics: coordinate
sort, Picard MarkDuplicates with -v semantics, FLAG 0x400 applied, bins recomputed, header
regenerated).  Workload at N=1: configs[1]+[2] -- a 300M-read (150M pairs) 30x WGS-shaped synthetic
read set (SURVEY.md §8d C2 generator, seed 1234).

value (SURVEY §8d timing rule, BAM in -> BAM out, BGZF at -c 6): one step is the whole
`mergesort -M` chain over a BGZF BAM file resident in HBM when the timed region starts
(oge_mergesort_bgzf_dev: framing index, inflate + CRC-32, record walk, sort + dedup, header,
GPU deflate, EOF block; the output BAM file ends in HBM).  The input file is made once before the
timed region by the library's own GPU deflate from the device generator.  The GPU deflate is a greedy
single-candidate parse (DEFLATE_SEARCH below), not zlib's level-6 lazy hash-chain search: its output is
~3% larger; config.deflate carries both ratios.

Also on the same JSON line:
  kernel_step   -- the sort+dedup device pipeline alone over records already decoded in HBM
                   (oge_sort_markdup_dev), the round-1 headline, with its stage times
  pcie_inclusive-- the same chain from a BAM file in page-locked host memory to one in host memory
                   (oge_mergesort_bgzf_host: upload overlapped with the framing index and inflate, the
                   download with the deflate), second call timed, the first reported (never `value`)
  roofline      -- the e2e step's dominant kernel: algorithmic bytes per launch / its HIP-event time
                   (events on the context stream), traffic from the committed rocprofv3 PMC summary
  cpu_baseline  -- the REFERENCE itself (oracle/_ref/ref_driver: OpenGE's own ReadSorter +
                   MarkDuplicates + BamSerializer modules compiled from its sources here, the
                   mergesort -M --nosplit chain with -v) timed on this box's host cores on a bounded
                   BAM-in/BAM-out sample of the same generator
  realign       -- configs[4]: openge localrealign on the C5 set (50k indel intervals)

Multi-GPU (torchrun, one rank per GPU): ONE 300M-read input BAM file split by byte range across the N
ranks (strong scaling); oge_mergesort_bgzf_shard has every rank inflate only the BGZF blocks of its
range (block and record boundaries joined with the neighbouring ranks), range-splits the ByPosition
keys with sampled splitters, exchanges the records with an all-to-all (RCCL over xGMI between GPUs; the
host-staged transport when ranks share a GPU), sorts each rank's slice and marks duplicates exactly
with hash-routed mate-join / pair-group exchanges.  value = reads / max-over-ranks wall
time.  --dump-dir writes every rank's output slice (tests/test_gpu_multiproc.py concatenates them).
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mreads/sec sort+dedup (and realign intervals/sec), 1/2/4/8 MI355X"
BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
# int32 VALU lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md: SIMD-32, a wave64
# VALU instruction issues over 2 cycles)
VALU_INT32_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
KERNEL_STAGES = ["input_pass", "sort_radix", "sort_ties", "meta_gather", "md_matejoin", "md_pairs", "md_frags",
                 "md_apply", "gather_offsets", "gather_records"]
DEDUP_STAGES = ["md_readends", "md_matejoin", "md_pairs", "md_frags", "md_apply"]
SUB_STAGES = ["md_pair_win", "md_frag_win", "md_pair_ovf", "md_frag_ovf"]  # nested in md_pairs / md_frags: which group path ran
E2E_STAGES = ["bgzf_index", "bgzf_inflate", "rec_walk"] + KERNEL_STAGES + ["bgzf_deflate"]
INFL_PHASES = ["infl_prep", "infl_huff", "infl_lz"]  # nested in bgzf_inflate: its two kernels' own times


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=150_000_000, help="read pairs (default 150M = 300M reads)")
    ap.add_argument("--seed", type=int, default=1234, help="C2 generator seed")
    ap.add_argument("--dump-dir", default=None, help="multi-GPU: write each rank's output slice here (tests)")
    ap.add_argument("--level", type=int, default=6, help="BGZF level of the input file and of the output")
    ap.add_argument("--kernel-steps", type=int, default=3, help="timed steps of the kernel-only leg")
    ap.add_argument("--cpu-sample-reads", type=int, default=2_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads for the reference (box CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-realign", action="store_true", help="skip the localrealign (C5) leg")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--realign-intervals", type=int, default=50_000)
    ap.add_argument("--realign-only", action="store_true", help="profiling aid: only the C5 realign leg")
    ap.add_argument("--e2e-only", action="store_true", help="profiling aid: skip every leg but the e2e steps")
    ap.add_argument("--kernel-only", action="store_true", help="profiling aid: only the kernel-only leg")
    return ap.parse_args()


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------- helpers
class DevBuf:
    """Device bytes from the library's allocator, or a view of one of the chain's reserved record arenas
    (oge_mergesort_reserve): the records and the staging file of the setup live in the arenas the chain
    then uses, so its first call does not re-acquire HBM the setup freed (the driver wipes freed HBM
    before handing it out again, ~35-45 GB/s: 4.3 s for the two 85.6 GB arenas, profiles/r05i_bench.log)."""

    def __init__(self, ctx, L, nbytes: int):
        import ctypes as C
        self.ctx, self.L = ctx, L
        p = C.c_void_p()
        L.check(L.lib().oge_dev_alloc(ctx.h, nbytes, C.byref(p)), ctx.h)
        self.ptr, self.nbytes = p.value, nbytes

    def put(self, off: int, data: bytes) -> None:
        b = bytearray(data)
        import ctypes as C
        src = (C.c_char * len(b)).from_buffer(b)
        self.L.check(self.L.lib().oge_memcpy(self.ctx.h, self.ptr + off, C.addressof(src), len(b), 1), self.ctx.h)

    def get(self, off: int, nbytes: int, host_ptr: int | None = None):
        """nbytes at off -> numpy array (or into host_ptr)"""
        import numpy as np
        out = None
        if host_ptr is None:
            out = np.empty(nbytes, np.uint8)
            host_ptr = out.ctypes.data
        self.L.check(self.L.lib().oge_memcpy(self.ctx.h, host_ptr, self.ptr + off, nbytes, 2), self.ctx.h)
        return out

    def free(self) -> None:
        if self.ptr and self.owned:
            self.L.check(self.L.lib().oge_dev_free(self.ctx.h, self.ptr), self.ctx.h)
        self.ptr = 0

    owned = True

    @classmethod
    def view(cls, ctx, L, ptr: int, nbytes: int) -> "DevBuf":
        """bytes the library owns (one of the chain's reserved arenas): free() only forgets them"""
        b = cls.__new__(cls)
        b.ctx, b.L, b.ptr, b.nbytes, b.owned = ctx, L, ptr, nbytes, False
        return b


def bam_header_bytes(header_text: str) -> bytes:
    """BamSerializer::open's header block (util/bam_serializer.h:54-76): magic, text, reference list."""
    refs = []
    for ln in header_text.splitlines():
        if ln.startswith("@SQ"):
            f = dict(x.split(":", 1) for x in ln.split("\t")[1:])
            refs.append((f["SN"], int(f["LN"])))
    t = header_text.encode()
    out = b"BAM\1" + struct.pack("<i", len(t)) + t + struct.pack("<i", len(refs))
    for nm, ln in refs:
        b = nm.encode() + b"\0"
        out += struct.pack("<i", len(b)) + b + struct.pack("<i", ln)
    return out


def stage_ms(ctx, names) -> dict:
    out = {}
    for s in names:
        v = ctx.timing(s)
        if v >= 0:
            out[s] = v
    return out


def pmc_files() -> list:
    """profiles/r<round><tag>_pmc.json oldest first: round, then tag by length and letters (r05z < r05aa)."""
    import re

    def key(f):
        m = re.match(r"r(\d+)([a-z]*)", f.name)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, f.name)
    return sorted((f for f in (ROOT / "profiles").glob("r*_pmc.json") if "realign" not in f.name), key=key)


def pmc_traffic(kernel: str, rec_bytes: int) -> dict | None:
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/r*_pmc.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md).  Scaled by record bytes when the profiled workload
    differed."""
    files = pmc_files()
    for fn in reversed(files):
        try:
            d = json.loads(fn.read_text())
        except Exception:
            continue
        for name, v in d.get("kernels", {}).items():
            if kernel in name:
                w = d.get("workload", {})
                b = w.get("record_bytes_rank0") or w.get("record_bytes_per_gpu") or rec_bytes
                return {"bytes": v["hbm_bytes"] * rec_bytes / b, "source": fn.name}
    return None


# kernel per e2e stage (the launch the stage time belongs to), its algorithmic bytes and what bounds it:
# the gather and the record parse stream HBM; the codec kernels are serial per-block chains (Huffman
# decode, greedy parse, bit emission) bound by VALU issue and latency, not by HBM bandwidth
def stage_kernels(B: int, zin: int, zout: int, n: int, seq_bytes: int) -> dict:
    return {
        "bgzf_inflate": ("k_infl", "BGZF inflate: compressed bytes read + payload bytes written", zin + B, "valu"),
        "infl_huff": ("k_infl_huff", "inflate phase 1, Huffman decode: compressed bytes read + every payload byte written "
                      "(literal or copy descriptor)", zin + B, "valu"),
        "infl_lz": ("k_infl_lz", "inflate phase 2, copies + CRC: payload bytes read + written", 2 * B, "valu"),
        "bgzf_deflate": ("k_defl", "BGZF deflate (greedy single-candidate, -c 6): payload read + compressed bytes written", B + zout, "valu"),
        "gather_records": ("k_gather16", "permutation gather + BAM re-encode: 2*B (SURVEY §8d sort bytes)", 2 * B, "hbm"),
        "input_pass": ("k_input_pass", "record parse: B - packed bases (SURVEY §8d dedup bytes) + 2N",
                       B - seq_bytes + 2 * n, "hbm"),
    }


def pmc_valu(kernel: str, rec_bytes: int) -> dict | None:
    """VALU lane-instructions per launch of a stage's kernels (SQ_INSTS_VALU x 64) from the newest
    committed PMC summary that has them, scaled by record bytes like pmc_traffic."""
    files = pmc_files()
    for fn in reversed(files):
        try:
            d = json.loads(fn.read_text())
        except Exception:
            continue
        for name, v in d.get("kernels", {}).items():
            if kernel in name and v.get("valu_insts"):
                w = d.get("workload", {})
                b = w.get("record_bytes_rank0") or w.get("record_bytes_per_gpu") or rec_bytes
                return {"lane_ops": 64 * v["valu_insts"] * rec_bytes / b, "source": fn.name}
    return None


def roofline_entry(stage: str, info: tuple, t_ms: float, B: int) -> dict:
    kname, what, abytes, bound = info
    ach = abytes / (t_ms / 1e3) / 1e9 if t_ms > 0 else 0.0
    pmc = pmc_traffic(kname, B)
    r = {"kernel": f"{kname} ({what})", "stage": stage, "bound": bound, "achieved": round(ach, 1),
         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
         "traffic": round(pmc["bytes"]) if pmc else None, "traffic_source": pmc["source"] if pmc else None,
         "traffic_ratio": round(pmc["bytes"] / abytes, 2) if pmc else None,
         "algorithmic_bytes": abytes, "avg_ms": t_ms}
    if bound == "valu":
        v = pmc_valu(kname, B)
        if v and t_ms > 0:
            a = v["lane_ops"] / (t_ms / 1e3) / 1e12
            r["valu"] = {"achieved": round(a, 2), "peak": round(VALU_INT32_PEAK_TOPS, 1), "unit": "T lane-ops/s",
                         "frac": round(a / VALU_INT32_PEAK_TOPS, 4), "source": v["source"]}
    return r


# --------------------------------------------------------------------------------------------- legs
def realign_leg(ctx, n_intervals: int, rank: int = 0, world: int = 1, cpu_threads: int = 0,
                dump_dir: str | None = None) -> dict | None:
    """configs[4]: openge localrealign on the C5 synthetic set (50k indel intervals, 24 contigs).
    Host phases (binning, consensus generation, decisions, mate fixing) + the HIP offset scan; the
    records are decoded in host memory before the timed region (the module's input queue).  With
    world > 1 every rank realigns its contig range (openge_amd/realign_shard.py, no exchange); the
    time is the max over ranks between barriers.  Returns the result on rank 0 (None elsewhere)."""
    from openge_amd import lib as L
    from openge_amd import realign_shard as RS

    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        p = L.realign_synth_params(n_intervals=n_intervals)
        fa, iv, bam = L.synth_realign(p, td, level=1, threads=16)
        b = L.Bam(bam, threads=16)
        import numpy as np
        offs = np.append(b.offs, np.uint64(b.recs.size))
        opts = L.realign_opts(threads=16)
        ref_lens = [int(dict(x.split(":", 1) for x in ln.split("\t")[1:])["LN"])
                    for ln in b.header_text.splitlines() if ln.startswith("@SQ")]
        lo, hi = RS.contig_slices(b.recs, offs, b.n, ref_lens, world)[rank]
        run = lambda: RS.localrealign_slice(ctx, b.header_text, b.recs, offs, lo, hi, fa, iv, opts,
                                            last=(rank == world - 1))
        # the whole command as a user runs it, in a fresh process: `openge localrealign` BAM file in -> BAM
        # file out (process start, HIP init, BGZF read, realign, mate fixing, BGZF write), beside the
        # reference's own chain timed the same way (cpu_baseline_realign); the in-process legs below time
        # the realigner itself on records already decoded
        cli = None
        if world == 1:
            cli = realign_cli_leg(fa, iv, bam, td)
        if world > 1:
            import torch
            import torch.distributed as dist
            dist.barrier()
        # the headline: the FIRST call in this process -- the realigner's cross-call
        # scratch (worker pool, record objects, event list, FASTA buffers) is built inside it, as in a fresh
        # `openge localrealign`; the second call (warm scratch) is reported beside it
        t0c = time.perf_counter()
        w_out, w_oo, first_st = run()
        first_call_s = time.perf_counter() - t0c
        if dump_dir:  # this rank's realigned records (tests concatenate the ranks' parts)
            Path(dump_dir, f"realign_{rank}.bin").write_bytes(np.asarray(w_out[:int(w_oo[-1])]).tobytes())
        ref_cpu = None
        if world == 1 and cpu_threads:  # the reference's own realigner on the same files, this box's host
            ref_cpu = cpu_baseline_realign(fa, iv, bam, n_intervals, cpu_threads, td)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        out, oo, st = run()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt, first_call_s], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt, first_call_s = float(t[0].item()), float(t[1].item())
            if rank != 0:
                return None
            return {"metric": "realign intervals/sec", "value": round(n_intervals / first_call_s, 1), "unit": "intervals/s",
                    "workload": f"C5: {n_intervals} indel intervals, 24 contigs, {b.n} reads (seed 1234)",
                    "seconds": round(first_call_s, 3), "warm_seconds": round(dt, 3),
                    "warm_value": round(n_intervals / dt, 1), "n_gpus": world, "scaling": "strong",
                    "parallelism": f"{world} ranks, contig-range shards, no exchange", "host_threads_per_rank": 16,
                    "rank0_reads": hi - lo, "rank0_stats": st}
    # VALU lane-ops per launch from the committed PMC pass (SQ_INSTS_VALU x 64; the instruction count
    # is fixed by the workload), divided by the live HIP-event time of the scan stage
    valu = realign_pmc_valu()
    t_k = st["scan_kernel_ms"] / 1e3
    ach = valu["lane_ops"] / t_k / 1e12 if (valu and t_k > 0 and n_intervals == 50_000) else None
    cmp_t = st["scan_ops"] / t_k / 1e12 if t_k > 0 else None
    # frac: SURVEY §8(d)'s algorithmic ops (#offsets x read length compare-accumulates per consensus x
    # altRead pair) per second over the int32 VALU peak; the bit-parallel kernel's own lane-ops (PMC) as a
    # secondary figure
    return {"metric": "realign intervals/sec", "value": round(n_intervals / first_call_s, 1), "unit": "intervals/s",
            "workload": f"C5: {n_intervals} indel intervals, 24 contigs, {b.n} reads (seed 1234)",
            "seconds": round(first_call_s, 3), "host_threads": 16, "stats": first_st,
            "timed_region": "the realigner on records already decoded in host memory, FIRST call in the process "
                            "(its scratch built inside the timed region; the leg runs before the 300M legs, on a "
                            "context of its own); warm_*: the second call; cli: the whole command, file to file, "
                            "fresh process",
            "warm_seconds": round(dt, 3), "warm_value": round(n_intervals / dt, 1), "warm_stats": st, "cli": cli,
            "roofline": {"kernel": "k_planes + k_scan_bp (findBestOffset over all consensus x altRead pairs, "
                                   "bit-parallel)",
                         "bound": "valu", "achieved": round(cmp_t, 2) if cmp_t else None,
                         "peak": round(VALU_INT32_PEAK_TOPS, 1), "unit": "T algorithmic compare-accumulates/s",
                         "frac": round(cmp_t / VALU_INT32_PEAK_TOPS, 4) if cmp_t else None,
                         "algorithmic_compares": st["scan_ops"], "avg_ms": st["scan_kernel_ms"],
                         "lane_ops": valu["lane_ops"] if valu else None,
                         "lane_ops_per_s_T": round(ach, 2) if ach is not None else None,
                         "lane_ops_frac": round(ach / VALU_INT32_PEAK_TOPS, 4) if ach is not None else None,
                         "lane_ops_source": valu["source"] if valu else None},
            "cpu_baseline": ref_cpu}


def realign_cli_leg(fa: str, iv: str, bam: str, td: str) -> dict:
    """`openge localrealign` (openge_amd/openge, this repo's CLI) as a fresh process on the C5 files, BAM
    file in -> BAM file out, wall time: the like-for-like counterpart of the reference's leg."""
    exe = ROOT / "openge_amd" / "openge"
    if not exe.exists():
        return {"seconds": None, "note": f"{exe} missing"}
    out = os.path.join(td, "gpu_realigned.bam")
    t0 = time.perf_counter()
    r = subprocess.run([str(exe), "localrealign", "--nopg", "-t", "16", "-R", fa, "-L", iv, bam, "-o", out],
                       capture_output=True, text=True, timeout=600)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        return {"seconds": None, "note": f"openge exit {r.returncode}: {r.stderr[-300:]}"}
    return {"seconds": round(dt, 3), "what": "openge localrealign -t 16 -R fa -L intervals in.bam -o out.bam --nopg, "
                                             "fresh process, BAM file in -> BAM file out (level-6 output)"}


def cpu_baseline_realign(fa: str, iv: str, bam: str, n_intervals: int, threads: int, td: str) -> dict:
    """The REFERENCE's LocalRealignment chain (oracle/_ref/ref_driver realign: FileReader ->
    LocalRealignment -> BamSerializer, cmd/command_localrealign.cpp:37-75, compiled from its sources)
    on the same C5 files, timed on this box's host cores in the same run (TEST INFRASTRUCTURE, the CPU
    baseline only)."""
    drv = ROOT / "oracle" / "_ref" / "ref_driver"
    if not drv.exists():
        return {"value": None, "kind": "reference", "note": f"{drv} missing (built only where /root/reference exists)"}
    out = os.path.join(td, "ref_realigned.bam")
    t0 = time.perf_counter()
    r = subprocess.run([str(drv), "realign", "-t", str(threads), "-R", fa, "-L", iv, bam, out], capture_output=True,
                       text=True, timeout=900)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        return {"value": None, "kind": "reference", "note": f"ref_driver exit {r.returncode}: {r.stderr[-300:]}"}
    return {"value": round(n_intervals / dt, 1), "unit": "intervals/s", "cores": threads, "kind": "reference",
            "sample": f"the same C5 set ({n_intervals} intervals), OpenGE's own localrealign chain "
                      f"(oracle/_ref/ref_driver realign -t {threads}), BAM file in -> BAM file out, wall time",
            "seconds": round(dt, 2)}


def realign_pmc_valu() -> dict | None:
    """VALU lane-ops per C5 scan (k_planes + k_scan_bp) from the newest profiles/r*_realign_pmc.json."""
    files = sorted((ROOT / "profiles").glob("r*_realign_pmc.json"))
    if not files:
        return None
    try:
        d = json.loads(files[-1].read_text())
        k = d["kernels"]
        return {"lane_ops": 64 * (k["k_planes"]["SQ_INSTS_VALU"] + k["k_scan_bp"]["SQ_INSTS_VALU"]),
                "source": files[-1].name}
    except Exception:
        return None


def cpu_baseline_reference(sample_reads: int, threads: int) -> dict:
    """The REFERENCE (TEST INFRASTRUCTURE, timed as the CPU baseline only): oracle/_ref/ref_driver is
    OpenGE's own FileReader -> ReadSorter -> MarkDuplicates -> BamSerializer<BgzfOutputStream> chain
    (command_mergesort.cpp:68-117 with -M --nosplit -v, n = 500,000 reads per run, level-0 temp runs,
    level-6 dedup temp file and output) compiled from its sources by oracle/Makefile.ref.  Timed
    BAM file in -> BAM file out on this box's host cores, on a bounded sample of the C2 generator."""
    from openge_amd import lib as L

    drv = ROOT / "oracle" / "_ref" / "ref_driver"
    if not drv.exists():
        return {"value": None, "kind": "reference", "note": f"{drv} missing (built only where /root/reference exists)"}
    n_pairs = sample_reads // 2
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        src, dst = os.path.join(td, "in.bam"), os.path.join(td, "out.bam")
        p = L.synth_params(n_pairs, preset="c2", seed=1234)
        recs, offs, hdr = L.synth_host(p, threads=threads)
        L.write_bam(src, hdr, recs, offs, len(offs) - 1, level=6, threads=threads)
        del recs, offs
        t0 = time.perf_counter()
        r = subprocess.run([str(drv), "sortdedup", "-v", "-t", str(threads), "-n", "500000", "-c", "6", "-T", td, src, dst],
                           capture_output=True, text=True, timeout=900)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            return {"value": None, "kind": "reference", "note": f"ref_driver exit {r.returncode}: {r.stderr[-300:]}"}
        marked = [ln for ln in r.stderr.splitlines() if "uplicate" in ln][-1:]
    n = 2 * n_pairs
    return {"value": round(n / dt / 1e6, 4), "unit": "Mreads/s", "cores": threads, "kind": "reference",
            "sample": f"{n} reads of the C2 generator (seed 1234) as a level-6 BAM file -> OpenGE's own "
                      f"mergesort -M --nosplit -v chain (oracle/_ref/ref_driver sortdedup -t {threads} -n 500000) "
                      "-> level-6 BAM file, wall time.  SIZE DIFFERS from the GPU leg (300M reads): at 300M the "
                      "reference merges 600 spilled runs through a std::multiset (util/read_stream_reader.h:132-153), "
                      "so its per-read cost there is higher and gpu_speedup is conservative",
            "seconds": round(dt, 2), "reference_log_tail": marked}


def kernel_leg(ctx, L, torch, dev, p, n, hlen, args) -> tuple[dict, DevBuf, int, object]:
    """Records generated straight into HBM after a `hlen`-byte BAM header prefix (the buffer later
    becomes the input file); the sort+dedup device pipeline alone over the resident records."""
    d_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), None)
    ctx.sync()
    B = int(d_offs[-1].item())
    X, Y, cap = ctx.mergesort_reserve(hlen + B)
    S = DevBuf.view(ctx, L, Y, cap)  # the chain's sorted-records arena holds the generated records
    d_offs += hlen
    ctx.synth_range_dev(p, 0, n, d_offs.data_ptr(), S.ptr)
    ctx.sync()
    import ctypes as C
    buf = C.create_string_buffer(1 << 16)
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
    hdr_text = buf.value.decode()
    opts, keep = L.markdup_opts_from_header(hdr_text, p.n_ref)
    res = {"skipped": True}
    if args.kernel_steps > 0:
        d_out = DevBuf.view(ctx, L, X, cap)
        d_out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_perm = torch.empty(n, dtype=torch.int32, device=dev)
        step = lambda: ctx.sort_markdup_dev(S.ptr, d_offs.data_ptr(), n, opts, d_perm.data_ptr(),
                                            d_out.ptr, d_out_off.data_ptr())
        step()  # first call: workspace growth, code-object load
        torch.cuda.synchronize(dev)
        tot = {s: 0.0 for s in KERNEL_STAGES + SUB_STAGES}
        t0 = time.perf_counter()
        for _ in range(args.kernel_steps):
            nd = step()
            for s, v in stage_ms(ctx, KERNEL_STAGES + SUB_STAGES).items():
                tot[s] += v
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / args.kernel_steps
        K = args.kernel_steps
        sms = {s: round(v / K, 3) for s, v in tot.items()}
        tg = sms["gather_records"] / 1e3
        res = {"what": "oge_sort_markdup_dev over records already decoded in HBM (no codec)",
               "ms_per_step": round(dt * 1e3, 2), "mreads_per_s": round(n / dt / 1e6, 1), "steps": K,
               "duplicates_flagged": nd, "stages_ms": sms,
               "mate_join": {k: ctx.counter("md_mate_" + k) for k in ("pairs", "left", "ovf", "redo")},
               "gather_roofline": {"kernel": "k_gather16", "achieved_GBps": round(2 * B / tg / 1e9, 1) if tg else None,
                                   "frac": round(2 * B / tg / 1e9 / HBM_PEAK_GBS, 4) if tg else None,
                                   "algorithmic_bytes": 2 * B}}
        # configs[2]: `openge dedup` on the sorted records -- oge_markdup_dev in place (record index = position in
        # the file, 0x400 set / cleared in the records themselves) over the records the steps above sorted
        # (their 0x400 bits are recomputed, not read).  The in-place path verifies the anchors never decrease
        # and then takes the windowed mate join and groups (markdup.hip oge_markdup_run).
        # (a context of its own, closed after the leg: without the fused chain's arena loan its workspaces are
        # ~17 GB that would otherwise stay allocated and shrink the e2e inflate's chunks)
        dctx = L.Context(torch.cuda.current_device(), stream=ctx.stream)
        d_dup = torch.empty(n + 1, dtype=torch.uint8, device=dev)
        md = lambda: dctx.markdup_dev(d_out.ptr, d_out_off.data_ptr(), n, opts, d_dup.data_ptr(), apply=True)
        md()
        torch.cuda.synchronize(dev)
        tot2 = {s: 0.0 for s in DEDUP_STAGES + SUB_STAGES}
        t0 = time.perf_counter()
        for _ in range(args.kernel_steps):
            nd2 = md()
            for s, v in stage_ms(dctx, DEDUP_STAGES + SUB_STAGES).items():
                tot2[s] += v
        torch.cuda.synchronize(dev)
        dt2 = (time.perf_counter() - t0) / args.kernel_steps
        sms2 = {s: round(v / K, 3) for s, v in tot2.items()}
        # dedup's algorithmic bytes = B - sum ceil(l_seq / 2) + 2 N (every record read once
        # except its packed bases, plus the flag write-back)
        dbytes = B - n * ((p.read_len + 1) // 2) + 2 * n
        res["dedup_inplace"] = {
            "what": "configs[2]: openge dedup's device path, oge_markdup_dev in place over the sorted records in HBM",
            "ms_per_step": round(dt2 * 1e3, 2), "mreads_per_s": round(n / dt2 / 1e6, 1), "steps": K,
            "duplicates_flagged": nd2, "equals_fused_chain": nd2 == nd,
            "windowed_paths": bool(dctx.counter("md_inplace_window")), "stages_ms": sms2,
            "algorithmic_bytes": dbytes, "hbm_frac_step": round(dbytes / dt2 / 1e9 / HBM_PEAK_GBS, 4)}
        dctx.close()
        del d_dup
        d_out.free()
        del d_out_off, d_perm
    del d_offs
    torch.cuda.empty_cache()
    return res, S, B, hdr_text


DEFLATE_SEARCH = ("GPU deflate (bgzf.hip): greedy parse, ONE hash candidate per position (4-byte prefix, 4096 "
                  "buckets, filled in rounds of 1024 positions), matches cut at 64-byte segment edges, no lazy "
                  "matching; one dynamic-Huffman block per 65,280-byte payload (length-limited to 15 bits). "
                  "Level 0 is stored, 1-7 this mode (it is not zlib's level-6 search), 8-9 add same-prefix chains "
                  "and lazy matching (level9_same_records)")


def zlib6_sample_ratio(S, off: int, nbytes: int, sample: int = 32 << 20) -> dict:
    """zlib level 6 (OpenGE's writer: util/bgzf_output_stream.cpp:74-79) over the first `sample` bytes of the
    record stream in 65,280-byte BGZF payloads (18 + 8 bytes of BGZF framing each), for comparison with the
    GPU deflate's ratio."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    pay = 65280
    n = max(pay, min(nbytes, sample) // pay * pay)
    h = S.get(off, n).tobytes()
    with ThreadPoolExecutor(16) as ex:
        z = sum(ex.map(lambda i: len(zlib.compress(h[i:i + pay], 6)) - 6 + 26, range(0, len(h), pay)))
    return {"ratio": round(z / len(h), 4), "sample_bytes": len(h),
            "what": "zlib level 6 per 65,280-byte payload + BGZF framing, first bytes of the same record stream"}


def build_input(ctx, L, S: DevBuf, total: int, level: int, chain_probe: dict | None = None) -> tuple[DevBuf, int]:
    """The input BAM file in HBM: the library's GPU deflate of [header][records] at `level` plus the
    EOF block, in a buffer of exactly its size (the records S and the bound-sized staging buffer are
    freed).  chain_probe (a dict): first one level-9 deflate of the same bytes (same-prefix chains + lazy
    matching, bgzf.hip) -- its stage time and size go into the dict."""
    bound = int(L.lib().oge_bgzf_bound(total))
    X, _, cap = ctx.mergesort_reserve(total)
    Z = DevBuf.view(ctx, L, X, cap)  # the chain's other arena stages the compressed file
    assert cap >= bound + 64
    zb = ctx.bgzf_deflate_dev(S.ptr, total, level, Z.ptr, bound)
    ctx.sync()
    d_z = DevBuf(ctx, L, zb + 28 + 64)
    L.check(L.lib().oge_memcpy(ctx.h, d_z.ptr, Z.ptr, zb, 3), ctx.h)
    d_z.put(zb, BGZF_EOF)
    if chain_probe is not None:  # after the level-`level` run, so its workspace is in place
        z9 = ctx.bgzf_deflate_dev(S.ptr, total, 9, Z.ptr, bound)
        chain_probe.update({"level": 9, "ms": round(ctx.timing("bgzf_deflate"), 1), "bytes": z9,
                            "ratio": round(z9 / total, 4),
                            "search": "levels 8-9: at every candidate the chain of earlier same-prefix positions "
                                      "(8 / 32 deep) and zlib-style lazy matching; levels 1-7 the greedy search"})
    S.free()
    Z.free()
    return d_z, zb + 28


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from openge_amd import lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # torch.distributed only bootstraps the library's RCCL communicator and times the steps (host
        # values): gloo.  The records move through oge_comm (RCCL over xGMI).
        dist.init_process_group(os.environ.get("OGE_DIST_BACKEND", "gloo"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # one stream for torch ops and our kernels (the default stream is the legacy null stream, which
    # the context's non-blocking stream would not order against)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = L.Context(local, stream=stream.cuda_stream)

    if args.realign_only:
        print(json.dumps(realign_leg(ctx, args.realign_intervals,
                                     cpu_threads=0 if args.no_cpu_baseline else args.cpu_threads,
                                     dump_dir=args.dump_dir)), flush=True)
        ctx.close()
        return

    p = L.synth_params(args.pairs, preset="c2", seed=args.seed)
    n_all = 2 * args.pairs
    if world > 1:
        multi_gpu(args, ctx, L, torch, dist, dev, p, n_all, world, rank)
        ctx.close()
        dist.destroy_process_group()
        return

    # ---- the C5 realign leg first, on a context of its own (closed after it): its "first call" is then the
    #      first realigner call of a fresh process, as in `openge localrealign`, not one that follows the 300M
    #      legs' host-memory churn (the pinned 60 + 57 GB of the PCIe leg)
    realign_res = None
    if not args.no_realign and not args.e2e_only and not args.kernel_only:
        log("realign leg")
        rctx = L.Context(local, stream=stream.cuda_stream)
        realign_res = realign_leg(rctx, args.realign_intervals, cpu_threads=0 if args.no_cpu_baseline else args.cpu_threads)
        rctx.close()
        torch.cuda.empty_cache()
    free0, total_mem = torch.cuda.mem_get_info(dev)
    log(f"HBM free {free0 / 1e9:.1f} / {total_mem / 1e9:.1f} GB")
    # ---- kernel-only leg; the generated records become the input file
    import ctypes as C
    buf = C.create_string_buffer(1 << 16)
    L.check(L.lib().oge_synth_finalize(C.byref(p)))
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
    hb = bam_header_bytes(buf.value.decode())
    n = n_all
    kargs = argparse.Namespace(**vars(args))
    if args.e2e_only:
        kargs.kernel_steps = 0
    kres, S, B, hdr_text = kernel_leg(ctx, L, torch, dev, p, n, len(hb), kargs)
    log(f"kernel leg: {kres.get('ms_per_step')} ms/step; records {B / 1e9:.2f} GB")
    if args.kernel_only:
        print(json.dumps(kres), flush=True)
        ctx.close()
        return
    S.put(0, hb)
    total = len(hb) + B
    seq_bytes = n * ((p.read_len + 1) // 2)

    # ---- the input BAM file in HBM (level-6 BGZF, GPU deflate), staging freed
    zref = zlib6_sample_ratio(S, len(hb), B)
    chain_probe = {}
    d_z, zbytes = build_input(ctx, L, S, total, args.level, chain_probe)
    torch.cuda.synchronize(dev)
    log(f"input BAM file in HBM: {zbytes / 1e9:.2f} GB (ratio {zbytes / total:.3f})")

    # ---- e2e steps: BAM file in HBM -> mergesort -M chain -> BAM file in HBM
    mopts = L.mergesort_opts(level=args.level, mark_duplicates=1)
    step = lambda: ctx.mergesort_bgzf_dev(d_z.ptr, zbytes, mopts)
    warm, cold_ws = [], None
    for _ in range(args.warmup):
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        warm.append(round((time.perf_counter() - tw) * 1e3, 1))
        if cold_ws is None:  # the first call on this context: its workspace allocations
            cold_ws = {"allocations": ctx.counter("ws_allocs"), "ms": round((ctx.counter("ws_alloc_us") or 0) / 1e3, 1)}
        log(f"warmup step {warm[-1]} ms; workspace allocations {ctx.counter('ws_allocs')} taking "
            f"{(ctx.counter('ws_alloc_us') or 0) / 1e3:.1f} ms; stages {stage_ms(ctx, E2E_STAGES)}")
    tot = {}
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out_bytes = nr = nd = 0
    for _ in range(args.steps):
        d_out, out_bytes, nr, nd = step()
        for s, v in stage_ms(ctx, E2E_STAGES + INFL_PHASES).items():
            tot[s] = tot.get(s, 0.0) + v
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    K = args.steps
    ms_step = dt / K * 1e3
    value = n * K / dt / 1e6
    sms = {s: round(v / K, 3) for s, v in tot.items()}
    fr, _ = torch.cuda.mem_get_info(dev)
    log(f"HBM free during e2e steps {fr / 1e9:.1f} GB")
    log(f"e2e: {ms_step:.1f} ms/step = {value:.1f} Mreads/s; stages {sms}")
    assert nr == n, (nr, n)

    # roofline: the dominant kernel of the e2e step (bound per stage; VALU fraction for the codec)
    kinfo = stage_kernels(B, zbytes, out_bytes, n, seq_bytes)
    t_dom, s_dom = max((sms.get(s, 0.0), s) for s in kinfo if s not in INFL_PHASES)
    roof = roofline_entry(s_dom, kinfo[s_dom], t_dom, B)
    others = [roofline_entry(s, kinfo[s], sms[s], B) for s in kinfo if sms.get(s, 0.0) > 0]

    # ---- PCIe-inclusive run (compressed bytes only cross PCIe): the file in page-locked host memory,
    #      oge_mergesort_bgzf_host overlaps its upload with the framing index and inflate, and the output's
    #      download with the deflate
    pcie = None
    if not args.no_pcie and not args.e2e_only:
        hz = torch.empty(zbytes, dtype=torch.uint8, pin_memory=True)
        d_z.get(0, zbytes, hz.data_ptr())
        d_z.free()
        del step
        ocap = out_bytes + (1 << 20)
        ho = torch.empty(ocap, dtype=torch.uint8, pin_memory=True)
        runs = []
        for _ in range(2):  # the first call grows the upload / segment buffers
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            ob, nr2, nd2 = ctx.mergesort_bgzf_host(hz.data_ptr(), zbytes, mopts, ho.data_ptr(), ocap)
            runs.append(time.perf_counter() - t1)
        assert (ob, nr2, nd2) == (out_bytes, nr, nd), (ob, nr2, nd2, out_bytes, nr, nd)
        tp = runs[-1]
        pcie = {"what": "oge_mergesort_bgzf_host: the input BAM file in page-locked host memory -> the output BAM "
                        "file in page-locked host memory; upload overlapped with the host framing index and the "
                        "inflate, download of each deflated segment with the next one's compression", "seconds": round(tp, 3),
                "first_call_seconds": round(runs[0], 3), "mreads_per_s": round(n / tp / 1e6, 1),
                "bytes_up": zbytes, "bytes_down": ob, "stages_ms": stage_ms(ctx, E2E_STAGES)}
        log(f"pcie-inclusive: {tp:.3f} s (first call {runs[0]:.3f} s); stages {pcie['stages_ms']}")
        del hz, ho
    else:
        d_z.free()
        del step

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "Mreads/s", "n_gpus": 1, "steps": K,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: C2 generator (SURVEY §8d) on device, seed 1234, as a level-6 BGZF BAM file resident in HBM",
        "config": {"workload": f"C2+C3 end to end: {n // 1000000}M-read BAM file -> mergesort -M --nosplit "
                               f"(sort + dedup -v) -> BGZF BAM file (-c {args.level}: GPU greedy single-candidate "
                               "deflate, see config.deflate), in HBM",
                   "reads_total": n, "record_bytes": B, "input_file_bytes": zbytes, "output_file_bytes": out_bytes,
                   "duplicates_flagged": nd, "parallelism": "1 GPU",
                   "deflate": {"search": DEFLATE_SEARCH, "gpu_ratio_input_file": round(zbytes / total, 4),
                               "gpu_ratio_output_file": round(out_bytes / total, 4), "zlib6_sample": zref,
                               "level9_same_records": chain_probe}},
        "roofline": roof, "roofline_stages": others, "stages_ms": sms, "warmup_ms": warm,
        "cold_ms": warm[0] if warm else None, "cold_over_warm": round(warm[0] / ms_step, 2) if warm else None,
        "cold_workspace": cold_ws,
        "kernel_step": kres, "pcie_inclusive": pcie,
    }
    torch.cuda.empty_cache()
    if realign_res is not None:
        out["realign"] = realign_res
        rc_ = (out["realign"] or {}).get("cpu_baseline") or {}
        if rc_.get("value"):
            rc_["gpu_speedup"] = round(out["realign"]["value"] / rc_["value"], 1)
            cli_s = ((out["realign"] or {}).get("cli") or {}).get("seconds")
            if cli_s and rc_.get("seconds"):  # like for like: both whole commands, file to file, fresh processes
                rc_["cli_speedup_file_to_file"] = round(rc_["seconds"] / cli_s, 1)
    if not args.no_cpu_baseline and not args.e2e_only:
        log("cpu baseline (reference)")
        cb = cpu_baseline_reference(args.cpu_sample_reads, args.cpu_threads)
        if cb.get("value"):
            cb["gpu_speedup"] = round(value / cb["value"], 1)
        out["cpu_baseline"] = cb
    print(json.dumps(out), flush=True)
    ctx.close()


DIST_STAGES = ["bgzf_index", "bgzf_inflate", "shard_edges", "rec_walk", "dist_split", "dist_exchange", "input_pass", "sort_radix",
               "sort_ties", "meta_gather", "dist_frags", "dist_join", "dist_pairs", "dist_reduce", "md_apply",
               "gather_offsets", "gather_records", "bgzf_deflate"]


def exchange_summary(per_rank: list) -> dict:
    """The last step's collectives (oge_comm_stats_json of every rank): per tag, bytes that crossed
    between ranks (sum over ranks of bytes sent), bytes kept on their rank, calls, and the slowest
    rank's time (host wall time of the collective calls, waiting for peers included), plus each rank's
    own list."""
    tags: dict = {}
    for r in per_rank:
        for x in r["exchanges"]:
            t = tags.setdefault(x["tag"], {"calls": x["calls"], "bytes_between_ranks": 0, "bytes_kept": 0, "max_ms": 0.0,
                                           "max_device_ms": 0.0, "mode": x.get("mode", "blocking")})
            t["bytes_between_ranks"] += x["bytes_sent"]
            t["bytes_kept"] += x["bytes_self"]
            t["max_ms"] = round(max(t["max_ms"], x["ms"]), 3)
            t["max_device_ms"] = round(max(t["max_device_ms"], x.get("device_ms", 0.0)), 3)
    return {"by_tag": tags, "per_rank": [r["exchanges"] for r in per_rank],
            "what": "last timed step; bytes_between_ranks = sum over ranks of bytes sent to other ranks; "
                    "ms = host wall time of the tag's collectives on a rank (peers' skew included); mode side_stream = "
                    "the peers' parts moved on a side stream while the rank's own records went through the input "
                    "pass (RCCL: ms is the time to queue them); device_ms (RCCL only) = the collectives' own time on their "
                    "stream from HIP events around them (RCCL calls are stream-ordered and not waited for), peers' skew "
                    "included"}


def multi_gpu(args, ctx, L, torch, dist, dev, p, n_all, world, rank):
    """N ranks, one process per GPU, RCCL over xGMI through the library's own communicator
    (oge_comm_init_rank; torch.distributed only bootstraps it and times the steps, on gloo).  ONE input
    BAM file (config 4: the node sorts one file): the C2 data set behind its header, BGZF level 6, made
    by the same seeded generator and deterministic GPU deflate on every rank before the timed region;
    rank g keeps only its byte range of it in its HBM (lib.shard_ranges: the blocks that start in
    [a_g, a_g + own_g), plus up to 64 KiB of the next range for its last block).  A step is the whole
    `mergesort -M --nosplit` chain over the one file (oge_mergesort_bgzf_shard): every rank indexes and
    inflates only its own blocks, the ranks join their block and record boundaries and hand over the
    records that straddle them, then the range-split exchange of the records, local sort, exact
    distributed dedup, and every rank deflating its slice of the one output file.  Strong scaling: the
    300M reads of the file are split over the N ranks."""
    import ctypes as C
    buf = C.create_string_buffer(1 << 16)
    L.check(L.lib().oge_synth_finalize(C.byref(p)))
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
    hb = bam_header_bytes(buf.value.decode())
    d_offs = torch.empty(n_all + 1, dtype=torch.int64, device=dev)
    ctx.synth_range_dev(p, 0, n_all, d_offs.data_ptr(), None)
    ctx.sync()
    B = int(d_offs[-1].item())
    # the whole file on every rank (library allocations, not the chain's arenas: a rank's chain holds 1/N of
    # the records), then only this rank's byte range kept
    total = len(hb) + B
    S = DevBuf(ctx, L, total + 64)
    ctx.synth_range_dev(p, 0, n_all, d_offs.data_ptr(), S.ptr + len(hb))
    S.put(0, hb)
    del d_offs
    torch.cuda.empty_cache()
    bound = int(L.lib().oge_bgzf_bound(total))
    Z = DevBuf(ctx, L, bound + 64)
    zb = ctx.bgzf_deflate_dev(S.ptr, total, args.level, Z.ptr, bound)
    ctx.sync()
    S.free()
    Z.put(zb, BGZF_EOF)
    zfile = zb + 28
    a, own, end = L.shard_ranges(zfile, world)[rank]
    d_zb = DevBuf(ctx, L, end - a + 64)
    L.check(L.lib().oge_memcpy(ctx.h, d_zb.ptr, Z.ptr + a, end - a, 3), ctx.h)
    Z.free()
    zbytes = end - a
    torch.cuda.synchronize(dev)
    obj = [L.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    comm = L.comm_init_rank(ctx, world, rank, obj[0])
    log(f"rank {rank}: file bytes [{a}, {a + own}) of {zfile} ({zbytes} held), transport {comm.transport}")
    mopts = L.mergesort_opts(level=args.level, mark_duplicates=1)
    step = lambda: comm.mergesort_bgzf_shard(d_zb.ptr, zbytes, own, mopts)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    tot, nr, nd, ob, d_last = {}, 0, 0, 0, 0
    for _ in range(args.steps):
        d_last, ob, nr, nd = step()
        for s_, v in stage_ms(ctx, DIST_STAGES).items():
            tot[s_] = tot.get(s_, 0.0) + v
    torch.cuda.synchronize(dev)
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    # per-rank record of the last step: every exchange's bytes and time, every stage's time, the share of
    # the file this rank decoded
    K = args.steps
    shard = {k: ctx.counter(k) for k in ("shard_blocks", "shard_zbytes", "shard_bytes", "shard_records")}
    shard.update({"file_range": [a, a + own], "output_bytes": ob})
    mine = {"exchanges": comm.exchange_stats(), "stages_ms": {k: round(v / K, 3) for k, v in tot.items()}, "shard": shard}
    per_rank = [None] * world
    dist.all_gather_object(per_rank, mine)
    assert nr == n_all, (nr, n_all)
    transport = comm.transport
    if args.dump_dir:  # this rank's slice of the output file (valid until the rank's next call)
        hs = torch.empty(max(ob, 1), dtype=torch.uint8)
        L.check(L.lib().oge_memcpy(ctx.h, hs.data_ptr(), d_last, ob, 2), ctx.h)
        Path(args.dump_dir, f"slice_{rank}.bam").write_bytes(hs[:ob].numpy().tobytes())
    comm.close()
    d_zb.free()
    torch.cuda.empty_cache()
    realign_multi = None
    if not args.no_realign:
        realign_multi = realign_leg(ctx, args.realign_intervals, rank, world, dump_dir=args.dump_dir)
    if rank == 0:
        out = {"metric": METRIC, "value": round(n_all * K / dt / 1e6, 2), "unit": "Mreads/s", "n_gpus": world,
               "steps": K, "warmup": args.warmup, "ms_per_step": round(dt / K * 1e3, 2), "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "u8",
               "data": "synthetic: C2 generator (SURVEY §8d) on device, seed 1234, ONE level-6 BGZF input file; rank g "
                       "holds its byte range of it in its HBM",
               "config": {"workload": f"C2+C3 end to end over {world} GPUs: one {n_all // 1000000}M-read BAM file, "
                                      "each rank decoding the BGZF blocks of its byte range -> mergesort -M --nosplit "
                                      "(range-split sort + exact distributed dedup) -> one BGZF "
                                      f"level-{args.level} BAM file as {world} rank slices, in HBM",
                          "reads_total": n_all, "input_file_bytes": zfile, "duplicates_flagged": nd,
                          "shard_per_rank": [r["shard"] for r in per_rank],
                          "parallelism": f"{world} ranks (one process per GPU), all-to-all via oge_comm_init_rank",
                          "transport": transport},
               "stages_ms_rank0": {k: round(v / K, 3) for k, v in tot.items()},
               "stages_ms_per_rank": [r["stages_ms"] for r in per_rank],
               "exchanges": exchange_summary(per_rank)}
        if realign_multi is not None:
            out["realign"] = realign_multi
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
