#!/usr/bin/env python
"""bench.py -- OpenGE post-alignment hot path on MI355X.

Metric (BASELINE.json): Mreads/s of sort+dedup (`openge mergesort -M --nosplit` semantics: coordinate
sort, Picard MarkDuplicates with -v semantics, output records re-encoded with bin recompute and
FLAG 0x400 applied).  Workload at N=1: configs[1]+[2] -- a 300M-read (150M pairs) 30x WGS-shaped
synthetic read set (SURVEY.md §8d C2 generator, seed 1234), generated straight into HBM; one step =
the whole device pipeline over the resident records (oge_sort_markdup_dev).

Multi-GPU (torchrun, one rank per GPU): the same 300M-read sample split across N ranks (strong
scaling); openge_amd/shard.py routes records to the rank owning their contig with an RCCL all-to-all
over xGMI (ghost copies of cross-rank mates keep MarkDuplicates exact), each rank sorts + dedups its
range, and the ranks' outputs concatenate into the single-GPU result.  value = reads / max-over-ranks
wall time.

Also reported on the same JSON line:
  roofline     -- dominant kernel (the permutation gather, algorithmic bytes 2*B per launch, B = record
                  bytes) timed live with HIP events on the stream it runs on; traffic from the committed
                  rocprofv3 PMC summary when present (profiles/)
  pipeline     -- the same for the whole step (algorithmic bytes of SURVEY §8d: sort 2B + dedup B-seq+2N)
  cpu_baseline -- the oracle port (oracle/oge_oracle.c, single thread, in memory) timed on this box's host
                  on a bounded C2-shaped sample
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mreads/sec sort+dedup (and realign intervals/sec), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
STAGES = ["input_pass", "sort_radix", "sort_ties", "meta_gather", "md_matejoin", "md_pairs", "md_frags", "md_apply",
          "gather_offsets", "gather_records"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=150_000_000, help="read pairs per GPU (default 150M = 300M reads)")
    ap.add_argument("--cpu-sample-reads", type=int, default=8_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-realign", action="store_true", help="skip the localrealign (C5) leg")
    ap.add_argument("--realign-intervals", type=int, default=50_000)
    ap.add_argument("--realign-only", action="store_true", help="profiling aid: only the C5 realign leg")
    return ap.parse_args()


VALU_INT32_PEAK_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12  # CUs x SIMDs x lanes/clk x 2.4 GHz (MI355X_MICROARCH.md)


def realign_leg(ctx, n_intervals: int, rank: int = 0, world: int = 1) -> dict | None:
    """configs[4]: openge localrealign on the C5 synthetic set (50k indel intervals, 24 contigs).
    Host phases (binning, consensus generation, decisions, mate fixing) + the HIP offset scan; the
    records are decoded in host memory before the timed region (the module's input queue).  With
    world > 1 every rank realigns its contig range (openge_amd/realign_shard.py, no exchange); the
    time is the max over ranks between barriers.  Returns the result on rank 0 (None elsewhere)."""
    import tempfile
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
        run()  # warm-up (first-touch, kernel load)
        if world > 1:
            import torch
            import torch.distributed as dist
            dist.barrier()
        t0 = time.perf_counter()
        out, oo, st = run()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            if rank != 0:
                return None
            return {"metric": "realign intervals/sec", "value": round(n_intervals / dt, 1), "unit": "intervals/s",
                    "workload": f"C5: {n_intervals} indel intervals, 24 contigs, {b.n} reads (seed 1234)",
                    "seconds": round(dt, 3), "n_gpus": world, "scaling": "strong",
                    "parallelism": f"{world} ranks, contig-range shards, no exchange", "host_threads_per_rank": 16,
                    "rank0_reads": hi - lo, "rank0_stats": st}
    # VALU lane-ops per launch from the committed PMC pass (SQ_INSTS_VALU x 64; the instruction count
    # is fixed by the workload), divided by the live HIP-event time of the scan stage
    valu = realign_pmc_valu()
    t_k = st["scan_kernel_ms"] / 1e3
    ach = valu["lane_ops"] / t_k / 1e12 if (valu and t_k > 0 and n_intervals == 50_000) else None
    return {"metric": "realign intervals/sec", "value": round(n_intervals / dt, 1), "unit": "intervals/s",
            "workload": f"C5: {n_intervals} indel intervals, 24 contigs, {b.n} reads (seed 1234)",
            "seconds": round(dt, 3), "host_threads": 16, "stats": st,
            "roofline": {"kernel": "k_planes + k_scan_bp (findBestOffset over all consensus x altRead pairs, "
                                   "bit-parallel)",
                         "bound": "valu", "achieved": round(ach, 2) if ach is not None else None,
                         "peak": round(VALU_INT32_PEAK_TOPS, 1), "unit": "T int32 lane-ops/s",
                         "frac": round(ach / VALU_INT32_PEAK_TOPS, 4) if ach is not None else None,
                         "lane_ops": valu["lane_ops"] if valu else None,
                         "lane_ops_source": valu["source"] if valu else None, "avg_ms": st["scan_kernel_ms"],
                         "algorithmic_compares": st["scan_ops"],
                         "compares_per_s_T": round(st["scan_ops"] / t_k / 1e12, 2) if t_k > 0 else None},
            "cpu_reference_here": {"value": 1520.0, "unit": "intervals/s", "cores": 8,
                                   "note": "oracle/_ref/ref_driver realign -t 8 on the same C5 set in the build "
                                           "container (32.9 s); the reference cannot run on the GPU box"}}


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


def cpu_baseline(sample_reads: int) -> dict:
    """The oracle port (TEST INFRASTRUCTURE, timed as the CPU baseline only) on a C2-shaped sample."""
    import oracle
    from openge_amd import lib as L

    p = L.synth_params(sample_reads // 2, preset="c2", seed=1234)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * (sample_reads // 2)
    t0 = time.perf_counter()
    perm = oracle.sort_perm(recs, offs, n)
    oracle.markdup(recs, offs[:-1][perm], n, hdr)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt / 1e6, 4), "unit": "Mreads/s", "cores": 1, "kind": "port",
            "sample": f"{n} reads of the C2 generator (seed 1234), in-memory oracle sort + markdup, 1 thread",
            "seconds": round(dt, 2)}


def pmc_traffic(kernel: str, rec_bytes: int) -> dict | None:
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/r*_pmc.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes).
    When the profiled workload had a different record-byte total, the count is scaled by bytes."""
    files = sorted(f for f in (ROOT / "profiles").glob("r*_pmc.json") if "realign" not in f.name)
    if not files:
        return None
    try:
        d = json.loads(files[-1].read_text())
    except Exception:
        return None
    for name, v in d.get("kernels", {}).items():
        if kernel in name:
            w = d.get("workload", {})
            b = w.get("record_bytes_rank0") or w.get("record_bytes_per_gpu") or rec_bytes
            return {"bytes": v["hbm_bytes"] * rec_bytes / b, "source": files[-1].name}
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from openge_amd import lib as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL on ROCm: all-to-all over xGMI.  OGE_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs.
        dist.init_process_group(os.environ.get("OGE_DIST_BACKEND", "nccl"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # one stream for torch ops and our kernels (the default stream is the legacy null stream, which
    # the context's non-blocking stream would not order against)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = L.Context(local, stream=stream.cuda_stream)

    if args.realign_only:
        print(json.dumps(realign_leg(ctx, args.realign_intervals)), flush=True)
        ctx.close()
        return

    # ---- inputs resident in HBM before the timed region.  One 300M-read sample (C2); with N ranks
    # each holds 1/N of it (an arbitrary slice of the unsorted input: strong scaling).
    p = L.synth_params(args.pairs, preset="c2", seed=1234)
    n_all = 2 * args.pairs
    s0, s1 = n_all * rank // world, n_all * (rank + 1) // world
    n = s1 - s0
    d_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.synth_range_dev(p, s0, n, d_offs.data_ptr(), None)
    ctx.sync()
    B = int(d_offs[-1].item())
    d_recs = torch.empty(B + 64, dtype=torch.uint8, device=dev)
    ctx.synth_range_dev(p, s0, n, d_offs.data_ptr(), d_recs.data_ptr())
    hdr_len = 1 << 16
    import ctypes as C
    buf = C.create_string_buffer(hdr_len)
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, hdr_len, None))
    opts, keep = L.markdup_opts_from_header(buf.value.decode(), p.n_ref)
    ctx.sync()

    shard_t = {}
    if world == 1:
        d_out = torch.empty(B + 64, dtype=torch.uint8, device=dev)
        d_out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_perm = torch.empty(n, dtype=torch.int32, device=dev)

        def step():
            return ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(),
                                        d_out.data_ptr(), d_out_off.data_ptr())
    else:
        from openge_amd import shard
        backend = shard.HipBackend(ctx)
        owners = shard.contig_owners([int(p.ref_len[i]) for i in range(p.n_ref)], world)

        def step():
            T = {}
            out, off, k = shard.sort_markdup_sharded(backend, d_recs, d_offs, n, p.n_ref, owners, opts, timings=T)
            for key, v in T.items():
                shard_t[key] = shard_t.get(key, 0.0) + v
            del out, off
            return k

    warmup_ms = []  # first-call costs (workspace growth, code-object load) stay out of the timed steps
    for _ in range(args.warmup):
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        warmup_ms.append(round((time.perf_counter() - tw) * 1e3, 2))
    shard_t.clear()
    stage_tot = {s: 0.0 for s in STAGES}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ndup = 0
    for _ in range(args.steps):
        ndup = step()
        if world == 1:
            for s in STAGES:  # HIP events recorded around each stage on the context stream
                stage_tot[s] += max(ctx.timing(s), 0.0)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    realign_multi = None
    if world > 1 and not args.no_realign:  # every rank realigns its contig range
        realign_multi = realign_leg(ctx, args.realign_intervals, rank, world)

    if rank == 0:
        K = args.steps
        ms_step = dt / K * 1e3
        value = n_all * K / dt / 1e6
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mreads/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: C2 generator (SURVEY §8d) on device, seed 1234; records resident in HBM",
            "config": {"workload": f"C2+C3 sort+dedup (mergesort -M --nosplit semantics), {n_all // 1000000}M reads "
                                   "in total" + (f", {world} contig-sharded ranks" if world > 1 else ""),
                       "reads_total": n_all, "reads_rank0": n, "record_bytes_rank0": B,
                       "parallelism": (f"{world} ranks: contig ownership + RCCL all-to-all + ghost mates"
                                       if world > 1 else "1 GPU")},
        }
        if world == 1:
            out["config"]["duplicates_flagged"] = ndup
            stages_ms = {s: round(v / K, 3) for s, v in stage_tot.items()}
            t_gather = stages_ms["gather_records"] / 1e3
            gather_bytes = 2 * B  # sort = 2*B (each record read once, written once)
            achieved = gather_bytes / t_gather / 1e9 if t_gather > 0 else 0.0
            seq_bytes = n * ((p.read_len + 1) // 2)
            pipe_bytes = 2 * B + (B - seq_bytes) + 2 * n
            pipe_gbs = pipe_bytes / (ms_step / 1e3) / 1e9
            pmc = pmc_traffic("k_gather16", B)
            out["roofline"] = {"kernel": "k_gather_records (permutation gather + BAM re-encode)", "bound": "hbm",
                               "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(achieved / HBM_PEAK_GBS, 4),
                               "traffic": round(pmc["bytes"]) if pmc else None,
                               "traffic_source": pmc["source"] if pmc else None,
                               "algorithmic_bytes": gather_bytes, "avg_ms": stages_ms["gather_records"]}
            out["pipeline"] = {"algorithmic_bytes": pipe_bytes, "achieved": round(pipe_gbs, 1), "unit": "GB/s",
                               "frac": round(pipe_gbs / HBM_PEAK_GBS, 4)}
            out["stages_ms"] = stages_ms
            out["warmup_ms"] = warmup_ms
            if not args.no_realign:
                out["realign"] = realign_leg(ctx, args.realign_intervals)
            if not args.no_cpu_baseline:
                cb = cpu_baseline(args.cpu_sample_reads)
                cb["gpu_speedup"] = round(value / cb["value"], 1)
                out["cpu_baseline"] = cb
        else:
            out["shard_rank0_s_per_step"] = {k: (round(v / K, 4) if isinstance(v, float) else v // K)
                                             for k, v in shard_t.items()}
            if realign_multi is not None:
                out["realign"] = realign_multi
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
