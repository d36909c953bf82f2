"""Out-of-core mergesort -M of 600M C2 reads (2x configs[1]) on ONE GPU.

    python tools/chunked_600m.py [reads=600000000] [chunk_bytes=0 (auto from free HBM)]

The records (~171 GB, more than the 288 GB of HBM can hold twice) are generated on the device slot
range by slot range and copied into one host arena; oge_sort_markdup_chunked then sorts them in runs
spilled back into the arena, cuts key ranges that fit HBM, marks duplicates over the whole input on a
device-resident summary array and hands the output range by range to a callback.  The callback checks
the cross-range order (last key of a range <= first key of the next) and counts records; the run
prints one JSON line (times, runs, ranges, duplicates, HBM/host footprint)."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from openge_amd import lib as L  # noqa: E402


def main():
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000_000
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    dev = torch.device("cuda", 0)
    ctx = L.Context(0)
    pairs = reads // 2
    n = 2 * pairs
    p = L.synth_params(pairs, preset="c2", seed=1234)
    L.check(L.lib().oge_synth_finalize(C.byref(p)))
    buf = C.create_string_buffer(1 << 16)
    L.check(L.lib().oge_synth_header_text(C.byref(p), buf, 1 << 16, None))
    opts, keep = L.markdup_opts_from_header(buf.value.decode(), p.n_ref)
    t0 = time.perf_counter()
    # sizes of every record, then the records slot range by slot range into the host arena
    offs = np.zeros(n + 1, np.uint64)
    step = 20_000_000
    d_off = torch.empty(step + 1, dtype=torch.int64, device=dev)
    sizes = []
    for s0 in range(0, n, step):
        m = min(step, n - s0)
        ctx.synth_range_dev(p, s0, m, d_off.data_ptr(), None)
        ctx.sync()
        o = d_off[:m + 1].cpu().numpy().view(np.uint64)
        sizes.append(np.diff(o))
    np.cumsum(np.concatenate(sizes), out=offs[1:])
    del sizes
    total = int(offs[-1])
    arena = np.empty(total + 64, np.uint8)
    d_rec = torch.empty(int(offs[min(step, n)]) * 2 + 64, dtype=torch.uint8, device=dev)
    for s0 in range(0, n, step):
        m = min(step, n - s0)
        ctx.synth_range_dev(p, s0, m, d_off.data_ptr(), None)
        ctx.synth_range_dev(p, s0, m, d_off.data_ptr(), d_rec.data_ptr())
        ctx.sync()
        b = int(offs[s0 + m] - offs[s0])
        L.check(L.lib().oge_memcpy(ctx.h, arena.ctypes.data + int(offs[s0]), d_rec.data_ptr(), b, 2), ctx.h)
    del d_rec, d_off
    torch.cuda.empty_cache()
    t_gen = time.perf_counter() - t0
    print(f"[chunked] {n} reads, {total / 1e9:.1f} GB in host memory ({t_gen:.1f} s)", file=sys.stderr, flush=True)

    state = {"n": 0, "ranges": 0, "last": None, "ok": True}

    def key_at(d_recs, d_off_p, i):
        o = np.empty(1, np.uint64)
        L.check(L.lib().oge_memcpy(ctx.h, o.ctypes.data, d_off_p + 8 * i, 8, 2), ctx.h)
        r = np.empty(12, np.uint8)
        L.check(L.lib().oge_memcpy(ctx.h, r.ctypes.data, d_recs + int(o[0]) + 4, 12, 2), ctx.h)
        ref = int(r[:4].view(np.int32)[0])
        pos = int(r[4:8].view(np.int32)[0])
        return (ref if ref >= 0 else 1 << 30, pos)

    def on_range(user, d_recs, d_off_p, m):
        try:
            if m:
                first, last = key_at(d_recs, d_off_p, 0), key_at(d_recs, d_off_p, m - 1)
                if state["last"] is not None and state["last"] > first:
                    state["ok"] = False
                state["last"] = last
            state["n"] += m
            state["ranges"] += 1
            print(f"[chunked] range {state['ranges']}: {m} reads", file=sys.stderr, flush=True)
            return 0
        except Exception:  # noqa: BLE001
            return -1

    cb = L.RANGE_CB(on_range)
    nd, nr, ng = C.c_uint64(), C.c_uint64(), C.c_uint64()
    fr0, tot = torch.cuda.mem_get_info(dev)
    t1 = time.perf_counter()
    L.check(L.lib().oge_sort_markdup_chunked(ctx.h, arena.ctypes.data, offs.ctypes.data, n, p.n_ref, C.byref(opts), chunk, cb,
                                             None, C.byref(nd), C.byref(nr), C.byref(ng)), ctx.h)
    dt = time.perf_counter() - t1
    stages = {s: round(ctx.timing(s), 1) for s in ("chunk_runs", "chunk_dedup", "chunk_output")}
    out = {"what": "out-of-core mergesort -M --nosplit on one MI355X (oge_sort_markdup_chunked), host arena in, ranges out",
           "reads": n, "record_bytes": total, "hbm_free_before_gb": round(fr0 / 1e9, 1), "hbm_total_gb": round(tot / 1e9, 1),
           "runs": nr.value, "ranges": ng.value, "duplicates_flagged": nd.value, "reads_out": state["n"],
           "cross_range_order_ok": state["ok"], "seconds": round(dt, 1), "mreads_per_s": round(n / dt / 1e6, 2),
           "stages_ms": stages, "generate_seconds": round(t_gen, 1)}
    print(json.dumps(out), flush=True)
    assert state["n"] == n and state["ok"]
    ctx.close()


if __name__ == "__main__":
    main()
