"""CPU: the product's threaded host code (bamio.cpp reader/writer threads, every realign.cpp phase on
its thread pool) built with AddressSanitizer and, separately, ThreadSanitizer (tests/native/
sanitize_main.cpp), run on the reference-made realignment cases; the output must still be the
reference's and no sanitizer may report.  The multi-GPU hub is covered under TSan by
test_dist_plan.py."""
import fcntl
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import bamutil
from test_realign import check_output, load_rl_case

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "tests" / "native"
SRCS = [NATIVE / "sanitize_main.cpp", ROOT / "openge_amd/csrc/realign.cpp", ROOT / "openge_amd/csrc/bamio.cpp"]
FLAGS = {"asan": ["-fsanitize=address", "-fno-omit-frame-pointer"], "tsan": ["-fsanitize=thread"]}


def _build(kind: str) -> Path:
    out = NATIVE / "_build" / f"sanitize_{kind}"
    out.parent.mkdir(exist_ok=True)
    # pytest-xdist workers may ask for the same binary at once: build under a lock, publish atomically
    with open(out.parent / f".sanitize_{kind}.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return _build_locked(kind, out)


def _build_locked(kind: str, out: Path) -> Path:
    deps = SRCS + list((ROOT / "openge_amd/csrc").glob("*.h")) + [ROOT / "oracle/oge_oracle.c"]
    if out.exists() and all(d.stat().st_mtime <= out.stat().st_mtime for d in deps):
        return out
    obj = out.parent / f"oge_oracle_{kind}.o"
    tmp = out.with_suffix(".tmp")
    subprocess.run(["gcc", "-O1", "-g", "-std=c99", *FLAGS[kind], "-c", str(ROOT / "oracle/oge_oracle.c"), "-o", str(obj)],
                   check=True)
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", *FLAGS[kind], f"-I{ROOT / 'include'}", "-o", str(tmp),
                    *map(str, SRCS), str(obj), "-lz", "-lpthread", "-ldl"], check=True)
    os.replace(tmp, out)
    return out


@pytest.mark.parametrize("kind", ["asan", "tsan"])
@pytest.mark.parametrize("name,maxrec", [("rl_small", 0), ("rl_edge", 0), ("rl_small", 40)])
def test_host_code_clean_under_sanitizer(kind, name, maxrec, tmp_path, built):
    exe = _build(kind)
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    env = {"PATH": "/usr/bin:/bin", "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
           "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}
    args = [str(exe), str(tmp_path / "reads.bam"), str(fa), str(iv), str(tmp_path / "o.bam"), "8"]
    if maxrec:
        args.append(str(maxrec))  # forces the mate fixer's single-writer rerun path too
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "ThreadSanitizer" not in r.stderr and "LeakSanitizer" not in r.stderr
    if maxrec == 0:
        _, _, orecs, ooffs = bamutil.read_bam(tmp_path / "o.bam")
        check_output(meta, arrays, orecs, np.append(ooffs, np.uint64(len(orecs))))
