"""Build libopenge_hip.so (HIP kernels for gfx950 + host codec + C ABI) and the `openge` CLI.

In-tree build with hipcc (no JIT cache): outputs land next to this file so they travel to the
GPU box with the repo snapshot.  Incremental: a target is rebuilt only when a source or header
is newer than it.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "libopenge_hip.so"
CLI = PKG / "openge"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
ARCH = "gfx950"

HIP_SRCS = ["prims.hip", "sort.hip", "records.hip", "markdup.hip", "capi_dev.hip", "realign.hip", "realign_prep.hip", "bgzf.hip", "inflate.hip", "inflate_lane.hip", "filter.hip", "sort_name.hip", "pipeline.hip", "dist.hip", "shard.hip", "chunked.hip"]
HOST_SRCS = ["bamio.cpp", "host_capi.cpp", "realign.cpp", "realign_synth.cpp"]
CLI_SRCS = ["openge_cli.cpp", "modules.cpp"]

COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"-I{ROOT / 'include'}"]


def _headers() -> list[Path]:
    return list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.exists() and d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


def _compile(src: Path, obj: Path, hip: bool) -> None:
    if not _stale(obj, [src] + _headers()):
        return
    obj.parent.mkdir(parents=True, exist_ok=True)
    if hip:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-x", "hip", *COMMON, "-c", str(src), "-o", str(obj)]
    else:
        cmd = [CXX, *COMMON, "-c", str(src), "-o", str(obj)]
    _run(cmd)


def build(verbose: bool = False) -> Path:
    jobs = []
    for s in HIP_SRCS:
        if (CSRC / s).exists():
            jobs.append((CSRC / s, BUILD / (s + ".o"), True))
    for s in HOST_SRCS:
        jobs.append((CSRC / s, BUILD / (s + ".o"), False))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        list(ex.map(lambda j: _compile(*j), jobs))
    objs = [j[1] for j in jobs]
    if _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(LIB), *map(str, objs), "-L/opt/rocm/lib", "-lrccl", "-lz", "-lpthread", "-ldl"])
        if verbose:
            print(f"built {LIB}")
    cli_srcs = [CSRC / s for s in CLI_SRCS if (CSRC / s).exists()]
    if len(cli_srcs) == len(CLI_SRCS):
        cli_objs = []
        for s in cli_srcs:
            o = BUILD / (s.name + ".o")
            _compile(s, o, False)
            cli_objs.append(o)
        if _stale(CLI, cli_objs + [LIB]):
            _run([HIPCC, "-o", str(CLI), *map(str, cli_objs), f"-L{PKG}", "-lopenge_hip",
                  f"-Wl,-rpath,$ORIGIN", "-lz", "-lpthread", "-ldl"])
    return LIB


if __name__ == "__main__":
    build(verbose=True)
