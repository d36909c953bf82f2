"""Build tests/native/_build/librealign_cpu.so (TEST INFRASTRUCTURE: product host realign phases +
oracle offset scan).  Rebuilt when any source is newer than the library."""
from __future__ import annotations

import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
SO = HERE / "_build" / "librealign_cpu.so"
SRCS = [HERE / "realign_cpu.cpp", ROOT / "openge_amd/csrc/realign.cpp", ROOT / "openge_amd/csrc/bamio.cpp"]
DEPS = SRCS + list((ROOT / "openge_amd/csrc").glob("*.h")) + [ROOT / "oracle/oge_oracle.c"]


def build() -> Path:
    if SO.exists() and all(d.stat().st_mtime <= SO.stat().st_mtime for d in DEPS):
        return SO
    SO.parent.mkdir(exist_ok=True)
    obj = SO.parent / "oge_oracle.o"
    subprocess.run(["gcc", "-O2", "-std=c99", "-fPIC", "-c", str(ROOT / "oracle/oge_oracle.c"), "-o", str(obj)], check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", f"-I{ROOT / 'include'}", "-o", str(SO),
                    *map(str, SRCS), str(obj), "-lz", "-lpthread"], check=True)
    return SO
