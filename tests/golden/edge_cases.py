"""Hand-crafted records covering the duplicate-marking and sort edge cases the reference code has
(Q2, Q4-Q8, Q10, Q16) -- deterministic, so the file is rebuilt on demand.
"""
from __future__ import annotations

import random
import struct

from bamutil import make_record

HEADER = ("@HD\tVN:1.4\tSO:unsorted\n"
          "@SQ\tSN:chrA\tLN:100000\n@SQ\tSN:chrB\tLN:50000\n"
          "@RG\tID:rgA\tLB:libA\tSM:s\n@RG\tID:rgB\tLB:libB\tSM:s\n@RG\tID:rgC\tSM:s\n"
          "@PG\tID:bwa\tPN:bwa\tVN:0.7\n@CO\tedge cases\n")
REFS = [("chrA", 100000), ("chrB", 50000)]


def rg(name: str) -> bytes:
    return b"RGZ" + name.encode() + b"\0"


def seq(n: int, rnd: random.Random) -> str:
    return "".join(rnd.choice("ACGT") for _ in range(n))


def quals(n: int, rnd: random.Random, lo=2, hi=40) -> bytes:
    return bytes(rnd.randint(lo, hi) for _ in range(n))


def build_edge_records(seed: int = 11) -> list[bytes]:
    rnd = random.Random(seed)
    R = []

    def pair(name, ref1, pos1, rev1, ref2, pos2, rev2, cig1="50M", cig2="50M", tag=b"", q1=None, q2=None, extra1=0,
             extra2=0):
        l1 = sum(int(x) for x in __import__("re").findall(r"(\d+)[MIS=X]", cig1))
        l2 = sum(int(x) for x in __import__("re").findall(r"(\d+)[MIS=X]", cig2))
        f1 = 0x1 | 0x40 | (0x10 if rev1 else 0) | (0x20 if rev2 else 0) | extra1
        f2 = 0x1 | 0x80 | (0x10 if rev2 else 0) | (0x20 if rev1 else 0) | extra2
        r1 = make_record(name, f1, ref1, pos1, cig1, seq(l1, rnd), q1 if q1 is not None else quals(l1, rnd),
                         mref=ref2, mpos=pos2, tags=tag)
        r2 = make_record(name, f2, ref2, pos2, cig2, seq(l2, rnd), q2 if q2 is not None else quals(l2, rnd),
                         mref=ref1, mpos=pos1, tags=tag)
        return r1, r2

    # 1. a cluster of duplicate pairs with distinct and tied scores, two read groups / libraries
    for i in range(6):
        a, b = pair(f"dupA{i}", 0, 1000, False, 0, 1200, True, tag=rg("rgA"),
                    q1=bytes([30] * 50) if i in (2, 4) else None, q2=bytes([30] * 50) if i in (2, 4) else None)
        R += [a, b]
    for i in range(3):
        a, b = pair(f"dupB{i}", 0, 1000, False, 0, 1200, True, tag=rg("rgB"))
        R += [a, b]
    # 2. fragments (mate unmapped) at a pair's 5' coordinate -> containsPairs: mark unpaired only
    for i in range(3):
        f = 0x1 | 0x40 | 0x8
        R.append(make_record(f"fragU{i}", f, 0, 1000, "50M", seq(50, rnd), quals(50, rnd), mref=0, mpos=1000,
                             tags=rg("rgA")))
        R.append(make_record(f"fragU{i}", 0x1 | 0x80 | 0x4, 0, 1000, "", seq(50, rnd), quals(50, rnd), mapq=0, mref=0,
                             mpos=1000, tags=rg("rgA")))
    # 3. pure fragment cluster (unpaired), clipped so unclipped starts coincide (5S45M at 2005 == 2000)
    R.append(make_record("solo1", 0, 0, 2000, "50M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    R.append(make_record("solo2", 0, 0, 2005, "5S45M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    R.append(make_record("solo3", 0, 0, 2003, "3H50M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    R.append(make_record("solo4", 0, 0, 2000, "50M", seq(50, rnd), bytes([40] * 50), tags=rg("rgA")))
    # 4. reverse fragments: unclipped end with D/N ops and trailing clips
    R.append(make_record("rev1", 0x10, 0, 3000, "20M5D30M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    R.append(make_record("rev2", 0x10, 0, 3000, "20M5N25M5S", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    R.append(make_record("rev3", 0x10, 0, 3010, "45M10S", seq(55, rnd), quals(55, rnd), tags=rg("rgA")))
    # 5. secondary with the same name (untouched, even with 0x400 preset); supplementary counts as primary
    a, b = pair("multi", 0, 4000, False, 0, 4300, True, tag=rg("rgA"))
    R += [a, b]
    R.append(make_record("multi", 0x1 | 0x40 | 0x100 | 0x400, 0, 4000, "50M", seq(50, rnd), quals(50, rnd), mref=0,
                         mpos=4300, tags=rg("rgA")))
    R.append(make_record("multi", 0x1 | 0x40 | 0x800, 1, 500, "30M20S", seq(50, rnd), quals(50, rnd), mref=0, mpos=4300,
                         tags=rg("rgA")))
    a, b = pair("multi2", 0, 4000, False, 0, 4300, True, tag=rg("rgA"))
    R += [a, b]
    # 6. pre-set 0x400 on a unique primary -> cleared
    R.append(make_record("preset", 0x400, 0, 5000, "50M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    # 7. missing qualities (0xFF) -> score wraps in int16 for long reads
    for i in range(3):
        a, b = pair(f"wrap{i}", 0, 6000, False, 0, 6300, True, cig1="150M", cig2="150M", tag=rg("rgA"),
                    q1=bytes([0xFF] * 150) if i == 0 else None, q2=bytes([0xFF] * 150) if i == 0 else None)
        R += [a, b]
    # 8. unmapped reads: refID -1 tail, and placed-unmapped (refID >= 0)
    for i in range(4):
        R.append(make_record(f"unm{i}", 0x4, -1, -1, "", seq(40, rnd), quals(40, rnd), mapq=0, tags=rg("rgA")))
    R.append(make_record("placed", 0x4, 1, 700, "", seq(40, rnd), quals(40, rnd), mapq=0, tags=rg("rgA")))
    # 9. name-prefix ties at one coordinate/strand; equal names differing by flag
    for nm in ["t10", "t1", "t", "t100", "s9"]:
        R.append(make_record(nm, 0, 1, 1000, "40M", seq(40, rnd), quals(40, rnd), tags=rg("rgB")))
    R.append(make_record("same", 0x1 | 0x40 | 0x8, 1, 1100, "40M", seq(40, rnd), quals(40, rnd), tags=rg("rgB")))
    R.append(make_record("same", 0x1 | 0x80 | 0x8, 1, 1100, "40M", seq(40, rnd), quals(40, rnd), tags=rg("rgB")))
    # 10. same name, different RG -> different pair keys; RG absent / unknown / without LB
    for tag in [rg("rgA"), rg("rgB"), rg("rgC"), rg("rgZ"), b""]:
        a, b = pair("samename", 1, 2000, False, 1, 2250, True, tag=tag)
        R += [a, b]
    # 11. inter-contig pairs; read2 earlier than read1 (swap branch); equal coordinates (first stays read1)
    for i in range(3):
        a, b = pair(f"inter{i}", 1, 3000, True, 0, 7000, False, tag=rg("rgA"))
        R += [a, b]
    for i in range(2):
        a, b = pair(f"eq{i}", 0, 8000, False, 0, 8000, True, tag=rg("rgA"))
        R += [b, a]
    # 12. orphan: mate mapped but never present
    R.append(make_record("orphan", 0x1 | 0x40, 0, 1000, "50M", seq(50, rnd), quals(50, rnd), mref=0, mpos=1200,
                         tags=rg("rgA")))
    # 13. tags of every type before RG (FindTag skipping), negative unclipped coordinate
    tags = (b"XAA" + b"q" + b"XBc" + b"\x05" + b"XCs" + struct.pack("<h", -3) + b"XDi" + struct.pack("<i", 7) +
            b"XEf" + struct.pack("<f", 1.5) + b"XFZhello\0" + b"XGBi" + struct.pack("<i", 2) + struct.pack("<ii", 1, 2) +
            rg("rgA"))
    R.append(make_record("tagged1", 0, 0, 2, "10S40M", seq(50, rnd), quals(50, rnd), tags=tags))
    R.append(make_record("tagged2", 0, 0, 0, "8S42M", seq(50, rnd), quals(50, rnd), tags=tags))
    R.append(make_record("tagged3", 0, 0, 2, "10S40M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    # 14. mate "mapped" but mate refID -1 (fragment isPaired() false, still a pair candidate)
    R.append(make_record("odd", 0x1 | 0x40, 0, 9000, "50M", seq(50, rnd), quals(50, rnd), mref=-1, mpos=-1,
                         tags=rg("rgA")))
    R.append(make_record("odd2", 0, 0, 9000, "50M", seq(50, rnd), quals(50, rnd), tags=rg("rgA")))
    rnd.shuffle(R)
    return R
