"""Test-side BAM helpers, independent of the product codec (pure Python + zlib/gzip).

Used to read the reference oracle's outputs, to craft edge-case records and to cross-check the
product's BAM reader/writer.
"""
from __future__ import annotations

import gzip
import struct
import zlib

import numpy as np


def read_bam(path) -> tuple[str, list[tuple[str, int]], np.ndarray, np.ndarray]:
    """-> (header_text, refs, recs u8, offs u64[n]) with records exactly as in the stream."""
    with open(path, "rb") as f:
        raw = gzip.decompress(f.read())
    assert raw[:4] == b"BAM\1", "not a BAM"
    (lt,) = struct.unpack_from("<i", raw, 4)
    text = raw[8:8 + lt].decode(errors="replace")
    p = 8 + lt
    (nref,) = struct.unpack_from("<i", raw, p)
    p += 4
    refs = []
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", raw, p)
        name = raw[p + 4:p + 4 + ln - 1].decode()
        (rl,) = struct.unpack_from("<i", raw, p + 4 + ln)
        refs.append((name, rl))
        p += 8 + ln
    recs = np.frombuffer(raw[p:], dtype=np.uint8).copy()
    offs = []
    q = 0
    while q < len(recs):
        offs.append(q)
        (bs,) = struct.unpack_from("<I", recs, q)
        q += 4 + bs
    return text, refs, recs, np.array(offs, dtype=np.uint64)


def rec_bytes(recs: np.ndarray, off: int) -> bytes:
    (bs,) = struct.unpack_from("<I", recs, int(off))
    return recs[int(off):int(off) + 4 + bs].tobytes()


def fields(rb: bytes) -> dict:
    refid, pos, lname, mapq, bin_, ncig, flag, lseq, mref, mpos, tlen = struct.unpack_from("<iiBBHHHiiii", rb, 4)
    name = rb[36:36 + lname - 1].decode()
    cig = struct.unpack_from(f"<{ncig}I", rb, 36 + lname)
    return dict(refid=refid, pos=pos, mapq=mapq, bin=bin_, flag=flag, lseq=lseq, mref=mref, mpos=mpos, tlen=tlen,
                name=name, cigar=cig)


def match_key(rb: bytes) -> bytes:
    """Record identity ignoring the bin field (recomputed on write) and the 0x400 bit."""
    b = bytearray(rb)
    b[14:16] = b"\0\0"
    b[19] &= ~0x04 & 0xFF  # flag bit 0x400 lives in the high byte of the flag (bytes 18-19)
    return bytes(b)


def perm_of(out_recs, out_offs, in_recs, in_offs) -> np.ndarray:
    """Input index of every output record (records must be unique under match_key)."""
    idx = {}
    for i, o in enumerate(in_offs):
        k = match_key(rec_bytes(in_recs, o))
        idx.setdefault(k, []).append(i)
    perm = np.empty(len(out_offs), dtype=np.uint32)
    for k, o in enumerate(out_offs):
        lst = idx[match_key(rec_bytes(out_recs, o))]
        perm[k] = lst.pop(0)
    return perm


def flags_of(recs, offs) -> np.ndarray:
    return np.array([struct.unpack_from("<H", recs, int(o) + 18)[0] for o in offs], dtype=np.uint16)


CIG = {c: i for i, c in enumerate("MIDNSHP=X")}


def make_record(name: str, flag: int, refid: int, pos: int, cigar: str = "", seq: str = "", qual=None, mapq: int = 60,
                mref: int = -1, mpos: int = -1, tlen: int = 0, tags: bytes = b"") -> bytes:
    ops = []
    num = ""
    for ch in cigar:
        if ch.isdigit():
            num += ch
        else:
            ops.append((int(num) << 4) | CIG[ch])
            num = ""
    lseq = len(seq)
    codes = {"=": 0, "A": 1, "C": 2, "M": 3, "G": 4, "R": 5, "S": 6, "V": 7, "T": 8, "W": 9, "Y": 10, "H": 11,
             "K": 12, "D": 13, "B": 14, "N": 15}
    sb = bytearray((lseq + 1) // 2)
    for i, ch in enumerate(seq):
        c = codes[ch.upper()]
        if i % 2 == 0:
            sb[i // 2] |= c << 4
        else:
            sb[i // 2] |= c
    if qual is None:
        qual = bytes([30] * lseq)
    nm = name.encode() + b"\0"
    body = struct.pack("<iiBBHHHiiii", refid, pos, len(nm), mapq, 4680, len(ops), flag, lseq, mref, mpos, tlen)
    body += nm + b"".join(struct.pack("<I", o) for o in ops) + bytes(sb) + bytes(qual) + tags
    return struct.pack("<I", len(body)) + body


def pack_records(recs: list[bytes]) -> tuple[np.ndarray, np.ndarray]:
    offs, acc = [], 0
    for r in recs:
        offs.append(acc)
        acc += len(r)
    return np.frombuffer(b"".join(recs) + b"\0" * 16, dtype=np.uint8).copy(), np.array(offs + [acc], dtype=np.uint64)


def bgzf_blocks(data: bytes, level: int = 6, payload: int = 65280) -> bytes:
    out = bytearray()
    for i in range(0, max(len(data), 1), payload):
        chunk = data[i:i + payload]
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        c = co.compress(chunk) + co.flush()
        bsize = 18 + len(c) + 8
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, ord("B"), ord("C"), 2, bsize - 1)
        out += c + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    c = co.compress(b"") + co.flush()
    out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, ord("B"), ord("C"), 2, 18 + len(c) + 8 - 1)
    out += c + struct.pack("<II", 0, 0)
    return bytes(out)


def write_bam_py(path, header_text: str, refs: list[tuple[str, int]], records: list[bytes]) -> None:
    ht = header_text.encode()
    body = b"BAM\1" + struct.pack("<i", len(ht)) + ht + struct.pack("<i", len(refs))
    for name, ln in refs:
        nb = name.encode() + b"\0"
        body += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
    body += b"".join(records)
    with open(path, "wb") as f:
        f.write(bgzf_blocks(body))
