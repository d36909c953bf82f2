"""An independent restatement of MarkDuplicates' duplicate set (-v --nosplit semantics) in torch tensor
operations, for checking the product's FLAG 0x400 bits at sizes the C oracle cannot reach (the 300M-read
bench workload, on the GPU) -- TEST INFRASTRUCTURE, no product code.

Input: a coordinate-sorted record stream (buf u8, off i64[n]: the output of sort + dedup) and its header
text.  Output: the 0x400 bit MarkDuplicates gives every primary record (record index = stream position,
the -v semantics), computed from the other fields only (the bit itself is ignored), following
alg/mark_duplicates.cpp:
  D1 buildReadEnds :147-164 -- mapped (0x4 clear), refID != -1, primary (0x100 clear; 0x800 counts):
     5' coordinate = reverse ? pos + refLen - 1 + trailing S/H : pos - leading S/H (:88-129, refLen over
     M/D/N/=/X :44-61); score = int16 sum of the quality bytes >= 15 (:135-144); library = the LB of the
     record's RG (:282-318, "Unknown Library" otherwise)
  D2 mate join :200-245 -- paired with the mate mapped: ends of one RG:name pair up consecutively in
     index order (ReadEndsMap put / remove); read1 = the end with the smaller (seq, coord), ties keep the
     first; orientation from both ends' strands; score = int16(score1 + score2)
  D4 :326-414,488-540 -- pair chunks = equal (lib, r1Seq, r1Coord, orient, r2Seq, r2Coord), best = the
     first strict max of score in (read1 index, read2 index) order, every other pair marks both ends;
     fragment chunks = equal (lib, r1Seq, r1Coord, strand) over every ReadEnds, processed when larger
     than one and holding an unpaired end: with a paired end present mark the unpaired ends, else keep
     the first strict max (index order) and mark the rest.  A fragment end is "paired" when
     read2Sequence = mateRefID != -1.
The checker hashes read names (two independent 64-bit hashes + the length, compared as separate keys)
instead of comparing them.
"""
from __future__ import annotations

import torch

_M = 1 << 64


def _u8(buf, idx):
    return buf[idx].to(torch.int64)


def _u16(buf, idx):
    return _u8(buf, idx) | (_u8(buf, idx + 1) << 8)


def _u32(buf, idx):
    return _u8(buf, idx) | (_u8(buf, idx + 1) << 8) | (_u8(buf, idx + 2) << 16) | (_u8(buf, idx + 3) << 24)


def _i32(buf, idx):
    v = _u32(buf, idx)
    return torch.where(v >= (1 << 31), v - (1 << 32), v)


def _rg_libs(header_text: str) -> dict[bytes, str]:
    out = {}
    for ln in header_text.splitlines():
        if ln.startswith("@RG"):
            f = dict(x.split(":", 1) for x in ln.split("\t")[1:] if ":" in x)
            if "ID" in f:
                out[f["ID"].encode()] = f.get("LB", "")
    return out


def _hash_bytes(buf, start, length, maxlen, cap):
    """two 64-bit polynomial hashes of buf[start : start + length] (per record; length <= maxlen), int64 wrap"""
    h1 = torch.full_like(start, 0x6C62272E07BB0142)  # FNV-1a 64 (as int64)
    h2 = torch.full_like(start, 7)
    for k in range(maxlen):
        m = k < length
        b = _u8(buf, torch.where(m, start + k, torch.zeros_like(start)).clamp_(max=cap))
        h1 = torch.where(m, (h1 ^ b) * 0x100000001B3, h1)
        h2 = torch.where(m, (h2 + b + 1) * 0x5851F42D4C957F2D, h2)
    return h1, h2


def _rg_of(buf, off, end, tag0, cap):
    """(found, hash1, hash2, length) of each record's RG:Z value, by a vectorised walk of the aux tags"""
    n = off.numel()
    cur = tag0.clone()
    found = torch.zeros(n, dtype=torch.bool, device=off.device)
    rs = torch.zeros_like(off)
    rl = torch.zeros_like(off)
    active = cur + 3 <= end
    for _ in range(256):
        if not bool(active.any()):
            break
        c = torch.where(active, cur, torch.zeros_like(cur))
        t0, t1, ty = _u8(buf, c), _u8(buf, c + 1), _u8(buf, c + 2)
        size = torch.full_like(cur, -1)
        for chs, sz in ((b"AcC", 1), (b"sS", 2), (b"iIf", 4)):
            for ch in chs:
                size = torch.where(ty == ch, torch.full_like(size, 3 + sz), size)
        isz = (ty == ord("Z")) | (ty == ord("H"))
        if bool((active & isz).any()):  # string length: the first NUL from c + 3
            ln = torch.full_like(cur, -1)
            for k in range(2048):
                pend = active & isz & (ln < 0)
                if not bool(pend.any()):
                    break
                q = torch.where(pend, c + 3 + k, torch.zeros_like(c)).clamp_(max=cap)
                ln = torch.where(pend & (_u8(buf, q) == 0), torch.full_like(ln, k), ln)
            size = torch.where(isz, 3 + ln + 1, size)
            is_rg = active & (t0 == ord("R")) & (t1 == ord("G")) & (ty == ord("Z")) & ~found
            rs = torch.where(is_rg, c + 3, rs)
            rl = torch.where(is_rg, ln, rl)
            found = found | is_rg
        isb = ty == ord("B")
        if bool((active & isb).any()):
            st = _u8(buf, torch.where(active & isb, c + 3, torch.zeros_like(c)))
            es = torch.ones_like(st)
            for ch, sz in ((b"sS", 2), (b"iIf", 4)):
                for x in ch:
                    es = torch.where(st == x, torch.full_like(es, sz), es)
            cnt = _u32(buf, torch.where(active & isb, c + 4, torch.zeros_like(c)))
            size = torch.where(isb, 8 + cnt * es, size)
        bad = active & (size < 0)
        assert not bool(bad.any()), "unknown aux tag type"
        cur = torch.where(active, cur + size, cur)
        active = active & (cur + 3 <= end)
    return found, rs, rl


def expected_dups(buf: torch.Tensor, off: torch.Tensor, header_text: str, debug: dict | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """-> (primary mask, expected 0x400 bit) per record of the sorted stream.  debug (a dict) receives the
    pair arrays (read1 / read2 record, chunk keys, score, group id, in chunk order) and per-record
    coordinate / score / library."""
    dev = off.device
    n = off.numel()
    cap = buf.numel() - 1
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    bsz = _i32(buf, off)
    end = off + 4 + bsz
    ref, pos = _i32(buf, off + 4), _i32(buf, off + 8)
    lname, ncig, flag = _u8(buf, off + 12), _u16(buf, off + 16), _u16(buf, off + 18)
    lseq, mref = _i32(buf, off + 20), _i32(buf, off + 24)
    rev = (flag >> 4) & 1
    primary = (flag & 0x100) == 0
    ends = ((flag & 0x4) == 0) & (ref != -1) & primary          # buildReadEnds is called
    cand = ends & ((flag & 0x1) != 0) & ((flag & 0x8) == 0)     # the mate join
    frag_paired = cand & (mref != -1)                           # read2Sequence = mateRefID != -1
    # CIGAR: reference length, leading / trailing clips
    cig0 = off + 36 + lname
    reflen = torch.zeros_like(off)
    lead = torch.zeros_like(off)
    trail = torch.zeros_like(off)
    seen = torch.zeros(n, dtype=torch.bool, device=dev)
    for k in range(int(ncig.max().item()) if n else 0):
        m = k < ncig
        w = _u32(buf, torch.where(m, cig0 + 4 * k, torch.zeros_like(cig0)))
        op, ln = w & 15, w >> 4
        clip = (op == 4) | (op == 5)
        reflen += torch.where(m & ((op == 0) | (op == 2) | (op == 3) | (op == 7) | (op == 8)), ln, 0)
        lead += torch.where(m & clip & ~seen, ln, 0)
        trail = torch.where(m, torch.where(clip, trail + ln, torch.zeros_like(trail)), trail)
        seen = seen | (m & ~clip)
    coord = torch.where(rev == 1, pos + reflen - 1 + trail, pos - lead)
    # score: int16 sum of quality bytes >= 15
    q0 = cig0 + 4 * ncig + (lseq + 1) // 2
    score = torch.zeros_like(off)
    for k in range(int(lseq.max().item()) if n else 0):
        m = k < lseq
        b = _u8(buf, torch.where(m, q0 + k, torch.zeros_like(q0)))
        score += torch.where(m & (b >= 15), b, 0)
    score = ((score + 32768) % 65536) - 32768
    # library of the record's RG
    found, rs, rl = _rg_of(buf, off, end, q0 + lseq, cap)
    rh1, rh2 = _hash_bytes(buf, rs, torch.where(found, rl, torch.zeros_like(rl)), 64, cap)
    libs = _rg_libs(header_text)
    lib_ids: dict[str, int] = {}
    lib = torch.zeros_like(off)  # 0 = "Unknown Library" unless a header RG names another
    unknown = lib_ids.setdefault("Unknown Library", 0)
    for rg, lb in libs.items():
        t = torch.tensor(list(rg), dtype=torch.uint8, device=dev)
        h1, h2 = _hash_bytes(t, torch.zeros(1, dtype=torch.int64, device=dev), torch.tensor([len(rg)], device=dev),
                             len(rg), len(rg) - 1 if len(rg) else 0)
        lid = lib_ids.setdefault(lb if lb else "Unknown Library", len(lib_ids))
        hit = found & (rl == len(rg)) & (rh1 == h1) & (rh2 == h2)
        lib = torch.where(hit, torch.full_like(lib, lid), lib)
    assert unknown == 0 and len(lib_ids) < 32
    dup = torch.zeros(n, dtype=torch.bool, device=dev)
    assert int(ref.max().item()) < (1 << 24) if n else True

    # ---- D2: pairs.  key RG:name (hash of the RG value and of the name), consecutive occurrences pair up
    ci = torch.nonzero(cand).squeeze(1)
    if ci.numel():
        # the key RG:name as four sort keys (name hashes and length, RG hash): every one must be equal --
        # never folded into one word (r05: names differing in their last digit collided when the two name
        # hashes were XOR-ed together, and the restatement paired ends of different names)
        nh1, nh2 = _hash_bytes(buf, off[ci] + 36, lname[ci] - 1, int(lname.max().item()), cap)
        k_rg = torch.where(found[ci], rh1[ci] ^ (rl[ci] << 40), torch.full_like(ci, -1))
        k_rg2 = torch.where(found[ci], rh2[ci], torch.full_like(ci, -1))
        k_nm = nh1
        k_nm2 = nh2 ^ lname[ci]
        o = torch.argsort(k_nm2, stable=True)  # ci is in index order: stable sorts keep it within a key
        o = o[torch.argsort(k_nm[o], stable=True)]
        o = o[torch.argsort(k_rg2[o], stable=True)]
        o = o[torch.argsort(k_rg[o], stable=True)]
        s = ci[o]
        kn, kn2, kr, kr2 = k_nm[o], k_nm2[o], k_rg[o], k_rg2[o]
        del o, k_nm, k_nm2, k_rg, k_rg2, nh1, nh2
        newk = torch.ones_like(s, dtype=torch.bool)
        newk[1:] = (kn[1:] != kn[:-1]) | (kn2[1:] != kn2[:-1]) | (kr[1:] != kr[:-1]) | (kr2[1:] != kr2[:-1])
        start = torch.cummax(torch.where(newk, torch.arange(s.numel(), device=dev), torch.zeros_like(s)), 0).values
        rank = torch.arange(s.numel(), device=dev) - start
        nxt_same = torch.zeros_like(newk)
        nxt_same[:-1] = ~newk[1:]
        first = (rank % 2 == 0) & nxt_same  # the first end of a completed pair; its partner is next
        a = s[torch.nonzero(first).squeeze(1)]
        b = s[torch.nonzero(first).squeeze(1) + 1]
        del s, kn, kn2, kr, kr2, newk, start, rank, nxt_same, first
        # read1 = a unless b's (seq, coord) is smaller
        keep = (ref[b] > ref[a]) | ((ref[b] == ref[a]) & (coord[b] >= coord[a]))
        r1 = torch.where(keep, a, b)
        r2 = torch.where(keep, b, a)
        orient = rev[r1] * 2 + rev[r2]
        psc = ((score[a] + score[b] + 32768) % 65536) - 32768
        plib = lib[a]
        k1 = (plib << 58) | (ref[r1] << 33) | ((coord[r1] + (1 << 31)) << 1)
        k2 = (orient << 58) | (ref[r2] << 33) | ((coord[r2] + (1 << 31)) << 1)
        assert bool(((coord + (1 << 31)) >= 0).all()) and bool(((coord + (1 << 31)) < (1 << 32)).all())
        o = torch.argsort(r2, stable=True)
        o = o[torch.argsort(r1[o], stable=True)]
        o = o[torch.argsort(k2[o], stable=True)]
        o = o[torch.argsort(k1[o], stable=True)]
        k1, k2, psc, r1, r2 = k1[o], k2[o], psc[o], r1[o], r2[o]
        del o, a, b, keep, orient, plib
        newg = torch.ones_like(k1, dtype=torch.bool)
        newg[1:] = (k1[1:] != k1[:-1]) | (k2[1:] != k2[:-1])
        gid = torch.cumsum(newg.to(torch.int64), 0) - 1
        G = int(gid[-1].item()) + 1
        gmax = torch.full((G,), -(1 << 20), dtype=torch.int64, device=dev).scatter_reduce(0, gid, psc, "amax")
        p = torch.arange(k1.numel(), device=dev)
        cand_best = torch.where(psc == gmax[gid], p, torch.full_like(p, 1 << 62))
        best = torch.full((G,), 1 << 62, dtype=torch.int64, device=dev).scatter_reduce(0, gid, cand_best, "amin")
        lose = p != best[gid]
        dup[r1[lose]] = True
        dup[r2[lose]] = True
        if debug is not None:
            debug.update(pr1=r1, pr2=r2, pk1=k1, pk2=k2, psc=psc, pgid=gid)
        del k1, k2, psc, r1, r2, newg, gid, gmax, p, cand_best, best, lose
    if debug is not None:
        debug.update(coord=coord, score=score, lib=lib, ends=ends, cand=cand, frag_paired=frag_paired)
    # ---- D4 fragments: every ReadEnds
    fi = torch.nonzero(ends).squeeze(1)
    if fi.numel():
        fk = (lib[fi] << 58) | (ref[fi] << 33) | ((coord[fi] + (1 << 31)) << 1) | rev[fi]
        o = torch.argsort(fk, stable=True)  # index order within a chunk (the chunk's order for the
        s, fk = fi[o], fk[o]                # unpaired-only case, the only one where it matters)
        del o
        newg = torch.ones_like(fk, dtype=torch.bool)
        newg[1:] = fk[1:] != fk[:-1]
        gid = torch.cumsum(newg.to(torch.int64), 0) - 1
        G = int(gid[-1].item()) + 1
        pr = frag_paired[s].to(torch.int64)
        size = torch.zeros(G, dtype=torch.int64, device=dev).scatter_add(0, gid, torch.ones_like(gid))
        npair = torch.zeros(G, dtype=torch.int64, device=dev).scatter_add(0, gid, pr)
        has_pairs = npair[gid] > 0
        has_frags = (size - npair)[gid] > 0
        proc = (size[gid] > 1) & has_frags
        sc = score[s]
        gmax = torch.full((G,), -(1 << 20), dtype=torch.int64, device=dev).scatter_reduce(0, gid, sc, "amax")
        p = torch.arange(s.numel(), device=dev)
        cand_best = torch.where(sc == gmax[gid], p, torch.full_like(p, 1 << 62))
        best = torch.full((G,), 1 << 62, dtype=torch.int64, device=dev).scatter_reduce(0, gid, cand_best, "amin")
        mark = proc & torch.where(has_pairs, pr == 0, p != best[gid])
        dup[s[mark]] = True
    return primary, dup
