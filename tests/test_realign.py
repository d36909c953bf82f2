"""CPU: local realignment.

* the oracle's literal findBestOffset restatement against an independent closed form (min over
  (score, visit rank)) -- the formula the HIP kernel implements;
* the product's host realignment phases (binning, consensus generation, decisions, CIGAR/tag surgery,
  mate fixing), run with the oracle scan in place of the GPU kernel, against the REFERENCE's own
  outputs (tests/golden/rl_*, made by oracle/_ref from the reference sources).
"""
import hashlib
import json

import numpy as np
import pytest

import bamutil
import oracle
import realign_util as R
from goldens import GOLDEN
from openge_amd import lib as L

RL_CASES = ["rl_small", "rl_edge", "rl_qual", "rl_short", "rl_c5_2k"]
REGULAR = set(b"ACGTacgt*")


def closed_form(cons: bytes, read: bytes, quals: bytes, orig: int, max_start: int):
    """S(k) = sum of w_i over regular mismatches + 99 per base past the end; argmin of (S, rank)."""
    C, Lr = len(cons), len(read)
    w = [((q + 33) & 0xFF) - (256 if ((q + 33) & 0xFF) > 127 else 0) - 33 for q in quals]
    best = None
    for k in range(max(orig, max_start) + 1):
        s = 0
        for i in range(Lr):
            if k + i >= C:
                s += 99
            elif read[i] in REGULAR and cons[k + i] in REGULAR and read[i] != cons[k + i]:
                s += w[i]
        rank = 0 if k == orig else (k + 1 if k < orig else k)
        if best is None or (s, rank) < best[0]:
            best = ((s, rank), k)
    return best[1], best[0][0]


def random_batch(rng, n_cons=6, reads_per=5, cons_len=(20, 90), read_len=(5, 40), alphabet=b"ACGTN*acgt",
                 qual_max=60):
    cons, co, bases, quals, ro, pairs = [], [0], [], [], [0], []
    for c in range(n_cons):
        s = rng.choice(list(b"ACGT" if rng.random() < .5 else alphabet), rng.integers(*cons_len)).astype(np.uint8).tobytes()
        cons.append(s)
        co.append(co[-1] + len(s))
        for _ in range(reads_per):
            ln = int(rng.integers(*read_len))
            if rng.random() < .5 and len(s) > ln:  # a read that matches somewhere, with a few errors
                k = int(rng.integers(0, len(s) - ln))
                r = bytearray(s[k:k + ln].upper())
                for _ in range(int(rng.integers(0, 3))):
                    r[int(rng.integers(0, ln))] = int(rng.choice(list(b"ACGT")))
                r = bytes(r)
            else:
                r = rng.choice(list(alphabet), ln).astype(np.uint8).tobytes()
            q = bytes(rng.integers(0, qual_max + 1, ln).astype(np.uint8))
            bases.append(r)
            quals.append(q)
            ro.append(ro[-1] + ln)
            orig = int(rng.integers(0, len(s) + 5))
            ms = len(s) - ln - int(rng.integers(-3, 4))
            pairs.append([c, len(ro) - 2, orig, ms])
    u8 = lambda bs: np.frombuffer(b"".join(bs) + b"\0", np.uint8)[:-1].copy()
    assert co[-1] == sum(map(len, cons)) and ro[-1] == sum(map(len, bases))
    return (u8(cons), np.array(co, np.uint64), u8(bases), u8(quals), np.array(ro, np.uint64),
            np.array(pairs, np.int32))


@pytest.mark.parametrize("seed", range(6))
def test_oracle_scan_equals_closed_form(built, seed):
    """With every weight >= 0 the reference's early exits cannot change the answer, so it equals the
    minimum of (score, visit rank).  Qualities >= 95 make weights negative ((signed char)(q + 33) - 33)
    and the early exits then matter; the kernel runs the literal scan for such reads."""
    rng = np.random.default_rng(seed)
    b = random_batch(rng, qual_max=120 if seed % 2 else 45)
    bi, bs = oracle.realign_scan(*b)
    cons, co, bases, quals, ro, pairs = b
    for p, (c, r, orig, ms) in enumerate(pairs):
        if quals[ro[r]:ro[r + 1]].max(initial=0) >= 95:
            continue  # negative weights: only the literal early-exit semantics apply (GPU test covers it)
        k, s = closed_form(cons[co[c]:co[c + 1]].tobytes(), bases[ro[r]:ro[r + 1]].tobytes(),
                           quals[ro[r]:ro[r + 1]].tobytes(), int(orig), int(ms))
        assert (bi[p], bs[p]) == (k, s), (p, c, r, orig, ms)


def load_rl_case(name, tmp_path):
    meta = json.loads((GOLDEN / name / "meta.json").read_text())
    arrays = dict(np.load(GOLDEN / name / "arrays.npz")) if (GOLDEN / name / "arrays.npz").exists() else {}
    p = L.realign_synth_params(**{k: v for k, v in meta["spec"].items()})
    fa, iv, bam = L.synth_realign(p, tmp_path)
    h, _, recs, offs = bamutil.read_bam(bam)
    inp = meta["input"]
    assert hashlib.sha256(open(fa, "rb").read()).hexdigest() == inp["fasta_sha256"]
    assert hashlib.sha256(open(iv, "rb").read()).hexdigest() == inp["intervals_sha256"]
    assert R.digest(recs, offs)["stream_sha256"] == inp["records_sha256"] and h == inp["header"]
    recs = np.concatenate([recs, np.zeros(16, np.uint8)])
    offs = np.append(offs, np.uint64(len(recs) - 16))
    return meta, arrays, h, recs, offs, fa, iv


def check_output(meta, arrays, out, oo):
    d = R.digest(out, oo[:-1])
    assert len(oo) - 1 == meta["n_out"]
    if d["stream_sha256"] != meta["stream_sha256"]:
        if "per_record" in arrays:
            bad = np.nonzero(d["per_record"] != arrays["per_record"])[0]
            k = int(bad[0])
            raise AssertionError(f"{len(bad)} records differ from the reference output; first at {k}: "
                                 f"{bamutil.fields(bamutil.rec_bytes(out, oo[k]))}")
        raise AssertionError("output stream differs from the reference output")


@pytest.mark.parametrize("name", RL_CASES)
def test_host_realign_phases_match_reference(built, tmp_path, name):
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    out, oo = R.realign_cpu(h, recs, offs, len(offs) - 1, fa, iv)
    check_output(meta, arrays, out, oo)


@pytest.mark.parametrize("max_records", [0, 7, 60, 400])
def test_parallel_mate_fixing_equals_one_writer(built, tmp_path, max_records):
    """Per-contig writer segments (run in parallel) against one writer over the whole stream, with
    MAX_RECORDS_IN_MEMORY small enough to force flushes inside segments and at contig boundaries
    (the latter sends the product to its sequential fallback)."""
    meta, arrays, h, recs, offs, fa, iv = load_rl_case("rl_c5_2k", tmp_path)
    n = len(offs) - 1
    st_par, st_seq = {}, {}
    a = R.realign_cpu(h, recs, offs, n, fa, iv, threads=4, max_records=max_records, stats=st_par)
    b = R.realign_cpu(h, recs, offs, n, fa, iv, threads=4, max_records=max_records, mate_sequential=True, stats=st_seq)
    assert st_seq["mate_segments"] == 1
    if max_records == 0:
        assert st_par["mate_segments"] > 1
        check_output(meta, arrays, *a)
    assert a[1].tolist() == b[1].tolist()
    assert a[0].tobytes() == b[0].tobytes()


def _ref_lens(header):
    return [int(dict(x.split(":", 1) for x in ln.split("\t")[1:])["LN"]) for ln in header.splitlines()
            if ln.startswith("@SQ")]


@pytest.mark.parametrize("world", [2, 3, 5])
def test_contig_sharded_realign_equals_whole(built, tmp_path, world):
    """realignment of contig-range shards (openge_amd/realign_shard.py), concatenated in
    rank order, is the single-process output (here: the reference's own output)."""
    from openge_amd import realign_shard as RS
    meta, arrays, h, recs, offs, fa, iv = load_rl_case("rl_c5_2k", tmp_path)
    n = len(offs) - 1
    sl = RS.contig_slices(recs, offs, n, _ref_lens(h), world)
    assert sl[0][0] == 0 and sl[-1][1] == n and all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
    parts, stats = [], []
    for lo, hi in sl:
        st = {}
        out, oo = R.realign_cpu(h, recs, offs[lo:hi + 1], hi - lo, fa, iv, stats=st)
        parts.append(bytes(out[:oo[-1]]))
        stats.append(st)
    assert all(st["tail_waiting"] < 150000 for st in stats[:-1])
    whole = b"".join(parts)
    d = R.digest(np.frombuffer(whole + b"\0" * 16, np.uint8), _offsets_of(whole))
    assert d["stream_sha256"] == meta["stream_sha256"]


def _offsets_of(stream: bytes) -> np.ndarray:
    o, out = 0, []
    while o < len(stream):
        out.append(o)
        o += 4 + int.from_bytes(stream[o:o + 4], "little")
    return np.array(out, np.uint64)


def test_realign_synth_is_deterministic(built, tmp_path):
    p = L.realign_synth_params(n_intervals=40, n_ref=2, seed=5)
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    A = L.synth_realign(p, tmp_path / "a", threads=1)
    B = L.synth_realign(p, tmp_path / "b", threads=5)
    for x, y in zip(A[:2], B[:2]):
        assert open(x, "rb").read() == open(y, "rb").read()
    assert bamutil.read_bam(A[2])[2].tobytes() == bamutil.read_bam(B[2])[2].tobytes()
