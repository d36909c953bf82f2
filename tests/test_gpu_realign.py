"""GPU: local realignment through the C ABI.

* oge_realign_scan (the HIP offset-scan kernels: bit-plane k_scan_bp, byte-wise k_realign_scan for
  batches with lower-case/'*' bases) against the oracle's literal findBestOffset restatement on
  random batches, including long consensuses/reads (the byte-wise kernel's LDS-overflow path),
  offsets past the consensus end and negative quality weights (literal early-exit path);
* oge_localrealign (host phases + GPU scan) against the REFERENCE's own outputs (tests/golden/rl_*).
"""
import numpy as np
import pytest

import oracle
from test_realign import RL_CASES, _offsets_of, _ref_lens, check_output, load_rl_case, random_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(8))
def test_gpu_scan_matches_oracle(ctx, seed):
    rng = np.random.default_rng(100 + seed)
    b = random_batch(rng, n_cons=12, reads_per=8, qual_max=(120 if seed % 3 == 0 else 60))
    gi, gs = ctx.realign_scan(*b)
    oi, os_ = oracle.realign_scan(*b)
    assert np.array_equal(gs, os_)
    assert np.array_equal(gi, oi)


@pytest.mark.parametrize("seed", range(8))
def test_gpu_scan_bitplane_path(ctx, seed):
    """Upper-case batches run k_planes + k_scan_bp (2-bit planes); lower case / '*' anywhere in a
    batch sends it to the byte-wise kernel (covered above).  Multi-word reads, offsets past the
    consensus end, zero and negative weights."""
    rng = np.random.default_rng(500 + seed)
    b = random_batch(rng, n_cons=16, reads_per=10, cons_len=(30, 700), read_len=(5, 300), alphabet=b"ACGTN",
                     qual_max=(120 if seed % 2 else 93))
    gi, gs = ctx.realign_scan(*b)
    oi, os_ = oracle.realign_scan(*b)
    assert np.array_equal(gs, os_)
    assert np.array_equal(gi, oi)


def test_gpu_scan_realistic_sizes(ctx):
    rng = np.random.default_rng(7)
    b = random_batch(rng, n_cons=64, reads_per=24, cons_len=(250, 600), read_len=(100, 151), alphabet=b"ACGT",
                     qual_max=41)
    gi, gs = ctx.realign_scan(*b)
    oi, os_ = oracle.realign_scan(*b)
    assert np.array_equal(gs, os_) and np.array_equal(gi, oi)


def test_gpu_scan_big_path(ctx):
    rng = np.random.default_rng(3)
    b1 = random_batch(rng, n_cons=2, reads_per=3, cons_len=(41000, 43000), read_len=(60, 90), alphabet=b"ACGT")
    b2 = random_batch(rng, n_cons=2, reads_per=2, cons_len=(4500, 5200), read_len=(4200, 4400), alphabet=b"ACGTN")
    for b in (b1, b2):
        gi, gs = ctx.realign_scan(*b)
        oi, os_ = oracle.realign_scan(*b)
        assert np.array_equal(gs, os_) and np.array_equal(gi, oi)


def test_gpu_scan_rejects_bad_pairs(ctx):
    rng = np.random.default_rng(1)
    cons, co, bases, quals, ro, pairs = random_batch(rng, n_cons=2, reads_per=2)
    bad = pairs.copy()
    bad[0, 0] = 99  # consensus index out of range
    from openge_amd import lib as L
    with pytest.raises(L.OgeError, match="out of range"):
        ctx.realign_scan(cons, co, bases, quals, ro, bad)


@pytest.mark.parametrize("name", RL_CASES)
def test_gpu_localrealign_matches_reference(ctx, tmp_path, name):
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    out, oo, stats = ctx.localrealign(h, recs, offs, len(offs) - 1, fa, iv)
    check_output(meta, arrays, out, oo)
    assert stats["scan_pairs"] > 0 and stats["intervals_cleaned"] > 0


@pytest.mark.parametrize("world", [3, 8])
def test_gpu_contig_sharded_realign_equals_reference(ctx, tmp_path, world):
    """Multi-GPU realign (openge_amd/realign_shard.py): each rank's contig range through the C ABI,
    concatenated, equals the reference's single-process output."""
    import realign_util as R
    from openge_amd import realign_shard as RS
    meta, arrays, h, recs, offs, fa, iv = load_rl_case("rl_c5_2k", tmp_path)
    n = len(offs) - 1
    sl = RS.contig_slices(recs, offs, n, _ref_lens(h), world)
    parts = []
    for r, (lo, hi) in enumerate(sl):
        out, oo, st = RS.localrealign_slice(ctx, h, recs, offs, lo, hi, fa, iv, None, last=(r == world - 1))
        parts.append(bytes(out[:int(oo[-1])]))
    whole = b"".join(parts)
    d = R.digest(np.frombuffer(whole + b"\0" * 16, np.uint8), _offsets_of(whole))
    assert d["stream_sha256"] == meta["stream_sha256"]


def _realign_both(ctx, monkeypatch, h, recs, offs, fa, iv):
    monkeypatch.setenv("OGE_REALIGN_DEVICE_PREP", "0")
    out0, oo0, st0 = ctx.localrealign(h, recs, offs, len(offs) - 1, fa, iv)
    monkeypatch.setenv("OGE_REALIGN_DEVICE_PREP", "1")
    out1, oo1, st1 = ctx.localrealign(h, recs, offs, len(offs) - 1, fa, iv)
    monkeypatch.delenv("OGE_REALIGN_DEVICE_PREP")
    assert st0["device_prep"] == 0 and st1["device_prep"] == 1
    b0, b1 = bytes(out0[:int(oo0[-1])]), bytes(out1[:int(oo1[-1])])
    assert b0 == b1 and list(oo0) == list(oo1)
    for k in ("scan_pairs", "scan_ops", "intervals_cleaned", "reads_realigned"):
        assert st0[k] == st1[k], k
    return st1


@pytest.mark.parametrize("name", RL_CASES)
def test_gpu_device_consensus_generation_equals_host(ctx, tmp_path, monkeypatch, name):
    """Phase B on the device (realign_prep.hip: left-alignment, mismatch sums, consensus set, batch) and on
    the host threads (realign.cpp) give the same records, the same scan pairs and compare counts -- on the
    reference's own rl_* cases (the default path is pinned to them by test_gpu_localrealign_matches_reference)."""
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    st = _realign_both(ctx, monkeypatch, h, recs, offs, fa, iv)
    assert st["prep_device_intervals"] > 0


@pytest.mark.parametrize("seed,knobs", [
    (11, {}),
    (12, {"clip_ppm": 300000, "n_ppm": 20000, "lower_ppm": 50000}),
    (13, {"gapped_ppm": 200000, "alt_indel_ppm": 300000, "noindel_ppm": 200000}),
    (14, {"qual_min": 0, "qual_max": 93, "dup_ppm": 200000, "mapq0_ppm": 100000, "clip_ppm": 100000}),
])
def test_gpu_device_consensus_generation_stress(ctx, tmp_path, monkeypatch, seed, knobs):
    """Synthetic C5-shaped sets with soft clips, N and lower-case bases, gapped (N) reads, competing indels,
    a wide quality range, duplicates: device and host phase B give the same output (qualities >= 95, whose
    weights are negative, are in the rl_qual golden)."""
    from openge_amd import lib as L
    p = L.realign_synth_params(n_intervals=1500, seed=seed, **knobs)
    fa, iv, bam = L.synth_realign(p, tmp_path, level=1)
    b = L.Bam(bam)
    offs = np.append(b.offs, np.uint64(b.recs.size))
    st = _realign_both(ctx, monkeypatch, b.header_text, b.recs, offs, fa, iv)
    assert st["prep_device_intervals"] > 0 and st["scan_pairs"] > 0


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("name", ["rl_short", "rl_c5_2k"])
def test_gpu_realign_interval_sharded_over_contexts(ctx, tmp_path, name, G):
    """oge_localrealign_multi: phase B + C over G contexts (one device here; G devices on a node) by interval
    ranges -- inside the one contig of rl_short -- equals the reference's output."""
    from openge_amd import lib as L
    meta, arrays, h, recs, offs, fa, iv = load_rl_case(name, tmp_path)
    more = [L.Context(0) for _ in range(G - 1)]
    try:
        out, oo, st = ctx.localrealign(h, recs, offs, len(offs) - 1, fa, iv, more=more)
        check_output(meta, arrays, out, oo)
        assert st["prep_devices"] == G and all(st[f"prep_rank{g}_intervals"] > 0 for g in range(G))
    finally:
        for c in more:
            c.close()
