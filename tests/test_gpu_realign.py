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
from test_realign import RL_CASES, check_output, load_rl_case, random_batch

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
