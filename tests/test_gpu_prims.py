"""GPU: the device radix sort every pipeline sort runs on (onesweep, decoupled look-back), against
numpy's stable sort on the masked key bits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sort(ctx, keys, vals, mask):
    import torch
    dev = torch.device("cuda", 0)
    n = len(keys)
    k = torch.from_numpy(keys.view(np.int64)).to(dev)
    kt = torch.empty_like(k)
    v = vt = None
    if vals is not None:
        v = torch.from_numpy(vals.view(np.int32)).to(dev)
        vt = torch.empty_like(v)
    p = lambda t: t.data_ptr() if t is not None else None
    in_tmp = ctx.radix_sort_pairs_dev(p(k), p(v), p(kt), p(vt), n, mask)
    torch.cuda.synchronize()
    ko = (kt if in_tmp else k).cpu().numpy().view(np.uint64)
    vo = (vt if in_tmp else v).cpu().numpy().view(np.uint32) if vals is not None else None
    return ko, vo


def _expect(keys, vals, mask):
    order = np.argsort(keys & np.uint64(mask), kind="stable")
    return keys[order], (vals[order] if vals is not None else None)


@pytest.mark.parametrize("n,mask,with_vals", [
    (1, 0xFF, True), (2, 0xFF, True), (4095, 0xFFFF, True), (4097, 0xFFFF, False),
    (100_003, (1 << 34) - 1, True), (1_000_000, 0xFFFF_0000_FFFF_0000, True),
    (3_000_017, (1 << 48) - 1, False), (20_000_000, (1 << 36) - 1, True),
])
def test_radix_sort_matches_stable_sort(ctx, n, mask, with_vals):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
    if n > 1000:
        keys[: n // 3] &= np.uint64(0xFFFF_FFFF_FFFF_00FF)  # a skewed digit: many equal keys in a run
    vals = np.arange(n, dtype=np.uint32)[::-1].copy() if with_vals else None
    ko, vo = _sort(ctx, keys, vals, mask)
    ek, ev = _expect(keys, vals, mask)
    assert np.array_equal(ko & np.uint64(mask), ek & np.uint64(mask))
    assert np.array_equal(ko, ek)
    if with_vals:
        assert np.array_equal(vo, ev)


def test_radix_sort_all_equal(ctx):
    n = 300_000
    keys = np.full(n, 0x1234, dtype=np.uint64)
    vals = np.arange(n, dtype=np.uint32)
    ko, vo = _sort(ctx, keys, vals, 0xFFFF)
    assert np.array_equal(vo, vals) and np.array_equal(ko, keys)
