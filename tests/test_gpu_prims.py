"""GPU: the device radix sort every pipeline sort runs on (reduce-then-scan passes), against numpy's
stable sort on the masked key bits; the exclusive scan behind every compaction and offset table."""
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


@pytest.mark.parametrize("elem", [4, 8])
@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 4095, 4096, 4097, 2048 * 3 + 1, 1 << 20, 300_007, 12_345_678])
@pytest.mark.parametrize("shift", [0, 1])
@pytest.mark.parametrize("inplace", [False, True])
def test_exclusive_scan(ctx, elem, n, shift, inplace):
    """Aligned buffers take the 16-byte-chunk reduce-then-scan (ragged tails element by element),
    misaligned ones (shift = one element) the narrow kernels; both against numpy, wrapping like the
    unsigned device arithmetic."""
    import torch
    if n > (1 << 20) and (shift or inplace):
        pytest.skip("large case: aligned out-of-place only")
    dt = np.uint32 if elem == 4 else np.uint64
    rng = np.random.default_rng(n + elem)
    hi = 1 << 20 if elem == 4 else 1 << 40
    a = rng.integers(0, hi, size=n, dtype=np.uint64).astype(dt)
    want = np.zeros(n, dtype=dt)
    if n:
        want[1:] = np.cumsum(a[:-1], dtype=dt)
    tdt = torch.int32 if elem == 4 else torch.int64
    dev = torch.device("cuda", 0)
    buf = torch.zeros(n + shift + 8, dtype=tdt, device=dev)
    buf[shift:shift + n] = torch.from_numpy(a.view(np.int32 if elem == 4 else np.int64)).to(dev)
    out = buf if inplace else torch.full((n + shift + 8,), -1, dtype=tdt, device=dev)
    base = buf.data_ptr() + shift * elem
    ctx.exclusive_scan_dev(base, out.data_ptr() + shift * elem, n, elem)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(dt)
    assert np.array_equal(got[shift:shift + n], want)
    if not inplace:  # nothing written outside [0, n)
        assert (got[shift + n:] == dt(-1 & (0xFFFFFFFF if elem == 4 else 0xFFFFFFFFFFFFFFFF))).all()
        if shift:
            assert got[0] == dt(0xFFFFFFFF if elem == 4 else 0xFFFFFFFFFFFFFFFF)
