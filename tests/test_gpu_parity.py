"""GPU parity: HIP path (through the C ABI) vs the CPU oracle on identical seeded inputs."""
import numpy as np
import pytest

import oracle
from openge_amd import lib as L

pytestmark = pytest.mark.gpu

CASES = [("mix", 3000, 7), ("c1", 50000, 1234), ("c2", 20000, 99)]


def _expected_flags(recs, offs, n, dup):
    f = np.array([int.from_bytes(recs[int(o) + 18:int(o) + 20].tobytes(), "little") for o in offs[:n]], dtype=np.uint16)
    return np.where(dup == 2, f, np.where(dup == 1, f | 0x400, f & np.uint16(0xFBFF))).astype(np.uint16)


@pytest.mark.parametrize("preset,npairs,seed", CASES)
def test_sort_perm_matches_oracle(ctx, preset, npairs, seed):
    p = L.synth_params(npairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * npairs
    perm = ctx.sort_coord(recs, offs, n, p.n_ref)
    assert np.array_equal(perm, oracle.sort_perm(recs, offs, n))


@pytest.mark.parametrize("preset,npairs,seed", CASES)
def test_markdup_matches_oracle(ctx, preset, npairs, seed):
    p = L.synth_params(npairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * npairs
    perm = oracle.sort_perm(recs, offs, n)
    # sorted input, as dedup sees it after mergesort
    from bamutil import rec_bytes, pack_records
    srecs, soffs = pack_records([rec_bytes(recs, offs[i]) for i in perm])
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    dup, nd = ctx.markdup(srecs, soffs, n, opts)
    odup, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond
    assert np.array_equal(dup, odup)
    # unsorted input too (dedup does not require sorted input)
    dup2, nd2 = ctx.markdup(recs, offs, n, opts)
    odup2, ond2 = oracle.markdup(recs, offs, n, hdr)
    assert nd2 == ond2 and np.array_equal(dup2, odup2)


def test_markdup_compat_nonverbose(ctx):
    p = L.synth_params(2000, preset="mix", seed=3)
    recs, offs, hdr = L.synth_host(p)
    n = 4000
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref, compat_nonverbose=True)
    dup, nd = ctx.markdup(recs, offs, n, opts)
    odup, ond = oracle.markdup(recs, offs, n, hdr, compat_nonverbose=True)
    assert nd == ond <= 1 and np.array_equal(dup, odup)


def test_synth_device_matches_host(ctx):
    torch = pytest.importorskip("torch")
    p = L.synth_params(5000, preset="c2", seed=5)
    recs, offs, _ = L.synth_host(p)
    n = 10000
    d_offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    ctx.synth_dev(p, d_offs.data_ptr(), None)
    ctx.sync()
    assert np.array_equal(d_offs.cpu().numpy().view(np.uint64), offs)
    d_recs = torch.zeros(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
    ctx.synth_dev(p, d_offs.data_ptr(), d_recs.data_ptr())
    ctx.sync()
    assert np.array_equal(d_recs.cpu().numpy()[: int(offs[-1])], recs[: int(offs[-1])])


@pytest.mark.parametrize("preset,npairs,seed", CASES)
def test_fused_sort_markdup(ctx, preset, npairs, seed):
    torch = pytest.importorskip("torch")
    from bamutil import rec_bytes, pack_records
    p = L.synth_params(npairs, preset=preset, seed=seed)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * npairs
    tot = int(offs[-1])
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(tot + 16, dtype=torch.uint8, device="cuda")
    d_out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                              d_out_off.data_ptr())
    ctx.sync()
    perm = d_perm.cpu().numpy().view(np.uint32)
    operm = oracle.sort_perm(recs, offs, n)
    assert np.array_equal(perm, operm)
    srecs, soffs = pack_records([rec_bytes(recs, offs[i]) for i in operm])
    odup, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond
    out = d_out.cpu().numpy()
    oo = d_out_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(oo, soffs)
    # expected bytes: sorted records, bin recomputed (generator bins are already exact), 0x400 applied
    exp = srecs.copy()
    fl = _expected_flags(srecs, soffs, n, odup)
    for k in range(n):
        o = int(soffs[k])
        exp[o + 18:o + 20] = np.frombuffer(int(fl[k]).to_bytes(2, "little"), dtype=np.uint8)
    assert np.array_equal(out[:tot], exp[:tot])


@pytest.mark.parametrize("bits", [1, 6, 12])
def test_markdup_forced_hash_collisions(ctx, bits):
    """Truncating the pair-key hash forces long hash runs and colliding 2-runs of non-mates:
    the exact key confirmation must keep the result identical to the oracle."""
    p = L.synth_params(1500, preset="mix", seed=11)
    recs, offs, hdr = L.synth_host(p)
    n = 3000
    perm = oracle.sort_perm(recs, offs, n)
    so = np.append(offs[:-1][perm], 0).astype(np.uint64)
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    opts.debug_hash_bits = bits
    dup, nd = ctx.markdup(recs, so, n, opts)
    odup, ond = oracle.markdup(recs, so, n, hdr)
    assert nd == ond and np.array_equal(dup, odup)


@pytest.mark.parametrize("bits", [1, 12])
def test_sort_markdup_forced_hash_collisions(ctx, bits):
    """The fused pipeline with truncated hashes: mate-join runs and the pair-chunk runs (grouped on
    hash bits, split into exact keys by k_pair_groups_h) hold many keys; FLAG bits must still equal
    the oracle's."""
    import torch
    p = L.synth_params(4000, preset="mix", seed=23)
    recs, offs, hdr = L.synth_host(p)
    n = 8000
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(recs.size, dtype=torch.uint8, device="cuda")
    d_oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    opts.debug_hash_bits = bits
    nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                              d_oo.data_ptr())
    ctx.sync()
    perm = d_perm.cpu().numpy().view(np.uint32)
    operm = oracle.sort_perm(recs, offs, n)
    assert np.array_equal(perm, operm)
    odup, ond = oracle.markdup(recs, offs[:-1][operm], n, hdr)
    assert nd == ond
    out, oo = d_out.cpu().numpy(), d_oo.cpu().numpy().view(np.uint64)
    for k in range(n):
        f = int.from_bytes(out[int(oo[k]) + 18:int(oo[k]) + 20].tobytes(), "little")
        if odup[k] != 2:
            assert bool(f & 0x400) == bool(odup[k]), k


@pytest.mark.parametrize("long_name", [False, True])
def test_long_tie_runs(ctx, long_name):
    """Equal-coordinate runs longer than 32 (k_tie_large_meta: LDS rows up to 2,048 members; the record-byte
    path past that, or when a member's name overflows the 32-byte slot): names sharing prefixes, exact
    name ties broken by flag and then by input index.  Sort-only and fused sort + dedup orders equal the
    oracle's, and so do the fused pipeline's FLAG bits."""
    import torch
    from bamutil import make_record, pack_records, rec_bytes
    rng = np.random.default_rng(11)
    recs = []
    for pos, cnt in [(100, 33), (200, 40), (300, 257), (400, 1000), (500, 2048), (600, 2049), (700, 3000)]:
        for j in range(cnt):
            nm = f"q{int(rng.integers(0, cnt // 3 + 1)):05d}" if j % 5 else f"q{int(rng.integers(0, 40))}"
            if long_name and pos == 400 and j == 7:
                nm = "L" * 40
            flag = int(rng.choice([0, 0x1 | 0x40 | 0x8, 0x1 | 0x80 | 0x8, 0x100]))
            recs.append(make_record(nm, flag, 0, pos, "20M", "A" * 20))
    for j in range(500):  # ragged background
        recs.append(make_record(f"b{j}", 0x10 if j & 1 else 0, 0, int(rng.integers(0, 1000)), "20M", "C" * 20))
    order = rng.permutation(len(recs))
    rr, oo = pack_records([recs[i] for i in order])
    n = len(recs)
    hdr = "@HD\tVN:1.0\tSO:unsorted\n@SQ\tSN:c0\tLN:10000\n"
    operm = oracle.sort_perm(rr, oo, n)
    assert np.array_equal(ctx.sort_coord(rr, oo, n, 1), operm)
    opts, keep = L.markdup_opts_from_header(hdr, 1)
    nd, fl, perm, _ = _fused_dup_flags(ctx, rr, oo, n, opts)
    assert np.array_equal(perm, operm)
    srecs, soffs = pack_records([rec_bytes(rr, oo[i]) for i in operm])
    odup, ond = oracle.markdup(srecs, soffs, n, hdr)
    assert nd == ond
    assert np.array_equal(fl, _expected_flags(srecs, soffs, n, odup))


def _fused_dup_flags(ctx, recs, offs, n, opts):
    import torch
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(recs.size + 16, dtype=torch.uint8, device="cuda")
    d_oo = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                              d_oo.data_ptr())
    ctx.sync()
    win = (ctx.timing("md_frag_win") >= 0, ctx.timing("md_pair_win") >= 0)
    out, oo = d_out.cpu().numpy(), d_oo.cpu().numpy().view(np.uint64)
    fl = np.array([int.from_bytes(out[int(oo[k]) + 18:int(oo[k]) + 20].tobytes(), "little") for k in range(n)])
    return nd, fl, d_perm.cpu().numpy().view(np.uint32), win


# (preset, pairs, seed, overrides, piles expected): the last case packs 40k pairs onto 3 kb of one
# contig (~27 reads per position), so the fragment windows overflow and those tiles' fragments go
# through the sort-based stage (k_win_collect)
WIN_CASES = [("c2", 30000, 5, {}, False), ("mix", 4000, 17, {}, False), ("c1", 20000, 8, {"clip_ppm": 300_000}, False),
             ("c1", 40000, 9, {"ref_len": [3000], "dup_ppm": 300_000}, True)]


@pytest.mark.parametrize("preset,npairs,seed,over,windowed", WIN_CASES)
def test_fused_windowed_groups_equal_sorted_groups(ctx, preset, npairs, seed, over, windowed):
    """The windowed fragment / pair group stages (k_frag_win, k_pair_win) against the sort-based
    ones (debug_sort_groups) and the oracle; dense piles overflow the windows and must fall back."""
    p = L.synth_params(npairs, preset=preset, seed=seed, **over)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * npairs
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    nd_w, fl_w, perm, win = _fused_dup_flags(ctx, recs, offs, n, opts)
    assert win == (True, True)
    assert (ctx.timing("md_frag_ovf") >= 0) == windowed
    opts.debug_sort_groups = 1
    nd_s, fl_s, perm_s, win_s = _fused_dup_flags(ctx, recs, offs, n, opts)
    assert win_s == (False, False)
    assert np.array_equal(perm, perm_s) and nd_w == nd_s and np.array_equal(fl_w, fl_s)
    operm = oracle.sort_perm(recs, offs, n)
    odup, ond = oracle.markdup(recs, offs[:-1][operm], n, hdr)
    assert nd_w == ond
    prim = odup != 2
    assert np.array_equal((fl_w[prim] & 0x400) != 0, odup[prim] == 1)


@pytest.mark.parametrize("cap", ["1", "300"])
def test_fused_windowed_groups_overflow_path(ctx, monkeypatch, cap):
    """OGE_MD_WINCAP shrinks the window caps: (nearly) every tile overflows, so the fragment and pair
    groups go through k_win_collect + the sort-based kernels; the result must not change."""
    p = L.synth_params(6000, preset="mix", seed=31)
    recs, offs, hdr = L.synth_host(p)
    n = 12000
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    monkeypatch.setenv("OGE_MD_WINCAP", cap)
    nd_w, fl_w, perm, win = _fused_dup_flags(ctx, recs, offs, n, opts)
    assert win == (True, True)
    assert ctx.timing("md_frag_ovf") >= 0 and ctx.timing("md_pair_ovf") >= 0
    monkeypatch.delenv("OGE_MD_WINCAP")
    operm = oracle.sort_perm(recs, offs, n)
    odup, ond = oracle.markdup(recs, offs[:-1][operm], n, hdr)
    assert nd_w == ond
    prim = odup != 2
    assert np.array_equal((fl_w[prim] & 0x400) != 0, odup[prim] == 1)


@pytest.mark.parametrize("width", [1, 4, 15, 16, 23])
def test_markdup_read_group_widths(ctx, width):
    """Read-group ids of every width around the input pass's word compare (<= 15 bytes: the padded
    16-byte table; longer: byte by byte), two of them sharing a prefix, plus an id missing from the header:
    libraries (RG -> LB) and pair keys (RG + name) must give the oracle's dup flags."""
    from bamutil import rec_bytes, pack_records
    p = L.synth_params(3000, preset="mix", seed=41)
    recs, offs, hdr = L.synth_host(p)
    n = 2 * 3000
    ids = {k: (f"g{k}" + "x" * width)[:width] if width > 1 else chr(ord("a") + k) for k in range(1, p.n_rg + 1)}
    if width > 2:
        ids[2] = ids[1][:-1] + "Y"  # same length, same prefix as group 1
    lines = []
    for line in hdr.splitlines():
        if line.startswith("@RG"):
            f = line.split("\t")
            k = int(f[1][len("ID:rg"):])
            f[1] = "ID:" + ids[k]
            line = "\t".join(f)
        lines.append(line)
    hdr2 = "\n".join(lines) + "\n"
    out = []
    for i in range(n):
        b = bytearray(rec_bytes(recs, offs[i]))
        assert bytes(b[-7:-4]) == b"RGZ"
        k = b[-2] - ord("0")
        v = ids[k] if i % 97 else "unlisted" + "z" * (width % 5)
        b = b[:-4] + v.encode() + b"\0"
        b[0:4] = (len(b) - 4).to_bytes(4, "little")
        out.append(bytes(b))
    r2, o2 = pack_records(out)
    perm = oracle.sort_perm(r2, o2, n)
    srecs, soffs = pack_records([rec_bytes(r2, o2[i]) for i in perm])
    opts, keep = L.markdup_opts_from_header(hdr2, p.n_ref)
    dup, nd = ctx.markdup(srecs, soffs, n, opts)
    odup, ond = oracle.markdup(srecs, soffs, n, hdr2)
    assert nd == ond and np.array_equal(dup, odup)


def test_sort_markdup_output_offsets_alignment(ctx):
    """The output offsets come from one fused scan over the sorted keys when d_out_off is 16-byte aligned and
    from the sizes kernel + scan otherwise: the same offsets and records either way."""
    import torch
    p = L.synth_params(3000, preset="mix", seed=29)
    recs, offs, hdr = L.synth_host(p)
    n = 6000
    opts, keep = L.markdup_opts_from_header(hdr, p.n_ref)
    d_recs = torch.from_numpy(recs).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    outs = []
    for shift in (0, 1):
        d_perm = torch.empty(n, dtype=torch.int32, device="cuda")
        d_out = torch.zeros(recs.size, dtype=torch.uint8, device="cuda")
        buf = torch.full((n + 2 + shift,), -1, dtype=torch.int64, device="cuda")
        d_oo = buf[shift:shift + n + 1]
        assert (d_oo.data_ptr() % 16 == 0) == (shift == 0)
        nd = ctx.sort_markdup_dev(d_recs.data_ptr(), d_offs.data_ptr(), n, opts, d_perm.data_ptr(), d_out.data_ptr(),
                                  d_oo.data_ptr())
        ctx.sync()
        outs.append((nd, d_oo.cpu().numpy().copy(), d_out.cpu().numpy()))
    assert outs[0][0] == outs[1][0]
    assert np.array_equal(outs[0][1], outs[1][1]) and outs[0][1][0] == 0 and outs[0][1][-1] == int(offs[-1])
    assert np.array_equal(outs[0][2], outs[1][2])
