// shard.hip -- ONE BGZF BAM file decoded by G ranks, each from its own byte range (config 4: the
// 8-GPU node reading one input file).  The reference reads the file on one thread, block after block
// (util/bgzf_input_stream.cpp:65-142,180-206 reader thread; util/bam_deserializer.h:143-193 record walk),
// and SplitByChromosome routes the decoded records to its chains afterwards
// (alg/split_by_chromosome.cpp:30-58, cmd/command_mergesort.cpp:118-179).  Here every rank inflates
// only the BGZF blocks that start in its byte range, so the codec scales with G:
//
//   framing   rank g scans its range [a_g, a_g + own_g) for block headers (inflate.hip's range index)
//             and walks the exact block chain from its first candidate; the chain of rank g - 1 ends at
//             the first block start at or past a_g, so a rank's guess is confirmed (or corrected) by
//             its predecessor's exit -- one allgather per round, one round unless a guess was wrong
//   inflate   the rank's blocks -> U_g, its part of the decompressed stream (bytes [B_g, B_g + T_g))
//   edges     every rank fetches the first 16 KiB after its part from the next ranks (the record that
//             starts in U_g and ends in U_{g+1}: at most 4 + 10000 bytes, bam_deserializer.h:160-163) --
//             an all-to-all of neighbour-sized messages; rank 0 parses the BAM header and shares it
//   records   rank g owns the records that START in U_g: rank 0 from the header's end, rank g > 0 from a
//             plausibility guess confirmed by rank g - 1's walk exit (the same join as the framing)
//
// The result on rank g: the records of its part in file order, complete in its own HBM (the last one
// may end in the fetched tail) -- contiguous input ranges in rank order, which is what the range-split
// sort + dedup (dist.hip) takes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "bamio.h"
#include "bgzf_dev.h"
#include "oge_ctx.h"

using namespace oge;

namespace {

constexpr uint64_t kNoPos = ~0ull;
constexpr uint64_t kLook = 16384;  // >= the largest record the walk accepts (4 + 10000 bytes)

struct Shard {
    oge_comm *comm;
    oge_ctx *ctx;
    int G, r;

    template <class T>
    int gather(const char *tag, const T &mine, std::vector<T> &all) {
        all.assign(G, T());
        return oge_comm_allgather(comm, tag, &mine, all.data(), sizeof(T));
    }
    // every rank learns whether any rank failed (keeps the collectives in step)
    int agree(int rc) {
        std::vector<int> all;
        if (const int r2 = gather("status", rc, all)) return r2;
        for (int g = 0; g < G; ++g)
            if (all[g]) return rc ? rc : oge_fail(ctx, OGE_ERR_HIP, ("sharded decode: rank " + std::to_string(g) + " failed").c_str());
        return OGE_OK;
    }
};

// Positions joined across ranks.  Rank g computes, from its start s_g (global), its exit x_g = the first
// position at or past its range's end; the chain is exact when s_0 = start0, s_g = x_{g-1} for every
// g > 0 and x_{G-1} = stream_end.  compute(s, slow, &x) returns 0 (x valid), 1 (s is not a start / the
// fast check could not confirm it) or < 0 (a device error).  A rank whose start is already the confirmed
// expectation but whose fast check failed gets one slow try (the host walk); after that a failure is
// a corrupt stream.  Every round extends the confirmed prefix by at least one rank.
template <class F>
int join_ranks(Shard &S, const char *tag, const char *what, uint64_t start0, uint64_t s, uint64_t x, int st, uint64_t stream_end,
               F &&compute, uint64_t *s_out, uint64_t *x_out) {
    int hard = st < 0 ? st : 0;
    uint64_t ok = st == 0 ? 1 : 0, slow_done = 0;
    auto run = [&](bool slow) {
        uint64_t xx = kNoPos;
        const int rc = s == kNoPos ? 1 : compute(s, slow, &xx);
        if (rc < 0 && !hard) hard = rc;
        ok = rc == 0 ? 1 : 0;
        x = rc == 0 ? xx : kNoPos;
    };
    for (int round = 0; round <= 2 * S.G + 2; ++round) {
        struct P {
            uint64_t s, x, ok, slow, hard;
        } mine{s, x, ok, slow_done, (uint64_t)(hard != 0)}, *all;
        std::vector<P> v;
        if (const int rc = S.gather(tag, mine, v)) return rc;
        all = v.data();
        for (int g = 0; g < S.G; ++g)
            if (all[g].hard) return hard ? hard : oge_fail(S.ctx, OGE_ERR_HIP, ("sharded decode: rank " + std::to_string(g) + " failed").c_str());
        int c = 0;  // confirmed prefix
        uint64_t expect = start0;
        for (; c < S.G; ++c) {
            if (all[c].s != expect || !all[c].ok) break;
            expect = all[c].x;
        }
        if (c == S.G) {
            if (expect != stream_end)
                return oge_fail(S.ctx, OGE_ERR_IO, (std::string(what) + ": the last rank's walk does not end at the end of the stream").c_str());
            *s_out = s;
            *x_out = x;
            return OGE_OK;
        }
        if (all[c].s == expect && !all[c].ok && all[c].slow)
            return oge_fail(S.ctx, OGE_ERR_IO, (std::string(what) + ": invalid data in rank " + std::to_string(c) + "'s range").c_str());
        if (S.r == c && s == expect && !ok) {
            run(true);
            slow_done = 1;
        } else if (S.r >= c) {
            const uint64_t want = S.r == 0 ? start0 : all[S.r - 1].x;
            if (want != kNoPos && want != s) {
                s = want;
                slow_done = 0;
                run(false);
            }
        }
    }
    return oge_fail(S.ctx, OGE_ERR_IO, (std::string(what) + ": the ranks' walks did not join").c_str());
}

// The host walk of the blocks that start in [0, lim) of h (the framing fallback; the same acceptance
// as oge_bgzf_index), positions offset by `at`.
int host_walk_range(oge_ctx *ctx, const uint8_t *h, uint64_t hb, uint64_t lim, uint64_t at, std::vector<uint64_t> &d0,
                    std::vector<uint64_t> &d1, std::vector<uint64_t> &uo, std::vector<uint32_t> &crc, uint64_t *xend) {
    auto rd16 = [](const uint8_t *p) { return (uint32_t)(p[0] | (p[1] << 8)); };
    auto rd32 = [](const uint8_t *p) { return (uint32_t)p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); };
    uint64_t p = 0, total = 0;
    d0.clear(), d1.clear(), uo.clear(), crc.clear();
    while (p < lim) {
        if (hb - p < 18 || h[p] != 31 || h[p + 1] != 139 || h[p + 2] != 8 || h[p + 3] != 4)
            return oge_fail(ctx, OGE_ERR_IO, "not a BGZF stream or truncated block header");
        const uint64_t xend_f = p + 12 + rd16(h + p + 10);
        if (xend_f > hb) return oge_fail(ctx, OGE_ERR_IO, "truncated BGZF extra field");
        uint64_t bsize = 0;
        for (uint64_t x = p + 12; x + 4 <= xend_f;) {
            const uint32_t sl = rd16(h + x + 2);
            if (h[x] == 'B' && h[x + 1] == 'C' && sl == 2) bsize = (uint64_t)rd16(h + x + 4) + 1;
            x += 4 + sl;
        }
        if (!bsize) return oge_fail(ctx, OGE_ERR_IO, "BGZF block without BC field");
        if (p + bsize > hb || bsize < xend_f - p + 8) return oge_fail(ctx, OGE_ERR_IO, "truncated BGZF block");
        const uint32_t isize = rd32(h + p + bsize - 4);
        if (isize > oge_bgzf::kSlot) return oge_fail(ctx, OGE_ERR_IO, "BGZF block payload larger than 64 KiB");
        if (isize) {
            d0.push_back(at + xend_f);
            d1.push_back(at + p + bsize - 8);
            uo.push_back(total);
            crc.push_back(rd32(h + p + bsize - 8));
            total += isize;
        }
        p += bsize;
    }
    uo.push_back(total);
    *xend = at + p;
    return OGE_OK;
}

}  // namespace

int oge_decode_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own, uint8_t **Xo, uint64_t **xoff_o, uint64_t *n_o,
                     std::vector<uint8_t> *header) {
    oge_ctx *ctx = oge_comm_ctx(comm);
    Shard S{comm, ctx, oge_comm_size(comm), oge_comm_rank(comm)};
    int rc = OGE_OK;
    if (own > zbytes || (zbytes && !d_z)) rc = oge_fail(ctx, OGE_ERR_ARG, "sharded decode: own_bytes > zbytes or null buffer");
    if ((rc = S.agree(rc))) return rc;

    // ---- ranges: rank g owns block starts in [a_g, a_g + own_g) of the file
    std::vector<uint64_t> owns;
    if ((rc = S.gather("shard_plan", own, owns))) return rc;
    uint64_t a = 0, zf = 0;
    for (int g = 0; g < S.G; ++g) {
        if (g < S.r) a += owns[g];
        zf += owns[g];
    }
    if (S.r == S.G - 1 && zbytes != own) rc = oge_fail(ctx, OGE_ERR_ARG, "sharded decode: the last rank's buffer must end at the end of the file");
    if ((rc = S.agree(rc))) return rc;

    // ---- framing: the exact block chain of every range, joined across ranks
    OgeStageTimer *tm = ctx->begin_stage("bgzf_index");
    OgeBgzfIndex ix;
    std::vector<uint64_t> h0, h1, hu;
    std::vector<uint32_t> hc;
    auto frame = [&](uint64_t sg, bool slow, uint64_t *xg) -> int {
        if (sg < a) return 1;
        const uint64_t ls = sg - a;
        if (ls >= own) {  // no block starts in this range
            ix = OgeBgzfIndex();
            *xg = sg;
            return 0;
        }
        if (!slow) {
            uint64_t xe = 0;
            const int r2 = oge_bgzf_index_range_ws(ctx, d_z, zbytes, ls, own, &ix, nullptr, &xe);
            if (r2 < 0) return r2;
            if (r2) return 1;
            *xg = a + xe;
            return 0;
        }
        std::vector<uint8_t> h(zbytes - ls);  // the host walk from a confirmed start (false candidates inside the range)
        OGE_HIP_TRY(ctx, hipMemcpyAsync(h.data(), d_z + ls, h.size(), hipMemcpyDeviceToHost, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        uint64_t xe = 0;
        if (host_walk_range(ctx, h.data(), h.size(), own - ls, ls, h0, h1, hu, hc, &xe)) return 1;
        const uint64_t nb = h0.size();
        uint64_t *dd = (uint64_t *)ctx->ws("shard_ix", (3 * nb + 2) * 8);
        uint32_t *dc = (uint32_t *)ctx->ws("shard_ixc", (nb + 1) * 4);
        if (!dd || !dc) return OGE_ERR_HIP;
        if (nb) {
            OGE_HIP_TRY(ctx, hipMemcpyAsync(dd, h0.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
            OGE_HIP_TRY(ctx, hipMemcpyAsync(dd + nb, h1.data(), nb * 8, hipMemcpyHostToDevice, ctx->stream));
            OGE_HIP_TRY(ctx, hipMemcpyAsync(dc, hc.data(), nb * 4, hipMemcpyHostToDevice, ctx->stream));
        }
        OGE_HIP_TRY(ctx, hipMemcpyAsync(dd + 2 * nb, hu.data(), (nb + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        OGE_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        ix.d0 = dd, ix.d1 = dd + nb, ix.uoff = dd + 2 * nb, ix.crc = dc, ix.nblk = nb, ix.total = hu[nb];
        *xg = a + xe;
        return 0;
    };
    uint64_t s0 = kNoPos, x0 = kNoPos;
    int st = 1;
    if (S.r == 0) {
        st = frame(0, false, &x0);
        s0 = 0;
    } else if (own) {  // the first candidate of the range as the guess
        uint64_t su = kNoPos, xe = 0;
        st = oge_bgzf_index_range_ws(ctx, d_z, zbytes, kIndexFirst, own, &ix, &su, &xe);
        if (st == 2) {
            st = 1;
        } else {
            s0 = su == kNoPos ? kNoPos : a + su;
            if (st == 0) x0 = a + xe;
        }
        if (st > 0) st = 1;
    }
    uint64_t s_blk = 0;
    uint64_t x_blk = 0;
    rc = join_ranks(S, "shard_framing", "BGZF framing", 0, s0, x0, st, zf, frame, &s_blk, &x_blk);
    ctx->end_stage(tm);
    if (rc) return rc;
    ctx->counters["shard_blocks"] = ix.nblk;
    ctx->counters["shard_zbytes"] = x_blk - s_blk;

    // ---- inflate this range's blocks: U_g, then room for the fetched tail
    const uint64_t T = ix.total;
    uint8_t *X = (uint8_t *)ctx->ws("pipe_x", T + kLook + 64);
    if (!X) rc = OGE_ERR_HIP;
    if (!rc && ix.nblk) rc = oge_bgzf_inflate_dev(ctx, d_z, zbytes, ix.d0, ix.d1, ix.uoff, ix.crc, ix.nblk, X);
    if ((rc = S.agree(rc))) return rc;

    // ---- edges: bases of the parts, the tails that straddle them, the header
    tm = ctx->begin_stage("shard_edges");
    std::vector<uint64_t> Ts;
    if ((rc = S.gather("shard_plan", T, Ts))) return rc;
    std::vector<uint64_t> Bs(S.G + 1, 0);
    for (int g = 0; g < S.G; ++g) Bs[g + 1] = Bs[g] + Ts[g];
    const uint64_t B = Bs[S.r], Ut = Bs[S.G];
    // fetch global bytes [lo, hi) of the decompressed stream into dst (every rank takes part)
    auto fetch = [&](const char *tag, uint64_t lo, uint64_t hi, uint8_t *dst) -> int {
        struct Rq {
            uint64_t lo, hi;
        };
        std::vector<Rq> rq;
        int r2 = S.gather("shard_plan", Rq{lo, hi}, rq);
        if (r2) return r2;
        std::vector<uint64_t> sb(S.G, 0), so(S.G, 0), rb(S.G, 0), ro(S.G, 0);
        for (int p = 0; p < S.G; ++p) {
            const uint64_t l1 = std::max(rq[p].lo, B), h1_ = std::min(rq[p].hi, B + T);  // p's request in my part
            if (p != S.r && h1_ > l1) sb[p] = h1_ - l1, so[p] = l1 - B;
            const uint64_t l2 = std::max(lo, Bs[p]), h2 = std::min(hi, Bs[p + 1]);  // my request in p's part
            if (p != S.r && h2 > l2) rb[p] = h2 - l2, ro[p] = l2 - lo;
        }
        return oge_comm_alltoallv_dev(comm, tag, X, sb.data(), so.data(), dst, rb.data(), ro.data());
    };
    const uint64_t look_hi = std::min(Ut, B + T + kLook), L = look_hi - (B + T);
    rc = fetch("shard_edges", B + T, look_hi, X + T);
    if ((rc = S.agree(rc))) return rc;
    // rank 0: the header from the stream's first bytes (its own part, the fetched tail, and more when a
    // header is larger than both); shared with every rank
    BamFile f;
    size_t rec_base = 0;
    std::vector<uint8_t> hdr;
    {
        uint64_t have = T + L, need = std::min<uint64_t>(have, 1 << 20);
        int parsed = 0;
        for (int it = 0; it < 64; ++it) {
            if (S.r == 0 && !parsed && !rc) {
                std::vector<uint8_t> h(need);
                const uint64_t own_part = std::min(need, T + L);
                if (own_part && hipMemcpyAsync(h.data(), X, own_part, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = OGE_ERR_HIP;
                if (!rc && need > own_part) {
                    const uint8_t *tail = (const uint8_t *)ctx->ws("shard_hdr_tail", 1);
                    if (hipMemcpyAsync(h.data() + own_part, tail, need - own_part, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
                        rc = OGE_ERR_HIP;
                }
                if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = OGE_ERR_HIP;
                if (rc) rc = oge_fail(ctx, OGE_ERR_HIP, "sharded decode: header copy");
                std::string err;
                if (!rc && bam_parse_header(h.data(), h.size(), f, err, &rec_base)) {
                    parsed = 1;
                    hdr.assign(h.begin(), h.begin() + rec_base);
                } else if (!rc && need >= Ut) {
                    rc = oge_fail(ctx, OGE_ERR_IO, ("BAM header: " + err).c_str());
                }
            }
            struct Hs {
                uint64_t parsed, need, rc;
            };
            std::vector<Hs> hs;
            if (const int r2 = S.gather("shard_header", Hs{(uint64_t)parsed, need, (uint64_t)(rc != 0)}, hs)) return r2;
            for (int g = 0; g < S.G; ++g)
                if (hs[g].rc) return rc ? rc : oge_fail(ctx, OGE_ERR_IO, "sharded decode: rank 0 could not read the BAM header");
            if (hs[0].parsed) break;
            // the header runs past rank 0's part and tail: rank 0 fetches more of the stream
            const uint64_t want = std::min<uint64_t>(Ut, std::max<uint64_t>(hs[0].need * 8, 1 << 20));
            if (S.r == 0) {
                if (want > have) {
                    uint8_t *tail = (uint8_t *)ctx->ws("shard_hdr_tail", want - have + 64);
                    rc = tail ? fetch("shard_header", have, want, tail) : OGE_ERR_HIP;
                } else {
                    rc = fetch("shard_header", 0, 0, X);
                }
                need = want;
            } else {
                rc = fetch("shard_header", 0, 0, X);
            }
            if ((rc = S.agree(rc))) return rc;
        }
        uint64_t hl = hdr.size();
        std::vector<uint64_t> hls;
        if ((rc = S.gather("shard_header", hl, hls))) return rc;
        hl = hls[0];
        if (!hl) return oge_fail(ctx, OGE_ERR_IO, "BAM header: not found");
        std::vector<uint8_t> hall((size_t)S.G * hl, 0), mine(hl, 0);
        if (S.r == 0) mine = hdr;
        if ((rc = oge_comm_allgather(comm, "shard_header", mine.data(), hall.data(), hl))) return rc;
        hdr.assign(hall.begin(), hall.begin() + hl);
        std::string err;
        f = BamFile();
        if (!bam_parse_header(hdr.data(), hdr.size(), f, err, &rec_base)) return oge_fail(ctx, OGE_ERR_IO, ("BAM header: " + err).c_str());
    }
    ctx->end_stage(tm);
    const int32_t n_ref = (int32_t)f.ref_names.size();

    // ---- records that start in this part, joined across ranks
    tm = ctx->begin_stage("rec_walk");
    const bool at_end = look_hi == Ut;
    auto walk = [&](uint64_t sg, bool, uint64_t *xg) -> int {
        if (sg < B) return 1;
        const uint64_t ls = sg - B;
        if (ls >= T) {
            *xg = sg;
            return 0;
        }
        uint64_t n = 0, xe = 0;
        const int r2 = oge_record_walk(ctx, X, ls, T, T + L, at_end, n_ref, nullptr, 0, &n, &xe);
        if (r2 == OGE_ERR_IO) return 1;
        if (r2) return r2;
        *xg = B + xe;
        return 0;
    };
    uint64_t rs = kNoPos, rx = kNoPos;
    st = 1;
    if (S.r == 0) {
        rs = rec_base;
        st = walk(rs, false, &rx);
    } else if (T) {
        uint64_t gl = kNoPos;
        st = oge_record_guess(ctx, X, T, T + L, at_end, n_ref, &gl);
        if (st == 0) {
            if (gl == kNoPos) {
                st = 1;
            } else {
                rs = B + gl;
                st = walk(rs, false, &rx);
            }
        }
    }
    uint64_t s_rec = 0, x_rec = 0;
    rc = join_ranks(S, "shard_records", "BAM records", rec_base, rs, rx, st, Ut, walk, &s_rec, &x_rec);
    if (rc) return rc;
    uint64_t n = 0, xe = 0;
    uint64_t *xoff = nullptr;
    if (s_rec - B >= T || s_rec < B) {  // no record starts in this part
        xoff = (uint64_t *)ctx->ws("pipe_xoff", 8);
        if (!xoff) rc = OGE_ERR_HIP;
        const uint64_t z = 0;
        if (!rc && hipMemcpyAsync(xoff, &z, 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) rc = OGE_ERR_HIP;
        if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = OGE_ERR_HIP;
    } else {
        rc = oge_record_walk(ctx, X, s_rec - B, T, T + L, at_end, n_ref, nullptr, 0, &n, &xe, true);
        if (!rc) {
            xoff = (uint64_t *)ctx->ws("pipe_xoff", (n + 1) * 8);
            rc = xoff ? oge_record_walk(ctx, X, s_rec - B, T, T + L, at_end, n_ref, xoff, n + 1, &n, &xe, true) : OGE_ERR_HIP;
        }
    }
    ctx->end_stage(tm);
    if ((rc = S.agree(rc))) return rc;
    ctx->counters["shard_bytes"] = T;
    ctx->counters["shard_records"] = n;
    *Xo = X;
    *xoff_o = xoff;
    *n_o = n;
    if (header) *header = hdr;
    return OGE_OK;
}

extern "C" int oge_bgzf_decode_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own_bytes, const uint8_t **d_recs,
                                     const uint64_t **d_off, uint64_t *n, uint8_t *hdr_out, uint64_t hdr_cap, uint64_t *hdr_len) {
    if (!comm) return oge_fail(nullptr, OGE_ERR_ARG, "null communicator");
    oge_ctx *ctx = oge_comm_ctx(comm);
    if (!d_recs || !d_off || !n) return oge_fail(ctx, OGE_ERR_ARG, "null argument");
    (void)hipSetDevice(ctx->device);
    ctx->reset_timing();
    ctx->timing_hold++;
    oge_comm_reset_stats(comm);
    uint8_t *X = nullptr;
    uint64_t *xoff = nullptr, m = 0;
    std::vector<uint8_t> h;
    const int rc = oge_decode_shard(comm, d_z, zbytes, own_bytes, &X, &xoff, &m, &h);
    ctx->timing_hold--;
    if (rc) return rc;
    if (hdr_len) *hdr_len = h.size();
    if (hdr_out && hdr_cap < h.size()) return oge_fail(ctx, OGE_ERR_LIMIT, "hdr_cap is smaller than the BAM header");
    if (hdr_out && !h.empty()) memcpy(hdr_out, h.data(), h.size());
    *d_recs = X;
    *d_off = xoff;
    *n = m;
    return OGE_OK;
}
