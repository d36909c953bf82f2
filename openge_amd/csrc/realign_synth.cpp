// realign_synth.cpp -- deterministic synthetic local-realignment data set (SURVEY.md §8d C5 shape):
// a random reference FASTA (+ .fai), a target-interval list and a coordinate-sorted BAM of read
// pairs around one true indel per interval.
//
// Per interval (contig c, site p): a 1-10 bp insertion or deletion at p (a fraction of intervals
// has none).  Fragments are placed so one read of the pair overlaps the site; the mate lies
// `insert` bp away, outside the interval.  Reads are cut from the sample haplotype (reference with
// the indel applied); a read spanning the indel is aligned gapped (aM LI/LD bM) with probability
// gapped_ppm, else ungapped (it then mismatches the reference past p).  alt_indel_ppm of the gapped
// reads carry the indel 3 bp to the right (a misaligned second consensus).  Sequencing errors,
// soft clips, MAPQ 0, duplicate flags, lower-case / N reference bases and NM/MD/UQ tags exercise the
// realigner's side paths.  Uniform draws use explicit modulo arithmetic on std::mt19937_64 (fully
// specified), so output is identical on every platform.
#include "../../include/openge_hip.h"
#include "bamio.h"
#include "capi_common.h"
#include "synth.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace {

struct Rec {
    uint64_t key;  // ref << 33 | pos << 1 | rev  (ByPosition up to the name)
    std::string name;
    uint16_t flag;
    std::vector<uint8_t> bytes;
};

const char kBases[] = "ACGT";

template <class F>
void par_for(size_t n, int threads, F f) {
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    std::atomic<size_t> next(0);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&]() {
            for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
        });
    for (auto &t : ts) t.join();
}

uint8_t code4(char b) {
    switch (b) {
        case 'A': return 1; case 'C': return 2; case 'G': return 4; case 'T': return 8;
        default: return 15;
    }
}

std::vector<uint8_t> encode(const std::string &name, uint16_t flag, int32_t ref, int32_t pos, uint8_t mapq,
                            const std::vector<uint32_t> &cig, const std::string &seq, const std::string &qual,
                            int32_t mref, int32_t mpos, int32_t tlen, const std::string &tags) {
    std::vector<uint8_t> b;
    const uint32_t lname = (uint32_t)name.size() + 1, l = (uint32_t)seq.size();
    const uint32_t bs = 32 + lname + 4 * (uint32_t)cig.size() + (l + 1) / 2 + l + (uint32_t)tags.size();
    b.resize(4 + bs);
    uint8_t *p = b.data();
    int32_t end = pos;
    for (uint32_t op : cig) {
        uint32_t t = op & 0xF;
        if (t == 0 || t == 2 || t == 3 || t == 7 || t == 8) end += (int32_t)(op >> 4);
    }
    uint32_t bin = oge_reg2bin(pos, end);
    uint32_t core[9] = {bs, (uint32_t)ref, (uint32_t)pos, (bin << 16) | ((uint32_t)mapq << 8) | lname,
                        ((uint32_t)flag << 16) | (uint32_t)cig.size(), l, (uint32_t)mref, (uint32_t)mpos, (uint32_t)tlen};
    memcpy(p, core, 36);
    p += 36;
    memcpy(p, name.c_str(), lname);
    p += lname;
    memcpy(p, cig.data(), 4 * cig.size());
    p += 4 * cig.size();
    for (uint32_t i = 0; i < l; i += 2) {
        uint8_t hi = code4(seq[i]), lo = i + 1 < l ? code4(seq[i + 1]) : 0;
        *p++ = (uint8_t)(hi << 4 | lo);
    }
    for (uint32_t i = 0; i < l; ++i) *p++ = (uint8_t)qual[i];
    memcpy(p, tags.data(), tags.size());
    return b;
}

void tag_i(std::string &t, const char *k, int32_t v) {
    t += k;
    t += 'i';
    t.append((const char *)&v, 4);
}
void tag_z(std::string &t, const char *k, const std::string &v) {
    t += k;
    t += 'Z';
    t += v;
    t += '\0';
}

struct Gen {
    const oge_realign_synth_params &P;
    std::mt19937_64 g;
    explicit Gen(const oge_realign_synth_params &p, uint64_t a, uint64_t b) : P(p), g(oge_rng(p.seed, a, b)) {}
    uint64_t u(uint64_t n) { return n ? g() % n : 0; }
    bool ppm(uint32_t x) { return (uint32_t)(g() % 1000000ull) < x; }
};

}  // namespace

extern "C" {

void oge_realign_synth_defaults(oge_realign_synth_params *p) {
    memset(p, 0, sizeof(*p));
    p->seed = 1234;
    p->n_ref = 24;
    p->n_intervals = 50000;
    p->spacing = 2000;
    p->read_len = 150;
    p->frags_per_interval = 40;
    p->qual_min = 10;
    p->qual_max = 40;
    p->ins_min = 250;
    p->ins_max = 450;
    p->err_ppm = 2000;
    p->noindel_ppm = 100000;
    p->gapped_ppm = 600000;
    p->alt_indel_ppm = 100000;
    p->dup_ppm = 30000;
    p->mapq0_ppm = 20000;
    p->clip_ppm = 50000;
    p->lower_ppm = 20000;
    p->n_ppm = 500;
    p->md_ppm = 500000;
    p->uq_ppm = 250000;
}

int oge_synth_realign(const oge_realign_synth_params *pp, const char *fasta_path, const char *intervals_path,
                      const char *bam_path, int level, int threads) {
    if (!pp || !fasta_path || !intervals_path || !bam_path) return oge_fail(nullptr, OGE_ERR_ARG, "oge_synth_realign: null argument");
    const oge_realign_synth_params &P = *pp;
    const uint32_t rl = P.read_len;
    if (P.n_ref == 0 || P.n_intervals == 0 || rl < 40 || rl > 250 || P.spacing < 2 * (P.ins_max + rl) ||
        P.ins_min < rl || P.ins_max < P.ins_min || P.qual_max < P.qual_min || P.qual_max > 93)
        return oge_fail(nullptr, OGE_ERR_ARG, "oge_synth_realign: parameters out of range");
    const uint32_t per = (P.n_intervals + P.n_ref - 1) / P.n_ref;
    const uint32_t margin = 1000;
    const int32_t clen = (int32_t)(2 * margin + per * P.spacing);

    // ---- reference
    std::vector<std::string> ref(P.n_ref);
    par_for(P.n_ref, threads, [&](size_t c) {
        Gen G(P, 1000003ull + c, 1);
        std::string &s = ref[c];
        s.resize((size_t)clen);
        for (int32_t i = 0; i < clen; ++i) {
            char b = kBases[G.u(4)];
            if (G.ppm(P.n_ppm)) b = 'N';
            else if (G.ppm(P.lower_ppm)) b = (char)(b + 32);
            s[(size_t)i] = b;
        }
    });
    {
        FILE *f = fopen(fasta_path, "wb");
        if (!f) return oge_fail(nullptr, OGE_ERR_IO, "oge_synth_realign: cannot write FASTA");
        std::string fai;
        long off = 0;
        for (uint32_t c = 0; c < P.n_ref; ++c) {
            std::string hdr = ">chr" + std::to_string(c + 1) + "\n";
            fputs(hdr.c_str(), f);
            off += (long)hdr.size();
            fai += "chr" + std::to_string(c + 1) + "\t" + std::to_string(clen) + "\t" + std::to_string(off) + "\t60\t61\n";
            for (int32_t i = 0; i < clen; i += 60) {
                int32_t k = std::min(60, clen - i);
                fwrite(ref[c].data() + i, 1, (size_t)k, f);
                fputc('\n', f);
                off += k + 1;
            }
        }
        fclose(f);
        FILE *fi = fopen((std::string(fasta_path) + ".fai").c_str(), "wb");
        if (!fi) return oge_fail(nullptr, OGE_ERR_IO, "oge_synth_realign: cannot write .fai");
        fputs(fai.c_str(), fi);
        fclose(fi);
    }

    // ---- intervals + reads
    // Reads of interval gi lie within +-(ins_max + read_len) of its site and sites are `spacing`
    // apart (>= 2 (ins_max + read_len)), so sorting each interval's records and concatenating the
    // intervals in order gives the coordinate sort.
    std::vector<std::vector<Rec>> per_iv(P.n_intervals);
    std::vector<std::string> ivline(P.n_intervals);
    auto upper = [](char b) { return (b >= 'a' && b <= 'z') ? (char)(b - 32) : b; };
    par_for(P.n_intervals, threads, [&](size_t gi_) {
        const uint32_t gi = (uint32_t)gi_;
        std::vector<Rec> &recs = per_iv[gi];
        const uint32_t c = gi / per, j = gi % per;
        const std::string &R = ref[c];
        Gen G(P, gi, 2);
        const int32_t p = (int32_t)(margin + j * P.spacing + P.spacing / 2);
        const bool has = !G.ppm(P.noindel_ppm);
        const bool ins = G.u(2) == 0;
        const int32_t L = 1 + (int32_t)G.u(10);
        std::string insSeq;
        for (int32_t k = 0; k < L; ++k) insSeq += kBases[G.u(4)];
        ivline[gi] = "chr" + std::to_string(c + 1) + ":" + std::to_string(p - 25 + 1) + "-" + std::to_string(p + 25 + 1) + "\n";
        // haplotype base at reference coordinate t (t < p: reference; t >= p: after the indel)
        // read bases of a read whose first base sits at reference coordinate t
        auto cut = [&](int32_t t, std::string &seq) {
            seq.clear();
            for (int32_t k = 0; k < (int32_t)rl; ++k) {
                int32_t x = t + k;
                char b;
                if (!has || x < p) b = R[(size_t)x];
                else if (ins) b = (x - p < L) ? insSeq[(size_t)(x - p)] : R[(size_t)(x - L)];
                else b = R[(size_t)(x + L)];
                seq += upper(b);
            }
        };
        for (uint32_t f = 0; f < P.frags_per_interval; ++f) {
            const int32_t s = p - (int32_t)rl + 10 + (int32_t)G.u(rl + 5 - 10);
            const int32_t isz = (int32_t)(P.ins_min + G.u(P.ins_max - P.ins_min + 1));
            const bool r2ovl = G.u(2) == 1;
            const bool dupf = G.ppm(P.dup_ppm);
            const std::string name = "i" + std::to_string(gi) + "f" + std::to_string(f);
            int32_t start[2];  // read1 (forward), read2 (reverse) first base, reference coordinates
            if (!r2ovl) {
                start[0] = s;
                start[1] = s + isz - (int32_t)rl;
            } else {
                start[1] = s;
                start[0] = s - isz + (int32_t)rl;
            }
            int32_t apos[2];
            std::vector<uint32_t> cig[2];
            std::string seq[2], qual[2], tags[2];
            uint8_t mapq[2];
            for (int m = 0; m < 2; ++m) {
                const int32_t t = start[m];
                // the haplotype bases the read carries; for reads right of the site, the read's
                // reference coordinate is its haplotype coordinate minus the indel shift
                int32_t rt = t;
                bool spans = has && t < p && t + (int32_t)rl > p;
                std::string sq;
                if (has && t >= p) {
                    // sample coordinate t maps to reference t - L (insertion) / t + L (deletion)
                    rt = ins ? t - L : t + L;
                    if (ins && rt < p) rt = p;  // starts inside the insertion: place at p
                }
                cut(t, sq);
                std::vector<uint32_t> cg;
                int32_t a = p - t;
                bool gapped = false;
                int32_t site = p;
                if (spans && G.ppm(P.gapped_ppm)) {
                    if (G.ppm(P.alt_indel_ppm)) site = p + 3;
                    a = site - t;
                    int32_t b = ins ? (int32_t)rl - a - L : (int32_t)rl - a;
                    if (a >= 5 && b >= 5) {
                        gapped = true;
                        cg.push_back((uint32_t)a << 4 | 0);
                        cg.push_back((uint32_t)L << 4 | (ins ? 1u : 2u));
                        cg.push_back((uint32_t)b << 4 | 0);
                    }
                }
                if (!gapped) cg.push_back(rl << 4 | 0);
                // sequencing errors (never inside inserted bases)
                for (int32_t k = 0; k < (int32_t)rl; ++k) {
                    bool inIns = has && ins && t + k >= p && t + k < p + L;
                    if (!inIns && G.ppm(P.err_ppm)) {
                        const char *q = strchr(kBases, sq[(size_t)k]);
                        int bi = q ? (int)(q - kBases) : 0;
                        sq[(size_t)k] = kBases[(bi + 1 + (int)G.u(3)) % 4];
                    }
                }
                int32_t pos = rt;
                if (G.ppm(P.clip_ppm) && (cg[0] >> 4) > 10) {
                    // 5 leading bases soft-clipped: first M block shortened, alignment start +5
                    std::vector<uint32_t> c2;
                    c2.push_back(5u << 4 | 4);
                    c2.push_back(((cg[0] >> 4) - 5) << 4 | (cg[0] & 0xF));
                    c2.insert(c2.end(), cg.begin() + 1, cg.end());
                    cg.swap(c2);
                    pos += 5;
                }
                std::string ql;
                for (uint32_t k = 0; k < rl; ++k) ql += (char)(P.qual_min + G.u(P.qual_max - P.qual_min + 1));
                std::string tg;
                tag_z(tg, "RG", "rg1");
                int32_t nm = gapped ? L : 0;
                tag_i(tg, "NM", nm);
                if (G.ppm(P.md_ppm)) tag_z(tg, "MD", std::to_string(rl));
                if (G.ppm(P.uq_ppm)) tag_i(tg, "UQ", 0);
                apos[m] = pos;
                cig[m] = cg;
                seq[m] = sq;
                qual[m] = ql;
                tags[m] = tg;
                mapq[m] = G.ppm(P.mapq0_ppm) ? 0 : 60;
            }
            for (int m = 0; m < 2; ++m) {
                uint16_t flag = 0x1 | 0x2 | (m == 0 ? (0x40 | 0x20) : (0x80 | 0x10));
                if (dupf) flag |= 0x400;
                int32_t tlen = m == 0 ? isz : -isz;
                Rec r;
                r.key = ((uint64_t)c << 33) | ((uint64_t)(uint32_t)(apos[m] + 1) << 1) | (m == 1 ? 1u : 0u);
                r.name = name;
                r.flag = flag;
                r.bytes = encode(name, flag, (int32_t)c, apos[m], mapq[m], cig[m], seq[m], qual[m], (int32_t)c, apos[1 - m],
                                 tlen, tags[m]);
                recs.push_back(std::move(r));
            }
        }
        std::sort(recs.begin(), recs.end(), [](const Rec &a, const Rec &b) {
            if (a.key != b.key) return a.key < b.key;
            if (a.name != b.name) return a.name < b.name;
            return a.flag < b.flag;
        });
    });
    std::string ivtext;
    for (auto &l : ivline) ivtext += l;
    {
        FILE *f = fopen(intervals_path, "wb");
        if (!f) return oge_fail(nullptr, OGE_ERR_IO, "oge_synth_realign: cannot write intervals");
        fputs(ivtext.c_str(), f);
        fclose(f);
    }
    std::string htext = "@HD\tVN:1.4\tSO:coordinate\n";
    for (uint32_t c = 0; c < P.n_ref; ++c) htext += "@SQ\tSN:chr" + std::to_string(c + 1) + "\tLN:" + std::to_string(clen) + "\n";
    htext += "@RG\tID:rg1\tLB:lib1\tSM:sample1\tPL:illumina\n";
    oge::BamHeaderModel h;
    std::string err;
    if (!h.parse(htext, err)) return oge_fail(nullptr, OGE_ERR_ARG, err.c_str());
    FILE *f = fopen(bam_path, "wb");
    if (!f) return oge_fail(nullptr, OGE_ERR_IO, "oge_synth_realign: cannot write BAM");
    {
        oge::BgzfWriter w(f, level, threads <= 0 ? 8 : threads);
        std::vector<uint8_t> hb = oge::bam_encode_header(h);
        w.write(hb.data(), hb.size());
        for (auto &v : per_iv)
            for (auto &r : v) w.write(r.bytes.data(), r.bytes.size());
        w.close();
    }
    fclose(f);
    return OGE_OK;
}

}  // extern "C"
