// host_capi.cpp -- host-only entry points of libopenge_hip.so: synthetic data, BAM files.
#include "../../include/openge_hip.h"
#include "bamio.h"
#include "capi_common.h"
#include "synth.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

using namespace oge;

template <class F>
static void host_parallel(uint64_t n, int threads, F f) {
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    uint64_t chunk = std::max<uint64_t>(4096, (n + threads * 8 - 1) / (threads * 8));
    std::atomic<uint64_t> next(0);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&]() {
            for (;;) {
                uint64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                uint64_t e = std::min(n, b + chunk);
                for (uint64_t i = b; i < e; ++i) f(i);
            }
        });
    for (auto &t : ts) t.join();
}

extern "C" {

uint64_t oge_synth_params_size(void) { return sizeof(oge_synth_params); }

int oge_synth_finalize(void *params) {
    oge_synth_params *P = (oge_synth_params *)params;
    if (!P || P->n_ref == 0 || P->n_ref > OGE_SYNTH_MAX_REF || P->read_len == 0 || P->read_len > 250 ||
        P->n_rg == 0 || P->n_rg > 9 || P->ins_max < P->ins_min || P->qual_max < P->qual_min || P->qual_max > 255)
        return oge_fail(nullptr, OGE_ERR_ARG, "oge_synth_finalize: parameters out of range");
    P->ref_cum[0] = 0;
    for (uint32_t i = 0; i < P->n_ref; ++i) {
        if (P->ref_len[i] <= (uint64_t)P->ins_max + 1 || P->ref_len[i] > 0x7FFFFFFFull)
            return oge_fail(nullptr, OGE_ERR_ARG, "oge_synth_finalize: contig shorter than the insert size");
        P->ref_cum[i + 1] = P->ref_cum[i] + P->ref_len[i];
    }
    return OGE_OK;
}

int oge_synth_offsets_host(const void *params, uint64_t *offs, int threads) {
    const oge_synth_params *P = (const oge_synth_params *)params;
    uint64_t n = 2 * P->n_pairs;
    std::vector<uint32_t> sz(n);
    host_parallel(n, threads, [&](uint64_t s) { sz[s] = oge_synth_slot_bytes(P, s); });
    uint64_t acc = 0;
    for (uint64_t s = 0; s < n; ++s) { offs[s] = acc; acc += sz[s]; }
    offs[n] = acc;
    return OGE_OK;
}

int oge_synth_records_host(const void *params, const uint64_t *offs, uint8_t *out, int threads) {
    const oge_synth_params *P = (const oge_synth_params *)params;
    uint64_t n = 2 * P->n_pairs;
    host_parallel(n, threads, [&](uint64_t s) { oge_synth_write_slot(P, s, out + offs[s]); });
    return OGE_OK;
}

int oge_synth_header_text(const void *params, char *buf, uint64_t cap, uint64_t *len_out) {
    const oge_synth_params *P = (const oge_synth_params *)params;
    std::string t = "@HD\tVN:1.4\tSO:unsorted\n";
    for (uint32_t i = 0; i < P->n_ref; ++i)
        t += "@SQ\tSN:chr" + std::to_string(i + 1) + "\tLN:" + std::to_string(P->ref_len[i]) + "\n";
    for (uint32_t g = 1; g <= P->n_rg; ++g)
        t += "@RG\tID:rg" + std::to_string(g) + "\tLB:lib" + std::to_string(g) + "\tSM:sample1\n";
    if (len_out) *len_out = t.size();
    if (buf && cap) {
        size_t k = std::min<size_t>(cap - 1, t.size());
        memcpy(buf, t.data(), k);
        buf[k] = 0;
    }
    return OGE_OK;
}

struct oge_bam { BamFile f; };

int oge_bam_read(const char *path, int threads, oge_bam **out) {
    if (!path || !out) return oge_fail(nullptr, OGE_ERR_ARG, "oge_bam_read: null argument");
    oge_bam *b = new oge_bam();
    std::string err;
    if (!bam_read_file(path, b->f, threads <= 0 ? 8 : threads, err)) {
        delete b;
        return oge_fail(nullptr, OGE_ERR_IO, ("oge_bam_read: " + err).c_str());
    }
    *out = b;
    return OGE_OK;
}
void oge_bam_free(oge_bam *b) { delete b; }
uint64_t oge_bam_count(const oge_bam *b) { return b->f.offsets.size(); }
const uint8_t *oge_bam_records(const oge_bam *b, uint64_t *bytes_out) {
    if (bytes_out) *bytes_out = b->f.rec_bytes();
    return b->f.recs();
}
const uint64_t *oge_bam_offsets(const oge_bam *b) { return b->f.offsets.data(); }
int32_t oge_bam_n_ref(const oge_bam *b) { return (int32_t)b->f.ref_names.size(); }

int oge_bam_header_text(const oge_bam *b, char *buf, uint64_t cap, uint64_t *len_out) {
    std::string t = b->f.header.to_string();
    if (len_out) *len_out = t.size();
    if (buf && cap) {
        size_t k = std::min<size_t>(cap - 1, t.size());
        memcpy(buf, t.data(), k);
        buf[k] = 0;
    }
    return OGE_OK;
}

int oge_bam_markdup_opts(const oge_bam *b, oge_markdup_opts *opts, char **rg_ids_buf, int16_t **rg_lib_buf) {
    // Library naming follows getLibraryName (algorithms/mark_duplicates.cpp:301-318): the LB of
    // the record's @RG if present and non-empty, else "Unknown Library".  Distinct names get
    // distinct ids; which id a name gets does not change any duplicate decision.
    const auto &rgs = b->f.header.rg;
    std::map<std::string, int16_t> lib_ids;
    std::string ids;
    int16_t *libs = (int16_t *)malloc(sizeof(int16_t) * std::max<size_t>(1, rgs.size()));
    int16_t next = 1;
    for (size_t i = 0; i < rgs.size(); ++i) {
        std::string lib = rgs[i].lb.empty() ? std::string("Unknown Library") : rgs[i].lb;
        auto it = lib_ids.find(lib);
        if (it == lib_ids.end()) it = lib_ids.emplace(lib, next++).first;
        libs[i] = it->second;
        ids += rgs[i].id;
        ids.push_back('\0');
    }
    auto unk = lib_ids.find("Unknown Library");
    int16_t unknown = unk != lib_ids.end() ? unk->second : next++;
    char *idbuf = (char *)malloc(std::max<size_t>(1, ids.size()));
    memcpy(idbuf, ids.data(), ids.size());
    memset(opts, 0, sizeof(*opts));
    opts->n_ref = (int32_t)b->f.ref_names.size();
    opts->rg_ids = idbuf;
    opts->rg_ids_bytes = ids.size();
    opts->rg_lib = libs;
    opts->n_rg = (int32_t)rgs.size();
    opts->unknown_lib = unknown;
    *rg_ids_buf = idbuf;
    *rg_lib_buf = libs;
    return OGE_OK;
}

int oge_bam_write(const char *path, const char *header_text, uint64_t header_len, int sort_order,
                  const uint8_t *recs, const uint64_t *offs, uint64_t n, const uint32_t *order,
                  const uint16_t *flags, int level, int threads) {
    BamHeaderModel h;
    std::string err;
    if (!h.parse(std::string(header_text, header_len), err))
        return oge_fail(nullptr, OGE_ERR_ARG, ("oge_bam_write: " + err).c_str());
    if (sort_order >= 0) h.sort_order = (BamHeaderModel::SortOrder)sort_order;
    FILE *f = (strcmp(path, "-") == 0 || strcmp(path, "stdout") == 0) ? stdout : fopen(path, "wb");
    if (!f) return oge_fail(nullptr, OGE_ERR_IO, "oge_bam_write: cannot open output");
    {
        BgzfWriter w(f, level, threads <= 0 ? 8 : threads);
        std::vector<uint8_t> hb = bam_encode_header(h);
        w.write(hb.data(), hb.size());
        std::vector<uint8_t> tmp;
        for (uint64_t k = 0; k < n; ++k) {
            uint64_t i = order ? order[k] : k;
            const uint8_t *r = recs + offs[i];
            uint32_t bs;
            memcpy(&bs, r, 4);
            // BamSerializer::write recomputes bin on every record (util/bam_serializer.h:112-116)
            tmp.assign(r, r + 4 + bs);
            oge_wr_u16(tmp.data() + OGE_OFF_BIN, oge_rec_bin(tmp.data()));
            if (flags) oge_wr_u16(tmp.data() + OGE_OFF_FLAG, flags[i]);
            w.write(tmp.data(), tmp.size());
        }
        w.close();
    }
    if (f != stdout) fclose(f);
    return OGE_OK;
}

} // extern "C"

// ----------------------------------------------------------------------------- Filter (mergesort -r/-q)
extern "C" void oge_filter_opts_init(oge_filter_opts *o) {  // Filter::Filter (filter.cpp:185-194)
    if (!o) return;
    memset(o, 0, sizeof *o);
    o->max_len = INT32_MAX;
    o->count_limit = INT32_MAX;
}

// Filter::ParseRegionString (filter.cpp:31-137): the same parse (atoi on the pieces, so "chr:5-9"
// reads as the single position 5), the last dictionary entry of that name, the same range checks.
extern "C" int oge_parse_region(const char *region, const char *ref_names, int32_t n_ref, const int64_t *ref_len,
                                oge_filter_opts *o) {
    if (!region || !o || (n_ref > 0 && (!ref_names || !ref_len))) return oge_fail(nullptr, OGE_ERR_ARG, "null argument");
    const std::string rs = region;
    const std::string bad = "ERROR: could not parse region'" + rs + "'";
    if (rs.empty()) return oge_fail(nullptr, OGE_ERR_ARG, bad.c_str());
    std::string chrom;
    int start, stop;
    const size_t c1 = rs.find(':');
    if (c1 == std::string::npos) {
        chrom = rs;
        start = 0;
        stop = -1;
    } else {
        chrom = rs.substr(0, c1);
        const size_t dots = rs.find("..", c1 + 1);
        if (dots == std::string::npos) {
            start = atoi(rs.substr(c1 + 1).c_str());
            stop = start;
        } else {
            start = atoi(rs.substr(c1 + 1, dots - c1 - 1).c_str());
            if (rs.find(':', dots + 1) != std::string::npos) return oge_fail(nullptr, OGE_ERR_ARG, bad.c_str());
            stop = atoi(rs.substr(dots + 2).c_str());
        }
    }
    int ref = -1;
    const char *p = ref_names;
    for (int i = 0; i < n_ref; ++i) {
        if (chrom == p) ref = i;
        p += strlen(p) + 1;
    }
    if (ref == -1) return oge_fail(nullptr, OGE_ERR_ARG, ("Can't find chromosome'" + chrom + "'").c_str());
    const int len = (int)ref_len[ref];
    if (start >= len)
        return oge_fail(nullptr, OGE_ERR_ARG,
                        ("Start position (" + std::to_string(start) + ") after end of the reference sequence (" +
                         std::to_string(len) + ")").c_str());
    if (stop > len)  // the reference's message says "Start" here too (filter.cpp:125)
        return oge_fail(nullptr, OGE_ERR_ARG,
                        ("Start position (" + std::to_string(stop) + ") after end of the reference sequence (" +
                         std::to_string(len) + ")").c_str());
    if (stop == -1) stop = len;
    o->has_region = 1;
    o->ref_id = ref;
    o->left_pos = start;
    o->right_pos = stop;
    return OGE_OK;
}
