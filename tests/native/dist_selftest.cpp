// dist_selftest.cpp -- CPU harness for the multi-GPU partition code (openge_amd/csrc/dist_plan.h,
// dist_local.h): G threads run the same schedule dist.hip runs on G GPUs -- sample keys, pool the
// samples, choose range splitters, route every key to its owner, plan and run the all-to-all, sort
// locally -- over the in-process hub with memcpy as the transport.  Checks: the rank slices
// concatenate into the global sorted order, equal keys never straddle ranks, load max/mean, and the
// max reduce-scatter the dedup uses.  Built and run by tests/test_dist_plan.py (also under TSan).
//
//   dist_selftest KEYS_FILE G...      (KEYS_FILE: little-endian u64 ByPosition keys in input order)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

#include "dist_local.h"
#include "dist_plan.h"

using namespace oge_dist;

struct HostOps {
    int copy(void *d, const void *s, size_t n) {
        memcpy(d, s, n);
        return 0;
    }
    int sync() { return 0; }
    int max_into(uint8_t *acc, const uint8_t *src, size_t n) {
        for (size_t i = 0; i < n; ++i) acc[i] = std::max(acc[i], src[i]);
        return 0;
    }
};

static int run(const std::vector<uint64_t> &keys, int G, double *balance) {
    Hub hub(G);
    const uint64_t N = keys.size();
    std::vector<std::vector<uint64_t>> slices(G);
    std::vector<int> fail(G, 0);
    std::vector<std::vector<uint8_t>> rs_out(G);
    auto rank_main = [&](int r) {
        HostOps ops;
        LocalColl<HostOps> c{hub, r, ops};
        const uint64_t lo = N * r / G, hi = N * (r + 1) / G, n = hi - lo;
        const uint64_t *mine = keys.data() + lo;
        // samples
        const uint32_t m = (uint32_t)std::min<uint64_t>(n, kSamples);
        std::vector<uint64_t> samp(kSamples, 0);
        for (uint32_t i = 0; i < m; ++i) samp[i] = mine[sample_pos(n, m, i)];
        std::vector<uint64_t> all((size_t)G * kSamples);
        c.allgather_host(samp.data(), all.data(), kSamples * 8);
        const uint64_t nm[2] = {n, m};
        std::vector<uint64_t> allnm(2 * G);
        c.allgather_host(nm, allnm.data(), 16);
        std::vector<std::vector<uint64_t>> per(G);
        std::vector<uint64_t> ns(G);
        for (int g = 0; g < G; ++g) {
            ns[g] = allnm[2 * g];
            per[g].assign(all.begin() + (size_t)g * kSamples, all.begin() + (size_t)g * kSamples + allnm[2 * g + 1]);
        }
        const std::vector<uint64_t> spl = choose_splitters(per, ns, G);
        // route (stable by input order)
        std::vector<std::vector<uint64_t>> by(G);
        for (uint64_t i = 0; i < n; ++i) by[owner_of(mine[i], spl.data(), (uint32_t)spl.size())].push_back(mine[i]);
        std::vector<uint64_t> cnt(G), send;
        for (int g = 0; g < G; ++g) {
            cnt[g] = by[g].size();
            send.insert(send.end(), by[g].begin(), by[g].end());
        }
        std::vector<uint64_t> allc((size_t)G * G);
        c.allgather_host(cnt.data(), allc.data(), G * 8);
        const Plan p = plan_from_counts(allc, G, r);
        std::vector<uint64_t> sb(G), so(G), rb(G), ro(G);
        for (int g = 0; g < G; ++g) sb[g] = 8 * p.scnt[g], so[g] = 8 * p.soff[g], rb[g] = 8 * p.rcnt[g], ro[g] = 8 * p.roff[g];
        std::vector<uint64_t> recv(p.rtot + 1);
        if (c.alltoallv(send.data(), sb.data(), so.data(), recv.data(), rb.data(), ro.data())) fail[r] = 1;
        recv.resize(p.rtot);
        std::stable_sort(recv.begin(), recv.end());
        slices[r] = recv;
        // max reduce-scatter: rank r marks byte i of chunk g when (i * 7 + r) % (G + 3) == 0
        const size_t chunk = 1000;
        std::vector<uint8_t> pad((size_t)G * chunk, 0);
        for (size_t i = 0; i < pad.size(); ++i) pad[i] = (uint8_t)(((i * 7 + r) % (G + 3)) == 0 ? 1 + r : 0);
        rs_out[r].assign(chunk, 0);
        if (c.reduce_scatter_max_u8(pad.data(), rs_out[r].data(), chunk)) fail[r] = 1;
    };
    std::vector<std::thread> ts;
    for (int r = 0; r < G; ++r) ts.emplace_back(rank_main, r);
    for (auto &t : ts) t.join();
    for (int r = 0; r < G; ++r)
        if (fail[r]) return fprintf(stderr, "rank %d: collective failed\n", r), 1;
    // concatenation == global sort
    std::vector<uint64_t> cat, ref = keys;
    for (auto &s : slices) cat.insert(cat.end(), s.begin(), s.end());
    std::stable_sort(ref.begin(), ref.end());
    if (cat != ref) return fprintf(stderr, "G=%d: slices do not concatenate into the sorted order\n", G), 1;
    for (int r = 0; r + 1 < G; ++r)
        if (!slices[r].empty() && !slices[r + 1].empty() && slices[r].back() == slices[r + 1].front())
            return fprintf(stderr, "G=%d: a key straddles ranks %d and %d\n", G, r, r + 1), 1;
    uint64_t mx = 0;
    for (auto &s : slices) mx = std::max<uint64_t>(mx, s.size());
    *balance = N ? (double)mx / ((double)N / G) : 1.0;
    // reduce-scatter expectation
    for (int r = 0; r < G; ++r)
        for (size_t i = 0; i < 1000; ++i) {
            uint8_t want = 0;
            for (int q = 0; q < G; ++q) {
                const size_t gi = (size_t)r * 1000 + i;
                want = std::max<uint8_t>(want, ((gi * 7 + q) % (G + 3)) == 0 ? 1 + q : 0);
            }
            if (rs_out[r][i] != want) return fprintf(stderr, "G=%d: reduce-scatter mismatch\n", G), 1;
        }
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) return fprintf(stderr, "usage: dist_selftest KEYS_FILE G...\n"), 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return perror(argv[1]), 2;
    std::vector<uint64_t> keys;
    uint64_t k;
    while (fread(&k, 8, 1, f) == 1) keys.push_back(k);
    fclose(f);
    printf("{");
    for (int a = 2; a < argc; ++a) {
        const int G = atoi(argv[a]);
        double bal = 0;
        if (run(keys, G, &bal)) return 1;
        printf("%s\"%d\": %.4f", a > 2 ? ", " : "", G, bal);
    }
    printf("}\n");
    return 0;
}
