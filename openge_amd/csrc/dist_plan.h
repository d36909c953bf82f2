// dist_plan.h -- host-side planning of the multi-GPU sort + dedup (dist.hip): range splitters on the
// packed coordinate key, the owner of a key, and the all-to-all exchange plan.  Plain C++ (also
// built into the CPU test harness tests/native/dist_selftest.cpp); OGE_DIST_HD functions also run on the
// device.
//
// Replaces the reference's split-by-chromosome routing (alg/split_by_chromosome.cpp:30-58: chain =
// refID % K) and re-merge (alg/sorted_merge.cpp:66-101): rank r owns the key range
// [spl[r-1], spl[r]) of the ByPosition key (refID', pos, strand) (bt/Sort.h:116-127), so rank
// outputs concatenate into the global order and records that tie on the key (ordered by name and
// flag, :128-132) never straddle two ranks.
#pragma once
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#define OGE_DIST_HD __host__ __device__
#else
#define OGE_DIST_HD
#endif

namespace oge_dist {

// Samples per rank: pooled over 8 ranks, the quantile error of a range is ~1/sqrt(8 * m) of the total
// (0.3%), well inside the 1.05 max/mean bound.
constexpr uint32_t kSamples = 16384;

// position of sample i of m in an array of n (evenly spaced, midpoints)
OGE_DIST_HD inline uint64_t sample_pos(uint64_t n, uint32_t m, uint32_t i) { return (n * (2ull * i + 1)) / (2ull * m); }

// owner rank of a key: the number of splitters <= key (equal keys share an owner)
OGE_DIST_HD inline uint32_t owner_of(uint64_t key, const uint64_t *spl, uint32_t nspl) {
    uint32_t lo = 0, hi = nspl;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (spl[mid] <= key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Splitters from every rank's sample: samples[r] holds up to kSamples keys of rank r, which holds
// n[r] records, so each of its samples stands for n[r] / |samples[r]| records.  Splitter j is the
// first pooled key whose cumulative weight reaches j / G of the total.  With no records at all every
// splitter is the largest key (everything on rank 0).
inline std::vector<uint64_t> choose_splitters(const std::vector<std::vector<uint64_t>> &samples,
                                              const std::vector<uint64_t> &n, int G) {
    std::vector<std::pair<uint64_t, double>> w;
    double total = 0;
    for (size_t r = 0; r < samples.size(); ++r) {
        if (samples[r].empty()) continue;
        const double each = (double)n[r] / (double)samples[r].size();
        for (uint64_t k : samples[r]) w.push_back({k, each});
        total += (double)n[r];
    }
    std::sort(w.begin(), w.end());
    std::vector<uint64_t> spl(G > 1 ? G - 1 : 0, ~0ull);
    double cum = 0;
    size_t i = 0;
    for (int j = 1; j < G; ++j) {
        const double target = total * j / G;
        while (i < w.size() && cum + w[i].second <= target) cum += w[i++].second;
        spl[j - 1] = i < w.size() ? w[i].first : ~0ull;
    }
    return spl;
}

// All-to-all plan of one rank from every rank's per-destination counts (cnt[src * G + dst]).
struct Plan {
    std::vector<uint64_t> scnt, soff, rcnt, roff;  // G each (+1 for the offsets)
    uint64_t stot = 0, rtot = 0;
};
inline Plan plan_from_counts(const std::vector<uint64_t> &cnt, int G, int rank) {
    Plan p;
    p.scnt.assign(cnt.begin() + (size_t)rank * G, cnt.begin() + (size_t)(rank + 1) * G);
    p.soff.assign(G + 1, 0);
    p.rcnt.assign(G, 0);
    p.roff.assign(G + 1, 0);
    for (int d = 0; d < G; ++d) p.soff[d + 1] = p.soff[d] + p.scnt[d];
    for (int s = 0; s < G; ++s) p.rcnt[s] = cnt[(size_t)s * G + rank];
    for (int s = 0; s < G; ++s) p.roff[s + 1] = p.roff[s] + p.rcnt[s];
    p.stot = p.soff[G];
    p.rtot = p.roff[G];
    return p;
}

// Owner of the hash-routed exchanges (mate join by RG:name hash, pair groups by chunk-key hash).
OGE_DIST_HD inline uint32_t hash_owner(uint64_t h, uint32_t G) {
    h ^= h >> 29;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 32;
    return (uint32_t)(((h & 0xffffffffull) * G) >> 32);
}

}  // namespace oge_dist
