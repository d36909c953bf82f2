// dist_selftest.cpp -- CPU harness for the multi-GPU partition code (openge_amd/csrc/dist_plan.h,
// dist_local.h): G threads run the same schedule dist.hip runs on G GPUs -- sample keys, pool the
// samples, choose range splitters, route every key to its owner, plan and run the all-to-all, sort
// locally -- over the in-process hub with memcpy as the transport.  Checks: the rank slices
// concatenate into the global sorted order, equal keys never straddle ranks, load max/mean, and the
// max reduce-scatter the dedup uses.  Built and run by tests/test_dist_plan.py (also under TSan).
//
// The same schedule also runs over the host-staged transport (dist_shm.h) between G forked PROCESSES
// meeting in a shared file mapping, with a staging area small enough to force many rounds (--shm), and
// with one rank's copy operation failing (--fail-copy): every rank must return, the failing one with
// its error, instead of hanging in the next collective.
//
//   dist_selftest KEYS_FILE G...          (KEYS_FILE: little-endian u64 ByPosition keys in input order)
//   dist_selftest --shm KEYS_FILE G...
//   dist_selftest --fail-copy G...
//   dist_selftest --dead-rank G...        (the last rank's process exits after joining: the others must
//                                          return with an error long before OGE_COMM_TIMEOUT)
#include <sys/wait.h>
#include <unistd.h>

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
#include "dist_shm.h"

using namespace oge_dist;

struct HostOps {
    bool fail = false;  // --fail-copy: this rank's copies fail
    int copy(void *d, const void *s, size_t n) {
        if (fail) return -1;
        memcpy(d, s, n);
        return 0;
    }
    int d2h(void *d, const void *s, size_t n) { return copy(d, s, n); }
    int h2d(void *d, const void *s, size_t n) { return copy(d, s, n); }
    int d2d(void *d, const void *s, size_t n) { return copy(d, s, n); }
    int sync() { return 0; }
    int max_into(uint8_t *acc, const uint8_t *src, size_t n) {
        for (size_t i = 0; i < n; ++i) acc[i] = std::max(acc[i], src[i]);
        return 0;
    }
};

// One rank's schedule over any collective (LocalColl over the hub, ShmColl over the shared segment):
// sample, splitters, route, plan, exchange, local sort; then the max reduce-scatter.  Returns 0 / 1.
template <class Coll>
static int rank_schedule(Coll &c, int r, int G, const std::vector<uint64_t> &keys, std::vector<uint64_t> &slice,
                         std::vector<uint8_t> &rs_out) {
    const uint64_t N = keys.size();
    const uint64_t lo = N * r / G, hi = N * (r + 1) / G, n = hi - lo;
    const uint64_t *mine = keys.data() + lo;
    const uint32_t m = (uint32_t)std::min<uint64_t>(n, kSamples);
    std::vector<uint64_t> samp(kSamples, 0);
    for (uint32_t i = 0; i < m; ++i) samp[i] = mine[sample_pos(n, m, i)];
    std::vector<uint64_t> all((size_t)G * kSamples);
    int fail = 0;
    if (c.allgather_host(samp.data(), all.data(), kSamples * 8)) fail = 1;
    const uint64_t nm[2] = {n, m};
    std::vector<uint64_t> allnm(2 * G);
    if (c.allgather_host(nm, allnm.data(), 16)) fail = 1;
    std::vector<std::vector<uint64_t>> per(G);
    std::vector<uint64_t> ns(G);
    for (int g = 0; g < G; ++g) {
        ns[g] = allnm[2 * g];
        per[g].assign(all.begin() + (size_t)g * kSamples, all.begin() + (size_t)g * kSamples + allnm[2 * g + 1]);
    }
    const std::vector<uint64_t> spl = choose_splitters(per, ns, G);
    std::vector<std::vector<uint64_t>> by(G);
    for (uint64_t i = 0; i < n; ++i) by[owner_of(mine[i], spl.data(), (uint32_t)spl.size())].push_back(mine[i]);
    std::vector<uint64_t> cnt(G), send;
    for (int g = 0; g < G; ++g) {
        cnt[g] = by[g].size();
        send.insert(send.end(), by[g].begin(), by[g].end());
    }
    std::vector<uint64_t> allc((size_t)G * G);
    if (c.allgather_host(cnt.data(), allc.data(), G * 8)) fail = 1;
    const Plan p = plan_from_counts(allc, G, r);
    std::vector<uint64_t> sb(G), so(G), rb(G), ro(G);
    for (int g = 0; g < G; ++g) sb[g] = 8 * p.scnt[g], so[g] = 8 * p.soff[g], rb[g] = 8 * p.rcnt[g], ro[g] = 8 * p.roff[g];
    std::vector<uint64_t> recv(p.rtot + 1);
    if (c.alltoallv(send.data(), sb.data(), so.data(), recv.data(), rb.data(), ro.data())) fail = 1;
    recv.resize(p.rtot);
    std::stable_sort(recv.begin(), recv.end());
    slice = recv;
    // max reduce-scatter: rank r marks byte i of chunk g when (i * 7 + r) % (G + 3) == 0
    const size_t chunk = 1000;
    std::vector<uint8_t> pad((size_t)G * chunk, 0);
    for (size_t i = 0; i < pad.size(); ++i) pad[i] = (uint8_t)(((i * 7 + r) % (G + 3)) == 0 ? 1 + r : 0);
    rs_out.assign(chunk, 0);
    if (c.reduce_scatter_max_u8(pad.data(), rs_out.data(), chunk)) fail = 1;
    return fail;
}

// the rank slices concatenate into the global sorted order, no key straddles two ranks, and the
// reduce-scatter gives the elementwise max
static int verify(const std::vector<uint64_t> &keys, int G, const std::vector<std::vector<uint64_t>> &slices,
                  const std::vector<std::vector<uint8_t>> &rs_out, double *balance) {
    const uint64_t N = keys.size();
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
    for (int r = 0; r < G; ++r) {
        if (rs_out[r].size() != 1000) return fprintf(stderr, "G=%d: reduce-scatter output missing\n", G), 1;
        for (size_t i = 0; i < 1000; ++i) {
            uint8_t want = 0;
            for (int q = 0; q < G; ++q) {
                const size_t gi = (size_t)r * 1000 + i;
                want = std::max<uint8_t>(want, ((gi * 7 + q) % (G + 3)) == 0 ? 1 + q : 0);
            }
            if (rs_out[r][i] != want) return fprintf(stderr, "G=%d: reduce-scatter mismatch\n", G), 1;
        }
    }
    return 0;
}

// G threads over the in-process hub; fail_rank >= 0: that rank's copies fail
static int run(const std::vector<uint64_t> &keys, int G, double *balance, int fail_rank = -1) {
    Hub hub(G);
    std::vector<std::vector<uint64_t>> slices(G);
    std::vector<int> fail(G, 0);
    std::vector<std::vector<uint8_t>> rs_out(G);
    auto rank_main = [&](int r) {
        HostOps ops;
        ops.fail = r == fail_rank;
        LocalColl<HostOps> c{hub, r, ops};
        fail[r] = rank_schedule(c, r, G, keys, slices[r], rs_out[r]);
    };
    std::vector<std::thread> ts;
    for (int r = 0; r < G; ++r) ts.emplace_back(rank_main, r);
    for (auto &t : ts) t.join();  // every rank returned
    if (fail_rank >= 0) return fail[fail_rank] ? 0 : (fprintf(stderr, "hub: the failing rank reported success\n"), 1);
    for (int r = 0; r < G; ++r)
        if (fail[r]) return fprintf(stderr, "rank %d: collective failed\n", r), 1;
    return verify(keys, G, slices, rs_out, balance);
}

// G forked processes over the host-staged transport (shared file mapping); results come back in files
static int run_shm(const std::vector<uint64_t> &keys, int G, double *balance, int fail_rank = -1, int dead_rank = -1,
                   int foreign_rank = -1) {
    char dir[] = "/tmp/oge_shm_selftestXXXXXX";
    if (!mkdtemp(dir)) return perror("mkdtemp"), 1;
    char name[64];
    snprintf(name, sizeof name, "oge_comm_selftest_%d_%d", (int)getpid(), G);
    const uint64_t W = ShmSeg::default_stage_bytes();
    std::vector<pid_t> kids;
    for (int r = 0; r < G; ++r) {
        const pid_t pid = fork();
        if (pid < 0) return perror("fork"), 1;
        if (pid == 0) {
            std::string err;
            ShmSeg *seg = ShmSeg::open(name, G, r, W, "selftest", &err);
            if (!seg) {
                fprintf(stderr, "rank %d: %s\n", r, err.c_str());
                _exit(3);
            }
            if (r == foreign_rank) {  // a rank in another pid namespace: its posted pid does not exist here
                seg->pose_as_foreign();
                usleep(1500 * 1000);  // the others wait (and check liveness) long enough to have judged it
            }
            if (r == dead_rank) _exit(7);  // gone before the first collective
            HostOps ops;
            ops.fail = r == fail_rank;
            ShmColl<HostOps> c{*seg, ops};
            std::vector<uint64_t> slice;
            std::vector<uint8_t> rs;
            const int f = rank_schedule(c, r, G, keys, slice, rs);
            const std::string out = std::string(dir) + "/rank" + std::to_string(r);
            FILE *o = fopen(out.c_str(), "wb");
            const uint64_t ns = slice.size();
            fwrite(&ns, 8, 1, o);
            fwrite(slice.data(), 8, ns, o);
            fwrite(rs.data(), 1, rs.size(), o);
            fclose(o);
            delete seg;
            _exit(f ? 4 : 0);
        }
        kids.push_back(pid);
    }
    std::vector<int> status(G);
    for (int k = 0; k < G; ++k) {  // reap in exit order (a launcher does: an exited rank is no zombie)
        int st = 0;
        const pid_t pid = waitpid(-1, &st, 0);
        for (int r = 0; r < G; ++r)
            if (kids[r] == pid) status[r] = WIFEXITED(st) ? WEXITSTATUS(st) : 128;
    }
    std::vector<std::vector<uint64_t>> slices(G);
    std::vector<std::vector<uint8_t>> rs_out(G);
    for (int r = 0; r < G; ++r) {
        const std::string in = std::string(dir) + "/rank" + std::to_string(r);
        FILE *f = fopen(in.c_str(), "rb");
        uint64_t ns = 0;
        if (f && fread(&ns, 8, 1, f) == 1) {
            slices[r].resize(ns);
            if (fread(slices[r].data(), 8, ns, f) != ns) slices[r].clear();
            rs_out[r].resize(1000);
            if (fread(rs_out[r].data(), 1, 1000, f) != 1000) rs_out[r].clear();
        }
        if (f) fclose(f);
        unlink(in.c_str());
    }
    rmdir(dir);
    if (fail_rank >= 0) {
        for (int r = 0; r < G; ++r)
            if (status[r] != (r == fail_rank ? 4 : 0))
                return fprintf(stderr, "shm: rank %d exited %d\n", r, status[r]), 1;
        return 0;
    }
    if (dead_rank >= 0) {
        for (int r = 0; r < G; ++r)
            if (status[r] != (r == dead_rank ? 7 : 4))
                return fprintf(stderr, "shm: rank %d exited %d\n", r, status[r]), 1;
        return 0;
    }
    for (int r = 0; r < G; ++r)
        if (status[r]) return fprintf(stderr, "shm: rank %d exited %d\n", r, status[r]), 1;
    return verify(keys, G, slices, rs_out, balance);
}

static std::vector<uint64_t> load_keys(const char *path) {
    std::vector<uint64_t> keys;
    FILE *f = fopen(path, "rb");
    if (!f) return perror(path), keys;
    uint64_t k;
    while (fread(&k, 8, 1, f) == 1) keys.push_back(k);
    fclose(f);
    return keys;
}

int main(int argc, char **argv) {
    if (argc < 3) return fprintf(stderr, "usage: dist_selftest [--shm] KEYS_FILE G... | --fail-copy G...\n"), 2;
    if (!strcmp(argv[1], "--fail-copy")) {
        std::vector<uint64_t> keys(50000);
        std::mt19937_64 rng(5);
        for (auto &k : keys) k = rng() >> 20;
        for (int a = 2; a < argc; ++a) {
            const int G = atoi(argv[a]);
            double bal = 0;
            if (run(keys, G, &bal, G - 1) || run_shm(keys, G, &bal, G - 1)) return 1;
        }
        printf("{}\n");
        return 0;
    }
    if (!strcmp(argv[1], "--foreign-pid") || !strcmp(argv[1], "--foreign-dead")) {
        // a live rank posting a pid that does not exist in this namespace must not be taken for dead; a
        // foreign rank that exits is found by its stopped heartbeat (OGE_COMM_STALE_S)
        const bool dies = !strcmp(argv[1], "--foreign-dead");
        std::vector<uint64_t> keys(50000);
        std::mt19937_64 rng(7);
        for (auto &k : keys) k = rng() >> 20;
        for (int a = 2; a < argc; ++a) {
            const int G = atoi(argv[a]);
            double bal = 0;
            if (run_shm(keys, G, &bal, -1, dies ? G - 1 : -1, G - 1)) return 1;
        }
        printf("{}\n");
        return 0;
    }
    if (!strcmp(argv[1], "--dead-rank")) {
        std::vector<uint64_t> keys(50000);
        std::mt19937_64 rng(6);
        for (auto &k : keys) k = rng() >> 20;
        for (int a = 2; a < argc; ++a) {
            const int G = atoi(argv[a]);
            double bal = 0;
            if (run_shm(keys, G, &bal, -1, G - 1)) return 1;
        }
        printf("{}\n");
        return 0;
    }
    const bool shm = !strcmp(argv[1], "--shm");
    const int a0 = shm ? 3 : 2;
    const std::vector<uint64_t> keys = load_keys(argv[a0 - 1]);
    printf("{");
    for (int a = a0; a < argc; ++a) {
        const int G = atoi(argv[a]);
        double bal = 0;
        if (shm ? run_shm(keys, G, &bal) : run(keys, G, &bal)) return 1;
        printf("%s\"%d\": %.4f", a > a0 ? ", " : "", G, bal);
    }
    printf("}\n");
    return 0;
}
