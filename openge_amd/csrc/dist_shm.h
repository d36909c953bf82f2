// dist_shm.h -- the host-staged transport of the multi-GPU path: ranks that are processes (or threads)
// of one node meet in a shared file mapping and move device buffers through it (device -> host slot ->
// device).  It is what `oge_comm_init_rank` uses when ranks share a GPU (RCCL refuses two ranks on one
// device), so the one-process-per-rank bootstrap of bench.py / the CLI runs unchanged on a one-GPU box;
// between distinct GPUs the same calls go over RCCL (dist.hip).
//
// Segment layout: ShmCtl (barrier words, per-rank posts) | rank 0 outbox (W bytes) | ... | rank G-1
// outbox.  An outbox is cut into G slots of S bytes: slot (from, to).  A collective moves its data in
// rounds of at most S bytes per pair; every rank runs the same number of rounds (the maximum over all
// ranks, read from the posts), each round = copy out, barrier, copy in, barrier, so a rank whose own
// copies fail still keeps every barrier and the collective ends on all ranks (its status is returned).
//
// The schedule is plain C++; Ops supplies the memory operations (HIP copies on the context stream in
// the library, memcpy in tests/native/dist_selftest.cpp, which runs it across forked processes).
//   Ops: int d2h(void *h, const void *d, size_t n); int h2d(void *d, const void *h, size_t n);
//        int d2d(void *d, const void *s, size_t n); int sync();   (0 = ok)
#pragma once
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <cerrno>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace oge_dist {

constexpr int kShmMaxRanks = 64;

struct ShmRankPost {
    char bus[64];         // PCI bus id of the rank's device (the meeting's question)
    int64_t pid;
    uint64_t pidns;       // inode of the rank's /proc/self/ns/pid: its pid means something here only if equal
    std::atomic<uint64_t> beat;  // bumped by the rank's heartbeat thread while its segment is open
    uint64_t stage_bytes; // W as this rank computed it (must agree)
    uint64_t maxb;        // largest byte count this rank sends to another rank in the current collective
    uint64_t sb[kShmMaxRanks];  // bytes for each destination in the current collective
    uint8_t pad[48];
};

struct ShmCtl {
    std::atomic<uint32_t> joined;
    std::atomic<uint32_t> count;
    std::atomic<uint32_t> gen;
    std::atomic<uint32_t> broken;  // a rank timed out: every barrier fails from now on
    uint8_t pad0[48];
    ShmRankPost post[kShmMaxRanks];
};

class ShmSeg {
public:
    ~ShmSeg() {
        stop_.store(true);
        if (hb_.joinable()) hb_.join();
        if (base_) munmap(base_, size_);
    }
    int size() const { return G_; }
    int rank() const { return rank_; }
    uint64_t stage_bytes() const { return W_; }
    uint64_t slot_bytes() const { return S_; }
    ShmRankPost &post(int r) { return ctl_->post[r]; }
    uint8_t *outbox(int r) { return base_ + hdr_ + (uint64_t)r * W_; }
    uint8_t *slot(int from, int to) { return outbox(from) + (uint64_t)to * S_; }
    const std::string &error() const { return err_; }

    // Directory of the segment: OGE_COMM_DIR, else /dev/shm when its size holds the segment with room
    // to spare, else /tmp.  A rule of the node's mounts only, so every rank picks the same place.
    static std::string dir_for(uint64_t bytes) {
        if (const char *d = getenv("OGE_COMM_DIR")) return d;
        struct statvfs v;
        if (statvfs("/dev/shm", &v) == 0 && (uint64_t)v.f_blocks * v.f_frsize >= 4 * bytes) return "/dev/shm";
        return "/tmp";
    }
    static uint64_t default_stage_bytes() {  // per-rank outbox, OGE_COMM_STAGE_MB (default 32)
        const char *e = getenv("OGE_COMM_STAGE_MB");
        const long mb = e && *e ? atol(e) : 32;
        return (uint64_t)std::min<long>(std::max<long>(mb, 1), 4096) << 20;
    }
    // A wait ends early when a peer process is gone: its posted pid no longer exists (only trusted when the
    // peer posted this process's pid namespace), or -- for a peer in another pid namespace (containers
    // sharing one IPC namespace) -- its heartbeat has not moved for OGE_COMM_STALE_S seconds.  The wall-clock
    // limit (OGE_COMM_TIMEOUT, default 1800 s) is only the backstop for a live peer that never arrives, so
    // a slow rank (a larger input, a GPU under contention) does not break the communicator.
    // Trade-off: the heartbeat thread of a LIVE peer that is frozen or starved of CPU (SIGSTOP, a
    // frozen cgroup, a checkpoint) stops moving too, and once it has been still for the stale limit the
    // communicator breaks for good, exactly as if the peer had died.  So the limit is a large fraction of the
    // timeout rather than a fixed few seconds: by default a quarter of OGE_COMM_TIMEOUT, at least 60 s (450 s
    // with the default timeout; a heartbeat moves every 100 ms), and OGE_COMM_STALE_S overrides it.  Only
    // peers in another pid namespace are judged this way; a peer in this one is judged by its pid alone.
    static double stale_beat_s() {
        const char *e = getenv("OGE_COMM_STALE_S");
        const double t = e && *e ? atof(e) : 0.0;
        return t > 0 ? t : std::max(60.0, timeout_s() / 4);
    }
    static uint64_t pid_namespace() {
        struct stat st;
        return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0;
    }
    static double timeout_s() {
        const char *e = getenv("OGE_COMM_TIMEOUT");
        const double t = e && *e ? atof(e) : 1800.0;
        return t > 0 ? t : 1800.0;
    }

    // Every rank calls open with the same name; returns after all G ranks have joined (or nullptr on a
    // failure / timeout, with *err set).  The file is unlinked once everyone has it mapped.  meet_s > 0 bounds
    // the wait for the others (else OGE_COMM_TIMEOUT).
    static ShmSeg *open(const std::string &name, int G, int rank, uint64_t W, const char *bus, std::string *err,
                        double meet_s = 0) {
        if (G < 1 || G > kShmMaxRanks || rank < 0 || rank >= G) {
            *err = "host transport: bad rank / size";
            return nullptr;
        }
        auto *s = new ShmSeg();
        s->G_ = G, s->rank_ = rank, s->W_ = W;
        s->S_ = (W / (uint64_t)G) & ~(uint64_t)4095;
        if (s->S_ == 0) {
            delete s;
            *err = "host transport: staging area too small for the rank count";
            return nullptr;
        }
        s->hdr_ = (sizeof(ShmCtl) + 4095) & ~(size_t)4095;
        s->size_ = s->hdr_ + (size_t)G * W;
        const std::string path = dir_for(s->size_) + "/" + name;
        const int fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0600);
        if (fd < 0) {
            *err = "host transport: cannot open " + path + ": " + strerror(errno);
            delete s;
            return nullptr;
        }
        // every rank extends the file to the same size (idempotent; never shrinks what a peer wrote)
        struct stat st;
        int rc = fstat(fd, &st);
        if (rc == 0 && (uint64_t)st.st_size < s->size_) rc = ftruncate(fd, (off_t)s->size_);
        void *p = rc == 0 ? mmap(nullptr, s->size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
        ::close(fd);
        if (p == MAP_FAILED) {
            *err = "host transport: cannot map " + path + ": " + strerror(errno);
            delete s;
            return nullptr;
        }
        s->base_ = (uint8_t *)p;
        s->ctl_ = (ShmCtl *)p;
        ShmRankPost &me = s->ctl_->post[rank];
        snprintf(me.bus, sizeof me.bus, "%s", bus ? bus : "");
        me.pid = (int64_t)getpid();
        me.pidns = pid_namespace();
        me.stage_bytes = W;
        s->my_ns_ = me.pidns;
        s->seen_.assign(G, {0, std::chrono::steady_clock::now()});
        s->hb_ = std::thread([s, rank]() {  // liveness for peers that cannot check this rank's pid
            while (!s->stop_.load()) {
                s->ctl_->post[rank].beat.fetch_add(1, std::memory_order_relaxed);
                std::this_thread::sleep_for(std::chrono::milliseconds(100));
            }
        });
        s->ctl_->joined.fetch_add(1, std::memory_order_acq_rel);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t it = 0; s->ctl_->joined.load(std::memory_order_acquire) < (uint32_t)G; ++it) {
            // a rank that joined last and exited at once is not a failure of the meeting (the next
            // barrier sees it): re-check the count after a failed wait
            if (s->waited_too_long(t0, it, meet_s) && s->ctl_->joined.load(std::memory_order_acquire) < (uint32_t)G) {
                if (rank == 0) unlink(path.c_str());
                *err = "host transport: not every rank joined " + path + " in time";
                delete s;
                return nullptr;
            }
        }
        if (rank == 0) unlink(path.c_str());  // every rank holds its mapping: the name is no longer needed
        for (int r = 0; r < G; ++r)
            if (s->ctl_->post[r].stage_bytes != W) {
                *err = "host transport: ranks disagree on OGE_COMM_STAGE_MB";
                s->ctl_->broken.store(1);
                delete s;
                return nullptr;
            }
        return s;
    }

    // 0 when all G ranks arrived; -2 on a timeout (or after any rank timed out)
    int barrier() {
        if (ctl_->broken.load(std::memory_order_acquire)) return -2;
        const uint32_t g = ctl_->gen.load(std::memory_order_acquire);
        if (ctl_->count.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)G_) {
            ctl_->count.store(0, std::memory_order_relaxed);
            ctl_->gen.fetch_add(1, std::memory_order_release);
            return 0;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t it = 0; ctl_->gen.load(std::memory_order_acquire) == g; ++it) {
            if (ctl_->broken.load(std::memory_order_acquire)) return -2;
            if (waited_too_long(t0, it) && ctl_->gen.load(std::memory_order_acquire) == g) {
                ctl_->broken.store(1, std::memory_order_release);
                return -2;
            }
        }
        return 0;
    }

private:
    bool waited_too_long(std::chrono::steady_clock::time_point t0, uint64_t it, double limit_s = 0) {
        if (it < 4096) {
            sched_yield();
            return false;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if ((it & 1023) != 0) return false;
        if (peer_gone()) return true;
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > (limit_s > 0 ? limit_s : timeout_s());
    }
    bool peer_gone() {  // a rank that posted its pid and whose process has exited
        const auto now = std::chrono::steady_clock::now();
        for (int r = 0; r < G_; ++r) {
            if (r == rank_) continue;
            const ShmRankPost &p = ctl_->post[r];
            if (p.pid <= 0) continue;  // not joined yet
            if (my_ns_ && p.pidns == my_ns_) {
                if (kill((pid_t)p.pid, 0) != 0 && errno == ESRCH) return true;
                continue;
            }
            const uint64_t b = p.beat.load(std::memory_order_relaxed);  // another pid namespace: the heartbeat
            if (b != seen_[r].first) {
                seen_[r] = {b, now};
            } else if (std::chrono::duration<double>(now - seen_[r].second).count() > stale_beat_s()) {
                return true;
            }
        }
        return false;
    }

public:
    // test hook (tests/native/dist_selftest.cpp --foreign-pid): post a pid that does not exist here, under
    // another pid namespace, as a rank of a container sharing the segment would
    void pose_as_foreign() {
        ctl_->post[rank_].pidns = my_ns_ + 1;
        ctl_->post[rank_].pid = 0x7ffffff0;
    }

private:
    uint64_t my_ns_ = 0;
    std::vector<std::pair<uint64_t, std::chrono::steady_clock::time_point>> seen_;
    std::thread hb_;
    std::atomic<bool> stop_{false};
    int G_ = 0, rank_ = 0;
    uint64_t W_ = 0, S_ = 0;
    size_t hdr_ = 0, size_ = 0;
    uint8_t *base_ = nullptr;
    ShmCtl *ctl_ = nullptr;
    std::string err_;
};

// bytes of round k (of S each) out of a total of n
inline uint64_t shm_part(uint64_t n, uint64_t k, uint64_t S) {
    const uint64_t a = k * S;
    return n > a ? std::min(S, n - a) : 0;
}

template <class Ops>
struct ShmColl {
    ShmSeg &seg;
    Ops &ops;

    // wait for every copy queued so far, whatever happened before; rc keeps the first error
    void drain(int &rc) {
        const int s = ops.sync();
        if (!rc) rc = s;
    }

    // device buffers: rank r's bytes for rank p are send + soff[p], sbytes[p]; they land at recv + roff[r]
    // of rank p.  0 = ok, -1 = this rank's copies failed or the byte counts disagree, -2 = the protocol
    // broke (timeout).
    int alltoallv(const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
                  const uint64_t *roff) {
        const int G = seg.size(), r = seg.rank();
        const uint64_t S = seg.slot_bytes();
        ShmRankPost &me = seg.post(r);
        uint64_t mx = 0;
        for (int p = 0; p < G; ++p) {
            me.sb[p] = sbytes[p];
            if (p != r) mx = std::max(mx, sbytes[p]);
        }
        me.maxb = mx;
        if (seg.barrier()) return -2;
        int rc = 0;
        uint64_t M = 0;
        for (int p = 0; p < G; ++p) {
            if (seg.post(p).sb[r] != rbytes[p]) rc = -1;
            M = std::max(M, seg.post(p).maxb);
        }
        if (!rc && sbytes[r]) rc = ops.d2d((uint8_t *)recv + roff[r], (const uint8_t *)send + soff[r], sbytes[r]);
        for (uint64_t k = 0; k * S < M; ++k) {
            for (int p = 0; p < G && !rc; ++p) {
                const uint64_t n = p == r ? 0 : shm_part(sbytes[p], k, S);
                if (n) rc = ops.d2h(seg.slot(r, p), (const uint8_t *)send + soff[p] + k * S, n);
            }
            drain(rc);  // the slot is filled before the peers read it (always: no copy outlives its round)
            if (seg.barrier()) return -2;
            for (int p = 0; p < G && !rc; ++p) {
                const uint64_t n = p == r ? 0 : shm_part(rbytes[p], k, S);
                if (n) rc = ops.h2d((uint8_t *)recv + roff[p] + k * S, seg.slot(p, r), n);
            }
            drain(rc);  // read out before the sender refills the slot
            if (seg.barrier()) return -2;
        }
        drain(rc);
        if (seg.barrier()) return -2;  // every rank has read the posts before the next collective rewrites them
        return rc;
    }

    // host buffers, the same byte count on every rank: out[p * bytes ...] = rank p's in
    int allgather_host(const void *in, void *out, size_t bytes) {
        const int G = seg.size(), r = seg.rank();
        const uint64_t W = seg.stage_bytes();
        for (uint64_t k = 0; k * W < bytes; ++k) {
            const uint64_t n = shm_part(bytes, k, W);
            memcpy(seg.outbox(r), (const uint8_t *)in + k * W, n);
            if (seg.barrier()) return -2;
            for (int p = 0; p < G; ++p) memcpy((uint8_t *)out + (size_t)p * bytes + k * W, seg.outbox(p), n);
            if (seg.barrier()) return -2;
        }
        return 0;
    }

    // in: G * chunk device bytes per rank; out (chunk device bytes) = elementwise max over the ranks of
    // their chunk `rank`
    int reduce_scatter_max_u8(const uint8_t *in, uint8_t *out, size_t chunk) {
        const int G = seg.size(), r = seg.rank();
        const uint64_t S = seg.slot_bytes();
        std::vector<uint8_t> acc(std::min<uint64_t>(chunk, S));
        int rc = 0;
        for (uint64_t k = 0; k * S < chunk; ++k) {
            const uint64_t n = shm_part(chunk, k, S);
            for (int p = 0; p < G && !rc; ++p) rc = ops.d2h(seg.slot(r, p), in + (size_t)p * chunk + k * S, n);
            drain(rc);
            if (seg.barrier()) return -2;
            if (!rc) {
                memcpy(acc.data(), seg.slot(0, r), n);
                for (int p = 1; p < G; ++p) {
                    const uint8_t *s = seg.slot(p, r);
                    for (uint64_t i = 0; i < n; ++i) acc[i] = std::max(acc[i], s[i]);
                }
                rc = ops.h2d(out + k * S, acc.data(), n);
            }
            drain(rc);  // acc and the slots are reused next round
            if (seg.barrier()) return -2;
        }
        return rc;
    }
};

}  // namespace oge_dist
