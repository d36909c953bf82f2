// dist_local.h -- the in-process ("local") transport of the multi-GPU path: G ranks are G threads
// of one process that meet at a Hub, post their buffers and copy from each other.  The schedule is
// plain C++; Ops supplies the memory operations (HIP copies between HBM buffers in the library,
// memcpy in the CPU test harness), so the same code carries records between contexts sharing one
// GPU, between GPUs of one process, and between host buffers in tests/native/dist_selftest.cpp.
//
// Every rank calls the collectives in the same order; each collective passes two barriers whatever
// happens inside it, so one rank's failure is reported by that rank without hanging the others.
// A rank drains its own stream before posting a buffer (ops.sync), so peers read finished data --
// the ordering RCCL gets from running on the producer's stream.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

namespace oge_dist {

class Hub {
public:
    explicit Hub(int G) : G_(G), slots_(G) {}
    int size() const { return G_; }
    struct Slot {
        const void *p = nullptr;
        const uint64_t *bytes = nullptr, *off = nullptr;
    };
    void post(int rank, const Slot &s) { slots_[rank] = s; }
    const Slot &slot(int r) const { return slots_[r]; }
    void barrier() {
        std::unique_lock<std::mutex> l(m_);
        const uint64_t gen = gen_;
        if (++arrived_ == G_) {
            arrived_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(l, [&] { return gen_ != gen; });
        }
    }

private:
    int G_;
    std::vector<Slot> slots_;
    std::mutex m_;
    std::condition_variable cv_;
    int arrived_ = 0;
    uint64_t gen_ = 0;
};

// Ops: int copy(void *dst, const void *src, size_t n); int sync(); int max_into(uint8_t *acc,
// const uint8_t *src, size_t n) (acc[i] = max(acc[i], src[i])); 0 = ok.
template <class Ops>
struct LocalColl {
    Hub &hub;
    int rank;
    Ops &ops;

    // rank r's bytes for rank p: send + soff[p], sbytes[p]; they land at recv + roff[r] of rank p
    int alltoallv(const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv, const uint64_t *rbytes,
                  const uint64_t *roff) {
        const int rc0 = ops.sync();  // this rank's producers of `send` have finished before peers read it
        hub.post(rank, {send, sbytes, soff});
        hub.barrier();
        int rc = rc0;
        for (int p = 0; p < hub.size() && !rc; ++p) {
            const Hub::Slot &s = hub.slot(p);
            const uint64_t nb = s.bytes[rank];
            if (nb != rbytes[p]) rc = -1;
            else if (nb) rc = ops.copy((uint8_t *)recv + roff[p], (const uint8_t *)s.p + s.off[rank], nb);
        }
        if (!rc) rc = ops.sync();
        hub.barrier();  // a sender's buffer stays valid until every receiver has copied out of it
        return rc;
    }
    // host buffers: out[p * bytes ...] = rank p's in
    int allgather_host(const void *in, void *out, size_t bytes) {
        hub.post(rank, {in, nullptr, nullptr});
        hub.barrier();
        for (int p = 0; p < hub.size(); ++p) memcpy((uint8_t *)out + (size_t)p * bytes, hub.slot(p).p, bytes);
        hub.barrier();
        return 0;
    }
    // in: G * chunk bytes per rank; out (chunk bytes) = elementwise max over ranks of their chunk `rank`
    int reduce_scatter_max_u8(const uint8_t *in, uint8_t *out, size_t chunk) {
        const int rc0 = ops.sync();
        hub.post(rank, {in, nullptr, nullptr});
        hub.barrier();
        int rc = rc0 ? rc0 : chunk ? ops.copy(out, (const uint8_t *)hub.slot(0).p + (size_t)rank * chunk, chunk) : 0;
        for (int p = 1; p < hub.size() && !rc && chunk; ++p)
            rc = ops.max_into(out, (const uint8_t *)hub.slot(p).p + (size_t)rank * chunk, chunk);
        if (!rc) rc = ops.sync();
        hub.barrier();
        return rc;
    }
};

}  // namespace oge_dist
