// oge_ctx.h -- internal device context: stream, grow-only workspace, HIP-event stage timing.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <deque>
#include <map>
#include <string>
#include <vector>

#include "../../include/openge_hip.h"
#include "capi_common.h"

struct OgeStageTimer {
    hipEvent_t start, stop;
};

struct oge_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    struct Buf { void *p = nullptr; size_t cap = 0; };
    std::map<std::string, Buf> bufs;
    // stage -> list of (start, stop) event pairs recorded during the last pipeline call
    std::map<std::string, std::vector<OgeStageTimer>> stage_events;
    std::deque<OgeStageTimer> event_pool;  // deque: begin_stage's pointers stay valid while stages nest
    size_t event_pool_used = 0;
    bool timing = true;
    int timing_hold = 0;  // > 0: a composite entry point (the pipeline) keeps its sub-calls' stage events
    bool pool = false;  // allocate from the device's stream-ordered pool and keep freed memory in it
    hipStream_t side[4] = {nullptr, nullptr, nullptr, nullptr};  // extra streams a stage pipelines over
    hipStream_t side_stream(int i);
    int ncu = 0;  // compute units of `device` (persistent grids), looked up once per context
    int cu_count() {
        if (!ncu) {
            int c = 0;
            (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device);
            ncu = c > 0 ? c : 256;
        }
        return ncu;
    }
    void *alloc(size_t bytes);
    void release(void *p);
    // the last count-only record walk: its converged chunk starts and offsets stay in the "rec_walk"
    // workspace, so the offsets call that follows (same stream and range) goes straight to the fill: from
    // the count walk's record slots (rel, a trusted internal caller's `keep`), else a second walk that is
    // checked to join and count the same
    struct RecWalk {
        const void *stream = nullptr;
        uint64_t base = 0, limit = 0, end = 0, n = 0, C = 0, x = 0;
        int32_t n_ref = 0;
        const uint16_t *rel = nullptr;
        uint32_t sc = 0;
    } recwalk;
    // the inflate's phase-1 bitmap buffer and how many of its bytes are known clear (inflate_lane.hip)
    const void *infl_clean_ptr = nullptr;
    uint64_t infl_clean_bytes = 0, infl_clean_next = 0;
    std::map<std::string, uint64_t> counters;  // per call: work counts a stage reports (oge_ctx_counter)
    bool last_scan_generic = false;  // realign scan fell back to the byte-wise kernel
    double scan_t[3] = {0, 0, 0};    // realign scan host timings: validate, upload, device + download

    // Grow-only named scratch buffer; contents are undefined between calls.
    void *ws(const char *name, size_t bytes);
    // Loaned scratch: while a loan is active (lend), scratch() bump-allocates from the caller's buffer
    // (the fused pipeline lends its output arena, which is only written by the final gather), else it
    // is ws().  Only for buffers that are dead before the lender writes its buffer.
    uint8_t *loan_base = nullptr;
    size_t loan_cap = 0, loan_used = 0;
    void *scratch(const char *name, size_t bytes);
    void lend(void *p, size_t bytes) { loan_base = (uint8_t *)p; loan_cap = p ? bytes : 0; loan_used = 0; }
    void end_loan() { loan_base = nullptr; loan_cap = loan_used = 0; }
    OgeStageTimer *begin_stage(const char *name);
    void end_stage(OgeStageTimer *t);
    void reset_timing();
};

#define OGE_HIP_TRY(ctx, expr)                                                                     \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            std::string _m = std::string(#expr) + ": " + hipGetErrorString(_e);                   \
            return oge_fail((ctx), OGE_ERR_HIP, _m.c_str());                                       \
        }                                                                                          \
    } while (0)

// Launch-error check after a kernel launch (names the launch site).
#define OGE_STR2(x) #x
#define OGE_STR(x) OGE_STR2(x)
#define OGE_LAUNCH_CHECK(ctx)                                                                      \
    do {                                                                                           \
        hipError_t _e = hipGetLastError();                                                         \
        if (_e != hipSuccess)                                                                      \
            return oge_fail((ctx), OGE_ERR_HIP,                                                    \
                            (std::string("kernel launch at " __FILE__ ":" OGE_STR(__LINE__) ": ") + \
                             hipGetErrorString(_e)).c_str());                                      \
    } while (0)

static inline uint32_t oge_ceil_div(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// ---- device primitives (prims.hip) ----
// In-place-or-not exclusive scans. `out` may alias `in`.
int oge_exclusive_scan_u32(oge_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n);
int oge_exclusive_scan_u64(oge_ctx *ctx, const uint64_t *in, uint64_t *out, uint64_t n);
// out[0..n] = the exclusive scan of the record sizes in sorted keys' payload bits (key >> 50), out[n] = their
// total, in one reduce-then-scan (keys and out 16-byte aligned; returns 1 without work otherwise)
int oge_offsets_from_keys(oge_ctx *ctx, const uint64_t *keys, uint64_t n, uint64_t *out);
// Stable LSD radix sort of (key, value) pairs on key bits selected by `bit_mask` (only bits set
// in the mask are sorted; set bits are grouped into digit passes of <= 8 contiguous bits).
// Buffers: keys/vals hold the input; ktmp/vtmp scratch of the same size.  On return *kout/*vout
// point at whichever pair of buffers holds the result.  vals == NULL sorts keys only.
int oge_radix_sort_pairs(oge_ctx *ctx, uint64_t *keys, uint32_t *vals, uint64_t *ktmp, uint32_t *vtmp,
                         uint64_t n, uint64_t bit_mask, uint64_t **kout, uint32_t **vout);
// OR / AND reduction of a u64 array (for choosing the varying key bits).
int oge_reduce_or_and_u64(oge_ctx *ctx, const uint64_t *in, uint64_t n, uint64_t mask, uint64_t *or_out, uint64_t *and_out);

// ---- BGZF framing index on the device (inflate.hip) ----
struct OgeBgzfIndex {
    uint64_t *d0 = nullptr, *d1 = nullptr, *uoff = nullptr;  // nblk, nblk, nblk + 1 entries (device)
    uint32_t *crc = nullptr;
    uint64_t nblk = 0, total = 0;
};
// 0 = ok, 1 = candidates are not an exact block chain (use the host walk), < 0 = error
int oge_bgzf_index_ws(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, OgeBgzfIndex *ix);
// The blocks that start in [s, own) of d_z (zbytes >= own bytes readable: the last block may end past
// own): s = kIndexFirst takes the range's first candidate (*s_used), else s must be a candidate; the
// chain must be exact from s to its last block, whose end (>= own) goes to *xend.  0 = ok, 1 = not an
// exact chain, 2 = no candidate in the range (or s >= own: no block), < 0 = error.
constexpr uint64_t kIndexFirst = ~0ull;
int oge_bgzf_index_range_ws(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t s, uint64_t own, OgeBgzfIndex *ix,
                            uint64_t *s_used, uint64_t *xend);
// The record walk of oge_bam_record_offsets_dev generalised to a window: records that start in
// [start, limit) of d (bytes readable up to bufend, so the last record may end past limit); at_end says
// bufend is the end of the stream (a guess chain may stop there).  *exit = the end of the last record
// (= the first record start at or past limit); d_off (cap >= n + 1) gets the offsets and d_off[n] = *exit.
// keep (a count call of an internal caller that fills next, on the same unchanged stream): the walk also
// stores each chunk's record positions (in rel_buf when it holds rel_cap >= the slots' bytes, else
// workspace "rec_rel"), and the fill call expands them instead of walking the stream again.
int oge_record_walk(oge_ctx *ctx, const uint8_t *d, uint64_t start, uint64_t limit, uint64_t bufend, bool at_end, int32_t n_ref,
                    uint64_t *d_off, uint64_t cap, uint64_t *n_out, uint64_t *exit, bool keep = false, void *rel_buf = nullptr,
                    uint64_t rel_cap = 0);
// The first plausible record start in [0, lim) of d (bufend readable) as k_rec_guess judges it, or ~0.
int oge_record_guess(oge_ctx *ctx, const uint8_t *d, uint64_t lim, uint64_t bufend, bool at_end, int32_t n_ref, uint64_t *out);
// the framing walk of a host buffer with T threads (inflate.hip); false: use oge_bgzf_index
bool oge_bgzf_index_host_mt(const uint8_t *z, uint64_t zbytes, int T, std::vector<uint64_t> &d0, std::vector<uint64_t> &d1,
                            std::vector<uint64_t> &uoff, std::vector<uint32_t> &crc);
// lane-per-block BGZF inflate (inflate_lane.hip); err/zpow as in oge_bgzf_inflate_dev
int oge_inflate_lanes(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                      const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                      const uint32_t *zpow);

// ---- multi-GPU internals (dist.hip)
oge_ctx *oge_comm_ctx(oge_comm *comm);
// in place: v[0..count) = the sum over the communicator's ranks (collective, host values)
int oge_comm_sum_u64(oge_comm *comm, uint64_t *v, int count);
// host allgather (every rank `bytes` bytes, out = G * bytes in rank order) and the device all-to-all-v,
// recorded under `tag` in the communicator's exchange statistics
int oge_comm_allgather(oge_comm *comm, const char *tag, const void *in, void *out, size_t bytes);
int oge_comm_alltoallv_dev(oge_comm *comm, const char *tag, const void *send, const uint64_t *sbytes, const uint64_t *soff, void *recv,
                           const uint64_t *rbytes, const uint64_t *roff);
void oge_comm_reset_stats(oge_comm *comm);
// shard.hip: this rank's records of one BGZF BAM file decoded by byte range (see oge_bgzf_decode_shard);
// *X / *xoff are workspace ("pipe_x", "pipe_xoff"), *header the raw BAM header bytes.  Collective.
int oge_decode_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own, uint8_t **X, uint64_t **xoff, uint64_t *n,
                     std::vector<uint8_t> *header);
