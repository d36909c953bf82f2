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
    void *alloc(size_t bytes);
    void release(void *p);
    // the last count-only oge_bam_record_offsets_dev call: its converged chunk starts and offsets stay
    // in the "rec_walk" workspace, so the offsets call that follows (same stream and range) goes
    // straight to the fill walk, which is checked to join and count the same
    struct RecWalk {
        const void *stream = nullptr;
        uint64_t base = 0, end = 0, n = 0, C = 0;
        int32_t n_ref = 0;
    } recwalk;
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
// lane-per-block BGZF inflate (inflate_lane.hip); err/zpow as in oge_bgzf_inflate_dev
int oge_inflate_lanes(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d0, const uint64_t *d1,
                      const uint64_t *uoff, const uint32_t *crc, uint64_t nblk, uint8_t *out, uint32_t *err,
                      const uint32_t *zpow);

// ---- multi-GPU internals (dist.hip)
oge_ctx *oge_comm_ctx(oge_comm *comm);
// in place: v[0..count) = the sum over the communicator's ranks (collective, host values)
int oge_comm_sum_u64(oge_comm *comm, uint64_t *v, int count);
