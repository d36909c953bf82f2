// shard.hip -- routing kernel of the multi-GPU (contig-sharded) sort + dedup.
//
// The reference's only data-parallel split is SplitByChromosome (algorithms/split_by_chromosome.cpp:
// 30-58: chain = refID % K, re-merged by SortedMerge).  Here ranks own contiguous refID ranges
// (owner table monotone in refID, refID -1 on the last rank), so the ranks' sorted outputs
// concatenate into the global order with no merge.  A record whose mate lies on another rank's
// contigs is ALSO sent there as a read-only "ghost", so every MarkDuplicates pair group is complete on
// the rank that owns its read1 contig (read1 = the lower refID end, mark_duplicates.cpp:226-241);
// that rank's decision for the ghost is sent back to the ghost's owner (openge_amd/shard.py).
#include "oge_ctx.h"
#include "bam_layout.h"
#include "dev_util.h"

namespace {

constexpr int kT = 256;

// dest  = owner(refID)                                       (every record)
// ghost = owner(mate refID) when the record is a mate-join candidate whose mate is owned elsewhere
//         (paired, mate mapped, mate refID valid), else -1
// back  = dest when this rank holds the record as a ghost (dest != my_rank) and its mate is the
//         pair's read1 (mate refID < refID), i.e. this rank decides the record's 0x400 bit, else -1
__global__ __launch_bounds__(kT) void k_route(const uint8_t *__restrict__ recs, const uint64_t *__restrict__ off, uint64_t n,
                                               const int32_t *__restrict__ owner, int32_t n_ref, int32_t my_rank,
                                               int32_t *__restrict__ dest, int32_t *__restrict__ ghost,
                                               int32_t *__restrict__ back) {
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    const uint8_t *r = recs + off[i];
    const int32_t ref = (int32_t)oge_ldu32(r + OGE_OFF_REFID);
    const int32_t mref = (int32_t)oge_ldu32(r + OGE_OFF_MREFID);
    const uint32_t flag = oge_ldu16(r + OGE_OFF_FLAG);
    const int32_t d = owner[(ref >= 0 && ref < n_ref) ? ref : n_ref];
    if (dest) dest[i] = d;
    const bool cand = (flag & OGE_F_PAIRED) && !(flag & OGE_F_MUNMAP) && mref >= 0 && mref < n_ref && ref >= 0;
    if (ghost) ghost[i] = (cand && owner[mref] != d) ? owner[mref] : -1;
    if (back) back[i] = (d != my_rank && cand && mref < ref) ? d : -1;
}

}  // namespace

extern "C" int oge_shard_route_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                                   const int32_t *d_owner, int32_t n_ref, int32_t my_rank, int32_t *d_dest,
                                   int32_t *d_ghost, int32_t *d_back) {
    if (!ctx || (n && (!d_recs || !d_off || !d_owner)) || n_ref < 0) return oge_fail(ctx, OGE_ERR_ARG, "oge_shard_route_dev: bad argument");
    hipSetDevice(ctx->device);
    if (!n) return OGE_OK;
    hipLaunchKernelGGL(k_route, dim3(oge_ceil_div(n, kT)), dim3(kT), 0, ctx->stream, d_recs, d_off, n, d_owner, n_ref, my_rank,
                       d_dest, d_ghost, d_back);
    OGE_LAUNCH_CHECK(ctx);
    return OGE_OK;
}
