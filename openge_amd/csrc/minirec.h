// minirec.h -- minimal records for exact mate-join key compares away from the record arena (the
// multi-GPU owner's join, dist.hip; the out-of-core global join, chunked.hip).  Included by one TU
// each; the kernels live in an anonymous namespace.
#pragma once
#include "bam_layout.h"
#include "dev_util.h"
#include "rec_parse.h"
#include "records.h"

namespace {

// Minimal record for an exact pair-key compare on another rank: the 36-byte core with l_read_name,
// n_cigar = 0, l_seq = 0, the name, and the record's RG tag (type and value bytes) when it has one --
// what pair_key_of / same_pair_key (markdup.hip) read.
__device__ __forceinline__ uint32_t minirec_size(const uint8_t *r, const uint8_t **rg, uint32_t *rgl) {
    const uint32_t bs = oge_ldu32(r);
    const uint32_t lname = r[OGE_OFF_LNAME], nc = oge_ldu16(r + OGE_OFF_NCIGAR), lseq = oge_ldu32(r + OGE_OFF_LSEQ);
    const uint8_t *tags = r + OGE_OFF_NAME + lname + 4 * nc + (lseq + 1) / 2 + lseq;
    if (!find_rg(tags, r + 4 + bs, rg, rgl)) *rgl = 0xffffffffu;
    return OGE_OFF_NAME + lname + (*rgl != 0xffffffffu ? 3 + *rgl + 1 : 0);
}

// cand_only: 0 bytes for summaries that are not mate-join candidates (their src is never followed)
__global__ __launch_bounds__(256) void k_minirec_sizes(const uint8_t *__restrict__ recs, const RecMeta *__restrict__ cm, uint64_t n,
                                                       bool cand_only, uint64_t *__restrict__ sz) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) {
        const uint8_t *rg;
        uint32_t rgl;
        sz[k] = (cand_only && !(cm[k].m & OGE_M_CAND)) ? 0 : minirec_size(recs + cm[k].src, &rg, &rgl);
    } else if (k == n) {
        sz[k] = 0;
    }
}

// writes the minimal records and points each summary's src at its record, relative to the byte chunk
// of its destination (chunk0[d]: first byte of destination d's chunk; dend[d]: its first entry after)
__global__ __launch_bounds__(256) void k_minirec_write(const uint8_t *__restrict__ recs, RecMeta *__restrict__ cm, uint64_t n,
                                                      const uint64_t *__restrict__ moff, const uint64_t *__restrict__ dend,
                                                      uint32_t G, uint8_t *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    if (moff[k + 1] == moff[k]) return;  // no record (cand_only sizing)
    const uint8_t *r = recs + cm[k].src;
    const uint8_t *rg;
    uint32_t rgl;
    const uint32_t sz = minirec_size(r, &rg, &rgl);
    uint8_t *o = out + moff[k];
    const uint32_t lname = r[OGE_OFF_LNAME];
    for (uint32_t b = 0; b < 4; ++b) o[b] = (uint8_t)((sz - 4) >> (8 * b));
    for (uint32_t b = 4; b < OGE_OFF_NAME; ++b) o[b] = 0;
    o[OGE_OFF_LNAME] = (uint8_t)lname;
    for (uint32_t b = 0; b < lname; ++b) o[OGE_OFF_NAME + b] = r[OGE_OFF_NAME + b];
    if (rgl != 0xffffffffu) {
        uint8_t *t = o + OGE_OFF_NAME + lname;
        for (uint32_t b = 0; b < 3; ++b) t[b] = rg[(int)b - 3];
        for (uint32_t b = 0; b < rgl; ++b) t[3 + b] = rg[b];
        t[3 + rgl] = 0;
    }
    uint32_t d = 0;
    while (d + 1 < G && k >= dend[d]) ++d;
    cm[k].src = moff[k] - (d ? moff[dend[d - 1]] : 0);
}

}  // namespace
