// markdup_stages.h -- the stages of the device MarkDuplicates (markdup.hip), callable one by one so
// the multi-GPU path (dist.hip) can run them on ReadEnds exchanged between ranks:
//
//   cand_frag   per-record pass over the sorted summaries: mate-join candidate keys, fragment group
//               keys (fk/fv), gather descriptors (mark_duplicates.cpp:147-164,185-205)
//   join_build  ReadEndsMap pairing of consecutive occurrences of each RG:name key and the pair
//               ReadEnds (read1/read2 choice, orientation, int16 score sum; :210-245)
//   pair_groups markDuplicatePairs over equal (lib, r1Seq, r1Coord, orient, r2Seq, r2Coord) (:488-507)
//   frag_groups markDuplicateFragments over equal (lib, r1Seq, r1Coord, orient) (:515-540)
//   apply_desc  0x400 set / cleared on primaries, counted (:443-465)
//
// dup[] is indexed by whatever the stage's index arrays hold: the record index on one GPU, a padded
// global index (home rank * stride + sorted position) on several.
#pragma once
#include "oge_ctx.h"
#include "records.h"

struct OgeMdFrags {
    uint32_t *cpos = nullptr;   // n + 1: exclusive scan of the candidate flags
    uint64_t *fk = nullptr;     // n fragment group keys (bit 46: not a fragment; bit 63: paired)
    uint32_t *fv = nullptr;     // n record indices
    uint64_t *cval = nullptr;   // n candidate keys (hash bits << ib | index)
    uint64_t *desc0 = nullptr;  // n gather descriptors (optional)
    uint32_t nc = 0;            // candidates (when cpos_scanned)
    bool cpos_scanned = true;   // false: cpos holds the 0/1 flags (the windowed mate join needs no scan;
                                // oge_md_join_build scans them if it falls back to the sort path)
    bool desc_ovf = false;      // a record offset does not fit the descriptor
    const uint64_t *skeys = nullptr;  // sorted coordinate keys (windowed fragment groups), optional
    unsigned long long *dev = nullptr;  // per-block maxima of the fragment (then pair) coordinates' deviation from the anchors
    bool fused = false;         // written by oge_md_cand_frag_gather (the scan / read-back not done yet)
    bool defer_apply = false;   // (oge_markdup_finish_pre's pre, set by the caller) descriptors wanted: leave
                                // the apply to the record gather (desc0 + dup, MODE 3); *n_dup_out is then
                                // the gather's to count
};

struct OgeMdPairs {  // pair ReadEnds, np entries (see k_pair_build for the packing of hi / lo)
    uint64_t *hi = nullptr, *lo = nullptr, *hk = nullptr;
    uint2 *idx = nullptr;  // (read1 index, read2 index)
    uint32_t *val = nullptr;
    int64_t *pax = nullptr;  // anchor of each pair's first record (windowed pair groups), optional
    unsigned long long *dev = nullptr;
    uint32_t np = 0;
};

// skeys (optional): the records' coordinate sort keys when meta is in that sorted order; enables the
// windowed group stages (oge_md_*_groups_win)
int oge_md_cand_frag(oge_ctx *ctx, const oge_markdup_opts *opts, const RecMeta *meta, uint64_t n, bool want_desc,
                     OgeMdFrags *f, const uint64_t *skeys = nullptr);
// The same products written by the summary gather itself (out[i] = in[perm[i]], perm the final sorted order);
// oge_markdup_finish_pre(..., f) then runs the rest.  Launch only: f is finished by oge_markdup_finish_pre.
// desc0_buf (optional): where the descriptors go (default: context scratch, which a caller lending its output
// buffer as scratch must not read once the output is written -- the deferred apply reads them in the gather)
int oge_md_cand_frag_gather(oge_ctx *ctx, const oge_markdup_opts *opts, const RecMeta *in, const uint32_t *perm, uint64_t n,
                            RecMeta *out, bool want_desc, const uint64_t *skeys, OgeMdFrags *f, uint64_t *desc0_buf = nullptr);
int oge_markdup_finish_pre(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n, const oge_markdup_opts *opts,
                           const RecMeta *meta, uint8_t *d_dup, int apply, uint64_t *n_dup_out, uint64_t *d_desc, bool *desc_ok,
                           const uint64_t *skeys, const OgeMdFrags *pre);
// recs: the bytes RecMeta.src points into (only read for names that do not fit the summary)
int oge_md_join_build(oge_ctx *ctx, const oge_markdup_opts *opts, const uint8_t *recs, const RecMeta *meta, uint64_t n,
                      const OgeMdFrags &f, OgeMdPairs *p);
int oge_md_pair_groups(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdPairs &p, uint8_t *dup);
int oge_md_frag_groups(oge_ctx *ctx, uint64_t *fk, uint32_t *fv, uint64_t n, uint8_t *dup);
// The same two stages without a global sort, for items in sorted order (see k_frag_win / k_pair_win);
// *done = false (nothing written) when a window overflows or the anchors are missing: run the sort
// based stage instead.
int oge_md_frag_groups_win(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdFrags &f, uint64_t n, uint8_t *dup,
                           bool *done);
int oge_md_pair_groups_win(oge_ctx *ctx, const oge_markdup_opts *opts, const OgeMdPairs &p, uint8_t *dup, bool *done);
int oge_md_apply_inplace(oge_ctx *ctx, uint8_t *recs, const uint64_t *off, uint64_t n, const RecMeta *meta, uint8_t *dup,
                         uint64_t *n_dup_out);
int oge_md_apply_desc(oge_ctx *ctx, const uint64_t *desc0, uint64_t n, uint8_t *dup, uint64_t *desc, uint64_t *n_dup_out);
// hk (the chunk-key hash k_pair_build writes) and val = 0..np-1 for pairs received from other ranks
int oge_md_pairs_rehash(oge_ctx *ctx, OgeMdPairs *p);
