// realign_dev.h -- the offset-scan batch resident on the device (realign_prep.hip builds it, realign.hip's
// k_planes / k_scan_bp read it in place) and the device consensus-generation entry point.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "realign.h"

struct oge_ctx;

struct RsDevBatch {
    const uint8_t *cons;        // consensus bytes back to back
    const uint64_t *cons_off;   // n_cons + 1
    uint32_t n_cons;
    const uint64_t *cwo;        // plane word offsets of the consensuses (n_cons + 1: one spare word each)
    uint64_t cons_words;
    const uint8_t *bases, *quals;  // altRead bases (characters) and raw qualities
    const uint64_t *read_off;   // n_reads + 1
    uint32_t n_reads;
    const uint64_t *rwo;        // n_reads + 1
    uint64_t read_words;
    const int4 *pairs;          // (consensus, read, orig, maxStart)
    uint64_t n_pairs;
};

// findBestOffset of every pair of a device batch -> best_index / best_score (host arrays, n_pairs each);
// *generic: the byte-wise kernel ran (lower-case bases or '*' in the batch)
int realign_scan_devbatch(oge_ctx *ctx, const RsDevBatch &b, int32_t *best_index, int32_t *best_score, bool *generic);
// phase B + the batch + the scan on the device (realign_prep.hip); d_recs = the staged record arena
int oge_realign_prep_run(oge_ctx *ctx, const uint8_t *d_recs, const oge::DevPrepBatch &B, oge::DevPrepOut &O);
