// records.h -- per-record metadata shared by records.hip (producer) and markdup.hip (consumer).
#pragma once
#include <stdint.h>

// RecMeta.m (u64):
//   [0,16)  score (int16, getScore)        [16,32) library id
//   bit 32 fragment ReadEnds exists (mapped, refID != -1, primary)   bit 33 reverse strand
//   bit 34 pair candidate (paired && mate mapped)                    bit 35 primary (0x100 clear)
//   bit 36 isPaired() (read2Sequence = mate refID != -1)             bit 37 whole name in `name`
//   [40,48) original FLAG >> 8
//   [48,64) bin the writer must store (recomputed, util/bam_serializer.h:112-116)
constexpr uint64_t OGE_M_FRAG = 1ull << 32, OGE_M_REV = 1ull << 33, OGE_M_CAND = 1ull << 34,
                   OGE_M_PRIMARY = 1ull << 35, OGE_M_PAIRED = 1ull << 36, OGE_M_NAMEFIT = 1ull << 37;
constexpr uint32_t OGE_NAME_SLOT = 32;

// 64-byte record summary (array-of-structs: one 64-byte access moves a record's metadata).  The
// read name rides along (NUL-terminated, zero-padded) so mates can be confirmed without touching
// the record arena; names longer than the slot fall back to the record bytes.
struct alignas(16) RecMeta {
    uint64_t m;
    uint64_t src;    // byte offset of the record in the input arena
    int32_t seq;     // read1Sequence (refID)
    int32_t coord;   // unclipped 5' coordinate (0-based)
    int16_t rgi;     // read group of the record: index in the header table, -2 = no/empty RG tag,
                     // -1 = RG value not in the table (pair keys then compare the RG bytes)
    uint16_t hash_hi;
    uint32_t hash;   // hash_hi:hash = 48-bit hash of RG ":" name (pair key), candidates only
    uint8_t name[OGE_NAME_SLOT];
};
constexpr int32_t OGE_RGI_NONE = -2, OGE_RGI_UNLISTED = -1;
constexpr int32_t OGE_MAX_RG = 32767;  // read groups addressable by RecMeta.rgi
__host__ __device__ inline uint64_t oge_meta_hash48(const RecMeta &M) { return ((uint64_t)M.hash_hi << 32) | M.hash; }

// Read-group table on the device: ids back to back, off[g]..off[g+1]-1 is "ID\0" of group g; idw[g]
// the same id zero-padded to 16 bytes when it has at most 15 (a word compare in the input pass).
struct OgeRgTable {
    const uint8_t *ids;
    const uint4 *idw;
    const uint32_t *off;
    const int16_t *lib;
    int32_t n_rg;
    int16_t unknown_lib;
    int32_t split_k;  // > 1: split-by-chromosome emulation, the pair key carries the chain refID % K
};

// Sort-key packing of the KEYS output (see sort.hip for the layout).
constexpr uint64_t OGE_SORT_KEY_MASK = (1ull << 50) - 1;

struct OgePassArgs {
    const uint8_t *recs;     // input arena
    const uint64_t *off;     // n record offsets into recs
    uint64_t n;
    // input pass outputs (either may be NULL)
    RecMeta *meta;           // summary of input record i
    OgeRgTable rg;
    uint64_t *keys;          // coordinate sort key of input record i (+ byte size payload)
    uint32_t *vals;          // = ibase + i
    uint64_t ibase;          // index of the pass's first record in a larger array (a pass over a sub-range)
    int32_t n_ref;
    unsigned int *bad;       // bit 0: refID/pos out of range, bit 1: block_size out of [32, 10000]
    // KEYS: when set, keyred[0] |= every key's sort bits, keyred[1] |= their complement (the sort's varying
    // bits without a reduction pass of its own) and bad[1] = 1 says they were written
    unsigned long long *keyred;
    // gather pass: output record k = input record perm[k] (or meta[k].src when smeta is given)
    const uint32_t *perm;
    const RecMeta *smeta;    // summaries in OUTPUT order (bin, flags, src offset), optional
    const uint8_t *dup;      // output order: 1 sets 0x400, 0 clears it (primary records only)
    const uint64_t *desc;    // output order, replaces smeta + dup when given: src (40 bits) | bin << 40 |
                             // final FLAG high byte << 56 (written by k_apply); with ndup: k_cand_frag's desc0
                             // (primary bit 39, FLAG byte before the dup bit), finished here with dup[]
    unsigned int *ndup;      // with desc0 + dup: primaries flagged, counted into 64 counters 32 words apart
    uint8_t *out;
    const uint64_t *out_off; // n+1 output offsets
    // input pass of the in-place dedup (oge_markdup_run, META + KEYS): each record's mate-join / fragment key
    // words from the summary just built (md_keys.h cand_frag_one) and the fragments' deviation maxima into
    // cf_dev's slots; cf_f == NULL: not written
    uint32_t *cf_f;
    uint64_t *cf_fk, *cf_cval;
    uint32_t *cf_fv;
    unsigned long long *cf_dev;
    uint32_t cf_sb, cf_lb, cf_ib, cf_hb;
    int32_t cf_split;
};

struct oge_ctx;
// oge_sort_keys_dev_hook: called after the tie sort with the final permutation (perm[k] = input index of
// output record k) and the sorted keys; it gathers the summaries itself (and whatever it derives from them)
struct OgeSortGatherHook {
    int (*fn)(void *user, oge_ctx *ctx, const uint32_t *perm, const uint64_t *skeys);
    void *user;
};
int oge_input_pass(oge_ctx *ctx, const OgePassArgs &a);
int oge_gather_pass(oge_ctx *ctx, const OgePassArgs &a);
// Output offsets (from the sorted keys' size payload, or from the records) + the record gather.
int oge_gather_with_sizes(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, const uint32_t *d_perm,
                          const uint64_t *sorted_keys, uint64_t n, uint8_t *d_out, uint64_t *d_out_off,
                          const RecMeta *smeta, const uint8_t *d_dup, const uint64_t *desc = nullptr,
                          unsigned int *ndup = nullptr);
