// synth.h -- deterministic synthetic paired-end BAM record generator.
//
// One definition compiled twice: by hipcc for the device generator (bench inputs are
// generated straight into HBM) and by the host compiler for small BAM files (oracle
// goldens, CPU tests).  Every record is a pure function of (params, slot), so the two
// agree byte for byte and the generator needs no sequential state.
//
// Read model (SURVEY.md §8d C1/C2 shapes): pairs of `read_len` reads on `n_ref` contigs,
// insert U[ins_min, ins_max], `dup_ppm` duplicate pairs that copy the placement of an
// earlier non-duplicate pair, `inter_ppm` inter-contig pairs, `munmap_ppm` pairs whose
// second mate is unmapped and placed at its mate, `clip_ppm` soft-clipped reads,
// `n_rg` read groups rg1..rgN (library libK), quals U[qual_min, qual_max], names
// "r%010llu" of the pair index, records shuffled by a Feistel permutation of the slots.
#pragma once
#include "bam_layout.h"

#define OGE_SYNTH_MAX_REF 64

typedef struct oge_synth_params {
    uint64_t seed;
    uint64_t n_pairs;        // records = 2 * n_pairs
    uint32_t n_ref;          // <= OGE_SYNTH_MAX_REF
    uint32_t read_len;       // <= 250
    uint32_t ins_min, ins_max;
    uint32_t dup_ppm, inter_ppm, munmap_ppm, clip_ppm;
    uint32_t n_rg;           // 1..9
    uint32_t qual_min, qual_max;
    uint32_t shuffle;        // 0 = pair order, 1 = shuffled slots
    uint64_t ref_len[OGE_SYNTH_MAX_REF];
    uint64_t ref_cum[OGE_SYNTH_MAX_REF + 1];  // filled by oge_synth_finalize
} oge_synth_params;

OGE_HD uint64_t oge_mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
OGE_HD uint64_t oge_rng(uint64_t seed, uint64_t a, uint64_t b) {
    return oge_mix64(seed ^ oge_mix64(a * 0xD1B54A32D192ED03ull + b));
}
OGE_HD uint32_t oge_ppm(uint64_t r) { return (uint32_t)((r >> 11) % 1000000ull); }

// ---- Feistel permutation of [0, n) (cycle walking over the next power of 4) ----
OGE_HD uint64_t oge_feistel_once(uint64_t x, uint32_t half_bits, uint64_t seed) {
    uint64_t mask = (half_bits >= 32) ? 0xFFFFFFFFull : ((1ull << half_bits) - 1);
    uint64_t l = x >> half_bits, r = x & mask;
    for (int round = 0; round < 4; ++round) {
        uint64_t f = oge_mix64(r ^ (seed + 0x632BE59BD9B4E019ull * (uint64_t)(round + 1))) & mask;
        uint64_t nl = r, nr = l ^ f;
        l = nl; r = nr;
    }
    return (l << half_bits) | r;
}
OGE_HD uint64_t oge_permute(uint64_t slot, uint64_t n, uint64_t seed) {
    uint32_t bits = 2;
    while ((1ull << bits) < n) bits += 2;
    uint32_t half = bits / 2;
    uint64_t x = slot;
    do { x = oge_feistel_once(x, half, seed); } while (x >= n);
    return x;
}

typedef struct oge_pair_place {
    int32_t ref[2], pos[2];
    uint8_t rev[2];
    uint8_t kind;      // 0 = FR pair, 1 = inter-contig, 2 = second mate unmapped
    uint8_t pad;
    int32_t ins;
    uint64_t src;      // pair whose placement (and read group) this pair copies
} oge_pair_place;

OGE_HD int oge_synth_is_dup(const oge_synth_params *P, uint64_t p) {
    return p > 0 && oge_ppm(oge_rng(P->seed, p, 2)) < P->dup_ppm;
}

OGE_HD void oge_synth_pick(const oge_synth_params *P, uint64_t r, int32_t *ref, int32_t *pos, uint32_t span) {
    uint64_t G = P->ref_cum[P->n_ref];
    uint64_t g = r % G;
    uint32_t lo = 0, hi = P->n_ref - 1;
    while (lo < hi) {                      // last contig with cum <= g
        uint32_t mid = (lo + hi + 1) >> 1;
        if (P->ref_cum[mid] <= g) lo = mid; else hi = mid - 1;
    }
    uint64_t len = P->ref_len[lo];
    uint64_t room = len > span ? len - span : 1;
    *ref = (int32_t)lo;
    *pos = (int32_t)((g - P->ref_cum[lo]) % room);
}

OGE_HD oge_pair_place oge_synth_base_place(const oge_synth_params *P, uint64_t q) {
    oge_pair_place pl;
    uint64_t r0 = oge_rng(P->seed, q, 1);
    uint32_t u = oge_ppm(r0);
    uint64_t r1 = oge_rng(P->seed, q, 20);
    uint64_t r2 = oge_rng(P->seed, q, 21);
    uint32_t L = P->read_len;
    int32_t ins = (int32_t)(P->ins_min + (r2 >> 20) % (P->ins_max - P->ins_min + 1));
    int32_t ref, pos;
    oge_synth_pick(P, r1, &ref, &pos, P->ins_max + 1);
    pl.ins = ins;
    pl.pad = 0;
    if (u < P->munmap_ppm) {
        pl.kind = 2;
        pl.ref[0] = pl.ref[1] = ref;
        pl.pos[0] = pl.pos[1] = pos;
        pl.rev[0] = (uint8_t)(r2 & 1);
        pl.rev[1] = 0;
    } else if (u < P->munmap_ppm + P->inter_ppm && P->n_ref > 1) {
        pl.kind = 1;
        pl.ref[0] = ref; pl.pos[0] = pos;
        uint64_t r3 = oge_rng(P->seed, q, 22);
        int32_t ref2, pos2;
        oge_synth_pick(P, r3, &ref2, &pos2, L + 1);
        if (ref2 == ref) ref2 = (ref + 1) % (int32_t)P->n_ref;
        if ((uint64_t)pos2 + L >= P->ref_len[ref2]) pos2 = 0;
        pl.ref[1] = ref2; pl.pos[1] = pos2;
        pl.rev[0] = (uint8_t)(r2 & 1);
        pl.rev[1] = (uint8_t)((r2 >> 1) & 1);
    } else {
        pl.kind = 0;
        int32_t left = pos, right = pos + ins - (int32_t)L;
        if (r2 & 1) {  // read 1 is the left (forward) end
            pl.ref[0] = ref; pl.pos[0] = left; pl.rev[0] = 0;
            pl.ref[1] = ref; pl.pos[1] = right; pl.rev[1] = 1;
        } else {
            pl.ref[0] = ref; pl.pos[0] = right; pl.rev[0] = 1;
            pl.ref[1] = ref; pl.pos[1] = left; pl.rev[1] = 0;
        }
    }
    return pl;
}

OGE_HD oge_pair_place oge_synth_place(const oge_synth_params *P, uint64_t p) {
    uint64_t src = p;
    if (oge_synth_is_dup(P, p)) {
        for (uint64_t k = 0; k < 8; ++k) {
            uint64_t q = oge_rng(P->seed, p, 3 + k) % p;
            if (!oge_synth_is_dup(P, q)) { src = q; break; }
        }
    }
    oge_pair_place pl = oge_synth_base_place(P, src);
    pl.src = src;
    return pl;
}

// Per-read soft clip: returns clip length (0 = none), *at_start = clip before the M block.
OGE_HD uint32_t oge_synth_clip(const oge_synth_params *P, uint64_t p, int m, int *at_start) {
    uint64_t r = oge_rng(P->seed, p, 16 + (uint64_t)m);
    *at_start = (int)((r >> 3) & 1);
    if (oge_ppm(r) >= P->clip_ppm) return 0;
    uint32_t c = 1 + (uint32_t)((r >> 40) % 20);
    if (c * 2 >= P->read_len) c = P->read_len / 4;
    return c;
}

OGE_HD int oge_synth_mapped(const oge_pair_place *pl, int m) { return !(pl->kind == 2 && m == 1); }

OGE_HD uint32_t oge_synth_ncigar(const oge_synth_params *P, const oge_pair_place *pl, uint64_t p, int m) {
    if (!oge_synth_mapped(pl, m)) return 0;
    int at_start;
    return oge_synth_clip(P, p, m, &at_start) ? 2u : 1u;
}

#define OGE_SYNTH_NAME_LEN 12u   /* "r%010llu" + NUL */
#define OGE_SYNTH_TAG_LEN 7u     /* "RG" 'Z' "rgK" NUL */

// Total bytes of record (p, m) including the 4-byte block_size prefix.
OGE_HD uint32_t oge_synth_rec_bytes(const oge_synth_params *P, const oge_pair_place *pl, uint64_t p, int m) {
    uint32_t L = P->read_len;
    return 4 + 32 + OGE_SYNTH_NAME_LEN + 4 * oge_synth_ncigar(P, pl, p, m) + (L + 1) / 2 + L + OGE_SYNTH_TAG_LEN;
}

OGE_HD uint64_t oge_synth_slot_record(const oge_synth_params *P, uint64_t slot) {
    uint64_t n = 2 * P->n_pairs;
    return P->shuffle ? oge_permute(slot, n, P->seed ^ 0x5EED5EED5EEDull) : slot;
}

OGE_HD uint32_t oge_synth_slot_bytes(const oge_synth_params *P, uint64_t slot) {
    uint64_t rec = oge_synth_slot_record(P, slot);
    uint64_t p = rec >> 1;
    int m = (int)(rec & 1);
    oge_pair_place pl = oge_synth_place(P, p);
    return oge_synth_rec_bytes(P, &pl, p, m);
}

// Write the record held by `slot` at `out` (oge_synth_slot_bytes(P, slot) bytes).
OGE_HD void oge_synth_write_slot(const oge_synth_params *P, uint64_t slot, uint8_t *out) {
    uint64_t rec = oge_synth_slot_record(P, slot);
    uint64_t p = rec >> 1;
    int m = (int)(rec & 1);
    int o = 1 - m;
    oge_pair_place pl = oge_synth_place(P, p);
    uint32_t L = P->read_len;
    int mapped = oge_synth_mapped(&pl, m);
    int mate_mapped = oge_synth_mapped(&pl, o);
    int at_start = 0;
    uint32_t clip = mapped ? oge_synth_clip(P, p, m, &at_start) : 0;
    uint32_t ncig = mapped ? (clip ? 2u : 1u) : 0u;
    uint32_t bytes = oge_synth_rec_bytes(P, &pl, p, m);

    uint32_t flag = OGE_F_PAIRED | (m ? OGE_F_READ2 : OGE_F_READ1);
    if (pl.kind == 0) flag |= OGE_F_PROPER;
    if (!mapped) flag |= OGE_F_UNMAP;
    if (!mate_mapped) flag |= OGE_F_MUNMAP;
    if (mapped && pl.rev[m]) flag |= OGE_F_REVERSE;
    if (mate_mapped && pl.rev[o]) flag |= OGE_F_MREVERSE;

    // A soft clip before the aligned block moves the alignment start right, so the unclipped
    // 5' end (what MarkDuplicates keys on) stays at the fragment end, as an aligner reports it.
    int32_t pos = pl.pos[m] + ((mapped && clip && at_start) ? (int32_t)clip : 0);
    int mate_at_start = 0;
    uint32_t mate_clip = mate_mapped ? oge_synth_clip(P, p, o, &mate_at_start) : 0;
    int32_t mpos = pl.pos[o] + ((mate_mapped && mate_clip && mate_at_start) ? (int32_t)mate_clip : 0);
    int32_t tlen = 0;
    if (pl.kind == 0) tlen = (pl.pos[m] <= pl.pos[o] && !pl.rev[m]) ? pl.ins : -pl.ins;
    uint32_t mlen = L - clip;
    int32_t end = mapped ? pos + (int32_t)mlen : pos;

    oge_wr_u32(out + OGE_OFF_BLOCK, bytes - 4);
    oge_wr_u32(out + OGE_OFF_REFID, (uint32_t)pl.ref[m]);
    oge_wr_u32(out + OGE_OFF_POS, (uint32_t)pos);
    out[OGE_OFF_LNAME] = (uint8_t)OGE_SYNTH_NAME_LEN;
    out[OGE_OFF_MAPQ] = mapped ? 60 : 0;
    oge_wr_u16(out + OGE_OFF_BIN, (uint16_t)oge_reg2bin(pos, end));
    oge_wr_u16(out + OGE_OFF_NCIGAR, (uint16_t)ncig);
    oge_wr_u16(out + OGE_OFF_FLAG, (uint16_t)flag);
    oge_wr_u32(out + OGE_OFF_LSEQ, L);
    oge_wr_u32(out + OGE_OFF_MREFID, (uint32_t)pl.ref[o]);
    oge_wr_u32(out + OGE_OFF_MPOS, (uint32_t)mpos);
    oge_wr_u32(out + OGE_OFF_TLEN, (uint32_t)tlen);

    uint8_t *q = out + OGE_OFF_NAME;
    q[0] = 'r';
    uint64_t v = p;
    for (int i = 10; i >= 1; --i) { q[i] = (uint8_t)('0' + v % 10); v /= 10; }
    q[11] = 0;
    q += OGE_SYNTH_NAME_LEN;

    if (ncig == 1) {
        oge_wr_u32(q, (L << 4) | OGE_CIG_M); q += 4;
    } else if (ncig == 2) {
        if (at_start) { oge_wr_u32(q, (clip << 4) | OGE_CIG_S); oge_wr_u32(q + 4, (mlen << 4) | OGE_CIG_M); }
        else          { oge_wr_u32(q, (mlen << 4) | OGE_CIG_M); oge_wr_u32(q + 4, (clip << 4) | OGE_CIG_S); }
        q += 8;
    }

    // sequence: 4-bit codes A=1 C=2 G=4 T=8, 32 bases per 64-bit draw
    uint64_t rs = 0;
    for (uint32_t i = 0; i < L; i += 2) {
        if ((i & 31) == 0) rs = oge_rng(P->seed, rec, 1000 + i / 32);
        uint32_t b0 = 1u << ((rs >> (2 * (i & 31))) & 3);
        uint32_t b1 = (i + 1 < L) ? (1u << ((rs >> (2 * ((i + 1) & 31))) & 3)) : 0u;
        q[i >> 1] = (uint8_t)((b0 << 4) | b1);
    }
    q += (L + 1) / 2;

    uint32_t qspan = P->qual_max - P->qual_min + 1;
    uint64_t rq = 0;
    for (uint32_t i = 0; i < L; ++i) {
        if ((i & 3) == 0) rq = oge_rng(P->seed, rec, 5000 + i / 4);
        uint32_t u16 = (uint32_t)((rq >> (16 * (i & 3))) & 0xFFFF);
        q[i] = (uint8_t)(P->qual_min + ((u16 * qspan) >> 16));
    }
    q += L;

    uint32_t rg = 1 + (uint32_t)(oge_rng(P->seed, pl.src, 5) % P->n_rg);
    q[0] = 'R'; q[1] = 'G'; q[2] = 'Z'; q[3] = 'r'; q[4] = 'g'; q[5] = (uint8_t)('0' + rg); q[6] = 0;
}
