/* oge_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of OpenGE's coordinate sort order and MarkDuplicates, used as the parity
 * checker for the HIP path (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg).
 * It is never linked into or called by the product library.  Pinned against the reference
 * itself: oracle/_ref/ref_driver (the reference's own modules compiled from /root/reference by
 * oracle/Makefile.ref) produced the goldens in tests/golden/, and tests/test_oracle.py checks
 * this file against them.
 *
 * Records are BAM records as stored in a decompressed stream (block_size + core + data),
 * addressed by byte offsets.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OFF_REFID 4
#define OFF_POS 8
#define OFF_LNAME 12
#define OFF_NCIGAR 16
#define OFF_FLAG 18
#define OFF_LSEQ 20
#define OFF_MREFID 24
#define OFF_NAME 36

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static int32_t rdi32(const uint8_t *p) { return (int32_t)rd32(p); }
static uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

typedef struct {
    const uint8_t *recs;
    const uint64_t *offs;
} rec_set;

static const uint8_t *REC(const rec_set *s, uint64_t i) { return s->recs + s->offs[i]; }

/* ---------------------------------------------------------------------------------------
 * Sort::ByPosition (util/bamtools/Sort.h:116-133), with the heap-address tie-break (:132)
 * replaced by input order (the reference's address order is not reproducible).
 * refID == -1 compares "not less" both ways (:119-120), so the unmapped tail is a tie block;
 * a stable sort keeps it in input order.
 * ------------------------------------------------------------------------------------- */
static int bypos_less(const rec_set *s, uint32_t a, uint32_t b) {
    const uint8_t *l = REC(s, a), *r = REC(s, b);
    int32_t lr = rdi32(l + OFF_REFID), rr = rdi32(r + OFF_REFID);
    if (lr == -1) return 0;
    if (rr == -1) return 1;
    if (lr != rr) return lr < rr;
    int32_t lp = rdi32(l + OFF_POS), rp = rdi32(r + OFF_POS);
    if (lp != rp) return lp < rp;
    int lrev = (rd16(l + OFF_FLAG) & 0x10) != 0, rrev = (rd16(r + OFF_FLAG) & 0x10) != 0;
    if (lrev != rrev) return lrev ? 0 : 1;
    /* std::string operator< on the names (getName drops the NUL, BamAlignment.h:226) */
    uint32_t ln = l[OFF_LNAME] ? l[OFF_LNAME] - 1u : 0u, rn = r[OFF_LNAME] ? r[OFF_LNAME] - 1u : 0u;
    uint32_t m = ln < rn ? ln : rn;
    int c = memcmp(l + OFF_NAME, r + OFF_NAME, m);
    if (c != 0) return c < 0;
    if (ln != rn) return ln < rn;
    uint16_t lf = rd16(l + OFF_FLAG), rf = rd16(r + OFF_FLAG);
    if (lf != rf) return lf < rf;
    return 0; /* equal: stable order */
}

static void merge_sort_idx(const rec_set *s, uint32_t *a, uint32_t *tmp, uint64_t n) {
    if (n < 2) return;
    uint64_t h = n / 2;
    merge_sort_idx(s, a, tmp, h);
    merge_sort_idx(s, a + h, tmp, n - h);
    uint64_t i = 0, j = h, k = 0;
    while (i < h && j < n) {
        if (bypos_less(s, a[j], a[i])) tmp[k++] = a[j++];
        else tmp[k++] = a[i++];
    }
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(uint32_t));
}

/* perm[k] = input index at sorted position k */
int oracle_sort_perm(const uint8_t *recs, const uint64_t *offs, uint64_t n, uint32_t *perm) {
    rec_set s = {recs, offs};
    uint32_t *tmp = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    if (!tmp) return -1;
    for (uint64_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
    merge_sort_idx(&s, perm, tmp, n);
    free(tmp);
    return 0;
}

/* ---------------------------------------------------------------------------------------
 * MarkDuplicates (algorithms/mark_duplicates.cpp) restated.
 * ------------------------------------------------------------------------------------- */
enum { RE_NONE, RE_F, RE_R, RE_FF, RE_RR, RE_FR, RE_RF }; /* util/picard_structures.h:24-27 */

typedef struct {
    int16_t libraryId, score;
    int32_t orientation;
    int32_t read1Sequence, read1Coordinate;
    int64_t read1IndexInFile;
    int32_t read2Sequence, read2Coordinate;
    int64_t read2IndexInFile;
} ReadEnds; /* util/picard_structures.h:29-53 */

static void readends_init(ReadEnds *e) {
    e->libraryId = -1; e->score = -1; e->orientation = RE_NONE;
    e->read1Sequence = -1; e->read1Coordinate = -1; e->read1IndexInFile = -1;
    e->read2Sequence = -1; e->read2Coordinate = -1; e->read2IndexInFile = -1;
}

/* ReadEnds::compare (util/picard_structures.h:56-68) */
static int readends_compare(const ReadEnds *l, const ReadEnds *r) {
    int ret = 0;
    if (ret == 0) ret = l->libraryId - r->libraryId;
    if (ret == 0) ret = l->read1Sequence - r->read1Sequence;
    if (ret == 0) ret = l->read1Coordinate - r->read1Coordinate;
    if (ret == 0) ret = l->orientation - r->orientation;
    if (ret == 0) ret = l->read2Sequence - r->read2Sequence;
    if (ret == 0) ret = l->read2Coordinate - r->read2Coordinate;
    if (ret == 0) ret = (int)(l->read1IndexInFile - r->read1IndexInFile);
    if (ret == 0) ret = (int)(l->read2IndexInFile - r->read2IndexInFile);
    return ret;
}
static int cmp_re_ptr(const void *a, const void *b) {
    return readends_compare(*(const ReadEnds *const *)a, *(const ReadEnds *const *)b);
}

/* cigar walk helpers (mark_duplicates.cpp:44-129) */
static const uint8_t *cigar_ptr(const uint8_t *r) { return r + OFF_NAME + r[OFF_LNAME]; }
static int reference_length(const uint8_t *r) {
    int len = 0;
    uint32_t nc = rd16(r + OFF_NCIGAR);
    const uint8_t *c = cigar_ptr(r);
    for (uint32_t i = 0; i < nc; ++i) {
        uint32_t op = rd32(c + 4 * i), t = op & 0xF;
        if (t == 0 || t == 2 || t == 3 || t == 7 || t == 8) len += (int)(op >> 4); /* M D N = X */
    }
    return len;
}
static int unclipped_start(const uint8_t *r) {
    int pos = rdi32(r + OFF_POS);
    uint32_t nc = rd16(r + OFF_NCIGAR);
    const uint8_t *c = cigar_ptr(r);
    for (uint32_t i = 0; i < nc; ++i) {
        uint32_t op = rd32(c + 4 * i), t = op & 0xF;
        if (t == 4 || t == 5) pos -= (int)(op >> 4); else break;
    }
    return pos;
}
static int unclipped_end(const uint8_t *r) {
    int flag = rd16(r + OFF_FLAG);
    int pos = (flag & 0x4) ? -1 : rdi32(r + OFF_POS) + reference_length(r) - 1; /* getAlignmentEnd :73-79 */
    uint32_t nc = rd16(r + OFF_NCIGAR);
    const uint8_t *c = cigar_ptr(r);
    for (int i = (int)nc - 1; i >= 0; --i) {
        uint32_t op = rd32(c + 4 * i), t = op & 0xF;
        if (t == 4 || t == 5) pos += (int)(op >> 4); else break;
    }
    return pos;
}
/* getScore (:135-144): short accumulator of qual bytes >= 15 */
static int16_t get_score(const uint8_t *r) {
    int16_t score = 0;
    uint32_t lseq = rd32(r + OFF_LSEQ), nc = rd16(r + OFF_NCIGAR);
    const uint8_t *q = cigar_ptr(r) + 4 * nc + (lseq + 1) / 2;
    for (uint32_t i = 0; i < lseq; ++i) {
        uint8_t b = (uint8_t)(q[i] + 33 - 33);
        if (b >= 15) score = (int16_t)(score + b);
    }
    return score;
}

/* BamAlignment::GetTag<std::string>("RG") with FindTag/SkipToNextTag semantics
 * (util/bamtools/BamAlignment.cpp:270-294,699-780, BamAlignment.h:576-606). */
static int tag_skip(char type, const uint8_t **p, const uint8_t *end) {
    switch (type) {
    case 'A': case 'c': case 'C': *p += 1; return 1;
    case 's': case 'S': *p += 2; return 1;
    case 'f': case 'i': case 'I': *p += 4; return 1;
    case 'Z': case 'H':
        while (*p < end && **p) ++*p;
        ++*p; return 1;
    case 'B': {
        if (*p + 5 > end) return 0;
        char at = (char)(*p)[0];
        int32_t cnt = rdi32(*p + 1);
        *p += 5;
        int sz;
        switch (at) {
        case 'c': case 'C': sz = 1; break;
        case 's': case 'S': sz = 2; break;
        case 'f': case 'i': case 'I': sz = 4; break;
        default: return 0;
        }
        *p += (int64_t)cnt * sz;
        return 1;
    }
    default: return 0;
    }
}
static int get_rg(const uint8_t *r, const uint8_t **val, uint32_t *len) {
    uint32_t bs = rd32(r);
    uint32_t lseq = rd32(r + OFF_LSEQ), nc = rd16(r + OFF_NCIGAR);
    const uint8_t *p = cigar_ptr(r) + 4 * nc + (lseq + 1) / 2 + lseq;
    const uint8_t *end = r + 4 + bs;
    if (p >= end) return 0;
    while (p < end) {
        const uint8_t *tag = p, *type = p + 2;
        p += 3;
        if (tag[0] == 'R' && tag[1] == 'G') {
            const uint8_t *s = p;
            while (s < end && *s) ++s;
            *val = p; *len = (uint32_t)(s - p);
            return 1;
        }
        if (*type == 0) return 0;
        if (!tag_skip((char)*type, &p, end)) return 0;
        if (p >= end || *p == 0) return 0;
    }
    return 0;
}

/* ---- string-keyed map for the pair table (ReadEndsMap, util/picard_structures.h:82-109) */
typedef struct { uint64_t h; char *key; uint32_t klen; ReadEnds *val; } slot_t;
typedef struct { slot_t *s; uint64_t cap, used; } smap;
static uint64_t fnv(const char *k, uint32_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; ++i) { h ^= (uint8_t)k[i]; h *= 1099511628211ull; }
    return h | 1;
}
static void smap_grow(smap *m);
static slot_t *smap_find(smap *m, const char *k, uint32_t n, uint64_t h, int create) {
    if (create && (m->used + 1) * 2 > m->cap) smap_grow(m);
    uint64_t i = h & (m->cap - 1);
    for (;;) {
        slot_t *s = &m->s[i];
        if (s->h == 0) {
            if (!create) return NULL;
            s->h = h; s->klen = n; s->key = (char *)malloc(n ? n : 1); memcpy(s->key, k, n); s->val = NULL;
            m->used++;
            return s;
        }
        if (s->h == h && s->klen == n && memcmp(s->key, k, n) == 0) return s;
        i = (i + 1) & (m->cap - 1);
    }
}
static void smap_grow(smap *m) {
    uint64_t oc = m->cap;
    slot_t *os = m->s;
    m->cap = oc ? oc * 2 : 1024;
    m->s = (slot_t *)calloc(m->cap, sizeof(slot_t));
    m->used = 0;
    for (uint64_t i = 0; i < oc; ++i)
        if (os[i].h) {
            slot_t *d = smap_find(m, os[i].key, os[i].klen, os[i].h, 1);
            free(d->key);
            d->key = os[i].key; d->val = os[i].val;
        }
    free(os);
}
/* erase with backward-shift deletion */
static void smap_erase(smap *m, slot_t *s) {
    uint64_t i = (uint64_t)(s - m->s);
    free(s->key);
    m->s[i].h = 0;
    m->used--;
    uint64_t j = i;
    for (;;) {
        j = (j + 1) & (m->cap - 1);
        if (m->s[j].h == 0) break;
        uint64_t home = m->s[j].h & (m->cap - 1);
        int move = (i <= j) ? (home <= i || home > j) : (home <= i && home > j);
        if (move) { m->s[i] = m->s[j]; m->s[j].h = 0; i = j; }
    }
}

typedef struct {
    const char *rg_ids; uint64_t rg_ids_bytes; const int16_t *rg_lib; int32_t n_rg; int16_t unknown_lib;
} libmap;

static int16_t library_id(const libmap *L, const uint8_t *rgv, uint32_t rglen, int has_rg) {
    if (!has_rg || rglen == 0) return L->unknown_lib;
    const char *p = L->rg_ids;
    for (int32_t i = 0; i < L->n_rg; ++i) {
        size_t n = strlen(p);
        if (n == rglen && memcmp(p, rgv, n) == 0) return L->rg_lib[i];
        p += n + 1;
    }
    return L->unknown_lib;
}

typedef struct { ReadEnds **v; uint64_t n, cap; } revec;
static void push(revec *v, ReadEnds *e) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 1024; v->v = (ReadEnds **)realloc(v->v, v->cap * sizeof(*v->v)); }
    v->v[v->n++] = e;
}

static int orientation_byte(int r1neg, int r2neg) { /* getOrientationByte :169-178 */
    if (r1neg) return r2neg ? RE_RR : RE_RF;
    return r2neg ? RE_FR : RE_FF;
}

static ReadEnds *build_read_ends(const libmap *L, int64_t index, const uint8_t *r) { /* :147-164 */
    ReadEnds *e = (ReadEnds *)malloc(sizeof(ReadEnds));
    readends_init(e);
    uint16_t flag = rd16(r + OFF_FLAG);
    int rev = (flag & 0x10) != 0;
    e->read1Sequence = rdi32(r + OFF_REFID);
    e->read1Coordinate = rev ? unclipped_end(r) : unclipped_start(r);
    e->orientation = rev ? RE_R : RE_F;
    e->read1IndexInFile = index;
    e->score = get_score(r);
    if ((flag & 0x1) && !(flag & 0x8)) e->read2Sequence = rdi32(r + OFF_MREFID);
    const uint8_t *rgv = NULL; uint32_t rgl = 0;
    int has = get_rg(r, &rgv, &rgl);
    e->libraryId = library_id(L, rgv, rgl, has);
    return e;
}

static int comparable(const ReadEnds *a, const ReadEnds *b, int r2) { /* :402-414 */
    int ret = a->libraryId == b->libraryId && a->read1Sequence == b->read1Sequence &&
              a->read1Coordinate == b->read1Coordinate && a->orientation == b->orientation;
    if (ret && r2) ret = a->read2Sequence == b->read2Sequence && a->read2Coordinate == b->read2Coordinate;
    return ret;
}

static void add_dup(uint8_t *is_dup, uint64_t n, int64_t idx, uint64_t *count) {
    if (idx >= 0 && (uint64_t)idx < n) is_dup[idx] = 1;
    ++*count;
}

static void mark_pairs(ReadEnds **list, uint64_t n, uint8_t *is_dup, uint64_t nrec, uint64_t *cnt) { /* :488-507 */
    int16_t max = 0; ReadEnds *best = NULL;
    for (uint64_t i = 0; i < n; ++i)
        if (list[i]->score > max || best == NULL) { max = list[i]->score; best = list[i]; }
    for (uint64_t i = 0; i < n; ++i)
        if (list[i] != best) {
            add_dup(is_dup, nrec, list[i]->read1IndexInFile, cnt);
            add_dup(is_dup, nrec, list[i]->read2IndexInFile, cnt);
        }
}

static void mark_frags(ReadEnds **list, uint64_t n, int contains_pairs, uint8_t *is_dup, uint64_t nrec, uint64_t *cnt) { /* :515-540 */
    if (contains_pairs) {
        for (uint64_t i = 0; i < n; ++i)
            if (list[i]->read2Sequence == -1) add_dup(is_dup, nrec, list[i]->read1IndexInFile, cnt);
    } else {
        int16_t max = 0; ReadEnds *best = NULL;
        for (uint64_t i = 0; i < n; ++i)
            if (list[i]->score > max || best == NULL) { max = list[i]->score; best = list[i]; }
        for (uint64_t i = 0; i < n; ++i)
            if (list[i] != best) add_dup(is_dup, nrec, list[i]->read1IndexInFile, cnt);
    }
}

/* dup_out[i]: 1 = set 0x400, 0 = primary with 0x400 cleared, 2 = non-primary (untouched).
 * Returns the number of records flagged. */
int64_t oracle_markdup(const uint8_t *recs, const uint64_t *offs, uint64_t n,
                       const char *rg_ids, uint64_t rg_ids_bytes, const int16_t *rg_lib, int32_t n_rg,
                       int16_t unknown_lib, int compat_nonverbose_index, uint8_t *dup_out) {
    rec_set s = {recs, offs};
    libmap L = {rg_ids, rg_ids_bytes, rg_lib, n_rg, unknown_lib};
    smap tmp = {0, 0, 0};
    smap_grow(&tmp);
    revec pairs = {0, 0, 0}, frags = {0, 0, 0};
    int64_t index = 0;
    char *key = (char *)malloc(1024);
    /* buildSortedReadEndLists (:185-279) */
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *r = REC(&s, i);
        uint16_t flag = rd16(r + OFF_FLAG);
        int32_t refid = rdi32(r + OFF_REFID);
        if ((flag & 0x4) || refid == -1) {
            /* unmapped / no coordinate: written through */
        } else if (!(flag & 0x100)) {
            ReadEnds *frag = build_read_ends(&L, index, r);
            push(&frags, frag);
            if ((flag & 0x1) && !(flag & 0x8)) {
                const uint8_t *rgv = NULL; uint32_t rgl = 0;
                if (!get_rg(r, &rgv, &rgl)) rgl = 0;
                uint32_t nl = r[OFF_LNAME] ? r[OFF_LNAME] - 1u : 0u;
                uint32_t kl = rgl + 1 + nl;
                memcpy(key, rgv, rgl); key[rgl] = ':'; memcpy(key + rgl + 1, r + OFF_NAME, nl);
                uint64_t h = fnv(key, kl);
                slot_t *sl = smap_find(&tmp, key, kl, h, 0);
                ReadEnds *pe = sl ? sl->val : NULL;
                if (sl) smap_erase(&tmp, sl);
                if (pe == NULL) {
                    pe = build_read_ends(&L, index, r);
                    slot_t *ns = smap_find(&tmp, key, kl, h, 1);
                    ns->val = pe;
                } else {
                    int seq = frag->read1Sequence, coord = frag->read1Coordinate;
                    int rev = (flag & 0x10) != 0;
                    if (seq > pe->read1Sequence || (seq == pe->read1Sequence && coord >= pe->read1Coordinate)) {
                        pe->read2Sequence = seq; pe->read2Coordinate = coord; pe->read2IndexInFile = index;
                        pe->orientation = orientation_byte(pe->orientation == RE_R, rev);
                    } else {
                        pe->read2Sequence = pe->read1Sequence; pe->read2Coordinate = pe->read1Coordinate;
                        pe->read2IndexInFile = pe->read1IndexInFile;
                        pe->read1Sequence = seq; pe->read1Coordinate = coord; pe->read1IndexInFile = index;
                        pe->orientation = orientation_byte(rev, pe->orientation == RE_R);
                    }
                    pe->score = (int16_t)(pe->score + get_score(r));
                    push(&pairs, pe);
                }
            }
        }
        /* :250 -- the index only advances when verbose */
        if (!compat_nonverbose_index) ++index;
    }
    free(key);
    qsort(pairs.v, pairs.n, sizeof(ReadEnds *), cmp_re_ptr);
    qsort(frags.v, frags.n, sizeof(ReadEnds *), cmp_re_ptr);

    uint8_t *is_dup = (uint8_t *)calloc(n ? n : 1, 1);
    uint64_t cnt = 0;
    /* generateDuplicateIndexes (:326-400) */
    {
        ReadEnds *first = NULL;
        uint64_t start = 0;
        for (uint64_t i = 0; i < pairs.n; ++i) {
            ReadEnds *nx = pairs.v[i];
            if (first == NULL) { first = nx; start = i; }
            else if (comparable(first, nx, 1)) { }
            else {
                if (i - start > 1) mark_pairs(pairs.v + start, i - start, is_dup, n, &cnt);
                start = i; first = nx;
            }
        }
        if (pairs.n) mark_pairs(pairs.v + start, pairs.n - start, is_dup, n, &cnt);
    }
    {
        ReadEnds *first = NULL;
        uint64_t start = 0;
        int cp = 0, cf = 0;
        for (uint64_t i = 0; i < frags.n; ++i) {
            ReadEnds *nx = frags.v[i];
            if (first != NULL && comparable(first, nx, 0)) {
                cp = cp || nx->read2Sequence != -1;
                cf = cf || nx->read2Sequence == -1;
            } else {
                if (i - start > 1 && cf) mark_frags(frags.v + start, i - start, cp, is_dup, n, &cnt);
                start = i; first = nx;
                cp = nx->read2Sequence != -1;
                cf = nx->read2Sequence == -1;
            }
        }
        if (frags.n) mark_frags(frags.v + start, frags.n - start, cp, is_dup, n, &cnt);
    }
    /* apply (:440-465): primary records get 0x400 set/cleared, others untouched */
    int64_t flagged = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *r = REC(&s, i);
        uint16_t flag = rd16(r + OFF_FLAG);
        if (!(flag & 0x100)) { dup_out[i] = is_dup[i]; flagged += is_dup[i]; }
        else dup_out[i] = 2;
    }
    for (uint64_t i = 0; i < pairs.n; ++i) free(pairs.v[i]);
    for (uint64_t i = 0; i < frags.n; ++i) free(frags.v[i]);
    for (uint64_t i = 0; i < tmp.cap; ++i) if (tmp.s[i].h) { free(tmp.s[i].key); free(tmp.s[i].val); }
    free(tmp.s); free(pairs.v); free(frags.v); free(is_dup);
    return flagged;
}

/* Split-by-chromosome: cmd/command_dedup.cpp:71-106 feeds record i to chain
 * refID % K (refID < 0 -> chain 0, algorithms/split_by_chromosome.cpp:45-48); every chain is its
 * own MarkDuplicates over its records in stream order, and SortedMerge puts the records back in
 * stream order (chains never hold equal-position records of one another).  Restated literally:
 * one oracle_markdup per chain. */
int64_t oracle_markdup_split(const uint8_t *recs, const uint64_t *offs, uint64_t n,
                             const char *rg_ids, uint64_t rg_ids_bytes, const int16_t *rg_lib, int32_t n_rg,
                             int16_t unknown_lib, int compat_nonverbose_index, int chains, uint8_t *dup_out) {
    if (chains <= 1)
        return oracle_markdup(recs, offs, n, rg_ids, rg_ids_bytes, rg_lib, n_rg, unknown_lib, compat_nonverbose_index,
                              dup_out);
    uint64_t *sub = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
    uint64_t *idx = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
    uint8_t *d = (uint8_t *)malloc(n ? n : 1);
    int64_t total = 0;
    for (int c = 0; c < chains; ++c) {
        uint64_t m = 0;
        for (uint64_t i = 0; i < n; ++i) {
            int32_t refid = rdi32(recs + offs[i] + OFF_REFID);
            int chain = refid < 0 ? 0 : refid % chains;
            if (chain == c) { sub[m] = offs[i]; idx[m] = i; ++m; }
        }
        total += oracle_markdup(recs, sub, m, rg_ids, rg_ids_bytes, rg_lib, n_rg, unknown_lib, compat_nonverbose_index, d);
        for (uint64_t j = 0; j < m; ++j) dup_out[idx[j]] = d[j];
    }
    free(sub); free(idx); free(d);
    return total;
}

/* ------------------------------------------------------------------------------------------
 * Local realignment offset scan: LocalRealignment::findBestOffset
 * (algorithms/local_realignment.cpp:1126-1164) over mismatchQualitySumIgnoreCigar (:641-679),
 * restated literally -- including its early exits (quitAboveThisValue, the return at score 0)
 * and its two loops -- so the HIP kernel's closed form (min over (score, visit rank)) is checked
 * against the reference's control flow, not against itself.  Qualities are ASCII chars
 * (phred + 33, kept as char: values above 94 wrap negative as in the reference); isRegularBase is
 * util/gatk/BaseUtils.h:49-57.  Offsets past the consensus end (Q26: the reference reads out of
 * range there) count 99 per base, the defined behaviour the product also uses.
 * ------------------------------------------------------------------------------------------ */
static int is_regular_base(char b) {
    return b == 'A' || b == 'C' || b == 'G' || b == 'T' || b == 'a' || b == 'c' || b == 'g' || b == 't' || b == '*';
}

static int mismatch_quality_sum(const char *read, const char *quals, int64_t rlen, const char *ref, int64_t reflen,
                                int64_t refIndex, int quit) {
    int sum = 0;
    int64_t common = refIndex >= reflen ? 0 : (rlen < reflen - refIndex - 1 ? rlen : reflen - refIndex - 1);
    int64_t readIndex = 0;
    for (; readIndex < common && sum <= quit; refIndex++, readIndex++) {
        char refChr = ref[refIndex], readChr = read[readIndex];
        if (!is_regular_base(readChr) || !is_regular_base(refChr)) continue;
        if (readChr != refChr) sum += (int)quals[readIndex] - 33;
    }
    for (; readIndex < rlen && sum <= quit; refIndex++, readIndex++) {
        if (refIndex >= reflen) {
            sum += 99; /* MAX_QUAL */
        } else {
            char refChr = ref[refIndex], readChr = read[readIndex];
            if (!is_regular_base(readChr) || !is_regular_base(refChr)) continue;
            if (readChr != refChr) sum += (int)quals[readIndex] - 33;
        }
    }
    return sum;
}

/* quals_phred: raw BAM quality bytes (converted to the reference's ASCII chars here) */
int oracle_find_best_offset(const char *cons, int64_t cons_len, const char *read, const uint8_t *quals_phred, int64_t rlen,
                            int orig, int max_start, int *best_score) {
    char *q = (char *)malloc((size_t)(rlen > 0 ? rlen : 1));
    for (int64_t i = 0; i < rlen; ++i) q[i] = (char)(quals_phred[i] + 33);
    int bestScore = mismatch_quality_sum(read, q, rlen, cons, cons_len, orig, 0x7FFFFFFF);
    int bestIndex = orig;
    if (bestScore == 0) goto done;
    for (int i = 0; i < orig; i++) {
        int score = mismatch_quality_sum(read, q, rlen, cons, cons_len, i, bestScore);
        if (score < bestScore) { bestScore = score; bestIndex = i; }
        if (bestScore == 0) goto done;
    }
    for (int i = orig + 1; i <= max_start; i++) {
        int score = mismatch_quality_sum(read, q, rlen, cons, cons_len, i, bestScore);
        if (score < bestScore) { bestScore = score; bestIndex = i; }
        if (bestScore == 0) goto done;
    }
done:
    free(q);
    *best_score = bestScore;
    return bestIndex;
}

/* Batch form with the layout of oge_realign_scan (include/openge_hip.h). */
int oracle_realign_scan(const uint8_t *cons, const uint64_t *cons_off, const uint8_t *bases, const uint8_t *quals,
                        const uint64_t *read_off, const int32_t *pairs, uint64_t n_pairs, int32_t *best_index,
                        int32_t *best_score) {
    for (uint64_t p = 0; p < n_pairs; ++p) {
        const int32_t *P = pairs + 4 * p;
        const uint64_t c0 = cons_off[P[0]], c1 = cons_off[P[0] + 1], r0 = read_off[P[1]], r1 = read_off[P[1] + 1];
        int s;
        best_index[p] = oracle_find_best_offset((const char *)cons + c0, (int64_t)(c1 - c0), (const char *)bases + r0,
                                                quals + r0, (int64_t)(r1 - r0), P[2], P[3], &s);
        best_score[p] = s;
    }
    return 0;
}

/* ---------------------------------------------------------------------------------------
 * mergesort extras.
 *
 * Filter::runInternal (algorithms/filter.cpp:205-249): keep[i] = 1 for the records the module
 * passes on, in input order; at most count_limit are kept (the loop stops pulling at the limit).
 * len = BamAlignment::getLength() = l_seq; the region test is refID in [L, R], pos + len >= left,
 * pos <= right (filter.cpp:230-236).  Returns the number kept. */
uint64_t oracle_filter(const uint8_t *recs, const uint64_t *offs, uint64_t n, int has_region, int32_t ref_id,
                       int32_t left_pos, int32_t right_pos, int32_t mapq_min, int32_t min_len, int32_t max_len,
                       int32_t trim_total, uint64_t count_limit, uint8_t *keep) {
    uint64_t count = 0, i;
    for (i = 0; i < n; ++i) {
        const uint8_t *r = recs + offs[i];
        int32_t len = rdi32(r + OFF_LSEQ), mapq = r[13], ok;
        ok = mapq >= mapq_min && len >= min_len && len <= max_len && len > trim_total;
        if (has_region) {
            int32_t ref = rdi32(r + OFF_REFID), pos = rdi32(r + OFF_POS);
            ok = ok && ref >= ref_id && (int32_t)((uint32_t)pos + (uint32_t)len) >= left_pos && ref <= ref_id &&
                 pos <= right_pos;
        }
        ok = ok && count < count_limit;
        keep[i] = (uint8_t)ok;
        count += ok;
    }
    return count;
}

/* Sort::ByName (util/bamtools/Sort.h:67-90): std::string < on the read names (unsigned bytewise,
 * shorter prefix first); equal names keep input order here (the reference's std::sort leaves
 * them in an implementation-defined order). */
static const rec_set *g_name_set;
static int name_cmp(uint32_t a, uint32_t b) {
    const uint8_t *ra = REC(g_name_set, a), *rb = REC(g_name_set, b);
    int la = ra[OFF_LNAME] - 1, lb = rb[OFF_LNAME] - 1, m = la < lb ? la : lb;
    int c = memcmp(ra + OFF_NAME, rb + OFF_NAME, (size_t)m);
    if (c) return c;
    if (la != lb) return la < lb ? -1 : 1;
    return a < b ? -1 : a > b;
}
static int name_cmp_q(const void *x, const void *y) { return name_cmp(*(const uint32_t *)x, *(const uint32_t *)y); }

int oracle_sort_name(const uint8_t *recs, const uint64_t *offs, uint64_t n, uint32_t *perm) {
    rec_set s = {recs, offs};
    uint64_t i;
    for (i = 0; i < n; ++i) perm[i] = (uint32_t)i;
    g_name_set = &s;
    qsort(perm, n, sizeof(uint32_t), name_cmp_q);
    g_name_set = 0;
    return 0;
}
