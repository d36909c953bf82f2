// defl_model.c -- CPU model of the GPU deflate parse (bgzf.hip k_defl_parse) and of level-6-class
// variants, to price each search feature in compressed bytes before it is built (profiling aid, not a
// test, not shipped).  Per 65,280-byte payload: hash candidates visible in rounds of R positions (a
// position sees the table as the earlier rounds left it), K candidates per position (a prev chain over
// earlier rounds), optional lazy evaluation (zlib's: at p with match L, look at p+1; take the literal
// when p+1's match is longer), matches cut at S-byte segment edges (0: none).  Size = Huffman-coded
// symbols (code lengths limited to 15) + extra bits + a dynamic-header estimate + 26 bytes of BGZF framing.
//
//   gcc -O2 -o /tmp/defl_model tools/defl_model.c && /tmp/defl_model sample.bin R K lazy S hashbytes hashbits
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { PAY = 65280, HB = 12, NLIT = 286, NDIST = 30 };

static uint32_t rd32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

static void len_code(uint32_t L, int *sym, int *nb) {
    uint32_t l = L - 3;
    if (l < 8) *sym = 257 + l, *nb = 0;
    else if (l == 255) *sym = 285, *nb = 0;
    else {
        int lg = 31 - __builtin_clz(l);
        *sym = 257 + 4 * (lg - 1) + ((l >> (lg - 2)) & 3), *nb = lg - 2;
    }
}
static void dist_code(uint32_t D, int *sym, int *nb) {
    uint32_t d = D - 1;
    if (d < 4) *sym = d, *nb = 0;
    else {
        int lg = 31 - __builtin_clz(d);
        *sym = 2 * lg + ((d >> (lg - 1)) & 1), *nb = lg - 1;
    }
}

// Huffman code lengths (heap-free O(n^2) build, fine for <= 286 symbols), then limited to 15 bits by
// the usual overflow fix-up.
static void huff_lengths(const uint64_t *f, int n, int *len) {
    int m = 0, idx[NLIT];
    uint64_t w[2 * NLIT];
    int par[2 * NLIT];
    for (int i = 0; i < n; ++i) {
        len[i] = 0;
        if (f[i]) idx[m++] = i;
    }
    if (m == 0) return;
    if (m == 1) {
        len[idx[0]] = 1;
        return;
    }
    int alive[2 * NLIT], na = 0, nn = m;
    for (int i = 0; i < m; ++i) w[i] = f[idx[i]], alive[na++] = i;
    while (na > 1) {
        int a = 0, b = 1;
        if (w[alive[b]] < w[alive[a]]) a = 1, b = 0;
        for (int i = 2; i < na; ++i) {
            if (w[alive[i]] < w[alive[a]]) b = a, a = i;
            else if (w[alive[i]] < w[alive[b]]) b = i;
        }
        int x = alive[a], y = alive[b];
        w[nn] = w[x] + w[y];
        par[x] = par[y] = nn;
        int hi = a > b ? a : b, lo = a > b ? b : a;
        alive[hi] = alive[--na];
        alive[lo] = nn++;
        if (lo == na) alive[lo] = nn - 1;
    }
    par[nn - 1] = -1;
    for (int i = 0; i < m; ++i) {
        int d = 0;
        for (int k = i; par[k] >= 0; k = par[k]) ++d;
        len[idx[i]] = d;
    }
    // limit to 15: Kraft repair
    for (;;) {
        double kr = 0;
        int over = 0;
        for (int i = 0; i < n; ++i)
            if (len[i]) {
                if (len[i] > 15) len[i] = 15, over = 1;
                kr += 1.0 / (1 << len[i]);
            }
        if (kr <= 1.0 + 1e-12) break;
        (void)over;
        // lengthen the longest code below 15 with the smallest frequency
        int best = -1;
        for (int i = 0; i < n; ++i)
            if (len[i] && len[i] < 15 && (best < 0 || f[i] < f[best])) best = i;
        len[best]++;
    }
}

typedef struct {
    int R, K, lazy, S, hb, hbits, split;  // K: chain entries examined per position (< 0: -K slots per bucket)
} Cfg;

static uint64_t payload_bits(const uint8_t *in, int n, const Cfg *c) {
    static int32_t head[1 << 16], prev[PAY + 8];
    static int32_t rhead[1 << 16];
    static uint64_t FL[8][NLIT], FD[8][NDIST];
    uint64_t extra = 0;
    memset(FL, 0, sizeof FL), memset(FD, 0, sizeof FD);
    const int nsplit = c->split > 0 ? c->split : 1;
#define CH(pos) ((int)((int64_t)(pos) * nsplit / n))
    const int hbits = c->hbits;
    memset(head, 0, sizeof head);
    const uint32_t hmask = (1u << hbits) - 1;
    // visibility in rounds: build per round, parse after (positions see rounds < their own)
    // cands: for each position p, up to K earlier-round positions with the same prefix hash
    static int32_t cand[PAY][256];
    static uint8_t ncand[PAY];
    if (c->K < 0) {  // GPU-shaped: -K slots per bucket; a round touching a bucket shifts its slots down
        static int32_t slot[8][1 << 16];
        const int ns = -c->K;
        memset(slot, 0, sizeof slot);
        for (int r = 0; r < n; r += c->R) {
            int e = r + c->R < n ? r + c->R : n;
            for (int p = r; p < e; ++p) {
                ncand[p] = 0;
                if (p + 4 > n) continue;
                uint32_t w = rd32(in + p), h = (w * 2654435761u) >> (32 - hbits);
                int k = 0;
                for (int i = 0; i < ns; ++i) {
                    int j = slot[i][h];
                    if (j && p - (j - 1) <= 32768 && rd32(in + j - 1) == w) cand[p][k++] = j - 1;
                }
                ncand[p] = k;
            }
            static int32_t mx[1 << 16];
            for (int p = r; p < e; ++p)
                if (p + 4 <= n) mx[(rd32(in + p) * 2654435761u) >> (32 - hbits)] = 0;
            for (int p = r; p < e; ++p)
                if (p + 4 <= n) mx[(rd32(in + p) * 2654435761u) >> (32 - hbits)] = p + 1;
            for (int p = r; p < e; ++p) {
                if (p + 4 > n) continue;
                uint32_t h = (rd32(in + p) * 2654435761u) >> (32 - hbits);
                if (mx[h] != p + 1) continue;  // the bucket's round max does the shift
                for (int i = ns - 1; i > 0; --i) slot[i][h] = slot[i - 1][h];
                slot[0][h] = p + 1;
            }
        }
    }
    const char *lte = getenv("LT");  // long table: "keybytes,step,bits" (sparse insertion, lookups everywhere)
    if (lte && c->K < 0) {
        int kb = 8, st = 4, lb = 12;
        sscanf(lte, "%d,%d,%d", &kb, &st, &lb);
        static int32_t lt[1 << 16];
        memset(lt, 0, sizeof lt);
        for (int r = 0; r < n; r += c->R) {
            int e = r + c->R < n ? r + c->R : n;
            for (int p = r; p < e; ++p) {
                if (p + kb > n) continue;
                uint64_t w = 0;
                memcpy(&w, in + p, 8);
                if (kb < 8) w &= (1ull << (8 * kb)) - 1;
                uint32_t h = (uint32_t)((w * 0x9E3779B97F4A7C15ull) >> (64 - lb));
                int j = lt[h];
                if (j && p - (j - 1) <= 32768 && memcmp(in + j - 1, in + p, kb) == 0 && ncand[p] < 250) {
                    int dup = 0;
                    for (int k = 0; k < ncand[p]; ++k) dup |= cand[p][k] == j - 1;
                    if (!dup) cand[p][ncand[p]++] = j - 1;
                }
            }
            for (int p = r; p < e; ++p) {
                if (p + kb > n || p % st) continue;
                uint64_t w = 0;
                memcpy(&w, in + p, 8);
                if (kb < 8) w &= (1ull << (8 * kb)) - 1;
                lt[(uint32_t)((w * 0x9E3779B97F4A7C15ull) >> (64 - lb))] = p + 1;
            }
        }
    }
    const int gpuchain = getenv("GPUCHAIN") != NULL, firstv = getenv("FIRSTV") != NULL;
    for (int r = 0; c->K > 0 && r < n; r += c->R) {
        int e = r + c->R < n ? r + c->R : n;
        if (gpuchain)
            for (int p = r; p < e; ++p)
                if (p + 4 <= n) {
                    uint32_t w = rd32(in + p), key = c->hb == 3 ? (w & 0xffffff) : w;
                    uint32_t h = (key * 2654435761u) >> (32 - hbits);
                    rhead[h] = head[h];
                }
        for (int p = r; p < e; ++p) {
            ncand[p] = 0;
            if (p + 4 > n) continue;
            uint32_t w = rd32(in + p), key = c->hb == 3 ? (w & 0xffffff) : w;
            uint32_t h = (key * 2654435761u) >> (32 - hbits);
            int k = 0, ex = 0;
            const int sb = gpuchain && !getenv("NOSB") ? p / 32768 * 32768 : 0;  // links kept for the current sub-block only
            for (int j = head[h]; j && ex < c->K; j = (j - 1 >= sb ? prev[j - 1] : 0), ++ex) {
                if (p - (j - 1) > 32768) break;
                uint32_t wj = rd32(in + j - 1);
                if ((c->hb == 3 ? (wj & 0xffffff) : wj) == key) cand[p][k++] = j - 1;
                else if (ex == 0 && firstv) break;  // GPU: a position is a candidate when its first link verifies
            }
            ncand[p] = k;
        }
        for (int p = r; p < e; ++p) {  // insert the round (GPU: every position links to the head the round saw)
            if (p + 4 > n) continue;
            uint32_t w = rd32(in + p), key = c->hb == 3 ? (w & 0xffffff) : w;
            uint32_t h = (key * 2654435761u) >> (32 - hbits);
            prev[p] = gpuchain ? rhead[h] : head[h];
            head[h] = p + 1;
        }
    }
    (void)rhead;
    (void)hmask;
    // parse
    int p = 0;
    // best match at q (limited to the segment end)
#define BEST(q, outL, outD)                                                             \
    do {                                                                                \
        outL = 0, outD = 0;                                                             \
        int lim = c->S ? (((q) / c->S) + 1) * c->S : n;                                 \
        if (lim > n) lim = n;                                                           \
        int maxL = lim - (q) < 258 ? lim - (q) : 258;                                   \
        for (int k = 0; k < ncand[q]; ++k) {                                            \
            int j_ = cand[q][k], ml_ = 0;                                               \
            while (ml_ < maxL && in[j_ + ml_] == in[(q) + ml_]) ++ml_;                  \
            if (ml_ > outL) outL = ml_, outD = (q) - j_;                                \
        }                                                                               \
        if (outL < 3) outL = 0;                                                         \
    } while (0)
    while (p < n) {
        int L, D;
        BEST(p, L, D);
        if (L && c->lazy && p + 1 < n && L < 32 && (!c->S || (p + 1) % c->S)) {
            int L2, D2;
            BEST(p + 1, L2, D2);
            if (L2 > L) {
                FL[CH(p)][in[p]]++;
                p += 1;
                continue;
            }
        }
        if (L) {
            int s, nb;
            len_code(L, &s, &nb);
            FL[CH(p)][s]++, extra += nb;
            dist_code(D, &s, &nb);
            FD[CH(p)][s]++, extra += nb;
            p += L;
        } else {
            FL[CH(p)][in[p]]++;
            p += 1;
        }
    }
    uint64_t bits = extra;
    for (int b = 0; b < nsplit; ++b) {
        uint64_t *fl = FL[b], *fd = FD[b];
        fl[256]++;
        int ll[NLIT], dl[NDIST];
        huff_lengths(fl, NLIT, ll);
        huff_lengths(fd, NDIST, dl);
        int used = 0;
        for (int i = 0; i < NLIT; ++i) bits += fl[i] * ll[i], used += ll[i] > 0;
        for (int i = 0; i < NDIST; ++i) bits += fd[i] * dl[i], used += dl[i] > 0;
        bits += 17 + 19 * 3 + 4 * used + 40;  // header estimate
    }
    uint64_t stored = 8ull * (n + 5);
    return (bits < stored ? bits : stored) + 8 * 26;
}

int main(int argc, char **argv) {
    if (argc < 8) return fprintf(stderr, "usage: %s sample R K lazy S hashbytes hashbits\n", argv[0]), 2;
    FILE *fp = fopen(argv[1], "rb");
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t *buf = malloc(sz + 16);
    if (fread(buf, 1, sz, fp) != (size_t)sz) return 1;
    memset(buf + sz, 0, 16);
    Cfg c = {atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), argc > 8 ? atoi(argv[8]) : 1};
    uint64_t bits = 0;
    long nn = sz / PAY * PAY;
    for (long o = 0; o < nn; o += PAY) bits += payload_bits(buf + o, PAY, &c);
    printf("R=%d K=%d lazy=%d S=%d hb=%d hbits=%d split=%d ratio %.4f\n", c.R, c.K, c.lazy, c.S, c.hb, c.hbits, c.split, bits / 8.0 / nn);
    return 0;
}
