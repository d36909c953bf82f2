// realign.cpp -- LocalRealignment host phases A, B, D, E (see realign.h).  Offset scoring (phase C)
// goes through the ScanFn the caller binds (the HIP kernel in realign.hip).
//
// Every function below restates one reference routine; the citation names it (paths under
// openge/src/).  Quirks the parity target depends on are reproduced and marked "Q<n>" after
// SURVEY.md Appendix A.
#include "realign.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sys/mman.h>
#include <unistd.h>
#include <new>
#include <set>
#include <thread>
#include <unordered_map>

#include "bam_layout.h"

namespace oge {

// The first call in a process touches every page of its per-read arrays for the first time (the scratch
// keeps them for later calls): those are hvectors (uvector.h: 2 MiB pages, no serial zero fill on a
// resize -- the workers that fill them touch their pages first).
template <class T>
using BigVec = hvector<T>;

// =====================================================================================  threads
// Persistent workers (kept across calls with the run's Scratch).  run_static maps index i to worker
// i % size(); run hands indices out one at a time (prepare and decide: intervals differ in size; r03
// mapped them statically so each interval's frees stayed in its allocating thread's arena -- the
// interval objects are now reused instead of freed).
static thread_local int tl_worker = 0;  // the Pool worker running the current job (0 = the caller)

class Pool {
public:
    explicit Pool(int threads) {
        if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
        n_ = threads;
        for (int t = 1; t < n_; ++t) ts_.emplace_back([this, t]() { loop(t); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : ts_) t.join();
    }
    int size() const { return n_; }
    template <class F>
    void run_static(size_t n, F f) {
        if (n_ == 1 || n <= 1) {
            for (size_t i = 0; i < n; ++i) f(i);
            return;
        }
        exec([&](int t) {
            tl_worker = t;
            for (size_t i = (size_t)t; i < n; i += (size_t)n_) f(i);
        });
    }
    template <class F>
    void run(size_t n, F f) {  // dynamic: indices handed out one at a time
        if (n_ == 1 || n <= 1) {
            for (size_t i = 0; i < n; ++i) f(i);
            return;
        }
        std::atomic<size_t> next(0);
        exec([&](int t) {
            tl_worker = t;
            for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
        });
    }
    template <class F>
    void run_chunks(size_t n, size_t chunk, F f) {  // f(begin, end) over [0, n) in chunks
        run((n + chunk - 1) / chunk, [&](size_t c) { f(c * chunk, std::min(n, (c + 1) * chunk)); });
    }
    // f(0..n) handed out in increasing order to the workers while the calling thread runs lead() beside them
    // (and then helps with what is left); one thread: f over all, then lead
    template <class F, class G>
    void run_lead(size_t n, F f, G lead) {
        if (n_ == 1) {
            for (size_t i = 0; i < n; ++i) f(i);
            lead();
            return;
        }
        std::atomic<size_t> next(0);
        exec([&](int t) {
            tl_worker = t;
            if (t == 0) lead();
            for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
        });
    }

private:
    void exec(const std::function<void(int)> &job) {
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &job;
            busy_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        job(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return busy_ == 0; });
        job_ = nullptr;
    }
    void loop(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> g(m_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    int n_ = 1;
    std::vector<std::thread> ts_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Hand the pages of a large block about to be freed back to the kernel from all workers: one
// munmap of ~1 GB frees its pages serially.
static void release_pages(Pool &pool, void *p, size_t bytes) {
    const size_t pg = 4096, chunk = 64ull << 20;
    const uintptr_t b = ((uintptr_t)p + pg - 1) & ~(uintptr_t)(pg - 1), e = ((uintptr_t)p + bytes) & ~(uintptr_t)(pg - 1);
    if (e <= b + chunk) return;
    pool.run_chunks(e - b, chunk, [&](size_t lo, size_t hi) { madvise((void *)(b + lo), hi - lo, MADV_DONTNEED); });
}

// =====================================================================================  records
static const char kSeqChars[] = "=ACMGRSVTWYHKDBN";
static const char kCigChars[] = "MIDNSHP=X";

// packed byte -> its two base characters
static const struct SeqPairs {
    char p[256][2];
    SeqPairs() {
        for (int b = 0; b < 256; ++b) {
            p[b][0] = kSeqChars[b >> 4];
            p[b][1] = kSeqChars[b & 0xF];
        }
    }
} kSeqPairs;

std::string RRead::bases() const {
    std::string s(l_seq, 'N');
    char *o = &s[0];
    const uint32_t full = l_seq >> 1;
    for (uint32_t k = 0; k < full; ++k) memcpy(o + 2 * k, kSeqPairs.p[(uint8_t)seq4[k]], 2);
    if (l_seq & 1) o[l_seq - 1] = kSeqPairs.p[(uint8_t)seq4[full]][0];
    return s;
}

std::string RRead::quals_ascii() const {
    std::string q(qual);
    for (auto &c : q) c = (char)(c + 33);  // BamAlignmentSupportData::getQual (BamAlignment.cpp:846-851)
    return q;
}

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

// the same strings into a caller's (thread-local, reused) buffers: no allocation per read
static void bases_into(const RRead &r, std::string &s) {
    s.resize(r.l_seq);
    char *o = &s[0];
    const uint32_t full = r.l_seq >> 1;
    for (uint32_t k = 0; k < full; ++k) memcpy(o + 2 * k, kSeqPairs.p[(uint8_t)r.seq4[k]], 2);
    if (r.l_seq & 1) o[r.l_seq - 1] = kSeqPairs.p[(uint8_t)r.seq4[full]][0];
}

bool rread_decode(const uint8_t *rec, RRead &r, std::string &err) {
    uint32_t bs = rd32(rec);
    if (bs < 32 || bs > 10000) {  // BamDeserializer::read rejects these (util/bam_deserializer.h:160-163)
        err = "record block_size out of [32, 10000]";
        return false;
    }
    r.ref = (int32_t)rd32(rec + OGE_OFF_REFID);
    r.pos = (int32_t)rd32(rec + OGE_OFF_POS);
    uint32_t lname = rec[OGE_OFF_LNAME];
    r.mapq = rec[OGE_OFF_MAPQ];
    uint32_t nc = oge_rd_u16(rec + OGE_OFF_NCIGAR);
    r.flag = oge_rd_u16(rec + OGE_OFF_FLAG);
    r.l_seq = rd32(rec + OGE_OFF_LSEQ);
    r.mref = (int32_t)rd32(rec + OGE_OFF_MREFID);
    r.mpos = (int32_t)rd32(rec + OGE_OFF_MPOS);
    r.tlen = (int32_t)rd32(rec + OGE_OFF_TLEN);
    uint64_t need = 32ull + lname + 4ull * nc + (r.l_seq + 1) / 2 + r.l_seq;
    if (need > bs) {
        err = "record fields overrun block_size";
        return false;
    }
    const uint8_t *p = rec + OGE_OFF_NAME;
    r.name = std::string_view((const char *)p, lname ? lname - 1 : 0);
    p += lname;
    r.cigar.resize(nc);
    for (uint32_t i = 0; i < nc; ++i) {
        uint32_t op = rd32(p + 4 * i);
        r.cigar[i].t = kCigChars[(op & 0xF) < 9 ? (op & 0xF) : 0];
        r.cigar[i].n = op >> 4;
    }
    p += 4 * nc;
    r.seq4 = std::string_view((const char *)p, (r.l_seq + 1) / 2);
    p += (r.l_seq + 1) / 2;
    r.qual = std::string_view((const char *)p, r.l_seq);
    p += r.l_seq;
    r.tags_in = std::string_view((const char *)p, (size_t)(rec + 4 + bs - p));
    uint32_t h = 2166136261u;
    for (char ch : r.name) h = (h ^ (uint8_t)ch) * 16777619u;
    r.name_hash = h;
    r.tags_own.clear();
    r.tags_owned = false;
    r.mq_add = -1;
    r.cleaned = false;
    return true;
}

static uint32_t cig_code(char t) {
    const char *q = strchr(kCigChars, t);
    return q ? (uint32_t)(q - kCigChars) : 0;
}

// BamSerializer::write (util/bam_serializer.h:105-147): block size from the char data, bin
// recomputed from pos and GetEndPosition (M, D, N, =, X).  A pending mate-fixer MQ lands last, where
// AddTag would have put it.
size_t rread_encoded_size(const RRead &r) {
    return 36 + r.name.size() + 1 + 4 * r.cigar.size() + r.seq4.size() + r.qual.size() + r.tags().size() +
           (r.mq_add >= 0 ? 5 : 0);
}

void rread_encode_to(const RRead &r, uint8_t *p) {
    const uint32_t lname = (uint32_t)r.name.size() + 1;
    const uint32_t nc = (uint32_t)r.cigar.size();
    const std::string_view tags = r.tags();
    const uint32_t bs = (uint32_t)rread_encoded_size(r) - 4;
    int32_t end = r.pos;
    for (auto &c : r.cigar)
        if (c.t == 'M' || c.t == 'D' || c.t == 'N' || c.t == '=' || c.t == 'X') end += (int32_t)c.n;
    const uint32_t bin = oge_reg2bin(r.pos, end);
    uint32_t core[9];
    core[0] = bs;
    core[1] = (uint32_t)r.ref;
    core[2] = (uint32_t)r.pos;
    core[3] = (bin << 16) | ((uint32_t)r.mapq << 8) | lname;
    core[4] = ((uint32_t)r.flag << 16) | nc;
    core[5] = r.l_seq;
    core[6] = (uint32_t)r.mref;
    core[7] = (uint32_t)r.mpos;
    core[8] = (uint32_t)r.tlen;
    memcpy(p, core, 36);
    p += 36;
    memcpy(p, r.name.data(), r.name.size());
    p[r.name.size()] = 0;
    p += lname;
    for (uint32_t i = 0; i < nc; ++i) {
        uint32_t op = (r.cigar[i].n << 4) | cig_code(r.cigar[i].t);
        memcpy(p + 4 * i, &op, 4);
    }
    p += 4 * nc;
    memcpy(p, r.seq4.data(), r.seq4.size());
    p += r.seq4.size();
    memcpy(p, r.qual.data(), r.qual.size());
    p += r.qual.size();
    memcpy(p, tags.data(), tags.size());
    p += tags.size();
    if (r.mq_add >= 0) {
        p[0] = 'M';
        p[1] = 'Q';
        p[2] = 'S';
        p[3] = (uint8_t)(r.mq_add & 0xFF);
        p[4] = (uint8_t)((r.mq_add >> 8) & 0xFF);
    }
}

void rread_encode(const RRead &r, std::vector<uint8_t> &out) {
    size_t o = out.size();
    out.resize(o + rread_encoded_size(r));
    rread_encode_to(r, out.data() + o);
}

std::string cigar_to_string(const Cigar &c) {
    std::string s;
    for (auto &e : c) s += std::to_string(e.n) + e.t;
    return s;
}

// =====================================================================================  tags
// Walk of BamAlignment::FindTag / SkipToNextTag (util/bamtools/BamAlignment.cpp).
static size_t tag_value_len(std::string_view t, size_t at /* index of the type byte */) {
    char ty = t[at];
    size_t v = at + 1;
    switch (ty) {
        case 'A': case 'c': case 'C': return 1;
        case 's': case 'S': return 2;
        case 'i': case 'I': case 'f': return 4;
        case 'Z': case 'H': {
            size_t e = t.find('\0', v);
            return (e == std::string_view::npos ? t.size() : e + 1) - v;
        }
        case 'B': {
            if (v + 5 > t.size()) return t.size() - v;
            char sub = t[v];
            uint32_t cnt;
            memcpy(&cnt, t.data() + v + 1, 4);
            size_t el = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
            return 5 + el * cnt;
        }
        default: return t.size() - v;  // unknown type: the rest (reference fails the parse)
    }
}

bool tag_find(std::string_view t, const char *tag, size_t *at, size_t *len) {
    size_t p = 0;
    while (p + 3 <= t.size()) {
        size_t vl = tag_value_len(t, p + 2);
        if (t[p] == tag[0] && t[p + 1] == tag[1]) {
            if (at) *at = p;
            if (len) *len = 3 + vl;
            return true;
        }
        p += 3 + vl;
    }
    return false;
}

bool tag_add_int(std::string &t, const char *tag, char type, int64_t v, int bytes) {
    if (tag_find(t, tag, nullptr, nullptr)) return false;  // AddTag never overwrites (BamAlignment.h:305-310)
    t.push_back(tag[0]);
    t.push_back(tag[1]);
    t.push_back(type);
    uint64_t u = (uint64_t)v;
    for (int i = 0; i < bytes; ++i) t.push_back((char)(u >> (8 * i)));
    return true;
}

bool tag_add_string(std::string &t, const char *tag, const std::string &v) {
    if (tag_find(t, tag, nullptr, nullptr)) return false;
    t.push_back(tag[0]);
    t.push_back(tag[1]);
    t.push_back('Z');
    t += v;
    t.push_back('\0');
    return true;
}

void tag_remove(std::string &t, const char *tag) {
    size_t at, len;
    if (tag_find(t, tag, &at, &len)) t.erase(at, len);
}

static bool tag_get_string(std::string_view t, const char *tag, std::string &v) {
    size_t at, len;
    if (!tag_find(t, tag, &at, &len) || t[at + 2] != 'Z') return false;
    v.assign(t.data() + at + 3, len > 4 ? len - 4 : 0);
    return true;
}

// EditTag(tag, "i", int): RemoveTag + AddTag, so the tag moves to the end (BamAlignment.h:463-469)
static void tag_edit_i32(std::string &t, const char *tag, int32_t v) {
    tag_remove(t, tag);
    tag_add_int(t, tag, 'i', v, 4);
}

// =====================================================================================  FASTA
// FastaReader (util/fasta_reader.cpp): sequences by name; readSequence(name, start, length) returns
// the raw bytes (case preserved).
struct Fasta {
    std::unordered_map<std::string, std::string> seq;
    BigVec<char> data;  // the file (kept, like the sequences' storage, for the next load: see Scratch; no zero
                        // fill on a resize, the workers' preads touch its pages first)
    size_t find_nl(size_t from) const {
        if (from >= data.size()) return std::string::npos;
        const void *q = memchr(data.data() + from, '\n', data.size() - from);
        return q ? (size_t)((const char *)q - data.data()) : std::string::npos;
    }
    // Whole file in one read; contigs (">" lines) located serially, their bodies de-lined in
    // parallel.  Line handling as FastaReader: name up to the first blank, CR before LF dropped.
    bool load(const std::string &path, std::string &err, Pool &pool) {
        FILE *f = fopen(path.c_str(), "rb");
        if (!f) {
            err = "cannot open reference FASTA " + path;
            return false;
        }
        data.clear();
        if (fseeko(f, 0, SEEK_END) == 0) {  // regular file: 8 MiB preads on the workers
            const off_t sz = ftello(f);
            if (sz > 0) {
                data.resize((size_t)sz);
                const int fd = fileno(f);
                const size_t chunk = 8ull << 20;
                std::atomic<bool> shortr(false);
                pool.run_chunks((size_t)sz, chunk, [&](size_t o, size_t e) {
                    while (o < e) {
                        const ssize_t r = pread(fd, &data[o], e - o, (off_t)o);
                        if (r <= 0) {
                            shortr = true;
                            return;
                        }
                        o += (size_t)r;
                    }
                });
                if (shortr) {
                    fclose(f);
                    err = "short read on reference FASTA " + path;
                    return false;
                }
                fseeko(f, sz, SEEK_SET);
            }
        }
        char buf[1 << 16];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + k);  // non-seekable input
        fclose(f);
        std::vector<size_t> hs;
        const char *b = data.data(), *e = b + data.size();
        for (const char *q = b; q < e && (q = (const char *)memchr(q, '>', (size_t)(e - q))); ++q)
            if (q == b || q[-1] == '\n') hs.push_back((size_t)(q - b));
        // names first (serially: the map's entries are made here, the last of a repeated name wins),
        // then the bodies into the entries' strings (their storage reused across loads)
        std::vector<std::string> names(hs.size());
        std::vector<size_t> les(hs.size());
        for (size_t c = 0; c < hs.size(); ++c) {
            const size_t h = hs[c], stop = c + 1 < hs.size() ? hs[c + 1] : data.size();
            size_t le = find_nl(h);
            if (le == std::string::npos || le > stop) le = stop;
            size_t ne = h + 1;
            while (ne < le && data[ne] != ' ' && data[ne] != '\t' && data[ne] != '\r') ++ne;
            names[c].assign(data.data() + h + 1, ne - h - 1);
            les[c] = le;
        }
        std::unordered_map<std::string, size_t> last;
        for (size_t c = 0; c < hs.size(); ++c) last[names[c]] = c;
        for (auto it = seq.begin(); it != seq.end();)  // contigs of an earlier file that this one lacks
            it = last.count(it->first) ? std::next(it) : seq.erase(it);
        std::vector<std::string *> bodies(hs.size(), nullptr);
        for (auto &kv : last) bodies[kv.second] = &seq[kv.first];
        pool.run(hs.size(), [&](size_t c) {
            if (!bodies[c]) return;  // a repeated name: a later entry holds it
            const size_t stop = c + 1 < hs.size() ? hs[c + 1] : data.size(), le = les[c];
            std::string &out = *bodies[c];
            out.clear();
            out.reserve(stop > le ? stop - le : 0);
            size_t p = le + 1;
            while (p < stop) {
                size_t q = find_nl(p);
                if (q == std::string::npos || q > stop) q = stop;
                size_t qe = q;
                if (qe > p && data[qe - 1] == '\r') --qe;
                out.append(data.data() + p, qe - p);
                p = q + 1;
            }
        });
        if (seq.empty()) {
            err = "no sequences in reference FASTA " + path;
            return false;
        }
        return true;
    }
    const std::string *get(const std::string &name) const {
        auto it = seq.find(name);
        return it == seq.end() ? nullptr : &it->second;
    }
};

// =====================================================================================  GenomeLoc
struct GLoc {
    int contig = -1, start = 0, stop = 0;
    bool is_before(const GLoc &o) const {  // GenomeLoc::isBefore (GenomeLoc.cpp:290-293)
        return contig < o.contig || (contig == o.contig && stop < o.start);
    }
    bool overlaps(const GLoc &o) const {  // overlapsP = !disjointP (GenomeLoc.h:119-131)
        return !(contig != o.contig || start > o.stop || o.start > stop);
    }
};

// GenomeLocParser::createGenomeLoc(const OGERead&) (GenomeLocParser.cpp:377-400): length = l_seq
// + D - I - S - H (N ignored, H subtracted although not in SEQ); stop = max(end - 1, pos).
static GLoc read_loc(const RRead &r) {
    int length = (int)r.l_seq;
    for (auto &c : r.cigar) {
        if (c.t == 'D') length += (int)c.n;
        if (c.t == 'I') length -= (int)c.n;
        if (c.t == 'S' || c.t == 'H') length -= (int)c.n;
    }
    int end = r.mapped() ? std::max(r.pos + length, r.pos) : r.pos;
    GLoc g;
    g.contig = r.ref;
    g.start = r.pos;
    g.stop = std::max(end - 1, r.pos);
    return g;
}

// =====================================================================================  cigar utils
static Cigar unclip_cigar(const Cigar &c) {  // LocalRealignment::unclipCigar (:1393-1403)
    Cigar e;
    for (auto &x : c)
        if (!(x.t == 'S' || x.t == 'H' || x.t == 'P')) e.push_back(x);
    return e;
}
static bool is_clip(const CigOp &x) { return x.t == 'S' || x.t == 'H' || x.t == 'P'; }

// LocalRealignment::reclipCigar (:1409-1432), including its skip of one element after the
// leading clips.
static Cigar reclip_cigar(const Cigar &cigar, const RRead &read) {
    Cigar e;
    const Cigar &cd = read.cigar;
    size_t i = 0, n = cd.size();
    while (i < n && is_clip(cd[i])) e.push_back(cd[i++]);
    e.insert(e.end(), cigar.begin(), cigar.end());
    i++;
    while (i < n && !is_clip(cd[i])) i++;
    while (i < n && is_clip(cd[i])) e.push_back(cd[i++]);
    return e;
}

// AlignmentUtils::createIndelString (AlignmentUtils.cpp:724-783).  `ok` = false stands for both the
// empty-string and the NULL returns (Q26; the reference throws on the latter).
static std::string create_indel_string(const Cigar &cigar, int idx, const std::string &ref, const std::string &rs,
                                       int refIndex, int readIndex, bool &ok) {
    ok = false;
    const CigOp indel = cigar[idx];
    int64_t indelLength = indel.n;
    int64_t totalRefBases = 0;
    for (int i = 0; i < idx; ++i) {
        const CigOp &ce = cigar[i];
        switch (ce.t) {
            case 'M': readIndex += ce.n; refIndex += ce.n; totalRefBases += ce.n; break;
            case 'S': readIndex += ce.n; break;
            case 'N': refIndex += ce.n; totalRefBases += ce.n; break;
            default: break;
        }
    }
    const int64_t rsz = (int64_t)ref.size();
    if (totalRefBases + indelLength > rsz) indelLength -= (totalRefBases + indelLength - rsz);
    const int64_t altsz = rsz + (indel.t == 'D' ? -indelLength : indelLength);
    if (altsz < 0 || refIndex < 0 || refIndex > altsz || refIndex > rsz) return std::string();
    std::string alt((size_t)altsz, ' ');
    memcpy(&alt[0], ref.data(), (size_t)refIndex);
    int64_t cur = refIndex, ri = refIndex;
    if (indel.t == 'D') {
        ri += indelLength;
    } else {
        for (int64_t k = 0; k < indelLength; ++k)
            alt[(size_t)(cur + k)] = (readIndex + k) < (int64_t)rs.size() ? rs[(size_t)(readIndex + k)] : '\0';
        cur += indelLength;
    }
    // size_t arithmetic of the reference: refSeq.size() - refIndex > alt.size() - currentPos
    if ((uint64_t)(rsz - ri) > (uint64_t)(altsz - cur)) return std::string();
    if (ri < rsz) memcpy(&alt[(size_t)cur], ref.data() + ri, (size_t)(rsz - ri));
    ok = true;
    return alt;
}

static Cigar move_cigar_left(const Cigar &c, int idx) {  // AlignmentUtils::moveCigarLeft (:700-722)
    Cigar e;
    for (int i = 0; i < idx - 1; ++i) e.push_back(c[i]);
    CigOp ce = c[idx - 1];
    e.push_back({ce.t, ce.n - 1});
    e.push_back(c[idx]);
    if (idx + 1 < (int)c.size()) e.push_back({c[idx + 1].t, c[idx + 1].n + 1});
    else e.push_back({'M', 1});
    for (int i = idx + 2; i < (int)c.size(); ++i) e.push_back(c[i]);
    return e;
}

static Cigar clean_up_cigar(const Cigar &c) {  // AlignmentUtils::cleanUpCigar (:687-698)
    Cigar e;
    for (auto &x : c)
        if (x.n != 0 && (!e.empty() || x.t != 'D')) e.push_back(x);
    return e;
}

// AlignmentUtils::leftAlignIndel (:632-677)
static Cigar left_align_indel(Cigar cigar, const std::string &ref, const std::string &rs, int refIndex, int readIndex) {
    int idx = -1;
    for (int i = 0; i < (int)cigar.size(); ++i) {
        if (cigar[i].t == 'D' || cigar[i].t == 'I') {
            if (idx != -1) return cigar;
            idx = i;
        }
    }
    if (idx < 1) return cigar;
    const int indelLength = (int)cigar[idx].n;
    bool ok;
    std::string alt = create_indel_string(cigar, idx, ref, rs, refIndex, readIndex, ok);
    if (!ok || alt.empty()) return cigar;
    Cigar nc = cigar;
    for (int i = 0; i < indelLength; ++i) {
        nc = move_cigar_left(nc, idx);
        std::string na = create_indel_string(nc, idx, ref, rs, refIndex, readIndex, ok);
        bool reachedEnd = false;
        for (auto &x : nc)
            if (x.n == 0) reachedEnd = true;
        if (ok && alt == na) {
            cigar = nc;
            i = -1;
            if (reachedEnd) cigar = clean_up_cigar(cigar);
        }
        if (reachedEnd) break;
    }
    return cigar;
}

// =====================================================================================  AlignedRead
static inline bool is_regular(char b) {  // BaseUtils::isRegularBase (util/gatk/BaseUtils.h:49-57)
    return b == 'A' || b == 'C' || b == 'G' || b == 'T' || b == 'a' || b == 'c' || b == 'g' || b == 't' || b == '*';
}

// bytes of getUnclippedBases (:137-164) -- the M and I operations of the ORIGINAL cigar, each clipped
// to the read -- for the interval's arena
static size_t unclipped_len(const RRead &r) {
    size_t from = 0, n = 0;
    for (auto &ce : r.cigar) {
        if (ce.t == 'S') from += ce.n;
        else if (ce.t == 'M' || ce.t == 'I') {
            if (from < r.l_seq) n += std::min<size_t>(ce.n, r.l_seq - from);
            from += ce.n;
        }
    }
    return n;
}

struct AlignedRead {
    RRead *read;
    std::string_view bases, quals;  // getUnclippedBases (:137-164), in the interval's arena
    Cigar newCigar;
    int newStart = -1;
    int misRef = 0;
    long aligner = 0;

    // decodes the unclipped bases and their ASCII qualities into arena[0 .. 2 * unclipped_len(*r))
    AlignedRead(RRead *r, char *arena) : read(r) {
        const size_t n = unclipped_len(*r);
        char *b = arena, *q = arena + n;
        size_t from = 0, k = 0;
        for (auto &ce : r->cigar) {
            if (ce.t == 'S') from += ce.n;
            else if (ce.t == 'M' || ce.t == 'I') {
                if (from < r->l_seq) {
                    const size_t m = std::min<size_t>(ce.n, r->l_seq - from);
                    for (size_t j = 0; j < m; ++j, ++k) {
                        const size_t i = from + j;
                        b[k] = kSeqChars[((uint8_t)r->seq4[i >> 1] >> ((i & 1) ? 0 : 4)) & 15];
                        q[k] = (char)(r->qual[i] + 33);
                    }
                }
                from += ce.n;
            }
        }
        bases = std::string_view(b, n);
        quals = std::string_view(q, n);
    }
    int read_length() const { return bases.empty() ? (int)read->l_seq : (int)bases.size(); }
    const Cigar &cigar() const { return newCigar.empty() ? read->cigar : newCigar; }
    size_t cigar_length() const {  // getCigarLength (local_realignment.h:251-269)
        size_t len = 0;
        for (auto &c : cigar())
            if (!(c.t == 'H' || c.t == 'S' || c.t == 'D')) len += c.n;
        return len;
    }
    int alignment_start() const { return newStart != -1 ? newStart : read->pos; }
    // setCigar (:176-201)
    void set_cigar(const Cigar &in, bool fixClipped = true) {
        bool reclip = fixClipped && (int64_t)bases.size() < (int64_t)read->l_seq;
        Cigar c = reclip ? reclip_cigar(in, *read) : in;
        if (read->cigar == c) {
            newCigar.clear();
            return;
        }
        newCigar = c;
    }
};

// mismatchQualitySumIgnoreCigar (:641-679) with quit = INT_MAX (the raw mismatch score)
static int mismatch_sum_ignore_cigar(const AlignedRead &a, const std::string &ref, int refIndex) {
    const std::string_view rs = a.bases, q = a.quals;
    const int64_t L = (int64_t)rs.size(), R = (int64_t)ref.size();
    int sum = 0;
    for (int64_t i = 0; i < L; ++i) {
        int64_t k = refIndex + i;
        if (k >= R) {
            sum += 99;  // MAX_QUAL
            continue;
        }
        if (k < 0) continue;  // not reachable for reads inside their bin (Q26: defined behaviour)
        char rc = ref[(size_t)k], bc = rs[(size_t)i];
        if (!is_regular(bc) || !is_regular(rc)) continue;
        if (bc != rc) sum += (int)(signed char)q[(size_t)i] - 33;
    }
    return sum;
}

// AlignmentUtils::getMismatchCount (AlignmentUtils.cpp:58-108), mismatchQualities only
static long mismatching_qualities(const RRead &r, const std::string &ref, int refIndex) {
    long mq = 0;
    int readIdx = 0;
    const int endOnRead = (int)r.l_seq - 1;
    // bases and ASCII qualities read in place (the packed base's character, the phred byte + 33 as a
    // signed char: what getQueryBases / getQualities would hold), no per-read strings
    const uint8_t *s4 = (const uint8_t *)r.seq4.data(), *qp = (const uint8_t *)r.qual.data();
    for (auto &ce : r.cigar) {
        if (readIdx > endOnRead) break;
        switch (ce.t) {
            case 'M':
                for (uint32_t j = 0; j < ce.n; ++j, ++refIndex, ++readIdx) {
                    if (refIndex < 0 || refIndex >= (int)ref.size()) continue;
                    if (readIdx > endOnRead) break;
                    const char b = kSeqChars[(s4[readIdx >> 1] >> ((readIdx & 1) ? 0 : 4)) & 15];
                    if (b != ref[refIndex]) mq += (int)(signed char)(char)(qp[readIdx] + 33) - 33;
                }
                break;
            case 'I': case 'S': readIdx += ce.n; break;
            case 'D': case 'N': refIndex += ce.n; break;
            default: break;  // H, P (and '='/'X', which the reference asserts on)
        }
    }
    return mq;
}

struct Consensus {
    std::string str;
    size_t hash = 0;  // of str (duplicate check)
    Cigar cigar;
    int pos = 0;
    long sum = 0;
    std::vector<std::pair<int, int>> readIndexes;
};

// createAlternateConsensus from a read (:1022-1088)
static bool create_consensus(int indexOnRef, const Cigar &c, const std::string &ref, std::string_view readStr, Consensus &out) {
    if (indexOnRef < 0) return false;
    if (c.size() == 1 && c[0].t == 'M') return false;
    std::string sb;
    sb.reserve(ref.size() + 64);
    sb.append(ref, 0, std::min<size_t>((size_t)indexOnRef, ref.size()));
    Cigar el;
    int indelCount = 0, altIdx = 0;
    int64_t refIdx = indexOnRef;
    bool ok = true;
    for (auto &ce : c) {
        const int64_t n = ce.n;
        switch (ce.t) {
            case 'D':
                refIdx += n;
                indelCount++;
                el.push_back(ce);
                break;
            case 'M':
                altIdx += (int)n;
                // fall through
            case 'N':
                if ((int64_t)ref.size() < refIdx + n) ok = false;
                else sb.append(ref, (size_t)refIdx, (size_t)n);
                refIdx += n;
                el.push_back({'M', (uint32_t)n});
                break;
            case 'I':
                for (int64_t j = 0; j < n; ++j) {
                    char b = (altIdx + j) < (int64_t)readStr.size() ? readStr[(size_t)(altIdx + j)] : '\0';
                    if (!is_regular(b)) {
                        ok = false;
                        break;
                    }
                    sb.push_back(b);
                }
                altIdx += (int)n;
                indelCount++;
                el.push_back(ce);
                break;
            default: break;
        }
    }
    if (!ok || indelCount != 1 || (int64_t)ref.size() < refIdx) return false;
    sb.append(ref, (size_t)refIdx, std::string::npos);
    out.str = sb;
    out.cigar = el;
    out.pos = indexOnRef;
    return true;
}

// updateRead (:1166-1272)
static bool update_read(const Cigar &alt, int altPosOnRef, int myPosOnAlt, AlignedRead &a, int leftmost) {
    Cigar rc;
    if (alt.size() == 1) {
        a.newStart = leftmost + myPosOnAlt;
        rc.push_back({'M', (uint32_t)a.read_length()});
        a.set_cigar(rc);
        return true;
    }
    CigOp e1 = alt[0], e2 = alt[1], indel{'M', 0};
    int lead = 0;
    if (e1.t == 'I') {
        indel = e1;
        if (e2.t != 'M') return false;
    } else {
        if (e1.t != 'M') return false;
        if (e2.t == 'I' || e2.t == 'D') indel = e2;
        else return false;
        lead = (int)e1.n;
    }
    const int endOfFirst = altPosOnRef + lead;
    bool saw = false;
    const int rl = a.read_length();
    if (myPosOnAlt < endOfFirst) {
        a.newStart = leftmost + myPosOnAlt;
        saw = true;
        if (myPosOnAlt + rl <= endOfFirst) {
            a.newCigar.clear();
            return true;
        }
        rc.push_back({'M', (uint32_t)(endOfFirst - myPosOnAlt)});
    }
    if (indel.t == 'I') {
        if (myPosOnAlt + rl < endOfFirst + (int)indel.n) {
            int partial = myPosOnAlt + rl - endOfFirst;
            if (!saw) partial = rl;
            rc.push_back({'I', (uint32_t)partial});
            a.set_cigar(rc);
            return true;
        }
        if (!saw && myPosOnAlt < endOfFirst + (int)indel.n) {
            a.newStart = leftmost + endOfFirst;
            rc.push_back({'I', (uint32_t)((int)indel.n - (myPosOnAlt - endOfFirst))});
            saw = true;
        } else if (saw) {
            rc.push_back(indel);
        }
    } else if (indel.t == 'D') {
        if (saw) rc.push_back(indel);
    }
    if (!saw) {
        a.newCigar.clear();
        return true;
    }
    int remaining = (int)a.bases.size();
    for (auto &ce : rc)
        if (ce.t != 'D') remaining -= (int)ce.n;
    if (remaining > 0) rc.push_back({'M', (uint32_t)remaining});
    a.set_cigar(rc);
    return true;
}

// alternateReducesEntropy (:1274-1391)
static bool reduces_entropy(const std::vector<AlignedRead> &reads, const std::string &ref, int leftmost,
                            double mismatchThreshold) {
    const size_t n = ref.size();
    std::vector<int> om(n, 0), cm(n, 0), to(n, 0), tc(n, 0);
    for (const AlignedRead &a : reads) {
        int blocks = 0;
        for (auto &c : a.read->cigar)
            if (c.t == 'M' || c.t == '=' || c.t == 'X') blocks++;
        if (blocks > 1) continue;
        int refIdx = a.read->pos - leftmost;
        const std::string_view rs = a.bases, q = a.quals;
        for (size_t j = 0; j < rs.size(); ++j, ++refIdx) {
            if (refIdx < 0 || refIdx >= (int)n) break;
            int w = (int)(signed char)q[j] - 33;
            to[refIdx] += w;
            if (rs[j] != ref[refIdx]) om[refIdx] += w;
        }
        refIdx = a.alignment_start() - leftmost;
        int altIdx = 0;
        for (auto &ce : a.cigar()) {
            switch (ce.t) {
                case 'M':
                    for (uint32_t k = 0; k < ce.n; ++k, ++refIdx, ++altIdx) {
                        if (refIdx < 0 || refIdx >= (int)n) break;
                        char qc = altIdx < (int)q.size() ? q[altIdx] : '\0';
                        char bc = altIdx < (int)rs.size() ? rs[altIdx] : '\0';
                        int w = (int)(signed char)qc - 33;
                        tc[refIdx] += w;
                        if (bc != ref[refIdx]) cm[refIdx] += w;
                    }
                    break;
                case 'I': altIdx += (int)ce.n; break;
                case 'D': refIdx += (int)ce.n; break;
                default: break;
            }
        }
    }
    int oc = 0, cc = 0;
    for (size_t i = 0; i < n; ++i) {
        if (cm[i] == om[i]) continue;
        if (om[i] > to[i] * mismatchThreshold) {
            oc++;
            if (tc[i] > 0 && ((double)cm[i] / (double)tc[i]) > ((double)om[i] / (double)to[i]) * (1.0 - 0.75)) cc++;
        } else if (cm[i] > tc[i] * mismatchThreshold) {
            cc++;
        }
    }
    return oc == 0 || cc < oc;
}

static inline bool bases_equal(char l, char r) {  // SequenceUtil::basesEqual (SequenceUtil.cpp:91-99)
    if (l == r) return true;
    if (l > 90) l -= 32;
    if (r > 90) r -= 32;
    return l == r;
}

// SequenceUtil::calculateSamNmTag / sumQualitiesOfMismatches (SequenceUtil.cpp:134-228) over the
// read's alignment blocks (getAlignmentBlocks :55-88).  UQ sums ASCII qualities (Q23).
static void nm_uq(const RRead &r, const std::string &ref, int leftmost, int *nm, int *uq) {
    // bases and ASCII qualities read in place (as in mismatching_qualities)
    const uint8_t *s4 = (const uint8_t *)r.seq4.data(), *qp = (const uint8_t *)r.qual.data();
    const int nseq = (int)r.l_seq, nq = (int)r.qual.size();
    int readBase = 0, refBase = r.pos - leftmost, mis = 0, qs = 0;
    auto refc = [&](int k) -> char { return (k >= 0 && k < (int)ref.size()) ? ref[k] : '\0'; };
    auto readc = [&](int k) -> char { return (k >= 0 && k < nseq) ? kSeqChars[(s4[k >> 1] >> ((k & 1) ? 0 : 4)) & 15] : '\0'; };
    for (auto &e : r.cigar) {
        switch (e.t) {
            case 'S': case 'I': readBase += (int)e.n; break;
            case 'N': case 'D': refBase += (int)e.n; break;
            case 'M': case '=': case 'X':
                for (uint32_t i = 0; i < e.n; ++i) {
                    const int k = readBase + (int)i;
                    if (!bases_equal(readc(k), refc(refBase + (int)i))) {
                        mis++;
                        qs += (int)(signed char)(k < nq ? (char)(qp[k] + 33) : 0);
                    }
                }
                readBase += (int)e.n;
                refBase += (int)e.n;
                break;
            default: break;
        }
    }
    int ind = 0;
    for (auto &e : r.cigar)
        if (e.t == 'I' || e.t == 'D') ind += (int)e.n;
    *nm = mis + ind;
    *uq = qs;
}

// =====================================================================================  phase data
struct IntervalData {
    int interval = -1;                   // index into the interval list, -1 = invalid (None)
    std::vector<RRead *> toClean, notToClean;
    GLoc binLoc;                          // ReadBin::loc before padding
    bool hasLoc = false;
    // phase B/D results
    std::string reference;
    int leftmost = 0;
    long totalRaw = 0;
    std::vector<AlignedRead> alt;        // altReads, bases / qualities in `arena`
    std::vector<char> arena;
    std::vector<Consensus> cons;
    uint64_t pairBase = 0;
    std::vector<std::pair<RRead *, RRead>> pending;  // read -> updated copy (applied in phase E)
    bool cleanable = false;
    // back to a fresh interval, keeping the containers' capacity (the objects are reused across calls)
    void reset(int iv) {
        interval = iv;
        toClean.clear(), notToClean.clear();
        binLoc = GLoc();
        hasLoc = false;
        reference.clear();
        leftmost = 0;
        totalRaw = 0;
        alt.clear(), arena.clear(), cons.clear(), pending.clear();
        pairBase = 0;
        cleanable = false;
    }
};

enum EvType { EV_READ, EV_CLEAN, EV_LIST };
struct Event {
    EvType t;
    RRead *read;
    IntervalData *id;
};

struct ByPos {  // Sort::ByPosition (util/bamtools/Sort.h:116-133); idx stands in for the address (Q10)
    bool operator()(const RRead *a, const RRead *b) const {
        if (a->ref == -1) return false;
        if (b->ref == -1) return true;
        if (a->ref != b->ref) return a->ref < b->ref;
        if (a->pos != b->pos) return a->pos < b->pos;
        if (a->rev() != b->rev()) return !a->rev();
        if (a->name != b->name) return a->name < b->name;
        if (a->flag != b->flag) return a->flag < b->flag;
        return a->idx < b->idx;
    }
};

// =====================================================================================  phase E
// The writer's waitingReads multiset (ConstrainedMateFixingManager.h:94) as a binary heap.  Entries
// the comparator calls equivalent (only unmapped refID -1 reads; everything else is ordered down to
// idx) leave in insertion order, as they would from the multiset's upper-bound inserts.  The
// (refID, pos, strand) part of the comparison is cached in `key`; none of those fields changes
// while a read waits (setMateInfo moves an unmapped read only after the requeue erase).
class WaitQueue {
public:
    bool empty() const { return h_.empty(); }
    size_t size() const { return h_.size(); }
    RRead *top() const { return h_.front().r; }
    void insert(RRead *r) {
        h_.push_back({key(*r), seq_++, r});
        std::push_heap(h_.begin(), h_.end(), After());
    }
    RRead *pop() {
        std::pop_heap(h_.begin(), h_.end(), After());
        RRead *r = h_.back().r;
        h_.pop_back();
        return r;
    }
    // multiset::count / erase by key: every entry equivalent to r under ByPosition
    size_t count(const RRead *r) const {
        const uint64_t k = key(*r);
        size_t c = 0;
        for (auto &e : h_) c += equivalent(e, k, r);
        return c;
    }
    size_t erase(const RRead *r) {
        const uint64_t k = key(*r);
        size_t before = h_.size();
        h_.erase(std::remove_if(h_.begin(), h_.end(), [&](const Entry &e) { return equivalent(e, k, r); }), h_.end());
        if (h_.size() != before) std::make_heap(h_.begin(), h_.end(), After());
        return before - h_.size();
    }

private:
    struct Entry {
        uint64_t key, seq;
        RRead *r;
    };
    // Sort::ByPosition (util/bamtools/Sort.h:116-133): refID -1 sorts last and ties with itself
    static uint64_t key(const RRead &r) {
        if (r.ref == -1) return ~0ull;
        return ((uint64_t)(uint32_t)r.ref << 33) | ((uint64_t)(uint32_t)(r.pos + 1) << 1) | (r.rev() ? 1u : 0u);
    }
    static int tail_cmp(const RRead &a, const RRead &b) {  // name, flag, idx (Q10)
        int c = a.name.compare(b.name);
        if (c) return c;
        if (a.flag != b.flag) return a.flag < b.flag ? -1 : 1;
        if (a.idx != b.idx) return a.idx < b.idx ? -1 : 1;
        return 0;
    }
    static bool equivalent(const Entry &e, uint64_t k, const RRead *r) {
        return e.key == k && (k == ~0ull || tail_cmp(*e.r, *r) == 0);
    }
    struct After {  // heap order: true when a leaves after b
        bool operator()(const Entry &a, const Entry &b) const {
            if (a.key != b.key) return a.key > b.key;
            if (a.key != ~0ull) {
                int c = tail_cmp(*a.r, *b.r);
                if (c) return c > 0;
            }
            return a.seq > b.seq;
        }
    };
    std::vector<Entry> h_;
    uint64_t seq_ = 0;
};

// The writer's forMateMatching map (read name -> read, modified) as an open-addressing table keyed
// on the precomputed name hash; removal shifts the probe run back (no tombstones).
class MateTable {
public:
    struct Slot {
        RRead *r;
        bool modified;
    };
    MateTable() { t_.assign(1024, Slot{nullptr, false}); }
    Slot *find(const RRead *k) {
        for (size_t i = k->name_hash & mask(); t_[i].r; i = (i + 1) & mask())
            if (t_[i].r->name_hash == k->name_hash && t_[i].r->name == k->name) return &t_[i];
        return nullptr;
    }
    void insert(RRead *r, bool modified) {  // caller checked find() == nullptr
        if (2 * (n_ + 1) > t_.size()) grow();
        size_t i = r->name_hash & mask();
        while (t_[i].r) i = (i + 1) & mask();
        t_[i] = Slot{r, modified};
        n_++;
    }
    void erase(Slot *s) {
        size_t i = (size_t)(s - t_.data());
        t_[i].r = nullptr;
        n_--;
        for (size_t j = (i + 1) & mask(); t_[j].r; j = (j + 1) & mask()) {
            const size_t home = t_[j].r->name_hash & mask();
            // move j back into the hole at i when its home is not in the cyclic range (i, j]
            if ((j > i && (home <= i || home > j)) || (j < i && (home <= i && home > j))) {
                t_[i] = t_[j];
                t_[j].r = nullptr;
                i = j;
            }
        }
    }
    void erase_name(const RRead *k) {
        if (Slot *s = find(k)) erase(s);
    }
    void clear() {
        if (n_) std::fill(t_.begin(), t_.end(), Slot{nullptr, false});
        n_ = 0;
    }
    void purge_unmodified() {
        std::vector<Slot> keep;
        for (auto &s : t_)
            if (s.r && s.modified) keep.push_back(s);
        clear();
        for (auto &s : keep) insert(s.r, s.modified);
    }

private:
    size_t mask() const { return t_.size() - 1; }
    void grow() {
        std::vector<Slot> old;
        old.swap(t_);
        t_.assign(old.size() * 2, Slot{nullptr, false});
        n_ = 0;
        for (auto &s : old)
            if (s.r) insert(s.r, s.modified);
    }
    std::vector<Slot> t_;
    size_t n_ = 0;
};

// ConstrainedMateFixingManager (util/gatk/ConstrainedMateFixingManager.cpp), run in stream order.
class MateFixer {
public:
    // `counter` = reads added before this one's first (EMIT_FREQUENCY counts the whole stream)
    MateFixer(const RealignParams &P, BigVec<RRead *> &out, uint64_t counter = 0) : P_(P), out_(out), counter_(counter) {}
    size_t waiting() const { return waiting_.size(); }

    // canMoveReads (:245-251)
    bool can_move(const GLoc &earliest) const {
        return !hasLast_ || last_.contig != earliest.contig ||
               std::abs(last_.start - earliest.start) > P_.max_isize_for_movement;
    }

    void add(RRead *nr, bool modified, bool canFlush) {  // addReadInternal (:312-419)
        const bool tooMany = waiting_.size() >= (size_t)P_.max_records_in_memory;
        if ((canFlush && tooMany) || (!waiting_.empty() && waiting_.top()->ref != nr->ref)) {
            while (waiting_.size() > 1) write(pop());
            RRead *last = pop();
            if (last->ref == -1) {
                hasLast_ = false;
            } else {
                hasLast_ = true;
                last_ = read_loc(*last);
            }
            write(last);
            if (!tooMany) mates_.clear();
            else purge_unmodified();
        }
        if (nr->paired()) {
            MateTable::Slot *it = mates_.find(nr);
            if (it) {
                RRead *mate = it->r;
                bool doNotFix = !nr->mapped() && (!mate->mapped() || !waiting_.count(mate));
                if (!doNotFix) {
                    bool requeue = !mate->mapped() && nr->mapped();
                    if (requeue && waiting_.erase(mate) == 0) requeue = false;
                    set_mate_info(*mate, *nr);
                    if (requeue) waiting_.insert(mate);
                }
                mates_.erase(it);
            } else if (movable(*nr)) {
                mates_.insert(nr, modified);
            }
        }
        waiting_.insert(nr);
        if (++counter_ % 1000 == 0) {  // EMIT_FREQUENCY (ConstrainedMateFixingManager.h:66)
            while (!waiting_.empty()) {
                RRead *r = waiting_.top();
                if (cannot_move_before(r->pos, *nr) && (!movable(*r) || cannot_move_before(r->mpos, *nr))) {
                    mates_.erase_name(r);
                    write(pop());
                } else {
                    break;
                }
            }
        }
    }

    void close() {
        while (!waiting_.empty()) write(pop());
    }

private:
    bool cannot_move_before(int pos, const RRead &added) const {  // noReadCanMoveBefore (:253-255)
        return pos + 2 * P_.max_pos_move_allowed < added.pos;
    }
    bool too_big(const RRead &r) const {  // iSizeTooBigToMove (:433-436): query length used as isize (Q22)
        return (r.paired() && r.mapped() && r.ref != r.mref) || std::abs((int)r.l_seq) > P_.max_isize_for_movement;
    }
    bool movable(const RRead &r) const {  // pairedReadIsMovable (:449-454)
        return r.paired() && (r.mapped() || r.mate_mapped()) && !too_big(r);
    }
    RRead *pop() { return waiting_.pop(); }
    void write(RRead *r) { out_.push_back(r); }
    void purge_unmodified() { mates_.purge_unmodified(); }
    static int end_position(const RRead &r) {  // getEndPosition (:100-120)
        int len = 0;
        for (auto &c : r.cigar)
            if (c.t == 'M' || c.t == 'D' || c.t == 'N' || c.t == '=' || c.t == 'X') len += (int)c.n;
        return r.pos + len - 1;
    }
    static int insert_size(const RRead &a, const RRead &b) {  // computeInsertSize (:125-141)
        if (!a.mapped() || !b.mapped()) return 0;
        if ((a.ref == 0 ? 1 : 0) == b.ref) return 0;  // `!firstEnd.getRefID() == secondEnd.getRefID()` (Q22)
        const int p1 = a.rev() ? end_position(a) : a.pos;
        const int p2 = b.rev() ? end_position(b) : b.pos;
        return p2 - p1 + ((p2 >= p1) ? 1 : -1);
    }
    static void set_flag(RRead &r, uint16_t bit, bool on) { r.flag = on ? (r.flag | bit) : (r.flag & ~bit); }
    // AddTag("MQ", "S", ...) deferred to encode (nothing edits tags after the mate fixer), so the
    // common case copies no tag bytes; RemoveTag("MQ") drops a pending one first.
    static void add_mq(RRead &r, uint16_t mq) {
        if (r.mq_add < 0 && !tag_find(r.tags(), "MQ", nullptr, nullptr)) r.mq_add = mq;
    }
    static void remove_mq(RRead &r) {
        if (r.mq_add >= 0) r.mq_add = -1;
        else if (tag_find(r.tags(), "MQ", nullptr, nullptr)) tag_remove(r.tags_mut(), "MQ");
    }
    static void set_mate_info(RRead &r1, RRead &r2) {  // setMateInfo (:143-201)
        if (r1.mapped() && r2.mapped()) {
            r1.mref = r2.mref;  // Q22: the mate's mate reference, not its reference
            r1.mpos = r2.pos;
            set_flag(r1, 0x20, r2.rev());
            set_flag(r1, 0x8, false);
            add_mq(r1, r2.mapq);
            r2.mref = r1.ref;
            r2.mpos = r1.pos;
            set_flag(r2, 0x20, r1.rev());
            set_flag(r2, 0x8, false);
            add_mq(r2, r1.mapq);
        } else if (!r1.mapped() && !r2.mapped()) {
            r1.ref = -1; r1.pos = -1; r1.mref = -1; r1.mpos = -1;
            set_flag(r1, 0x20, r2.rev());
            set_flag(r1, 0x8, true);
            remove_mq(r2);
            r2.ref = -1; r2.pos = -1; r2.mref = -1; r2.mpos = -1;
            set_flag(r2, 0x20, r1.rev());
            set_flag(r2, 0x8, false);
            remove_mq(r2);
        } else {
            RRead &m = r1.mapped() ? r1 : r2;
            RRead &u = r1.mapped() ? r2 : r1;
            u.ref = m.ref;
            u.pos = m.pos;
            m.mref = u.ref;
            m.mpos = u.pos;
            set_flag(m, 0x20, u.rev());
            set_flag(m, 0x8, true);
            u.mref = m.ref;
            u.mpos = m.pos;
            set_flag(u, 0x20, m.rev());
            set_flag(u, 0x8, false);
        }
        int is = insert_size(r1, r2);
        if (is > 0) is--;
        if (is < 0) is++;
        r1.tlen = is;
        r2.tlen = -is;
    }

    const RealignParams &P_;
    BigVec<RRead *> &out_;
    uint64_t counter_ = 0;
    WaitQueue waiting_;
    MateTable mates_;
    GLoc last_;
    bool hasLast_ = false;
};

// =====================================================================================  driver
static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// GenomeLocParser::parseGenomeLoc (GenomeLocParser.cpp:274-328): "contig:start[-stop]", 1-based.
static bool parse_intervals(const std::string &path, const std::vector<std::string> &names, std::vector<GLoc> &out,
                            std::string &err) {
    std::ifstream f(path);
    if (!f) {
        err = "cannot open intervals file " + path;
        return false;
    }
    std::unordered_map<std::string, int> idx;
    for (size_t i = 0; i < names.size(); ++i) idx[names[i]] = (int)i;
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty()) break;  // the reference stops at the first empty line (:326-331)
        size_t colon = line.find(':');
        if (colon == std::string::npos) {
            err = "Could not find colon in interval file: " + line;
            return false;
        }
        size_t hy = line.find('-');
        std::string contig = line.substr(0, std::min(colon, hy));
        GLoc g;
        g.start = (int)strtol(line.c_str() + colon + 1, nullptr, 10) - 1;
        g.stop = g.start;
        if (hy != std::string::npos) g.stop = (int)strtol(line.c_str() + hy + 1, nullptr, 10) - 1;
        auto it = idx.find(contig);
        if (it == idx.end()) {
            err = "Contig '" + contig + "' does not match any contig in the sequence dictionary";
            return false;
        }
        g.contig = it->second;
        out.push_back(g);
    }
    if (out.empty()) {
        err = "Error parsing intervals file. Aborting.";
        return false;
    }
    return true;
}

// doNotTryToClean (:555-575)
static bool do_not_clean(const RRead &r, const RealignParams &P) {
    std::string rg;
    bool is454 = tag_get_string(r.tags(), "RG", rg) && rg.find("454") != std::string::npos;
    bool tooBig = (r.paired() && r.mapped() && r.ref != r.mref) || std::abs((int)r.l_seq) > P.max_isize_for_movement;
    return !r.mapped() || (r.flag & 0x100) || (r.flag & 0x200) || r.mapq == 0 || r.pos == -1 || tooBig || is454;
}

// A worker pool and the run's large containers, kept across calls (taken from this cache and handed
// back at the end; concurrent calls each get their own).  r03 started and joined 16 threads per call
// (~20 ms on the GPU box), allocated the record array, the event list, the scan batch and 50k interval
// objects afresh -- first touch of every page -- and freed them at return (~0.15 s of destructors and
// munmap).  Reused containers are cleared, not freed: their capacity carries over.
struct Scratch {
    std::unique_ptr<Pool> pool;
    RRead *rmem = nullptr;  // the decoded records: [0, rlive) constructed and kept across calls (the decode
    uint64_t rcap = 0, rlive = 0;  // overwrites every field; cigar / owned-tag storage is reused)
    BigVec<int32_t> lstop;
    BigVec<uint8_t> dnc;
    std::vector<std::unique_ptr<IntervalData>> ids;
    BigVec<Event> ev;
    std::vector<IntervalData *> work;
    ScanBatch B;
    hvector<int32_t> bidx, bscore;
    BigVec<RRead *> order;
    std::vector<DevPrepBatch> DB;  // phase B on the devices: their inputs and results
    std::vector<DevPrepOut> DO;
    Fasta fa;
    ~Scratch() {
        for (uint64_t i = 0; i < rlive; ++i) rmem[i].~RRead();
        std::free(rmem);
    }
};
static std::mutex g_scratch_mu;
// never destroyed: no static destructor joins worker threads at exit (a forked child that exits
// through them would join threads it does not have)
static std::vector<std::unique_ptr<Scratch>> &g_scratch = *new std::vector<std::unique_ptr<Scratch>>();
struct ScratchLease {
    std::unique_ptr<Scratch> s;
    explicit ScratchLease(int threads) {
        if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
        {
            std::lock_guard<std::mutex> g(g_scratch_mu);
            for (auto it = g_scratch.begin(); it != g_scratch.end(); ++it)
                if ((*it)->pool->size() == threads) {
                    s = std::move(*it);
                    g_scratch.erase(it);
                    break;
                }
        }
        if (!s) {
            s.reset(new Scratch());
            s->pool.reset(new Pool(threads));
        }
    }
    ~ScratchLease() {
        std::lock_guard<std::mutex> g(g_scratch_mu);
        g_scratch.push_back(std::move(s));
    }
};

// per-worker busy seconds of a parallel phase: max and mean say how well its work is balanced
struct Busy {
    std::vector<double> t;
    explicit Busy(int threads) : t((size_t)std::max(threads, 1), 0.0) {}
    void add(size_t, double s) { t[(size_t)tl_worker % t.size()] += s; }  // each worker only touches its own slot
    void report(RealignStats &st, const char *name) const {
        double mx = 0, sum = 0;
        for (double x : t) mx = std::max(mx, x), sum += x;
        st.more.emplace_back(std::string(name) + "_busy_max", mx);
        st.more.emplace_back(std::string(name) + "_busy_avg", sum / (double)t.size());
    }
};

int realign_run(const std::vector<std::string> &ref_names, const uint8_t *recs, const uint64_t *offs, uint64_t n,
                const std::string &fasta_path, const std::string &intervals_path, const RealignParams &P, const ScanFn &scan,
                ByteBuf &out, std::vector<uint64_t> &out_off, RealignStats &st, std::string &err, const DevPrep *dev) {
    double t0 = now_s();
    ScratchLease lease(P.threads);
    Scratch &S = *lease.s;
    // phase B on the device: the record arena goes up now, beside the FASTA load, decode and binning
    uint64_t span_lo = 0;
    if (dev && n) {
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint64_t i = 0; i < n; ++i) lo = std::min(lo, offs[i]), hi = std::max(hi, offs[i]);
        hi += 4 + rd32(recs + hi);
        span_lo = lo;
        for (int g = 0; g < std::max(1, dev->ndev); ++g)
            if (dev->stage(g, recs, lo, hi)) {
                err = "device consensus generation: staging the records failed";
                return -1;
            }
    }
    Pool &pool = *S.pool;
    st.more.emplace_back("t_pool", now_s() - t0);
    Fasta &fa = S.fa;
    if (!fa.load(fasta_path, err, pool)) return -4;
    std::vector<GLoc> ivs;
    if (!parse_intervals(intervals_path, ref_names, ivs, err)) return -1;
    st.intervals = ivs.size();

    const double tf = now_s();
    // decoded records, constructed (first-touched) and destroyed by the worker threads
    const uint64_t dchunk = 4096;
    struct ReadArray {
        RRead *p;
        uint64_t n;
        Pool &pool;
        RRead &operator[](uint64_t i) { return p[i]; }
    };
    if (S.rcap < std::max<uint64_t>(n, 1)) {
        pool.run_chunks(S.rlive, dchunk, [&](size_t b, size_t e) {
            for (size_t i = b; i < e; ++i) S.rmem[i].~RRead();
        });
        S.rlive = 0;
        std::free(S.rmem);
        S.rcap = 0;
        S.rmem = (RRead *)big_alloc(std::max<uint64_t>(n, 1) * sizeof(RRead));
        if (!S.rmem) {
            err = "out of host memory for the decoded records";
            return -1;
        }
        S.rcap = std::max<uint64_t>(n, 1);
    }
    RRead *rmem = S.rmem;
    ReadArray reads{rmem, 0, pool};
    if (S.rlive < n) {
        const uint64_t r0 = S.rlive;
        pool.run_chunks(n - r0, dchunk, [&](size_t b, size_t e) {
            for (size_t i = r0 + b; i < r0 + e; ++i) new (&rmem[i]) RRead();
        });
        S.rlive = n;
    }
    reads.n = n;
    std::atomic<bool> bad(false);
    std::mutex emu;
    std::string derr;
    // decode, plus what binning asks of every read (its GenomeLoc stop, doNotTryToClean), on the workers in
    // 4096-read chunks; the calling thread bins the reads in order beside them, waiting for each chunk (r06:
    // the binning walk was a serial 0.05 s after the decode)
    BigVec<int32_t> &lstop = S.lstop;  // (every entry written by the decode below)
    BigVec<uint8_t> &dnc = S.dnc;
    lstop.resize(n);
    dnc.resize(n);
    const uint64_t ndch = (n + dchunk - 1) / dchunk;
    std::unique_ptr<std::atomic<uint8_t>[]> cdone(new std::atomic<uint8_t>[ndch ? ndch : 1]);
    for (uint64_t c = 0; c < ndch; ++c) cdone[c].store(0, std::memory_order_relaxed);
    auto decode_chunk = [&](size_t c) {
        std::string e;
        const size_t b = c * dchunk, end = std::min<size_t>(n, b + dchunk);
        for (size_t i = b; i < end; ++i) {
            if (!rread_decode(recs + offs[i], reads[i], e)) {
                std::lock_guard<std::mutex> g(emu);
                bad = true;
                derr = e;
                continue;
            }
            reads[i].idx = (uint32_t)i;
            lstop[i] = read_loc(reads[i]).stop;
            dnc[i] = do_not_clean(reads[i], P);
        }
        cdone[c].store(1, std::memory_order_release);
    };

    // ---------------------------------------------------------------- A: map_func (:455-553)
    std::vector<std::unique_ptr<IntervalData>> &ids = S.ids;  // objects reused across calls
    size_t nids = 0;
    BigVec<Event> &ev = S.ev;
    ev.clear();
    ev.reserve(n + 2 * ivs.size() + 16);  // a read is one event at most, an interval two (no regrowth copies)
    auto new_id = [&](int interval) {
        if (nids == ids.size()) ids.emplace_back(new IntervalData());
        IntervalData *d = ids[nids++].get();
        d->reset(interval);
        return d;
    };
    size_t it = 0;
    IntervalData *loading = new_id(ivs.empty() ? -1 : 0);
    bool saw = false;
    auto bin_add = [&](IntervalData *d, RRead *r, const GLoc &l) {  // ReadBin::add (:263-275)
        if (!d->hasLoc) {
            d->binLoc = l;
            d->hasLoc = true;
        } else if (l.stop > d->binLoc.stop) {
            d->binLoc.stop = l.stop;
        }
        d->toClean.push_back(r);
    };
    // map_func; `continue` re-dispatches the read after the loading bin changed (the reference's
    // recursive calls).  Once the intervals are exhausted every read passes straight through (a bin
    // of its own in the reference, which emits it unchanged).
    bool badref = false;
    auto bin_all = [&]() {
        for (uint64_t i = 0; i < n; ++i) {
            if (i % dchunk == 0) {
                const uint64_t c = i / dchunk;
                while (!cdone[c].load(std::memory_order_acquire)) std::this_thread::yield();
                if (bad.load(std::memory_order_relaxed)) return;  // a record that does not decode: reported below
            }
            RRead *r = &reads[i];
            if (r->ref < -1 || r->ref >= (int)ref_names.size()) {
                badref = true;
                return;
            }
            for (;;) {
                if (loading->interval < 0) {
                    ev.push_back({EV_READ, r, loading});
                    break;
                }
                if (r->ref == -1) {
                    ev.push_back({EV_CLEAN, nullptr, loading});
                    it = ivs.size();
                    loading = new_id(-1);
                    saw = false;
                    continue;
                }
                GLoc loc;
                loc.contig = r->ref;
                loc.start = r->pos;
                loc.stop = lstop[i];
                GLoc rl = loc;
                if (rl.stop == 0) rl.stop = rl.start;
                const GLoc &cur = ivs[loading->interval];
                if (rl.is_before(cur)) {
                    if (!saw) ev.push_back({EV_READ, r, loading});
                    else loading->notToClean.push_back(r);
                } else if (rl.overlaps(cur)) {
                    saw = true;
                    if (dnc[i]) loading->notToClean.push_back(r);
                    else bin_add(loading, r, loc);
                    if ((int)(loading->toClean.size() + loading->notToClean.size()) >= P.max_reads) {
                        ev.push_back({EV_LIST, nullptr, loading});
                        ++it;
                        loading = new_id(it < ivs.size() ? (int)it : -1);
                        saw = false;
                    }
                } else {
                    ev.push_back({EV_CLEAN, nullptr, loading});
                    do {
                        ++it;
                    } while (it < ivs.size() && ivs[it].is_before(rl));
                    loading = new_id(it < ivs.size() ? (int)it : -1);
                    saw = false;
                    continue;
                }
                break;
            }
        }
    };
    pool.run_lead(ndch, decode_chunk, bin_all);
    if (bad) {  // (a decode error first, as when the whole input was decoded before the binning)
        err = derr;
        return -1;
    }
    if (badref) {
        err = "record refID outside the sequence dictionary";
        return -1;
    }
    const double td = now_s();
    st.t_fasta = tf - t0;
    st.t_decode = td - tf;  // decode and binning, side by side
    // onTraversalDone (:577-607)
    if (!loading->toClean.empty()) ev.push_back({EV_CLEAN, nullptr, loading});
    else if (!loading->notToClean.empty()) ev.push_back({EV_LIST, nullptr, loading});
    double t1 = now_s();
    st.t_bin = t1 - t0;

    // ---------------------------------------------------------------- B: prepare (:681-700, :918-999)
    std::vector<IntervalData *> &work = S.work;
    work.clear();
    for (auto &e : ev)
        if (e.t == EV_CLEAN && !e.id->toClean.empty()) work.push_back(e.id);
    const size_t nw = work.size();
    std::atomic<bool> ferr(false);
    std::string fmsg;
    // B.1 every interval's reference window: ReadBin::getReference (:277-293): pad 30, clamp, upper-case
    pool.run(nw, [&](size_t w) {
        IntervalData &d = *work[w];
        const std::string &contig = ref_names[d.binLoc.contig];
        const std::string *seq = fa.get(contig);
        int padLeft = std::max(d.binLoc.start - 30, 0);
        int padRight = seq ? std::min(d.binLoc.stop + 30, (int)seq->size() - 1) : -1;
        if (!seq || padRight < padLeft) {
            std::lock_guard<std::mutex> g(emu);
            ferr = true;
            fmsg = seq ? "Requested FASTA read beyond end of sequence " + contig : "Sequence " + contig + " not found in FASTA";
            return;
        }
        d.reference = seq->substr((size_t)padLeft, (size_t)(padRight - padLeft + 1));
        for (auto &c : d.reference) c = (char)toupper((unsigned char)c);
        d.leftmost = padLeft;
    });
    if (ferr) {
        err = fmsg;
        return -4;
    }
    // B.2 on the device(s) (realign_prep.hip): every toClean read's left-alignment, sums and consensus, each
    // interval's consensus set, and the offset scan of its pairs; intervals a device hands back run on the
    // host.  With several devices, device g takes the g-th contiguous range of work intervals (balanced by
    // toClean reads) and the results are stitched in interval order.
    std::vector<uint8_t> on_host(nw, 1);
    std::vector<const DevPrepRead *> iv_reads(nw, nullptr);  // interval w's first read result
    std::vector<int64_t> iv_traw(nw, 0);
    std::vector<uint64_t> iv_pbase(nw, 0);
    hvector<int32_t> dev_bi, dev_bs;
    uint64_t n_dev_iv = 0, ndev_pairs = 0;
    const int G = dev ? std::max(1, dev->ndev) : 0;
    if (dev && nw) {
        const double tb0 = now_s();
        S.DB.resize((size_t)G);
        S.DO.resize((size_t)G);
        std::vector<uint64_t> pre(nw + 1, 0);
        for (size_t w = 0; w < nw; ++w) pre[w + 1] = pre[w] + work[w]->toClean.size();
        std::vector<size_t> cut((size_t)G + 1, nw);
        cut[0] = 0;
        for (int g = 1; g < G; ++g)
            cut[(size_t)g] = (size_t)(std::lower_bound(pre.begin(), pre.end(), pre[nw] * (uint64_t)g / (uint64_t)G) - pre.begin());
        for (int g = 1; g <= G; ++g) cut[(size_t)g] = std::max(std::min(cut[(size_t)g], nw), cut[(size_t)g - 1]);
        for (int g = 0; g < G; ++g) {
            DevPrepBatch &DB = S.DB[(size_t)g];
            const size_t w0 = cut[(size_t)g], w1 = cut[(size_t)g + 1], m = w1 - w0;
            DB.ref_off.resize(m + 1);
            DB.rd_off.resize(m + 1);
            DB.ref_off[0] = DB.rd_off[0] = 0;
            for (size_t k = 0; k < m; ++k) {
                DB.ref_off[k + 1] = DB.ref_off[k] + work[w0 + k]->reference.size();
                DB.rd_off[k + 1] = DB.rd_off[k] + work[w0 + k]->toClean.size();
            }
            DB.ref.resize(DB.ref_off[m]);
            DB.rec.resize(DB.rd_off[m]);
            DB.start.resize(DB.rd_off[m]);
        }
        pool.run_static(nw, [&](size_t w) {
            const int g = (int)(std::upper_bound(cut.begin(), cut.end(), w) - cut.begin()) - 1;
            DevPrepBatch &DB = S.DB[(size_t)g];
            const size_t k0 = w - cut[(size_t)g];
            const IntervalData &d = *work[w];
            memcpy(DB.ref.data() + DB.ref_off[k0], d.reference.data(), d.reference.size());
            uint64_t k = DB.rd_off[k0];
            for (RRead *r : d.toClean) {
                DB.rec[k] = offs[r->idx] - span_lo;
                DB.start[k] = r->pos - d.leftmost;
                ++k;
            }
        });
        const double tb1 = now_s();
        std::vector<int> rcs((size_t)G, 0);
        if (G == 1) {
            rcs[0] = dev->run(0, S.DB[0], S.DO[0]);
        } else {
            std::vector<std::thread> ts;
            for (int g = 0; g < G; ++g) ts.emplace_back([&, g]() { rcs[(size_t)g] = dev->run(g, S.DB[(size_t)g], S.DO[(size_t)g]); });
            for (auto &t : ts) t.join();
        }
        for (int g = 0; g < G; ++g)
            if (rcs[(size_t)g]) {
                err = "device consensus generation failed (device " + std::to_string(g) + ")";
                return -1;
            }
        for (int g = 0; g < G; ++g) {
            const DevPrepOut &O = S.DO[(size_t)g];
            const DevPrepBatch &DB = S.DB[(size_t)g];
            uint64_t niv = 0;
            for (size_t w = cut[(size_t)g]; w < cut[(size_t)g + 1]; ++w) {
                const size_t k = w - cut[(size_t)g];
                on_host[w] = O.iv_host[k];
                n_dev_iv += !on_host[w], niv += !on_host[w];
                iv_reads[w] = O.reads.data() + DB.rd_off[k];
                iv_traw[w] = O.iv_total_raw[k];
                iv_pbase[w] = ndev_pairs + O.iv_pair_base[k];
            }
            if (G == 1) {  // the one device's results taken as they are (their buffers come back next call)
                dev_bi.swap(S.DO[0].best_index);
                dev_bs.swap(S.DO[0].best_score);
            } else {
                dev_bi.insert(dev_bi.end(), O.best_index.begin(), O.best_index.end());
                dev_bs.insert(dev_bs.end(), O.best_score.begin(), O.best_score.end());
            }
            ndev_pairs += O.pairs;
            if (G > 1) {
                const std::string pfx = "prep_rank" + std::to_string(g) + "_";
                st.more.emplace_back(pfx + "intervals", (double)niv);
                st.more.emplace_back(pfx + "reads", (double)DB.rec.size());
                st.more.emplace_back(pfx + "pairs", (double)O.pairs);
            }
        }
        st.more.emplace_back("t_prep_batch", tb1 - tb0);
        st.more.emplace_back("t_prep_device", now_s() - tb1);
        double tk = 0;
        for (auto &O : S.DO) tk = std::max(tk, O.t_device);
        st.more.emplace_back("t_prep_device_kernels", tk);
    }
    st.more.emplace_back("prep_devices", (double)G);
    st.more.emplace_back("prep_device_intervals", (double)n_dev_iv);
    st.more.emplace_back("prep_host_intervals", (double)(nw - n_dev_iv));
    const double tb2 = now_s();
    std::vector<uint64_t> wops(nw, 0);
    Busy bprep(pool.size());
    pool.run(nw, [&](size_t w) {  // (dynamic: intervals differ in size)
        const double tb = now_s();
        struct Acc {
            Busy &b;
            size_t w;
            double t;
            ~Acc() { b.add(w, now_s() - t); }
        } acc{bprep, w, tb};
        IntervalData &d = *work[w];
        const std::string &ref = d.reference;
        if (!on_host[w]) {
            // the device's results: the altReads (their bases and qualities decoded here: phase D reads them),
            // their cigars and sums, and the consensuses it kept, rebuilt from their creating reads
            const DevPrepRead *o = iv_reads[w];
            const size_t nt = d.toClean.size();
            size_t abytes = 0;
            for (size_t k = 0; k < nt; ++k)
                if (o[k].flags & DP_ALT) abytes += 2 * (size_t)o[k].ul;
            d.arena.resize(abytes);
            char *ap = d.arena.data();
            d.totalRaw = iv_traw[w];
            for (size_t k = 0; k < nt; ++k) {
                if (!(o[k].flags & DP_ALT)) continue;
                RRead *r = d.toClean[k];
                AlignedRead a(r, ap);
                ap += 2 * a.bases.size();
                if (o[k].flags & DP_NEWCIG) {
                    a.newCigar.resize(o[k].n_ops);
                    for (uint32_t i = 0; i < o[k].n_ops; ++i) a.newCigar[i] = CigOp{kCigChars[o[k].ops[i] & 15], o[k].ops[i] >> 4};
                }
                a.misRef = o[k].raw;
                a.aligner = o[k].aligner;
                if (o[k].flags & DP_KEPT) {
                    Consensus c;
                    if (!create_consensus(r->pos - d.leftmost, a.cigar(), ref, a.bases, c)) {
                        std::lock_guard<std::mutex> g(emu);
                        ferr = true;
                        fmsg = "device consensus generation: a kept consensus the host does not reproduce";
                        return;
                    }
                    d.cons.push_back(std::move(c));
                }
                d.alt.push_back(std::move(a));
            }
            if (!d.cons.empty()) {
                d.pairBase = iv_pbase[w];
                uint64_t ops = 0;  // findBestOffset's algorithmic compares (#offsets x read length per pair)
                for (auto &c : d.cons)
                    for (auto &a : d.alt) {
                        const int orig = a.read->pos - d.leftmost, ms = (int)c.str.size() - (int)a.cigar_length();
                        ops += (uint64_t)std::max(std::max(orig, ms) + 1, 0) * a.bases.size();
                    }
                wops[w] = ops;
            }
            return;
        }
        size_t abytes = 0;
        for (RRead *r : d.toClean)
            if (!r->cigar.empty()) abytes += 2 * unclipped_len(*r);
        d.arena.resize(abytes);  // sized once: the altReads' views into it stay valid
        char *ap = d.arena.data();
        thread_local std::string rb;
        for (RRead *r : d.toClean) {
            if (r->cigar.empty()) continue;  // refReads
            AlignedRead a(r, ap);
            ap += 2 * a.bases.size();
            int blocks = 0;
            for (auto &c : r->cigar)
                if (c.t == 'M' || c.t == '=' || c.t == 'X') blocks++;
            if (blocks == 2) {
                bases_into(*r, rb);
                Cigar nc = left_align_indel(unclip_cigar(r->cigar), ref, rb, r->pos - d.leftmost, 0);
                a.set_cigar(nc, false);
            }
            const int startOnRef = r->pos - d.leftmost;
            const int raw = mismatch_sum_ignore_cigar(a, ref, startOnRef);
            if (raw > 0) {
                if (!r->dup()) d.totalRaw += raw;
                a.misRef = raw;
                a.aligner = mismatching_qualities(*r, ref, startOnRef);
                if (blocks == 2) {
                    Consensus c;
                    if (create_consensus(startOnRef, a.cigar(), ref, a.bases, c)) {
                        c.hash = std::hash<std::string>()(c.str);
                        bool exists = false;
                        for (auto &o : d.cons)
                            if (o.hash == c.hash && o.str == c.str) exists = true;
                        if (!exists) d.cons.push_back(std::move(c));
                    }
                }
                d.alt.push_back(std::move(a));
            }
        }
    });
    if (ferr) {
        err = fmsg;
        return -1;
    }
    double t2 = now_s();
    st.t_prepare = t2 - t1;
    st.more.emplace_back("t_prep_finish", t2 - tb2);
    bprep.report(st, "t_prepare");

    // ---------------------------------------------------------------- C: offset scan (GPU)
    // the device intervals' pairs were scanned by dev->run (scores first in bidx / bscore); the host
    // intervals' batch: per-interval extents, prefix sums, then a parallel fill
    ScanBatch &B = S.B;  // (resized below; every byte written)
    const uint64_t ndev = ndev_pairs;
    std::vector<uint64_t> xc(nw + 1, 0), xcb(nw + 1, 0), xr(nw + 1, 0), xrb(nw + 1, 0), xp(nw + 1, 0);
    for (size_t w = 0; w < nw; ++w) {
        const IntervalData &d = *work[w];
        uint64_t cb = 0, rb = 0;
        const bool on = !d.cons.empty() && on_host[w];
        if (on) {
            for (auto &c : d.cons) cb += c.str.size();
            for (auto &a : d.alt) rb += a.bases.size();
        }
        xc[w + 1] = xc[w] + (on ? d.cons.size() : 0);
        xcb[w + 1] = xcb[w] + cb;
        xr[w + 1] = xr[w] + (on ? d.alt.size() : 0);
        xrb[w + 1] = xrb[w] + rb;
        xp[w + 1] = xp[w] + (on ? (uint64_t)d.cons.size() * d.alt.size() : 0);
    }
    B.cons.resize(xcb[nw]);
    B.cons_off.resize(xc[nw] + 1);
    B.bases.resize(xrb[nw]);
    B.quals.resize(xrb[nw]);
    B.read_off.resize(xr[nw] + 1);
    B.pairs.resize(xp[nw]);
    B.cons_off[0] = 0;
    B.read_off[0] = 0;
    pool.run_static(nw, [&](size_t w) {
        IntervalData &d = *work[w];
        if (d.cons.empty() || !on_host[w]) return;
        d.pairBase = ndev + xp[w];
        uint64_t cb = xcb[w], ci0 = xc[w];
        for (size_t c = 0; c < d.cons.size(); ++c) {
            memcpy(B.cons.data() + cb, d.cons[c].str.data(), d.cons[c].str.size());
            cb += d.cons[c].str.size();
            B.cons_off[ci0 + c + 1] = cb;
        }
        uint64_t rb = xrb[w], ri0 = xr[w];
        for (size_t j = 0; j < d.alt.size(); ++j) {
            const AlignedRead &a = d.alt[j];
            memcpy(B.bases.data() + rb, a.bases.data(), a.bases.size());
            for (size_t k = 0; k < a.quals.size(); ++k) B.quals[rb + k] = (uint8_t)(a.quals[k] - 33);
            rb += a.bases.size();
            B.read_off[ri0 + j + 1] = rb;
        }
        uint64_t pi = xp[w], ops = 0;
        for (uint32_t c = 0; c < d.cons.size(); ++c) {
            const int consLen = (int)d.cons[c].str.size();
            for (uint32_t j = 0; j < d.alt.size(); ++j) {
                const AlignedRead &a = d.alt[j];
                ScanPair &sp = B.pairs[pi++];
                sp.cons = (uint32_t)(ci0 + c);
                sp.read = (uint32_t)(ri0 + j);
                sp.orig = a.read->pos - d.leftmost;
                sp.max_start = consLen - (int)a.cigar_length();
                const int offsets = std::max(sp.orig, sp.max_start) + 1;
                ops += (uint64_t)std::max(offsets, 0) * a.bases.size();
            }
        }
        wops[w] = ops;
    });
    for (uint64_t o : wops) st.scan_ops += o;
    st.scan_pairs = ndev + B.pairs.size();
    st.t_scan_build = now_s() - t2;
    hvector<int32_t> &bidx = S.bidx, &bscore = S.bscore;
    bidx.swap(dev_bi);
    bscore.swap(dev_bs);
    if (G == 1 && nw && !S.DO.empty()) {  // the previous call's buffers back to the device's result slot (capacity kept)
        S.DO[0].best_index.swap(dev_bi);
        S.DO[0].best_score.swap(dev_bs);
    }
    if (!B.pairs.empty()) {
        std::vector<int32_t> hi, hs;
        int rc = scan(B, hi, hs);
        if (rc) {
            err = "offset scan failed";
            return rc;
        }
        bidx.insert(bidx.end(), hi.begin(), hi.end());
        bscore.insert(bscore.end(), hs.begin(), hs.end());
    }
    double t3 = now_s();
    st.t_scan = t3 - t2;

    // ---------------------------------------------------------------- D: decide (:713-892)
    Busy bdec(pool.size());
    pool.run(work.size(), [&](size_t w) {
        struct Acc {
            Busy &b;
            size_t w;
            double t;
            ~Acc() { b.add(w, now_s() - t); }
        } acc{bdec, w, now_s()};
        IntervalData &d = *work[w];
        if (d.cons.empty()) return;
        Consensus *best = nullptr;
        uint64_t pi = d.pairBase;
        for (auto &c : d.cons) {  // deterministic consensus order (Q19: the reference shuffles)
            c.sum = 0;
            for (size_t j = 0; j < d.alt.size(); ++j, ++pi) {
                AlignedRead &a = d.alt[j];
                int my = bscore[pi];
                if (my > a.aligner || my >= a.misRef) my = a.misRef;
                else c.readIndexes.push_back(std::make_pair((int)j, (int)bidx[pi]));
                if (!a.read->dup()) c.sum += my;
            }
            if (!best || best->sum > c.sum) best = &c;  // first strictly smaller sum (:764)
        }
        const double improvement = best ? (double)(d.totalRaw - best->sum) / 10.0 : -1;
        if (!(improvement >= P.lod_threshold)) return;
        best->cigar = left_align_indel(best->cigar, d.reference, best->str, best->pos, best->pos);
        for (auto &ip : best->readIndexes)
            if (!update_read(best->cigar, best->pos, ip.second, d.alt[ip.first], d.leftmost)) return;
        if (!reduces_entropy(d.alt, d.reference, d.leftmost, P.mismatch_threshold)) return;
        std::string reference = d.reference;
        int leftmost = d.leftmost;
        const std::string &contig = ref_names[ivs[d.interval].contig];
        const std::string *fseq = fa.get(contig);
        for (auto &ip : best->readIndexes) {
            AlignedRead &a = d.alt[ip.first];
            // constizeUpdate (:218-241)
            if (a.newCigar.empty()) continue;
            RRead u = *a.read;
            int ns = a.newStart == -1 ? u.pos : a.newStart;
            if (a.newStart != -1 && std::abs(a.newStart - u.pos) > P.max_pos_move_allowed) continue;
            if (!P.no_original_alignment_tags) {
                tag_add_string(u.tags_mut(), "OC", cigar_to_string(u.cigar));
                if (ns != u.pos) tag_add_int(u.tags_mut(), "OP", 'i', u.pos + 1, 4);
            }
            u.cigar = a.newCigar;
            u.pos = ns;
            if (u.mapq != 255) u.mapq = (uint16_t)std::min((int)u.mapq + 10, 254);
            // reference refetch for the tag fix-ups (:864-872); the refetched bases keep their case
            int64_t needL = (int64_t)leftmost - u.pos;
            int64_t needR = (int64_t)u.pos + (int64_t)u.l_seq - leftmost - (int64_t)reference.size() + 1;
            int needed = (int)std::max(needL, needR);
            if (needed > 0 && fseq) {
                int padLeft = std::max(leftmost - needed, 1);
                int64_t padRight =
                    std::min<int64_t>((int64_t)leftmost + (int64_t)reference.size() + needed, (int64_t)fseq->size());
                reference = fseq->substr((size_t)padLeft, (size_t)std::max<int64_t>(0, padRight - padLeft));
                leftmost = padLeft;
            }
            int nm, uq;
            nm_uq(u, reference, leftmost, &nm, &uq);
            if (tag_find(u.tags(), "NM", nullptr, nullptr)) tag_edit_i32(u.tags_mut(), "NM", nm);
            if (tag_find(u.tags(), "UQ", nullptr, nullptr)) tag_edit_i32(u.tags_mut(), "UQ", uq);
            if (tag_find(u.tags(), "MD", nullptr, nullptr)) tag_remove(u.tags_mut(), "MD");
            d.pending.push_back(std::make_pair(a.read, std::move(u)));
        }
        d.cleanable = true;
    });
    double t4 = now_s();
    st.t_decide = t4 - t3;
    bdec.report(st, "t_decide");

    // ---------------------------------------------------------------- E: emit + mate fixing
    // The writer (ConstrainedMateFixingManager) flushes everything waiting and forgets its mate map
    // whenever a read of another contig arrives; the stream is never empty at that point (the last
    // read added is still waiting).  So per-contig segments of the event stream run independently,
    // each on its own writer whose EMIT_FREQUENCY counter starts where the stream's would be -- with
    // one exception: a flush that also finds >= maxRecordsInMemory reads waiting keeps the modified
    // mate entries.  A segment ending that way sends the whole phase to the sequential path.
    auto emit_events = [&](size_t e0, size_t e1, uint64_t add0, BigVec<RRead *> &ord, uint64_t &cl, uint64_t &rr) {
        MateFixer mf(P, ord, add0);
        for (size_t k = e0; k < e1; ++k) {
            const Event &e = ev[k];
            if (e.t == EV_READ) {
                mf.add(e.read, false, true);
                continue;
            }
            IntervalData &d = *e.id;
            if (e.t == EV_CLEAN && !d.toClean.empty()) {
                // CleanAndEmitReadList::runJob (:435-453): clean only if the writer allows moves here
                if (mf.can_move(read_loc(*d.toClean[0])) && d.cleanable) {
                    cl++;
                    for (auto &pu : d.pending) {
                        *pu.first = pu.second;  // a copy: the sequential fallback may apply it again
                        pu.first->cleaned = true;
                    }
                    rr += d.pending.size();
                }
            }
            // emitReadLists (:370-376)
            std::vector<RRead *> lst = d.notToClean;
            lst.insert(lst.end(), d.toClean.begin(), d.toClean.end());
            std::stable_sort(lst.begin(), lst.end(), ByPos());
            for (RRead *r : lst) mf.add(r, r->cleaned, false);
        }
        const size_t left = mf.waiting();
        mf.close();
        return left;
    };
    struct Seg {
        size_t e0, e1;
        uint64_t add0;
        BigVec<RRead *> ord;
        uint64_t cl = 0, rr = 0;
        size_t left = 0;
    };
    const double tm0 = now_s();
    std::vector<Seg> segs;
    bool mixed = false;
    {
        // each event's contig and record count, chunk by chunk on the workers (an interval's lists are
        // walked: a bin whose records span two contigs sends the phase to the sequential path); then a
        // segment starts at every event with records whose contig differs from the previous such event
        struct Cut {
            size_t k;
            int32_t ref;
            uint64_t adds;  // records of the chunk before event k
        };
        struct Part {
            std::vector<Cut> cuts;  // events with records whose contig differs from the chunk's previous one
            uint64_t adds = 0;
            bool mixed = false;
        };
        const size_t echunk = 16384, nch = (ev.size() + echunk - 1) / echunk;
        std::vector<Part> parts(nch);
        pool.run(nch, [&](size_t c) {
            Part &pt = parts[c];
            int32_t cur = INT32_MIN;
            for (size_t k = c * echunk, ke = std::min(ev.size(), k + echunk); k < ke; ++k) {
                const Event &e = ev[k];
                int32_t ref = INT32_MIN;
                uint64_t cnt = 0;
                if (e.t == EV_READ) {
                    ref = e.read->ref;
                    cnt = 1;
                } else {
                    const IntervalData &d = *e.id;
                    for (const auto *v : {&d.notToClean, &d.toClean})
                        for (RRead *r : *v) {
                            if (ref == INT32_MIN) ref = r->ref;
                            else if (r->ref != ref) pt.mixed = true;
                            cnt++;
                        }
                }
                if (cnt && ref != cur) {
                    pt.cuts.push_back(Cut{k, ref, pt.adds});
                    cur = ref;
                }
                pt.adds += cnt;
            }
        });
        uint64_t adds = 0;
        int32_t cur = INT32_MIN;
        for (auto &pt : parts) {
            mixed |= pt.mixed;
            for (auto &ct : pt.cuts) {
                if (ct.ref == cur) continue;  // (a chunk's first cut continues the previous chunk's contig)
                if (!segs.empty()) segs.back().e1 = ct.k;
                segs.push_back(Seg{segs.empty() ? 0 : ct.k, ev.size(), adds + ct.adds, {}, 0, 0, 0});
                cur = ct.ref;
            }
            adds += pt.adds;
        }
    }
    bool sequential = mixed || segs.size() <= 1 || P.mate_sequential;
    st.more.emplace_back("t_mate_build", now_s() - tm0);
    if (!sequential) {
        std::vector<double> segt(segs.size(), 0.0);
        std::vector<size_t> big(segs.size());  // the largest segments handed out first
        for (size_t k = 0; k < segs.size(); ++k) big[k] = k;
        auto recs_in = [&](size_t k) { return (k + 1 < segs.size() ? segs[k + 1].add0 : (uint64_t)n) - segs[k].add0; };
        std::stable_sort(big.begin(), big.end(), [&](size_t a, size_t b) { return recs_in(a) > recs_in(b); });
        pool.run(segs.size(), [&](size_t j) {
            const size_t k = big[j];
            const double ts = now_s();
            Seg &g = segs[k];
            g.left = emit_events(g.e0, g.e1, g.add0, g.ord, g.cl, g.rr);
            segt[k] = now_s() - ts;
        });
        double smax = 0, ssum = 0;
        for (double x : segt) smax = std::max(smax, x), ssum += x;
        st.more.emplace_back("t_mate_seg_max", smax);
        st.more.emplace_back("t_mate_seg_sum", ssum);
        for (size_t k = 0; k + 1 < segs.size(); ++k)
            if (segs[k].left >= (size_t)P.max_records_in_memory) sequential = true;
        if (sequential) {  // undo: fresh records, then the one-writer path
            pool.run_chunks(n, dchunk, [&](size_t b, size_t end) {
                std::string e;
                for (size_t i = b; i < end; ++i) rread_decode(recs + offs[i], reads[i], e);
            });
        }
    }
    BigVec<RRead *> &order = S.order;
    order.clear();
    if (sequential) {
        order.reserve(n);
        st.tail_waiting = emit_events(0, ev.size(), 0, order, st.intervals_cleaned, st.reads_realigned);
    } else {  // the segments' orders side by side (copied by the workers)
        const double tc = now_s();
        std::vector<size_t> at(segs.size() + 1, 0);
        for (size_t k = 0; k < segs.size(); ++k) {
            at[k + 1] = at[k] + segs[k].ord.size();
            st.intervals_cleaned += segs[k].cl;
            st.reads_realigned += segs[k].rr;
        }
        st.tail_waiting = segs.back().left;
        order.resize(at.back());
        pool.run(segs.size(), [&](size_t k) {
            std::copy(segs[k].ord.begin(), segs[k].ord.end(), order.begin() + (ptrdiff_t)at[k]);
            BigVec<RRead *>().swap(segs[k].ord);
        });
        st.more.emplace_back("t_mate_concat", now_s() - tc);
    }
    st.mate_segments = sequential ? 1 : segs.size();
    st.t_mate = now_s() - t4;
    if (order.size() != n) {
        err = "internal: emitted " + std::to_string(order.size()) + " of " + std::to_string(n) + " records";
        return -1;
    }
    // output offsets: sizes and per-chunk sums in parallel, the chunk prefix serially, then the adds
    const uint64_t chunk = 4096;
    out_off.assign(n + 1, 0);
    const uint64_t nch = (n + chunk - 1) / chunk;
    std::vector<uint64_t> csum(nch + 1, 0);
    pool.run_chunks(n, chunk, [&](size_t b, size_t e) {
        uint64_t s = 0;
        for (size_t i = b; i < e; ++i) s += (out_off[i + 1] = rread_encoded_size(*order[i]));
        csum[b / chunk + 1] = s;
    });
    for (uint64_t c = 0; c < nch; ++c) csum[c + 1] += csum[c];
    pool.run_chunks(n, chunk, [&](size_t b, size_t e) {
        uint64_t run = csum[b / chunk];
        for (size_t i = b; i < e; ++i) run = (out_off[i + 1] += run);
    });
    if (!out.alloc(out_off[n])) {
        err = "out of host memory for the output records";
        return -1;
    }
    {  // fresh pages for ~1 GB of output: 2 MiB pages where the kernel allows them (512x fewer faults
       // in the parallel encode below)
        const uintptr_t a = ((uintptr_t)out.data() + (2ull << 20) - 1) & ~(uintptr_t)((2ull << 20) - 1);
        const uintptr_t e = ((uintptr_t)out.data() + out_off[n]) & ~(uintptr_t)((2ull << 20) - 1);
        if (e > a) madvise((void *)a, e - a, MADV_HUGEPAGE);
    }
    pool.run_chunks(n, chunk, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) rread_encode_to(*order[i], out.data() + out_off[i]);
    });
    st.t_emit = now_s() - t4;
    const double t5 = now_s();
    st.more.emplace_back("t_encode", t5 - t4 - st.t_mate);
    // teardown: the intervals reset on the workers (their containers keep their capacity for the next
    // call); the records and the large containers stay with the scratch (see Scratch)
    pool.run(nids, [&](size_t k) { ids[k]->reset(-1); });
    const double t6 = now_s();
    for (auto &g : segs) BigVec<RRead *>().swap(g.ord);
    st.t_release = now_s() - t5;
    st.more.emplace_back("t_release_intervals", t6 - t5);
    st.more.emplace_back("t_release_reads", now_s() - t6);
    st.more.emplace_back("t_at_return", now_s() - t0);  // t_run minus this: the locals' destructors
    return 0;
}

}  // namespace oge
