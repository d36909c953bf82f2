// bamio.cpp -- host BGZF/BAM codec (see bamio.h for the reference interfaces replaced).
#include "bamio.h"

#include <dlfcn.h>
#include <zlib.h>
#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <unistd.h>
#include <sys/mman.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <cstring>
#include <sstream>
#include <thread>

namespace oge {

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

template <class F>
static void parallel_for(size_t n, int threads, F f) {
    if (threads <= 1 || n < 2) { for (size_t i = 0; i < n; ++i) f(i); return; }
    std::atomic<size_t> next(0);
    std::vector<std::thread> ts;
    int t = (int)std::min<size_t>((size_t)threads, n);
    for (int k = 0; k < t; ++k)
        ts.emplace_back([&]() {
            for (;;) {
                size_t i = next.fetch_add(1);
                if (i >= n) break;
                f(i);
            }
        });
    for (auto &th : ts) th.join();
}

// ---------------- DEFLATE engine ----------------
// libdeflate (the image's libdeflate.so.0, loaded at run time) when present: 2-3x zlib's speed for
// both directions.  Compressed bytes are not part of parity, records are.
// OGE_BGZF_CODEC=zlib forces zlib.
struct LibDeflate {
    bool ok = false;
    void *(*alloc_c)(int) = nullptr;
    size_t (*compress)(void *, const void *, size_t, void *, size_t) = nullptr;
    void (*free_c)(void *) = nullptr;
    void *(*alloc_d)() = nullptr;
    int (*decompress)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    void (*free_d)(void *) = nullptr;
    uint32_t (*crc32)(uint32_t, const void *, size_t) = nullptr;
};

static const LibDeflate &libdeflate() {
    static LibDeflate L = [] {
        LibDeflate l;
        const char *env = getenv("OGE_BGZF_CODEC");
        if (env && std::string(env) == "zlib") return l;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return l;
        l.alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
        l.compress = (size_t(*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_deflate_compress");
        l.free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
        l.alloc_d = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        l.decompress = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_deflate_decompress");
        l.free_d = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        l.crc32 = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
        l.ok = l.alloc_c && l.compress && l.free_c && l.alloc_d && l.decompress && l.free_d && l.crc32;
        return l;
    }();
    return L;
}

static uint32_t block_crc(const uint8_t *p, size_t n) {
    const LibDeflate &L = libdeflate();
    return L.ok ? L.crc32(0, p, n) : (uint32_t)crc32(0L, p, (uInt)n);
}

// thread-local libdeflate handles (allocation is not free; one per worker thread and level)
struct DeflateTls {
    void *comp[10] = {nullptr};
    void *decomp = nullptr;
    ~DeflateTls() {
        const LibDeflate &L = libdeflate();
        if (!L.ok) return;
        for (void *c : comp)
            if (c) L.free_c(c);
        if (decomp) L.free_d(decomp);
    }
};
static thread_local DeflateTls tls_deflate;

const char *bgzf_codec_name() { return libdeflate().ok ? "libdeflate" : "zlib"; }

bool bgzf_host_codec_forced() {
    const char *env = getenv("OGE_BGZF_CODEC");
    return env && (std::string(env) == "zlib" || std::string(env) == "libdeflate");
}

// Large fresh buffers: ask for transparent huge pages before the first touch (a 5.7 GB stream is
// 1.4M 4-KiB page faults otherwise, which serialise in the kernel).
void want_huge_pages(void *p, size_t n) {
    if (n < (64ull << 20)) return;
    const uintptr_t a = ((uintptr_t)p + (2ull << 20) - 1) & ~(uintptr_t)((2ull << 20) - 1);
    const uintptr_t e = ((uintptr_t)p + n) & ~(uintptr_t)((2ull << 20) - 1);
    if (e > a) madvise((void *)a, e - a, MADV_HUGEPAGE);
}

// ---------------- BGZF inflate ----------------
bool bgzf_inflate_all(const uint8_t *src, size_t n, bytevec &out, int threads, std::string &err, size_t slack) {
    struct Blk { size_t coff, clen, cdata, dlen, uoff; };
    std::vector<Blk> blocks;
    size_t p = 0, total = 0;
    while (p < n) {
        if (n - p < 18 || src[p] != 31 || src[p + 1] != 139 || src[p + 2] != 8 || !(src[p + 3] & 4)) {
            err = "not a BGZF stream or truncated block header";
            return false;
        }
        uint16_t xlen = rd16(src + p + 10);
        size_t x = p + 12, xend = x + xlen, bsize = 0;
        if (xend > n) { err = "truncated BGZF extra field"; return false; }
        while (x + 4 <= xend) {
            uint16_t slen = rd16(src + x + 2);
            if (src[x] == 'B' && src[x + 1] == 'C' && slen == 2) bsize = (size_t)rd16(src + x + 4) + 1;
            x += 4 + slen;
        }
        if (!bsize) { err = "BGZF block without BC field"; return false; }
        if (p + bsize > n) { err = "truncated BGZF block (file cut short?)"; return false; }
        size_t cdata = xend;
        uint32_t isize = rd32(src + p + bsize - 4);
        blocks.push_back({p, bsize, cdata, isize, total});
        total += isize;
        p += bsize;
    }
    out.reserve(total + slack);
    want_huge_pages(out.data(), total + slack);
    out.resize(total + slack);
    memset(out.data() + total, 0, slack);
    out.resize(total);  // capacity keeps the zeroed slack
    std::atomic<bool> ok(true);
    parallel_for(blocks.size(), threads, [&](size_t i) {
        const Blk &b = blocks[i];
        if (b.dlen == 0) return;
        const LibDeflate &LD = libdeflate();
        if (LD.ok) {
            if (!tls_deflate.decomp) tls_deflate.decomp = LD.alloc_d();
            size_t got = 0;
            int rc = LD.decompress(tls_deflate.decomp, src + b.cdata, b.coff + b.clen - 8 - b.cdata, out.data() + b.uoff,
                                   b.dlen, &got);
            if (rc != 0 || got != b.dlen || block_crc(out.data() + b.uoff, b.dlen) != rd32(src + b.coff + b.clen - 8))
                ok = false;
            return;
        }
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (inflateInit2(&zs, -15) != Z_OK) { ok = false; return; }
        zs.next_in = (Bytef *)(src + b.cdata);
        zs.avail_in = (uInt)(b.coff + b.clen - 8 - b.cdata);
        zs.next_out = (Bytef *)(out.data() + b.uoff);
        zs.avail_out = (uInt)b.dlen;
        int rc = inflate(&zs, Z_FINISH);
        if (rc != Z_STREAM_END || zs.total_out != b.dlen) ok = false;
        else {
            uint32_t crc = (uint32_t)crc32(0L, out.data() + b.uoff, (uInt)b.dlen);
            if (crc != rd32(src + b.coff + b.clen - 8)) ok = false;
        }
        inflateEnd(&zs);
    });
    if (!ok) { err = "BGZF block failed to inflate (corrupt data)"; return false; }
    return true;
}

// ---------------- BGZF deflate ----------------
static const size_t kBlockPayload = 65280;

BgzfWriter::BgzfWriter(FILE *f, int level, int threads) : f_(f), level_(level), threads_(threads), closed_(false) {}
BgzfWriter::~BgzfWriter() {
    if (!closed_) close();
    drain();
}

void BgzfWriter::drain() {
    if (writer_.joinable()) writer_.join();
    writing_.clear();
}

void BgzfWriter::emit(std::vector<std::vector<uint8_t>> &&blocks) {
    drain();  // the previous batch goes out first
    writing_ = std::move(blocks);
    writer_ = std::thread([this]() {
        for (auto &o : writing_) put(o.data(), o.size());
    });
}

void BgzfWriter::put(const uint8_t *p, size_t n) {
    if (n && fwrite(p, 1, n, f_) != n) failed_ = true;
}

void BgzfWriter::abandon() {
    drain();
    pending_.clear();
    closed_ = true;
}

static void bgzf_block(const uint8_t *src, size_t n, int level, std::vector<uint8_t> &dst) {
    size_t bound = compressBound((uLong)n) + 64;
    dst.resize(18 + bound + 8);
    size_t clen = 0;
    const LibDeflate &LD = libdeflate();
    level = std::max(0, std::min(9, level));
    if (LD.ok) {
        if (!tls_deflate.comp[level]) tls_deflate.comp[level] = LD.alloc_c(level);
        clen = LD.compress(tls_deflate.comp[level], src, n, dst.data() + 18, bound);
    }
    if (!clen) {
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
        zs.next_in = (Bytef *)src;
        zs.avail_in = (uInt)n;
        zs.next_out = dst.data() + 18;
        zs.avail_out = (uInt)bound;
        deflate(&zs, Z_FINISH);
        clen = zs.total_out;
        deflateEnd(&zs);
    }
    size_t bsize = 18 + clen + 8;
    static const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0};
    memcpy(dst.data(), hdr, 16);
    dst[16] = (uint8_t)((bsize - 1) & 0xff);
    dst[17] = (uint8_t)((bsize - 1) >> 8);
    uint32_t crc = n ? block_crc(src, n) : 0;
    memcpy(dst.data() + 18 + clen, &crc, 4);
    uint32_t isz = (uint32_t)n;
    memcpy(dst.data() + 18 + clen + 4, &isz, 4);
    dst.resize(bsize);
}

const uint8_t kBgzfEof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

std::vector<uint8_t> bgzf_compress_host(const uint8_t *src, size_t n, int level) {
    std::vector<uint8_t> out, blk;
    for (size_t o = 0; o < n; o += kBlockPayload) {
        bgzf_block(src + o, std::min(kBlockPayload, n - o), level, blk);
        out.insert(out.end(), blk.begin(), blk.end());
    }
    return out;
}

void add_program_record(BamHeaderModel &h, const std::string &cl) {
    PgRecord pg;
    pg.id = "openge";
    auto has = [&](const std::string &id) {
        for (auto &p : h.pg)
            if (p.id == id) return true;
        return false;
    };
    for (int i = 2; has(pg.id); i++) pg.id = "openge-" + std::to_string(i);
    pg.vn = "0.3-dev";  // OPENGE_VERSION_STRING (oge/CMakeLists.txt:11-12)
    pg.cl = cl;
    h.pg.push_back(pg);
}

void BgzfWriter::write(const void *data, size_t n) {
    const uint8_t *p = (const uint8_t *)data;
    pending_.insert(pending_.end(), p, p + n);
    if (pending_.size() >= kBlockPayload * (size_t)std::max(1, threads_) * 64) flush_blocks(false);
}

void BgzfWriter::flush_blocks(bool final) {
    size_t nblk = pending_.size() / kBlockPayload;
    if (final && pending_.size() % kBlockPayload) nblk++;
    if (!nblk) return;
    std::vector<std::vector<uint8_t>> outs(nblk);
    parallel_for(nblk, threads_, [&](size_t i) {
        size_t off = i * kBlockPayload;
        size_t len = std::min(kBlockPayload, pending_.size() - off);
        bgzf_block(pending_.data() + off, len, level_, outs[i]);
    });
    emit(std::move(outs));
    size_t consumed = std::min(pending_.size(), nblk * kBlockPayload);
    pending_.erase(pending_.begin(), pending_.begin() + consumed);
}

void BgzfWriter::write_span(const uint8_t *data, size_t n) {
    // complete the partial block held in pending_, then compress the span's whole blocks in place
    if (!pending_.empty()) {
        const size_t fill = std::min(n, (kBlockPayload - pending_.size() % kBlockPayload) % kBlockPayload);
        pending_.insert(pending_.end(), data, data + fill);
        data += fill;
        n -= fill;
        if (pending_.size() % kBlockPayload == 0) flush_blocks(false);
    }
    const size_t whole = n / kBlockPayload;
    const size_t window = (size_t)std::max(1, threads_) * 64;  // blocks per parallel step (bounded memory)
    for (size_t b0 = 0; b0 < whole; b0 += window) {
        const size_t nb = std::min(window, whole - b0);
        std::vector<std::vector<uint8_t>> outs(nb);
        parallel_for(nb, threads_, [&](size_t i) {
            bgzf_block(data + (b0 + i) * kBlockPayload, kBlockPayload, level_, outs[i]);
        });
        emit(std::move(outs));  // written while the next window compresses
    }
    pending_.insert(pending_.end(), data + whole * kBlockPayload, data + n);
}

void BgzfWriter::write_compressed(const uint8_t *z, size_t n) {
    flush_blocks(true);
    drain();
    if (!n) return;
    // regular files: parallel pwrite at the stream position (page-cache copies on all threads)
    struct stat st;
    fflush(f_);
    const int fd = fileno(f_);
    const off_t at = ftello(f_);
    // pwrite ignores the offset on an O_APPEND descriptor (`>>` redirection): sequential there
    const int fl = fcntl(fd, F_GETFL);
    if (n >= (64ull << 20) && threads_ > 1 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && at >= 0 && fl >= 0 &&
        !(fl & O_APPEND)) {
        const size_t chunk = 32ull << 20, nch = (n + chunk - 1) / chunk;
        std::atomic<bool> ok(true);
        parallel_for(nch, threads_, [&](size_t c) {
            size_t o = c * chunk;
            const size_t e = std::min(n, o + chunk);
            while (o < e) {
                const ssize_t r = pwrite(fd, z + o, e - o, at + (off_t)o);
                if (r <= 0) {
                    ok = false;
                    return;
                }
                o += (size_t)r;
            }
        });
        if (ok && fseeko(f_, at + (off_t)n, SEEK_SET) == 0) return;
        fseeko(f_, at, SEEK_SET);  // fall back to one sequential write
    }
    put(z, n);
}

void BgzfWriter::close() {
    if (closed_) return;
    flush_blocks(true);
    drain();
    std::vector<uint8_t> eof;
    bgzf_block(nullptr, 0, level_, eof);
    put(eof.data(), eof.size());
    if (fflush(f_) != 0) failed_ = true;
    closed_ = true;
}

// ---------------- header model (util/bam_header.cpp:27-278) ----------------
static std::vector<std::string> split_tabs(const std::string &line) {
    std::vector<std::string> ret;
    size_t i = 0;
    for (;;) {
        size_t j = line.find('\t', i);
        if (j == std::string::npos) { ret.push_back(line.substr(i)); break; }
        ret.push_back(line.substr(i, j - i));
        i = j + 1;
    }
    return ret;
}

bool BamHeaderModel::parse(const std::string &text, std::string &err) {
    // getline loop that stops when the stream is no longer good: a final line without a
    // trailing newline is dropped (util/bam_header.cpp:113-116).
    std::string t(text);
    t.push_back('\0');  // the reference parses a text_len+1 buffer with a trailing NUL
    std::stringstream in(t);
    for (;;) {
        std::string line;
        std::getline(in, line);
        if (!in.good()) break;
        if (line.empty() || line[0] != '@') { err = "Sam header format problem: line doesn't begin with a '@'"; return false; }
        if (line.size() < 4 || line[3] != '\t') { err = "Sam header format problem: line doesn't have a tab after the tag"; return false; }
        std::string tag = line.substr(1, 2), data = line.substr(4);
        std::vector<std::string> segs = split_tabs(data);
        auto field = [&](const std::string &s, std::string &k, std::string &v) -> bool {
            if (s.size() < 3) { err = "malformed header field '" + s + "'"; return false; }
            k = s.substr(0, 2); v = s.substr(3); return true;
        };
        if (tag == "CO") {
            co.push_back(data);
        } else if (tag == "RG") {
            RgRecord r;
            for (auto &s : segs) {
                std::string k, v;
                if (!field(s, k, v)) return false;
                if (k == "ID") r.id = v; else if (k == "CN") r.cn = v; else if (k == "DS") r.ds = v;
                else if (k == "DT") r.dt = v; else if (k == "FO") r.fo = v; else if (k == "KS") r.ks = v;
                else if (k == "LB") r.lb = v; else if (k == "PG") r.pg = v; else if (k == "PI") r.pi = v;
                else if (k == "PL") r.pl = v; else if (k == "PU") r.pu = v; else if (k == "SM") r.sm = v;
            }
            if (r.id.empty()) { err = "Mandatory field missing in header read group line."; return false; }
            rg.push_back(r);
        } else if (tag == "SQ") {
            SqRecord r;
            for (auto &s : segs) {
                std::string k, v;
                if (!field(s, k, v)) return false;
                if (k == "SN") r.name = v; else if (k == "LN") r.length = (long long)(size_t)(long)atoi(v.c_str());
                else if (k == "AS") r.as = v; else if (k == "M5") r.m5 = v; else if (k == "SP") r.sp = v;
                else if (k == "UR") r.ur = v;
            }
            if (r.name.empty() || r.length == -1) { err = "Mandatory field missing in header sequence line."; return false; }
            sq.push_back(r);
        } else if (tag == "PG") {
            PgRecord r;
            for (auto &s : segs) {
                std::string k, v;
                if (!field(s, k, v)) return false;
                if (k == "ID") r.id = v; else if (k == "PN") r.pn = v; else if (k == "CL") r.cl = v;
                else if (k == "PP") r.pp = v; else if (k == "VN") r.vn = v;
            }
            if (r.id.empty()) { err = "Mandatory field missing in header program record line."; return false; }
            pg.push_back(r);
        } else if (tag == "HD") {
            std::string so;
            for (auto &s : segs) {
                std::string k, v;
                if (!field(s, k, v)) return false;
                if (k == "VN") format_version = v; else if (k == "SO") so = v;
            }
            if (so.empty() || format_version.empty()) { err = "Mandatory field missing in header HD line."; return false; }
            if (so == "unsorted") sort_order = UNSORTED;
            else if (so == "coordinate") sort_order = COORDINATE;
            else if (so == "queryname") sort_order = QUERYNAME;
            else if (so == "unknown") sort_order = UNKNOWN;
            else { err = "Unknown sort order '" + so + "'."; return false; }
        } else {
            err = "Sam header format problem: tag '" + tag + "' wasn't CO RG SQ PG or HD.";
            return false;
        }
    }
    if (format_version.empty()) { format_version = "1.4"; sort_order = UNKNOWN; }
    return true;
}

std::string BamHeaderModel::to_string() const {
    std::ostringstream s;
    static const char *so_names[] = {"unknown", "unsorted", "queryname", "coordinate"};
    s << "@HD\tVN:" << format_version << "\tSO:" << so_names[sort_order] << "\n";
    for (auto &r : sq) {
        s << "@SQ\tSN:" << r.name << "\tLN:" << (size_t)r.length;
        if (!r.as.empty()) s << "\tAS:" << r.as;
        if (!r.m5.empty()) s << "\tM5:" << r.m5;
        if (!r.sp.empty()) s << "\tSP:" << r.sp;
        if (!r.ur.empty()) s << "\tUR:" << r.ur;
        s << "\n";
    }
    for (auto &r : rg) {
        s << "@RG\tID:" << r.id;
        if (!r.cn.empty()) s << "\tCN:" << r.cn;
        if (!r.ds.empty()) s << "\tDS:" << r.ds;
        if (!r.dt.empty()) s << "\tDT:" << r.dt;
        if (!r.fo.empty()) s << "\tFO:" << r.fo;
        if (!r.ks.empty()) s << "\tKS:" << r.ks;
        if (!r.ks.empty()) s << "\tKS:" << r.ks;  // printed twice by the reference (bam_header.cpp:243-246)
        if (!r.lb.empty()) s << "\tLB:" << r.lb;
        if (!r.pg.empty()) s << "\tPG:" << r.pg;
        if (!r.pi.empty()) s << "\tPI:" << r.pi;
        if (!r.pl.empty()) s << "\tPL:" << r.pl;
        if (!r.pu.empty()) s << "\tPU:" << r.pu;
        if (!r.sm.empty()) s << "\tSM:" << r.sm;
        s << "\n";
    }
    for (auto &r : pg) {
        s << "@PG\tID:" << r.id;
        if (!r.pn.empty()) s << "\tPN:" << r.pn;
        if (!r.cl.empty()) s << "\tCL:" << r.cl;
        if (!r.pp.empty()) s << "\tPP:" << r.pp;
        if (!r.vn.empty()) s << "\tVN:" << r.vn;
        s << "\n";
    }
    for (auto &c : co) s << "@CO\t" << c << "\n";
    return s.str();
}

// ---------------- BAM ----------------
// Record offsets of the stream d[p, n) on all threads.  Each chunk but the first finds its first
// record by trying positions until 16 consecutive records look well-formed (block_size in
// [32, 10000], refIDs in range, NUL-terminated name, fixed fields inside the block), then walks to
// the first record at or past the next chunk's start.  The walks must meet exactly at every
// boundary and the last must end at n -- then the chain is the one a sequential walk from p takes
// (it is anchored at p); otherwise the caller falls back to the sequential walk, which also
// produces the reference's error messages for malformed input.
static bool plausible_record(const uint8_t *d, size_t s, size_t n, int32_t n_ref) {
    if (s + 36 > n) return false;
    const uint32_t bs = rd32(d + s);
    if (bs < 32 || bs > 10000 || s + 4 + bs > n) return false;
    const int32_t ref = (int32_t)rd32(d + s + 4), mref = (int32_t)rd32(d + s + 24);
    if (ref < -1 || ref >= n_ref || mref < -1 || mref >= n_ref) return false;
    const uint32_t lname = d[s + 12], nc = rd16(d + s + 16), lseq = rd32(d + s + 20);
    if (lname == 0 || d[s + 36 + lname - 1] != 0) return false;
    return 32ull + lname + 4ull * nc + (lseq + 1ull) / 2 + lseq <= bs;
}

static bool parse_offsets_parallel(const uint8_t *d, size_t p, size_t n, int32_t n_ref, int threads,
                                   std::vector<uint64_t> &offsets) {
    const int T = threads;
    std::vector<size_t> cut(T + 1);
    for (int i = 0; i <= T; ++i) cut[i] = p + (n - p) * (size_t)i / (size_t)T;
    std::vector<size_t> start(T, 0), stop(T, 0);
    std::vector<std::vector<uint64_t>> part(T);
    std::atomic<bool> ok(true);
    parallel_for((size_t)T, T, [&](size_t i) {
        size_t s = cut[i];
        if (i > 0) {
            const size_t lim = std::min(n, cut[i] + 20016);
            for (; s < lim; ++s) {
                size_t q = s;
                int k = 0;
                for (; k < 16 && q < n && plausible_record(d, q, n, n_ref); ++k) q += 4 + rd32(d + q);
                if (k == 16 || (q == n && k > 0)) break;
            }
            if (s >= lim) { ok = false; return; }
        }
        start[i] = s;
        std::vector<uint64_t> &o = part[i];
        o.reserve((cut[i + 1] - cut[i]) / 200 + 16);
        size_t q = s;
        while (q < cut[i + 1]) {
            if (q + 4 > n) { ok = false; return; }
            const uint32_t bs = rd32(d + q);
            if (bs < 32 || bs > 10000 || q + 4 + bs > n) { ok = false; return; }
            o.push_back(q - p);
            q += 4 + bs;
        }
        stop[i] = q;
    });
    if (!ok) return false;
    for (int i = 0; i + 1 < T; ++i)
        if (stop[i] != start[i + 1]) return false;
    if (stop[T - 1] != n) return false;
    std::vector<size_t> at(T + 1, 0);
    for (int i = 0; i < T; ++i) at[i + 1] = at[i] + part[i].size();
    offsets.resize(at[T]);
    parallel_for((size_t)T, T, [&](size_t i) { std::copy(part[i].begin(), part[i].end(), offsets.begin() + at[i]); });
    return true;
}

bool bam_parse_header(const uint8_t *d, size_t n, BamFile &out, std::string &err, size_t *rec_base) {
    if (n < 12 || memcmp(d, "BAM\1", 4) != 0) { err = "Error reading BAM stream header magic bytes."; return false; }
    uint32_t l_text = rd32(d + 4);
    if (8 + (size_t)l_text + 4 > n) { err = "Error reading BAM stream header text."; return false; }
    out.header_text.assign((const char *)d + 8, l_text);
    size_t p = 8 + l_text;
    if (!out.header.parse(out.header_text, err)) return false;
    uint32_t n_ref = rd32(d + p);
    p += 4;
    for (uint32_t i = 0; i < n_ref; ++i) {
        if (p + 4 > n) { err = "Error reading BAM stream reference sequence name length."; return false; }
        uint32_t ln = rd32(d + p);
        p += 4;
        if (p + ln + 4 > n || ln == 0) { err = "Error reading BAM stream reference sequence."; return false; }
        std::string name((const char *)d + p, ln - 1);
        p += ln;
        int32_t len = (int32_t)rd32(d + p);
        p += 4;
        out.ref_names.push_back(name);
        out.ref_lens.push_back(len);
        // util/bam_deserializer.h:126-133 -- binary list must match the text @SQ lines
        if (i >= out.header.sq.size() || out.header.sq[i].name != name || (int32_t)out.header.sq[i].length != len) {
            err = "BAM header text doesn't match sequence information.";
            return false;
        }
    }
    out.rec_base = p;
    *rec_base = p;
    return true;
}

bool bam_parse(bytevec &&raw, BamFile &out, std::string &err, int threads) {
    out.data = std::move(raw);
    const uint8_t *d = out.data.data();
    size_t n = out.data.size();
    size_t p = 0;
    if (!bam_parse_header(d, n, out, err, &p)) return false;
    uint32_t n_ref = (uint32_t)out.ref_names.size();
    out.offsets.clear();
    if (threads > 1 && n - p >= (64ull << 20) && parse_offsets_parallel(d, p, n, (int32_t)n_ref, threads, out.offsets))
        return true;
    out.offsets.clear();
    size_t q = p;
    while (q < n) {
        if (q + 4 > n) { err = "Expected more bytes reading BAM core. Is this file truncated or corrupted?"; return false; }
        uint32_t bs = rd32(d + q);
        // util/bam_deserializer.h:160-163
        if (bs < 32 || bs > 10000) { err = "Invalid BAM block size(" + std::to_string(bs) + ")."; return false; }
        if (q + 4 + bs > n) { err = "Expected more bytes reading BAM core. Is this file truncated or corrupted?"; return false; }
        out.offsets.push_back(q - p);
        q += 4 + bs;
    }
    return true;
}

bool read_file_bytes(const std::string &path, bytevec &comp, int threads, std::string &err) {
    FILE *f = (path == "-" || path == "stdin") ? stdin : fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    comp.clear();
    if (f != stdin && fseeko(f, 0, SEEK_END) == 0) {  // regular file: parallel preads into a sized buffer
        off_t sz = ftello(f);
        comp.reserve(sz > 0 ? (size_t)sz : 0);
        want_huge_pages(comp.data(), comp.capacity());
        comp.resize(sz > 0 ? (size_t)sz : 0);
        const int fd = fileno(f);
        const size_t chunk = 64ull << 20, nch = (comp.size() + chunk - 1) / chunk;
        std::atomic<bool> short_read(false);
        parallel_for(nch, threads, [&](size_t c) {
            size_t o = c * chunk, e = std::min(comp.size(), o + chunk);
            while (o < e) {
                ssize_t r = pread(fd, comp.data() + o, e - o, (off_t)o);
                if (r <= 0) {
                    short_read = true;
                    return;
                }
                o += (size_t)r;
            }
        });
        if (short_read) {
            fclose(f);
            err = "short read on " + path;
            return false;
        }
    } else {
        uint8_t buf[1 << 16];
        size_t r;
        while ((r = fread(buf, 1, sizeof(buf), f)) > 0) comp.insert(comp.end(), buf, buf + r);
    }
    if (f != stdin) fclose(f);
    return true;
}

bool bam_read_file(const std::string &path, BamFile &out, int threads, std::string &err) {
    static const bool dbg = getenv("OGE_IO_DEBUG") != nullptr;
    auto clk = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = clk();
    bytevec comp;
    if (!read_file_bytes(path, comp, threads, err)) return false;
    const auto t1 = clk();
    bytevec raw;
    if (!bgzf_inflate_all(comp.data(), comp.size(), raw, threads, err)) return false;
    const auto t2 = clk();
    const bool ok = bam_parse(std::move(raw), out, err, threads);
    if (dbg)
        fprintf(stderr, "[openge] read %s: file %.3f s, inflate %.3f s, parse %.3f s\n", path.c_str(),
                std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
                std::chrono::duration<double>(clk() - t2).count());
    return ok;
}

std::vector<uint8_t> bam_encode_header(const BamHeaderModel &h) {
    std::vector<uint8_t> o;
    auto put32 = [&](uint32_t v) { uint8_t b[4]; memcpy(b, &v, 4); o.insert(o.end(), b, b + 4); };
    std::string text = h.to_string();
    o.insert(o.end(), {'B', 'A', 'M', 1});
    put32((uint32_t)text.size());
    o.insert(o.end(), text.begin(), text.end());
    put32((uint32_t)h.sq.size());
    for (auto &s : h.sq) {
        put32((uint32_t)s.name.size() + 1);
        o.insert(o.end(), s.name.begin(), s.name.end());
        o.push_back(0);
        put32((uint32_t)(int32_t)s.length);
    }
    return o;
}

} // namespace oge
