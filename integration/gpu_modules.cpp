// gpu_modules.cpp -- see gpu_modules.h.
#include "gpu_modules.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <iostream>
#include <map>

namespace {

// One record in BAM encoding (the bytes BamSerializer::write emits, util/bam_serializer.h:105-147;
// the bin is recomputed by the library wherever it writes records).
void append_bam_record(std::string &arena, const OGERead &al) {
    const std::string &chars = al.getSupportData().getAllCharData();
    uint32_t w[9];
    w[0] = (uint32_t)chars.size() + 32;
    w[1] = (uint32_t)al.getRefID();
    w[2] = (uint32_t)al.getPosition();
    w[3] = (al.getMapQuality() << 8) | al.getNameLength();
    w[4] = (al.getAlignmentFlag() << 16) | al.getNumCigarOps();
    w[5] = (uint32_t)al.getLength();
    w[6] = (uint32_t)al.getMateRefID();
    w[7] = (uint32_t)al.getMatePosition();
    w[8] = (uint32_t)al.getInsertSize();
    arena.append((const char *)w, sizeof w);
    arena.append(chars);
}

// One more input record into the arena (offsets: n + 1 once `finish` ran).
void add(OGERead *r, std::vector<OGERead *> &reads, std::string &arena, std::vector<uint64_t> &off) {
    off.push_back(arena.size());
    append_bam_record(arena, *r);
    reads.push_back(r);
}
void finish(std::string &arena, std::vector<uint64_t> &off) {
    off.push_back(arena.size());
    arena.append(16, '\0');  // the library reads whole words at the end of a record
}

void fail(const char *what, oge_ctx *ctx) {
    std::cerr << what << ": " << oge_last_error(ctx) << std::endl;  // the reference's I/O error style
    exit(-1);
}

}  // namespace

const BamHeader &GpuReadSorter::getHeader() {  // as ReadSorter::getHeader (alg/read_sorter.cpp:234-262)
    while (!header_ready) usleep(10000);
    return header;
}

int GpuReadSorter::runInternal() {
    header = AlgorithmModule::getHeader();
    header.setSortOrder(BamHeader::SORT_COORDINATE);
    header_ready = true;
    std::vector<OGERead *> reads;
    std::string arena;
    std::vector<uint64_t> off;
    for (OGERead *r; (r = getInputAlignment()) != NULL;) add(r, reads, arena, off);
    finish(arena, off);
    oge_ctx *ctx = NULL;
    if (oge_ctx_create(device, &ctx)) fail("GpuReadSorter", NULL);
    std::vector<uint32_t> perm(reads.size() + 1);
    if (oge_sort_coord(ctx, (const uint8_t *)arena.data(), arena.size(), &off[0], reads.size(),
                       (int32_t)header.getSequences().size(), &perm[0]))
        fail("GpuReadSorter", ctx);
    oge_ctx_destroy(ctx);
    for (size_t k = 0; k < reads.size(); k++) putOutputAlignment(reads[perm[k]]);
    return 0;
}

int GpuMarkDuplicates::runInternal() {
    std::vector<OGERead *> reads;
    std::string arena;
    std::vector<uint64_t> off;
    for (OGERead *r; (r = getInputAlignment()) != NULL;) add(r, reads, arena, off);
    finish(arena, off);
    // read group -> library id as MarkDuplicates::getLibraryName / getLibraryId resolve it
    // (alg/mark_duplicates.cpp:282-318): first-seen order of the libraries, ids from 1
    const BamHeader &h = getHeader();
    std::string ids;
    std::vector<int16_t> libs;
    std::map<std::string, int16_t> lib_id;
    int16_t next = 1;
    for (BamReadGroupRecords::const_iterator g = h.getReadGroups().begin(); g != h.getReadGroups().end(); ++g) {
        const std::string lib = g->getLibrary().empty() ? std::string("Unknown Library") : g->getLibrary();
        std::map<std::string, int16_t>::iterator it = lib_id.find(lib);
        if (it == lib_id.end()) it = lib_id.insert(std::make_pair(lib, next++)).first;
        libs.push_back(it->second);
        ids += g->getId();
        ids.push_back('\0');
    }
    libs.push_back(0);
    std::map<std::string, int16_t>::iterator unk = lib_id.find("Unknown Library");
    oge_markdup_opts o;
    memset(&o, 0, sizeof o);
    o.n_ref = (int32_t)h.getSequences().size();
    o.rg_ids = ids.c_str();
    o.rg_ids_bytes = ids.size();
    o.rg_lib = &libs[0];
    o.n_rg = (int32_t)h.getReadGroups().size();
    o.unknown_lib = unk != lib_id.end() ? unk->second : next;
    oge_ctx *ctx = NULL;
    if (oge_ctx_create(device, &ctx)) fail("GpuMarkDuplicates", NULL);
    std::vector<uint8_t> dup(reads.size() + 1);
    uint64_t nd = 0;
    if (oge_markdup(ctx, (const uint8_t *)arena.data(), arena.size(), &off[0], reads.size(), &o, &dup[0], &nd))
        fail("GpuMarkDuplicates", ctx);
    oge_ctx_destroy(ctx);
    duplicates = nd;
    // the apply phase (alg/mark_duplicates.cpp:443-465): primaries get 0x400 set or cleared,
    // -r / -R drops the flagged ones (the receiver owns what it is handed; dropped reads are freed)
    for (size_t i = 0; i < reads.size(); i++) {
        OGERead *r = reads[i];
        if (dup[i] != 2) r->SetIsDuplicate(dup[i] == 1);
        if (removeDuplicates && dup[i] == 1) OGERead::deallocate(r);
        else putOutputAlignment(r);
    }
    return 0;
}
