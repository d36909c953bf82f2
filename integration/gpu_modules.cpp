// gpu_modules.cpp -- see gpu_modules.h.
#include "gpu_modules.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <iostream>
#include <map>
#include <sstream>

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

// An OGERead holding one BAM record (block_size + core + data), filled as BamDeserializer::read fills
// the records it reads (util/bam_deserializer.h:143-193).
OGERead *read_from_bam_record(const uint8_t *r) {
    uint32_t w[9];
    memcpy(w, r, sizeof w);
    OGERead *al = OGERead::allocate();
    al->setRefID((int32_t)w[1]);
    al->setPosition((int32_t)w[2]);
    const uint32_t lname = w[3] & 0xff;
    al->setMapQuality((w[3] >> 8) & 0xff);
    al->setBin(w[3] >> 16);
    const uint32_t ncig = w[4] & 0xffff;
    al->setAlignmentFlag(w[4] >> 16);
    al->setMateRefID((int32_t)w[6]);
    al->setMatePosition((int32_t)w[7]);
    al->setInsertSize((int32_t)w[8]);
    al->setBamStringData((const char *)r + 36, w[0] - 32, ncig, w[5], lname);
    return al;
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
    // -r / -R drops every record whose FLAG then carries 0x400 -- non-primaries keep the bit they came
    // with (:456) -- (the receiver owns what it is handed; dropped reads are freed)
    for (size_t i = 0; i < reads.size(); i++) {
        OGERead *r = reads[i];
        if (dup[i] != 2) r->SetIsDuplicate(dup[i] == 1);
        if (removeDuplicates && r->IsDuplicate()) OGERead::deallocate(r);
        else putOutputAlignment(r);
    }
    return 0;
}

int GpuLocalRealignment::runInternal() {
    // the sequence dictionary the realigner needs, as SAM header text (LocalRealignment::runInternal reads
    // getHeader().getSequences(), alg/local_realignment.cpp:1464)
    const BamHeader &h = getHeader();
    std::ostringstream ht;
    for (BamSequenceRecords::const_iterator sq = h.getSequences().begin(); sq != h.getSequences().end(); ++sq)
        ht << "@SQ\tSN:" << sq->getName() << "\tLN:" << sq->getLength() << "\n";
    const std::string hts = ht.str();
    // drain the input (coordinate-sorted, as the reference module requires); the module owns what it
    // is handed, so the input reads are freed once their bytes are in the arena
    std::string arena;
    std::vector<uint64_t> off;
    for (OGERead *r; (r = getInputAlignment()) != NULL;) {
        off.push_back(arena.size());
        append_bam_record(arena, *r);
        OGERead::deallocate(r);
    }
    const uint64_t n = off.size();
    finish(arena, off);
    oge_ctx *ctx = NULL;
    if (oge_ctx_create(device, &ctx)) fail("GpuLocalRealignment", NULL);
    oge_realign_opts o;
    oge_realign_opts_init(&o);
    oge_realign_result *res = NULL;
    if (oge_localrealign(ctx, hts.c_str(), hts.size(), (const uint8_t *)arena.data(), &off[0], n, reference_filename.c_str(),
                         intervals_filename.c_str(), &o, &res))
        fail("GpuLocalRealignment", ctx);
    if (verbose) std::cerr << "GpuLocalRealignment: " << oge_realign_result_stats(res) << std::endl;
    const uint64_t m = oge_realign_result_count(res);
    uint64_t nb = 0;
    const uint8_t *out = oge_realign_result_records(res, &nb);
    const uint64_t *oo = oge_realign_result_offsets(res);
    for (uint64_t k = 0; k < m; k++) putOutputAlignment(read_from_bam_record(out + oo[k]));
    oge_realign_result_free(res);
    oge_ctx_destroy(ctx);
    return 0;
}
