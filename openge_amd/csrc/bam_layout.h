// bam_layout.h -- BAM record layout helpers shared by host code and HIP kernels.
//
// A record in a record arena is stored exactly as in a decompressed BAM stream:
//   [0,4)  block_size (u32, bytes that follow)
//   [4,8)  refID  [8,12) pos  [12] l_read_name  [13] mapq  [14,16) bin
//   [16,18) n_cigar_op  [18,20) flag  [20,24) l_seq  [24,28) next_refID
//   [28,32) next_pos  [32,36) tlen  [36,...) read_name\0, cigar u32[], seq, qual, tags
// (the reference decodes the same bytes at util/bam_deserializer.h:143-193 and
// re-encodes them at util/bam_serializer.h:105-147).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define OGE_HD __host__ __device__ __forceinline__
#else
#define OGE_HD static inline
#endif

enum {
    OGE_OFF_BLOCK = 0, OGE_OFF_REFID = 4, OGE_OFF_POS = 8, OGE_OFF_LNAME = 12, OGE_OFF_MAPQ = 13,
    OGE_OFF_BIN = 14, OGE_OFF_NCIGAR = 16, OGE_OFF_FLAG = 18, OGE_OFF_LSEQ = 20,
    OGE_OFF_MREFID = 24, OGE_OFF_MPOS = 28, OGE_OFF_TLEN = 32, OGE_OFF_NAME = 36
};

enum {
    OGE_F_PAIRED = 0x1, OGE_F_PROPER = 0x2, OGE_F_UNMAP = 0x4, OGE_F_MUNMAP = 0x8,
    OGE_F_REVERSE = 0x10, OGE_F_MREVERSE = 0x20, OGE_F_READ1 = 0x40, OGE_F_READ2 = 0x80,
    OGE_F_SECONDARY = 0x100, OGE_F_QCFAIL = 0x200, OGE_F_DUP = 0x400, OGE_F_SUPPLEMENTARY = 0x800
};

// CIGAR op codes (BAM_CIGAR_LOOKUP "MIDNSHP=X")
enum { OGE_CIG_M = 0, OGE_CIG_I = 1, OGE_CIG_D = 2, OGE_CIG_N = 3, OGE_CIG_S = 4, OGE_CIG_H = 5,
       OGE_CIG_P = 6, OGE_CIG_EQ = 7, OGE_CIG_X = 8 };

OGE_HD uint32_t oge_rd_u32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
OGE_HD int32_t oge_rd_i32(const uint8_t *p) { return (int32_t)oge_rd_u32(p); }
OGE_HD uint16_t oge_rd_u16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
OGE_HD void oge_wr_u32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
OGE_HD void oge_wr_u16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

// Minimum BAM bin for [beg, end) -- util/bam_serializer.h:92-101 (the reference recomputes
// bin on every write, util/bam_serializer.h:112-116).  Arithmetic shifts on int, so
// pos = -1 with no CIGAR gives 4680.
OGE_HD uint32_t oge_reg2bin(int beg, int end) {
    --end;
    if ((beg >> 14) == (end >> 14)) return 4681 + (beg >> 14);
    if ((beg >> 17) == (end >> 17)) return 585 + (beg >> 17);
    if ((beg >> 20) == (end >> 20)) return 73 + (beg >> 20);
    if ((beg >> 23) == (end >> 23)) return 9 + (beg >> 23);
    if ((beg >> 26) == (end >> 26)) return 1 + (beg >> 26);
    return 0;
}

// Alignment end (half-open) the way BamAlignment::GetEndPosition computes it
// (util/bamtools/BamAlignment.cpp:311-350): pos + lengths of M, D, N, =, X ops.
OGE_HD int32_t oge_rec_end(const uint8_t *rec) {
    int32_t end = oge_rd_i32(rec + OGE_OFF_POS);
    uint32_t ncig = oge_rd_u16(rec + OGE_OFF_NCIGAR);
    const uint8_t *c = rec + OGE_OFF_NAME + rec[OGE_OFF_LNAME];
    for (uint32_t i = 0; i < ncig; ++i) {
        uint32_t op = oge_rd_u32(c + 4 * i);
        uint32_t t = op & 0xF;
        if (t == OGE_CIG_M || t == OGE_CIG_D || t == OGE_CIG_N || t == OGE_CIG_EQ || t == OGE_CIG_X)
            end += (int32_t)(op >> 4);
    }
    return end;
}

// The bin BamSerializer::write stores (util/bam_serializer.h:108-116).
OGE_HD uint16_t oge_rec_bin(const uint8_t *rec) {
    return (uint16_t)oge_reg2bin(oge_rd_i32(rec + OGE_OFF_POS), oge_rec_end(rec));
}
