// rec_parse.h -- device-side BAM record field parsing shared by records.hip and markdup.hip.
#pragma once
#include "dev_util.h"

// BamAlignment::GetTag<std::string>("RG") -- FindTag/SkipToNextTag semantics
// (util/bamtools/BamAlignment.cpp:270-294,699-780; BamAlignment.h:576-606).  p = tag area start.
__device__ __forceinline__ bool find_rg(const uint8_t *p, const uint8_t *end, const uint8_t **val, uint32_t *len) {
    while (p + 3 <= end) {
        const uint32_t w = oge_ldu32(p);
        const uint8_t t0 = (uint8_t)w, t1 = (uint8_t)(w >> 8), type = (uint8_t)(w >> 16);
        p += 3;
        if (t0 == 'R' && t1 == 'G') {
            const uint8_t *s = p;
            while (s < end && *s) ++s;
            *val = p;
            *len = (uint32_t)(s - p);
            return true;
        }
        if (type == 0) return false;
        switch (type) {
        case 'A': case 'c': case 'C': p += 1; break;
        case 's': case 'S': p += 2; break;
        case 'f': case 'i': case 'I': p += 4; break;
        case 'Z': case 'H':
            while (p < end && *p) ++p;
            ++p;
            break;
        case 'B': {
            if (p + 5 > end) return false;
            const uint8_t at = p[0];
            const int32_t cnt = (int32_t)oge_ldu32(p + 1);
            p += 5;
            const int sz = (at == 'c' || at == 'C') ? 1 : (at == 's' || at == 'S') ? 2 : (at == 'f' || at == 'i' || at == 'I') ? 4 : 0;
            if (!sz) return false;
            p += (int64_t)cnt * sz;
            break;
        }
        default: return false;
        }
        if (p >= end || *p == 0) return false;
    }
    return false;
}

__device__ __forceinline__ uint32_t fnv_step(uint32_t h, uint32_t b) { return (h ^ b) * 16777619u; }

