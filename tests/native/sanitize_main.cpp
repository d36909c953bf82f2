// sanitize_main.cpp -- TEST INFRASTRUCTURE ONLY: the product's threaded host code in one executable
// for AddressSanitizer / ThreadSanitizer builds (the reference's own races
// Q13/Q14 show why).  Exercised:
//   bamio.cpp    parallel pread + parallel BGZF inflate + record walk (bam_read_file), the BgzfWriter
//                compressing on worker threads with a background ordered writer thread
//   realign.cpp  every host phase of localrealign on a thread pool: parallel decode, binning,
//                per-interval prepare / decide / update, per-contig mate-fixer segments, parallel
//                encode (the offset scan is the oracle's restatement in place of the HIP kernel)
//   sanitize_main IN.bam REF.fa INTERVALS OUT.bam THREADS [MAX_RECORDS_IN_MEMORY]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../openge_amd/csrc/bamio.h"
#include "../../openge_amd/csrc/realign.h"

extern "C" int oracle_realign_scan(const uint8_t *cons, const uint64_t *cons_off, const uint8_t *bases,
                                   const uint8_t *quals, const uint64_t *read_off, const int32_t *pairs, uint64_t n_pairs,
                                   int32_t *best_index, int32_t *best_score);

int main(int argc, char **argv) {
    if (argc < 6) return fprintf(stderr, "usage: sanitize_main IN.bam REF.fa INTERVALS OUT.bam THREADS [MAXREC]\n"), 2;
    const int threads = atoi(argv[5]);
    oge::BamFile f;
    std::string err;
    if (!oge::bam_read_file(argv[1], f, threads, err)) return fprintf(stderr, "read: %s\n", err.c_str()), 1;
    std::vector<uint64_t> offs(f.offsets);
    offs.push_back(f.rec_bytes());
    oge::RealignParams P;
    P.threads = threads;
    if (argc > 6) P.max_records_in_memory = atoi(argv[6]);
    oge::ScanFn scan = [](const oge::ScanBatch &B, std::vector<int32_t> &bi, std::vector<int32_t> &bs) {
        bi.resize(B.pairs.size());
        bs.resize(B.pairs.size());
        return oracle_realign_scan(B.cons.data(), B.cons_off.data(), B.bases.data(), B.quals.data(), B.read_off.data(),
                                   (const int32_t *)B.pairs.data(), B.pairs.size(), bi.data(), bs.data());
    };
    oge::ByteBuf out;
    std::vector<uint64_t> oo;
    oge::RealignStats st;
    if (oge::realign_run(f.ref_names, f.recs(), offs.data(), f.offsets.size(), argv[2], argv[3], P, scan, out, oo, st, err))
        return fprintf(stderr, "realign: %s\n", err.c_str()), 1;
    FILE *o = fopen(argv[4], "wb");
    if (!o) return perror(argv[4]), 1;
    {
        oge::BgzfWriter w(o, 6, threads);
        const std::vector<uint8_t> hb = oge::bam_encode_header(f.header);
        w.write(hb.data(), hb.size());
        const uint64_t n = oo.size() - 1;
        if (n) w.write_span(out.data() + oo[0], oo[n] - oo[0]);
        w.close();
        if (!w.ok()) return fprintf(stderr, "write failed\n"), 1;
    }
    if (fclose(o)) return 1;
    printf("%zu records in, %zu out\n", f.offsets.size(), oo.size() - 1);
    if (getenv("OGE_REALIGN_STATS"))  // phase times of the host code (the scan here is the oracle's)
        printf("bin %.3f (fasta %.3f decode %.3f) prepare %.3f scan %.3f (build %.3f) decide %.3f emit %.3f (mate %.3f) "
               "release %.3f run %.3f\n",
               st.t_bin, st.t_fasta, st.t_decode, st.t_prepare, st.t_scan, st.t_scan_build, st.t_decide, st.t_emit,
               st.t_mate, st.t_release, st.t_run);
    return 0;
}
