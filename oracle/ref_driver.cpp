// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref harness).
//
// Own code (not copied from the reference).  It links against the reference's
// own algorithm modules, compiled from /root/reference by oracle/Makefile.ref,
// and wires the same module chains the reference commands build:
//   sort       : FileReader -> ReadSorter -> sink     (cmd/command_mergesort.cpp:77-117, no -M)
//   dedup      : FileReader -> MarkDuplicates -> sink (cmd/command_dedup.cpp:48-69, --nosplit)
//   sortdedup  : FileReader -> ReadSorter -> MarkDuplicates -> sink (command_mergesort.cpp:68-117, -M --nosplit)
//   realign    : FileReader -> LocalRealignment -> sink (cmd/command_localrealign.cpp:37-75)
// sort / sortdedup take mergesort's -r region / -q mapq (a Filter between reader and sorter,
// command_mergesort.cpp:82-92) and -b (sort by name, :104).
// With -K k (k > 1) dedup / sortdedup run the reference's default split-by-chromosome chain
// instead (cmd/command_dedup.cpp:71-106, command_mergesort.cpp:118-170):
//   ... -> SplitByChromosome -> k x MarkDuplicates -> SortedMerge -> sink
// The sink writes BGZF BAM through the reference's BamSerializer<BgzfOutputStream>,
// i.e. exactly the serializer FileWriter uses (alg/file_writer.cpp:144-166), with
// no @PG line (the `--nopg` behaviour).  Global settings mirror
// cmd/commands.cpp:67-84.
//
// It is never part of the product.  The built binary travels to the GPU box with the snapshot and
// runs there only as test infrastructure: bench.py's cpu_baseline legs (the reference's own chains
// timed beside the GPU path) and -m gpu tests that compare against the reference chain's output.

#include <cstdlib>

#include "algorithms/algorithm_module.h"
#include "algorithms/file_reader.h"
#include "algorithms/read_sorter.h"
#include "algorithms/mark_duplicates.h"
#include "algorithms/local_realignment.h"
#include "algorithms/split_by_chromosome.h"
#include "algorithms/sorted_merge.h"
#include "algorithms/filter.h"
#include "util/bam_serializer.h"
#include "util/bgzf_output_stream.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <iostream>

class CaptureSink : public AlgorithmModule {
public:
    std::string filename;
    int level;
    CaptureSink() : level(6) {}
protected:
    virtual int runInternal() {
        BamHeader header = getHeader();
        BamSerializer<BgzfOutputStream> writer;
        writer.getOutputStream().setCompressionLevel(level);
        if (!writer.open(filename, header)) {
            std::cerr << "ref_driver: cannot open " << filename << std::endl;
            exit(2);
        }
        while (true) {
            OGERead *r = getInputAlignment();
            if (!r) break;
            writer.write(*r);
            putOutputAlignment(r);
        }
        writer.close();
        return 0;
    }
};

static void usage() {
    fprintf(stderr,
            "usage: ref_driver sort|dedup|sortdedup|realign [-v] [-D] [-t N] [-n N] [-T tmpdir] [-c level] [-K chains]\n"
            "                  [-r region] [-q mapq] [-b] [-S seed] [-R ref.fa -L intervals] in.bam [in2.bam ...] out.bam\n");
    exit(2);
}

int main(int argc, char **argv) {
    if (argc < 4) usage();
    std::string mode = argv[1];
    bool verbose = false;
    int threads = 8, per_tmp = 500000, level = 6, chains = 0;
    std::string tmpdir = "/tmp", ref, intervals, region;
    int mapq = -1;
    bool byname = false, remove_dups = false;
    std::vector<std::string> pos;
    for (int i = 2; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-v") verbose = true;
        else if (a == "-t" && i + 1 < argc) threads = atoi(argv[++i]);
        else if (a == "-n" && i + 1 < argc) per_tmp = atoi(argv[++i]);
        else if (a == "-T" && i + 1 < argc) tmpdir = argv[++i];
        else if (a == "-c" && i + 1 < argc) level = atoi(argv[++i]);
        else if (a == "-K" && i + 1 < argc) chains = atoi(argv[++i]);
        else if (a == "-R" && i + 1 < argc) ref = argv[++i];
        else if (a == "-L" && i + 1 < argc) intervals = argv[++i];
        else if (a == "-r" && i + 1 < argc) region = argv[++i];
        else if (a == "-q" && i + 1 < argc) mapq = atoi(argv[++i]);
        else if (a == "-b") byname = true;
        else if (a == "-D") remove_dups = true;  // MarkDuplicates::removeDuplicates (mergesort/dedup -R)
        else if (a == "-S" && i + 1 < argc) srand((unsigned)atoi(argv[++i]));  // harness only: the realigner's
                                  // random_shuffle of tied consensuses draws from rand()
        else pos.push_back(a);
    }
    if (pos.size() < 2) usage();  // in.bam [in2.bam ...] out.bam: several inputs go through MultiReader
    tmpdir += "/";

    OGEParallelismSettings::setNumberThreads(threads);
    AlgorithmModule::setNothreads(false);
    AlgorithmModule::setVerbose(verbose);
    OGEParallelismSettings::enableMultithreading();

    FileReader reader;
    reader.setLoadStringData(false);
    for (size_t k = 0; k + 1 < pos.size(); ++k) reader.addFile(pos[k]);
    CaptureSink sink;
    sink.filename = pos.back();
    sink.level = level;

    if ((mode == "dedup" || mode == "sortdedup") && chains > 1) {
        ReadSorter sorter(tmpdir);
        SplitByChromosome split;
        SortedMerge merge;
        std::vector<MarkDuplicates *> md;
        if (mode == "sortdedup") {
            sorter.setSortBy(BamHeader::SORT_COORDINATE);
            sorter.setCompressTempFiles(false);
            sorter.setAlignmentsPerTempfile(per_tmp);
            reader.addSink(&sorter);
            sorter.addSink(&split);
        } else {
            reader.addSink(&split);
        }
        merge.addSink(&sink);
        for (int c = 0; c < chains; ++c) {
            md.push_back(new MarkDuplicates(tmpdir));
            md.back()->removeDuplicates = remove_dups;
            merge.addSource(md.back());
            split.addSink(md.back());
        }
        sink.runChain();
        for (size_t c = 0; c < md.size(); ++c) delete md[c];
    } else if (mode == "sort" || mode == "sortdedup") {
        ReadSorter sorter(tmpdir);
        MarkDuplicates md(tmpdir);
        md.removeDuplicates = remove_dups;
        Filter filter;
        sorter.setSortBy(byname ? BamHeader::SORT_QUERYNAME : BamHeader::SORT_COORDINATE);
        sorter.setCompressTempFiles(false);
        sorter.setAlignmentsPerTempfile(per_tmp);
        if (!region.empty() || mapq >= 0) {
            if (!region.empty()) filter.setRegion(region);
            if (mapq >= 0) filter.setQualityLimit(mapq);
            reader.addSink(&filter);
            filter.addSink(&sorter);
        } else {
            reader.addSink(&sorter);
        }
        if (mode == "sortdedup") {
            sorter.addSink(&md);
            md.addSink(&sink);
        } else {
            sorter.addSink(&sink);
        }
        sink.runChain();
    } else if (mode == "dedup") {
        MarkDuplicates md(tmpdir);
        md.removeDuplicates = remove_dups;
        reader.addSink(&md);
        md.addSink(&sink);
        sink.runChain();
    } else if (mode == "realign") {
        if (ref.empty() || intervals.empty()) usage();
        LocalRealignment lr;
        reader.addSink(&lr);
        lr.addSink(&sink);
        lr.verbose = verbose;
        lr.setReferenceFilename(ref);
        lr.setIntervalsFilename(intervals);
        reader.runChain();
    } else {
        usage();
    }
    OGERead::clearCachedAllocations();
    ThreadPool::closeSharedPool();
    return 0;
}
