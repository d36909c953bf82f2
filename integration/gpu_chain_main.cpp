// gpu_chain_main.cpp -- `openge mergesort -M --nopg` as cmd/command_mergesort.cpp:68-117 wires it,
// with the two GPU modules (gpu_modules.h) in place of ReadSorter and MarkDuplicates, the
// reference's own FileReader in front, and at the end a sink writing through the reference's
// BamSerializer<BgzfOutputStream> -- the serializer its FileWriter uses (alg/file_writer.cpp:144-166;
// FileWriter itself needs the CMake-generated openge_constants.h, which this image cannot make).
//   gpu_chain IN.bam OUT.bam [-R]
// and `openge localrealign` as cmd/command_localrealign.cpp:37-75 wires it, with GpuLocalRealignment in
// place of LocalRealignment:
//   gpu_chain realign REF.fa INTERVALS IN.bam OUT.bam
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <iostream>

#include "algorithms/file_reader.h"
#include "gpu_modules.h"
#include "util/bam_serializer.h"
#include "util/bgzf_output_stream.h"
#include "util/thread_pool.h"

class BamFileSink : public AlgorithmModule {
public:
    std::string filename;
protected:
    virtual int runInternal() {
        BamSerializer<BgzfOutputStream> w;
        w.getOutputStream().setCompressionLevel(6);
        if (!w.open(filename, getHeader())) {
            std::cerr << "Error opening BAM file to write." << std::endl;
            exit(-1);
        }
        for (OGERead *r; (r = getInputAlignment()) != NULL;) {
            w.write(*r);
            putOutputAlignment(r);
        }
        w.close();
        return 0;
    }
};

static void on_abort(int sig) {  // where an abort came from, for the test log
    void *bt[64];
    const int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char **argv) {
    signal(SIGABRT, on_abort);
    signal(SIGSEGV, on_abort);
    const bool realign = argc > 1 && !strcmp(argv[1], "realign");
    if (argc < 3 || (realign && argc < 6)) {
        std::cerr << "usage: gpu_chain IN.bam OUT.bam [-R] | gpu_chain realign REF.fa INTERVALS IN.bam OUT.bam" << std::endl;
        return 2;
    }
    OGEParallelismSettings::setNumberThreads(8);  // as cmd/commands.cpp:67-84 sets up the pool
    OGEParallelismSettings::enableMultithreading();
    AlgorithmModule::setNothreads(false);
    AlgorithmModule::setVerbose(false);
    FileReader reader;
    BamFileSink sink;
    int rc;
    if (realign) {
        GpuLocalRealignment lr;
        reader.addFile(argv[4]);
        sink.filename = argv[5];
        reader.addSink(&lr);
        lr.addSink(&sink);
        lr.setReferenceFilename(argv[2]);
        lr.setIntervalsFilename(argv[3]);
        rc = reader.runChain();
    } else {
        GpuReadSorter sorter;
        GpuMarkDuplicates md;
        reader.addFile(argv[1]);
        sink.filename = argv[2];
        md.removeDuplicates = argc > 3 && !strcmp(argv[3], "-R");
        reader.addSink(&sorter);
        sorter.addSink(&md);
        md.addSink(&sink);
        rc = reader.runChain();
        std::cerr << "Marked " << md.duplicates << " records as duplicates." << std::endl;
    }
    OGERead::clearCachedAllocations();
    ThreadPool::closeSharedPool();
    return rc;
}
