// gpu_modules.h -- the modules an OpenGE maintainer adds to openge/src/algorithms to run the sort,
// duplicate marking and local realignment on MI355X: AlgorithmModule subclasses (alg/algorithm_module.h:33-107) that drain
// their input queue into a BAM-record arena, make one call into libopenge_hip.so
// (include/openge_hip.h), and emit the same OGERead objects in the new order / with the new flags,
// keeping the module contract (ownership passes on with putOutputAlignment; header via getHeader).
// Written in the reference's dialect (C++98) and built against its headers by integration/Makefile;
// tests/test_integration.py compiles and links it, tests/test_gpu_integration.py runs the chain.
#ifndef OGE_GPU_MODULES_H
#define OGE_GPU_MODULES_H

#include <string>
#include <vector>

#include "algorithms/algorithm_module.h"
#include "openge_hip.h"

// Drop-in for ReadSorter (alg/read_sorter.h:32-105) with SORT_COORDINATE: oge_sort_coord.
class GpuReadSorter : public AlgorithmModule {
public:
    explicit GpuReadSorter(int device = 0) : device(device), header_ready(false) {}
    virtual const BamHeader &getHeader();
    // the reference's knobs, kept for drop-in compatibility (one device sort replaces the spilled runs)
    void setCompressTempFiles(bool) {}
    void setAlignmentsPerTempfile(int) {}

protected:
    virtual int runInternal();
    int device;
    BamHeader header;
    bool header_ready;
};

// Drop-in for LocalRealignment (alg/local_realignment.h:67-527, wired by
// cmd/command_localrealign.cpp:37-75): the same setters and public `verbose`; oge_localrealign runs
// the whole module (binning, consensuses, the offset scan on the GPU, decisions, CIGAR / tag updates,
// mate fixing) over the drained records and the realigned records are emitted in the module's order.
class GpuLocalRealignment : public AlgorithmModule {
public:
    explicit GpuLocalRealignment(int device = 0) : verbose(false), device(device) {}
    bool verbose;
    void setReferenceFilename(const std::string &filename) { reference_filename = filename; }
    void setIntervalsFilename(const std::string &filename) { intervals_filename = filename; }

protected:
    virtual int runInternal();
    int device;
    std::string reference_filename, intervals_filename;
};

// Drop-in for MarkDuplicates (alg/mark_duplicates.h:27-68, -v --nosplit semantics): oge_markdup.
class GpuMarkDuplicates : public AlgorithmModule {
public:
    explicit GpuMarkDuplicates(int device = 0) : removeDuplicates(false), duplicates(0), device(device) {}
    bool removeDuplicates;
    size_t duplicates;

protected:
    virtual int runInternal();
    int device;
};

#endif
