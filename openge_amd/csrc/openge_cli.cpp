// openge_cli.cpp -- the `openge` command-line drop-in for OpenGE's hot-path commands
// (oge/main.cpp:24-42, commands/commands.cpp:34-169): mergesort (+ the `sort` alias),
// dedup and localrealign, with the reference's option names and defaults.  Each command builds the
// same module chain the reference builds (commands/command_mergesort.cpp:68-117,
// command_dedup.cpp:48-69, command_localrealign.cpp:37-75) out of the modules in modules.h.
//
// Deliberate differences: dedup defaults to `-v --nosplit` semantics (Q1, Q3).
// --compat-nonverbose-dedup reproduces the non-verbose index bug; --split-chains K reproduces K
// split-by-chromosome chains, and --compat-split the reference's own rule for them (without
// --nosplit/--nothreads: K = min(12, threads / 2), command_dedup.cpp:46-48).  Sort by name (-b)
// gives the true name order (the reference merges name-sorted temp runs by position,
// util/read_stream_reader.h:94-97, so its output is name-sorted only within one run of -n reads).
// SAM/FASTQ output is not provided and fails loudly.
#include <sys/resource.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "modules.h"

using namespace oge;

namespace {

struct Opt {
    const char *shortname, *longname;
    bool takes_value;
};

// global_options + io_options (commands.cpp:117-132) and each command's getOptions()
const Opt kGlobal[] = {{"v", "verbose", false}, {"t", "threads", true}, {"d", "nothreads", false},
                       {"T", "tmpdir", true},   {"", "nosplit", false},  {"i", "in", true},
                       {"F", "format", true},   {"c", "compression", true}, {"", "nopg", false},
                       {"", "device", true},    {"", "compat-nonverbose-dedup", false},
                       {"", "split-chains", true}, {"", "compat-split", false}, {"", "gpus", true}};
const Opt kMergesort[] = {{"o", "out", true}, {"r", "region", true},  {"q", "mapq", true},
                          {"b", "byname", false}, {"n", "n", true}, {"C", "compresstempfiles", false},
                          {"M", "markduplicates", false}, {"R", "removeduplicates", false}};
const Opt kDedup[] = {{"o", "out", true}, {"r", "remove", false}};
const Opt kRealign[] = {{"o", "out", true}, {"R", "reference", true}, {"L", "intervals", true}};

struct Parsed {
    std::map<std::string, std::vector<std::string>> vm;  // long name -> values ("" for flags)
    std::vector<std::string> inputs;
    bool count(const char *k) const { return vm.count(k) != 0; }
    std::string get(const char *k, const std::string &def) const {
        auto it = vm.find(k);
        return it == vm.end() || it->second.empty() ? def : it->second.back();
    }
};

bool parse(int argc, const char **argv, const std::vector<Opt> &opts, Parsed &p) {
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        const Opt *o = nullptr;
        std::string val;
        bool have_val = false;
        if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
            std::string k = a.substr(2);
            size_t eq = k.find('=');
            if (eq != std::string::npos) {
                val = k.substr(eq + 1);
                k = k.substr(0, eq);
                have_val = true;
            }
            for (auto &x : opts)
                if (k == x.longname) o = &x;
        } else if (a.size() >= 2 && a[0] == '-' && a != "-") {
            std::string k = a.substr(1, 1);
            for (auto &x : opts)
                if (k == x.shortname) o = &x;
            if (o && a.size() > 2) {
                val = a.substr(2);
                have_val = true;
            }
        } else {
            p.inputs.push_back(a);
            continue;
        }
        if (!o) {
            fprintf(stderr, "Error: unrecognised option '%s'\n", a.c_str());
            return false;
        }
        if (o->takes_value && !have_val) {
            if (i + 1 >= argc) {
                fprintf(stderr, "Error: the required argument for option '--%s' is missing\n", o->longname);
                return false;
            }
            val = argv[++i];
        }
        p.vm[o->longname].push_back(o->takes_value ? val : "");
    }
    for (auto &v : p.vm["in"]) p.inputs.push_back(v);
    p.vm.erase("in");
    return true;
}

void usage_top() {
    fprintf(stderr, "Usage:\n    openge command [options]\n\nCommands: mergesort (alias: sort), dedup, localrealign, version\n");
}

}  // namespace

int main(int argc, const char **argv) {
    if (argc == 1) {
        usage_top();
        return 0;
    }
    std::string cmd = argv[1];
    if (cmd == "sort") cmd = "mergesort";  // the reference has no `sort` command
    if (cmd == "version") {
        printf("openge 0.3-dev (openge_amd MI355X path: %s)\n", oge_version());
        return 0;
    }
    if (cmd == "help") {
        usage_top();
        return 0;
    }
    std::vector<Opt> opts(std::begin(kGlobal), std::end(kGlobal));
    if (cmd == "mergesort") opts.insert(opts.end(), std::begin(kMergesort), std::end(kMergesort));
    else if (cmd == "dedup") opts.insert(opts.end(), std::begin(kDedup), std::end(kDedup));
    else if (cmd == "localrealign") opts.insert(opts.end(), std::begin(kRealign), std::end(kRealign));
    else {
        fprintf(stderr, "Unknown command %s.\n", argv[1]);
        return -1;
    }
    // command_line (commands.cpp:36-40): "openge " + every argument after `openge`, space-terminated
    std::string command_line = "openge ";
    for (int i = 1; i < argc; ++i) {
        command_line += argv[i];
        command_line += " ";
    }
    Parsed p;
    if (!parse(argc - 1, argv + 1, opts, p)) return -1;
    if (p.inputs.empty()) p.inputs.push_back("stdin");

    ChainContext cc;
    cc.verbose = p.count("verbose");
    cc.threads = atoi(p.get("threads", std::to_string(std::max(1u, std::thread::hardware_concurrency()))).c_str());
    cc.device = atoi(p.get("device", "0").c_str());
    cc.gpus = std::max(1, atoi(p.get("gpus", "1").c_str()));  // ranks over RCCL / xGMI
    AlgorithmModule::setVerbose(cc.verbose);
    const int level = atoi(p.get("compression", "6").c_str());
    const bool compat = p.count("compat-nonverbose-dedup");
    int split = atoi(p.get("split-chains", "0").c_str());
    if (p.count("compat-split") && !p.count("nosplit") && !p.count("nothreads")) split = std::min(12, cc.threads / 2);
    if (split > 1 && compat) {
        fprintf(stderr, "openge: split chains with --compat-nonverbose-dedup are not supported\n");
        return -1;
    }
    timeval t0;
    gettimeofday(&t0, nullptr);
    // one input file on one GPU: its bytes come off the disk / page cache while HIP initialises
    if (p.inputs.size() == 1 && p.inputs[0] != "stdin" && cc.gpus == 1) prefetch_input(p.inputs[0]);
    if (oge_ctx_create(cc.device, &cc.ctx)) {
        fprintf(stderr, "openge: %s\n", oge_last_error(nullptr));
        return -1;
    }
    const char *pool = getenv("OGE_POOL");  // default on: the chain's modules share one memory pool
    if (!(pool && std::string(pool) == "0") && oge_ctx_set_pool(cc.ctx, 1)) {
        fprintf(stderr, "openge: %s\n", oge_last_error(cc.ctx));
        return -1;
    }

    FileReader reader;
    FileWriter writer;
    reader.addFiles(p.inputs);
    writer.setFilename(p.get("out", "stdout"));
    if (!p.count("nopg")) writer.addProgramLine(command_line);
    writer.setCompressionLevel(level);
    if (p.count("format") && writer.setFormat(p.get("format", "bam"))) return -1;

    int ret = 0;
    if (cmd == "mergesort") {
        bool dedup = p.count("markduplicates") || p.count("removeduplicates");
        Filter filter;
        ReadSorter sorter;
        MarkDuplicates md;
        sorter.setSortBy(p.count("byname") ? BamHeaderModel::QUERYNAME : BamHeaderModel::COORDINATE);
        sorter.setCompressTempFiles(p.count("compresstempfiles"));
        sorter.setAlignmentsPerTempfile(atoi(p.get("n", "500000").c_str()));
        if (p.count("region") || p.count("mapq")) {  // command_mergesort.cpp:82-92
            if (p.count("region")) filter.setRegion(p.get("region", ""));
            if (p.count("mapq")) filter.setQualityLimit(atoi(p.get("mapq", "0").c_str()));
            reader.addSink(&filter);
            filter.addSink(&sorter);
        } else {
            reader.addSink(&sorter);
        }
        if (dedup) {
            md.removeDuplicates = p.count("removeduplicates");
            md.compatNonverbose = compat;
            md.splitChains = split;
            sorter.addSink(&md);
            md.addSink(&writer);
        } else {
            sorter.addSink(&writer);
        }
        ret = writer.runChain(cc);
        if (cc.verbose && dedup) fprintf(stderr, "Marked %llu records as duplicates.\n", (unsigned long long)md.duplicates);
    } else if (cmd == "dedup") {
        MarkDuplicates md;
        md.removeDuplicates = p.count("remove");
        md.compatNonverbose = compat;
        md.splitChains = split;
        reader.addSink(&md);
        md.addSink(&writer);
        ret = writer.runChain(cc);
        if (cc.verbose) fprintf(stderr, "Marked %llu records as duplicates.\n", (unsigned long long)md.duplicates);
    } else {
        if (!p.count("reference") || p.vm["reference"].size() != 1) {
            fprintf(stderr, "One FASTA reference file is required.\n");
            return -1;
        }
        if (!p.count("intervals") || p.vm["intervals"].size() != 1) {
            fprintf(stderr, "One intervals file is required.\n");
            return -1;
        }
        LocalRealignment lr;
        lr.verbose = cc.verbose;
        lr.setReferenceFilename(p.get("reference", ""));
        lr.setIntervalsFilename(p.get("intervals", ""));
        reader.addSink(&lr);
        lr.addSink(&writer);
        ret = writer.runChain(cc);
    }
    cc.close_ranks();
    oge_ctx_destroy(cc.ctx);
    if (cc.verbose) {  // commands.cpp:91-108
        rusage r;
        getrusage(RUSAGE_SELF, &r);
        timeval t1;
        gettimeofday(&t1, nullptr);
        double el = (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
        fprintf(stderr, "Elapsed time: %3ldm%06.3fs\n", (long)el / 60, el - 60 * ((long)el / 60));
        fprintf(stderr, "Max mem: %6ld MB\n", r.ru_maxrss / 1024);
    }
    return ret;
}
