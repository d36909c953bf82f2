/* openge_hip.h -- C ABI of libopenge_hip.so, the MI355X (gfx950) drop-in for OpenGE's
 * post-alignment hot path: coordinate sort, duplicate marking, local-realignment scoring.
 *
 * Conventions: every entry point returns 0 on success and a negative oge_status on failure
 * (message via oge_last_error); no C++ exceptions cross the ABI; plain pointers and sizes
 * only.  Record buffers hold BAM records exactly as in a decompressed BAM stream
 * (block_size u32 + 32-byte core + variable data, util/bam_deserializer.h:143-193) and are
 * addressed by a u64 byte offset per record.
 *
 * Entry points named *_dev take device (HBM) pointers and run on the context's HIP stream;
 * the others take host buffers and copy in/out.  One context per host thread and GPU.
 *
 * Reference interfaces replaced (paths under openge/src/):
 *   oge_sort_coord*      <- ReadSorter (algorithms/read_sorter.h:32-105, .cpp:48-232) with
 *                           Sort::ByPosition (util/bamtools/Sort.h:116-136) and the
 *                           MultiReader run merge (util/read_stream_reader.h:132-153)
 *   oge_gather_records*  <- BamSerializer::write's record encode incl. bin recompute
 *                           (util/bam_serializer.h:105-147) applied to the sorted stream
 *   oge_markdup*         <- MarkDuplicates::runInternal/buildSortedReadEndLists/
 *                           generateDuplicateIndexes (algorithms/mark_duplicates.cpp:185-475)
 *   oge_realign_scan*    <- LocalRealignment::findBestOffset + mismatchQualitySumIgnoreCigar
 *                           (algorithms/local_realignment.cpp:641-679,1126-1164)
 */
#ifndef OPENGE_HIP_H
#define OPENGE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum oge_status {
    OGE_OK = 0,
    OGE_ERR_ARG = -1,      /* bad argument / malformed record */
    OGE_ERR_HIP = -2,      /* HIP runtime error (no device, launch failure, OOM) */
    OGE_ERR_LIMIT = -3,    /* input outside supported limits */
    OGE_ERR_IO = -4        /* file / codec error */
} oge_status;

typedef struct oge_ctx oge_ctx;

/* ---- context ---------------------------------------------------------------------- */
int oge_ctx_create(int device, oge_ctx **out);
/* number of HIP devices visible to the process (0 when there is none) */
int oge_device_count(void);
/* stream: a hipStream_t (0 = the context's own non-blocking stream) */
int oge_ctx_set_stream(oge_ctx *ctx, void *stream);
void *oge_ctx_stream(oge_ctx *ctx);
int oge_ctx_sync(oge_ctx *ctx);
void oge_ctx_destroy(oge_ctx *ctx);
const char *oge_last_error(const oge_ctx *ctx);   /* ctx may be NULL (thread-local last error) */
/* last pipeline's kernel timings in ms, measured with HIP events on the context stream */
int oge_ctx_timing(oge_ctx *ctx, const char *stage, double *ms_out);
/* A work count of the context's last pipeline call (e.g. "shard_blocks", "shard_zbytes",
 * "shard_bytes", "shard_records" of oge_bgzf_decode_shard: this rank's BGZF blocks, their compressed
 * and decompressed bytes, its records).  OGE_ERR_ARG when the call recorded no such count. */
int oge_ctx_counter(oge_ctx *ctx, const char *name, uint64_t *value);
/* version string of the library, gfx target it was built for */
const char *oge_version(void);

/* ---- device buffers (for host code that stages records in HBM without HIP headers) ---- */
int oge_dev_alloc(oge_ctx *ctx, uint64_t bytes, void **out);
int oge_dev_free(oge_ctx *ctx, void *p);
/* kind: 1 = host->device, 2 = device->host, 3 = device->device, 4 = any (also between two GPUs'
 * HBM); synchronous on the ctx stream */
int oge_memcpy(oge_ctx *ctx, void *dst, const void *src, uint64_t bytes, int kind);
/* enable != 0: device buffers (oge_dev_alloc and the library's workspaces) come from the device's
 * stream-ordered pool and freed memory stays reserved for the next allocation of this process
 * (a module chain then reuses one module's buffers for the next).  Call before any allocation;
 * buffers must be freed with the same setting. */
int oge_ctx_set_pool(oge_ctx *ctx, int enable);
/* Page-locked host memory (DMA at full PCIe rate) for staging compressed output. */
int oge_host_alloc(oge_ctx *ctx, uint64_t bytes, void **out);
int oge_host_free(oge_ctx *ctx, void *p);

/* ---- coordinate sort (ReadSorter + Sort::ByPosition) ------------------------------ */
/* perm_out[k] = input index of the record at sorted position k.  Order: refID ascending with
 * refID == -1 last; pos; forward before reverse; read name bytes; flag; input index (the
 * reference's final tie-break is the record's heap address).  Records with
 * refID == -1 keep input order (reference order there is implementation-defined, Q11).
 * n_ref: number of reference sequences (refIDs must lie in [-1, n_ref)). */
int oge_sort_coord(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off,
                   uint64_t n, int32_t n_ref, uint32_t *perm_out);
int oge_sort_coord_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                       int32_t n_ref, uint32_t *d_perm);

/* ---- permutation gather with BAM re-encode (bin recompute) ------------------------- */
/* out record k = record perm[k] with its bin field recomputed as the reference writer does.
 * d_out_off (n+1 entries) receives the output offsets; d_out must hold the same byte total. */
int oge_gather_records_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, const uint32_t *d_perm,
                           uint64_t n, uint8_t *d_out, uint64_t *d_out_off);

/* Device primitive used by every sort above, exposed for tests: stable LSD radix sort of
 * (u64 key, u32 value) pairs on the key bits in bit_mask (d_vals/d_vtmp may be NULL).  The sorted
 * pairs end in (d_keys, d_vals) when *in_tmp_out == 0, in (d_ktmp, d_vtmp) when 1. */
int oge_radix_sort_pairs_dev(oge_ctx *ctx, uint64_t *d_keys, uint32_t *d_vals, uint64_t *d_ktmp, uint32_t *d_vtmp,
                             uint64_t n, uint64_t bit_mask, int *in_tmp_out);

/* Device primitive behind every compaction and offset table, exposed for tests: exclusive prefix sum
 * of n unsigned elements of elem_bytes (4 or 8) bytes, d_out may equal d_in.  Synchronous. */
int oge_exclusive_scan_dev(oge_ctx *ctx, const void *d_in, void *d_out, uint64_t n, int elem_bytes);

/* ---- duplicate marking (MarkDuplicates) ------------------------------------------- */
typedef struct oge_markdup_opts {
    int32_t n_ref;
    /* Read-group -> library table: rg_ids is n_rg NUL-terminated IDs back to back; rg_lib[i] is
     * the library id (>= 1) of rg i.  Records whose RG is absent / unknown / has no LB use
     * unknown_lib (getLibraryName, algorithms/mark_duplicates.cpp:301-318). */
    const char *rg_ids;
    uint64_t rg_ids_bytes;
    const int16_t *rg_lib;
    int32_t n_rg;
    int16_t unknown_lib;
    /* Test knob: 1 = group fragments / pairs with the sort-based stages even where the windowed
     * ones apply (records in sorted order on one GPU).  Results must not change. */
    int16_t debug_sort_groups;
    /* Reproduce the reference's non-verbose index bug: the record index only
     * advances under -v, so every ReadEnds carries index 0.  Default 0 = -v semantics. */
    int32_t compat_nonverbose_index;
    /* 1 = drop duplicates from the output (-r/-R); affects oge_markdup's n_kept only */
    int32_t remove_duplicates;
    /* Test knob: keep only this many bits (1..47) of the 48-bit pair-key hash, to force the
     * collision paths of the mate join.  0 = full hash.  Results must not change. */
    int32_t debug_hash_bits;
    /* Split-by-chromosome emulation (cmd/command_dedup.cpp:71-106,
     * algorithms/split_by_chromosome.cpp:45-48): K > 1 gives the result of K MarkDuplicates chains
     * fed refID % K (refID < 0 -> chain 0) -- mates in different chains never pair.  The
     * reference's default when --nosplit is absent, with K = min(12, threads / 2).  0 or 1 =
     * --nosplit.  Not combinable with compat_nonverbose_index. */
    int32_t split_chains;
} oge_markdup_opts;

/* dup_out[i] (per input record, input order = record index): 1 if record i is flagged
 * 0x400, 0 if a primary record that gets 0x400 cleared, 2 if non-primary (flag untouched).
 * flags_out (optional, may be NULL): the record's new FLAG field. */
int oge_markdup(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n,
                const oge_markdup_opts *opts, uint8_t *dup_out, uint64_t *n_dup_out);
/* Device form: also rewrites FLAG 0x400 in place in d_recs when apply != 0. */
int oge_markdup_dev(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                    const oge_markdup_opts *opts, uint8_t *d_dup, int apply, uint64_t *n_dup_out);

/* ---- fused sort + markdup (mergesort -M --nosplit) on device-resident records -------- */
/* d_out/d_out_off receive the sorted records with bin recomputed and 0x400 applied.
 * d_perm (n) receives the permutation. */
int oge_sort_markdup_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                         const oge_markdup_opts *opts, uint32_t *d_perm, uint8_t *d_out, uint64_t *d_out_off,
                         uint64_t *n_dup_out);

/* Allocate the mergesort chain's two record arenas for streams of up to `total` decompressed bytes now
 * (a long-running caller reserves them once; HBM re-acquired inside a call is wiped by the driver first,
 * ~35-45 GB/s).  *x / *y (cap bytes each) may hold the caller's data between chain calls. */
int oge_mergesort_reserve(oge_ctx *ctx, uint64_t total, void **x, void **y, uint64_t *cap);

/* ---- the whole mergesort chain on a BAM file resident in HBM -------------------------- */
/* FileReader -> ReadSorter -> [MarkDuplicates] -> FileWriter as MergeSortCommand::runCommand wires
 * it (commands/command_mergesort.cpp:68-117), every stage on the device: BGZF framing index,
 * inflate + CRC check, record walk, coordinate sort (+ duplicate marking, -M), optional removal
 * (-R), header regeneration (SO:coordinate, @PG unless program_line is NULL = --nopg), BGZF
 * deflate, EOF block.  d_z = the whole input file (4-byte aligned).  On success *d_out points at
 * the whole output BAM file in HBM, valid until the next call on ctx. */
typedef struct oge_mergesort_opts {
    int32_t level;                   /* output BGZF level 0..9 (FileWriter -c; default 6) */
    int32_t mark_duplicates;         /* -M */
    int32_t remove_duplicates;       /* -R (with -M) */
    int32_t compat_nonverbose_index; /* oge_markdup_opts field of the same name */
    int32_t split_chains;            /* oge_markdup_opts field of the same name */
    int32_t pad0;
    const char *program_line;        /* @PG CL, or NULL (--nopg) */
} oge_mergesort_opts;
void oge_mergesort_opts_init(oge_mergesort_opts *o);
int oge_mergesort_bgzf_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const oge_mergesort_opts *o,
                           const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads, uint64_t *n_dup);
/* The same chain on a BAM file in HOST memory with the PCIe transfers overlapped (replaces the reader and
 * writer threads of BgzfInputStream / BgzfOutputStream, util/bgzf_input_stream.cpp:180-206,
 * util/bgzf_output_stream.cpp:252-285): h_z goes up in chunks on a copy stream while the host indexes its
 * framing and the chunks already up are inflated; after the sort the output is deflated in block-aligned
 * segments whose copies down into h_out (out_cap bytes) run on a high-priority stream while the next
 * segment is compressed (OGE_HOSTPIPE_DIRECT=1 with a page-locked h_out of header + oge_bgzf_bound + 28
 * bytes: the deflate writes straight into h_out instead).  The output bytes equal
 * oge_mergesort_bgzf_dev's.  h_z and h_out should be page-locked (oge_host_alloc). */
int oge_mergesort_bgzf_host(oge_ctx *ctx, const uint8_t *h_z, uint64_t zbytes, const oge_mergesort_opts *o, uint8_t *h_out,
                            uint64_t out_cap, uint64_t *out_bytes, uint64_t *n_reads, uint64_t *n_dup);

/* ---- inputs larger than HBM (replaces ReadSorter's spilled runs + k-way merge) ---------- */
/* Receives one output range: n records in HBM (d_off: n + 1 offsets from d_recs), valid during the
 * call; ranges arrive in output order.  Non-zero return aborts the sort with that status. */
typedef int (*oge_range_cb)(void *user, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n);
/* mergesort [-M] of records in HOST memory of any size on one GPU (alg/read_sorter.cpp:48-190,
 * util/read_stream_reader.h:132-153): sorted runs of <= chunk_bytes (0 = sized from free HBM) are
 * written back over the input arena (h_recs is the spill space and holds the runs afterwards;
 * h_off[0..n] is read-only), key ranges that fit HBM are cut from the runs and sorted on the device,
 * and with opts != NULL the duplicate marks of the whole input are computed on a device-resident
 * summary array first (64 B/read + ~140 B/read of scratch).  Output = oge_sort_markdup_dev's, handed
 * to cb range by range.  *n_runs / *n_ranges (optional) report the cut. */
int oge_sort_markdup_chunked(oge_ctx *ctx, uint8_t *h_recs, const uint64_t *h_off, uint64_t n, int32_t n_ref,
                             const oge_markdup_opts *opts, uint64_t chunk_bytes, oge_range_cb cb, void *user,
                             uint64_t *n_dup, uint64_t *n_runs, uint64_t *n_ranges);
/* free / total bytes of the context's device memory */
int oge_mem_info(oge_ctx *ctx, uint64_t *free_bytes, uint64_t *total_bytes);

/* ---- multi-GPU sort + duplicate marking (replaces SplitByChromosome / SortedMerge) ------ */
/* One rank per GPU.  The reference parallelises mergesort -M / dedup by routing refID % K to K
 * MarkDuplicates chains and re-merging them (alg/split_by_chromosome.cpp:30-58,
 * alg/sorted_merge.cpp:66-101, wired by cmd/command_mergesort.cpp:118-179 and
 * cmd/command_dedup.cpp:70-113); here G ranks split the ByPosition key range with sampled
 * splitters, exchange records over RCCL (xGMI), and mark duplicates exactly (= --nosplit on one
 * GPU) with hash-routed mate-join and pair-group exchanges.  Every call below is collective: all
 * ranks of a communicator make it, in the same order. */
typedef struct oge_comm oge_comm;
/* Communicator id for oge_comm_init_rank (made by one rank, shared by the caller): RCCL's unique id
 * plus a random nonce naming the node-local meeting of ranks that share a GPU. */
uint64_t oge_comm_unique_id_bytes(void);
int oge_comm_unique_id(uint8_t *id_out, uint64_t bytes);
/* One rank per process (or per host thread): rank `rank` of `nranks`, every rank with the same id,
 * concurrently.  Transport (OGE_COMM = auto | rccl | host, default auto): RCCL over xGMI between
 * distinct GPUs; "host" (device -> shared host segment -> device, dist_shm.h) when ranks share a GPU,
 * which RCCL refuses -- so the same bootstrap runs on a one-GPU box.  auto takes RCCL when the
 * process sees >= nranks devices, else compares the ranks' PCI bus ids in the shared segment
 * (OGE_COMM_DIR, default /dev/shm or /tmp; OGE_COMM_STAGE_MB per-rank staging, default 32). */
int oge_comm_init_rank(oge_ctx *ctx, int nranks, int rank, const uint8_t *id, oge_comm **out);
/* The same with the transport chosen by the caller (mode "auto" | "rccl" | "host" | "node"; NULL =
 * OGE_COMM).  In auto mode with fewer visible devices than ranks, the shared-segment meeting is tried
 * only when the launcher says every rank is on this node (LOCAL_WORLD_SIZE / OMPI_COMM_WORLD_LOCAL_SIZE /
 * MPI_LOCALNRANKS == nranks); otherwise RCCL, the only transport that reaches other hosts.  "node" =
 * OGE_COMM's choice with every rank known to be on this node.  The CLI, whose ranks are threads of one
 * process, passes "host" when they share a device, else "node".  RCCL ranks on one node exchange their
 * small host-side values (statuses, counts, splitter samples) through a shared segment instead of a
 * device round trip (OGE_COMM_HOSTX=0: the device round trip). */
int oge_comm_init_rank_mode(oge_ctx *ctx, int nranks, int rank, const uint8_t *id, const char *mode, oge_comm **out);
/* Per-exchange record of the communicator's last oge_sort_markdup_dist / oge_mergesort_bgzf_dist /
 * oge_mergesort_bgzf_shard / oge_bgzf_decode_shard call:
 * a JSON array of {tag, calls, bytes_sent, bytes_recv, bytes_self, ms, device_ms, mode} (bytes to / from
 * other ranks and kept on this rank; host wall time of the collectives, waiting for peers included; RCCL's
 * time on its stream; mode: blocking | side_stream for device exchanges, host_memory | device_round_trip
 * for the host-side allgathers).  Returns the JSON
 * length; writes it (NUL-terminated) when cap > length. */
int64_t oge_comm_stats_json(const oge_comm *comm, char *buf, uint64_t cap);
/* One process, n contexts in one call (test harness): RCCL when the contexts' devices are distinct,
 * else (or with OGE_COMM=local) an in-process hub of device-to-device copies.  out[0..n) receives one
 * communicator per context.  The CLI uses oge_comm_init_rank from one thread per rank instead. */
int oge_comm_init(oge_ctx **ctxs, int n, oge_comm **out);
void oge_comm_destroy(oge_comm *comm);
int oge_comm_rank(const oge_comm *comm);
int oge_comm_size(const oge_comm *comm);
const char *oge_comm_transport(const oge_comm *comm); /* "rccl", "host" or "local" */
/* This rank's shard of the input: contiguous input ranges in rank order (any sizes, empty ones
 * included).  sort != 0 (mergesort [-M]): -> this rank's slice of the globally sorted output, with
 * bin recomputed and, when opts != NULL, 0x400 set/cleared exactly as oge_sort_markdup_dev does on
 * the whole input.  sort == 0 (dedup): the shard keeps its records and their order, marked exactly
 * as oge_markdup_dev marks the whole input (record index = input position).  compat_nonverbose_index
 * is one-GPU only.  Concatenating the slices in rank order gives the one-GPU output.  *d_out /
 * *d_out_off (*n_out + 1 offsets) are owned by the rank's context and valid until its next call;
 * *n_dup_total = 0x400 records over all ranks.  d_off[i] are byte offsets from d_recs. */
/* The whole mergesort [-M] [-R] chain (oge_mergesort_bgzf_dev) over the communicator's ranks: rank g
 * passes its own input BAM file (resident in its HBM; the output header is rank 0's file's, as
 * MultiReader takes the first file's), and *d_out receives rank g's slice of the one output file --
 * rank 0's begins with the header, the last rank's ends with the EOF block, so the slices concatenate
 * in rank order (valid until the rank's next call).  *n_reads_total: records written by all ranks. */
int oge_mergesort_bgzf_dist(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, const oge_mergesort_opts *o,
                            const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads_total, uint64_t *n_dup_total);
int oge_sort_markdup_dist(oge_comm *comm, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, int32_t n_ref, int sort,
                          const oge_markdup_opts *opts, uint8_t **d_out, uint64_t **d_out_off, uint64_t *n_out,
                          uint64_t *n_dup_total);
/* ONE BGZF BAM file read by every rank from its own byte range (config 4 on the node; replaces the
 * reader thread of BgzfInputStream util/bgzf_input_stream.cpp:180-206 + BamDeserializer::read
 * util/bam_deserializer.h:143-193 feeding SplitByChromosome, cmd/command_mergesort.cpp:118-179).  Rank g
 * holds the file's bytes [a_g, a_g + zbytes) in HBM, a_g = the sum of the earlier ranks' own_bytes, and
 * decodes the BGZF blocks that START in [a_g, a_g + own_bytes): the buffer must hold them whole (own_bytes
 * + 65536 bytes, or up to the end of the file, which the last rank's buffer ends at; zbytes >= own_bytes).
 * The ranks confirm their first block / first record with their predecessors' walk exits (allgathers)
 * and fetch the <= 16 KiB tail of the record that straddles their part's end from the next ranks (an
 * all-to-all).  Out: this rank's records -- those that START in its part of the decompressed stream, in
 * file order, complete in its HBM (*d_off: n + 1 offsets into *d_recs, library workspace valid until the
 * next call on the rank's context) -- and the raw BAM header (rank 0's, shared), copied to hdr_out when
 * hdr_cap holds it (*hdr_len = its length; OGE_ERR_LIMIT otherwise).  The rank shards are contiguous
 * input ranges in rank order: oge_sort_markdup_dist's input.  Collective. */
int oge_bgzf_decode_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own_bytes, const uint8_t **d_recs,
                          const uint64_t **d_off, uint64_t *n, uint8_t *hdr_out, uint64_t hdr_cap, uint64_t *hdr_len);
/* oge_mergesort_bgzf_dist over ONE input file sharded by byte range as oge_bgzf_decode_shard takes it:
 * every rank inflates ~1/G of the blocks, then the range-split sort + exact dedup, then every rank
 * deflates its slice of the output file (rank 0's with the header, the last rank's with the EOF block). */
int oge_mergesort_bgzf_shard(oge_comm *comm, const uint8_t *d_z, uint64_t zbytes, uint64_t own_bytes, const oge_mergesort_opts *o,
                             const uint8_t **d_out, uint64_t *out_bytes, uint64_t *n_reads_total, uint64_t *n_dup_total);
/* Device synthetic generation of the slot range [slot0, slot0 + nslots) of a data set (one rank's
 * shard of a multi-GPU input). */
int oge_synth_offsets_range_dev(oge_ctx *ctx, const void *params, uint64_t slot0, uint64_t nslots, uint64_t *d_offs);
int oge_synth_records_range_dev(oge_ctx *ctx, const void *params, uint64_t slot0, uint64_t nslots,
                                const uint64_t *d_offs, uint8_t *d_out);

/* ---- local realignment (LocalRealignment) ----------------------------------------- */
/* Offset scan, the realigner's hot loop: for every pair (consensus c, altRead r) the best
 * offset of r on c and its mismatch-quality score, exactly as findBestOffset returns them
 * (algorithms/local_realignment.cpp:1126-1164 over mismatchQualitySumIgnoreCigar :641-679).
 * cons / bases are ASCII bases; quals are raw phred bytes (BAM layout) aligned with bases;
 * pairs holds n_pairs x {cons index, read index, orig offset, maxPossibleStart}. */
typedef struct oge_realign_scan_batch {
    const uint8_t *cons;
    uint64_t cons_bytes;
    const uint64_t *cons_off;   /* n_cons + 1 */
    uint32_t n_cons;
    uint32_t n_reads;
    const uint8_t *bases;
    const uint8_t *quals;
    uint64_t read_bytes;
    const uint64_t *read_off;   /* n_reads + 1 */
    const int32_t *pairs;
    uint64_t n_pairs;
} oge_realign_scan_batch;
int oge_realign_scan(oge_ctx *ctx, const oge_realign_scan_batch *batch, int32_t *best_index, int32_t *best_score);

/* LocalRealignment's tunables (constructor constants, algorithms/local_realignment.cpp:1434-1460) */
typedef struct oge_realign_opts {
    double lod_threshold;            /* 5.0 */
    double mismatch_threshold;       /* 0.15 (entropy) */
    int32_t max_records_in_memory;   /* 150000 */
    int32_t max_isize_for_movement;  /* 3000 */
    int32_t max_pos_move_allowed;    /* 200 */
    int32_t max_reads;               /* 20000 */
    int32_t no_original_alignment_tags;
    int32_t threads;                 /* host threads, 0 = all cores */
} oge_realign_opts;
void oge_realign_opts_init(oge_realign_opts *opts);

/* Whole LocalRealignment module (map_func binning, consensus generation, offset scan on the GPU,
 * LOD / entropy decision, CIGAR + tag updates, ConstrainedMateFixingManager emission) over
 * coordinate-sorted records; replaces LocalRealignment::runInternal
 * (algorithms/local_realignment.cpp:1462-1490) with the writer chain of
 * cmd/command_localrealign.cpp:37-75.  header_text supplies the sequence dictionary. */
typedef struct oge_realign_result oge_realign_result;
int oge_localrealign(oge_ctx *ctx, const char *header_text, uint64_t header_len, const uint8_t *recs,
                     const uint64_t *rec_off, uint64_t n, const char *fasta_path, const char *intervals_path,
                     const oge_realign_opts *opts, oge_realign_result **out);
/* The same over n_ctx devices (realign sharded by interval ranges).  The work intervals are cut
 * into n_ctx contiguous ranges balanced by the reads to clean -- cuts fall inside contigs as well, a
 * single-contig input included -- and device g generates the consensuses of range g and scans their pairs
 * (realign_prep.hip, realign.hip); binning, decisions and the mate-fixing writer run once on the host over
 * the whole input, so the output equals oge_localrealign's for any input and no writer state crosses a cut.
 * Per-device counts are in the result's stats (prep_rank<g>_intervals / _reads / _pairs).  Errors and
 * messages go to ctxs[0]. */
int oge_localrealign_multi(oge_ctx *const *ctxs, int n_ctx, const char *header_text, uint64_t header_len, const uint8_t *recs,
                           const uint64_t *rec_off, uint64_t n, const char *fasta_path, const char *intervals_path,
                           const oge_realign_opts *opts, oge_realign_result **out);
uint64_t oge_realign_result_count(const oge_realign_result *r);
const uint8_t *oge_realign_result_records(const oge_realign_result *r, uint64_t *bytes_out);
const uint64_t *oge_realign_result_offsets(const oge_realign_result *r);   /* count + 1 entries */
const char *oge_realign_result_stats(const oge_realign_result *r);          /* JSON */
void oge_realign_result_free(oge_realign_result *r);

/* ---- synthetic data (bench / tests) ------------------------------------------------ */
/* params: a pointer to oge_synth_params (openge_amd/csrc/synth.h) */
int oge_synth_finalize(void *params);
uint64_t oge_synth_params_size(void);
/* Host generation of slots [0, 2*n_pairs): sizes first (offs gets n+1 prefix offsets), then bytes. */
int oge_synth_offsets_host(const void *params, uint64_t *offs, int threads);
int oge_synth_records_host(const void *params, const uint64_t *offs, uint8_t *out, int threads);
int oge_synth_header_text(const void *params, char *buf, uint64_t cap, uint64_t *len_out);
/* Local-realignment data set (SURVEY §8d C5 shape; openge_amd/csrc/realign_synth.cpp): writes a
 * reference FASTA (+ .fai), a target-interval list and a coordinate-sorted BAM. */
typedef struct oge_realign_synth_params {
    uint64_t seed;
    uint32_t n_ref, n_intervals, spacing, read_len, frags_per_interval;
    uint32_t qual_min, qual_max, ins_min, ins_max;
    uint32_t err_ppm, noindel_ppm, gapped_ppm, alt_indel_ppm, dup_ppm, mapq0_ppm, clip_ppm;
    uint32_t lower_ppm, n_ppm, md_ppm, uq_ppm;
} oge_realign_synth_params;
void oge_realign_synth_defaults(oge_realign_synth_params *p);   /* C5: 50k intervals, 24 contigs */
int oge_synth_realign(const oge_realign_synth_params *p, const char *fasta_path, const char *intervals_path,
                      const char *bam_path, int level, int threads);
/* Device generation straight into HBM. */
int oge_synth_offsets_dev(oge_ctx *ctx, const void *params, uint64_t *d_offs);
int oge_synth_records_dev(oge_ctx *ctx, const void *params, const uint64_t *d_offs, uint8_t *d_out);

/* ---- BAM file helpers (host) -------------------------------------------------------- */
typedef struct oge_bam oge_bam;
int oge_bam_read(const char *path, int threads, oge_bam **out);
void oge_bam_free(oge_bam *b);
uint64_t oge_bam_count(const oge_bam *b);
const uint8_t *oge_bam_records(const oge_bam *b, uint64_t *bytes_out);
const uint64_t *oge_bam_offsets(const oge_bam *b);
int32_t oge_bam_n_ref(const oge_bam *b);
/* regenerated header text (BamHeader::toString, util/bam_header.cpp:184-214) */
int oge_bam_header_text(const oge_bam *b, char *buf, uint64_t cap, uint64_t *len_out);
/* Build the RG -> library table MarkDuplicates derives from the header. Caller frees with free(). */
int oge_bam_markdup_opts(const oge_bam *b, oge_markdup_opts *opts, char **rg_ids_buf, int16_t **rg_lib_buf);
/* Write a BGZF BAM: header from `header_text`, records in the given order (order may be NULL
 * for identity), optional FLAG overrides (flags may be NULL). sort_order: -1 keep, else
 * BamHeader::sort_order_t. */
int oge_bam_write(const char *path, const char *header_text, uint64_t header_len, int sort_order,
                  const uint8_t *recs, const uint64_t *offs, uint64_t n, const uint32_t *order,
                  const uint16_t *flags, int level, int threads);

/* ---- BGZF compression on the device (replaces BgzfOutputStream's deflate workers,
 * util/bgzf_output_stream.cpp:59-250; crc32 at :139) ---------------------------------- */
/* Worst-case size of the BGZF stream for n payload bytes (one 64 KiB slot per 65,280-byte block). */
uint64_t oge_bgzf_bound(uint64_t n);
/* Compress n bytes at d_src into consecutive BGZF blocks (65,280-byte payloads; dynamic-Huffman
 * deflate, or stored blocks for level 0 / incompressible payloads) written back to back at d_dst.
 * No EOF marker is appended.  dst_cap must be >= oge_bgzf_bound(n); *out_bytes = stream size.
 * Levels 1-7: greedy one-candidate parse; 8-9: same-prefix match chains (8 / 32 deep) with lazy
 * matching, ~1 % smaller output at 1.7-3x the time.  Deterministic: the same input gives the same bytes. */
int oge_bgzf_deflate_dev(oge_ctx *ctx, const uint8_t *d_src, uint64_t n, int level, uint8_t *d_dst,
                         uint64_t dst_cap, uint64_t *out_bytes);
/* Host-buffer form (uploads, compresses, downloads); dst_cap >= the compressed size. */
int oge_bgzf_deflate(oge_ctx *ctx, const uint8_t *src, uint64_t n, int level, uint8_t *dst, uint64_t dst_cap,
                     uint64_t *out_bytes);
/* ---- BGZF decompression and BAM record boundaries on the device (replaces BgzfInputStream,
 * util/bgzf_input_stream.cpp:65-142,208-240, and BamDeserializer's record walk,
 * util/bam_deserializer.h:143-193) ------------------------------------------------------ */
/* Host: index the BGZF framing of z.  For each block with a non-empty payload (at most cap):
 * d0/d1 = byte range of its deflate data in z, uoff = payload offset (uoff has cap + 1 entries;
 * uoff[nblk] = total), crc = the stored CRC-32.  Any array may be NULL.  *nblk = block count
 * (OGE_ERR_ARG when it exceeds cap). */
int oge_bgzf_index(const uint8_t *z, uint64_t zbytes, uint64_t *d0, uint64_t *d1, uint64_t *uoff, uint32_t *crc,
                   uint64_t cap, uint64_t *nblk);
/* Device form of oge_bgzf_index for a stream resident in HBM (d_z 4-byte aligned): every byte
 * position is tested for a block header in parallel and the candidates are accepted only when they
 * form the exact block chain from offset 0 to zbytes (otherwise the host walk runs on a copy, with
 * its error messages).  Same outputs and capacity rule as oge_bgzf_index, as device arrays; with every
 * array NULL it only counts (*nblk). */
int oge_bgzf_index_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, uint64_t *d_d0, uint64_t *d_d1,
                       uint64_t *d_uoff, uint32_t *d_crc, uint64_t cap, uint64_t *nblk);
/* Inflate the indexed blocks of d_z (4-byte aligned) into d_out + uoff[i]; d_crc (may be NULL)
 * checks every payload's CRC-32.  Fails with OGE_ERR_IO on corrupt data. */
int oge_bgzf_inflate_dev(oge_ctx *ctx, const uint8_t *d_z, uint64_t zbytes, const uint64_t *d_d0, const uint64_t *d_d1,
                         const uint64_t *d_uoff, const uint32_t *d_crc, uint64_t nblk, uint8_t *d_out);
/* Host-buffer form: the whole BGZF stream z -> out (out_cap >= payload total). */
int oge_bgzf_inflate(oge_ctx *ctx, const uint8_t *z, uint64_t zbytes, uint8_t *out, uint64_t out_cap,
                     uint64_t *out_bytes);
/* Record boundaries of the decompressed BAM stream d_stream[rec_base, end): d_off[i] = absolute
 * offset of record i, d_off[n] = end (cap >= n + 1; d_off NULL = count only).  Equals the sequential
 * block_size walk; block_size outside [32, 10000] or a record past the end fails (OGE_ERR_IO). */
int oge_bam_record_offsets_dev(oge_ctx *ctx, const uint8_t *d_stream, uint64_t rec_base, uint64_t end, int32_t n_ref,
                               uint64_t *d_off, uint64_t cap, uint64_t *n_out);
/* Recompute every record's bin field in place (BamSerializer::write, util/bam_serializer.h:112-116). */
int oge_fix_bins_dev(oge_ctx *ctx, uint8_t *d_recs, const uint64_t *d_off, uint64_t n);
/* Copy the records whose FLAG has none of flag_mask set, in order, to d_out / d_out_off (n_out
 * records): the writer side of -r/-R (MarkDuplicates::runInternal, mark_duplicates.cpp:456-458). */
int oge_drop_flagged_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, uint16_t flag_mask,
                         uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_out);

/* ---- mergesort extras: Filter (-r region / -q mapq) and sort by name (-b) ----------- */
/* Filter::runInternal's predicate (algorithms/filter.cpp:205-249) with the module's setters
 * (filter.h:34-47).  len = l_seq (BamAlignment::getLength).  A record is kept when
 *   mapq >= mapq_min && min_len <= len <= max_len && len > trim_total
 *   [&& ref_id <= refID <= ref_id && pos + len >= left_pos && pos <= right_pos   if has_region]
 * and at most count_limit records (the first ones kept, in input order) are kept. */
typedef struct oge_filter_opts {
    int32_t has_region;
    int32_t ref_id;       /* region refID (Filter::ParseRegionString) */
    int32_t left_pos;     /* region start, 0-based as the reference compares it */
    int32_t right_pos;    /* region stop */
    int32_t mapq_min;     /* setQualityLimit, default 0 */
    int32_t min_len;      /* setMinimumReadLength, default 0 */
    int32_t max_len;      /* setMaximumReadLength, default INT32_MAX */
    int32_t trim_total;   /* trim_begin_length + trim_end_length, default 0 */
    uint64_t count_limit; /* setCountLimit, default INT32_MAX */
} oge_filter_opts;
/* Defaults of Filter::Filter() (filter.cpp:185-194). */
void oge_filter_opts_init(oge_filter_opts *o);
/* Filter::ParseRegionString (filter.cpp:31-137): "chr", "chr:pos" or "chr:start..stop" against the
 * header's sequence dictionary (ref_names = n_ref NUL-terminated names back to back, ref_len =
 * their LN).  Fills has_region/ref_id/left_pos/right_pos; OGE_ERR_ARG with the reference's message
 * (oge_last_error(NULL)) when the region does not parse or lies outside the sequence. */
int oge_parse_region(const char *region, const char *ref_names, int32_t n_ref, const int64_t *ref_len,
                     oge_filter_opts *o);
/* Copy the records the filter keeps, in input order, to d_out / d_out_off (*n_out records). */
int oge_filter_records_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n,
                           const oge_filter_opts *o, uint8_t *d_out, uint64_t *d_out_off, uint64_t *n_out);
/* Sort::ByName (util/bamtools/Sort.h:67-90) as ReadSorter uses it for SORT_QUERYNAME
 * (algorithms/read_sorter.cpp:202-203): read names compared bytewise (std::string <); records
 * with equal names keep input order (the reference's std::sort leaves their order
 * implementation-defined).  d_perm (n) receives the input index of each output position. */
int oge_sort_name_dev(oge_ctx *ctx, const uint8_t *d_recs, const uint64_t *d_off, uint64_t n, uint32_t *d_perm);
int oge_sort_name(oge_ctx *ctx, const uint8_t *recs, uint64_t rec_bytes, const uint64_t *rec_off, uint64_t n,
                  uint32_t *perm_out);

#ifdef __cplusplus
}
#endif
#endif /* OPENGE_HIP_H */
