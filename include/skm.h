/*
 * skm.h -- C-ABI of libskm, the MI355X-native signature-k-mer engine.
 *
 * This is the drop-in boundary for the reference's hot path (olsonanl/signature_kmers @ 2024-11-15).
 * The reference has no FFI; its boundary is a C++ template API.  Each entry point below names the
 * reference interface it replaces (paths relative to the reference's src/).
 *
 * Conventions
 *   - Plain C types only.  No exceptions cross the boundary.
 *   - Return value: 0 = OK, < 0 = error class (SKM_E_*).  skm_last_error() holds a message
 *     (thread-local).
 *   - Host buffers passed in are caller-owned and are copied before the call returns.
 *   - Buffers returned in out-structs are library-owned; release them with the matching *_free.
 *   - A k-mer key is the 8 residue bytes as a little-endian uint64 (byte 0 = first residue),
 *     i.e. Kmer<8> = std::array<char,8> reinterpreted (kmer_data.h:37).
 *   - Handles are driven from one host thread at a time.
 */
#ifndef SKM_H
#define SKM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKM_OK 0
#define SKM_E_ARG -1      /* invalid argument / limit exceeded                    */
#define SKM_E_HIP -2      /* HIP runtime error (incl. no device)                  */
#define SKM_E_OOM -3      /* device or host allocation failed                     */
#define SKM_E_IO -4       /* file I/O or format error                             */
#define SKM_E_COMM -5     /* RCCL error                                           */
#define SKM_E_STATE -6    /* call out of order                                    */

#define SKM_UNDEFINED_FUNCTION 0xFFFFu /* kmer_data.h:23 UndefinedFunction */

/* StoredKmerData (kmer_data.h:114-128): five little-endian u16, 10 bytes, the kmer_data.dat
 * record (perfect_hash.h:62 writes sizeof(StoredKmerData)=10 per MPH slot).  Natural layout:
 * sizeof 10, alignof 2, offsets 0/2/4/6/8 -- equal to the reference as g++ compiles it
 * (tests/golden/ref_split.npz `layout`, tests/test_ref_pin_cpu.py). */
typedef struct skm_stored_kmer_data {
    uint16_t avg_from_end;
    uint16_t function_index;
    uint16_t mean;
    uint16_t median;
    uint16_t var;
} skm_stored_kmer_data;

/* KmerCall (call_functions.h:23-48). 24 bytes. */
typedef struct skm_kmer_call {
    uint32_t start;
    uint32_t end;
    int32_t count;
    uint16_t function_index;
    uint16_t pad;
    uint32_t protein_length_median;
    float protein_length_med_avg_dev;
} skm_kmer_call;

const char* skm_last_error(void);
const char* skm_version(void);
int skm_device_count(int* n);

/* ------------------------------------------------------------------------------------------
 * Signature build.  Replaces SignatureBuilder<K>::extract_kmers + process_kmers
 * (signature_build.h:55-110, signature_build.tcc:48-293) as driven by kmers-build-signatures.cc
 * :193-196, and the consumers kept_kmers()/kmer_stats() (signature_build.h:106-107).
 * ------------------------------------------------------------------------------------------ */
typedef struct skm_build skm_build;

typedef struct skm_build_opts {
    int32_t k;                  /* must be 8 (kmers-build-signatures.cc:17 K=8)                 */
    uint32_t max_seqs_per_file; /* 100000 (kmers-build-signatures.cc:18); informational        */
    uint32_t n_functions;       /* size of function.index (FunctionIndex upper bound, < 65535)  */
    int32_t canonical_order;    /* 1: n_threads=1 reference semantics (the only mode)           */
    int32_t rank;               /* this process's rank (0 for single GPU)                        */
    int32_t world_size;         /* number of GPUs/processes: 1, 2, 4 or 8                        */
} skm_build_opts;

/* Kept k-mers (KeptKmers<8>, signature_build.h:52-53) + KmerStatistics (:44-50). */
typedef struct skm_kept {
    uint64_t* keys;                  /* [n] k-mer keys, sorted ascending                       */
    skm_stored_kmer_data* data;      /* [n] packed 10-byte records                              */
    uint64_t n;                      /* kept k-mers ("Kept N kmers")                            */
    uint32_t* distinct_functions;    /* [n_functions] kept k-mers per best function              */
    uint32_t* seqs_with_func;        /* [n_functions] sequences per function                    */
    uint32_t n_functions;
    uint64_t n_seqs_with_signature;  /* "num_seqs_with_a_signature="                            */
    uint64_t distinct_signatures;    /* "distinct_signatures="                                  */
    uint64_t n_windows;              /* windows examined (metric units)                         */
    uint64_t n_records;              /* valid windows (occurrences)                             */
} skm_kept;

/* devices: HIP device ordinals (n_devices == 1 per process; multi-GPU is one process per GPU). */
int skm_build_create(skm_build** out, const int* devices, int n_devices, const skm_build_opts* opts);

/* One batch of sequences in reference emission order (file order, then sequence order).
 * residues: concatenated residue bytes; sequence s is residues[seq_off[s] .. +seq_len[s]).
 * seq_func: FunctionIndex of the sequence's assigned function, or 0xFFFF when the sequence has
 *           no kept function (the reference skips it, signature_build.tcc:133-158).
 * seq_id:   file_number*max_seqs_per_file + k (signature_build.tcc:91,138).                   */
int skm_build_add_batch(skm_build* b, const uint8_t* residues, const uint64_t* seq_off,
                        const uint32_t* seq_len, const uint16_t* seq_func, const uint32_t* seq_id,
                        size_t n_seqs);

/* Optional capacity hint: the total residues and sequences that will be added, so the HBM
 * residue buffer is allocated once instead of grown.  Batches stream to HBM as they are added,
 * packed into two pinned staging buffers that alternate (the host packs one while the DMA engine
 * copies the other); the caller may overlap parsing with add_batch (kmers-build-signatures does).
 * Replaces nothing in the reference (its build reads the FASTA into host memory,
 * signature_build.tcc:48-70); new in this port. */
int skm_build_reserve(skm_build* b, uint64_t n_residues, uint64_t n_seqs);

/* Flush the last staging buffer, pack the metadata into HBM (idempotent). */
int skm_build_prepare(skm_build* b);
/* Run the device pipeline over the resident input; results stay on the device. */
int skm_build_run(skm_build* b);
/* Device time (ms) of the last run's phases: [0]=extract-count [1]=scan [2]=extract-scatter
 * [3]=bucket-process (partition + group-by) [4]=overflow (own stream, overlaps [3]) [5]=chains
 * [6]=stats (+ reductions) [7]=total [8]=exchange (world_size > 1) [9]=level-2 partition kernel
 * [10]=group-by kernel alone [11]=groups of > 64 members (k_big_groups + append);
 * returns entries written. */
int skm_build_last_timings(skm_build* b, float* ms, int cap);
/* [12] of skm_build_last_timings: the long-chain tail -- device time from the end of the last
 * key-range pass on the group-by stream until the last stashed P^2 / variance chain is done.
 * [13], [14]: the start and end of the run's first giant-chain launch (k_heavy's chains of
 * >= 2^giant_class samples; with route_first the heavy-only pass 0's), in ms from the run's
 * start; -1 when no giant chain ran. */
/* Per-kernel device time (diagnostics and the bench's roofline): with enable != 0 every kernel
 * launch of a run -- or only the launches of the kernel named `only` (e.g. "k_bucket_process";
 * NULL = all) -- is bracketed by an event pair on its stream, and after the run's host
 * synchronisation the durations are summed by kernel name.  skm_build_kernel_timings returns the
 * number of kernels of the last run and writes, for the first `cap`, the total ms and launch count
 * and (names != NULL) their names, one per line.  New in this port (the reference has no device
 * code; its only timing is the stderr phase banners, kmers-build-signatures.cc:178-325). */
int skm_build_set_kernel_timing(skm_build* b, int enable, const char* only);
int skm_build_kernel_timings(skm_build* b, char* names, size_t names_cap, float* ms, uint64_t* launches, int cap);
/* Counters of the last run: [0]=windows [1]=kept (owned by this rank) [2]=overflow sub-buckets
 * [3]=chain jobs [4]=chain samples [5]=sequences [6]=occurrences grouped on this rank
 * [7]=occurrences in overflow sub-buckets [8]=k-mers kept by the overflow path
 * [9]=groups of > 64 members handed to k_big_groups [10]=k-mers kept among them
 * [11]=key-range passes [12]=valid windows (occurrences) this rank extracts [13]=giant chains
 * (heavy k-mers whose P^2 / variance chains start right after k_heavy) [14]=the longest of them
 * [15]=redone steps since create (a run that outgrew a data-sized work buffer -- the overflow
 * scratch, the split path, the stashed long chains -- records its demand and is redone once with
 * the buffers grown; the capacities persist, so later runs on the same input are not)
 * [16..19]=capacities of those buffers (overflow scratch elements, split-path elements, stashed
 * long-chain samples, stashed long jobs) [20..23]=the last run's demands on them [24]=samples of
 * the stashed long chains (chains of >= 2^14 samples with key-range passes) [25]=occurrences of
 * heavy k-mers routed into the first half of the key-range passes ("route_heavy_min");
 * [26]=host microseconds in skm_build_add_batch (all calls; the residues are packed by a pool of
 * host threads, SKM_HOST_THREADS or min(16, hardware threads)), and prepare's phases in
 * microseconds: [27] the residue / metadata upload, [28] the pass plan (device tallies of the pass
 * sizes, heavy-key routing sketch and filter), [29] allocations and the rest; [30] residue scans
 * per run that emit the key-range passes' window positions (k_pass_emit, one per group of up to
 * four passes; 0 without key-range passes); [31] of [26]: microseconds packing residues into the
 * pinned staging buffers, [32] of [26]: microseconds waiting for a staging buffer's DMA to end;
 * totals over the passes of the run; the last skm_build_finish / _finish_slice's kept-set
 * hand-off (device radix sort in key-range chunks, streamed through pinned staging): [33] its
 * host microseconds, [34] of them waiting for the device / PCIe, [35] copying pieces out on the
 * host pool, [36] chunks, and its device microseconds summed over the chunks: [37] selection,
 * [38] radix sort, [39] gather, [40] the D2H pieces; [41] the largest hand-off chunk (k-mers),
 * [42] 1 if the hand-off used 64-bit arena indices (>= 2^32 k-mers); [43] the kept arena's
 * capacity (k-mers); [44] device bytes free after prepare; [45] 1 if the passes alternate two
 * element buffers ("recs_rot"); returns entries written. */
int skm_build_counters(skm_build* b, uint64_t* out, int cap);
/* Host transport: the rank collectives of a multi-process build run by the caller on host
 * buffers, for ranks joined by a channel other than RCCL (the tests drive it with
 * torch.distributed gloo; production multi-GPU runs use skm_build_set_comm).  The library stages
 * device data through host memory around each call.  Every callback returns 0 on success. */
typedef struct skm_transport {
    void* ctx;
    /* variable all-to-all (bytes): send + soff[q] (scnt[q] bytes) goes to rank q, which receives
     * it at recv + roff[p] (rcnt[p] bytes) for source p */
    int (*alltoallv)(void* ctx, const void* send, const uint64_t* scnt, const uint64_t* soff, void* recv,
                     const uint64_t* rcnt, const uint64_t* roff);
    /* in-place element-wise reduction over the ranks: op 0 = u32 sum (mod 2^32), 1 = u8 max */
    int (*allreduce)(void* ctx, void* data, uint64_t count, int op);
    /* every rank's bytes_per_rank[r] bytes, concatenated in rank order into recv */
    int (*allgatherv)(void* ctx, const void* send, void* recv, const uint64_t* bytes_per_rank);
} skm_transport;
/* Join the ranks through a host transport instead of RCCL (world_size > 1; copied). */
int skm_build_set_transport(skm_build* b, const skm_transport* tp);
/* Test hooks (host only, no device): the exchange planning of one key-range pass as rank `rank`
 * of `world`: bucket_starts [world*nb1+1] are this rank's owner-major level-1 bucket starts; the
 * per-bucket counts go through tp->alltoallv; out: recv_off/recv_cnt [world] (elements, source
 * order) and vstart [nb1+1] (bucket-major starts of the received elements).  And a self-check of
 * the three callbacks (returns 0 when every collective gave the expected result). */
int skm_debug_exchange_plan(const skm_transport* tp, int rank, int world, uint32_t nb1, const uint64_t* bucket_starts,
                            uint64_t* recv_off, uint64_t* recv_cnt, uint64_t* vstart);
int skm_debug_transport_check(const skm_transport* tp, int rank, int world);

/* Build options beyond skm_build_opts (take effect at the next prepare/run):
 *   "key_range_passes"        0 = automatic; else P = 1, 2, 4 .. 64 passes over disjoint k-mer
 *                             ranges (top bits of the key hash).  The reference holds the whole
 *                             proteome in one multimap (signature_build.h:61,122); a GPU shard
 *                             whose occurrences exceed the work buffers is grouped pass by pass,
 *                             with identical results (each k-mer lives in exactly one pass).
 *   "device_memory_budget_mb" memory the automatic pass count plans for (0 = free memory).
 * Diagnostic tunables (defaults are the tuned values): "overflow_heavy_min",
 *   "overflow_inline_min", "overflow_inline_prio", "overflow_long_class", "overflow_chain_wgs",
 *   "chain_prio", "bucket_prio", "chain_lds_kb", "host_timing",
 *   "heavy_min" (occurrences that send a k-mer to the heavy path), "split_min" (overflow
 *   sub-buckets at least this large are split into heavy keys + a light remainder),
 *   "heavy_lsd" (1: every heavy k-mer through round 3's Boyer-Moore + LSD-sort path instead of
 *   the one-read bucketed path; it is the fallback for > 4096 functions or crowded buckets),
 *   "giant_class" (heavy chains of >= 2^class samples start right after the heavy kernel on
 *   their own streams; 0 = off; default: 14 with one pass or world_size > 1, off with key-range
 *   passes on one GPU),
 *   "giant_passes", "prefetch" (the next pass group's positions, k_pass_emit, during the group-by of the group's
 *   last pass, 1),
 *   "overflow_grid" / "split_grid" / "chain_grid" (persistent-grid sizes), "stream_priority"
 *   (1: the group-by stream at the highest priority), "chain_batches" (key-range passes: the
 *   stashed long chains leave in this many batches, 2) / "chain_streams" (over 1..4 streams, 1),
 *   "work_buffer_elements" (capacity of the data-sized work buffers; tests force the
 *   grow-and-redo path with a small value; 0 = automatic), "poison_jobs" (tests: canary jobs in
 *   the stashed long-job list), "route_heavy_min" (one GPU, >= 4 key-range passes: k-mers with at
 *   least this many occurrences -- estimated at prepare from a count-min sketch of 1/64 of the
 *   windows -- are grouped in the first half of the passes, so their long P^2 chains run beside
 *   the later passes instead of after the last one; 16384; 0 = off), "route_vacate" (the last
 *   this many passes hold no routed heavy key, whose keys are spread over the others by hash;
 *   0 = the second half, mapped to pass - P/2), "route_first" (every routed heavy k-mer in a
 *   heavy-only pass 0, the light keys of pass 0 spread over the others, the pass count doubled
 *   below four passes: 1 = on, 0 = off; default on at world_size > 1), "route_first_min" (its
 *   occurrence threshold, 131072), "tail_async" (one GPU, key-range passes: a pass's big groups,
 *   chains and accounting on their own stream beside the next pass's staging; 1),
 *   "stage_round" (key-range
 *   passes: 1 = the staged position scatter in half rounds of 2048 elements, four workgroups
 *   per CU, the default; 0 = rounds of 4096), "partition_round"
 *   (k_partition staging rounds: 0 = 2048 elements, three 512-thread workgroups per CU (default);
 *   1 = 4096, one per CU; 2 = 4096, one 1024-thread workgroup per CU), "flag_check" (1: the
 *   group-by reads a sequence's signature flag before storing it; 0), "serial_overflow"
 *   (diagnostics: 1 = a pass's overflow path starts after its group-by kernel; 0), "chain_cus"
 *   (the stashed long chains' stream confined to this many CUs, a multiple of 8; 0 = all),
 *   "side_cus" (the same for the overflow streams and the next pass's selection), "overlap"
 *   (key-range passes on one GPU: 1 = pipelined passes -- a second element buffer set when it
 *   fits, so a pass's overflow path runs beside the next pass's extract and partition; 0 = each
 *   pass waits for its overflow path, the default), "heavy_grid" (k_heavy's persistent grid, 512),
 *   "lane_long" (key-range passes: stashed long chains below this many samples run one lane each,
 *   64 chains per wave, instead of on a wave pair; 2^20; 0 = all on wave pairs), "lane_grid"
 *   (their grid, 256), "lane_tail" (the threshold for the batch after the last pass, 2^16),
 *   "lane_streams" (their batches rotate over 1..4 streams, 1), "chain_queue" (1: chain waves take
 *   64-job blocks from a work queue instead of a fixed stride), "flag_bits" (1: signature flags
 *   kept as bits during the run, read before an atomic set; 0: a byte store per kept
 *   occurrence), "sub_target" (k_partition's target elements per level-2 sub-bucket; 0 = 768),
 *   "big_split" (tail_async: the two big-group size classes on two tail streams; 0),
 *   "emit_group" (key-range passes emitted per residue scan: 0 = 4, or 1, 2, 4, 8, 16),
 *   "tail_defer" (tail_async: a pass's tail issued after the next pass's scan kernels; 0),
 *   "recs_rot" (tail_async: the passes alternate two element buffers, so a split does not wait
 *   for the previous pass's tail; +16 B per element of the largest pass when it fits; 0),
 *   "handoff_index_limit" / "handoff_max_chunk" (tests: force the hand-off's 64-bit indices /
 *   small chunks),
 *   "diag" (diagnostics only, wrong results: skips of flag stores / the heavy sort / chain
 *   kernels / overflow entry classes).
 * Unknown names and out-of-range values return SKM_E_ARG. */
int skm_build_set_option(skm_build* b, const char* name, int64_t value);
/* Diagnostics: copy the per-phase cycle sums of the last run (if enabled) into out, then
 * enable/disable stamping for subsequent runs. */
int skm_build_debug_stamps(skm_build* b, int enable, uint64_t* out, int cap);
/* Diagnostics: lengths of the first cap chain jobs of the last pass in execution order (longest
 * first; the overflow's list when the pass had overflow sub-buckets). */
int skm_build_debug_jobs(skm_build* b, uint32_t* out, int cap);
/* Diagnostics: element counts of the last pass's overflow sub-buckets as the partition listed
 * them; returns how many there are (at most cap written). */
int skm_build_debug_overflow(skm_build* b, uint32_t* out, int cap);
/* Diagnostics: device time of the chain kernel on njobs synthetic jobs of length n
 * (mode 0: the build's choice by length, 1: one lane per chain, 2: one wave pair per chain;
 *  3 / 5: the P^2 wave alone, previous / current walk; 4: the variance wave alone). */
int skm_debug_chain_bench(uint32_t n, uint32_t njobs, int mode, float* ms);
/* Diagnostics: the P^2 median and the variance (raw doubles) of one chain of n samples in visit
 * order, by the per-lane (mode 1) or the wave-pair (mode 2) chain code. */
int skm_debug_chain_eval(const uint32_t* samples, uint32_t n, int mode, double* median, double* var);
/* Diagnostics: device exact-division helpers (reciprocal + corrected quotient used by the
 * statistics recurrences) against IEEE division: m = 1..nm, then nm*per random pairs. */
int skm_debug_div_check(uint64_t nm, uint32_t per, uint64_t* mismatches);
/* Run (if not yet run since the last prepare) and download the result, keys ascending (sorted
 * on the device in key-range chunks and streamed to the host arrays; the reference's KeptKmers is
 * a hash map, kmers-build-signatures.cc:206-221, so any order is valid).  At most 2^32 - 1 kept
 * k-mers per call (use skm_build_finish_slice beyond).  With world_size > 1 this is collective:
 * rank 0 receives every rank's kept k-mers, the other ranks the k-mers they own; the statistics
 * are global on every rank. */
int skm_build_finish(skm_build* b, skm_kept* out);
/* The kept k-mers of one output slice: those whose slice hash -- MurmurHash3's fmix64 of the
 * little-endian key, top slice_bits bits -- equals `slice` (0 <= slice < 2^slice_bits, slice_bits
 * <= 16; slice_bits 0 = every kept k-mer), keys sorted, with the build's global statistics.  The
 * 2^slice_bits slices partition the kept set, so a caller streams an output too large for one
 * host copy slice by slice (the 50M-protein build keeps ~2.9G k-mers).  The reference writes
 * final.kmers / the .dat from one in-memory KeptKmers map (kmers-build-signatures.cc:198-264);
 * its order is hash order, so slices written one after another are a valid final.kmers.
 * n_seqs_with_signature counts sequences (not distinct seq ids).  With world_size > 1: this
 * rank's own k-mers of the slice (not collective for the keys; distinct_signatures is global). */
int skm_build_finish_slice(skm_build* b, int slice_bits, uint32_t slice, skm_kept* out);
/* The last run's per-sequence signature flags (KmerStatistics::seqs_with_a_signature, signature_
 * build.tcc:275, as a bitmap over the sequences with a kept function in add order; world_size > 1:
 * every rank's sequences in rank order): min(cap, sequences) bytes of 0/1. */
int skm_build_signature_flags(skm_build* b, uint8_t* out, uint64_t cap);
void skm_kept_free(skm_kept* k);
void skm_build_destroy(skm_build* b);

/* ------------------------------------------------------------------------------------------
 * Multi-GPU (one process per GPU; opts.rank / opts.world_size, a power of two).  Rank r adds
 * the r-th contiguous range of files (emission order is rank order).  Rank 0 calls
 * skm_comm_unique_id, the caller broadcasts the 128 bytes (e.g. torch.distributed over gloo),
 * every rank passes them to skm_build_set_comm (collective) before prepare/run.  Owner of a
 * k-mer = top bits of its hashed key; occurrence elements are exchanged with one RCCL
 * all-to-all over xGMI, then per-function counts (sum) and signature flags (max) are
 * all-reduced.  prepare / run / finish are collective.
 * ------------------------------------------------------------------------------------------ */
int skm_comm_unique_id(uint8_t id[128]);
int skm_build_set_comm(skm_build* b, const uint8_t id[128]);
/* Test/diagnostic transport: run n handles of ranks 0..n-1 (world_size n) in this process,
 * exchanging through device copies instead of RCCL; skm_build_finish on any member afterwards. */
int skm_build_group_run(skm_build* const* bs, int n);

/* ------------------------------------------------------------------------------------------
 * Signature DB (CmphKmerDb<StoredKmerData,8>, cmph_kmer.h:28-164).  Reads a cmph BDZ dump
 * (<dir>/kmer_data.mph) + the dense record file (<dir>/kmer_data.dat) and lays g, the rank table
 * and the records out contiguously in HBM.
 * ------------------------------------------------------------------------------------------ */
typedef struct skm_db skm_db;

int skm_db_open(skm_db** out, const char* mph_path, const char* dat_path, int device);
int skm_db_open_mem(skm_db** out, const uint8_t* mph, size_t mph_len, const uint8_t* dat,
                    size_t dat_len, int device);
/* Exact-key DB over the kept k-mers of a build: KeptKmerDB<K> (kept_kmer_db.h:9-31), used by the
 * recall pass of kmers-build-signatures (kmers-build-signatures.cc:238-349).  A window hits only
 * if its k-mer is one of keys (record data[i]); keys must be distinct and non-zero.  Laid out in
 * HBM as an open-addressing table (load <= 1/2) + the 10-byte records.  skm_db_lookup returns
 * the record index, or n for a miss.                                                          */
int skm_db_open_kept(skm_db** out, const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, int device);
/* cmph_size() (cmph_kmer.h:102); for an exact DB the number of kept k-mers */
int skm_db_size(skm_db* db, uint32_t* m);
/* Batched cmph_search(hash, key, 8) (cmph_kmer.h:90-92); idx >= size is a miss. */
int skm_db_lookup(skm_db* db, const uint64_t* keys, size_t n, uint32_t* idx_out);
/* test hook: the same search through the generic bdz_search walk (any b), bypassing the b == 7
 * (g word, rank) pair lines that skm_db_lookup / the annotate kernels use when present */
int skm_debug_db_lookup_generic(skm_db* db, const uint64_t* keys, size_t n, uint32_t* idx_out);
void skm_db_close(skm_db* db);

/* Build a BDZ minimal perfect hash over keys (build_perfect_hash, perfect_hash.h:11-69):
 * writes a cmph-compatible .mph image and the .dat records (data[i] goes to slot search(key i)).
 * seed: initial PRNG seed for the hash seed draws (cmph uses rand() % 15).                     */
int skm_mph_build(const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, uint32_t seed,
                  const char* mph_path, const char* dat_path);

/* skm_mph_build with the construction on a GPU: same parameters and image format, the
 * 3-hypergraph peeled in parallel rounds and g assigned round by round on `device`, the rank
 * table and records placed from the device lookup.  Deterministic for a given (keys, seed).
 * device < 0 (or fewer than 1024 keys) runs the host builder.                                */
int skm_mph_build_device(const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, uint32_t seed,
                         const char* mph_path, const char* dat_path, int device);

/* skm_mph_build_device with phase times and an optional on-device check, for builds up to the
 * headline kept set (cmph's 32-bit m, n = 3r: n < 2^32, i.e. about 3.4 G keys).  mph_path /
 * dat_path may be NULL (that image is not written).  verify != 0: every key's slot is < n and
 * distinct (a slot bitmap), the annotate kernels' b == 7 pair-line search equals the generic
 * bdz_search for every key, and .dat[slot] equals the key's record; a failure returns
 * SKM_E_STATE.  Replaces build_perfect_hash (perfect_hash.h:11-69) as kmers-build-signatures
 * runs it over the whole kept set (kmers-build-signatures.cc:253-264). */
typedef struct skm_mph_stats {
    double upload_s, peel_s, assign_s, rank_s, place_s, verify_s, write_s, total_s;
    uint64_t n_keys, n_vertices;
    uint32_t attempts, peel_rounds;
    int32_t verified;      /* 1: the check above ran and passed */
    int32_t pad;
} skm_mph_stats;
int skm_mph_build_device_ex(const uint64_t* keys, const skm_stored_kmer_data* data, size_t n, uint32_t seed,
                            const char* mph_path, const char* dat_path, int device, int verify,
                            skm_mph_stats* stats);

/* ------------------------------------------------------------------------------------------
 * Function calling.  Replaces FunctionCaller<CmphKmerDb>::process_aa_seq for a batch of query
 * sequences (call_functions.tcc:259-338 + HitSet :6-108, window iterator kmer_data.h:76-102).
 * find_best_call (call_functions.tcc:347-659) stays on the host: skm_find_best_call.
 * ------------------------------------------------------------------------------------------ */
typedef struct skm_annot_opts {
    int32_t min_hits;      /* 5   (call_functions.h:66)                                   */
    int32_t max_gap;       /* 200                                                          */
    int32_t ignore_hypo;   /* --ignore-hypo                                                */
    int32_t hypo_index;    /* index of "hypothetical protein" in function.index           */
    int32_t mean_mode;     /* Boost.Math mean: 0 = >=1.76 four-lane (default), 1 = <=1.75  */
    int32_t mad_mode;      /* MAD: 0 = |x(mid)-median| (>=1.76), 1 = |x(mid)| (older Boost,  */
                           /* libstdc++ nth_element order)                      */
} skm_annot_opts;

typedef struct skm_calls {
    uint64_t* call_off;    /* [n_seqs+1] CSR offsets                                       */
    skm_kmer_call* calls;  /* [n_calls]                                                    */
    uint64_t n_seqs;
    uint64_t n_calls;
    uint64_t n_windows;    /* query windows examined                                       */
} skm_calls;

typedef struct skm_query skm_query;
/* Upload a batch of query sequences (residues/seq_off/seq_len as in skm_build_add_batch). */
int skm_query_create(skm_query** out, skm_db* db, const uint8_t* residues, const uint64_t* seq_off,
                     const uint32_t* seq_len, size_t n_seqs);
/* Device pipeline (window lookup + HitSet) on resident queries; calls stay on the device. */
int skm_query_run(skm_query* q, const skm_annot_opts* opts);
int skm_query_last_timings(skm_query* q, float* ms, int cap);
/* Download the calls of the last run. */
int skm_query_calls(skm_query* q, skm_calls* out);
/* The last run's per-window hits as the device lookup produced them (diagnostics and parity tests
 * of the device window iterator, kmer_data.h:76-102, and fetch, cmph_kmer.h:139-147; the CLI's
 * --debug-hits prints them as the reference's hit_cb does, kmers-call-functions.cc:109-118):
 * hit_off [n_seqs+1] CSR offsets; for the first `cap` hits pos = the window's offset in its
 * sequence and fm = function_index << 16 | mean of its record (either array may be NULL).
 * *n_out = the total number of hits. */
int skm_query_window_hits(skm_query* q, uint64_t* hit_off, uint32_t* pos, uint32_t* fm, uint64_t cap, uint64_t* n_out);
void skm_query_destroy(skm_query* q);
/* Convenience: create + run + calls, through one query object the DB keeps for these calls (its
 * device buffers, stream and host threads reused from batch to batch; released by
 * skm_db_close).  A batch laid out packed -- seq_off[s] = sum over t < s of (seq_len[t] + 1),
 * i.e. one byte after every sequence -- is uploaded as it is (the bytes between sequences are not
 * read as residues); any other layout is packed on the host first.  Like every call on a handle,
 * from one host thread at a time per DB. */
int skm_annotate(skm_db* db, const uint8_t* residues, const uint64_t* seq_off, const uint32_t* seq_len,
                 size_t n_seqs, const skm_annot_opts* opts, skm_calls* out);
void skm_calls_free(skm_calls* c);

/* ------------------------------------------------------------------------------------------
 * All-vs-all shared-signature-k-mer counts.  Replaces MatrixDistance::compute
 * (matrix_distance.h:45-170) as run by kmers-matrix-distance (kmers-matrix-distance.cc:94-212):
 * process_aa_seq with ignore_hypothetical(true) feeds hit_cb (:123-152: hits whose seqlen lies
 * outside mean +/- 2 sd of the record are dropped; sd = sqrt(var), or 0.1 seqlen when var == 0),
 * kmer_hit_map[kmer] = set of SeqIdMap indices (seq_id_map.h:12-27), seq_dist[id1][id2]++ for
 * every id1 < id2 of a k-mer's set (:176-196).
 * ------------------------------------------------------------------------------------------ */
typedef struct skm_matrix skm_matrix;

typedef struct skm_matrix_opts {
    int32_t hypo_index;       /* function index of "hypothetical protein" (dropped); -1: none    */
    uint32_t row_begin;       /* count only pairs with id1 in [row_begin, row_end): this GPU's    */
    uint32_t row_end;         /* tile of the triangle (skm_matrix_tile_rows); 0, 0 = every row    */
    uint32_t pad;
    uint64_t max_tile_bytes;  /* reserved (0): the counts live in per-row LDS histograms, no dense
                                 tile is allocated in HBM                                        */
} skm_matrix_opts;

typedef struct skm_pairs {
    uint32_t* pairs;          /* [n][3] = (id1, id2, count), id1 < id2, sorted by (id1, id2)      */
    uint64_t n;
    uint64_t n_hits;          /* (kmer, sequence) hit records that passed the filters            */
} skm_pairs;

/* seq_idx[s]: SeqIdMap index of sequence s (index of the first sequence with its id, in input
 * order; < n_idx).  residues / seq_off / seq_len as in skm_build_add_batch. */
int skm_matrix_create(skm_matrix** out, skm_db* db, const uint8_t* residues, const uint64_t* seq_off,
                      const uint32_t* seq_len, const uint32_t* seq_idx, size_t n_seqs, uint32_t n_idx);
/* Device pipeline on the resident queries; the pairs stay on the device. */
int skm_matrix_run(skm_matrix* m, const skm_matrix_opts* opts);
/* Multi-GPU matrix distance: rank `rank` of `world` created its handle over its
 * own contiguous range of the query sequences, with the global SeqIdMap indices and n_idx (every
 * rank's the same).  After joining the ranks -- a host transport (copied) or an RCCL communicator
 * (rank 0's skm_comm_unique_id, collective) -- skm_matrix_run is collective: each rank looks up
 * only its own queries (kmers-matrix-distance.cc:123-152 hit_cb), every (k-mer, index) hit goes
 * to the k-mer's owner GPU (all-to-all), the owner builds its k-mers' kmer_hit_map entries and
 * sends each one's index set to the GPUs whose row band (skm_matrix_tile_rows) it has pairs in
 * (all-to-all), and each GPU counts the pairs of its band (:176-196); opts row_begin / row_end are
 * ignored, and skm_matrix_pairs returns the band's pairs (concatenate the ranks' in rank order). */
int skm_matrix_set_transport(skm_matrix* m, int rank, int world, const skm_transport* tp);
int skm_matrix_set_comm(skm_matrix* m, int rank, int world, const uint8_t id[128]);
/* [0]=hits [1]=group (hash + sort) [2]=pair increments [3]=compaction [4]=total (ms) */
int skm_matrix_last_timings(skm_matrix* m, float* ms, int cap);
/* [0]=windows [1]=hit records [2]=pair increments [3]=nonzero pairs [4]=distinct hit k-mers
 * (kmer_hit_map.size(), kmers-matrix-distance.cc:169; with ranks: the k-mers this rank owns)
 * [5]=hits of this handle's queries [6]=with ranks: index entries routed to this rank's band */
int skm_matrix_counters(skm_matrix* m, uint64_t* out, int cap);
int skm_matrix_pairs(skm_matrix* m, skm_pairs* out);
void skm_pairs_free(skm_pairs* p);
void skm_matrix_destroy(skm_matrix* m);
/* Row band of rank `rank` of `world` GPUs with (nearly) equal triangle area. */
int skm_matrix_tile_rows(uint32_t n_idx, int rank, int world, uint32_t* row_begin, uint32_t* row_end);

/* find_best_call (call_functions.tcc:347-659) on the host.  function_index: nfunc C strings
 * (function.index column 1).  out_func receives the called function (NUL-terminated).      */
int skm_find_best_call(const skm_kmer_call* calls, size_t ncalls, const char* const* function_index,
                       size_t nfunc, uint16_t* out_fi, float* out_score, float* out_offset,
                       char* out_func, size_t out_func_cap);

#ifdef __cplusplus
}
#endif

#endif /* SKM_H */
