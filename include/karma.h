/*
 * karma.h — C ABI of libkarma_hip.so, the MI355X (gfx950) implementation of
 * lmfaber/karma's k-mer profile + shared-read graph hot path.
 *
 * Plain C types only (pointers + sizes); no torch / HIP types in signatures
 * (streams are passed as void*).  Every function returns an int status
 * (KARMA_OK = 0, negative = error; message via karma_last_error()).
 *
 * Reference interfaces replaced (file:line under lmfaber/karma):
 *   karma_contigs_*, karma_kmer_*   KmerClustering.__calc_kmer_profile   karma/kmer.py:199-264
 *                                   (__extract_kmers :146-179, __kmers_of_seq :181-197,
 *                                    __count_kmer_occurence :56-92, fill_array_for_contig :108-122,
 *                                    is_palindrome :46-54)
 *   karma_graph_records             ReadGraph.from_contigs               karma/read_graph.py:19-50
 *                                   + Contig readsets                    karma/contig.py:4-35
 *                                   and ReadGraph.update_graph           karma/read_graph.py:192-221
 *   karma_graph_eq                  ReadGraph.from_equivalence_classes   karma/read_graph.py:61-148
 *   karma_pairs_merge{,_runs} /     (new) multi-GPU edge merge, SURVEY.md §8(e)
 *   _split / _totals
 *   karma_edges_*                   the normalised weight (s/|A| + s/|B|)/2  read_graph.py:39-42, :128-130
 *   karma_synth_*                   (new) deterministic synthetic inputs, SURVEY.md §8(d)
 *   karma_fasta_*                   read_fasta_file                      karma/karma.py:40-61
 *   karma_eq_*                      eq_classes.txt parse                 karma/read_graph.py:75-92
 *   karma_sam_*                     Contig readsets from SAM lines       karma/contig.py:24,34, hisat2.py:49-53
 *   karma_adj_*                     graph consumers: unconnected nodes, node weights, edge_list
 *                                   karma/read_graph.py:150-190, :315-357
 *   karma_adj_cross_sums            --rearrange subcluster connections  karma/karma.py:103-118
 *
 * The reference is pure Python and has no FFI; INTEGRATION.md shows the ctypes
 * binding (karma_amd/_lib.py) that the Python classes mirroring the reference
 * API (karma_amd/kmer.py, read_graph.py, contig.py) use.
 */
#ifndef KARMA_H
#define KARMA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define KARMA_OK 0
#define KARMA_ERR_ARG (-1)       /* invalid argument / unsupported size                       */
#define KARMA_ERR_KMER (-2)      /* unsupported k (supported: 1..8 and "5p6")                 */
#define KARMA_ERR_HIP (-3)       /* HIP runtime error (no device, launch failure, ...)        */
#define KARMA_ERR_OOM (-4)       /* device allocation failed                                  */
#define KARMA_ERR_ZERO_DIV (-5)  /* non-zero count over a zero normaliser (ZeroDivisionError) */
#define KARMA_ERR_UNSORTED (-6)  /* records not grouped by read (read ids must not decrease)  */
#define KARMA_ERR_STATE (-7)     /* call out of order (e.g. profile before finalize)          */
#define KARMA_ERR_PARSE (-8)     /* input text outside what the C++ parser reproduces exactly */
#define KARMA_ERR_COMM (-9)      /* RCCL communicator error                                   */
#define KARMA_ERR_STALL (-10)    /* a deferred step's status did not arrive (stalled peer/device) */

#define KARMA_KMER_5P6 (-1) /* kmer.py:69 "5p6": all 5-mers + string-palindromic 6-mers */

int karma_version(void);
const char* karma_last_error(void);
/* Build identity as a JSON object: {"arch", "defines" (extra -D flags of a
 * variant build; "" for the shipped library), "src_sha256_16", "flags"}.
 * bench.py prints it and refuses a non-default build. */
const char* karma_build_info(void);
int karma_device_count(int* n);
/* Layout of a context's mapped host region (diagnostic; no device needed):
 * one fixed slot per user, offsets[s] / bytes[s] for s < min(cap, *n). */
int karma_mapped_slots(int64_t* offsets, int64_t* bytes, int cap, int* n);
/* HIP runtime (and RCCL) calls this thread has made through the library that
 * enqueue work, wait, or manage streams, events and memory (launches, copies,
 * memsets, event records, stream waits, synchronisations, collectives). */
int karma_api_calls(uint64_t* n);

/* ---- context: one device, one HIP stream --------------------------------- */
typedef struct karma_ctx karma_ctx;
int karma_ctx_create(int device, karma_ctx** out);
int karma_ctx_destroy(karma_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream. */
int karma_ctx_set_stream(karma_ctx* ctx, void* hip_stream);
int karma_ctx_sync(karma_ctx* ctx);
/* Per-kernel HIP-event timing on the launch stream (for bench.py's roofline). */
int karma_timing_enable(karma_ctx* ctx, int on);
/* Restrict timing to launches of one kernel name (NULL or "": every kernel), so a
 * timed region carries two events per launch of that kernel only. */
int karma_timing_only(karma_ctx* ctx, const char* name);
int karma_timing_reset(karma_ctx* ctx);
/* Fills up to cap entries: name (NUL-separated into names[cap*64]), total ms, launches.
 * Returns number of distinct kernels in *n. Synchronises the stream. */
int karma_timing_read(karma_ctx* ctx, char* names, double* total_ms, int64_t* launches, int cap, int* n);

/* ---- device memory helpers (for callers without their own allocator) ------ */
int karma_dev_alloc(karma_ctx* ctx, size_t bytes, void** out);
int karma_dev_free(karma_ctx* ctx, void* p);
int karma_memcpy(karma_ctx* ctx, void* dst, const void* src, size_t bytes, int kind /*0 H2D,1 D2H,2 D2D*/);
/* The same, ordered on the context's stream and not waited for (host memory
 * must stay valid until the stream reaches the copy). */
int karma_memcpy_async(karma_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);
/* Pinned host memory for results (device -> host copies into it run at the
 * full PCIe rate): blocks are cached by size class after karma_host_free. */
int karma_host_alloc(size_t bytes, void** out);
int karma_host_free(void* p);
int karma_memset_async(karma_ctx* ctx, void* dst, int value, size_t bytes);
/* Average ms of `reps` hipMemsetAsync of `bytes` at dst (HIP events on the
 * context's stream): the device's write ceiling for a buffer of that size. */
int karma_memset_timed(karma_ctx* ctx, void* dst, size_t bytes, int reps, double* ms);
/* Streams owned by the library (a side stream for the profile, a high-priority
 * main stream); priority: 0 normal, < 0 higher (hipStreamCreateWithPriority). */
int karma_stream_create(karma_ctx* ctx, int priority, void** stream);
int karma_stream_destroy(karma_ctx* ctx, void* stream);
int karma_stream_sync(karma_ctx* ctx, void* stream);

/* ---- RCCL communicator (one per device and process) ----
 * The multi-GPU build's two exchange steps (presence MAX-allreduce + exception
 * all-gather for the column table; pair all-to-all-v + totals all-gather for the
 * graph) run on it, enqueued on the bound context's stream.  The 128-byte unique
 * id made by one rank reaches the others through the caller's bootstrap
 * (karma_amd/hostgroup.py).  Replaces nothing in the reference (single process). */
typedef struct karma_comm karma_comm;
#define KARMA_DT_U8 0
#define KARMA_DT_I32 1
#define KARMA_DT_I64 2
#define KARMA_DT_U64 3
#define KARMA_DT_F64 4
#define KARMA_OP_SUM 0
#define KARMA_OP_MAX 1
#define KARMA_OP_MIN 2
int karma_comm_id_bytes(void);
int karma_comm_unique_id(uint8_t* id);
int karma_comm_create(karma_ctx* ctx, const uint8_t* id, int world, int rank, karma_comm** out);
/* The same with flags.  KARMA_COMM_SIDE: a second communicator over the same
 * ranks (its own unique id) for collectives enqueued on a side stream.  One
 * communicator's operations must be issued in the same order on every rank; a
 * job with collectives on two streams gives each stream its own communicator,
 * so the two orders never interleave differently across ranks. */
#define KARMA_COMM_SIDE 1
int karma_comm_create_ex(karma_ctx* ctx, const uint8_t* id, int world, int rank, int flags, karma_comm** out);
int karma_comm_destroy(karma_comm* c);
int karma_comm_info(karma_comm* c, int* world, int* rank);
/* In place on device memory, stream-ordered. */
int karma_comm_allreduce(karma_comm* c, void* buf_dev, int64_t count, int dtype, int op);
/* Host scalars (at most max(64, 8 * world) bytes); synchronises the stream. */
int karma_comm_allreduce_host(karma_comm* c, void* buf_host, int64_t count, int dtype, int op);
int karma_comm_barrier(karma_comm* c);
/* recv_dev[r * bytes_per_rank ...] = rank r's send_dev; in place when
 * send_dev == recv_dev + rank * bytes_per_rank. */
int karma_comm_allgather(karma_comm* c, const void* send_dev, void* recv_dev, int64_t bytes_per_rank);
/* recv_host[r] = send_host[rank] of rank r (world int64 each; synchronises). */
int karma_comm_exchange_counts(karma_comm* c, const int64_t* send_host, int64_t* recv_host);
/* Bytes send_dev[send_off[r], send_off[r+1]) go to rank r and land in its
 * recv_dev[recv_off[me], ...); offsets are host arrays of world + 1 entries. */
int karma_comm_alltoallv(karma_comm* c, const void* send_dev, const int64_t* send_off, void* recv_dev,
                         const int64_t* recv_off);
/* The same for a list held as two arrays of equal element size (keys and
 * counts): part a and part b of each slice go as two grouped sends, so the
 * sender needs no interleaved copy.  Offsets (bytes) apply to both parts. */
int karma_comm_alltoallv_kv(karma_comm* c, const void* send_a, const void* send_b, const int64_t* send_off,
                            void* recv_a, void* recv_b, const int64_t* recv_off);

/* ---- contig store (device-resident, 2-bit packed + exception mask) -------- */
typedef struct karma_contigs karma_contigs;
/* seq: concatenated sequence bytes (latin-1 code points of the reference's str
 * values), offsets[n+1] into seq, key_len[n] = len(FASTA dict key) — the
 * reference's normaliser (kmer.py:213 iterates the dict's keys).
 * is_device = 0: host pointers, copied; 1: device pointers, referenced (must
 * outlive the store).  Packs A,C,G,T to 2 bits on the device; any other byte is
 * an exception base handled through a byte-key path. */
int karma_contigs_create(karma_ctx* ctx, const uint8_t* seq, const int64_t* offsets, const int32_t* key_len,
                         int64_t n, int is_device, karma_contigs** out);
int karma_contigs_destroy(karma_contigs* c);
int karma_contigs_info(karma_contigs* c, int64_t* n, int64_t* total_bases, int64_t* exception_bases,
                       int64_t* packed_bytes);

/* ---- k-mer profile (kmer.py:146-264) -------------------------------------- */
typedef struct karma_kmer_plan karma_kmer_plan;
/* Presence pass over the (local) contig store. kmode: 1..8 or KARMA_KMER_5P6. */
int karma_kmer_plan_create(karma_ctx* ctx, karma_contigs* c, int kmode, karma_kmer_plan** out);
int karma_kmer_plan_destroy(karma_kmer_plan* p);
/* Multi-rank exchange points: the ACGT presence bitmap (OR /
 * max-reduce across ranks) and the non-ACGT ("exception") k-mer keys (union). */
int karma_kmer_presence_words(karma_kmer_plan* p, int64_t* nwords);
int karma_kmer_presence_get(karma_kmer_plan* p, uint32_t* dst_dev);
int karma_kmer_presence_set(karma_kmer_plan* p, const uint32_t* src_dev);
/* presence = OR of n_sets bitmaps of presence_words each, back to back in
 * device memory (the ranks' bitmaps after an all-gather). */
int karma_kmer_presence_merge(karma_kmer_plan* p, const uint32_t* all_dev, int n_sets);
int karma_kmer_exceptions_count(karma_kmer_plan* p, int64_t* n);
int karma_kmer_exceptions_get(karma_kmer_plan* p, uint64_t* dst_dev);
int karma_kmer_exceptions_set(karma_kmer_plan* p, const uint64_t* src_dev, int64_t n);
/* Column table = sorted() union of present k-mers (kmer.py:172-177). */
int karma_kmer_plan_finalize(karma_kmer_plan* p, int64_t* M);
/* The same in two halves: _async enqueues the column table and M's readback;
 * _wait waits for those alone (not for later work on the stream).  One
 * finalize in flight per context. */
int karma_kmer_plan_finalize_async(karma_kmer_plan* p);
int karma_kmer_plan_finalize_wait(karma_kmer_plan* p, int64_t* M);
/* Column keys: byte-packed u64, big-endian bytes from bit 63; for k < 8 and 5p6
 * the low byte holds the k-mer length (so u64 order == Python str order). */
int karma_kmer_columns(karma_kmer_plan* p, uint64_t* keys_host);
/* Dense float64 profile, row r = contig r of the store, stride ld >= M:
 * out[r*ld + col] = count / key_len[r] (kmer.py:120, :231-233), zeros written. */
int karma_kmer_profile(karma_kmer_plan* p, double* out, int64_t ld, int out_is_device);
/* Rows [row_lo, row_hi) of the same profile: row r of out is contig row_lo + r
 * (SURVEY.md §8(e) streaming: a profile larger than host or device memory is
 * produced and copied out one row block at a time; host output synchronises). */
int karma_kmer_profile_rows(karma_kmer_plan* p, int64_t row_lo, int64_t row_hi, double* out, int64_t ld,
                            int out_is_device);
/* karma_kmer_profile into device memory, launched on `side` (a hipStream_t)
 * after everything already enqueued on the context's stream -- or, while a
 * karma_graph_records_begin job is open, after that job's classify kernel and
 * this plan's column table -- so it overlaps the rest of the stream's work.  Call karma_ctx_join
 * before the plan or the output are used or destroyed.  side = NULL: the
 * context's stream. */
int karma_kmer_profile_side(karma_kmer_plan* plan, double* out_dev, int64_t ld, void* side);
/* The context's stream waits (on the device) for the work enqueued on `side`. */
int karma_ctx_join(karma_ctx* ctx, void* side);
/* Block slots per CU the side-stream profile's grid leaves free for the main
 * stream (default 0: the profile's 3 blocks per CU take the chip; a free slot
 * measured slower). */
int karma_ctx_set_side_headroom(karma_ctx* ctx, int blocks_per_cu);
/* Number of k-mer occurrences per contig (0 => the all-zero row of kmer.py:250-258). */
int karma_kmer_row_totals(karma_kmer_plan* p, int64_t* dst_host);

/* ---- shared-read graph ----------------------------------------------------- */
/* A pair list: unique keys (a << 32 | b, a <= b) sorted ascending with int64
 * counts (and, for eq classes, the first emission position). */
typedef struct karma_pairs karma_pairs;
#define KARMA_REC_SORTED 0   /* records grouped by read, read ids non-decreasing (SAM order) */
#define KARMA_REC_UNSORTED 1 /* any order: sorted by read on the device first */
#define KARMA_REC_FLAGGED 2  /* records as n_records x u32: contig | (first record of its read) << 31, grouped by
                              * read.  The graph depends only on which records share a read (read_graph.py:31-49
                              * intersects readsets), so the read ids give way to read-start flags: 4 bytes per
                              * record instead of 8.  Record 0 always starts a read; contig ids < 2^31. */
/* records: n_records x {u32 read_id, u32 contig} interleaved (or, flags =
 * KARMA_REC_FLAGGED, n_records x u32 flagged contigs; records is then a
 * uint32_t array of n_records entries).  Deduplicates
 * (read, contig) (contig.py:11 keeps QNAMEs in a set); emits for every read's
 * contig set S every pair a <= b of S: the diagonal (a, a) counts |readset(a)|,
 * (a, b) counts |R_a ∩ R_b| (read_graph.py:34). */
int karma_graph_records(karma_ctx* ctx, const uint32_t* records, int64_t n_records, int64_t n_contigs, int flags,
                        int is_device, karma_pairs** out);
/* karma_graph_records in two halves.  _begin enqueues the pipeline up to its
 * one host synchronisation and returns; the caller may enqueue other work (on
 * another stream) before _end waits, checks and assembles the list.  Device
 * records must stay valid until _end.  One open job per context; _end always
 * consumes the job (also on error). */
typedef struct karma_graph_job karma_graph_job;
int karma_graph_records_begin(karma_ctx* ctx, const uint32_t* records, int64_t n_records, int64_t n_contigs,
                              int flags, int is_device, karma_graph_job** job);
int karma_graph_records_end(karma_graph_job* job, karma_pairs** out);
/* Owner bounds (nranks + 1 contig ids) of the exchange that will split the
 * next records job's list on this context: the job finds each owner's start
 * on the device as it builds the list, and karma_pairs_split with the same
 * bounds then answers without a launch or a synchronisation.  Applies to one
 * job; at most 64 ranks. */
int karma_graph_split_hint(karma_ctx* ctx, const int64_t* bounds, int nranks);
/* Salmon eq classes (read_graph.py:75-114): cls_off[n_classes+1] into members
 * (contig indices as listed, duplicates kept), counts[n_classes], pair_skip[c]=1
 * when the eq_size token is "1" (read_graph.py:102).  Totals (read_graph.py:86-92)
 * go to the pair list's totals array; pairs carry first-emission positions. */
int karma_graph_eq(karma_ctx* ctx, const int64_t* cls_off, const uint32_t* members, const int64_t* counts,
                   const uint8_t* pair_skip, int64_t n_classes, int64_t n_contigs, int is_device, karma_pairs** out);
/* karma_graph_eq from compact host inputs (10 bytes per class fewer over PCIe):
 * sizes[C] = member count (<= 127) | 0x80 when the class's eq_size token is
 * "1" (pair_skip), counts[C] as u32; n_members = the sizes' sum (KARMA_ERR_ARG
 * when they disagree, checked on the device).  Same pairs, firsts and totals. */
int karma_graph_eq_compact(karma_ctx* ctx, const uint8_t* sizes, const uint32_t* members, int64_t n_members,
                           const uint32_t* counts, int64_t C, int64_t n_contigs, karma_pairs** out);
/* Merge (key, count) lists in any order into one sorted unique list (exchange merge). */
int karma_pairs_merge(karma_ctx* ctx, const uint64_t* keys, const int64_t* counts, int64_t n, int is_device,
                      karma_pairs** out);
/* Merge runs [run_off[r], run_off[r + 1]) of (key, count), each sorted by key
 * (the slices an exchange owner receives, one per sender), into one sorted
 * unique list: a pairwise merge tree, then equal keys summed.
 * KARMA_ERR_UNSORTED when a run is not sorted.  run_off is a host array of
 * n_runs + 1 offsets starting at 0. */
int karma_pairs_merge_runs(karma_ctx* ctx, const uint64_t* keys, const int64_t* counts, const int64_t* run_off,
                           int n_runs, int is_device, karma_pairs** out);
/* The exchange's wire format: n x {i64 key, i64 count} interleaved in device
 * memory.  _get_kc writes the list in it (stream-ordered, not waited for);
 * _merge_runs_kc merges received runs of it (at most 64 runs: without a host
 * synchronisation, equal keys of different runs left adjacent for the edge
 * stage; accessors of the list sum them first). */
int karma_pairs_get_kc(karma_pairs* p, int64_t* kc_dev);
int karma_pairs_merge_runs_kc(karma_ctx* ctx, const int64_t* kc_dev, const int64_t* run_off, int n_runs,
                              karma_pairs** out);
int karma_pairs_destroy(karma_pairs* p);
/* Later kernels on p run on ctx's stream (after p's current stream is drained);
 * p's memory stays with the allocator that made it.  Lets a list built on a
 * second context (concurrent graph build) join the main stream's exchange. */
int karma_pairs_rebind(karma_pairs* p, karma_ctx* ctx);
int karma_pairs_count(karma_pairs* p, int64_t* n);
/* Device pointers of the list (valid until destroy): keys u64[n], counts i64[n]. */
int karma_pairs_device(karma_pairs* p, const uint64_t** keys, const int64_t** counts);
/* Copy the list out.  Host copies (is_device = 0) have completed on return;
 * device copies (is_device = 1) are ordered on p's stream and not waited for. */
int karma_pairs_get(karma_pairs* p, uint64_t* keys, int64_t* counts, uint64_t* first, int is_device);
/* Index of the first key with a >= bounds[r] for r = 0..nranks (host out; searched on the device). */
int karma_pairs_split(karma_pairs* p, const int64_t* bounds, int nranks, int64_t* starts);
/* karma_pairs_split and karma_pairs_get_kc in one launch (the exchange's send
 * side): starts on the host when it returns, kc_dev (n x {key, count}) written. */
int karma_pairs_split_kc(karma_pairs* p, const int64_t* bounds, int nranks, int64_t* starts, int64_t* kc_dev);
/* totals[c] = count of the diagonal pair (c, c) (readset sizes) for c in [0, n_contigs). */
int karma_pairs_totals(karma_pairs* p, int64_t* totals_dev, int64_t n_contigs);

typedef struct karma_edges karma_edges;
#define KARMA_MODE_READS 0 /* diagonal = readset sizes; off-diagonal = shared reads   */
#define KARMA_MODE_EQ 1    /* totals from the eq pass; diagonal pairs are self-loops */
/* Edges with non-zero shared count and weight (s/tot[a] + s/tot[b]) / 2.
 * totals_dev: int64[n_contigs] device array, or NULL to take it from the pair
 * list (diagonal in READS mode, eq totals in EQ mode). */
int karma_edges_from_pairs(karma_ctx* ctx, karma_pairs* p, int mode, const int64_t* totals_dev, int64_t n_contigs,
                           karma_edges** out, int64_t* n_edges);
/* The same in two halves, for an all-gather of the totals in between (the
 * sharded build: each owner's diagonal holds the readset sizes of the contigs
 * it owns).  _begin takes the totals from the list (as totals_dev = NULL
 * above), launches the edge count and returns the device totals array
 * (int64[n_contigs], owned by the edges) for the caller to fill further;
 * _end launches the weights and synchronises.  p must stay valid until _end.
 * A list from karma_pairs_merge_runs_kc may hold equal adjacent keys (not yet
 * summed): the edge stage sums them, and reports KARMA_ERR_UNSORTED for a
 * merge input that was not sorted. */
int karma_edges_begin(karma_ctx* ctx, karma_pairs* p, int mode, int64_t n_contigs, karma_edges** out,
                      int64_t** totals_dev);
int karma_edges_end(karma_edges* e, int64_t* n_edges);
/* n_edges = NULL: _end launches the weights and returns at once; the edge
 * count, and the zero-total and merge-order errors, come with the first
 * karma_edges_count / _get / _totals (one synchronisation there). */
int karma_edges_count(karma_edges* e, int64_t* n_edges);
int karma_edges_destroy(karma_edges* e);
/* Any output pointer may be NULL. first is only meaningful in EQ mode. */
int karma_edges_get(karma_edges* e, uint32_t* a, uint32_t* b, int64_t* shared, double* weight, uint64_t* first,
                    int is_device);
int karma_edges_totals(karma_edges* e, int64_t* totals, int is_device);
/* karma_edges_get and karma_edges_totals with one synchronisation. */
int karma_edges_get_all(karma_edges* e, uint32_t* a, uint32_t* b, int64_t* s, double* w, uint64_t* first,
                        int64_t* totals, int is_device);
/* Eq-class edge stages (KARMA_MODE_EQ) only: a, b, w[E] in the reference's
 * insertion order -- edges grouped by a ascending, inside a group by the pair's
 * first emission (read_graph.py:96-131 adds (u, v) from u as pairs are first
 * seen; cls(incoming_graph_data=) keeps that order, read_graph.py:148).  The
 * order is computed on the device; one synchronisation. */
int karma_edges_get_ordered(karma_edges* e, uint32_t* a, uint32_t* b, double* w, int is_device);

/* ---- one rank's step of the sharded build ---------------
 * The whole hot path of one batch on this rank as one call: the records job
 * (read_graph.py:19-50 via Contig readsets, contig.py:4-35) on a main stream,
 * the k-mer column table and dense profile (kmer.py:146-264) on a side stream,
 * and, with several owners, the owners' split, the key/count all-to-all-v, the
 * owner's merge and the edge stage around the totals all-gather.  Replaces the
 * Python per-step sequence of karma_amd/distributed.py (which stays for the
 * host-staged rehearsal transport).
 * comm: the communicator (NULL or world 1: one process); by default every
 * collective of a step goes to it on ONE stream, in the same order on every rank.
 * side_comm: NULL (or comm) for that default; a distinct KARMA_COMM_SIDE
 * communicator puts the column-set exchange on it, on the side stream.
 * bounds[nranks + 1]: owner contig ranges tiling [0, n_glob); this rank's store
 * holds [bounds[rank], bounds[rank + 1]) (nranks = 1: any shard of the n_glob
 * contig ids, no exchange).  One process with nranks > 1 emulates
 * rank `rank` of an nranks-rank job (the exchange's local work, no collectives).
 * The step owns two streams; inputs stay on the device (records: n x {u32 read,
 * u32 contig}, grouped by read). */
typedef struct karma_step karma_step;
#define KARMA_STEP_KEEP 1       /* outputs kept for karma_step_profile / _columns / _edges */
#define KARMA_STEP_SEQUENTIAL 2 /* every kernel on the main stream (per-kernel timing) */
#define KARMA_STEP_FLAGGED 8    /* records_dev in the KARMA_REC_FLAGGED format (n_records x u32) */
#define KARMA_STEP_DEFER 4      /* outputs not read: the step returns without waiting for anything (its
                                 * checks arrive through mapped memory and are read <= 3 steps later; a
                                 * step needing the general path runs again synchronously; a status later
                                 * than KARMA_STEP_STALL_S seconds (120) is KARMA_ERR_STALL).  Several ranks:
                                 * once a synchronous step has sized the
                                 * exchange's slots and the store is ACGT-only on every rank (else the
                                 * step runs synchronously, its edge count not read back); every rank
                                 * learns every rank's re-run verdict from the exchange, so all of them
                                 * re-run the same steps.  Every rank must pass the same flags.
                                 * Inputs must stay valid until the next non-deferred step or
                                 * karma_step_sync. */
int karma_step_create(karma_ctx* ctx, karma_comm* comm, karma_comm* side_comm, int kmode, int64_t n_glob,
                      const int64_t* bounds, int nranks, int rank, karma_step** out);
/* info (may be NULL): [0] M, [1] local edges (-1: not read), [2] local pair list
 * size, [3] its summed counts (the last two with KARMA_STEP_KEEP, else -1). */
int karma_step_run(karma_step* s, karma_contigs* store, const uint32_t* records_dev, int64_t n_records, int flags,
                   int64_t* info);
/* Waits for every enqueued step and checks the deferred ones. */
int karma_step_sync(karma_step* s);
/* [M, E, pairs, entries, synchronous steps, deferred steps, re-run steps, pending, host ns inside
 * karma_step_run, of which ns waiting for a deferred step's status, deferred steps on two main
 * streams, deferred steps whose tail ran on the exchange stream, mode bits (1 one communicator,
 * 2 exchange stream allowed, 4 deferral across ranks allowed), ranks, deferred records jobs on the
 * step's own (pre-zeroed) control block] (first n).  After
 * karma_step_sync, M and E are the newest step's also when it was deferred (E: this rank's
 * edges). */
int karma_step_info(karma_step* s, int64_t* info, int n);
/* Outputs (valid until the next run).  _profile: the newest step's profile
 * (device, rows x M dense f64; a deferred step's once karma_step_sync has read
 * its column count).  _columns and _edges: the last KARMA_STEP_KEEP step's
 * column keys and edges (owned by the step: read with karma_edges_get /
 * _totals, never destroyed). */
int karma_step_profile(karma_step* s, double** dev, int64_t* rows, int64_t* M);
int karma_step_columns(karma_step* s, uint64_t* keys_host);
int karma_step_edges(karma_step* s, karma_edges** e);
/* The newest step's graph as this rank owns it (edges with a in its owner
 * range; one process: all), valid after karma_step_sync until the next run.
 * A deferred step's come from its own tail buffers -- the outputs of the
 * kernels a stream of deferred batches runs (step_edge_count / _write, and with
 * an exchange step_pack / step_merge) -- a synchronous one's (a re-run
 * included) from its karma_edges.  *n_edges = E; *deferred (may be NULL) = 1
 * for a deferred step's.  a, b, shared, weight: E entries each (E <= cap, else
 * KARMA_ERR_ARG), sorted by (a, b), a < b, weight (s/|A| + s/|B|)/2
 * (read_graph.py:19-50, :34-42); totals: n_glob readset sizes.  Any pointer may
 * be NULL (all NULL: only the count). */
int karma_step_newest_edges(karma_step* s, uint32_t* a, uint32_t* b, int64_t* shared, double* weight,
                            int64_t* totals, int64_t cap, int is_device, int64_t* n_edges, int* deferred);
int karma_step_destroy(karma_step* s);

/* ---- synthetic inputs (spec in karma_amd/synth.py) ------- */
int karma_synth_contig_lengths(uint64_t seed, int64_t n, int32_t len_min, int32_t len_span, int64_t* lengths);
/* Fills seq[total] given offsets[n+1] (prefix sums of the lengths). */
int karma_synth_contig_bases(uint64_t seed, const int64_t* offsets, int64_t n, int32_t n_rate, uint8_t* seq);
int karma_synth_n_genes(uint64_t seed, int64_t n_contigs, int32_t gene_max, int64_t* n_genes);
int karma_synth_genes(uint64_t seed, int64_t n_contigs, int32_t gene_max, int64_t* gene_first, int32_t* gene_size);
/* Records of fragments [frag_lo, frag_hi): per-fragment record counts first
 * (rec_count[frag_hi-frag_lo]), then the records themselves. */
int karma_synth_read_counts(uint64_t seed, const int64_t* gene_first, const int32_t* gene_size, int64_t n_genes,
                            int64_t frag_lo, int64_t frag_hi, int paired, int32_t* rec_count);
int karma_synth_read_records(uint64_t seed, const int64_t* gene_first, const int32_t* gene_size, int64_t n_genes,
                             int64_t frag_lo, int64_t frag_hi, int paired, const int64_t* rec_off, uint32_t* records);
/* Salmon-style eq classes of fragments [frag_lo, frag_hi): each fragment's
 * deduplicated contig set, aggregated in order of first appearance (the
 * karma_graph_eq input).  cls_off == NULL: only *n_classes and *n_members. */
int karma_synth_eq_classes(uint64_t seed, const int64_t* gene_first, const int32_t* gene_size, int64_t n_genes,
                           int64_t frag_lo, int64_t frag_hi, int paired, int64_t* n_classes, int64_t* n_members,
                           int64_t* cls_off, uint32_t* members, int64_t* counts);

/* ---- host ingestion (C++, std::threads; no device needed) ----------------
 * Parsers over an in-memory file image, with Python text-mode semantics
 * (strict UTF-8, universal newlines).  Input the parser cannot reproduce
 * exactly (a malformed line, a non-ASCII integer, a duplicate eq name, ...)
 * returns KARMA_ERR_PARSE; the Python front end then raises the reference's
 * own exception.  threads <= 0: hardware concurrency. */
typedef struct karma_fasta karma_fasta;
/* read_fasta_file: records in OrderedDict order, keys with ">" kept.
 * seq: seq_bytes + 16 zero bytes of padding (the karma_contigs_create layout);
 * key_len in code points; ascii = 1 when every byte is < 0x80. */
int karma_fasta_parse(const char* data, size_t len, int threads, karma_fasta** out);
int karma_fasta_info(karma_fasta* f, int64_t* n, int64_t* seq_bytes, int64_t* key_bytes, int* ascii);
int karma_fasta_get(karma_fasta* f, uint8_t* seq, int64_t* seq_off, char* keys, int64_t* key_off,
                    int32_t* key_len);
/* Zero-copy view of the parsed arrays (valid until karma_fasta_destroy). */
int karma_fasta_view(karma_fasta* f, const uint8_t** seq, const int64_t** seq_off, const char** keys,
                     const int64_t** key_off, const int32_t** key_len);
int karma_fasta_destroy(karma_fasta* f);

typedef struct karma_eq karma_eq;
/* eq_classes.txt -> names + the karma_graph_eq arrays (cls_off[C+1], members,
 * counts, pair_skip = eq_size token == "1"). */
int karma_eq_parse(const char* data, size_t len, int threads, karma_eq** out);
int karma_eq_info(karma_eq* q, int64_t* n_contigs, int64_t* n_classes, int64_t* n_members, int64_t* name_bytes);
int karma_eq_get(karma_eq* q, char* names, int64_t* name_off, int64_t* cls_off, uint32_t* members, int64_t* counts,
                 uint8_t* pair_skip);
/* The same classes in the compact form karma_graph_eq_compact takes: sizes[C] =
 * member count | 0x80 when the eq_size token is "1", counts[C] as u32 (names,
 * name_off, members as karma_eq_get).  KARMA_ERR_ARG, nothing written, when a
 * class has more than 127 members or a count past 2^32 - 1. */
int karma_eq_get_compact(karma_eq* q, char* names, int64_t* name_off, uint8_t* sizes, uint32_t* members,
                         uint32_t* counts);
int karma_eq_destroy(karma_eq* q);

typedef struct karma_sam karma_sam;
/* SAM lines -> one (read id, contig id) record per line (the karma_graph_records
 * input, unsorted); contig ids number RNAMEs in order of first appearance, read
 * ids are an injective numbering of QNAMEs below read_id_bound.  q_start/q_len
 * locate each line's QNAME in the caller's buffer. */
int karma_sam_parse(const char* data, size_t len, int skip_headers, int threads, karma_sam** out);
int karma_sam_info(karma_sam* s, int64_t* n_records, int64_t* n_reads, int64_t* n_contigs, int64_t* rname_bytes,
                   int64_t* read_id_bound);
int karma_sam_get(karma_sam* s, uint32_t* records, char* rnames, int64_t* rname_off, int64_t* q_start,
                  int32_t* q_len);
int karma_sam_destroy(karma_sam* s);

/* ---- graph consumers --------------------------------
 * read_graph.py:150-172 (get_unconnected_nodes / get_connected_nodes),
 * :174-190 + :315-344 (node weights, representative sequences) and :350-357
 * (edge_list, MCL stdin), as karma.py:255-395 uses them on
 * ReadGraph(full_graph.subgraph(cluster)).  A karma_adj is a graph laid out as
 * networkx iterates it: nodes in iteration order (positions 0..n-1, each with an
 * id into the caller's name table) and per node its neighbours (positions) and
 * weights in adjacency-dict order. */
typedef struct karma_adj karma_adj;
/* add_edge(a[e], b[e], weight=w[e]) for e = 0..n_edges-1 on a graph whose n
 * nodes were added first (positions = ids order when ids == NULL). */
int karma_adj_from_edges(karma_ctx* ctx, int64_t n, const uint32_t* ids, const uint32_t* a, const uint32_t* b,
                         const double* w, int64_t n_edges, int is_device, karma_adj** out);
/* An exported adjacency: off[n+1] into nbr (positions) / w, in dict order. */
int karma_adj_from_lists(karma_ctx* ctx, int64_t n, const uint32_t* ids, const int64_t* off, const uint32_t* nbr,
                         const double* w, int is_device, karma_adj** out);
/* nx.Graph(G.subgraph(nodes)) of G = src: order[k] = distinct src positions in
 * the view's node order (host).  Adjacency rebuilt as from_dict_of_dicts does.
 * Stream-ordered: no host synchronisation. */
int karma_adj_view(karma_adj* src, const int64_t* order, int64_t k, karma_adj** out);
/* The consumers of a small view in one launch and one host synchronisation:
 * for nx.Graph(G.subgraph(nodes)) of G = src (order as karma_adj_view), deg[k]
 * (karma_adj_degrees), w[k] (karma_adj_node_weights) and, when with_text, the
 * edge_list text (karma_adj_edge_list; names / name_off on the device) into
 * text[text_cap].  *done = 0 (nothing computed) when the view exceeds one
 * block: k > 1024 nodes, > 4096 adjacency entries or text over text_cap (or
 * about 1 MB); the caller then takes karma_adj_view and the calls above. */
int karma_adj_view_summary(karma_adj* src, const int64_t* order, int64_t k, const uint8_t* names,
                           const int64_t* name_off, int with_text, int64_t* deg, double* w, uint8_t* text,
                           int64_t text_cap, int64_t* text_len, int* done);
/* G.remove_nodes_from: keep[n] (host, 1 = stays), n_keep = ones in keep;
 * remaining orders unchanged.  No host synchronisation. */
int karma_adj_keep(karma_adj* src, const uint8_t* keep, int64_t n_keep, karma_adj** out);
int karma_adj_info(karma_adj* g, int64_t* n, int64_t* n_entries);
/* Host copies of the layout (any pointer may be NULL). */
int karma_adj_get(karma_adj* g, uint32_t* ids, int64_t* off, uint32_t* nbr, double* w);
/* len(G.adj[u]) per position (nx.all_neighbors, a self-loop once). */
int karma_adj_degrees(karma_adj* g, int64_t* deg_host);
/* 0 + w_1 + w_2 + ... over G.adj[u] in order, f64 left to right (read_graph.py:183-187). */
int karma_adj_node_weights(karma_adj* g, double* w_host);
/* Both of the above in one pass (either pointer may be NULL). */
int karma_adj_node_stats(karma_adj* g, int64_t* deg_host, double* w_host);
/* "\n".join(f"{A} {B} {w}" for A, B, w in G.edges(data="weight")) as UTF-8:
 * names[name_off[i]:name_off[i+1]] is the UTF-8 name of id i; w is written as
 * Python repr(float).  out == NULL: only *len (the text is kept for the copying call). */
int karma_adj_edge_list(karma_adj* g, const uint8_t* names, const int64_t* name_off, int64_t n_names,
                        int names_on_device, uint8_t* out, int64_t cap, int64_t* len);
/* --rearrange (karma.py:103-118): sub[u] = subcluster
 * index of position u (-1: none; each node in at most one), rank[u] = its index
 * in that subcluster's node list.  For every pair A < B joined by an edge:
 * pair = A << 32 | B, sum = 0 + w_1 + w_2 + ... over the edges between them in
 * itertools.product(nodes_A, nodes_B) order, n_edges = their count, n_over = how
 * many of the partial sums exceed cutoff (the reference appends [A, B] once per
 * such edge); sorted by (A, B).  All outputs NULL: only *n_pairs. */
int karma_adj_cross_sums(karma_adj* g, const int32_t* sub, const int32_t* rank, double cutoff, uint64_t* pair,
                         double* sum, int64_t* n_edges, int64_t* n_over, int64_t cap, int64_t* n_pairs);
int karma_adj_destroy(karma_adj* g);
/* Host build of the device's repr(float) formatter, for tests: one line per value. */
int karma_repr_f64_host(const double* x, int64_t n, char* out, int64_t cap, int64_t* len);

#ifdef __cplusplus
}
#endif
#endif /* KARMA_H */
