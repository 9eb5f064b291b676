// karma_internal.h — shared host/device plumbing of libkarma_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/karma.h"

namespace karma {

void set_error(const char* fmt, ...);

// HIP runtime calls made on this thread that enqueue work, wait, or manage
// streams/events/memory (launches, copies, memsets, event records, stream
// waits, synchronisations): karma_api_calls, the bench's api_calls_per_step.
// hipGetLastError and hipSetDevice (no queue traffic) are not counted.
extern thread_local uint64_t t_hip_calls;
constexpr bool counted_call(const char* e) {
    return !((e[0] == 'h' && e[1] == 'i' && e[2] == 'p' && e[3] == 'G' && e[4] == 'e' && e[5] == 't' && e[6] == 'L') ||
             (e[0] == 'h' && e[1] == 'i' && e[2] == 'p' && e[3] == 'S' && e[4] == 'e' && e[5] == 't' && e[6] == 'D'));
}

#define KARMA_HIP(expr)                                                                     \
    do {                                                                                    \
        if (::karma::counted_call(#expr)) ++::karma::t_hip_calls;                           \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            ::karma::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
            return _e == hipErrorOutOfMemory ? KARMA_ERR_OOM : KARMA_ERR_HIP;               \
        }                                                                                   \
    } while (0)

#define KARMA_CHECK(cond, code, ...)      \
    do {                                  \
        if (!(cond)) {                    \
            ::karma::set_error(__VA_ARGS__); \
            return (code);                \
        }                                 \
    } while (0)

#define KARMA_TRY(expr)          \
    do {                         \
        int _rc = (expr);        \
        if (_rc != KARMA_OK) return _rc; \
    } while (0)

struct TimedLaunch {
    const char* name;
    hipEvent_t start, stop;
};

}  // namespace karma

struct karma_ctx {
    int device = 0;
    int cu_count = 256;  // compute units of the device
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // exact-size caching allocator: repeated steps of identical shape never hipMalloc
    // cached device blocks by (stream they were allocated on, bytes): a block
    // is reused only by allocations on that same stream, whose later work
    // stream order puts after every earlier reader there (a side stream's
    // temporaries never reach the main stream's allocations while its kernels
    // may still read them).  Work on another stream that reads a block is
    // joined back before its owner frees it (the side-stream profile: ctx_join).
    std::multimap<std::pair<hipStream_t, size_t>, void*> free_list;
    std::map<void*, std::pair<size_t, hipStream_t>> live;  // bytes, allocating stream
    size_t cached_bytes = 0;
    // per-kernel event timing
    bool timing = false;
    std::string timing_only;  // empty: time every kernel
    std::vector<karma::TimedLaunch> launches;
    std::vector<hipEvent_t> event_pool;
    // pinned host scratch for small status readbacks (one async copy + one sync)
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    // a split graph call (karma_graph_records_begin/_end) keeps its control-block
    // readback here until _end, so calls in between may use `pinned`
    void* job_pinned = nullptr;
    size_t job_pinned_bytes = 0;
    bool job_open = false;
    hipEvent_t side_ev = nullptr;  // main -> side stream ordering (karma_kmer_profile_side)
    int grid_headroom = 0;         // blocks per CU resident_grid leaves free (a side-stream launch)
    int side_headroom = 0;         // grid_headroom of karma_kmer_profile_side (karma_ctx_set_side_headroom)
    hipEvent_t mark_ev = nullptr;  // recorded by an open graph job after its classify kernel
    bool mark_set = false;
    int mark_pos = -1;  // where an open graph job records mark_ev (SetsJob::launch); -1: the default
    int64_t* fin_pinned = nullptr;  // M of an in-flight karma_kmer_plan_finalize_async
    // mapped, coherent pinned host memory that kernels read and write directly
    // (one-launch consumers of small views: no copy launches)
    void* mapped = nullptr;
    void* mapped_dev = nullptr;
    size_t mapped_bytes = 0;
    // owner bounds for the next records graph job (karma_graph_split_hint): its
    // final kernel also finds where each owner's slice starts (no split launch)
    std::vector<int64_t> split_bounds;
    // resident blocks per CU by (kernel, block size, dynamic LDS): the occupancy
    // query costs host microseconds and is asked on every call of a step
    std::map<std::pair<const void*, std::pair<int, size_t>>, int> occupancy;
    // a records graph job's second branch (general reads' pairs: general,
    // pair partition, pair reduce) runs here beside the code branch, forked
    // after classify and joined before the final kernel (SetsJob::launch)
    hipStream_t fork_stream = nullptr;
    hipEvent_t fork_a = nullptr, fork_b = nullptr;
    hipEvent_t xfer_ev[4] = {};  // the eq path's staged host->device copies on fork_stream
    bool no_fork = false;        // the next records job keeps its general branch on its own stream
    // an idle stream of the caller's to fork onto instead of fork_stream (a
    // step's spare main stream): every stream the process creates takes one of
    // its 4 hardware queues in turn, and a 6th stream shares the 2nd's -- a
    // records job's main stream (config 3: 1.52 against 1.2 ms per step)
    hipStream_t fork_use = nullptr;
    int64_t eq_pair_cap = 0;     // the eq path's previous pair total (its speculative scratch size)
    // a zeroed control block the next deferred records job may use instead of
    // its own (a native step's, kept zero by the step's status kernel): no
    // clearing launch ahead of classify, no relabel probe (classify votes)
    int64_t* job_ctrl = nullptr;
    int64_t job_ctrl_words = 0;
    // the next k-mer plan may take this zeroed block for its presence bitmap
    // and exception counter (no clearing memset); its column table kernel
    // clears it again (karma_step, per side stream)
    uint32_t* plan_zeroed = nullptr;
    int64_t plan_zeroed_words = 0;
};

namespace karma {

int ctx_alloc(karma_ctx* ctx, size_t bytes, void** out);
void ctx_free(karma_ctx* ctx, void* p);
int ctx_begin(karma_ctx* ctx);  // hipSetDevice
// Grid of one round: blocks that fit on the device at once for this kernel,
// block size and dynamic LDS (at least 1, at most `work` blocks).
int resident_grid(karma_ctx* ctx, const void* kernel, int block, size_t lds, int64_t work);
// Pinned host scratch of >= bytes (valid until the next call on this ctx).
int ctx_fork(karma_ctx* ctx);  // creates ctx->fork_stream and its two events on first use
int ctx_pinned(karma_ctx* ctx, size_t bytes, void** out);
// Mapped coherent pinned host memory that kernels read and write directly.
// One region per context, allocated once and freed only with the context, cut
// into fixed per-user slots, so two users never alias (a side-stream
// collective's scalars beside a main-stream status word, say) and no address
// handed out is ever freed while a stream may still use it.
enum MappedSlot : int {
    kMapConsumers = 0,  // karma_adj_view_summary inputs and results (1 MiB)
    kMapCommScalar,     // karma_comm_allreduce_host: host scalars (8 x world)
    kMapCommCounts,     // karma_comm_exchange_counts: sent and received counts (16 x world)
    kMapSplit,          // karma_pairs_split{,_kc}: bounds and starts (2 x (nranks + 1) x 8)
    kMapMerge,          // karma_pairs_merge_runs: unique-key count, order flag
    kMapEdges,          // karma_edges_end: zero-division flag, edge count, order flag
    kMapStep,           // karma_step: per-step status words (deferred checks)
    kMapSideScalar,     // the side-stream communicator's host scalars (8 x world)
    kMapSlots
};
// Byte offset and capacity of each slot (karma_ctx_mapped_layout exposes them).
int64_t mapped_slot_offset(int slot);
int64_t mapped_slot_bytes(int slot);
int ctx_mapped(karma_ctx* ctx, int slot, size_t bytes, void** host, void** dev);
// Pinned scratch owned by the open split graph call (valid until its _end).
int ctx_job_pinned(karma_ctx* ctx, size_t bytes, void** out);
// Wrap a launch with HIP events when timing is on.
void timing_start(karma_ctx* ctx, const char* name, hipEvent_t* ev_stop);
void timing_stop(karma_ctx* ctx, hipEvent_t ev_stop);

template <typename T>
struct DevArray {
    karma_ctx* ctx = nullptr;
    T* ptr = nullptr;
    size_t n = 0;
    DevArray() = default;
    DevArray(const DevArray&) = delete;
    DevArray& operator=(const DevArray&) = delete;
    ~DevArray() { release(); }
    int alloc(karma_ctx* c, size_t count) {
        release();
        ctx = c;
        n = count;
        void* p = nullptr;
        int rc = ctx_alloc(c, (count ? count : 1) * sizeof(T), &p);
        ptr = static_cast<T*>(p);
        return rc;
    }
    void release() {
        if (ptr) ctx_free(ctx, ptr);
        ptr = nullptr;
        n = 0;
    }
    void swap(DevArray& o) {
        std::swap(ctx, o.ctx);
        std::swap(ptr, o.ptr);
        std::swap(n, o.n);
    }
};

#define KARMA_LAUNCH(ctx, name, kernel, grid, block, shmem, ...)                         \
    do {                                                                                \
        hipEvent_t _stop = nullptr;                                                     \
        ::karma::timing_start((ctx), (name), &_stop);                                   \
        ++::karma::t_hip_calls;                                                         \
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), (shmem), (ctx)->stream, __VA_ARGS__); \
        ::karma::timing_stop((ctx), _stop);                                             \
        KARMA_HIP(hipGetLastError());                                                   \
    } while (0)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Generic (key u64, count i64[, first u64]) sort + reduce-by-key on the device.
// Used by the low-volume paths (eq classes, exchange merge, bucket overflow).
int sort_reduce_pairs(karma_ctx* ctx, const uint64_t* keys_in, const int64_t* counts_in, const uint64_t* first_in,
                      int64_t n, int key_bits, DevArray<uint64_t>& keys_out, DevArray<int64_t>& counts_out,
                      DevArray<uint64_t>* first_out, int64_t* n_out);

// sort.hip: the library's own single-launch look-back scans, stable LSD radix
// sorts (u32 values move with the keys; vin == NULL: the input positions;
// vout == NULL: keys only) and the reduce-by-key of a sorted array (counts
// summed and the smallest "first" per group, both read through perm when given;
// cin == NULL counts 1 each, fin == NULL takes the position itself; uc / uf
// may be NULL; the group count lands in *n_out_dev on the device).
int scan_excl_i64(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n);
int scan_excl_u32(karma_ctx* ctx, const uint32_t* in, int64_t* out, int64_t n);
// out[c] = sum over classes before c of m (m - 1) / 2 (0 where skip[c]), c <= C
int scan_excl_pairs(karma_ctx* ctx, const int64_t* off, const uint8_t* skip, int64_t C, int64_t* out);
// compact eq classes: off[c] = sum of (sizes & 0x7F) before c (c <= C), skip[c] = sizes[c] >> 7
int scan_excl_sizes(karma_ctx* ctx, const uint8_t* sizes, uint8_t* skip, int64_t C, int64_t* off);
int radix_sort_u64(karma_ctx* ctx, const uint64_t* kin, const uint32_t* vin, int64_t n, int key_bits,
                   uint64_t* kout, uint32_t* vout);
int radix_sort_u32(karma_ctx* ctx, const uint32_t* kin, const uint32_t* vin, int64_t n, int key_bits,
                   uint32_t* kout, uint32_t* vout);
int reduce_sorted(karma_ctx* ctx, const uint64_t* keys, const uint32_t* perm, const int64_t* cin,
                  const uint64_t* fin, int64_t n, uint64_t* uk, int64_t* uc, uint64_t* uf, int64_t* n_out_dev);

// k-mer plan internals for karma_step (kmer.hip)
int64_t kmer_m_cap(const karma_kmer_plan* p);
int kmer_finalize_device(karma_kmer_plan* p, int64_t* m_out, int64_t* m_host);
int kmer_profile_device_m(karma_kmer_plan* p, double* out_dev, const int64_t* m_dev);
int kmer_set_m(karma_kmer_plan* p, int64_t M);
// graph.hip: a pending edge stage's status words (see karma_edges_end), handed over
const int64_t* edges_take_pending(karma_edges* e);

}  // namespace karma

struct karma_pairs {
    karma_ctx* ctx = nullptr;
    int64_t n = 0;
    int64_t n_contigs = 0;
    karma::DevArray<uint64_t> keys;
    karma::DevArray<int64_t> counts;
    karma::DevArray<uint64_t> first;   // eq path only
    karma::DevArray<int64_t> totals;   // eq path only
    bool has_first = false;
    bool has_totals = false;
    // An owner's merge of received runs may leave equal keys adjacent (dups):
    // the edge stage and the totals sum such groups themselves; every other
    // accessor compacts the list first (graph.hip compact_pairs).  bad: the
    // merge's order check (device flag), read at the next synchronisation.
    bool dups = false;
    karma::DevArray<int64_t> bad;
    // karma_pairs_split's answer for split_bounds, found by the records job
    // that built the list (empty: search on demand)
    std::vector<int64_t> split_bounds, split_starts;
};

namespace karma {
// The graph's input records (karma_graph_records, karma_step_run): either
// interleaved {u32 read id, u32 contig} grouped by read (pr; KARMA_REC_SORTED),
// or one u32 per record, contig | first-of-its-read << 31 (fw;
// KARMA_REC_FLAGGED): the graph depends only on which records share a read, so
// the read ids are replaced by read-start flags and the records take 4 bytes.
struct RecIn {
    const uint2* pr = nullptr;
    const uint32_t* fw = nullptr;
    __host__ __device__ bool flagged() const { return fw != nullptr; }
    __device__ __forceinline__ uint32_t contig(int64_t i) const { return fw ? fw[i] & 0x7FFFFFFFu : pr[i].y; }
    // record i (> 0) belongs to the read of record i - 1
    __device__ __forceinline__ bool cont(int64_t i) const { return fw ? (int)fw[i] >= 0 : pr[i].x == pr[i - 1].x; }
};
// set-partition records pipeline (graph_sets.hip)
int records_to_pairs_sets(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, karma_pairs* out);
// The same in two halves: sets_begin enqueues every kernel up to the control
// block readback and returns; sets_end synchronises and assembles the list.
// Only for N <= sets_max_contigs() (the compact path); `rec` must stay valid
// until sets_end.
struct SetsJob;
int64_t sets_max_contigs();
int sets_begin(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, SetsJob** job);
int sets_end(SetsJob* job, karma_pairs* out);  // frees the job
void sets_free(SetsJob* job);
// A records job launched without its control-block readback (karma_step's
// deferred steps): nothing waits for it; the list and the words that say
// whether the common path held stay on the device.
struct SetsDeferred {
    const uint64_t* keys = nullptr;  // the final kernel's list: sorted unique keys ...
    const int64_t* counts = nullptr;  // ... and counts, dst[B] of them
    int64_t cap = 0;                  // capacity of keys / counts
    const int64_t* dst = nullptr;     // per-bucket list offsets (B + 1; dst[B] = list length)
    const int64_t* split_loc = nullptr;  // per split bound: keys of its bucket below it
    std::vector<int64_t> split_b;     // the split bounds (host)
    int B = 0, bw = 0;
    const int* flags = nullptr;       // [0] unsorted, [1] contig range, [2] pair capacity, [3] partition check
    const unsigned* counters = nullptr;  // [0] big reads, [3] relabel vote
    const uint8_t* ovf = nullptr;     // per bucket: overflowed the LDS tables (generic path needed)
    int64_t* ctrl = nullptr;          // the caller's control block when the job used it (ctx->job_ctrl), else null
    int64_t ctrl_need = 0;            // words of control block the job needed (a larger ctx->job_ctrl next time)
};
int sets_begin_deferred(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, SetsJob** job, SetsDeferred* view);
// Frees a deferred job's buffers to the allocator (stream-ordered; no wait).
void sets_release(SetsJob* job);
}  // namespace karma
