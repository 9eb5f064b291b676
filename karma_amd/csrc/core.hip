// core.hip — context, errors, caching allocator, per-kernel event timing.
#include <algorithm>
#include <cstdarg>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "karma_internal.h"

namespace karma {

static thread_local std::string g_err;
thread_local uint64_t t_hip_calls = 0;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

int ctx_begin(karma_ctx* ctx) {
    KARMA_CHECK(ctx, KARMA_ERR_ARG, "null karma_ctx");
    KARMA_HIP(hipSetDevice(ctx->device));
    return KARMA_OK;
}

int ctx_alloc(karma_ctx* ctx, size_t bytes, void** out) {
    bytes = (bytes + 255) & ~size_t(255);
    auto it = ctx->free_list.find({ctx->stream, bytes});
    if (it != ctx->free_list.end()) {
        *out = it->second;
        ctx->free_list.erase(it);
        ctx->cached_bytes -= bytes;
        ctx->live[*out] = {bytes, ctx->stream};
        return KARMA_OK;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
        // drop the cache and retry once
        (void)hipGetLastError();
        hipDeviceSynchronize();  // cached blocks of every stream are idle
        for (auto& kv : ctx->free_list) hipFree(kv.second);
        ctx->free_list.clear();
        ctx->cached_bytes = 0;
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess) {
        set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        return KARMA_ERR_OOM;
    }
    ctx->live[p] = {bytes, ctx->stream};
    *out = p;
    return KARMA_OK;
}

void ctx_free(karma_ctx* ctx, void* p) {
    if (!p || !ctx) return;
    auto it = ctx->live.find(p);
    if (it == ctx->live.end()) return;
    // stream-ordered reuse: later work on the same stream runs after earlier frees' readers
    ctx->free_list.emplace(std::make_pair(it->second.second, it->second.first), p);
    ctx->cached_bytes += it->second.first;
    ctx->live.erase(it);
}

void timing_start(karma_ctx* ctx, const char* name, hipEvent_t* ev_stop) {
    *ev_stop = nullptr;
    if (!ctx->timing) return;
    if (!ctx->timing_only.empty() && ctx->timing_only != name) return;
    hipEvent_t a, b;
    if (ctx->event_pool.size() >= 2) {
        a = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        b = ctx->event_pool.back();
        ctx->event_pool.pop_back();
    } else {
        hipEventCreate(&a);
        hipEventCreate(&b);
    }
    hipEventRecord(a, ctx->stream);
    ctx->launches.push_back({name, a, b});
    *ev_stop = b;
}

void timing_stop(karma_ctx* ctx, hipEvent_t ev_stop) {
    if (ev_stop) hipEventRecord(ev_stop, ctx->stream);
}

int ctx_job_pinned(karma_ctx* ctx, size_t bytes, void** out) {
    if (ctx->job_pinned_bytes < bytes) {
        if (ctx->job_pinned) KARMA_HIP(hipHostFree(ctx->job_pinned));
        ctx->job_pinned = nullptr;
        ctx->job_pinned_bytes = 0;
        const size_t want = std::max<size_t>(bytes, 64 * 1024);
        KARMA_HIP(hipHostMalloc(&ctx->job_pinned, want, hipHostMallocDefault));
        ctx->job_pinned_bytes = want;
    }
    *out = ctx->job_pinned;
    return KARMA_OK;
}

int resident_grid(karma_ctx* ctx, const void* kernel, int block, size_t lds, int64_t work) {
    const auto key = std::make_pair(kernel, std::make_pair(block, lds));
    auto it = ctx->occupancy.find(key);
    int per_cu = 0;
    if (it != ctx->occupancy.end()) {
        per_cu = it->second;
    } else {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess || per_cu < 1)
            per_cu = 1;
        ctx->occupancy.emplace(key, per_cu);
    }
    per_cu = std::max(1, per_cu - ctx->grid_headroom);
    return (int)std::max<int64_t>(1, std::min<int64_t>(work, (int64_t)per_cu * ctx->cu_count));
}

// the context's second stream (a records job's general branch, the eq path's
// staged copies), created on first use at the highest priority
int ctx_fork(karma_ctx* ctx) {
    if (!ctx->fork_a) {
        KARMA_HIP(hipEventCreateWithFlags(&ctx->fork_a, hipEventDisableTiming));
        KARMA_HIP(hipEventCreateWithFlags(&ctx->fork_b, hipEventDisableTiming));
    }
    if (!ctx->fork_stream && !ctx->fork_use) {
        int lo = 0, hi = 0;
        KARMA_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        KARMA_HIP(hipStreamCreateWithPriority(&ctx->fork_stream, hipStreamNonBlocking, hi));
    }
    return KARMA_OK;
}

int ctx_pinned(karma_ctx* ctx, size_t bytes, void** out) {
    if (ctx->pinned_bytes < bytes) {
        if (ctx->pinned) KARMA_HIP(hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        const size_t want = std::max<size_t>(bytes, 64 * 1024);
        KARMA_HIP(hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault));
        ctx->pinned_bytes = want;
    }
    *out = ctx->pinned;
    return KARMA_OK;
}

// Slot capacities (bytes, multiples of 256); offsets are their prefix sums.
static constexpr int64_t kMapCap[kMapSlots] = {
    int64_t(1) << 20,  // consumers
    8 * 1024,          // comm scalars: world <= 1024
    16 * 1024,         // comm counts: world <= 1024
    16 * 1024 + 256,   // split: nranks <= 1023
    256,               // merge status
    256,               // edge status
    8192,              // step status (64 entries of 64 B) and column counts (64 x 8 B)
    8 * 1024,          // side communicator scalars
};

int64_t mapped_slot_bytes(int slot) { return slot >= 0 && slot < kMapSlots ? kMapCap[slot] : 0; }

int64_t mapped_slot_offset(int slot) {
    int64_t o = 0;
    for (int s = 0; s < slot && s < kMapSlots; ++s) o += kMapCap[s];
    return o;
}

int ctx_mapped(karma_ctx* ctx, int slot, size_t bytes, void** host, void** dev) {
    KARMA_CHECK(slot >= 0 && slot < kMapSlots, KARMA_ERR_ARG, "mapped slot %d out of range", slot);
    KARMA_CHECK((int64_t)bytes <= kMapCap[slot], KARMA_ERR_ARG, "mapped slot %d holds %lld bytes, %zu asked", slot,
                (long long)kMapCap[slot], bytes);
    if (!ctx->mapped) {  // allocated once, freed with the context
        const size_t total = (size_t)mapped_slot_offset(kMapSlots);
        KARMA_HIP(hipHostMalloc(&ctx->mapped, total, hipHostMallocMapped | hipHostMallocCoherent));
        ctx->mapped_bytes = total;
        KARMA_HIP(hipHostGetDevicePointer(&ctx->mapped_dev, ctx->mapped, 0));
    }
    const int64_t o = mapped_slot_offset(slot);
    *host = static_cast<uint8_t*>(ctx->mapped) + o;
    *dev = static_cast<uint8_t*>(ctx->mapped_dev) + o;
    return KARMA_OK;
}


// ---- pinned host blocks for results (karma_host_alloc) ---------------------------
// A D2H copy into pageable memory runs at about half the rate of one into
// pinned memory (8 MB of eq edges: 0.257 against 0.152 ms, profiles/r04/measurements.md (meas_c)),
// and hipHostMalloc itself costs far more than the copy, so freed blocks are
// kept by size class (powers of two from 4 KiB) for the next caller.
namespace {
std::mutex g_host_mu;
std::map<size_t, std::vector<void*>> g_host_free;  // size class -> free blocks
std::map<void*, size_t> g_host_live;                // block -> size class
size_t g_host_cached = 0;
constexpr size_t kHostCacheMax = size_t(1) << 30;  // free bytes kept at most
size_t host_class(size_t bytes) {
    size_t c = 4096;
    while (c < bytes) c <<= 1;
    return c;
}
}  // namespace

}  // namespace karma

using namespace karma;

extern "C" {

int karma_version(void) { return 1; }

// The build's identity, for the bench line and the default-build check:
// KARMA_BUILD_DEFINES holds the -D flags a variant build added on top of the
// Makefile's (empty for the shipped library), KARMA_SRC_HASH the first 16 hex
// digits of sha256 over the sources (Makefile).
#ifndef KARMA_BUILD_DEFINES
#define KARMA_BUILD_DEFINES "unknown (not built by karma_amd/csrc/Makefile)"
#endif
#ifndef KARMA_SRC_HASH
#define KARMA_SRC_HASH "unknown"
#endif
const char* karma_build_info(void) {
    return "{\"arch\": \"gfx950\", \"defines\": \"" KARMA_BUILD_DEFINES "\", \"src_sha256_16\": \"" KARMA_SRC_HASH
           "\", \"flags\": \"-O3 -ffp-contract=off -fno-fast-math\"}";
}

const char* karma_last_error(void) { return g_err.c_str(); }

int karma_api_calls(uint64_t* n) {
    KARMA_CHECK(n, KARMA_ERR_ARG, "null out");
    *n = t_hip_calls;
    return KARMA_OK;
}

int karma_mapped_slots(int64_t* offsets, int64_t* bytes, int cap, int* n) {
    KARMA_CHECK(n && (cap <= 0 || (offsets && bytes)), KARMA_ERR_ARG, "karma_mapped_slots: bad arguments");
    for (int s = 0; s < kMapSlots && s < cap; ++s) {
        offsets[s] = mapped_slot_offset(s);
        bytes[s] = mapped_slot_bytes(s);
    }
    *n = kMapSlots;
    return KARMA_OK;
}

int karma_device_count(int* n) {
    KARMA_CHECK(n, KARMA_ERR_ARG, "null out");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
        return KARMA_ERR_HIP;
    }
    *n = c;
    return KARMA_OK;
}

int karma_ctx_create(int device, karma_ctx** out) {
    KARMA_CHECK(out, KARMA_ERR_ARG, "null out");
    int n = 0;
    KARMA_HIP(hipGetDeviceCount(&n));
    KARMA_CHECK(device >= 0 && device < n, KARMA_ERR_ARG, "device %d out of range (%d devices)", device, n);
    KARMA_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    KARMA_HIP(hipGetDeviceProperties(&prop, device));
    KARMA_CHECK(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, KARMA_ERR_HIP,
                "device %d is %s; libkarma_hip is built for gfx950 only", device, prop.gcnArchName);
    karma_ctx* ctx = new karma_ctx();
    ctx->device = device;
    ctx->cu_count = prop.multiProcessorCount;
    hipError_t e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        set_error("hipStreamCreate: %s", hipGetErrorString(e));
        return KARMA_ERR_HIP;
    }
    ctx->stream = ctx->own_stream;
    *out = ctx;
    return KARMA_OK;
}

int karma_ctx_destroy(karma_ctx* ctx) {
    if (!ctx) return KARMA_OK;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->free_list) hipFree(kv.second);
    for (auto& kv : ctx->live) hipFree(kv.first);
    for (auto& l : ctx->launches) {
        hipEventDestroy(l.start);
        hipEventDestroy(l.stop);
    }
    for (auto e : ctx->event_pool) hipEventDestroy(e);
    if (ctx->fork_stream) {
        hipStreamSynchronize(ctx->fork_stream);
        hipStreamDestroy(ctx->fork_stream);
    }
    if (ctx->fork_a) hipEventDestroy(ctx->fork_a);
    if (ctx->fork_b) hipEventDestroy(ctx->fork_b);
    for (hipEvent_t e : ctx->xfer_ev)
        if (e) hipEventDestroy(e);
    if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
    if (ctx->pinned) hipHostFree(ctx->pinned);
    if (ctx->job_pinned) hipHostFree(ctx->job_pinned);
    if (ctx->side_ev) hipEventDestroy(ctx->side_ev);
    if (ctx->mark_ev) hipEventDestroy(ctx->mark_ev);
    if (ctx->fin_pinned) hipHostFree(ctx->fin_pinned);
    if (ctx->mapped) hipHostFree(ctx->mapped);
    delete ctx;
    return KARMA_OK;
}

int karma_ctx_set_stream(karma_ctx* ctx, void* s) {
    KARMA_CHECK(ctx, KARMA_ERR_ARG, "null ctx");
    ctx->stream = s ? static_cast<hipStream_t>(s) : ctx->own_stream;
    return KARMA_OK;
}

int karma_ctx_sync(karma_ctx* ctx) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int karma_timing_enable(karma_ctx* ctx, int on) {
    KARMA_CHECK(ctx, KARMA_ERR_ARG, "null ctx");
    ctx->timing = on != 0;
    return KARMA_OK;
}

int karma_timing_only(karma_ctx* ctx, const char* name) {
    KARMA_CHECK(ctx, KARMA_ERR_ARG, "null ctx");
    ctx->timing_only = name ? name : "";
    return KARMA_OK;
}

int karma_timing_reset(karma_ctx* ctx) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    for (auto& l : ctx->launches) {
        ctx->event_pool.push_back(l.start);
        ctx->event_pool.push_back(l.stop);
    }
    ctx->launches.clear();
    return KARMA_OK;
}

int karma_timing_read(karma_ctx* ctx, char* names, double* total_ms, int64_t* launches, int cap, int* n) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<std::string> order;
    std::map<std::string, std::pair<double, int64_t>> acc;
    for (auto& l : ctx->launches) {
        float ms = 0.f;
        KARMA_HIP(hipEventElapsedTime(&ms, l.start, l.stop));
        auto it = acc.find(l.name);
        if (it == acc.end()) {
            order.push_back(l.name);
            acc[l.name] = {ms, 1};
        } else {
            it->second.first += ms;
            it->second.second += 1;
        }
    }
    int k = 0;
    for (auto& nm : order) {
        if (k >= cap) break;
        std::strncpy(names + 64 * k, nm.c_str(), 63);
        names[64 * k + 63] = 0;
        total_ms[k] = acc[nm].first;
        launches[k] = acc[nm].second;
        ++k;
    }
    *n = (int)order.size();
    return KARMA_OK;
}

int karma_dev_alloc(karma_ctx* ctx, size_t bytes, void** out) {
    KARMA_TRY(ctx_begin(ctx));
    return ctx_alloc(ctx, bytes, out);
}

int karma_dev_free(karma_ctx* ctx, void* p) {
    KARMA_TRY(ctx_begin(ctx));
    ctx_free(ctx, p);
    return KARMA_OK;
}

int karma_memcpy(karma_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
    KARMA_TRY(ctx_begin(ctx));
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    KARMA_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int karma_memcpy_async(karma_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
    KARMA_TRY(ctx_begin(ctx));
    if (!bytes) return KARMA_OK;
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    KARMA_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->stream));
    return KARMA_OK;
}

// The write ceiling of this device for a buffer of `bytes`: hipMemsetAsync
// timed with events on the context's stream (bench.py reports the profile's
// write rate against it, measured in the same process).
int karma_memset_timed(karma_ctx* ctx, void* dst, size_t bytes, int reps, double* ms) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(dst && ms && reps >= 1, KARMA_ERR_ARG, "karma_memset_timed: bad arguments");
    hipEvent_t a, b;
    KARMA_HIP(hipEventCreate(&a));
    KARMA_HIP(hipEventCreate(&b));
    KARMA_HIP(hipMemsetAsync(dst, 0, bytes, ctx->stream));  // warm
    KARMA_HIP(hipEventRecord(a, ctx->stream));
    for (int r = 0; r < reps; ++r) KARMA_HIP(hipMemsetAsync(dst, r & 1, bytes, ctx->stream));
    KARMA_HIP(hipEventRecord(b, ctx->stream));
    KARMA_HIP(hipEventSynchronize(b));
    float t = 0.f;
    KARMA_HIP(hipEventElapsedTime(&t, a, b));
    hipEventDestroy(a);
    hipEventDestroy(b);
    *ms = t / reps;
    return KARMA_OK;
}

int karma_host_alloc(size_t bytes, void** out) {
    KARMA_CHECK(out, KARMA_ERR_ARG, "karma_host_alloc: null out");
    const size_t c = host_class(std::max<size_t>(bytes, 1));
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = g_host_free.find(c);
        if (it != g_host_free.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            g_host_cached -= c;
            g_host_live[*out] = c;
            return KARMA_OK;
        }
    }
    void* p = nullptr;
    KARMA_HIP(hipHostMalloc(&p, c, hipHostMallocDefault));
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_live[p] = c;
    *out = p;
    return KARMA_OK;
}

int karma_host_free(void* p) {
    if (!p) return KARMA_OK;
    size_t c = 0;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = g_host_live.find(p);
        KARMA_CHECK(it != g_host_live.end(), KARMA_ERR_ARG, "karma_host_free: not a karma_host_alloc block");
        c = it->second;
        g_host_live.erase(it);
        if (g_host_cached + c <= kHostCacheMax) {
            g_host_free[c].push_back(p);
            g_host_cached += c;
            return KARMA_OK;
        }
    }
    KARMA_HIP(hipHostFree(p));
    return KARMA_OK;
}

int karma_memset_async(karma_ctx* ctx, void* dst, int value, size_t bytes) {
    KARMA_TRY(ctx_begin(ctx));
    if (!bytes) return KARMA_OK;
    KARMA_HIP(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return KARMA_OK;
}

int karma_stream_create(karma_ctx* ctx, int priority, void** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out, KARMA_ERR_ARG, "null out");
    int lo = 0, hi = 0;
    KARMA_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));  // hi is the numerically smallest (highest)
    const int p = std::max(hi, std::min(lo, priority));
    hipStream_t s = nullptr;
    KARMA_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p));
    *out = s;
    return KARMA_OK;
}

int karma_stream_destroy(karma_ctx* ctx, void* s) {
    KARMA_TRY(ctx_begin(ctx));
    if (!s) return KARMA_OK;
    KARMA_CHECK(s != ctx->own_stream, KARMA_ERR_ARG, "the context's own stream is destroyed with the context");
    if (ctx->stream == s) ctx->stream = ctx->own_stream;
    KARMA_HIP(hipStreamSynchronize(static_cast<hipStream_t>(s)));
    // its cached blocks are idle now: hand them to the context's own stream
    // (a later stream may reuse this handle value)
    for (auto it = ctx->free_list.begin(); it != ctx->free_list.end();) {
        if (it->first.first == s) {
            ctx->free_list.emplace(std::make_pair(ctx->own_stream, it->first.second), it->second);
            it = ctx->free_list.erase(it);
        } else {
            ++it;
        }
    }
    KARMA_HIP(hipStreamDestroy(static_cast<hipStream_t>(s)));
    return KARMA_OK;
}

int karma_stream_sync(karma_ctx* ctx, void* s) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_HIP(hipStreamSynchronize(s ? static_cast<hipStream_t>(s) : ctx->stream));
    return KARMA_OK;
}

}  // extern "C"
