// capi.hip — the C ABI (include/svo_c.h): contexts, device-resident pyramid sets, alignment batches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "svo_internal.h"
#include "svo_math.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define SVO_HIP(call)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) return fail(SVO_ERR_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                                        \
    } while (0)

svo::LevelGeom make_geom(int32_t w, int32_t h, int32_t levels) {
    svo::LevelGeom g{};
    int64_t off = 0;
    for (int l = 0; l < levels; ++l) {
        g.w[l] = w; g.h[l] = h; g.off[l] = off;
        off += ((int64_t)w * h + 255) / 256 * 256;  // 256-B aligned level planes (16-B row-block loads)
        w = (w + 1) / 2;
        h = (h + 1) / 2;
    }
    g.frame_bytes = off;
    g.levels = levels;
    return g;
}

}  // namespace

constexpr int32_t kSplitMin = 64;  // batches of at least this many pairs run as kSplits concurrent chains
constexpr int kSplits = 2;         // measured on MI355X at 512 pairs: 1 / 2 / 3 / 4 chains = 335k / 355k / 359k / 352k pairs/s
// reference mode on K2V (one pair per CU for the whole robust scale): more chains give the other chains' K1 / K3 more
// ways into the CUs a K2V launch frees pair by pair (MI355X, round 5, same box: 512 pairs 2 / 4 chains = 172.4-172.9k /
// 173.7-174.0k pairs/s; 1024 pairs 174.4-175.0k / 177.9-178.0k; 3 chains at 512: 169.6-170.2k)
constexpr int kSplitsRefv = 4;
constexpr int32_t kSplitsRefvMin = 512;

struct svo_ctx {
    int32_t device;
    // the context stream; every use goes through ctx_stream(), which first joins a batch's pending chains (below)
    hipStream_t stream_raw;
    hipStream_t sides[4];         // extra streams: a batch runs as concurrent sub-batch chains
    hipEvent_t fork, joins[4];    // sides wait for stream at fork; stream waits for each side at its join
    // Chains of a batch run are joined into the context stream lazily: a run leaves its side chains pending, the
    // next run of the same batch (same split) lets each chain follow its own previous run on its own stream, and any
    // other use of the context stream joins them first (ctx_stream).  So back-to-back runs of one batch are ordered
    // per chain -- the only data dependency between them: chain i reads and writes only its own pairs -- instead of
    // every chain of run k + 1 waiting for the slowest chain of run k.  SVO_DEFER_JOIN=0 joins after every run.
    const struct svo_align_batch* pending_batch = nullptr;
    int pending_chains = 0;
    hipEvent_t chain_marks[3][2 + 3 * svo::kMaxLevels];  // launch marks of chains 0..2 (staggered starts)
    hipEvent_t events[16];
    // svo_align_batch_set_pairs uploads on its own stream, so the copies overlap a pyramid build queued
    // on `stream`; staged: the upload is done; stage_free: the last scatter out of a staging block is done
    hipStream_t copy;
    hipEvent_t staged, stage_free;
    // svo_pyramid_set_build_async builds on its own stream, after everything queued on `stream` so far (prep_gate),
    // so that the next batch's pyramids build while the current batch aligns
    hipStream_t prep = nullptr;
    hipEvent_t prep_gate = nullptr;
    // grow-only scratch of the synchronous per-call entry points (FeatureAlignment): no device
    // allocation per call once warm
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    // pinned host staging of the same calls (fixed size, ctx_pinned): one H2D and one D2H copy per call
    void* pinned = nullptr;
    void* pinned_dev = nullptr;  // the same block as the device addresses it (stage_copy)
    size_t pinned_bytes = 0;
    // svo_align_batch_set_pair stages into the same block as a ring without waiting for its copies;
    // every other user of the block first drains them (ctx_pinned)
    size_t ring_off = 0;
    bool ring_pending = false;
    // pyramid sets with a build_async the context stream has not waited for yet (set_join removes them); the
    // batches' runs join the sets their pairs read from this list (a batch never dereferences a set it keeps)
    std::vector<svo_pyramid_set*> pending_sets;
};

// the context stream after the pending chains of the last batch run (see svo_ctx::pending_batch)
static hipStream_t ctx_stream(svo_ctx* c) {
    if (c->pending_batch) {
        for (int i = 1; i < c->pending_chains; ++i) {
            const hipError_t e = hipStreamWaitEvent(c->stream_raw, c->joins[i], 0);
            if (e != hipSuccess) {  // (valid handles: not expected) fall back to a full wait so nothing overlaps
                (void)hipStreamSynchronize(c->sides[i]);
                (void)hipGetLastError();
            }
        }
        c->pending_batch = nullptr;
        c->pending_chains = 0;
    }
    return c->stream_raw;
}

// at least `bytes` of the context's scratch (the previous contents are not kept)
static hipError_t ctx_scratch(svo_ctx* c, size_t bytes, void** out) {
    if (bytes > c->scratch_bytes) {
        if (c->scratch) (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_bytes = 0;
        const size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes + bytes / 2;
        const hipError_t e = hipMalloc(&c->scratch, want);
        if (e != hipSuccess) return e;
        c->scratch_bytes = want;
    }
    *out = c->scratch;
    return hipSuccess;
}

// the context's pinned host staging (kPinnedCap bytes, allocated once on first use and never resized:
// measured on the MI355X boxes, copies into a pinned block allocated after a hipHostFree of the previous
// one failed with "invalid argument").  Calls whose payload exceeds it (or when pinning fails) stage in
// pageable memory or copy straight from the caller's arrays.
constexpr size_t kPinnedCap = (size_t)8 << 20;
static hipError_t ctx_pinned_alloc(svo_ctx* c) {
    if (c->pinned) return hipSuccess;
    hipError_t e = hipHostMalloc(&c->pinned, kPinnedCap, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&c->pinned_dev, c->pinned, 0);
    if (e != hipSuccess) {
        if (c->pinned) (void)hipHostFree(c->pinned);
        c->pinned = c->pinned_dev = nullptr;
        return e;
    }
    c->pinned_bytes = kPinnedCap;
    return hipSuccess;
}

static hipError_t ctx_ring_drain(svo_ctx* c) {
    if (!c->ring_pending) return hipSuccess;
    const hipError_t e = hipStreamSynchronize(ctx_stream(c));
    c->ring_pending = false;
    c->ring_off = 0;
    return e;
}

static hipError_t ctx_pinned(svo_ctx* c, size_t bytes, void** out) {
    if (bytes > kPinnedCap) return hipErrorInvalidValue;
    if (hipError_t e = ctx_ring_drain(c)) return e;
    if (hipError_t e = ctx_pinned_alloc(c)) return e;
    *out = c->pinned;
    return hipSuccess;
}

// Copies between the context's pinned block and device memory as a kernel that reads / writes the mapped
// pinned block itself, not on a copy engine.  Measured on MI355X (tools/dev/fa_latency.py, rocprofv3 memory-copy
// trace): once a process has run and freed a large alignment batch, every small SDMA transfer starts ~100 us
// after it is queued, so each synchronous call paid ~200 us for its two copies (config 3 FeatureAlignment
// 0.07 -> 0.28 ms per call, BENCH_r02 `secondary`).  A kernel copy is dispatched like the call's own kernel.
// Copies that do not touch the pinned block (pageable memory) stay hipMemcpyAsync.
namespace {
__global__ void pinned_copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t bytes) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)dst | (uintptr_t)src) & 7u) == 0) {
        const uint64_t n8 = bytes / 8;
        uint64_t* d = reinterpret_cast<uint64_t*>(dst);
        const uint64_t* q = reinterpret_cast<const uint64_t*>(src);
        for (uint64_t i = t; i < n8; i += nt) d[i] = q[i];
        for (uint64_t i = n8 * 8 + t; i < bytes; i += nt) dst[i] = src[i];
    } else {
        for (uint64_t i = t; i < bytes; i += nt) dst[i] = src[i];
    }
}
}  // namespace

static bool in_pinned(const svo_ctx* c, const void* p, size_t bytes) {
    const char* b = static_cast<const char*>(c->pinned);
    const char* q = static_cast<const char*>(p);
    return b && q >= b && q + bytes <= b + c->pinned_bytes;
}
static hipError_t stage_copy(svo_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    const bool h2d = kind == hipMemcpyHostToDevice;
    const void* host = h2d ? src : dst;
    if (!(kind == hipMemcpyHostToDevice || kind == hipMemcpyDeviceToHost) || !in_pinned(c, host, bytes))
        return hipMemcpyAsync(dst, src, bytes, kind, s);
    const ptrdiff_t off = static_cast<const char*>(host) - static_cast<const char*>(c->pinned);
    char* hd = static_cast<char*>(c->pinned_dev) + off;
    const uint64_t blocks = std::min<uint64_t>((bytes / 8 + 255) / 256 + 1, 1024);
    hipLaunchKernelGGL(pinned_copy_kernel, dim3((uint32_t)blocks), dim3(256), 0, s,
                       h2d ? static_cast<uint8_t*>(dst) : reinterpret_cast<uint8_t*>(hd),
                       h2d ? reinterpret_cast<const uint8_t*>(hd) : static_cast<const uint8_t*>(src), (uint64_t)bytes);
    return hipGetLastError();
}

struct svo_pyramid_set {
    svo_ctx* ctx;
    int32_t n_frames, width, height, levels;
    svo::LevelGeom geom;
    int64_t grad_off, stride;
    uint8_t* d_base;
    hipEvent_t ready = nullptr;  // svo_pyramid_set_build_async: recorded on the prep stream after the build
    bool pending = false;        // a build_async whose `ready` the context stream has not waited for yet
};

// the context stream waits for the set's last asynchronous build.  Every user of a set's planes on the context
// stream goes through this first: uploads, builds, downloads, the batches' set_pair / set_pairs and runs
// (join_pending), FeatureAlignment, the depth filter and feature detection / selection.
static void pending_remove(svo_ctx* c, const svo_pyramid_set* p) {
    auto& v = c->pending_sets;
    v.erase(std::remove(v.begin(), v.end(), p), v.end());
}
static hipError_t set_join(const svo_pyramid_set* cp) {
    svo_pyramid_set* p = const_cast<svo_pyramid_set*>(cp);
    if (!p || !p->pending) return hipSuccess;
    p->pending = false;
    pending_remove(p->ctx, p);
    hipError_t e = hipSetDevice(p->ctx->device);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx_stream(p->ctx), p->ready, 0);
    return e;
}
// the sets among `sets` that still have a pending asynchronous build (matched by address against the context's
// list, so a set destroyed since it was recorded is never touched)
static hipError_t join_pending(svo_ctx* c, const std::vector<const svo_pyramid_set*>& sets) {
    for (const svo_pyramid_set* q : sets) {
        if (std::find(c->pending_sets.begin(), c->pending_sets.end(), q) == c->pending_sets.end()) continue;
        const hipError_t e = set_join(q);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

struct svo_align_batch {
    svo_ctx* ctx;
    svo_camera cam;
    svo_align_params params;
    int32_t n_pairs, max_f, half, area;
    int64_t key_stride;
    uint16_t* d_keys;
    uint32_t* d_sel;      // median_mode 1: K2R scratch
    int64_t sel_stride;
    uint32_t* d_win;
    int64_t win_stride;
    uint32_t win_levels;
    svo::LevelGeom geom;
    std::vector<svo::PairDesc> h_pairs;
    std::vector<uint8_t> pair_set;
    svo::PairDesc* d_pairs;
    svo::PairState* d_state;
    double *d_px, *d_bearing, *d_point, *d_xw, *d_partials, *d_cproj, *d_scratch, *d_pose_out, *d_err;
    uint32_t* d_arrive;
    int32_t feat_iters, chunks;
    uint8_t *d_has_point, *d_fvis;
    int32_t* d_status;
    svo_level_trace* d_traces;
    bool ran;
    uint8_t* d_stage = nullptr;  // svo_align_batch_set_pairs: packed features + row offsets (grow-only)
    size_t stage_bytes = 0;
    // per pair the ref / lastKF / cur sets its planes come from (run joins their pending builds)
    std::vector<std::array<const svo_pyramid_set*, 3>> pair_sets;
};
// the distinct sets the batch's pairs read now
static std::vector<const svo_pyramid_set*> batch_sets(const svo_align_batch* b) {
    std::vector<const svo_pyramid_set*> v;
    for (const auto& t : b->pair_sets)
        for (const svo_pyramid_set* p : t)
            if (p && std::find(v.begin(), v.end(), p) == v.end()) v.push_back(p);
    return v;
}

extern "C" {

const char* svo_last_error(void) { return g_err.c_str(); }
int svo_abi_version(void) { return SVO_ABI_VERSION; }

int svo_device_count(int32_t* count) {
    if (!count) return fail(SVO_ERR_ARG, "count is null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SVO_OK;
}

int svo_ctx_create(int32_t device, svo_ctx** out) {
    if (!out) return fail(SVO_ERR_ARG, "out is null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(SVO_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(SVO_ERR_ARG, "device %d out of range [0,%d)", device, n);
    hipDeviceProp_t prop;
    SVO_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SVO_ERR_NODEV, "device %d is %s; this build targets gfx950 (MI355X)", device, prop.gcnArchName);
    SVO_HIP(hipSetDevice(device));
    svo_ctx* c = new (std::nothrow) svo_ctx{};
    if (!c) return fail(SVO_ERR_ARG, "out of host memory");
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream_raw, hipStreamNonBlocking);
    for (int i = 1; i < 4 && e == hipSuccess; ++i) e = hipStreamCreateWithFlags(&c->sides[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->prep, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->prep_gate, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->staged, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->stage_free, hipEventDisableTiming);
    for (int i = 1; i < 4 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->joins[i], hipEventDisableTiming);
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 2 + 3 * svo::kMaxLevels && e == hipSuccess; ++i)
            e = hipEventCreateWithFlags(&c->chain_marks[k][i], hipEventDisableTiming);
    for (int i = 0; i < 16 && e == hipSuccess; ++i) e = hipEventCreate(&c->events[i]);
    if (e != hipSuccess) {
        delete c;
        return fail(SVO_ERR_HIP, "hipStreamCreate/hipEventCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return SVO_OK;
}

int svo_ctx_destroy(svo_ctx* c) {
    if (!c) return SVO_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(ctx_stream(c));
    for (hipEvent_t ev : c->events)
        if (ev) (void)hipEventDestroy(ev);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->prep) (void)hipStreamSynchronize(c->prep);
    if (c->prep) (void)hipStreamDestroy(c->prep);
    if (c->prep_gate) (void)hipEventDestroy(c->prep_gate);
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->staged) (void)hipEventDestroy(c->staged);
    if (c->stage_free) (void)hipEventDestroy(c->stage_free);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    for (auto& row : c->chain_marks)
        for (hipEvent_t ev : row)
            if (ev) (void)hipEventDestroy(ev);
    for (int i = 1; i < 4; ++i) {
        if (c->joins[i]) (void)hipEventDestroy(c->joins[i]);
        if (c->sides[i]) (void)hipStreamDestroy(c->sides[i]);
    }
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->pinned) (void)hipHostFree(c->pinned);
    (void)hipStreamDestroy(c->stream_raw);
    delete c;
    return SVO_OK;
}

int svo_ctx_synchronize(svo_ctx* c) {
    if (!c) return fail(SVO_ERR_ARG, "ctx is null");
    SVO_HIP(hipSetDevice(c->device));
    SVO_HIP(hipStreamSynchronize(ctx_stream(c)));
    return SVO_OK;
}

void* svo_ctx_stream(svo_ctx* c) { return c ? (void*)ctx_stream(c) : nullptr; }

int svo_ctx_event_record(svo_ctx* c, int32_t slot) {
    if (!c || slot < 0 || slot >= 16) return fail(SVO_ERR_ARG, "bad context or event slot");
    SVO_HIP(hipSetDevice(c->device));
    SVO_HIP(hipEventRecord(c->events[slot], ctx_stream(c)));
    return SVO_OK;
}

int svo_ctx_event_elapsed(svo_ctx* c, int32_t a, int32_t b, float* ms) {
    if (!c || !ms || a < 0 || a >= 16 || b < 0 || b >= 16) return fail(SVO_ERR_ARG, "bad context or event slot");
    SVO_HIP(hipSetDevice(c->device));
    SVO_HIP(hipEventSynchronize(c->events[b]));
    SVO_HIP(hipEventElapsedTime(ms, c->events[a], c->events[b]));
    return SVO_OK;
}

// ------------------------------------------------------------------ pyramid sets
int svo_pyramid_set_create(svo_ctx* c, int32_t n_frames, int32_t width, int32_t height, int32_t levels,
                           svo_pyramid_set** out) {
    if (!c || !out) return fail(SVO_ERR_ARG, "null argument");
    *out = nullptr;
    if (n_frames <= 0 || width < 3 || height < 3 || levels < 1 || levels > svo::kMaxLevels)
        return fail(SVO_ERR_ARG, "bad pyramid geometry n=%d %dx%d levels=%d", n_frames, width, height, levels);
    if (width > 4096) return fail(SVO_ERR_ARG, "width %d > 4096 (the gradient kernel stages two rows per run)", width);
    SVO_HIP(hipSetDevice(c->device));
    svo_pyramid_set* p = new (std::nothrow) svo_pyramid_set{};
    if (!p) return fail(SVO_ERR_ARG, "out of host memory");
    p->ctx = c;
    p->n_frames = n_frames; p->width = width; p->height = height; p->levels = levels;
    p->geom = make_geom(width, height, levels);
    p->grad_off = (p->geom.frame_bytes + 255) / 256 * 256;
    p->stride = (p->grad_off + p->geom.frame_bytes + 255) / 256 * 256;
    // +64 B: 16-B aligned window-row loads may run up to 31 B past the last plane (zero-weight cells)
    hipError_t e = hipMalloc(&p->d_base, (size_t)p->stride * n_frames + 64);
    if (e != hipSuccess) {
        delete p;
        return fail(SVO_ERR_HIP, "hipMalloc(pyramids %lld B): %s", (long long)p->stride * n_frames, hipGetErrorString(e));
    }
    *out = p;
    return SVO_OK;
}

int svo_pyramid_set_destroy(svo_pyramid_set* p) {
    if (!p) return SVO_OK;
    (void)hipSetDevice(p->ctx->device);
    (void)hipStreamSynchronize(ctx_stream(p->ctx));
    if (p->ready) {
        (void)hipStreamSynchronize(p->ctx->prep);
        (void)hipEventDestroy(p->ready);
    }
    pending_remove(p->ctx, p);
    (void)hipFree(p->d_base);
    delete p;
    return SVO_OK;
}

static int upload_impl(svo_pyramid_set* p, int32_t first, int32_t count, const uint8_t* src, hipMemcpyKind kind) {
    if (!p || !src) return fail(SVO_ERR_ARG, "null argument");
    if (first < 0 || count < 0 || first + count > p->n_frames) return fail(SVO_ERR_ARG, "frames out of range");
    SVO_HIP(hipSetDevice(p->ctx->device));
    SVO_HIP(set_join(p));
    const size_t img = (size_t)p->width * p->height;
    SVO_HIP(hipMemcpy2DAsync(p->d_base + (size_t)first * p->stride, (size_t)p->stride, src, img, img, count, kind,
                             ctx_stream(p->ctx)));
    return SVO_OK;
}

int svo_pyramid_set_upload(svo_pyramid_set* p, int32_t first, int32_t count, const uint8_t* host_images) {
    return upload_impl(p, first, count, host_images, hipMemcpyHostToDevice);
}

int svo_pyramid_set_upload_device(svo_pyramid_set* p, int32_t first, int32_t count, const uint8_t* dev_images) {
    return upload_impl(p, first, count, dev_images, hipMemcpyDeviceToDevice);
}

int svo_pyramid_set_build(svo_pyramid_set* p, int32_t first, int32_t count) {
    if (!p) return fail(SVO_ERR_ARG, "null argument");
    if (first < 0 || count < 0 || first + count > p->n_frames) return fail(SVO_ERR_ARG, "frames out of range");
    if (count == 0) return SVO_OK;
    SVO_HIP(hipSetDevice(p->ctx->device));
    SVO_HIP(set_join(p));
    svo::launch_pyramid(p->d_base, p->geom, first, count, ctx_stream(p->ctx));
    SVO_HIP(hipGetLastError());
    return SVO_OK;
}

int svo_pyramid_set_build_async(svo_pyramid_set* p, int32_t first, int32_t count) {
    if (!p) return fail(SVO_ERR_ARG, "null argument");
    if (first < 0 || count < 0 || first + count > p->n_frames) return fail(SVO_ERR_ARG, "frames out of range");
    if (count == 0) return SVO_OK;
    svo_ctx* c = p->ctx;
    SVO_HIP(hipSetDevice(c->device));
    if (!p->ready) SVO_HIP(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
    // after everything the context stream holds now (the uploads of these frames, and the alignment that
    // last read the planes), and after an earlier asynchronous build of this set (the prep stream is in order)
    SVO_HIP(hipEventRecord(c->prep_gate, ctx_stream(c)));
    SVO_HIP(hipStreamWaitEvent(c->prep, c->prep_gate, 0));
    svo::launch_pyramid(p->d_base, p->geom, first, count, c->prep);
    SVO_HIP(hipGetLastError());
    SVO_HIP(hipEventRecord(p->ready, c->prep));
    p->pending = true;
    if (std::find(c->pending_sets.begin(), c->pending_sets.end(), p) == c->pending_sets.end()) c->pending_sets.push_back(p);
    return SVO_OK;
}

int svo_pyramid_set_download(const svo_pyramid_set* p, int32_t frame, int32_t level, int32_t gradient, uint8_t* out) {
    if (!p || !out) return fail(SVO_ERR_ARG, "null argument");
    if (frame < 0 || frame >= p->n_frames || level < 0 || level >= p->levels) return fail(SVO_ERR_ARG, "index out of range");
    SVO_HIP(hipSetDevice(p->ctx->device));
    SVO_HIP(set_join(p));
    const uint8_t* src = p->d_base + (size_t)frame * p->stride + (gradient ? p->grad_off : 0) + p->geom.off[level];
    SVO_HIP(hipMemcpyAsync(out, src, (size_t)p->geom.w[level] * p->geom.h[level], hipMemcpyDeviceToHost, ctx_stream(p->ctx)));
    SVO_HIP(hipStreamSynchronize(ctx_stream(p->ctx)));
    return SVO_OK;
}

int svo_pyramid_level_size(const svo_pyramid_set* p, int32_t level, int32_t* w, int32_t* h) {
    if (!p || !w || !h) return fail(SVO_ERR_ARG, "null argument");
    if (level < 0 || level >= p->levels) { *w = 0; *h = 0; return SVO_OK; }
    *w = p->geom.w[level];
    *h = p->geom.h[level];
    return SVO_OK;
}

// ------------------------------------------------------------------ image alignment batches
static void free_batch(svo_align_batch* b) {
    void* ptrs[] = {b->d_pairs, b->d_px, b->d_bearing, b->d_point, b->d_has_point, b->d_xw, b->d_keys, b->d_sel,
                    b->d_state, b->d_partials, b->d_arrive, b->d_fvis, b->d_cproj, b->d_scratch, b->d_pose_out, b->d_err, b->d_status, b->d_traces,
                    b->d_win, b->d_stage};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
}

int svo_align_batch_create(svo_ctx* c, const svo_camera* cam, const svo_align_params* prm, int32_t n_pairs,
                           int32_t max_features, svo_align_batch** out) {
    if (!c || !cam || !prm || !out) return fail(SVO_ERR_ARG, "null argument");
    *out = nullptr;
    if (n_pairs <= 0 || max_features <= 0) return fail(SVO_ERR_ARG, "n_pairs and max_features must be > 0");
    if (prm->patch_size < 1 || prm->patch_size / 2 > svo::align_max_half())
        return fail(SVO_ERR_ARG, "patch_size %d unsupported (<= 19)", prm->patch_size);
    if (prm->min_level < 0 || prm->max_level < prm->min_level || prm->max_level >= svo::kMaxLevels)
        return fail(SVO_ERR_ARG, "bad level range [%d,%d]", prm->min_level, prm->max_level);
    if (prm->median_mode != SVO_MEDIAN_EXACT && prm->median_mode != SVO_MEDIAN_REFERENCE)
        return fail(SVO_ERR_ARG, "median_mode %d unknown (0 = exact order statistics, 1 = the reference's nth_element)",
                    prm->median_mode);
    const int half = prm->patch_size / 2, area = (2 * half + 1) * (2 * half + 1);
    if ((int64_t)max_features * area >= (1ll << 31)) return fail(SVO_ERR_ARG, "max_features too large");
    if (prm->median_mode == SVO_MEDIAN_REFERENCE && (int64_t)max_features * area > SVO_REF_MAX_SLOTS)
        return fail(SVO_ERR_ARG, "median_mode 1 supports up to %d residual slots per pair (max_features * patch^2)",
                    SVO_REF_MAX_SLOTS);
    SVO_HIP(hipSetDevice(c->device));
    svo_align_batch* b = new (std::nothrow) svo_align_batch{};
    if (!b) return fail(SVO_ERR_ARG, "out of host memory");
    b->ctx = c; b->cam = *cam; b->params = *prm; b->n_pairs = n_pairs; b->max_f = max_features;
    b->half = half; b->area = area;
    b->geom = make_geom(cam->width, cam->height, prm->max_level + 1);
    b->h_pairs.assign(n_pairs, svo::PairDesc{});
    b->pair_set.assign(n_pairs, 0);
    b->pair_sets.assign(n_pairs, {nullptr, nullptr, nullptr});
    const size_t F = (size_t)n_pairs * max_features;
    hipError_t e = hipSuccess;
#define ALLOC(ptr, bytes) if (e == hipSuccess) e = hipMalloc(&ptr, bytes)
    ALLOC(b->d_pairs, sizeof(svo::PairDesc) * n_pairs);
    ALLOC(b->d_px, F * 2 * sizeof(double));
    ALLOC(b->d_bearing, F * 3 * sizeof(double));
    ALLOC(b->d_point, F * 3 * sizeof(double));
    ALLOC(b->d_has_point, F);
    ALLOC(b->d_xw, F * 3 * sizeof(double));
    ALLOC(b->d_state, sizeof(svo::PairState) * n_pairs);
    {
        b->feat_iters = svo::align_feat_iters();
        b->chunks = svo::align_chunks(max_features, half, b->feat_iters);
    }
    ALLOC(b->d_partials, (size_t)n_pairs * b->chunks * 28 * sizeof(double));
    ALLOC(b->d_arrive, (size_t)n_pairs * sizeof(uint32_t));
    ALLOC(b->d_fvis, F);
    const int64_t slots = (int64_t)area * ((max_features + 63) / 64 * 64);  // pixel-major slots, see AlignArgs
    b->key_stride = slots;
    ALLOC(b->d_cproj, F * 2 * sizeof(double));
    if (prm->median_mode == SVO_MEDIAN_REFERENCE) {
        // K2R: K1's exact residuals in the reference's feature-major slot order, and the selection scratch
        b->sel_stride = svo::ref_sel_stride((int64_t)max_features * area);
        ALLOC(b->d_scratch, (size_t)n_pairs * b->key_stride * sizeof(double));
        ALLOC(b->d_sel, (size_t)n_pairs * b->sel_stride * sizeof(uint32_t));
    } else {
        ALLOC(b->d_scratch, (size_t)n_pairs * b->key_stride * sizeof(double));
        ALLOC(b->d_keys, (size_t)n_pairs * b->key_stride * sizeof(uint16_t));
    }
    // window levels: where K3 re-gathering the level's planes would cost more than K1 handing over the
    // windows (3 planes' bytes >= 4x the windows written + read); SVO_WIN_LEVELS (a level bitmask)
    // overrides, for measurements
    {
        const int64_t wdw = svo::align_win_dwords(half), fpad = (max_features + 63) / 64 * 64;
        b->win_stride = wdw * fpad;
        b->win_levels = 0;
        for (int l = prm->min_level; l <= prm->max_level; ++l)
            if (3ll * b->geom.w[l] * b->geom.h[l] >= 4ll * 4 * wdw * max_features) b->win_levels |= 1u << l;
        if (const char* ov = getenv("SVO_WIN_LEVELS")) b->win_levels = (uint32_t)strtoul(ov, nullptr, 0);
        if (b->win_levels) ALLOC(b->d_win, (size_t)n_pairs * b->win_stride * sizeof(uint32_t));
    }
    ALLOC(b->d_pose_out, (size_t)n_pairs * 7 * sizeof(double));
    ALLOC(b->d_err, (size_t)n_pairs * sizeof(double));
    ALLOC(b->d_status, (size_t)n_pairs * sizeof(int32_t));
    ALLOC(b->d_traces, (size_t)n_pairs * (prm->max_level + 1) * sizeof(svo_level_trace));
#undef ALLOC
    if (e != hipSuccess) {
        free_batch(b);
        delete b;
        return fail(SVO_ERR_HIP, "hipMalloc(align batch): %s", hipGetErrorString(e));
    }
    *out = b;
    return SVO_OK;
}

int svo_align_batch_destroy(svo_align_batch* b) {
    if (!b) return SVO_OK;
    (void)hipSetDevice(b->ctx->device);
    (void)hipStreamSynchronize(ctx_stream(b->ctx));
    free_batch(b);
    delete b;
    return SVO_OK;
}

static int check_frame(const svo_align_batch* b, const svo_pyramid_set* pyr, int32_t f) {
    if (!pyr) return fail(SVO_ERR_ARG, "null pyramid set");
    if (pyr->ctx != b->ctx) return fail(SVO_ERR_ARG, "pyramid set belongs to another context");
    if (pyr->width != b->cam.width || pyr->height != b->cam.height || pyr->levels < b->params.max_level + 1)
        return fail(SVO_ERR_ARG, "pyramid geometry %dx%d/%d does not match camera %dx%d / max_level %d", pyr->width,
                    pyr->height, pyr->levels, b->cam.width, b->cam.height, b->params.max_level);
    if (f < 0 || f >= pyr->n_frames) return fail(SVO_ERR_ARG, "frame index %d out of range", f);
    return SVO_OK;
}

int svo_align_batch_set_pair(svo_align_batch* b, int32_t pair, const svo_pyramid_set* ref_set, int32_t ref_frame,
                             const svo_pyramid_set* kf_set, int32_t kf_frame, const svo_pyramid_set* cur_set,
                             int32_t cur_frame, const double* ref_pose, const double* kf_pose,
                             const double* cur_pose, int32_t n_ref, int32_t n_kf, const double* px,
                             const double* bearing, const double* point, const uint8_t* has_point) {
    if (!b || !ref_pose || !kf_pose || !cur_pose) return fail(SVO_ERR_ARG, "null argument");
    if (pair < 0 || pair >= b->n_pairs) return fail(SVO_ERR_ARG, "pair %d out of range", pair);
    if (n_ref < 0 || n_kf < 0 || n_ref + n_kf > b->max_f)
        return fail(SVO_ERR_ARG, "n_ref+n_kf = %d exceeds max_features %d", n_ref + n_kf, b->max_f);
    const int32_t nf = n_ref + n_kf;
    if (nf > 0 && (!px || !bearing || !point || !has_point)) return fail(SVO_ERR_ARG, "null feature array");
    int rc;
    if ((rc = check_frame(b, ref_set, ref_frame)) != SVO_OK) return rc;
    if ((rc = check_frame(b, kf_set, kf_frame)) != SVO_OK) return rc;
    if ((rc = check_frame(b, cur_set, cur_frame)) != SVO_OK) return rc;
    SVO_HIP(hipSetDevice(b->ctx->device));
    SVO_HIP(set_join(ref_set));
    SVO_HIP(set_join(kf_set));
    SVO_HIP(set_join(cur_set));
    b->pair_sets[pair] = {ref_set, kf_set, cur_set};
    svo::PairDesc& d = b->h_pairs[pair];
    d.ref_pyr = ref_set->d_base + (size_t)ref_frame * ref_set->stride;
    d.kf_pyr = kf_set->d_base + (size_t)kf_frame * kf_set->stride;
    d.cur_pyr = cur_set->d_base + (size_t)cur_frame * cur_set->stride;
    std::memcpy(d.ref_pose, ref_pose, 7 * sizeof(double));
    std::memcpy(d.kf_pose, kf_pose, 7 * sizeof(double));
    std::memcpy(d.cur_pose, cur_pose, 7 * sizeof(double));
    d.n_ref = n_ref;
    d.n_kf = n_kf;
    const size_t fo = (size_t)pair * b->max_f;
    svo_ctx* c = b->ctx;
    hipStream_t s = ctx_stream(c);
    // stage the pair's arrays in the context's pinned ring and return without waiting: the copies are
    // ordered before any later work on the stream, and the ring drains when it wraps or another call
    // needs the pinned block (large pairs, or no pinned memory: direct copies and a wait, as before)
    auto r8 = [](size_t v) { return (v + 7) / 8 * 8; };
    const size_t n = (size_t)nf;
    const size_t need = r8(sizeof(d)) + n * 16 + n * 24 * 2 + r8(n);
    if (need <= kPinnedCap && ctx_pinned_alloc(c) == hipSuccess) {
        if (c->ring_off + need > kPinnedCap) SVO_HIP(ctx_ring_drain(c));
        char* h = static_cast<char*>(c->pinned) + c->ring_off;
        // claim the slice before enqueueing: if an enqueue fails part way, copies already queued may still
        // read it, so the ring stays pending (the next pinned user drains it) and the slice is not reused
        c->ring_off += need;
        c->ring_pending = true;
        std::memcpy(h, &d, sizeof(d));
        char* hp = h + r8(sizeof(d));
        if (nf > 0) {
            std::memcpy(hp, px, n * 16);
            std::memcpy(hp + n * 16, bearing, n * 24);
            std::memcpy(hp + n * 40, point, n * 24);
            std::memcpy(hp + n * 64, has_point, n);
            SVO_HIP(stage_copy(c, b->d_px + 2 * fo, hp, n * 16, hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_bearing + 3 * fo, hp + n * 16, n * 24, hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_point + 3 * fo, hp + n * 40, n * 24, hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_has_point + fo, hp + n * 64, n, hipMemcpyHostToDevice, s));
        }
        SVO_HIP(stage_copy(c, b->d_pairs + pair, h, sizeof(d), hipMemcpyHostToDevice, s));
    } else {
        (void)hipGetLastError();
        SVO_HIP(ctx_ring_drain(c));
        if (nf > 0) {
            SVO_HIP(stage_copy(c, b->d_px + 2 * fo, px, nf * 2 * sizeof(double), hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_bearing + 3 * fo, bearing, nf * 3 * sizeof(double), hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_point + 3 * fo, point, nf * 3 * sizeof(double), hipMemcpyHostToDevice, s));
            SVO_HIP(stage_copy(c, b->d_has_point + fo, has_point, nf, hipMemcpyHostToDevice, s));
        }
        SVO_HIP(stage_copy(c, b->d_pairs + pair, &d, sizeof(d), hipMemcpyHostToDevice, s));
        SVO_HIP(hipStreamSynchronize(s));
    }
    b->pair_set[pair] = 1;
    return SVO_OK;
}

}  // extern "C"

namespace {
// svo_align_batch_set_pairs: pair i's packed rows [off[i], off[i+1]) to its slots from (first + i) * max_f.
// One workgroup per pair; each array is copied as a flat run of its elements (coalesced both sides).
__global__ void scatter_features_kernel(const int64_t* __restrict__ off, const double* __restrict__ px,
                                        const double* __restrict__ bearing, const double* __restrict__ point,
                                        const uint8_t* __restrict__ has_point, double* __restrict__ dpx,
                                        double* __restrict__ dbearing, double* __restrict__ dpoint,
                                        uint8_t* __restrict__ dhas, int32_t first, int32_t max_f) {
    const int64_t o = off[blockIdx.x], n = off[blockIdx.x + 1] - o;
    const int64_t d = (int64_t)(first + (int32_t)blockIdx.x) * max_f;
    for (int64_t e = threadIdx.x; e < 2 * n; e += blockDim.x) dpx[2 * d + e] = px[2 * o + e];
    for (int64_t e = threadIdx.x; e < 3 * n; e += blockDim.x) dbearing[3 * d + e] = bearing[3 * o + e];
    for (int64_t e = threadIdx.x; e < 3 * n; e += blockDim.x) dpoint[3 * d + e] = point[3 * o + e];
    for (int64_t e = threadIdx.x; e < n; e += blockDim.x) dhas[d + e] = has_point[o + e];
}
}  // namespace

extern "C" {

int svo_align_batch_set_pairs(svo_align_batch* b, int32_t first, int32_t count, const svo_pyramid_set* ref_set,
                              const svo_pyramid_set* kf_set, const svo_pyramid_set* cur_set, const int32_t* frames,
                              const double* poses, const int32_t* n_feat, const double* px, const double* bearing,
                              const double* point, const uint8_t* has_point, int32_t features_on_device) {
    if (!b || !frames || !poses || !n_feat) return fail(SVO_ERR_ARG, "null argument");
    if (first < 0 || count < 0 || (int64_t)first + count > b->n_pairs)
        return fail(SVO_ERR_ARG, "pairs [%d, %d) out of range (n_pairs %d)", first, first + count, b->n_pairs);
    if (count == 0) return SVO_OK;
    std::vector<int64_t> off((size_t)count + 1, 0);
    int rc;
    for (int32_t i = 0; i < count; ++i) {
        const int32_t n_ref = n_feat[2 * i], n_kf = n_feat[2 * i + 1];
        if (n_ref < 0 || n_kf < 0 || n_ref + n_kf > b->max_f)
            return fail(SVO_ERR_ARG, "pair %d: n_ref+n_kf = %d exceeds max_features %d", first + i, n_ref + n_kf, b->max_f);
        if ((rc = check_frame(b, ref_set, frames[3 * i])) != SVO_OK) return rc;
        if ((rc = check_frame(b, kf_set, frames[3 * i + 1])) != SVO_OK) return rc;
        if ((rc = check_frame(b, cur_set, frames[3 * i + 2])) != SVO_OK) return rc;
        off[i + 1] = off[i] + n_ref + n_kf;
    }
    const int64_t T = off[count];
    if (T > 0 && (!px || !bearing || !point || !has_point)) return fail(SVO_ERR_ARG, "null feature array");
    SVO_HIP(hipSetDevice(b->ctx->device));
    SVO_HIP(set_join(ref_set));
    SVO_HIP(set_join(kf_set));
    SVO_HIP(set_join(cur_set));
    for (int32_t i = 0; i < count; ++i) b->pair_sets[first + i] = {ref_set, kf_set, cur_set};
    for (int32_t i = 0; i < count; ++i) {
        svo::PairDesc& d = b->h_pairs[first + i];
        d.ref_pyr = ref_set->d_base + (size_t)frames[3 * i] * ref_set->stride;
        d.kf_pyr = kf_set->d_base + (size_t)frames[3 * i + 1] * kf_set->stride;
        d.cur_pyr = cur_set->d_base + (size_t)frames[3 * i + 2] * cur_set->stride;
        std::memcpy(d.ref_pose, poses + 21 * i, 7 * sizeof(double));
        std::memcpy(d.kf_pose, poses + 21 * i + 7, 7 * sizeof(double));
        std::memcpy(d.cur_pose, poses + 21 * i + 14, 7 * sizeof(double));
        d.n_ref = n_feat[2 * i];
        d.n_kf = n_feat[2 * i + 1];
    }
    // device staging: the row offsets, the pair descriptors, then (host features) the packed arrays
    const size_t off_bytes = ((size_t)(count + 1) * sizeof(int64_t) + 255) / 256 * 256;
    const size_t desc_bytes = (sizeof(svo::PairDesc) * count + 255) / 256 * 256;
    const size_t host_bytes = features_on_device ? 0 : (size_t)T * 65 + 4 * 256;
    const size_t need = off_bytes + desc_bytes + host_bytes;
    if (need > b->stage_bytes) {
        if (b->d_stage) {  // a scatter queued on the stream, or an upload left on the copy stream by an
                           // earlier call's error exit, may still touch the old block
            SVO_HIP(hipStreamSynchronize(b->ctx->copy));
            SVO_HIP(hipStreamSynchronize(ctx_stream(b->ctx)));
            SVO_HIP(hipFree(b->d_stage));
        }
        b->d_stage = nullptr;
        b->stage_bytes = 0;
        SVO_HIP(hipMalloc(&b->d_stage, need + need / 4));
        b->stage_bytes = need + need / 4;
    }
    svo_ctx* c = b->ctx;
    hipStream_t s = ctx_stream(c), cs = c->copy;
    SVO_HIP(ctx_ring_drain(c));  // set_pair copies still reading the ring go first (stream order anyway)
    // the upload runs on the copy stream, behind only the previous scatter out of staging (not behind
    // whatever else `stream` holds, e.g. the pyramid build these pairs read); `stream` then waits for it
    SVO_HIP(hipStreamWaitEvent(cs, c->stage_free, 0));
    int64_t* d_off = reinterpret_cast<int64_t*>(b->d_stage);
    svo::PairDesc* d_desc = reinterpret_cast<svo::PairDesc*>(b->d_stage + off_bytes);
    SVO_HIP(hipMemcpyAsync(d_off, off.data(), (size_t)(count + 1) * sizeof(int64_t), hipMemcpyHostToDevice, cs));
    SVO_HIP(hipMemcpyAsync(d_desc, b->h_pairs.data() + first, sizeof(svo::PairDesc) * count, hipMemcpyHostToDevice,
                           cs));
    const double *spx = px, *sbr = bearing, *spt = point;
    const uint8_t* shp = has_point;
    if (!features_on_device && T > 0) {
        auto r256 = [](size_t v) { return (v + 255) / 256 * 256; };
        uint8_t* p = b->d_stage + off_bytes + desc_bytes;
        double* dpx = reinterpret_cast<double*>(p);
        double* dbr = reinterpret_cast<double*>(p + r256((size_t)T * 16));
        double* dpt = reinterpret_cast<double*>(p + r256((size_t)T * 16) + r256((size_t)T * 24));
        uint8_t* dhp = p + r256((size_t)T * 16) + 2 * r256((size_t)T * 24);
        SVO_HIP(hipMemcpyAsync(dpx, px, (size_t)T * 16, hipMemcpyHostToDevice, cs));
        SVO_HIP(hipMemcpyAsync(dbr, bearing, (size_t)T * 24, hipMemcpyHostToDevice, cs));
        SVO_HIP(hipMemcpyAsync(dpt, point, (size_t)T * 24, hipMemcpyHostToDevice, cs));
        SVO_HIP(hipMemcpyAsync(dhp, has_point, (size_t)T, hipMemcpyHostToDevice, cs));
        spx = dpx; sbr = dbr; spt = dpt; shp = dhp;
    }
    SVO_HIP(hipEventRecord(c->staged, cs));
    SVO_HIP(hipStreamWaitEvent(s, c->staged, 0));
    SVO_HIP(hipMemcpyAsync(b->d_pairs + first, d_desc, sizeof(svo::PairDesc) * count, hipMemcpyDeviceToDevice, s));
    if (T > 0)
        hipLaunchKernelGGL(scatter_features_kernel, dim3(count), dim3(256), 0, s, d_off, spx, sbr, spt, shp, b->d_px,
                           b->d_bearing, b->d_point, b->d_has_point, first, b->max_f);
    SVO_HIP(hipGetLastError());
    SVO_HIP(hipEventRecord(c->stage_free, s));
    // the offsets, descriptors and (host) features are read from memory the caller and this call own:
    // wait for the upload only; the scatter stays queued on `stream` behind earlier work (device features:
    // the caller's arrays are read by the scatter itself, so wait for it too)
    SVO_HIP(hipStreamSynchronize(cs));
    if (features_on_device && T > 0) SVO_HIP(hipStreamSynchronize(s));
    for (int32_t i = 0; i < count; ++i) b->pair_set[first + i] = 1;
    return SVO_OK;
}

int svo_align_batch_set_initial_poses(svo_align_batch* b, const double* poses) {
    if (!b || !poses) return fail(SVO_ERR_ARG, "null argument");
    SVO_HIP(hipSetDevice(b->ctx->device));
    for (int32_t i = 0; i < b->n_pairs; ++i) std::memcpy(b->h_pairs[i].cur_pose, poses + 7 * i, 7 * sizeof(double));
    SVO_HIP(hipMemcpyAsync(b->d_pairs, b->h_pairs.data(), sizeof(svo::PairDesc) * b->n_pairs, hipMemcpyHostToDevice,
                           ctx_stream(b->ctx)));
    SVO_HIP(hipStreamSynchronize(ctx_stream(b->ctx)));
    return SVO_OK;
}

// the largest residual vector (n_ref + n_kf) * patch area among pairs [p0, p0 + n): the reference-mode robust
// scale kernel is chosen per launch by the vectors the pairs actually hold (src/image_alignment.cpp:30-38 sizes
// the vector per frame), not by the batch's capacity
static int32_t batch_max_slots(const svo_align_batch* b, int32_t p0, int32_t n) {
    int32_t m = 0;
    for (int32_t i = p0; i < p0 + n; ++i) m = std::max(m, b->h_pairs[i].n_ref + b->h_pairs[i].n_kf);
    return m * b->area;
}

// Pairs [p0, p0 + n) of a batch as a batch of their own (every per-pair array offset by p0).
static svo::AlignArgs sub_batch(const svo::AlignArgs& a, const svo_align_batch* b, int32_t p0, int32_t n) {
    svo::AlignArgs s = a;
    const int64_t F = (int64_t)p0 * b->max_f;
    s.pairs += p0; s.state += p0;
    s.px += 2 * F; s.bearing += 3 * F; s.point += 3 * F; s.has_point += F; s.xw += 3 * F; s.fvis += F;
    s.cproj += 2 * F;
    s.partials += (int64_t)p0 * b->chunks * 28; s.arrive += p0;
    if (s.keys) s.keys += (int64_t)p0 * b->key_stride;
    if (s.scratch) s.scratch += (int64_t)p0 * b->key_stride;
    if (s.sel) s.sel += (int64_t)p0 * b->sel_stride;
    if (s.win) s.win += (int64_t)p0 * b->win_stride;
    s.pose_out += 7 * (int64_t)p0; s.err_out += p0; s.status_out += p0;
    s.traces += (int64_t)p0 * (b->params.max_level + 1);
    s.n_pairs = n;
    s.pair_base = a.pair_base + p0;
    s.max_slots = batch_max_slots(b, p0, n);
    return s;
}

static int run_batch(svo_align_batch* b, hipEvent_t* marks) {
    if (!b) return fail(SVO_ERR_ARG, "null argument");
    for (int32_t i = 0; i < b->n_pairs; ++i)
        if (!b->pair_set[i]) return fail(SVO_ERR_STATE, "pair %d was never set", i);
    SVO_HIP(hipSetDevice(b->ctx->device));
    // a set the pairs read may have been rebuilt asynchronously since set_pair(s) (build_async after the hand-over)
    SVO_HIP(join_pending(b->ctx, batch_sets(b)));
    svo::AlignArgs a;
    a.pairs = b->d_pairs;
    a.px = b->d_px; a.bearing = b->d_bearing; a.point = b->d_point; a.has_point = b->d_has_point;
    a.xw = b->d_xw; a.keys = b->d_keys; a.key_stride = b->key_stride; a.state = b->d_state; a.partials = b->d_partials;
    a.sel = b->d_sel; a.sel_stride = b->sel_stride; a.median_mode = b->params.median_mode;
    a.arrive = b->d_arrive;
    a.win = b->d_win; a.win_stride = b->win_stride; a.win_levels = b->win_levels;
    a.feat_iters = b->feat_iters; a.chunks = b->chunks; a.fvis = b->d_fvis; a.cproj = b->d_cproj; a.scratch = b->d_scratch;
    a.pose_out = b->d_pose_out; a.err_out = b->d_err; a.status_out = b->d_status; a.traces = b->d_traces;
    a.n_pairs = b->n_pairs; a.pair_base = 0; a.max_f = b->max_f; a.half = b->half; a.area = b->area;
    a.max_slots = batch_max_slots(b, 0, b->n_pairs);
    a.min_level = b->params.min_level; a.max_level = b->params.max_level;
    a.fx = b->cam.fx; a.fy = b->cam.fy; a.cx = b->cam.cx; a.cy = b->cam.cy;
    a.geom = b->geom;
    svo_ctx* c = b->ctx;
    // SVO_CHAINS=1 (measurement knob, read once): the whole batch as one chain
    static const bool one_chain = getenv("SVO_CHAINS") && atoi(getenv("SVO_CHAINS")) == 1;
    if (marks || b->n_pairs < kSplitMin || one_chain) {
        svo::launch_align(a, ctx_stream(c), marks);
    } else {
        // two independent half-batch chains on two streams: one chain's latency-bound stages (the
        // per-pair robust scale) overlap the other chain's feature stages.  Results are per pair and
        // independent of the split.
        static const int env_chains = getenv("SVO_CHAINS") ? atoi(getenv("SVO_CHAINS")) : 0;  // (measurement knobs,
        static const int env_stagger = getenv("SVO_STAGGER") ? atoi(getenv("SVO_STAGGER")) : -1;  //  read once)
        const bool k2v = svo::scale_impl() != SVO_SCALE_K2R && (int64_t)a.max_slots <= svo::refv_max_slots();
        const bool refv = b->params.median_mode == SVO_MEDIAN_REFERENCE && k2v;
        const int ns = env_chains ? std::max(2, std::min(4, env_chains))
                                  : (refv && b->n_pairs >= kSplitsRefvMin ? kSplitsRefv : kSplits);
        const int32_t per = (b->n_pairs / ns + 7) / 8 * 8;
        // Reference semantics with K2R: chain 1 starts when chain 0's first K1 is done (launch mark 2), so that
        // each chain's K1 / K3 run under the other chain's K2R instead of both chains meeting in K1 / K3 at every
        // level (MI355X, 512 pairs: 88.4k vs 78.4k pairs/s; marks 3 / 4 / 7: 79k / 74k / 67k).  The exact mode
        // runs unstaggered (round 1: staggering by 1-3 kernels cost 1-6 %).  SVO_STAGGER=k overrides.
        // K2V (the default reference-mode kernel whenever the vector fits its registers) fills whole CUs, so
        // the other chain's K1 / K3 run only between its launches whatever the stagger: unstaggered measured
        // best (MI355X, 512 pairs: stagger 0 / 1 / 2 / 3 = 119.1k / 118.4k / 117.3k / 117.4k pairs/s).
        const int stagger = env_stagger >= 0 ? env_stagger
                                             : (b->params.median_mode == SVO_MEDIAN_REFERENCE && !k2v ? 2 : 0);
        if (stagger < 0 || stagger > 1 + 3 * (b->params.max_level - b->params.min_level + 1))
            return fail(SVO_ERR_ARG, "SVO_STAGGER=%d outside the chain's launch marks", stagger);
        // Chains join the context stream lazily (svo_ctx::pending_batch): a run that follows a run of this same batch
        // and split, with nothing else queued in between, lets chain i follow its own previous run on its own stream
        // (chain i reads and writes only its own pairs) instead of forking after every chain of that run.
        static const bool defer = !getenv("SVO_DEFER_JOIN") || atoi(getenv("SVO_DEFER_JOIN")) != 0;  // (read once)
        const bool lazy = defer && stagger == 0;
        const bool cont = lazy && c->pending_batch == b && c->pending_chains == ns;
        hipStream_t s0 = cont ? c->stream_raw : ctx_stream(c);  // (ctx_stream joins any other pending chains)
        if (!cont) {
            SVO_HIP(hipEventRecord(c->fork, s0));
            for (int i = 1; i < ns; ++i) SVO_HIP(hipStreamWaitEvent(c->sides[i], c->fork, 0));
        }
        for (int i = 0; i < ns; ++i) {
            const int32_t p0 = i * per, cnt = i == ns - 1 ? b->n_pairs - p0 : std::min(per, b->n_pairs - p0);
            if (cnt <= 0) break;  // (later chains would be empty too)
            if (i >= 1 && stagger > 0) SVO_HIP(hipStreamWaitEvent(c->sides[i], c->chain_marks[i - 1][stagger], 0));
            svo::launch_align(sub_batch(a, b, p0, cnt), i == 0 ? s0 : c->sides[i],
                              i < ns - 1 && stagger > 0 ? c->chain_marks[i] : nullptr);
        }
        for (int i = 1; i < ns; ++i) SVO_HIP(hipEventRecord(c->joins[i], c->sides[i]));
        if (lazy) {
            c->pending_batch = b;  // joined by the next ctx_stream()
            c->pending_chains = ns;
        } else {
            for (int i = 1; i < ns; ++i) SVO_HIP(hipStreamWaitEvent(s0, c->joins[i], 0));
        }
    }
    SVO_HIP(hipGetLastError());
    b->ran = true;
    return SVO_OK;
}

int svo_align_batch_run(svo_align_batch* b) { return run_batch(b, nullptr); }

int svo_align_batch_profile(svo_align_batch* b, float* stage_ms) {
    if (!b || !stage_ms) return fail(SVO_ERR_ARG, "null argument");
    SVO_HIP(hipSetDevice(b->ctx->device));
    const int levels = b->params.max_level - b->params.min_level + 1;
    const int n = 2 + 3 * levels;
    std::vector<hipEvent_t> ev(n, nullptr);
    int rc = SVO_OK;
    for (int i = 0; i < n && rc == SVO_OK; ++i)
        if (hipEventCreate(&ev[i]) != hipSuccess) rc = fail(SVO_ERR_HIP, "hipEventCreate failed");
    if (rc == SVO_OK) rc = run_batch(b, ev.data());
    if (rc == SVO_OK && hipEventSynchronize(ev[n - 1]) != hipSuccess) rc = fail(SVO_ERR_HIP, "hipEventSynchronize failed");
    if (rc == SVO_OK) {
        for (int k = 0; k < 5; ++k) stage_ms[k] = 0.0f;
        for (int i = 0; i + 1 < n; ++i) {
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, ev[i], ev[i + 1]) != hipSuccess) { rc = fail(SVO_ERR_HIP, "hipEventElapsedTime failed"); break; }
            stage_ms[i == 0 ? 0 : 1 + (i - 1) % 3] += ms;  // [4] stays 0: the LM step runs inside K3
        }
    }
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

int svo_align_batch_results(svo_align_batch* b, double* poses, double* err, int32_t* status) {
    if (!b) return fail(SVO_ERR_ARG, "null argument");
    if (!b->ran) return fail(SVO_ERR_STATE, "batch has not been run");
    SVO_HIP(hipSetDevice(b->ctx->device));
    svo_ctx* c = b->ctx;
    hipStream_t s = ctx_stream(c);
    const size_t np = (size_t)b->n_pairs, bp = np * 7 * sizeof(double), be = np * sizeof(double), bs = np * sizeof(int32_t);
    void* host = nullptr;
    if (ctx_pinned(c, bp + be + bs, &host) == hipSuccess) {  // through the pinned block: kernel copies (stage_copy)
        char* h = static_cast<char*>(host);
        if (poses) SVO_HIP(stage_copy(c, h, b->d_pose_out, bp, hipMemcpyDeviceToHost, s));
        if (err) SVO_HIP(stage_copy(c, h + bp, b->d_err, be, hipMemcpyDeviceToHost, s));
        if (status) SVO_HIP(stage_copy(c, h + bp + be, b->d_status, bs, hipMemcpyDeviceToHost, s));
        SVO_HIP(hipStreamSynchronize(s));
        if (poses) std::memcpy(poses, h, bp);
        if (err) std::memcpy(err, h + bp, be);
        if (status) std::memcpy(status, h + bp + be, bs);
        return SVO_OK;
    }
    (void)hipGetLastError();
    if (poses) SVO_HIP(hipMemcpyAsync(poses, b->d_pose_out, bp, hipMemcpyDeviceToHost, s));
    if (err) SVO_HIP(hipMemcpyAsync(err, b->d_err, be, hipMemcpyDeviceToHost, s));
    if (status) SVO_HIP(hipMemcpyAsync(status, b->d_status, bs, hipMemcpyDeviceToHost, s));
    SVO_HIP(hipStreamSynchronize(s));
    return SVO_OK;
}

int svo_align_batch_traces(svo_align_batch* b, int32_t pair, svo_level_trace* out) {
    if (!b || !out) return fail(SVO_ERR_ARG, "null argument");
    if (!b->ran) return fail(SVO_ERR_STATE, "batch has not been run");
    if (pair < 0 || pair >= b->n_pairs) return fail(SVO_ERR_ARG, "pair out of range");
    SVO_HIP(hipSetDevice(b->ctx->device));
    const int L = b->params.max_level + 1;
    const size_t bytes = L * sizeof(svo_level_trace);
    svo_ctx* c = b->ctx;
    void* host = nullptr;
    if (ctx_pinned(c, bytes, &host) == hipSuccess) {  // a kernel copy through the pinned block (as results)
        SVO_HIP(stage_copy(c, host, b->d_traces + (size_t)pair * L, bytes, hipMemcpyDeviceToHost, ctx_stream(c)));
        SVO_HIP(hipStreamSynchronize(ctx_stream(c)));
        std::memcpy(out, host, bytes);
        return SVO_OK;
    }
    (void)hipGetLastError();
    SVO_HIP(hipMemcpyAsync(out, b->d_traces + (size_t)pair * L, bytes, hipMemcpyDeviceToHost, ctx_stream(c)));
    SVO_HIP(hipStreamSynchronize(ctx_stream(c)));
    return SVO_OK;
}

int svo_robust_scale_capacity(int32_t impl, int64_t* slots) {
    if (!slots) return fail(SVO_ERR_ARG, "null argument");
    if (impl == SVO_SCALE_K2V) *slots = svo::refv_max_slots();
    else if (impl == SVO_SCALE_K2R) *slots = SVO_REF_MAX_SLOTS;
    else return fail(SVO_ERR_ARG, "impl %d has no capacity (SVO_SCALE_K2V or SVO_SCALE_K2R)", impl);
    return SVO_OK;
}

int svo_debug_robust_scale(svo_ctx* c, const double* values, int64_t n_slots, int64_t n_valid, int32_t impl, double* out,
                           int64_t out_len) {
    if (!c || !values || !out) return fail(SVO_ERR_ARG, "null argument");
    if (out_len < 2) return fail(SVO_ERR_ARG, "out_len %lld < 2", (long long)out_len);
    if (impl < SVO_SCALE_AUTO || impl > SVO_SCALE_K2V) return fail(SVO_ERR_ARG, "impl %d unknown", impl);
    if (n_slots < 1 || n_slots > 524288 || n_valid < 1 || n_valid > n_slots)
        return fail(SVO_ERR_ARG, "need 1 <= n_valid <= n_slots <= 524288 (got %lld, %lld)", (long long)n_valid,
                    (long long)n_slots);
    if (impl == SVO_SCALE_K2V && n_slots > svo::refv_max_slots())
        return fail(SVO_ERR_ARG, "K2V holds at most %lld slots (got %lld)", (long long)svo::refv_max_slots(),
                    (long long)n_slots);
    for (int64_t i = 0; i < n_slots; ++i)
        if (std::isnan(values[i])) return fail(SVO_ERR_ARG, "value %lld is NaN", (long long)i);
    SVO_HIP(hipSetDevice(c->device));
    const int64_t sel_stride = svo::ref_sel_stride(n_slots);  // u32
    const int64_t q = (n_slots + 63) / 64 * 64;
    constexpr int64_t kDiag = 206;  // the diagnostics either kernel writes
    // out_len past kDiag: K2V's round trace (development; align_refv.hip VDiag::tr) in the rest of out
    const int64_t ntr = impl == SVO_SCALE_K2V && out_len > kDiag ? std::min<int64_t>(out_len - kDiag, 1ll << 28) : 0;
    const size_t bytes = (size_t)q * 8 + (size_t)sel_stride * 4 + (size_t)(kDiag + ntr) * 8;
    void* base = nullptr;
    hipError_t e = ctx_scratch(c, bytes, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_debug_robust_scale: %s", hipGetErrorString(e));
    SVO_HIP(ctx_ring_drain(c));
    double* d_v = static_cast<double*>(base);
    uint32_t* d_sel = reinterpret_cast<uint32_t*>(d_v + q);
    double* d_out = reinterpret_cast<double*>(d_sel + sel_stride);
    SVO_HIP(hipMemsetAsync(d_out, 0, (size_t)(kDiag + ntr) * 8, ctx_stream(c)));
    SVO_HIP(hipMemcpyAsync(d_v, values, (size_t)n_slots * 8, hipMemcpyHostToDevice, ctx_stream(c)));
    // out_len 2 (med / mad only): K2V runs the product kernel's own code path instead of the debug kernel
    if (svo::launch_debug_robust_scale(d_v, (uint32_t)n_slots, (uint32_t)n_valid, d_sel, sel_stride, impl, d_out,
                                       ntr ? d_out + kDiag : nullptr, (uint32_t)ntr, ctx_stream(c), out_len == 2) != 0)
        return fail(SVO_ERR_ARG, "the vector does not fit the requested kernel");
    SVO_HIP(hipGetLastError());
    SVO_HIP(hipMemcpyAsync(out, d_out, (size_t)std::min<int64_t>(out_len, kDiag + ntr) * 8, hipMemcpyDeviceToHost, ctx_stream(c)));
    SVO_HIP(hipStreamSynchronize(ctx_stream(c)));
    return SVO_OK;
}

// ------------------------------------------------------------------ feature alignment
// One FeatureAlignment launch over n candidates whose reference gradient planes are rg[i].
static int feature_align_impl(svo_ctx* c, const svo_camera* cam, int32_t patch_size, const std::vector<const uint8_t*>& rg,
                              const svo_pyramid_set* cur_set, int32_t cur_frame, int32_t n, const double* ref_px,
                              double* px_inout, double* err, int32_t* status) {
    SVO_HIP(hipSetDevice(c->device));
    hipStream_t s = ctx_stream(c);
    // one block, same layout on both sides: ref planes | ref px | px | err | status (8-B aligned pieces);
    // one H2D copy of the inputs (planes .. px) and one D2H copy of the outputs (px .. status)
    const size_t nn = (size_t)n;
    const size_t in_bytes = nn * (sizeof(void*) + 4 * sizeof(double));
    const size_t out_off = nn * (sizeof(void*) + 2 * sizeof(double));
    const size_t total = nn * (sizeof(void*) + 5 * sizeof(double) + 8);
    void* base = nullptr;
    void* host = nullptr;
    std::vector<char> pageable;  // staging past kPinnedCap
    hipError_t e = ctx_scratch(c, total, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_align: %s", hipGetErrorString(e));
    if (ctx_pinned(c, total, &host) != hipSuccess) {
        (void)hipGetLastError();
        pageable.resize(total);
        host = pageable.data();
    }
    char* hb = static_cast<char*>(host);
    std::memcpy(hb, rg.data(), nn * sizeof(void*));
    std::memcpy(hb + nn * sizeof(void*), ref_px, nn * 2 * sizeof(double));
    std::memcpy(hb + out_off, px_inout, nn * 2 * sizeof(double));
    const uint8_t** d_rg = static_cast<const uint8_t**>(base);
    double* d_rpx = reinterpret_cast<double*>(d_rg + nn);
    double* d_px = d_rpx + 2 * nn;
    double* d_err = d_px + 2 * nn;
    int32_t* d_st = reinterpret_cast<int32_t*>(d_err + nn);
    e = stage_copy(c, base, hb, in_bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        svo::FeatureAlignArgs a;
        a.ref_grad = d_rg;
        a.cur_grad = cur_set->d_base + (size_t)cur_frame * cur_set->stride + cur_set->grad_off;
        a.ref_px = d_rpx;
        a.px = d_px;
        a.err = d_err;
        a.status = d_st;
        a.n = n;
        a.half = patch_size / 2;
        a.area = (2 * a.half + 1) * (2 * a.half + 1);
        a.width = cam->width;
        a.height = cam->height;
        svo::launch_feature_align(a, s);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = stage_copy(c, hb + out_off, static_cast<char*>(base) + out_off, total - out_off, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_align: %s", hipGetErrorString(e));
    std::memcpy(px_inout, hb + out_off, nn * 2 * sizeof(double));
    if (err) std::memcpy(err, hb + out_off + nn * 2 * sizeof(double), nn * sizeof(double));
    if (status) std::memcpy(status, hb + out_off + nn * 3 * sizeof(double), nn * sizeof(int32_t));
    return SVO_OK;
}

static int feature_align_check(svo_ctx* c, const svo_camera* cam, int32_t patch_size, const svo_pyramid_set* cur_set,
                               int32_t cur_frame, int32_t n, const double* ref_px, const double* px_inout) {
    if (!c || !cam || !cur_set || (n > 0 && (!ref_px || !px_inout))) return fail(SVO_ERR_ARG, "null argument");
    if (n < 0) return fail(SVO_ERR_ARG, "n < 0");
    if (patch_size < 1 || (2 * (patch_size / 2) + 1) * (2 * (patch_size / 2) + 1) > 128)
        return fail(SVO_ERR_ARG, "patch_size %d unsupported (footprint must be <= 128 px)", patch_size);
    if (cur_set->ctx != c) return fail(SVO_ERR_ARG, "pyramid set belongs to another context");
    if (cur_set->width != cam->width || cur_set->height != cam->height) return fail(SVO_ERR_ARG, "camera/pyramid size mismatch");
    if (cur_frame < 0 || cur_frame >= cur_set->n_frames) return fail(SVO_ERR_ARG, "cur_frame out of range");
    return SVO_OK;
}

int svo_feature_align(svo_ctx* c, const svo_camera* cam, int32_t patch_size, const svo_pyramid_set* ref_set,
                      const int32_t* ref_frames, int32_t ref_frame, const svo_pyramid_set* cur_set, int32_t cur_frame,
                      int32_t n, const double* ref_px, double* px_inout, double* err, int32_t* status) {
    if (int r = feature_align_check(c, cam, patch_size, cur_set, cur_frame, n, ref_px, px_inout)) return r;
    if (!ref_set) return fail(SVO_ERR_ARG, "null argument");
    if (ref_set->ctx != c) return fail(SVO_ERR_ARG, "pyramid set belongs to another context");
    if (ref_set->width != cam->width || ref_set->height != cam->height) return fail(SVO_ERR_ARG, "camera/pyramid size mismatch");
    if (n == 0) return SVO_OK;
    SVO_HIP(set_join(ref_set));
    SVO_HIP(set_join(cur_set));
    std::vector<const uint8_t*> rg(n);
    for (int32_t i = 0; i < n; ++i) {
        const int32_t f = ref_frames ? ref_frames[i] : ref_frame;
        if (f < 0 || f >= ref_set->n_frames) return fail(SVO_ERR_ARG, "ref frame %d out of range", f);
        rg[i] = ref_set->d_base + (size_t)f * ref_set->stride + ref_set->grad_off;
    }
    return feature_align_impl(c, cam, patch_size, rg, cur_set, cur_frame, n, ref_px, px_inout, err, status);
}

int svo_feature_align_multi(svo_ctx* c, const svo_camera* cam, int32_t patch_size, const svo_pyramid_set* const* ref_sets,
                            const int32_t* ref_frames, const svo_pyramid_set* cur_set, int32_t cur_frame, int32_t n,
                            const double* ref_px, double* px_inout, double* err, int32_t* status) {
    if (int r = feature_align_check(c, cam, patch_size, cur_set, cur_frame, n, ref_px, px_inout)) return r;
    if (n > 0 && (!ref_sets || !ref_frames)) return fail(SVO_ERR_ARG, "null argument");
    if (n == 0) return SVO_OK;
    std::vector<const uint8_t*> rg(n);
    for (int32_t i = 0; i < n; ++i) {
        const svo_pyramid_set* p = ref_sets[i];
        if (!p) return fail(SVO_ERR_ARG, "candidate %d: null pyramid set", i);
        if (p->ctx != c) return fail(SVO_ERR_ARG, "candidate %d: pyramid set belongs to another context", i);
        if (p->width != cam->width || p->height != cam->height) return fail(SVO_ERR_ARG, "camera/pyramid size mismatch");
        if (ref_frames[i] < 0 || ref_frames[i] >= p->n_frames) return fail(SVO_ERR_ARG, "ref frame %d out of range", ref_frames[i]);
        rg[i] = p->d_base + (size_t)ref_frames[i] * p->stride + p->grad_off;
        SVO_HIP(set_join(p));
    }
    SVO_HIP(set_join(cur_set));
    return feature_align_impl(c, cam, patch_size, rg, cur_set, cur_frame, n, ref_px, px_inout, err, status);
}

// ------------------------------------------------------------------ map reprojection (host planning)
// Frame::world2image (src/frame.cpp:83-92) with PinholeCamera::project2d (src/pinhole_camera.cpp:53-57):
// the same arithmetic, in the same order, as the device and oracle paths (no FMA contraction).
static inline void world2image(const svo_camera* cam, const svo::SE3& T, const double* p, double* px) {
    const svo::V3 c = svo::se3_act(T, svo::V3{p[0], p[1], p[2]});
    px[0] = cam->fx * (c.x / c.z) + cam->cx;
    px[1] = cam->fy * (c.y / c.z) + cam->cy;
}
static inline bool in_frame(const svo_camera* cam, const double* px, double b) {  // src/pinhole_camera.cpp:163-168
    return px[0] >= b && px[1] >= b && px[0] < cam->width - b && px[1] < cam->height - b;
}

int svo_world2image(const svo_camera* cam, const double* pose, int32_t n, const double* points, double* px) {
    if (!cam || !pose || n < 0 || (n > 0 && (!points || !px))) return fail(SVO_ERR_ARG, "null argument");
    const svo::SE3 T = svo::se3_load(pose);
    for (int32_t i = 0; i < n; ++i) world2image(cam, T, points + 3 * i, px + 2 * i);
    return SVO_OK;
}

int svo_map_reproject_plan(const svo_camera* cam, int32_t cell_size, int32_t n_cells, const int32_t* cell_order,
                           const double* cur_pose, uint64_t cur_id, int32_t n_kf, const int32_t* kf_feat_off,
                           const int32_t* feat_point, int32_t n_points, const double* point_pos,
                           const uint32_t* point_type, uint64_t* point_last, int32_t* overlap, int32_t* n_sel,
                           int32_t* sel_feat, int32_t* sel_cell, double* sel_px, int32_t* matches, int32_t* trials) {
    if (!cam || !cell_order || !cur_pose || !kf_feat_off || !overlap || !n_sel || !sel_feat || !sel_cell || !sel_px ||
        !matches || !trials || (n_points > 0 && (!point_pos || !point_type || !point_last)))
        return fail(SVO_ERR_ARG, "null argument");
    if (cell_size < 1) return fail(SVO_ERR_ARG, "cell_size %d", cell_size);
    const int32_t cols = (int32_t)std::ceil((double)cam->width / cell_size);  // src/map.cpp:226-227
    const int32_t rows = (int32_t)std::ceil((double)cam->height / cell_size);
    if (n_cells != cols * rows) return fail(SVO_ERR_ARG, "n_cells %d != %d x %d", n_cells, cols, rows);
    if (n_kf < 0 || (kf_feat_off[n_kf] > 0 && !feat_point)) return fail(SVO_ERR_ARG, "bad feature table");
    for (int32_t i = 0; i < n_cells; ++i)
        if (cell_order[i] < 0 || cell_order[i] >= n_cells) return fail(SVO_ERR_ARG, "cell_order[%d] out of range", i);
    const svo::SE3 T = svo::se3_load(cur_pose);
    std::vector<std::vector<int32_t>> cells(n_cells);  // resetGrid (:250-258)
    double px[2];
    for (int32_t k = 0; k < n_kf; ++k) {  // closeKeyframes: ref, then ref->lastKeyframe (:441-461)
        overlap[k] = 0;
        for (int32_t f = kf_feat_off[k]; f < kf_feat_off[k + 1]; ++f) {
            const int32_t p = feat_point[f];
            if (p < 0) continue;
            if (p >= n_points) return fail(SVO_ERR_ARG, "feature %d: point %d out of range", f, p);
            if (point_last[p] == cur_id) continue;
            point_last[p] = cur_id;
            world2image(cam, T, point_pos + 3 * p, px);  // reprojectPoint (:481-492)
            if (!in_frame(cam, px, 3.0)) continue;
            const uint32_t cell = (uint32_t)(int32_t)px[1] / (uint32_t)cell_size * (uint32_t)cols +
                                  (uint32_t)(int32_t)px[0] / (uint32_t)cell_size;
            cells[cell].push_back(f);
            ++overlap[k];
        }
    }
    int32_t m = 0, t = 0, ns = 0;
    for (int32_t i = 0; i < n_cells; ++i) {  // (:463-477)
        const int32_t idx = cell_order[i];
        std::vector<int32_t>& c = cells[idx];
        if (!c.empty()) {
            // reprojectCell (:505-570): std::sort by point type, descending (the reference's own
            // comparator, so cells past 16 candidates keep libstdc++'s order), first non-deleted wins;
            // its FeatureAlignment result is not used to accept or reject
            std::sort(c.begin(), c.end(), [&](int32_t a, int32_t b) { return point_type[feat_point[a]] > point_type[feat_point[b]]; });
            for (int32_t f : c) {
                ++t;
                if (point_type[feat_point[f]] == 1u) continue;  // Point::PointType::DELETED
                sel_feat[ns] = f;
                sel_cell[ns] = idx;
                world2image(cam, T, point_pos + 3 * feat_point[f], sel_px + 2 * ns);
                ++ns;
                ++m;
                break;
            }
        }
        if (m > 150) break;
    }
    *n_sel = ns;
    *matches = m;
    *trials = t;
    return SVO_OK;
}

// ------------------------------------------------------------------ depth filter
int svo_depth_seed_init(double depth_mean, double depth_min, svo_depth_seed* seed) {
    if (!seed) return fail(SVO_ERR_ARG, "null seed");
    seed->a = 10;                          // src/mixed_gaussian_filter.cpp:10-11
    seed->b = 10;
    seed->mu = 1.0 / depth_mean;           // :13
    seed->max_depth = 1.0 / depth_min;     // :14
    seed->sigma = seed->max_depth / 6;     // :18
    seed->var = seed->sigma * seed->sigma; // :20
    seed->valid = 1;                       // :21
    return SVO_OK;
}

int svo_depth_update(svo_ctx* c, const svo_camera* cam, int32_t n_kf, const svo_pyramid_set* const* kf_sets,
                     const int32_t* kf_frames, const double* kf_poses, const svo_pyramid_set* cur_set,
                     int32_t cur_frame, const double* cur_pose, int32_t n, svo_depth_seed* seeds,
                     int32_t* n_out, int32_t* outcome, double* cand_points, int32_t* cand_seed, int32_t* n_cand) {
    if (!c || !cam || !cur_set || !cur_pose || !n_out || !n_cand || (n_kf > 0 && (!kf_sets || !kf_frames || !kf_poses)))
        return fail(SVO_ERR_ARG, "null argument");
    if (n < 0 || n_kf < 0) return fail(SVO_ERR_ARG, "negative count");
    if (n > 0 && (!seeds || !cand_points || !cand_seed)) return fail(SVO_ERR_ARG, "null seed / candidate array");
    auto check_set = [&](const svo_pyramid_set* p, int32_t frame) -> int {
        if (!p) return fail(SVO_ERR_ARG, "null pyramid set");
        if (p->ctx != c) return fail(SVO_ERR_ARG, "pyramid set belongs to another context");
        if (p->width != cam->width || p->height != cam->height) return fail(SVO_ERR_ARG, "camera/pyramid size mismatch");
        if (frame < 0 || frame >= p->n_frames) return fail(SVO_ERR_ARG, "frame %d out of range", frame);
        SVO_HIP(set_join(p));
        return SVO_OK;
    };
    int rc;
    if ((rc = check_set(cur_set, cur_frame)) != SVO_OK) return rc;
    std::vector<const uint8_t*> kimg(n_kf > 0 ? n_kf : 1);
    for (int32_t k = 0; k < n_kf; ++k) {
        if ((rc = check_set(kf_sets[k], kf_frames[k])) != SVO_OK) return rc;
        kimg[k] = kf_sets[k]->d_base + (size_t)kf_frames[k] * kf_sets[k]->stride;  // intensity stack, level 0
    }
    for (int32_t i = 0; i < n; ++i)
        if (seeds[i].kf < 0 || seeds[i].kf >= n_kf) return fail(SVO_ERR_ARG, "seed %d: keyframe %d out of range", i, seeds[i].kf);
    *n_out = 0;
    *n_cand = 0;
    if (n == 0) return SVO_OK;
    SVO_HIP(hipSetDevice(c->device));
    hipStream_t s = ctx_stream(c);
    svo::DepthArgs a{};
    // one block, same layout on both sides: inputs (seeds | keyframe poses | keyframe planes | cur pose),
    // outputs (counts | survivors | outcomes | candidate points | candidate seeds), device-only scratch
    // (updated seeds | points); one H2D and one D2H copy through the context's pinned staging
    const size_t N = (size_t)n, K = (size_t)(n_kf > 0 ? n_kf : 1), SZ = sizeof(svo_depth_seed);
    auto r8 = [](size_t v) { return (v + 7) / 8 * 8; };
    const size_t o_seeds = 0, o_kpose = o_seeds + N * SZ, o_kimg = o_kpose + K * 56, o_cpose = o_kimg + K * 8,
                 in_end = o_cpose + 56;
    const size_t o_counts = in_end, o_out = o_counts + 8, o_outc = o_out + N * SZ, o_cpts = o_outc + r8(N * 4),
                 o_cseed = o_cpts + N * 24, out_end = o_cseed + r8(N * 4);
    const size_t o_new = out_end, o_points = o_new + N * SZ, total = o_points + N * 24;
    void* base = nullptr;
    void* host = nullptr;
    std::vector<char> pageable;  // staging past kPinnedCap
    hipError_t e = ctx_scratch(c, total, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_depth_update: %s", hipGetErrorString(e));
    if (ctx_pinned(c, out_end, &host) != hipSuccess) {
        (void)hipGetLastError();
        pageable.resize(out_end);
        host = pageable.data();
    }
    char* hb = static_cast<char*>(host);
    char* db = static_cast<char*>(base);
    std::memcpy(hb + o_seeds, seeds, N * SZ);
    if (n_kf > 0) {
        std::memcpy(hb + o_kpose, kf_poses, (size_t)n_kf * 56);
        std::memcpy(hb + o_kimg, kimg.data(), (size_t)n_kf * 8);
    }
    std::memcpy(hb + o_cpose, cur_pose, 56);
    e = stage_copy(c, db, hb, in_end, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        a.seeds = reinterpret_cast<svo_depth_seed*>(db + o_seeds);
        a.seeds_new = reinterpret_cast<svo_depth_seed*>(db + o_new);
        a.seeds_out = reinterpret_cast<svo_depth_seed*>(db + o_out);
        a.outcome = reinterpret_cast<int32_t*>(db + o_outc);
        a.points = reinterpret_cast<double*>(db + o_points);
        a.cand_points = reinterpret_cast<double*>(db + o_cpts);
        a.cand_seed = reinterpret_cast<int32_t*>(db + o_cseed);
        a.counts = reinterpret_cast<int32_t*>(db + o_counts);
        a.kf_imgs = reinterpret_cast<const uint8_t* const*>(db + o_kimg);
        a.kf_poses = reinterpret_cast<double*>(db + o_kpose);
        a.cur_img = cur_set->d_base + (size_t)cur_frame * cur_set->stride;
        a.cur_pose = reinterpret_cast<double*>(db + o_cpose);
        a.n = n; a.width = cam->width; a.height = cam->height;
        a.fx = cam->fx; a.fy = cam->fy; a.cx = cam->cx; a.cy = cam->cy;
        a.err_angle = std::atan(1.0 / (2.0 * cam->fx)) * 2.0;  // src/depth_estimator.cpp:202-206 (pixel noise 1)
        svo::launch_depth_update(a, s);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = stage_copy(c, hb + in_end, db + in_end, out_end - in_end, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_depth_update: %s", hipGetErrorString(e));
    int32_t counts[2];
    std::memcpy(counts, hb + o_counts, sizeof(counts));
    std::memcpy(seeds, hb + o_out, (size_t)counts[0] * SZ);
    if (outcome) std::memcpy(outcome, hb + o_outc, N * 4);
    std::memcpy(cand_points, hb + o_cpts, (size_t)counts[1] * 24);
    std::memcpy(cand_seed, hb + o_cseed, (size_t)counts[1] * 4);
    *n_out = counts[0];
    *n_cand = counts[1];
    return SVO_OK;
}

// ------------------------------------------------------------------ feature selection
int svo_feature_grid_size(int32_t width, int32_t height, int32_t cell_size, int32_t* rows, int32_t* cols) {
    if (!rows || !cols) return fail(SVO_ERR_ARG, "null argument");
    if (width < 1 || height < 1 || cell_size < 1) return fail(SVO_ERR_ARG, "bad grid geometry");
    *rows = height / cell_size + 1;  // src/feature_selection.cpp:21-22
    *cols = width / cell_size + 1;
    return SVO_OK;
}

static int fs_check(svo_ctx* c, const svo_pyramid_set* p, int32_t frame, int32_t threshold) {
    if (!c || !p) return fail(SVO_ERR_ARG, "null argument");
    if (p->ctx != c) return fail(SVO_ERR_ARG, "pyramid set belongs to another context");
    if (frame < 0 || frame >= p->n_frames) return fail(SVO_ERR_ARG, "frame %d out of range", frame);
    if (threshold < 0) return fail(SVO_ERR_ARG, "threshold < 0");
    if ((int64_t)p->width * p->height >= ((int64_t)1 << 24)) return fail(SVO_ERR_ARG, "image of 2^24 pixels or more");
    SVO_HIP(set_join(p));
    return SVO_OK;
}

// device detection into host keys; *n = keys above the threshold (may exceed capacity: nothing copied then)
static int fs_detect(svo_ctx* c, const svo_pyramid_set* p, int32_t frame, int32_t threshold, int32_t capacity,
                     uint32_t* keys, int32_t* n) {
    SVO_HIP(hipSetDevice(c->device));
    hipStream_t s = ctx_stream(c);
    const int64_t npx = (int64_t)p->width * p->height;
    const int nseg = svo::feature_detect_segments(npx);
    void* base = nullptr;
    hipError_t e = ctx_scratch(c, (size_t)npx * 4 + (size_t)nseg * 4 + 64, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_detect: %s", hipGetErrorString(e));
    uint32_t* d_keys = static_cast<uint32_t*>(base);
    int* d_n = reinterpret_cast<int*>(d_keys + npx);
    int* d_seg = d_n + 16;
    const uint8_t* plane = p->d_base + (size_t)frame * p->stride + p->grad_off;
    svo::launch_feature_detect(plane, p->width, p->height, threshold, d_seg, d_keys, d_n, s);
    e = hipGetLastError();
    // the count, then the keys, through the pinned staging when it is large enough
    void* host = nullptr;
    const bool staged = ctx_pinned(c, (size_t)npx * 4 + 64, &host) == hipSuccess;
    if (!staged) (void)hipGetLastError();
    int32_t cnt = 0;
    int32_t* h_n = staged ? static_cast<int32_t*>(host) : &cnt;
    if (e == hipSuccess) e = stage_copy(c, h_n, d_n, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    cnt = *h_n;
    if (e == hipSuccess && cnt <= capacity && cnt > 0) {
        if (staged) {
            uint32_t* hk = reinterpret_cast<uint32_t*>(static_cast<char*>(host) + 64);
            e = stage_copy(c, hk, d_keys, (size_t)cnt * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) std::memcpy(keys, hk, (size_t)cnt * 4);
        } else {
            e = hipMemcpy(keys, d_keys, (size_t)cnt * 4, hipMemcpyDeviceToHost);
        }
    }
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_detect: %s", hipGetErrorString(e));
    *n = cnt;
    return SVO_OK;
}

int svo_feature_detect(svo_ctx* c, const svo_pyramid_set* p, int32_t frame, int32_t threshold, int32_t capacity,
                       uint32_t* keys, int32_t* n_keys) {
    if (int r = fs_check(c, p, frame, threshold)) return r;
    if (!n_keys || (capacity > 0 && !keys)) return fail(SVO_ERR_ARG, "null argument");
    if (int r = fs_detect(c, p, frame, threshold, capacity, keys, n_keys)) return r;
    if (*n_keys > capacity) return fail(SVO_ERR_ARG, "%d keypoints exceed capacity %d", *n_keys, capacity);
    return SVO_OK;
}

int svo_feature_select_ssc(svo_ctx* c, const svo_pyramid_set* p, int32_t frame, int32_t threshold,
                           int32_t number_candidate, int32_t use_bucketing, int32_t cell_size, uint8_t* occupancy,
                           int32_t capacity, double* px_out, double* response_out, int32_t* n_out, int32_t* n_keypoints) {
    if (int r = fs_check(c, p, frame, threshold)) return r;
    if (!n_out || (capacity > 0 && (!px_out || !response_out))) return fail(SVO_ERR_ARG, "null argument");
    if (number_candidate < 2) return fail(SVO_ERR_ARG, "numberCandidate < 2 (SSC divides by numberCandidate - 1)");
    if (use_bucketing && (cell_size < 1 || !occupancy)) return fail(SVO_ERR_ARG, "bucketing needs cell_size and occupancy");
    const int32_t W = p->width, H = p->height;
    std::unique_ptr<uint32_t[]> keys(new (std::nothrow) uint32_t[(size_t)W * H]);  // not zero-filled
    if (!keys) return fail(SVO_ERR_ARG, "out of host memory");
    int32_t n = 0;
    if (int r = fs_detect(c, p, frame, threshold, W * H, keys.get(), &n)) return r;
    if (n_keypoints) *n_keypoints = n;
    svo::feature_sort_keys(keys.get(), n);  // :53-54
    std::vector<int32_t> xs(n), ys(n), sel;
    for (int32_t i = 0; i < n; ++i) {
        const int32_t idx = (int32_t)(keys[i] & 0xFFFFFFu);
        ys[i] = idx / W;
        xs[i] = idx - ys[i] * W;
    }
    svo::feature_ssc(xs.data(), ys.data(), n, number_candidate, 0.1f, W, H, sel);  // :57-58
    const int32_t gcols = use_bucketing ? W / cell_size + 1 : 0;
    int32_t m = 0;
    for (int32_t i : sel) {
        if (use_bucketing) {  // :60-76
            uint8_t& cell = occupancy[(xs[i] / cell_size) + (ys[i] / cell_size) * gcols];
            if (cell) continue;
            cell = 1;
        }
        if (m >= capacity) return fail(SVO_ERR_ARG, "more than capacity %d features", capacity);
        px_out[2 * m] = xs[i];
        px_out[2 * m + 1] = ys[i];
        response_out[m] = (double)(keys[i] >> 24);
        ++m;
    }
    if (use_bucketing) std::memset(occupancy, 0, (size_t)(H / cell_size + 1) * gcols);  // resetGridOccupancy
    *n_out = m;
    return SVO_OK;
}

int svo_feature_select_by_value(svo_ctx* c, const svo_pyramid_set* p, int32_t frame, int32_t threshold,
                                int32_t cell_size, uint8_t* occupancy, int32_t capacity, double* px_out,
                                double* response_out, int32_t* n_out) {
    if (int r = fs_check(c, p, frame, threshold)) return r;
    if (!occupancy || !n_out || (capacity > 0 && (!px_out || !response_out))) return fail(SVO_ERR_ARG, "null argument");
    if (cell_size < 1 || cell_size > 1024) return fail(SVO_ERR_ARG, "cell_size must be in [1, 1024]");
    const int32_t W = p->width, H = p->height, gr = H / cell_size + 1, gc = W / cell_size + 1, nc = gr * gc;
    SVO_HIP(hipSetDevice(c->device));
    hipStream_t s = ctx_stream(c);
    void* base = nullptr;
    hipError_t e = ctx_scratch(c, (size_t)nc * 5 + 64, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_select_by_value: %s", hipGetErrorString(e));
    uint32_t* d_px = static_cast<uint32_t*>(base);
    uint8_t* d_occ = reinterpret_cast<uint8_t*>(d_px + nc);
    // pinned staging when available: [cells (4 nc) | occupancy (nc)] on both sides
    void* host = nullptr;
    std::vector<uint32_t> pageable;
    uint32_t* cell_px;
    uint8_t* h_occ;
    if (ctx_pinned(c, (size_t)nc * 5, &host) == hipSuccess) {
        cell_px = static_cast<uint32_t*>(host);
        h_occ = reinterpret_cast<uint8_t*>(cell_px + nc);
        std::memcpy(h_occ, occupancy, nc);
    } else {
        (void)hipGetLastError();
        pageable.resize(nc);
        cell_px = pageable.data();
        h_occ = occupancy;
    }
    e = stage_copy(c, d_occ, h_occ, nc, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        const uint8_t* plane = p->d_base + (size_t)frame * p->stride + p->grad_off;
        svo::launch_feature_cell_max(plane, W, H, cell_size, gr, gc, d_occ, threshold, d_px, s);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = stage_copy(c, cell_px, d_px, (size_t)nc * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_feature_select_by_value: %s", hipGetErrorString(e));
    int32_t m = 0;
    for (int32_t k = 0; k < nc; ++k) {
        const uint32_t v = (uint32_t)cell_px[k];
        if (v == 0xFFFFFFFFu) continue;
        if (m >= capacity) return fail(SVO_ERR_ARG, "more than capacity %d features", capacity);
        const int32_t idx = (int32_t)(v & 0xFFFFFFu);
        px_out[2 * m] = idx % W;
        px_out[2 * m + 1] = idx / W;
        response_out[m] = (double)(v >> 24);
        ++m;
    }
    std::memset(occupancy, 0, nc);  // resetGridOccupancy (:141)
    *n_out = m;
    return SVO_OK;
}

// ------------------------------------------------------------------ trajectory output
int svo_pose_matrix3x4_inverse(const double* pose, double* out12) {
    if (!pose || !out12) return fail(SVO_ERR_ARG, "null argument");
    const svo::SE3 T{{pose[0], pose[1], pose[2], pose[3]}, {pose[4], pose[5], pose[6]}};
    const svo::SE3 Ti = svo::se3_inverse(T);  // Sophus SE3::inverse
    double R[3][3];
    svo::rotmat(Ti.q, R);  // SO3::matrix (Eigen toRotationMatrix)
    const double t[3] = {Ti.t.x, Ti.t.y, Ti.t.z};
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) out12[4 * r + c] = R[r][c];
        out12[4 * r + 3] = t[r];
    }
    return SVO_OK;
}

int svo_format_kitti_pose(const double* pose, char* buf, int32_t cap) {
    if (!buf || cap < 1) return fail(SVO_ERR_ARG, "null argument");
    double m[12];
    if (int r = svo_pose_matrix3x4_inverse(pose, m)) return r;
    int32_t o = 0;
    for (int i = 0; i < 12; ++i) {
        const int k = std::snprintf(buf + o, (size_t)(cap - o), i ? " %.6g" : "%.6g", m[i]);
        if (k < 0 || k >= cap - o) {
            buf[0] = 0;
            return fail(SVO_ERR_ARG, "buffer of %d bytes too short", cap);
        }
        o += k;
    }
    return SVO_OK;
}

// ------------------------------------------------------------------ pose-only bundle adjustment
int svo_pose_optimize(svo_ctx* c, int32_t n_frames, const int32_t* feat_off, const double* bearing, const double* point,
                      const uint8_t* has_point, uint8_t* vis_inout, double* poses_inout, double* err, int32_t* status) {
    if (!c || (n_frames > 0 && (!feat_off || !poses_inout || !err || !status))) return fail(SVO_ERR_ARG, "null argument");
    if (n_frames < 0) return fail(SVO_ERR_ARG, "n_frames < 0");
    if (n_frames == 0) return SVO_OK;
    if (feat_off[0] != 0) return fail(SVO_ERR_ARG, "feat_off[0] must be 0");
    for (int32_t f = 0; f < n_frames; ++f)
        if (feat_off[f + 1] < feat_off[f]) return fail(SVO_ERR_ARG, "feat_off not ascending at frame %d", f);
    const int64_t nf = feat_off[n_frames];
    if (nf > 0 && (!bearing || !point || !has_point || !vis_inout)) return fail(SVO_ERR_ARG, "null argument");
    if (nf >= ((int64_t)1 << 28)) return fail(SVO_ERR_ARG, "too many features");
    for (int64_t k = 0; k < nf; ++k)
        if (vis_inout[k] && !has_point[k])
            return fail(SVO_ERR_ARG, "feature %lld: visible from the previous call but without a point "
                                     "(the reference dereferences a null m_point)", (long long)k);
    SVO_HIP(hipSetDevice(c->device));
    hipStream_t s = ctx_stream(c);
    // one block, same layout on both sides: inputs (offsets | poses | bearing | point | has_point | flags)
    // then outputs (poses | err | status | flags) then device-only scratch (rows | weights); one H2D copy
    // of the inputs and one D2H copy of the outputs through the context's pinned staging
    const size_t F = (size_t)n_frames, N = (size_t)nf;
    auto r8 = [](size_t b) { return (b + 7) / 8 * 8; };
    const size_t o_off = 0, o_pin = o_off + r8((F + 1) * 4), o_bear = o_pin + F * 56, o_pt = o_bear + N * 24,
                 o_has = o_pt + N * 24, o_vin = o_has + r8(N), in_end = o_vin + r8(N);
    const size_t o_pout = in_end, o_err = o_pout + F * 56, o_st = o_err + F * 8, o_vout = o_st + r8(F * 4),
                 out_end = o_vout + r8(N);
    const size_t o_rows = out_end, o_wts = o_rows + N * 24, total = o_wts + N * 8;
    void* base = nullptr;
    void* host = nullptr;
    hipError_t e = ctx_scratch(c, total, &base);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_pose_optimize: %s", hipGetErrorString(e));
    const bool staged = ctx_pinned(c, out_end, &host) == hipSuccess;
    (void)hipGetLastError();
    char* hb = static_cast<char*>(host);
    char* db = static_cast<char*>(base);
    struct Piece { size_t off; const void* src; size_t bytes; };
    const Piece in[] = {{o_off, feat_off, (F + 1) * 4}, {o_pin, poses_inout, F * 56}, {o_bear, bearing, N * 24},
                        {o_pt, point, N * 24}, {o_has, has_point, N}, {o_vin, vis_inout, N}};
    for (const Piece& pc : in) {
        if (!pc.bytes) continue;
        if (staged) std::memcpy(hb + pc.off, pc.src, pc.bytes);
        else if (e == hipSuccess) e = stage_copy(c, db + pc.off, pc.src, pc.bytes, hipMemcpyHostToDevice, s);
    }
    if (staged && e == hipSuccess) e = stage_copy(c, db, hb, in_end, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        svo::PoseBAArgs a{reinterpret_cast<int32_t*>(db + o_off), reinterpret_cast<double*>(db + o_bear),
                          reinterpret_cast<double*>(db + o_pt), reinterpret_cast<uint8_t*>(db + o_has),
                          reinterpret_cast<uint8_t*>(db + o_vin), reinterpret_cast<uint8_t*>(db + o_vout),
                          reinterpret_cast<double*>(db + o_pin), reinterpret_cast<double*>(db + o_pout),
                          reinterpret_cast<double*>(db + o_err), reinterpret_cast<int32_t*>(db + o_st),
                          reinterpret_cast<double*>(db + o_rows), reinterpret_cast<double*>(db + o_wts), n_frames};
        svo::launch_pose_ba(a, s);
        e = hipGetLastError();
    }
    struct Out { size_t off; void* dst; size_t bytes; };
    const Out out[] = {{o_pout, poses_inout, F * 56}, {o_err, err, F * 8}, {o_st, status, F * 4}, {o_vout, vis_inout, N}};
    if (staged) {
        if (e == hipSuccess) e = stage_copy(c, hb + in_end, db + in_end, out_end - in_end, hipMemcpyDeviceToHost, s);
    } else {
        for (const Out& o : out)
            if (o.bytes && e == hipSuccess) e = stage_copy(c, o.dst, db + o.off, o.bytes, hipMemcpyDeviceToHost, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, "svo_pose_optimize: %s", hipGetErrorString(e));
    if (staged)
        for (const Out& o : out)
            if (o.bytes) std::memcpy(o.dst, hb + o.off, o.bytes);
    return SVO_OK;
}

}  // extern "C"
