// svo_internal.h — device-side argument blocks shared by the kernels and the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/svo_c.h"

namespace svo {

constexpr int kMaxLevels = 12;

struct LevelGeom {  // one pyramid geometry (all frames of a set share it)
    int32_t w[kMaxLevels], h[kMaxLevels];
    int64_t off[kMaxLevels];
    int64_t frame_bytes;  // bytes of one packed stack
    int32_t levels;
};

struct PairDesc {  // per frame pair, device resident (inputs; never written by the kernels)
    const uint8_t* ref_pyr;
    const uint8_t* kf_pyr;
    const uint8_t* cur_pyr;
    double ref_pose[7];
    double kf_pose[7];
    double cur_pose[7];
    int32_t n_ref, n_kf;
};

struct PairState {  // per frame pair, carried from stage to stage and level to level
    double pose[7];             // current estimate of cur->m_absPose
    double med, mad, sigma, c;  // robust scale of the current level (K2)
    double err;                 // RMSE of the last finished level
    uint32_t n, n_ref_vis;      // visible pixel slots / ref-visible features of the current level
    int32_t status, active;     // Optimizer::Status of the last level; 0 = nothing to align
    int32_t scale_kernel, pad;  // SVO_SCALE_* of the kernel that computed med / mad at the current level
};

struct AlignArgs {
    const PairDesc* pairs;
    PairState* state;         // [n_pairs]
    const double* px;         // [n_pairs*max_f][2]
    const double* bearing;    // [n_pairs*max_f][3]
    const double* point;      // [n_pairs*max_f][3]
    const uint8_t* has_point; // [n_pairs*max_f]
    double* xw;               // scratch [n_pairs*max_f][3]   world point per feature
    uint8_t* fvis;            // scratch [n_pairs*max_f]      bit0 ref visible, bit1 cur visible
    double* partials;         // scratch [n_pairs][chunks][28] per-workgroup J^T W J (21) | J^T W r (6) | chi2
    uint32_t* arrive;         // scratch [n_pairs] K3 workgroups of the current level that have published partials
    // Residual slots of a pair are pixel-major: slot (k, f) = k * fstride + f for pixel k of the patch and
    // feature f, fstride = n_features rounded up to 64 (one lane per feature, one 128-B key line per wave
    // and pixel).  Slots of features >= n_features are invisible.  Only the 16-bit keys are stored; exact
    // residuals are recomputed from the images where needed (K2 candidates, K3).
    double* cproj;            // scratch [n_pairs*max_f][2] projection (cu, cv) into the cur level (K1)
    double* scratch;          // scratch [n_pairs][key_stride] exact residuals: K2's exact paths (median_mode 0);
                              // median_mode 1: K1's residuals in the reference's feature-major slot order
    uint16_t* keys;           // scratch [n_pairs][key_stride] 16-bit monotone key per slot (0xFFFF = invisible)
    uint32_t* sel;            // median_mode 1: [n_pairs][sel_stride] K2R scratch (segment, mailbox, step records)
    int64_t sel_stride;       // u32 per pair: ref_sel_stride(max_f * area)
    int32_t median_mode;      // 0 exact order statistics (K2), 1 the reference's nth_element post-state (K2V, or
                              // K2R for vectors past K2V's registers: launch_scale_ref chooses by max_slots)
    int64_t key_stride;       // >= area * round_up(max_f, 64), multiple of 64
    uint32_t* win;            // scratch [n_pairs][win_stride] feature windows of the window levels (K1 -> K3)
    int64_t win_stride;       // dwords per pair: align_win_dwords(half) * round_up(max_f, 64)
    uint32_t win_levels;      // bit l: at level l K1 hands each visible feature's ref / cur windows to K3
                              // (K3 then reads them instead of gathering from the pyramid planes)
    double* pose_out;         // [n_pairs][7]
    double* err_out;          // [n_pairs]
    int32_t* status_out;      // [n_pairs]
    svo_level_trace* traces;  // [n_pairs][max_level+1]
    int32_t n_pairs, max_f, half, area, min_level, max_level;
    int32_t max_slots;        // largest (n_ref + n_kf) * area over these pairs: the reference-mode robust scale
                              // kernel is chosen by it (K2V when it fits), not by the batch capacity max_f
    int32_t pair_base;        // index of pair 0 of these arguments in the whole batch (sub-batch chains)
    int32_t feat_iters;       // feature groups one K1/K3 wave walks through
    int32_t chunks;           // K1/K3 workgroups per pair = align_chunks(max_f, half, feat_iters)
    double fx, fy, cx, cy;
    LevelGeom geom;
};

void launch_align(const AlignArgs& a, hipStream_t s, hipEvent_t* marks = nullptr);  // marks: see align.hip
void launch_scale_ref(const AlignArgs& a, int level, hipStream_t s);                 // K2R (align_ref.hip)
// svo_debug_robust_scale: impl SVO_SCALE_*; returns -1 if the vector does not fit the requested kernel
// plain (K2V): the product kernel's own code path (no diagnostics, out[0..1] only) instead of the debug kernel
int launch_debug_robust_scale(const double* v, uint32_t M, uint32_t n, uint32_t* sel, int64_t sel_stride, int impl,
                              double* out, double* trace, uint32_t trcap, hipStream_t s, bool plain = false);
int scale_impl();  // SVO_SCALE_IMPL knob (0 auto)
int64_t ref_sel_stride(int64_t max_slots);  // K2R scratch per pair (u32) for vectors of up to max_slots
// K2V (align_refv.hip): the same selection with the vector in registers, vectors of <= refv_max_slots()
int64_t refv_max_slots();
void launch_scale_refv(const AlignArgs& a, int level, hipStream_t s);
void launch_debug_robust_scale_v(const double* v, uint32_t M, uint32_t n, double* gseg, double* out, double* trace,
                                 uint32_t trcap, hipStream_t s, bool plain);
int align_max_half();  // largest patch half size the alignment kernels are instantiated for
int align_feat_iters();                                 // feature groups per K1/K3 wave
int align_win_dwords(int half);                         // window dwords per feature (win_stride / slots)
int align_chunks(int max_f, int half, int feat_iters);  // K1/K3 workgroups per pair
void launch_pyramid(uint8_t* stacks, const LevelGeom& g, int32_t first, int32_t count, hipStream_t s);

#if defined(SVO_TIMELINE)
// Diagnostic build only (make timeline -> build/timeline/): one record per workgroup of K1 / K2V / K3 with its start
// and end on the chip-wide 100 MHz clock and the CU it ran on, so a step's CU time can be split by kernel and idle
// (tools/timeline.py).  A TlScope at the top of a kernel body records the workgroup when it goes out of scope, early
// returns included; thread 0's clock stands for the workgroup.
struct TlRec {
    uint64_t t0, t1;
    uint32_t kind, level, block, hw, xcc, pair_base;
};
constexpr uint32_t kTlCap = 1u << 18;
enum : uint32_t { kTlK1 = 1, kTlK2V = 2, kTlK3 = 3 };
struct TlScope {
    TlRec* rec;
    uint32_t* n;
    uint64_t t0;
    uint32_t kind, level, pb;
    __device__ __forceinline__ TlScope(TlRec* r, uint32_t* nn, uint32_t k, uint32_t l, uint32_t p)
        : rec(r), n(nn), t0(__builtin_amdgcn_s_memrealtime()), kind(k), level(l), pb(p) {}
    __device__ __forceinline__ ~TlScope() {
        if (threadIdx.x == 0) {
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave, SIMD, CU, SH, SE
            const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
            const uint32_t i = __hip_atomic_fetch_add(n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (i < kTlCap) rec[i] = TlRec{t0, t1, kind, level, blockIdx.x, hw, xcc, pb};
        }
    }
};
#define SVO_TL_DEFINE(tag)                    \
    __device__ TlRec g_tl_rec_##tag[kTlCap]; \
    __device__ uint32_t g_tl_n_##tag;
#define SVO_TL_SCOPE(tag, kind, level, pb) TlScope tl_scope_(g_tl_rec_##tag, &g_tl_n_##tag, kind, (uint32_t)(level), (uint32_t)(pb))
// extern "C" int svo_debug_timeline_<tag>(void* out, size_t bytes, uint32_t* count, int reset): copy the records out
// (or, with reset, zero the count)
#define SVO_TL_READER(tag)                                                                                       \
    extern "C" int svo_debug_timeline_##tag(void* out, size_t bytes, uint32_t* count, int reset) {                \
        if (reset) {                                                                                             \
            const uint32_t z = 0;                                                                                \
            return hipMemcpyToSymbol(HIP_SYMBOL(g_tl_n_##tag), &z, sizeof z) == hipSuccess ? 0 : -2;             \
        }                                                                                                        \
        if (hipMemcpyFromSymbol(count, HIP_SYMBOL(g_tl_n_##tag), sizeof(uint32_t)) != hipSuccess) return -2;     \
        const size_t want = (size_t)(*count < kTlCap ? *count : kTlCap) * sizeof(TlRec);                         \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl_rec_##tag), bytes < want ? bytes : want) == hipSuccess ? 0 \
                                                                                                               : -2; \
    }
#else
#define SVO_TL_SCOPE(tag, kind, level, pb) \
    do {                                   \
    } while (0)
#endif

struct FeatureAlignArgs {
    const uint8_t* const* ref_grad;  // [n] level-0 gradient image of each candidate's reference frame
    const uint8_t* cur_grad;         // level-0 gradient image of the current frame
    const double* ref_px;       // [n][2]
    double* px;                 // [n][2] in/out
    double* err;                // [n]
    int32_t* status;            // [n]
    int32_t n, half, area, width, height;
};
void launch_feature_align(const FeatureAlignArgs& a, hipStream_t s);

struct DepthArgs {
    const svo_depth_seed* seeds;     // [n] input state
    svo_depth_seed* seeds_new;       // [n] state after the update (scratch)
    svo_depth_seed* seeds_out;       // [n] survivors, compacted (stable)
    int32_t* outcome;                // [n] SVO_DEPTH_*
    double* points;                  // [n][3] candidate point of a converged seed (scratch)
    double* cand_points;             // [n][3] candidates in the update loop's order
    int32_t* cand_seed;              // [n] their seed index
    int32_t* counts;                 // [2] survivors, candidates
    const uint8_t* const* kf_imgs;   // [n_kf] level-0 intensity image of each keyframe
    const double* kf_poses;          // [n_kf][7]
    const uint8_t* cur_img;          // level-0 intensity image of the current frame
    const double* cur_pose;          // [7]
    int32_t n, width, height;
    double fx, fy, cx, cy, err_angle;
};
void launch_depth_update(const DepthArgs& a, hipStream_t s);

struct PoseBAArgs {  // BundleAdjustment::optimizePose over a batch of frames (pose_ba.hip)
    const int32_t* feat_off;    // [n_frames + 1] feature range of each frame
    const double* bearing;      // [n_feat][3]
    const double* point;        // [n_feat][3] world position of the feature's point (any if none)
    const uint8_t* has_point;   // [n_feat]
    const uint8_t* vis_in;      // [n_feat] m_refVisibility before the call
    uint8_t* vis_out;           // [n_feat] after
    const double* poses;        // [n_frames][7]
    double* poses_out;          // [n_frames][7]
    double* err;                // [n_frames]
    int32_t* status;            // [n_frames]
    double* rows;               // scratch [3 * n_feat]
    double* wts;                // scratch [n_feat]
    int32_t n_frames;
};
void launch_pose_ba(const PoseBAArgs& a, hipStream_t s);

// FeatureSelection (feature_select.hip)
int feature_detect_segments(int64_t npx);
void launch_feature_detect(const uint8_t* plane, int width, int height, int thr, int* seg_counts, uint32_t* keys,
                           int* n_keys, hipStream_t s);
void launch_feature_cell_max(const uint8_t* plane, int width, int height, int cell, int grid_rows, int grid_cols,
                             const uint8_t* occupancy, int thr, uint32_t* cell_px, hipStream_t s);
}  // namespace svo

#include <vector>
namespace svo {
void feature_sort_keys(uint32_t* keys, int32_t n);
void feature_ssc(const int32_t* xs, const int32_t* ys, int32_t n, int32_t num_ret, float tolerance, int32_t cols,
                 int32_t rows, std::vector<int32_t>& out);
}  // namespace svo
