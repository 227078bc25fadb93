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

struct PairDesc {  // per frame pair, device resident
    const uint8_t* ref_pyr;
    const uint8_t* kf_pyr;
    const uint8_t* cur_pyr;
    double ref_pose[7];
    double kf_pose[7];
    double cur_pose[7];
    int32_t n_ref, n_kf;
};

struct AlignArgs {
    const PairDesc* pairs;
    const double* px;         // [n_pairs*max_f][2]
    const double* bearing;    // [n_pairs*max_f][3]
    const double* point;      // [n_pairs*max_f][3]
    const uint8_t* has_point; // [n_pairs*max_f]
    double* xw;               // scratch [n_pairs*max_f][3]   world point per feature
    double* jimg;             // scratch [n_pairs*max_f][12]  image Jacobian at the current level
    double* cuv;              // scratch [n_pairs*max_f][2]   projection into cur at the current level
    uint8_t* fvis;            // scratch [n_pairs*max_f]      bit0 ref visible, bit1 cur visible
    double* fsum;             // scratch [n_pairs*max_f][5]   per-feature S_xx S_xy S_yy S_xr S_yr
    double* res;              // scratch [n_pairs][res_stride] residual per pixel slot (+inf = invisible)
    int64_t res_stride;       // >= max_f*area + 1, even (16-B aligned rows for the double2 sweeps)
    double* pose_out;         // [n_pairs][7]
    double* err_out;          // [n_pairs]
    int32_t* status_out;      // [n_pairs]
    svo_level_trace* traces;  // [n_pairs][max_level+1]
    unsigned long long* stamps;  // diagnostics: [n_pairs][max_level+1][8] s_memtime per phase, or null
    int32_t n_pairs, max_f, half, area, min_level, max_level;
    double fx, fy, cx, cy;
    LevelGeom geom;
};

void launch_align(const AlignArgs& a, hipStream_t s);
int align_window_bytes(int half);  // LDS staging bytes one wave needs for this half patch size
int align_window_capacity();       // LDS staging bytes available per wave
void launch_pyramid(uint8_t* stacks, const LevelGeom& g, int32_t first, int32_t count, hipStream_t s);

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

}  // namespace svo
