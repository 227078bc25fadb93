/*
 * svo_c.h — C ABI of the MI355X-native direct-alignment hot path (libsvo_hip.so).
 *
 * This is the drop-in boundary for amin-abouee/semi-direct-visual-odometry's sparse image alignment,
 * feature alignment and image pyramid.  The reference has no plugin registry or FFI: its boundary is
 * the C++ class surface.  Each entry point below names the reference interface it
 * replaces (paths relative to the reference root).  The C++ host mirror of that class surface
 * (semi-direct-visual-odometry_amd/host/svo.hpp) and the Python mirror (svo_amd) sit on top of it.
 *
 * Conventions
 *   - every function returns int: 0 = SVO_OK, < 0 = error (svo_last_error() has the message);
 *     no C++ exception crosses the ABI;
 *   - host buffers are caller-owned and only read/written during the call (or until the documented
 *     synchronisation point for *_run);
 *   - device memory is owned by the context; one context per (host thread, GPU); not reentrant;
 *   - poses are world->camera SE(3) in Sophus params() order: qx, qy, qz, qw, tx, ty, tz
 *     (Frame::m_absPose, include/frame.hpp:198);
 *   - images are 8-bit grey, row-major, tightly packed (cv::Mat CV_8UC1, continuous).
 */
#ifndef SVO_C_H
#define SVO_C_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVO_ABI_VERSION 2

enum {
    SVO_OK = 0,
    SVO_ERR_ARG = -1,    /* bad argument (null pointer, size out of range, bad index) */
    SVO_ERR_HIP = -2,    /* HIP runtime error */
    SVO_ERR_NODEV = -3,  /* no usable gfx950 device */
    SVO_ERR_STATE = -4   /* object used in the wrong state (e.g. results before run) */
};

/* Optimizer::Status values (include/optimizer.hpp:21-33) reported per alignment. */
enum {
    SVO_STATUS_SUCCESS = 0,
    SVO_STATUS_MAX_COFF_DX = 1,
    SVO_STATUS_NON_IN_DX = 2,
    SVO_STATUS_SMALL_STEP_SIZE = 3,
    SVO_STATUS_LAMBDA_VALUE = 4,
    SVO_STATUS_NORM_INF_DIFF = 5,
    SVO_STATUS_NON_SUFF_POINTS = 6,
    SVO_STATUS_INCREASE_CHI_SQUARED_ERROR = 7,
    SVO_STATUS_SMALL_CHI_SQUARED_ERROR = 8,
    SVO_STATUS_FAILED = 9
};

typedef struct svo_ctx svo_ctx;
typedef struct svo_pyramid_set svo_pyramid_set;
typedef struct svo_align_batch svo_align_batch;

/* PinholeCamera without distortion (src/pinhole_camera.cpp:50-101; KITTI d = 0, resource/kitti.yaml). */
typedef struct {
    double fx, fy, cx, cy;
    int32_t width, height;
} svo_camera;

/* Robust-scale semantics of the Tukey weights (Optimizer::tukeyWeighting, src/optimizer.cpp:485-514, with
 * algorithm::computeMedian / computeMAD, src/algorithm.cpp:834-865).
 *   SVO_MEDIAN_REFERENCE: the reference's own values: std::nth_element on the full residual vector and,
 *     for an even length, vec[n/2 - 1] as libstdc++'s introselect leaves it (not always the (n/2 - 1)-th
 *     order statistic): the device re-runs the introselect -- K2V (csrc/align_refv.hip, the vector in one
 *     CU's registers) whenever every pair of a launch holds at most svo_robust_scale_capacity(SVO_SCALE_K2V)
 *     slots, K2R (csrc/align_ref.hip, segments in LDS / global scratch) otherwise; the same bits either way;
 *   SVO_MEDIAN_EXACT: true order statistics ((n/2 - 1)-th and n/2-th), the robust statistic the
 *     reference means; faster (K2). */
enum { SVO_MEDIAN_EXACT = 0, SVO_MEDIAN_REFERENCE = 1 };
/* SVO_MEDIAN_REFERENCE: largest residual vector per pair (max_features * patch_size^2) */
#define SVO_REF_MAX_SLOTS 524288

/* ImageAlignment(patchSize, minLevel, maxLevel, numParameters=6) (include/image_alignment.hpp:18).
 * median_mode: SVO_MEDIAN_EXACT or SVO_MEDIAN_REFERENCE (above). */
typedef struct {
    int32_t patch_size;
    int32_t min_level;
    int32_t max_level;
    int32_t median_mode;
} svo_align_params;

/* Per pair, per pyramid level record of the single LM step (mirrors Optimizer state after
 * optimizeLM, src/optimizer.cpp:162-370).  H is the damped 6x6 (row-major), g the gradient. */
typedef struct {
    int32_t level, n_ref_vis, n_vis, status;
    double median, mad, sigma, chi2, lambda, err;
    double H[36], g[6], dx[6];
    int32_t scale_kernel; /* the device kernel that computed median / MAD at this level: SVO_SCALE_K2R,
                             SVO_SCALE_K2V or SVO_SCALE_K2 (exact mode); 0 if the level did not run */
    int32_t reserved;
} svo_level_trace;

/* ---------------------------------------------------------------- context */
int svo_device_count(int32_t* count);
int svo_ctx_create(int32_t device, svo_ctx** out);
int svo_ctx_destroy(svo_ctx* ctx);
int svo_ctx_synchronize(svo_ctx* ctx);
/* hipStream_t of the context (all work of the context is enqueued on it), for event timing. */
void* svo_ctx_stream(svo_ctx* ctx);
const char* svo_last_error(void);
int svo_abi_version(void);
/* hipEvent timing on the context stream: record event `slot` (0..15) now; elapsed ms between two
 * recorded slots (waits for the later one). */
int svo_ctx_event_record(svo_ctx* ctx, int32_t slot);
int svo_ctx_event_elapsed(svo_ctx* ctx, int32_t slot_begin, int32_t slot_end, float* ms);

/* ---------------------------------------------------------------- ImagePyramid
 * Replaces ImagePyramid::createImagePyramid (src/image_pyramid.cpp:36-52), called from the Frame
 * constructor (src/frame.cpp:26): per frame an intensity stack (level 0 = input, level l = pyrDown
 * of level l-1) and a gradient stack (level 0 = Simd::AbsGradientSaturatedSum, level l = pyrDown of
 * gradient l-1).  A set holds n_frames device-resident stacks of equal geometry, packed level after
 * level; level sizes are ((w+1)/2, (h+1)/2) per step (cv::pyrDown default). */
int svo_pyramid_set_create(svo_ctx* ctx, int32_t n_frames, int32_t width, int32_t height, int32_t levels,
                           svo_pyramid_set** out);
int svo_pyramid_set_destroy(svo_pyramid_set* set);
/* Copy `count` base images (count*width*height bytes) into frames [first, first+count). Async. */
int svo_pyramid_set_upload(svo_pyramid_set* set, int32_t first, int32_t count, const uint8_t* host_images);
/* Same, from device memory (e.g. a decoder's output), stream-ordered. */
int svo_pyramid_set_upload_device(svo_pyramid_set* set, int32_t first, int32_t count, const uint8_t* dev_images);
/* Build both stacks for frames [first, first+count) on the device.  Async (context stream). */
int svo_pyramid_set_build(svo_pyramid_set* set, int32_t first, int32_t count);
/* The same build on the context's prep stream, after everything queued on the context stream so far, so that it
 * overlaps work queued later (the next batch's pyramids building while the current batch aligns:
 * src/frame.cpp:26 -> src/image_pyramid.cpp:36-52 for the frames of the next call).  Every later use of the set's
 * planes through this ABI (upload, build, download, svo_align_batch_set_pair / set_pairs) waits for it. */
int svo_pyramid_set_build_async(svo_pyramid_set* set, int32_t first, int32_t count);
/* ImagePyramid::getImageAtLevel / getGradientAtLevel (src/image_pyramid.cpp:54-124): copy one level
 * to the host (synchronous).  gradient = 0 for the intensity stack, 1 for the gradient stack. */
int svo_pyramid_set_download(const svo_pyramid_set* set, int32_t frame, int32_t level, int32_t gradient, uint8_t* out);
/* ImagePyramid::getImageSizeAtLevel (src/image_pyramid.cpp:110-116). */
int svo_pyramid_level_size(const svo_pyramid_set* set, int32_t level, int32_t* width, int32_t* height);

/* ---------------------------------------------------------------- ImageAlignment
 * Replaces ImageAlignment::align(refFrame, curFrame) (src/image_alignment.cpp:25-67, declared
 * include/image_alignment.hpp:25; called src/system.cpp:313).  A batch holds n_pairs independent
 * (ref, ref->lastKeyframe, cur) problems; each is the reference's whole coarse-to-fine call:
 * for level = max..min: Jacobian of the ref patches, one Tukey-weighted Nielsen-damped LM step,
 * pose <- pose * exp(-dx).  Features are the ref frame's, then the last keyframe's, in vector order
 * (slots exist for features without a point, src/image_alignment.cpp:81-121). */
int svo_align_batch_create(svo_ctx* ctx, const svo_camera* cam, const svo_align_params* params, int32_t n_pairs,
                           int32_t max_features, svo_align_batch** out);
int svo_align_batch_destroy(svo_align_batch* batch);
/* Describe pair `pair`: each frame is (pyramid set, frame index); the sets must outlive the batch's runs.
 *   px       (n_ref+n_kf) x 2   Feature::m_pixelPosition at level 0 (include/feature.hpp:31)
 *   bearing  (n_ref+n_kf) x 3   Feature::m_bearingVec (include/feature.hpp:33-34)
 *   point    (n_ref+n_kf) x 3   Point::m_position in world coordinates (include/point.hpp:28)
 *   has_point(n_ref+n_kf)       Feature::m_point != nullptr
 * The host arrays are consumed on return (copied into the context's pinned staging ring, or read
 * directly for pairs too large for it); the device copies are stream-ordered before any later work on
 * the context stream and are not waited for.  A copy that fails after this call returned is reported
 * by a later call on the context (the next run, results or pinned-memory user). */
int svo_align_batch_set_pair(svo_align_batch* batch, int32_t pair, const svo_pyramid_set* ref_set, int32_t ref_frame,
                             const svo_pyramid_set* kf_set, int32_t kf_frame, const svo_pyramid_set* cur_set,
                             int32_t cur_frame, const double* ref_pose, const double* kf_pose,
                             const double* cur_pose, int32_t n_ref, int32_t n_kf, const double* px,
                             const double* bearing, const double* point, const uint8_t* has_point);
/* Describe pairs [first, first + count) in one call (the bulk form of svo_align_batch_set_pair): one copy
 * per array for all of them, then a device scatter into the pairs' feature slots.
 *   frames   count x 3   frame indices (ref, kf, cur) in ref_set / kf_set / cur_set
 *   poses    count x 21  ref, kf, cur poses (7 each, as set_pair)
 *   n_feat   count x 2   n_ref, n_kf
 *   px, bearing, point, has_point: the pairs' feature rows packed pair after pair (pair i's rows start at
 *   the sum of the earlier pairs' n_ref + n_kf), layouts as set_pair.  With features_on_device != 0 they
 *   are device pointers on the context's device (e.g. FeatureSelection output), else host memory.
 * Every host array is consumed on return; the upload runs on a copy stream of the context (overlapping
 * earlier work queued there, e.g. a pyramid build) and the scatter is queued on the context stream,
 * ordered before any later work on it.  With features_on_device the call also waits for the scatter, so
 * the device arrays may be reused on return. */
int svo_align_batch_set_pairs(svo_align_batch* batch, int32_t first, int32_t count, const svo_pyramid_set* ref_set,
                              const svo_pyramid_set* kf_set, const svo_pyramid_set* cur_set, const int32_t* frames,
                              const double* poses, const int32_t* n_feat, const double* px, const double* bearing,
                              const double* point, const uint8_t* has_point, int32_t features_on_device);
/* Replace the initial cur poses of all pairs (n_pairs x 7).  Synchronous H2D. */
int svo_align_batch_set_initial_poses(svo_align_batch* batch, const double* poses);
/* Run every pair.  Asynchronous on the context stream; inputs stay untouched, so repeated runs are
 * identical (the result pose is written to a separate device buffer).  A large reference-mode batch runs as
 * sub-batch chains on the context's side streams; back-to-back runs of the same batch are ordered per chain (each
 * chain touches only its own pairs), and every other call that uses the context (results, traces, set_pair(s),
 * pyramid uploads / builds, FeatureAlignment, events, synchronize, destroy) first waits for all of them. */
int svo_align_batch_run(svo_align_batch* batch);
/* One run with a hipEvent between consecutive kernel launches (diagnostics; synchronous).  stage_ms[5]
 * receives the device time per stage summed over the levels: [0] world points + state, [1] residuals,
 * [2] robust scale, [3] weights + normal equations, [4] LM step.  No reference counterpart. */
int svo_align_batch_profile(svo_align_batch* batch, float* stage_ms);
/* Wait for the last run and copy results: poses n_pairs x 7 (the aligned cur->m_absPose), err
 * n_pairs (the RMSE of the finest level, as align() returns), status n_pairs (Optimizer::Status of
 * the finest level).  Any pointer may be NULL. */
int svo_align_batch_results(svo_align_batch* batch, double* poses, double* err, int32_t* status);
/* Per-level records of one pair (max_level+1 entries, indexed by level). */
int svo_align_batch_traces(svo_align_batch* batch, int32_t pair, svo_level_trace* out);

/* Device forms of the reference robust scale (SVO_MEDIAN_REFERENCE): K2V keeps the residual vector in
 * registers (vectors of <= 60 416 slots, 2416 features at patch 5; the faster of its two register layouts up
 * to 50 176 slots, config 2's 2000 features x 25), K2R runs its large rounds through global scratch (any size).
 * Both give the same bits. */
enum { SVO_SCALE_AUTO = 0, SVO_SCALE_K2R = 1, SVO_SCALE_K2V = 2, SVO_SCALE_K2 = 3 /* exact mode (trace only) */ };

/* Diagnostics (no reference counterpart): the SVO_MEDIAN_REFERENCE robust scale of an arbitrary residual
 * vector, i.e. algorithm::computeMAD(values, n_valid) (src/algorithm.cpp:855-865) and the median it uses, on
 * the device, with the kernel `impl` (SVO_SCALE_*; AUTO picks K2V where the vector fits).  values: n_slots
 * doubles, none NaN (an invisible slot is DBL_MAX).  out[0] = median, out[1] = MAD, then as many diagnostics
 * as out_len allows (out_len >= 2):
 *   K2V: [2 + 5p ..] per pass p: cycles, block rounds, one-wave rounds, heap select, chunked exchanges;
 *   K2R: with the environment variable SVO_DEBUG_STAMPS set, [2..9] cycles / block rounds / one-wave rounds
 *        / heap select per pass, [10..189] the block rounds, [190..205] cycles per round phase
 *        (tools/k2r_probe.py).
 * K2V with out_len > 206: out[206..] receives a round trace (development): per round 8 header doubles (pass + 10
 * kind, f, l, pivot, Ks, #GE, #LE, cut) and the vector's n_slots values after the round.
 * K2V with out_len == 2: no diagnostics; the vector runs through the product kernel's own code path (its layouts
 * and one-wave size), whereas the diagnostics kernel hands segments of <= 1024 positions to wave 0.
 * Synchronous.  SVO_ERR_ARG if impl is K2V and the vector does not fit it. */
int svo_debug_robust_scale(svo_ctx* ctx, const double* values, int64_t n_slots, int64_t n_valid, int32_t impl,
                           double* out, int64_t out_len);
/* The largest residual vector (slots = features x patch^2) the robust-scale kernel `impl` (SVO_SCALE_K2V or
 * SVO_SCALE_K2R) takes.  A reference-mode launch runs K2V when every pair's vector fits it, K2R otherwise. */
int svo_robust_scale_capacity(int32_t impl, int64_t* slots);

/* ---------------------------------------------------------------- FeatureAlignment
 * Replaces FeatureAlignment::align(refFeature, curFrame, pixelPos) (src/feature_alignment.cpp:25-62,
 * declared include/feature_alignment.hpp:25; called src/map.cpp:538,608) for n candidates at once:
 * 2-D translation + intensity bias on the level-0 GRADIENT images of the ref and cur frames, one
 * LM step, pixelPos <- flow.xy.  Candidate i's reference feature lives in frame ref_frames[i]
 * (refFeature->m_frame; NULL = every candidate in ref_frame) at ref_px[i] (its m_pixelPosition).
 * px_inout: n x 2 (initial pixel positions in, aligned out); err: the returned RMSE (NaN when the
 * patch left the frame); status: Optimizer::Status.  Synchronous. */
int svo_feature_align(svo_ctx* ctx, const svo_camera* cam, int32_t patch_size, const svo_pyramid_set* ref_set,
                      const int32_t* ref_frames, int32_t ref_frame, const svo_pyramid_set* cur_set, int32_t cur_frame,
                      int32_t n, const double* ref_px, double* px_inout, double* err, int32_t* status);

/* As svo_feature_align, with each candidate's reference frame in a pyramid set of its own:
 * candidate i reads ref_sets[i] frame ref_frames[i] (the batched call Map::reprojectCell and
 * Map::addCandidateToFrame make: their candidates come from different keyframes). */
int svo_feature_align_multi(svo_ctx* ctx, const svo_camera* cam, int32_t patch_size, const svo_pyramid_set* const* ref_sets,
                            const int32_t* ref_frames, const svo_pyramid_set* cur_set, int32_t cur_frame, int32_t n,
                            const double* ref_px, double* px_inout, double* err, int32_t* status);

/* ---------------------------------------------------------------- map reprojection (host side)
 * Frame::world2image (src/frame.cpp:83-92): px[i] = project2d(pose * points[i]) for n points (n x 3). */
int svo_world2image(const svo_camera* cam, const double* pose, int32_t n, const double* points, double* px);

/* The decisions of Map::reprojectMap (src/map.cpp:260-267, 436-478) with reprojectPoint (:481-492) and
 * reprojectCell (:495-570), before any FeatureAlignment: the reference accepts the aligned position of
 * the first non-deleted candidate of a cell whatever its error, so which candidates are aligned is fixed
 * by the geometry alone and the alignments can run as one batch (svo_feature_align_multi).
 * Grid: cell_size-pixel cells, n_cells = ceil(W / c) * ceil(H / c), visited in cell_order (the
 * reference shuffles it with an unseeded std::random_device; callers pass a seeded permutation).
 * Keyframes k < n_kf (ref frame, then its last keyframe) own features kf_feat_off[k] .. kf_feat_off[k+1]-1;
 * feat_point[f] is the feature's point (-1: none).  Points: position (n_points x 3), type
 * (Point::PointType: 0 GOOD, 1 DELETED, 2 CANDIDATE, 3 UNKNOWN), point_last = m_lastProjectedKFId
 * (updated: set to cur_id for every point projected).  Out: overlap[k] points of keyframe k in the
 * frame; the selected candidates in acceptance order (sel_feat, sel_cell, sel_px = the initial
 * pixel for the alignment; capacity n_cells); matches (m_matches) and trials (m_trials).  The caller
 * applies the per-candidate effects (:558-569): succeededProjection += 1, UNKNOWN -> GOOD past 10, a new
 * feature at the aligned pixel, and marks sel_cell visited. */
int svo_map_reproject_plan(const svo_camera* cam, int32_t cell_size, int32_t n_cells, const int32_t* cell_order,
                           const double* cur_pose, uint64_t cur_id, int32_t n_kf, const int32_t* kf_feat_off,
                           const int32_t* feat_point, int32_t n_points, const double* point_pos,
                           const uint32_t* point_type, uint64_t* point_last, int32_t* overlap, int32_t* n_sel,
                           int32_t* sel_feat, int32_t* sel_cell, double* sel_px, int32_t* matches, int32_t* trials);

/* ---------------------------------------------------------------- depth filter
 * One depth-filter seed: MixedGaussianFilter (include/mixed_gaussian_filter.hpp:28-38) and the feature
 * it refines (m_feature: pixel position and bearing in its keyframe). */
typedef struct {
    double a, b, mu, sigma, var, max_depth; /* Beta(a, b) inlier ratio; inverse-depth N(mu, var); 1 / depthMin */
    double px[2];                           /* m_feature->m_pixelPosition (keyframe, level 0) */
    double bearing[3];                      /* m_feature->m_bearingVec */
    int32_t kf;                             /* keyframe of m_feature->m_frame: index into the call's keyframe table */
    int32_t valid;                          /* m_validity */
} svo_depth_seed;

/* Outcome of one seed in svo_depth_update (no reference counterpart; the reference only logs it). */
enum {
    SVO_DEPTH_REJECTED = 0,  /* point behind / outside the current image: seed invalid (src/depth_estimator.cpp:229-237) */
    SVO_DEPTH_NO_MATCH = 1,  /* epipolar search failed: b += 1 (:252-258) */
    SVO_DEPTH_UPDATED = 2,   /* Gaussian x Beta update (:261-266) */
    SVO_DEPTH_CONVERGED = 3, /* sqrt(var) * 10 < max_depth: candidate point emitted, seed invalid (:281-291) */
    SVO_DEPTH_NAN = 4        /* inverse depth NaN: seed invalid (:292-297) */
};

/* MixedGaussianFilter(feature, depthMean, depthMin) (src/mixed_gaussian_filter.cpp:7-24): initial state
 * of a seed (px, bearing, kf are the caller's; valid = 1).  Host only. */
int svo_depth_seed_init(double depth_mean, double depth_min, svo_depth_seed* seed);

/* Replaces DepthEstimator::updateFilters(frame) (src/depth_estimator.cpp:192-309, with
 * algorithm::matchEpipolarConstraint src/algorithm.cpp:412-551, computeTau :342-357, updateFilter
 * :311-340): every seed against the current frame, then the reference's stable remove_if of invalid
 * seeds.  Keyframe k of the table is frame kf_frames[k] of kf_sets[k] (its level-0 intensity image) with
 * pose kf_poses[7k..7k+6]; the current frame is cur_frame of cur_set with pose cur_pose (Sophus params).
 *   seeds_inout   n_seeds in; the n_seeds_out survivors out (order kept)
 *   outcome       n_seeds (per input seed, SVO_DEPTH_*), may be NULL
 *   cand_points   n_seeds x 3 capacity: world points of the converged seeds (m_map->addNewCandidate),
 *   cand_seed     n_seeds capacity: their input seed index; both in the reference's loop order
 *                 (seeds visited from the last to the first); *n_cand entries.
 * Synchronous. */
int svo_depth_update(svo_ctx* ctx, const svo_camera* cam, int32_t n_kf, const svo_pyramid_set* const* kf_sets,
                     const int32_t* kf_frames, const double* kf_poses, const svo_pyramid_set* cur_set,
                     int32_t cur_frame, const double* cur_pose, int32_t n_seeds, svo_depth_seed* seeds_inout,
                     int32_t* n_seeds_out, int32_t* outcome, double* cand_points, int32_t* cand_seed,
                     int32_t* n_cand);

/* ---------------------------------------------------------------- FeatureSelection
 * Replaces FeatureSelection (src/feature_selection.cpp:19-287; constructed src/system.cpp:28 with the
 * image size and cell_pixel_size, called :81, :252-254, :428-430).  Its bool occupancy grid of
 * (height / cell_size + 1) rows x (width / cell_size + 1) columns (:19-25) is caller-owned bytes here
 * (`occupancy`, row-major, 1 = occupied): setExistingFeatures / setCellInGridOccupancy (:268-282) mark
 * it, the bucketing branches clear it on return (resetGridOccupancy, :75, :141).  The gradient magnitude
 * is the frame's level-0 gradient plane (computeImageGradient :250-266 is the same
 * Simd::AbsGradientSaturatedSum as the pyramid's); the orientation is 0 everywhere (:261).  Output
 * features are in Frame::addFeature order: pixel (x, y) and response = gradient magnitude. */
int svo_feature_grid_size(int32_t width, int32_t height, int32_t cell_size, int32_t* rows, int32_t* cols);
/* Device step of gradientMagnitudeWithSSC (:38-50): the level-0 gradient pixels of `frame` above
 * `threshold` in row-major order, as keys (response << 24 | y * width + x; width * height <= 2^24).
 * keys: capacity entries.  Synchronous. */
int svo_feature_detect(svo_ctx* ctx, const svo_pyramid_set* set, int32_t frame, int32_t threshold, int32_t capacity,
                       uint32_t* keys, int32_t* n_keys);
/* gradientMagnitudeWithSSC(frame, detectionThreshold, numberCandidate, useBucketing) (:27-89): device
 * detection, then std::sort by response (reference comparator) and SSC (:166-248, tolerance 0.1) on the
 * host.  n_keypoints (may be NULL): keypoints above the threshold.  Synchronous. */
int svo_feature_select_ssc(svo_ctx* ctx, const svo_pyramid_set* set, int32_t frame, int32_t threshold,
                           int32_t number_candidate, int32_t use_bucketing, int32_t cell_size, uint8_t* occupancy,
                           int32_t capacity, double* px_out, double* response_out, int32_t* n_out, int32_t* n_keypoints);
/* gradientMagnitudeByValue(frame, detectionThreshold, useBucketing = true) (:91-143): per free cell the
 * first maximum in row-major order, kept if above the threshold; cells in row-major order.  The
 * reference's useBucketing = false branch reads the 8-bit magnitude as float (:150) and is rejected.
 * Synchronous. */
int svo_feature_select_by_value(svo_ctx* ctx, const svo_pyramid_set* set, int32_t frame, int32_t threshold,
                                int32_t cell_size, uint8_t* occupancy, int32_t capacity, double* px_out,
                                double* response_out, int32_t* n_out);

/* ---------------------------------------------------------------- trajectory output (host only)
 * System::writeInFile (src/system.cpp:635-640, called per image from src/main.cpp:114-121): the ref
 * frame's camera->world pose m_absPose.inverse().matrix3x4() (Sophus) as one KITTI trajectory line.
 * out12: that 3x4 matrix, row-major. */
int svo_pose_matrix3x4_inverse(const double* pose, double* out12);
/* The same line as text: the 12 numbers row-major, single spaces, each as an std::ostream with
 * precision 6 prints a double ("%.6g"; Eigen IOFormat utils::eigenFormatIO, src/utils.cpp:10-13), NUL
 * terminated, no newline.  cap: bytes of buf (>= 12 * 14 is always enough). */
int svo_format_kitti_pose(const double* pose, char* buf, int32_t cap);

/* ---------------------------------------------------------------- pose-only bundle adjustment
 * Replaces BundleAdjustment::optimizePose(frame) (src/bundle_adjustment.cpp:35-69; BundleAdjustment(camera,
 * 0, 6) constructed src/system.cpp:31, the call itself is commented out at :388) for n_frames independent
 * frames: one LM step of Optimizer::optimizeLM<SE3d> on |bearing - normalise(T * P)| (three rows per
 * feature, only the third visible), pose <- exp(dx) * pose.  Frame f owns features feat_off[f] ..
 * feat_off[f+1]-1: bearing (x3), point (x3, the feature's m_point->m_position), has_point (m_point != null).
 * vis_inout is m_refVisibility of the BundleAdjustment object that optimises the frame, resized to the
 * frame's feature count (new entries 0): the residual step reads the flags the PREVIOUS call left (the
 * reference calls the residual functor before the Jacobian functor, src/optimizer.cpp:199 vs :242), so a
 * fresh object returns NaN and leaves the pose as exp(0) * pose; on return the flags are has_point.
 * poses_inout n_frames x 7; err: the returned RMSE (0 when the frame has no features, -1 on
 * Non_Suff_Points); status: Optimizer::Status, -1 when nothing ran (no features).  A stale flag on a
 * feature without a point (the reference dereferences null) is SVO_ERR_ARG.  Synchronous. */
int svo_pose_optimize(svo_ctx* ctx, int32_t n_frames, const int32_t* feat_off, const double* bearing,
                      const double* point, const uint8_t* has_point, uint8_t* vis_inout, double* poses_inout,
                      double* err, int32_t* status);

#ifdef __cplusplus
}
#endif

#endif /* SVO_C_H */
