// svo_synth.cpp — deterministic synthetic KITTI-shaped frame pairs for benchmarks and parity tests.
//
// Scene: a piecewise-planar street — road, two walls, a far plane — textured with a
// seeded integer-hash value noise (3 octaves), rendered by ray/plane intersection with 2x2 box
// supersampling.  World frame = last keyframe camera (identity pose, like the first keyframe in the
// reference, src/frame.cpp:13).  Camera convention: x right, y down, z forward; poses are world->camera
// (Sophus params qx,qy,qz,qw,tx,ty,tz), as Frame::m_absPose (include/frame.hpp:198).
//
// Features: half on the reference frame, half on the last keyframe, at distinct pixels whose
// Simd-style abs-gradient exceeds 50 (config/config.json:21), >= h+3 px from the border, with a seeded
// sub-pixel offset.  bearing = normalise(K^-1 [u v 1]) (src/feature.cpp:14, src/pinhole_camera.cpp:84-100),
// point = ray/scene intersection.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(mix64(seed)) {}
    uint64_t next() { s = mix64(s); return s; }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
    double uniform(double a, double b) { return a + (b - a) * uniform(); }
};

static inline double lattice(uint64_t seed, int64_t ix, int64_t iy, int oct, int plane) {
    uint64_t h = mix64(seed ^ mix64((uint64_t)ix * 0x632BE59BD9B4E019ull ^ mix64((uint64_t)iy + 0x1234567ull) ^
                                    ((uint64_t)oct << 48) ^ ((uint64_t)plane << 56)));
    return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}
static inline double smooth(double t) { return t * t * (3.0 - 2.0 * t); }
static double value_noise(uint64_t seed, double x, double y, int oct, int plane) {
    const double fx = std::floor(x), fy = std::floor(y);
    const int64_t ix = (int64_t)fx, iy = (int64_t)fy;
    const double tx = smooth(x - fx), ty = smooth(y - fy);
    const double a = lattice(seed, ix, iy, oct, plane), b = lattice(seed, ix + 1, iy, oct, plane);
    const double c = lattice(seed, ix, iy + 1, oct, plane), d = lattice(seed, ix + 1, iy + 1, oct, plane);
    const double ab = a + (b - a) * tx, cd = c + (d - c) * tx;
    return ab + (cd - ab) * ty;
}

struct Scene {
    uint64_t seed;
    double road_y = 1.65, wall_l = -3.6, wall_r = 3.9, far_z = 60.0;
    double freq[4] = {2.2, 1.7, 1.7, 0.45};  // base texture frequency per plane (1/m)
    double contrast = 160.0;
    // returns distance along the ray (unit direction d) and intensity
    bool hit(const double C[3], const double d[3], double* s_out, int* plane_out, double* u, double* v) const {
        double best = 1e300;
        int pl = -1;
        auto test = [&](double num, double den, int id) {
            if (std::fabs(den) < 1e-12) return;
            double s = num / den;
            if (s > 1e-6 && s < best) { best = s; pl = id; }
        };
        test(road_y - C[1], d[1], 0);
        test(wall_l - C[0], d[0], 1);
        test(wall_r - C[0], d[0], 2);
        test(far_z - C[2], d[2], 3);
        if (pl < 0) return false;
        const double P[3] = {C[0] + best * d[0], C[1] + best * d[1], C[2] + best * d[2]};
        switch (pl) {
            case 0: *u = P[0]; *v = P[2]; break;
            case 1: case 2: *u = P[2]; *v = P[1]; break;
            default: *u = P[0]; *v = P[1]; break;
        }
        *s_out = best;
        *plane_out = pl;
        return true;
    }
    double shade(int pl, double u, double v) const {
        double acc = 0.0, amp = 1.0, norm = 0.0, f = freq[pl];
        for (int o = 0; o < 3; ++o) {
            acc += amp * value_noise(seed, u * f, v * f, o, pl);
            norm += amp;
            amp *= 0.55;
            f *= 2.3;
        }
        double t = acc / norm;                      // ~[0,1], centred near 0.5
        t = 0.5 + 2.6 * (t - 0.5);                  // contrast
        const double base = (pl == 0) ? 110.0 : (pl == 3 ? 150.0 : 125.0);
        const double val = base + contrast * (t - 0.5);
        return std::min(255.0, std::max(0.0, val));
    }
};

struct Pose {  // world -> camera: x_c = R x_w + t ;  R row-major
    double R[3][3], t[3];
};
static void rot_y(double deg, double R[3][3]) {
    const double a = deg * M_PI / 180.0, c = std::cos(a), s = std::sin(a);
    double M[3][3] = {{c, 0, s}, {0, 1, 0}, {-s, 0, c}};
    std::memcpy(R, M, sizeof(M));
}
static void matmul(const double A[3][3], const double B[3][3], double C[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}
// camera-to-world rotation Rwc and centre C  ->  world-to-camera pose
static Pose from_center(const double Rwc[3][3], const double C[3]) {
    Pose p;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) p.R[i][j] = Rwc[j][i];
    for (int i = 0; i < 3; ++i) p.t[i] = -(p.R[i][0] * C[0] + p.R[i][1] * C[1] + p.R[i][2] * C[2]);
    return p;
}
static void to_params(const Pose& p, double* out7) {  // rotation matrix -> unit quaternion (x,y,z,w)
    const double(*R)[3] = p.R;
    double tr = R[0][0] + R[1][1] + R[2][2], qw, qx, qy, qz;
    if (tr > 0) {
        double s = std::sqrt(tr + 1.0) * 2;
        qw = 0.25 * s; qx = (R[2][1] - R[1][2]) / s; qy = (R[0][2] - R[2][0]) / s; qz = (R[1][0] - R[0][1]) / s;
    } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
        double s = std::sqrt(1.0 + R[0][0] - R[1][1] - R[2][2]) * 2;
        qw = (R[2][1] - R[1][2]) / s; qx = 0.25 * s; qy = (R[0][1] + R[1][0]) / s; qz = (R[0][2] + R[2][0]) / s;
    } else if (R[1][1] > R[2][2]) {
        double s = std::sqrt(1.0 + R[1][1] - R[0][0] - R[2][2]) * 2;
        qw = (R[0][2] - R[2][0]) / s; qx = (R[0][1] + R[1][0]) / s; qy = 0.25 * s; qz = (R[1][2] + R[2][1]) / s;
    } else {
        double s = std::sqrt(1.0 + R[2][2] - R[0][0] - R[1][1]) * 2;
        qw = (R[1][0] - R[0][1]) / s; qx = (R[0][2] + R[2][0]) / s; qy = (R[1][2] + R[2][1]) / s; qz = 0.25 * s;
    }
    double n = std::sqrt(qx * qx + qy * qy + qz * qz + qw * qw);
    out7[0] = qx / n; out7[1] = qy / n; out7[2] = qz / n; out7[3] = qw / n;
    out7[4] = p.t[0]; out7[5] = p.t[1]; out7[6] = p.t[2];
}
// Rodrigues
static void axis_angle(const double w[3], double R[3][3]) {
    double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double I[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    if (th < 1e-15) { std::memcpy(R, I, sizeof(I)); return; }
    double k[3] = {w[0] / th, w[1] / th, w[2] / th};
    double K[3][3] = {{0, -k[2], k[1]}, {k[2], 0, -k[0]}, {-k[1], k[0], 0}};
    double K2[3][3];
    matmul(K, K, K2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = I[i][j] + std::sin(th) * K[i][j] + (1 - std::cos(th)) * K2[i][j];
}

struct Cam { int w, h; double fx, fy, cx, cy; };

static void render(const Scene& sc, const Cam& cam, const Pose& pose, uint8_t* img, int nthreads) {
    // camera centre and camera->world rotation
    double Rwc[3][3], C[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rwc[i][j] = pose.R[j][i];
    for (int i = 0; i < 3; ++i) C[i] = -(Rwc[i][0] * pose.t[0] + Rwc[i][1] * pose.t[1] + Rwc[i][2] * pose.t[2]);
    auto rows = [&](int y0, int y1) {
        for (int y = y0; y < y1; ++y)
            for (int x = 0; x < cam.w; ++x) {
                double acc = 0.0;
                for (int sy = 0; sy < 2; ++sy)
                    for (int sx = 0; sx < 2; ++sx) {
                        // pixel (x,y) integer centre convention: sample offsets +-0.25 around the centre
                        const double u = x - 0.25 + 0.5 * sx, v = y - 0.25 + 0.5 * sy;
                        double dc[3] = {(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, 1.0};
                        double n = std::sqrt(dc[0] * dc[0] + dc[1] * dc[1] + dc[2] * dc[2]);
                        double dw[3];
                        for (int i = 0; i < 3; ++i) dw[i] = (Rwc[i][0] * dc[0] + Rwc[i][1] * dc[1] + Rwc[i][2] * dc[2]) / n;
                        double s, tu, tv;
                        int pl;
                        if (sc.hit(C, dw, &s, &pl, &tu, &tv)) acc += sc.shade(pl, tu, tv);
                        else acc += 128.0;
                    }
                img[(size_t)y * cam.w + x] = (uint8_t)std::lround(std::min(255.0, std::max(0.0, acc * 0.25)));
            }
    };
    if (nthreads <= 1) { rows(0, cam.h); return; }
    std::vector<std::thread> th;
    const int chunk = (cam.h + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        int a = t * chunk, b = std::min(cam.h, a + chunk);
        if (a < b) th.emplace_back(rows, a, b);
    }
    for (auto& t : th) t.join();
}

static inline int grad_at(const uint8_t* im, int w, int x, int y) {
    int dx = std::abs((int)im[(size_t)y * w + x + 1] - (int)im[(size_t)y * w + x - 1]);
    int dy = std::abs((int)im[(size_t)(y + 1) * w + x] - (int)im[(size_t)(y - 1) * w + x]);
    return std::min(dx + dy, 255);
}

static int pick_features(const Scene& sc, const Cam& cam, const Pose& pose, const uint8_t* img, int count, int margin,
                         double null_frac, int cell, Rng& rng, double* px, double* bearing, double* point,
                         uint8_t* has_point) {
    std::vector<int> cand;
    for (int y = margin; y < cam.h - margin - 1; ++y)
        for (int x = margin; x < cam.w - margin - 1; ++x)
            if (grad_at(img, cam.w, x, y) > 50) cand.push_back(y * cam.w + x);
    if ((int)cand.size() < count) {  // low-texture fallback: any interior pixel
        cand.clear();
        for (int y = margin; y < cam.h - margin - 1; ++y)
            for (int x = margin; x < cam.w - margin - 1; ++x) cand.push_back(y * cam.w + x);
    }
    for (int i = 0; i < count && i < (int)cand.size(); ++i) {  // partial Fisher-Yates
        size_t j = i + (size_t)(rng.next() % (uint64_t)(cand.size() - i));
        std::swap(cand[i], cand[j]);
    }
    if (cell > 0) {  // the detector's emission order: grid cells row-major, then pixel index
        const int n = std::min(count, (int)cand.size()), cols = cam.w / cell + 1;
        auto key = [&](int p) { return (int64_t)((p / cam.w) / cell * cols + (p % cam.w) / cell) * cam.w * cam.h + p; };
        std::sort(cand.begin(), cand.begin() + n, [&](int a, int b) { return key(a) < key(b); });
    }
    double Rwc[3][3], C[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rwc[i][j] = pose.R[j][i];
    for (int i = 0; i < 3; ++i) C[i] = -(Rwc[i][0] * pose.t[0] + Rwc[i][1] * pose.t[1] + Rwc[i][2] * pose.t[2]);
    int n = std::min(count, (int)cand.size());
    for (int i = 0; i < n; ++i) {
        const double u = (cand[i] % cam.w) + rng.uniform(), v = (cand[i] / cam.w) + rng.uniform();
        px[2 * i] = u;
        px[2 * i + 1] = v;
        double b[3] = {(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, 1.0};
        const double nb = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
        for (int k = 0; k < 3; ++k) bearing[3 * i + k] = b[k] * (1.0 / nb);
        double dw[3];
        for (int k = 0; k < 3; ++k) dw[k] = Rwc[k][0] * bearing[3 * i] + Rwc[k][1] * bearing[3 * i + 1] + Rwc[k][2] * bearing[3 * i + 2];
        double s, tu, tv;
        int pl;
        if (!sc.hit(C, dw, &s, &pl, &tu, &tv)) s = 30.0;
        for (int k = 0; k < 3; ++k) point[3 * i + k] = C[k] + s * dw[k];
        has_point[i] = rng.uniform() < null_frac ? 0 : 1;
    }
    return n;
}

}  // namespace

extern "C" {

typedef struct {
    int32_t width, height;
    double fx, fy, cx, cy;
    int32_t n_features;        // total features: n/2 on the ref frame, n - n/2 on the last keyframe
    int32_t patch_size;        // border margin = patch/2 + 3
    double null_point_fraction;
    double init_trans_err;     // metres (default 0.02)
    double init_rot_err_deg;   // degrees (default 0.2)
    int32_t nthreads;
    int32_t cell_order;        // 0: features in shuffled order; c > 0: in the order FeatureSelection's
                               // bucketing emits them (src/feature_selection.cpp:103-141): c-px grid cells
                               // row by row (config "cell_pixel_size": 30), pixel order within a cell
} svo_synth_config;

void svo_synth_default_config(svo_synth_config* c) {
    c->width = 1241; c->height = 376;                                   // config/config.json:10-11
    c->fx = 721.5377; c->fy = 721.5377; c->cx = 609.5593; c->cy = 172.8540;  // resource/kitti.yaml:7-8
    c->n_features = 2000;
    c->patch_size = 5;
    c->null_point_fraction = 0.0;
    c->init_trans_err = 0.02;
    c->init_rot_err_deg = 0.2;
    c->nthreads = 1;
    c->cell_order = 0;
}

// Renders one (last keyframe, ref, cur) triple and its features.  Returns the number of features
// written (n_ref + n_kf).  Buffers: images width*height each; poses 7 doubles; feature arrays sized
// for c->n_features entries (px x2, bearing x3, point x3, has_point x1).
int32_t svo_synth_pair(const svo_synth_config* c, uint64_t seed, uint8_t* kf_img, uint8_t* ref_img, uint8_t* cur_img,
                       double* kf_pose, double* ref_pose, double* cur_true_pose, double* cur_init_pose, int32_t* n_ref,
                       int32_t* n_kf, double* px, double* bearing, double* point, uint8_t* has_point) {
    Rng rng(seed);
    Scene sc;
    sc.seed = mix64(seed * 31 + 7);
    sc.wall_l = -3.6 - 0.6 * rng.uniform();
    sc.wall_r = 3.9 + 0.6 * rng.uniform();
    Cam cam{c->width, c->height, c->fx, c->fy, c->cx, c->cy};
    // poses: lastKF = identity; ref = +0.8 m forward, 0.3 deg yaw; cur = +0.8 m more, another 0.3 deg
    const double step = 0.8 * (1.0 + 0.1 * (rng.uniform() - 0.5));
    const double yaw = 0.3 * (1.0 + 0.2 * (rng.uniform() - 0.5));
    double I3[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    double C0[3] = {0, 0, 0};
    Pose P_kf = from_center(I3, C0);
    double Rr[3][3];
    rot_y(yaw, Rr);
    double Cr[3] = {0, 0, step};
    Pose P_ref = from_center(Rr, Cr);
    double Rc[3][3];
    rot_y(2 * yaw, Rc);
    double Cc[3] = {Cr[0] + Rr[0][2] * step, Cr[1] + Rr[1][2] * step, Cr[2] + Rr[2][2] * step};
    Pose P_cur = from_center(Rc, Cc);
    // initial guess: true pose composed with a seeded perturbation (|t| = init_trans_err, |w| = init_rot_err)
    double dir[3], ax[3];
    for (int k = 0; k < 3; ++k) { dir[k] = rng.uniform(-1, 1); ax[k] = rng.uniform(-1, 1); }
    double nd = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    double na = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    double w[3];
    for (int k = 0; k < 3; ++k) w[k] = ax[k] / na * (c->init_rot_err_deg * M_PI / 180.0);
    double dR[3][3];
    axis_angle(w, dR);
    Pose P_init;
    matmul(dR, P_cur.R, P_init.R);
    for (int i = 0; i < 3; ++i)
        P_init.t[i] = dR[i][0] * P_cur.t[0] + dR[i][1] * P_cur.t[1] + dR[i][2] * P_cur.t[2] + dir[i] / nd * c->init_trans_err;

    const int nt = std::max(1, (int)c->nthreads);
    render(sc, cam, P_kf, kf_img, nt);
    render(sc, cam, P_ref, ref_img, nt);
    render(sc, cam, P_cur, cur_img, nt);
    to_params(P_kf, kf_pose);
    to_params(P_ref, ref_pose);
    to_params(P_cur, cur_true_pose);
    to_params(P_init, cur_init_pose);

    const int margin = c->patch_size / 2 + 3;
    const int want_ref = c->n_features / 2, want_kf = c->n_features - c->n_features / 2;
    int nr = pick_features(sc, cam, P_ref, ref_img, want_ref, margin, c->null_point_fraction, c->cell_order, rng, px, bearing, point, has_point);
    int nk = pick_features(sc, cam, P_kf, kf_img, want_kf, margin, c->null_point_fraction, c->cell_order, rng, px + 2 * nr, bearing + 3 * nr,
                           point + 3 * nr, has_point + nr);
    *n_ref = nr;
    *n_kf = nk;
    return nr + nk;
}

// Fraction of pixels with Simd-style abs-gradient > thr (texture calibration helper).
double svo_synth_gradient_fraction(const uint8_t* img, int32_t w, int32_t h, int32_t thr) {
    int64_t cnt = 0;
    for (int y = 1; y < h - 1; ++y)
        for (int x = 1; x < w - 1; ++x) cnt += grad_at(img, w, x, y) > thr;
    return (double)cnt / ((double)w * h);
}

}  // extern "C"
