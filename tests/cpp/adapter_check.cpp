// adapter_check.cpp -- drives the compiled INTEGRATION.md adapter (tests/cpp/adapter.cpp) like the reference's
// callers do: Frame construction builds the pyramid (src/frame.cpp:26), System::trackFrame calls
// ImageAlignment::align (src/system.cpp:313), Map calls FeatureAlignment::align (src/map.cpp:538).  Test
// infrastructure for tests/test_adapter.py.
//   adapter_check <input.bin> run|fail
// input.bin: int32 W H levels patch min_level max_level; double fx fy cx cy; 3 images (ref, lastKF, cur) of W*H
// bytes; double poses ref[7] kf[7] cur[7]; int32 n_ref n_kf; double px[2n] bearing[3n] point[3n]; uint8 has[n];
// int32 n_fa; double fa_ref_px[2 n_fa] fa_init[2 n_fa] (FeatureAlignment(7) from the ref frame into cur).
// `fail` makes the adapter's context on a device index that does not exist first.
// Output lines: "err <v>", "pose <7 values>", "unchanged <0|1>" (the pose bits after vs before), "again <0|1>"
// (a second align from the same start gives the same bits), "fa <i> <x> <y> <err>", and the ref frame's pyramid
// through the ImagePyramid getters ("pyr", "lvl", "all" lines, see below).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

#include "ref_types.hpp"

template <class T>
static bool rd(std::ifstream& f, T* p, size_t n) {
    return (bool)f.read(reinterpret_cast<char*>(p), (std::streamsize)(n * sizeof(T)));
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    std::ifstream f(argv[1], std::ios::binary);
    int32_t hdr[6];
    double K[4];
    if (!rd(f, hdr, 6) || !rd(f, K, 4)) return 3;
    const int32_t W = hdr[0], H = hdr[1], levels = hdr[2], patch = hdr[3], minL = hdr[4], maxL = hdr[5];
    if (std::string(argv[2]) == "fail") g_svo_device = 1 << 20;
    auto cam = std::make_shared<PinholeCamera>(K[0], K[1], K[2], K[3], W, H);
    cv::Mat img[3];
    for (auto& m : img) {
        m.rows = H;
        m.cols = W;
        m.buf.resize((size_t)W * H);
        if (!rd(f, m.buf.data(), m.buf.size())) return 3;
    }
    double poses[21];
    int32_t nn[2];
    if (!rd(f, poses, 21) || !rd(f, nn, 2)) return 3;
    const int32_t n = nn[0] + nn[1];
    std::vector<double> px(2 * n), br(3 * n), pt(3 * n);
    std::vector<uint8_t> hp(n);
    if (!rd(f, px.data(), px.size()) || !rd(f, br.data(), br.size()) || !rd(f, pt.data(), pt.size()) ||
        !rd(f, hp.data(), hp.size()))
        return 3;
    int32_t nfa = 0;
    if (!rd(f, &nfa, 1)) return 3;
    std::vector<double> fref(2 * nfa), finit(2 * nfa);
    if (!rd(f, fref.data(), fref.size()) || !rd(f, finit.data(), finit.size())) return 3;

    auto ref = std::make_shared<Frame>(cam), kf = std::make_shared<Frame>(cam), cur = std::make_shared<Frame>(cam);
    std::shared_ptr<Frame> fr3[3] = {ref, kf, cur};
    for (int i = 0; i < 3; ++i) {
        fr3[i]->m_imagePyramid.createImagePyramid(img[i], (size_t)levels);   // src/frame.cpp:26
        std::memcpy(fr3[i]->m_absPose.data(), poses + 7 * i, 7 * sizeof(double));
    }
    ref->m_lastKeyframe = kf;
    cur->m_lastKeyframe = kf;
    for (int32_t i = 0; i < n; ++i) {
        auto ft = std::make_shared<Feature>();
        ft->m_frame = i < nn[0] ? ref : kf;
        ft->m_pixelPosition = {px[2 * i], px[2 * i + 1]};
        ft->m_bearingVec = {br[3 * i], br[3 * i + 1], br[3 * i + 2]};
        if (hp[i]) {
            ft->m_point = std::make_shared<Point>();
            ft->m_point->m_position = {pt[3 * i], pt[3 * i + 1], pt[3 * i + 2]};
        }
        ft->m_frame->m_features.push_back(ft);
    }
    // the pyramid getters (include/image_pyramid.hpp:75-140) on the ref frame, one level past the last included:
    // "pyr <levels> <base w> <base h>", then per level "lvl <l> <w> <h> <rows> <cols> <fnv1a(image)> <fnv1a(gradient)>"
    {
        const ImagePyramid& pyr = ref->m_imagePyramid;
        auto fnv = [](const cv::Mat& m) {
            uint64_t x = 1469598103934665603ull;
            for (uint8_t b : m.buf) x = (x ^ b) * 1099511628211ull;
            return (unsigned long long)x;
        };
        const cv::Size b = pyr.getBaseImageSize();
        std::printf("pyr %zu %d %d\n", pyr.getSizeImagePyramid(), b.width, b.height);
        for (int32_t l = 0; l <= levels; ++l) {
            const cv::Size sz = pyr.getImageSizeAtLevel((size_t)l);
            const cv::Mat& im = pyr.getImageAtLevel((size_t)l);
            const cv::Mat& gr = pyr.getGradientAtLevel((size_t)l);
            std::printf("lvl %d %d %d %d %d %llu %llu\n", l, sz.width, sz.height, im.rows, im.cols, fnv(im), fnv(gr));
        }
        const std::vector<cv::Mat>& all = pyr.getAllImages();
        const bool base_ok = fnv(pyr.getBaseImage()) == fnv(pyr.getImageAtLevel(0)) &&
                             fnv(pyr.getBaseGradientImage()) == fnv(pyr.getGradientAtLevel(0));
        std::printf("all %zu %d\n", all.size(), base_ok ? 1 : 0);
    }
    ImageAlignment ia((uint32_t)patch, minL, maxL, 6);
    const Sophus::SE3d before = cur->m_absPose;
    const double err = ia.align(ref, cur);
    const Sophus::SE3d after = cur->m_absPose;
    std::printf("err %.17g\npose", err);
    for (double v : after.p) std::printf(" %.17g", v);
    std::printf("\nunchanged %d\n", std::memcmp(before.p, after.p, sizeof before.p) == 0 ? 1 : 0);
    cur->m_absPose = before;
    const double err2 = ia.align(ref, cur);
    std::printf("again %d\n", (std::memcmp(cur->m_absPose.p, after.p, sizeof after.p) == 0 &&
                               (err2 == err || (err2 != err2 && err != err))) ? 1 : 0);
    FeatureAlignment fa(7, 0, 3);
    for (int32_t i = 0; i < nfa; ++i) {
        auto rf = std::make_shared<Feature>();
        rf->m_frame = ref;
        rf->m_pixelPosition = {fref[2 * i], fref[2 * i + 1]};
        Eigen::Vector2d p(finit[2 * i], finit[2 * i + 1]);
        const double e = fa.align(rf, cur, p);
        std::printf("fa %d %.17g %.17g %.17g\n", i, p.x(), p.y(), e);
    }
    return 0;
}
