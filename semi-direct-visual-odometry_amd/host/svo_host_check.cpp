// svo_host_check.cpp — drives the C++ class-surface mirror (host/svo.hpp, libsvo_host.so) from the tests.
//   svo_host_check io              poses on stdin (7 numbers a line, Sophus params) -> utils::writeInFile lines
//   svo_host_check fs W H CELL THR NUM BUCKET IMAGE.raw [EX EY]...
//                                  FeatureSelection::gradientMagnitudeWithSSC on a raw 8-bit image (GPU);
//                                  existing features (EX, EY) marked first; prints "x y response" per feature
//   svo_host_check fv W H CELL THR IMAGE.raw    gradientMagnitudeByValue (bucketing)
//   svo_host_check ba N DATA.bin   BundleAdjustment::optimizePose twice on one object (GPU); DATA.bin:
//                                  pose[7], then per feature bearing[3] point[3] has_point (as a double);
//                                  prints "err status qx qy qz qw tx ty tz" per call
//   svo_host_check depth DATA.bin KF.raw CUR.raw   DepthEstimator addKeyframe + updateFilters (GPU);
//                                  DATA.bin: fx fy cx cy W H, kf pose[7], cur pose[7], depth_mean, depth_min,
//                                  n, then n x (px[2] bearing[3]) as doubles; prints "filters M", then one
//                                  "cand X Y Z" line per candidate
//   svo_host_check map DATA.bin REF.raw KF.raw CUR.raw   Map::reprojectMap + addCandidateToFrame (GPU);
//                                  DATA.bin (doubles): fx fy cx cy W H cell, ref/kf/cur pose[7], n_ref n_kf
//                                  n_points n_cand n_cells, feat_px[2n], feat_point[n], point_pos[3p],
//                                  point_type[p], point_succ[p], cand_feat[c], cand_pos[3c], cell_order;
//                                  prints "counts matches trials", then "px X Y" per new cur feature;
//                                  an optional REPS argument also times REPS more runs on fresh object
//                                  graphs ("ms T": reprojectMap + addCandidateToFrame, average)
//   svo_host_check align DATA.bin REF.raw KF.raw CUR.raw PATCH MINL MAXL MEDIAN
//                                  ImageAlignment::align (GPU) twice on one object from the same initial
//                                  cur pose (the second call reuses the object's batch); DATA.bin (doubles):
//                                  fx fy cx cy W H, ref/kf/cur pose[7], n_ref n_kf, then per feature
//                                  px[2] bearing[3] point[3] has_point; prints "err status pose[7]" per call
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <memory>
#include <string>
#include <vector>

#include "svo.hpp"

using namespace svo_amd;

static std::vector<uint8_t> read_raw(const char* path, size_t n) {
    std::ifstream f(path, std::ios::binary);
    std::vector<uint8_t> v((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (v.size() != n) throw std::runtime_error("image size mismatch");
    return v;
}

int main(int argc, char** argv) {
    try {
        const std::string mode = argc > 1 ? argv[1] : "";
        if (mode == "io") {
            Pose p;
            while (std::cin >> p[0] >> p[1] >> p[2] >> p[3] >> p[4] >> p[5] >> p[6]) utils::writeInFile(p, std::cout);
            return 0;
        }
        if ((mode == "fs" && argc >= 9) || (mode == "fv" && argc >= 7)) {
            const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), cell = std::atoi(argv[4]), thr = std::atoi(argv[5]);
            const char* img_path = mode == "fs" ? argv[8] : argv[6];
            const std::vector<uint8_t> img = read_raw(img_path, (size_t)w * h);
            Context ctx(0);
            auto cam = std::make_shared<PinholeCamera>(PinholeCamera{w, h, 300.0, 300.0, w / 2.0, h / 2.0});
            auto frame = std::make_shared<Frame>(ctx, cam, img.data(), 1);
            FeatureSelection sel(ctx, w, h, cell);
            std::vector<std::shared_ptr<Feature>> existing;
            if (mode == "fs")
                for (int i = 9; i + 1 < argc; i += 2)
                    existing.push_back(std::make_shared<Feature>(frame.get(), Vec2{std::atof(argv[i]), std::atof(argv[i + 1])}));
            auto run = [&]() {
                frame->m_features.clear();
                sel.resetGridOccupancy();
                sel.setExistingFeatures(existing);
                if (mode == "fs") sel.gradientMagnitudeWithSSC(frame, thr, std::atoi(argv[6]), std::atoi(argv[7]) != 0);
                else sel.gradientMagnitudeByValue(frame, thr, true);
            };
            run();
            for (const auto& f : frame->m_features)
                std::printf("%.17g %.17g %.17g\n", f->m_pixelPosition[0], f->m_pixelPosition[1], f->m_gradientMagnitude);
            // SVO_CHECK_REPS=n: time n more calls (selection only; the grid reset / existing features are
            // inside the loop but cost nanoseconds) and report the average on stderr
            const char* reps_env = std::getenv("SVO_CHECK_REPS");
            const int reps = reps_env ? std::atoi(reps_env) : 0;
            if (reps > 0) {
                const auto t0 = std::chrono::steady_clock::now();
                for (int r = 0; r < reps; ++r) run();
                const auto t1 = std::chrono::steady_clock::now();
                std::fprintf(stderr, "ms %.6f\n", std::chrono::duration<double, std::milli>(t1 - t0).count() / reps);
            }
            return 0;
        }
        if (mode == "ba" && argc >= 4) {
            const int n = std::atoi(argv[2]);
            std::ifstream f(argv[3], std::ios::binary);
            std::vector<double> d(7 + 7 * (size_t)n);
            f.read(reinterpret_cast<char*>(d.data()), (std::streamsize)(d.size() * sizeof(double)));
            if (!f) throw std::runtime_error("short BA data file");
            Context ctx(0);
            auto cam = std::make_shared<PinholeCamera>(PinholeCamera{64, 64, 300.0, 300.0, 32.0, 32.0});
            std::vector<uint8_t> img(64 * 64, 0);
            auto frame = std::make_shared<Frame>(ctx, cam, img.data(), 1);
            for (int i = 0; i < 7; ++i) frame->m_absPose[i] = d[i];
            for (int k = 0; k < n; ++k) {
                const double* r = &d[7 + 7 * (size_t)k];
                auto feat = std::make_shared<Feature>(frame.get(), Vec2{0.0, 0.0});
                feat->m_bearingVec = {r[0], r[1], r[2]};
                if (r[6] != 0.0) feat->m_point = std::make_shared<Point>(Point{{r[3], r[4], r[5]}});
                frame->m_features.push_back(feat);
            }
            BundleAdjustment ba(ctx, cam, 0, 6);
            for (int call = 0; call < 2; ++call) {
                const double e = ba.optimizePose(frame);
                std::printf("%.17g %d", e, ba.lastStatus());
                for (double v : frame->m_absPose) std::printf(" %.17g", v);
                std::printf("\n");
            }
            return 0;
        }
        if (mode == "depth" && argc >= 5) {
            std::ifstream f(argv[2], std::ios::binary);
            std::vector<double> hdr(6 + 7 + 7 + 3);
            f.read(reinterpret_cast<char*>(hdr.data()), (std::streamsize)(hdr.size() * sizeof(double)));
            const int w = (int)hdr[4], h = (int)hdr[5], n = (int)hdr[22];
            std::vector<double> d(5 * (size_t)n);
            f.read(reinterpret_cast<char*>(d.data()), (std::streamsize)(d.size() * sizeof(double)));
            if (!f) throw std::runtime_error("short depth data file");
            const std::vector<uint8_t> kimg = read_raw(argv[3], (size_t)w * h), cimg = read_raw(argv[4], (size_t)w * h);
            Context ctx(0);
            auto cam = std::make_shared<PinholeCamera>(PinholeCamera{w, h, hdr[0], hdr[1], hdr[2], hdr[3]});
            auto kf = std::make_shared<Frame>(ctx, cam, kimg.data(), 1);
            auto cur = std::make_shared<Frame>(ctx, cam, cimg.data(), 1);
            for (int i = 0; i < 7; ++i) {
                kf->m_absPose[i] = hdr[6 + i];
                cur->m_absPose[i] = hdr[13 + i];
            }
            for (int k = 0; k < n; ++k) {
                const double* r = &d[5 * (size_t)k];
                auto feat = std::make_shared<Feature>(kf.get(), Vec2{r[0], r[1]});
                feat->m_bearingVec = {r[2], r[3], r[4]};
                kf->m_features.push_back(feat);
            }
            DepthEstimator de(ctx);
            de.addKeyframe(kf, hdr[20], hdr[21]);
            const auto cands = de.updateFilters(cur);
            std::printf("filters %zu\n", de.numberFilters());
            for (const auto& c : cands)
                std::printf("cand %.17g %.17g %.17g\n", c.second->m_position[0], c.second->m_position[1], c.second->m_position[2]);
            return 0;
        }
        if (mode == "align" && argc >= 10) {
            std::ifstream f(argv[2], std::ios::binary);
            f.seekg(0, std::ios::end);
            const size_t bytes = (size_t)f.tellg();
            f.seekg(0);
            std::vector<double> v(bytes / sizeof(double));
            f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
            size_t q = 0;
            auto take = [&]() { return v.at(q++); };
            const double fx = take(), fy = take(), cx = take(), cy = take();
            const int w = (int)take(), h = (int)take();
            Pose poses[3];
            for (auto& p : poses)
                for (double& x : p) x = take();
            const int nref = (int)take(), nkf = (int)take();
            const int patch = std::atoi(argv[6]), minl = std::atoi(argv[7]), maxl = std::atoi(argv[8]);
            const int median = std::atoi(argv[9]);
            const std::vector<uint8_t> rimg = read_raw(argv[3], (size_t)w * h), kimg = read_raw(argv[4], (size_t)w * h),
                                       cimg = read_raw(argv[5], (size_t)w * h);
            Context ctx(0);
            auto cam = std::make_shared<PinholeCamera>(PinholeCamera{w, h, fx, fy, cx, cy});
            auto kf = std::make_shared<Frame>(ctx, cam, kimg.data(), maxl + 1);
            auto ref = std::make_shared<Frame>(ctx, cam, rimg.data(), maxl + 1, kf);
            auto cur = std::make_shared<Frame>(ctx, cam, cimg.data(), maxl + 1, kf);
            ref->m_absPose = poses[0];
            kf->m_absPose = poses[1];
            for (int i = 0; i < nref + nkf; ++i) {
                const double ux = take(), uy = take();
                auto feat = std::make_shared<Feature>(i < nref ? ref.get() : kf.get(), Vec2{ux, uy});
                feat->m_bearingVec = {take(), take(), take()};
                const Vec3 pos{take(), take(), take()};
                if (take() != 0.0) feat->m_point = std::make_shared<Point>(Point{pos});
                (i < nref ? ref : kf)->m_features.push_back(feat);
            }
            ImageAlignment align(ctx, (uint32_t)patch, minl, maxl, 6, median);
            for (int call = 0; call < 2; ++call) {
                cur->m_absPose = poses[2];
                const double e = align.align(ref, cur);
                std::printf("%.17g %d", e, align.lastStatus());
                for (double x : cur->m_absPose) std::printf(" %.17g", x);
                std::printf("\n");
            }
            // REPS > 0: the per-frame latency of align() as src/system.cpp:313 pays it (median of REPS calls)
            const int reps = argc >= 11 ? std::atoi(argv[10]) : 0;
            if (reps > 0) {
                std::vector<double> ms;
                for (int i = 0; i < reps; ++i) {
                    cur->m_absPose = poses[2];
                    const auto t0 = std::chrono::steady_clock::now();
                    align.align(ref, cur);
                    ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
                }
                std::sort(ms.begin(), ms.end());
                std::printf("ms %.6f\n", ms[ms.size() / 2]);
            }
            return 0;
        }
        if (mode == "map" && argc >= 6) {
            std::ifstream f(argv[2], std::ios::binary);
            f.seekg(0, std::ios::end);
            const size_t bytes = (size_t)f.tellg();
            f.seekg(0);
            std::vector<double> v(bytes / sizeof(double));
            f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
            size_t q = 0;
            auto take = [&]() { return v.at(q++); };
            const double fx = take(), fy = take(), cx = take(), cy = take();
            const int w = (int)take(), h = (int)take(), cell = (int)take();
            Pose poses[3];
            for (auto& p : poses)
                for (double& x : p) x = take();
            const int nref = (int)take(), nkf = (int)take(), npt = (int)take(), nc = (int)take(), ncells = (int)take();
            const int nf = nref + nkf;
            std::vector<Vec2> px(nf);
            for (auto& p : px) p = {take(), take()};
            std::vector<int> fpt(nf);
            for (int& i : fpt) i = (int)take();
            std::vector<Vec3> ppos(npt);
            for (auto& p : ppos) p = {take(), take(), take()};
            std::vector<uint32_t> ptype(npt), psucc(npt);
            for (auto& t : ptype) t = (uint32_t)take();
            for (auto& t : psucc) t = (uint32_t)take();
            std::vector<int> cf(nc);
            for (int& i : cf) i = (int)take();
            std::vector<Vec3> cpos(nc);
            for (auto& p : cpos) p = {take(), take(), take()};
            std::vector<int32_t> order(ncells);
            for (int32_t& o : order) o = (int32_t)take();
            const std::vector<uint8_t> rimg = read_raw(argv[3], (size_t)w * h), kimg = read_raw(argv[4], (size_t)w * h),
                                       cimg = read_raw(argv[5], (size_t)w * h);
            const int reps = argc >= 7 ? std::atoi(argv[6]) : 0;  // > 0: time reprojectMap + addCandidateToFrame
            const bool twice = argc >= 8 && std::string(argv[7]) == "twice";  // then a second addCandidateToFrame
            Context ctx(0);
            auto cam = std::make_shared<PinholeCamera>(PinholeCamera{w, h, fx, fy, cx, cy});
            double total_ms = 0.0;
            for (int rep = 0; rep <= reps; ++rep) {
                // a fresh object graph per run (the calls mutate the map, the points and the cur frame)
                auto kf = std::make_shared<Frame>(ctx, cam, kimg.data(), 1);
                auto ref = std::make_shared<Frame>(ctx, cam, rimg.data(), 1, kf);
                auto cur = std::make_shared<Frame>(ctx, cam, cimg.data(), 1, kf);
                ref->m_absPose = poses[0];
                kf->m_absPose = poses[1];
                cur->m_absPose = poses[2];
                std::vector<std::shared_ptr<Point>> pts(npt);
                for (int i = 0; i < npt; ++i) {
                    pts[i] = std::make_shared<Point>(Point{ppos[i]});
                    pts[i]->m_type = (Point::PointType)ptype[i];
                    pts[i]->m_succeededProjection = psucc[i];
                }
                std::vector<std::shared_ptr<Feature>> feats(nf);
                for (int i = 0; i < nf; ++i) {
                    feats[i] = std::make_shared<Feature>(i < nref ? ref.get() : kf.get(), px[i]);
                    if (fpt[i] >= 0) feats[i]->m_point = pts[fpt[i]];
                    (i < nref ? ref : kf)->m_features.push_back(feats[i]);
                }
                Map map(ctx, cam, cell);
                for (int i = 0; i < nc; ++i) map.addNewCandidate(feats[cf[i]], std::make_shared<Point>(Point{cpos[i]}));
                map.setCellOrder(order);
                std::vector<std::pair<std::shared_ptr<Frame>, int32_t>> overlap;
                (void)svo_ctx_synchronize(ctx.get());
                const auto t0 = std::chrono::steady_clock::now();
                map.reprojectMap(ref, cur, overlap);
                map.addCandidateToFrame(cur);
                const auto t1 = std::chrono::steady_clock::now();
                if (rep > 0) total_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
                if (rep == 0) {
                    std::printf("counts %u %u\n", map.m_matches, map.m_trials);
                    for (const auto& ft : cur->m_features)
                        std::printf("px %.17g %.17g\n", ft->m_pixelPosition[0], ft->m_pixelPosition[1]);
                    if (twice) {  // a second frame (cur moved 5 cm along x): only unmatched candidates remain
                        std::printf("candidates %zu\n", map.m_candidates.size());
                        auto cur2 = std::make_shared<Frame>(ctx, cam, cimg.data(), 1, kf);
                        cur2->m_absPose = poses[2];
                        cur2->m_absPose[4] += 0.05;
                        map.addCandidateToFrame(cur2);
                        std::printf("candidates %zu\n", map.m_candidates.size());
                        for (const auto& ft : cur2->m_features)
                            std::printf("px2 %.17g %.17g\n", ft->m_pixelPosition[0], ft->m_pixelPosition[1]);
                    }
                }
            }
            if (reps > 0) std::printf("ms %.6f\n", total_ms / reps);
            return 0;
        }
        std::fprintf(stderr, "usage: svo_host_check io | fs W H CELL THR NUM BUCKET IMAGE [EX EY]... | fv W H CELL THR IMAGE\n");
        return 2;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "svo_host_check: %s\n", e.what());
        return 1;
    }
}
