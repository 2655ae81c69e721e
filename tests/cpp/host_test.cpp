// C++ host-layer test driver (built by tests/cpp/Makefile, run from
// tests/test_cpp_host.py).  Calls the reference-named C++ entry points of
// slam-indoor-code_amd/host/slamhip.hpp the way the reference's callers do
// and checks them against the CPU oracle (test infrastructure, linked here
// only).
//   host_test cpu   config / selection / ratio / Rodrigues (no GPU)
//   host_test gpu   FAST, SIFT, ORB, pair matching, BA, batch search vs oracle
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/oracle.h"
#include "../../slam-indoor-code_amd/host/slamhip.hpp"

using namespace slamhip;

static int g_fail = 0;
#define CHECK(cond)                                                                 \
    do {                                                                            \
        if (!(cond)) {                                                              \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
            ++g_fail;                                                               \
        }                                                                           \
    } while (0)

static const char* kConfig = R"({
  // the README example config (all 40 keys), with comments
  "onlyViz": false, "calibrate": false, "visualCalibration": true,
  "calibrationPath": "./config/samsung-hv.xml", "usePhotosCycle": false,
  "photosPathPattern": "", "videoSourcePath": "", "outputDataDir": "./data",
  "threadsCount": 1, "useUndistortion": false, "requiredExtractedPointsCount": 10000,
  "featureExtractingThreshold": 1, "framesBatchSize": 210, "skipFramesFromBatchHead": 0,
  "useFirstFitInBatch": true, "requiredMatchedPointsCount": 500, "useFM-SIFT-FLANN": true,
  "useFM-SIFT-BF": false, "useFM-ORB": false, "knnMatcherDistance": 0.7, "RPUseRANSAC": true,
  "RPRANSACProb": 0.999, "RPRANSACThreshold": 5.0, "RPDistanceThreshold": 200.0,
  "useBundleAdjustment": false, "BAMaxFramesCnt": 8, "BAThreadsCnt": 12,
  "BAUseTrivialLossFunction": false, "BAUseHuberLossFunction": true,
  "BAHuberLossFunctionParameter": 4.0, "BAUseCauchyLossFunction": false,
  "BACauchyLossFunctionParameter": 1.0, "BAUseArctanLossFunction": false,
  "BAArctanLossFunctionParameter": 1.0, "BAUseTukeyLossFunction": false,
  "BATukeyLossFunctionParameter": 1.0, /* triangulation */ "TriangleMaxDistance": 1.0,
  "TriangleEuclidDistanceWeight": 1.0, "TriangleColorDistance": 1.0, "TriangleMinimumPoints": 3
})";

static void test_cpu()
{
    ConfigService cfg;
    cfg.setConfigText(kConfig);
    CHECK(cfg.getValue<int>("framesBatchSize") == 210);
    CHECK(std::fabs(cfg.getValue<double>("knnMatcherDistance") - 0.7) < 1e-15);
    CHECK(cfg.getValue<bool>("useFM-SIFT-FLANN"));
    CHECK(cfg.getValue<std::string>("calibrationPath") == "./config/samsung-hv.xml");
    CHECK(getMatcherTypeIndex(cfg) == SIFT_FLANN);

    // checkJSON: a missing key and a wrong type are rejected with the reference's text
    std::string t = kConfig;
    {
        std::string bad = t;
        bad.replace(bad.find("\"useFM-ORB\": false"), 18, "\"useFM-ORB\": 3");
        bool threw = false;
        try { ConfigService c; c.setConfigText(bad); } catch (const ConfigError& e) {
            threw = std::string(e.what()).find("\"useFM-ORB\" missed or has incorrect type") != std::string::npos;
        }
        CHECK(threw);
    }
    {
        bool threw = false;
        try { ConfigService c; c.setConfigText("{\"onlyViz\": false}"); } catch (const ConfigError&) { threw = true; }
        CHECK(threw);
    }
    {
        bool threw = false;
        try { ConfigService c; c.setConfigText("{ not json"); } catch (const ConfigError&) { threw = true; }
        CHECK(threw);
    }
    // no matcher selected -> throw (featureMatchingCommon.cpp:20)
    {
        std::string none = t;
        none.replace(none.find("\"useFM-SIFT-FLANN\": true"), 24, "\"useFM-SIFT-FLANN\": false");
        ConfigService c;
        c.setConfigText(none);
        bool threw = false;
        try { getMatcherTypeIndex(c); } catch (const std::exception&) { threw = true; }
        CHECK(threw);
    }

    // selection rule vs the oracle
    std::mt19937 rng(5);
    for (int trial = 0; trial < 300; trial++) {
        const int n = rng() % 12;
        std::vector<int32_t> counts(n);
        for (auto& c : counts) c = rng() % 800;
        const int req = rng() % 900, skip = rng() % 4;
        const bool ff = rng() & 1;
        CHECK(selectGoodFrame(counts, req, skip, ff) == orc_select_good(counts.data(), n, req, skip, ff));
    }

    // ratio test: strict, double compare, missing neighbours skipped
    std::vector<int> idx{3, 4, 5, -1, 7, 8};
    std::vector<float> dist{6.9f, 10.f, 1.f, 0.f, 0.f, 0.f};
    std::vector<DMatch> good;
    getGoodMatches(idx, dist, 0.7, good);
    CHECK(good.size() == 1 && good[0].queryIdx == 0 && good[0].trainIdx == 3);
    dist[0] = 7.f;                       // 0.7 * 10.0 == 7.0 in double: the strict test rejects it
    getGoodMatches(idx, dist, 0.7, good);
    CHECK(good.empty());

    // Rodrigues both ways
    for (int trial = 0; trial < 50; trial++) {
        std::uniform_real_distribution<double> u(-1.5, 1.5);   // |r| < pi: unique angle-axis
        std::array<double, 3> r{u(rng), u(rng), u(rng)};
        const auto R = rodrigues(r);
        const auto r2 = rodrigues(R);
        for (int q = 0; q < 3; q++) CHECK(std::fabs(r[q] - r2[q]) < 1e-9);
    }
    CHECK(rodrigues(std::array<double, 9>{1, 0, 0, 0, 1, 0, 0, 0, 1})[0] == 0.0);
}

static std::vector<uint8_t> synth(int w, int h, int first, int count)
{
    std::vector<uint8_t> f((size_t)w * h * 3 * count);
    slam_synth_frames(w, h, first, count, 1234, f.data());
    return f;
}

static void test_gpu()
{
    configService.setConfigText(kConfig);
    const int w = 640, h = 480;
    auto frames = synth(w, h, 0, 3);
    Image im0{frames.data(), w, h, (size_t)w * 3, 3};
    Image im1{frames.data() + (size_t)w * h * 3, w, h, (size_t)w * 3, 3};

    // fastExtractor vs oracle: bit-exact, raster order
    std::vector<KeyPoint> kp0, kp1;
    fastExtractor(im0, kp0, 12, true);
    fastExtractor(im1, kp1, 12, true);
    std::vector<orc_kp> ref(w * h / 4);
    const int nref = orc_fast_bgr(im0.data, w, h, im0.step, 12, 1, ref.data(), (int)ref.size());
    CHECK((int)kp0.size() == nref && nref > 200);
    CHECK(std::memcmp(kp0.data(), ref.data(), sizeof(orc_kp) * std::min<size_t>(nref, kp0.size())) == 0);

    // extractDescriptor SIFT vs oracle: bit-exact
    Descriptors d0;
    std::vector<KeyPoint> k = kp0;
    extractDescriptor(im0, k, SIFT_FLANN, d0);
    std::vector<float> sref((size_t)kp0.size() * 128);
    orc_sift_compute(im0.data, w, h, im0.step, reinterpret_cast<const orc_kp*>(kp0.data()), (int)kp0.size(),
                     sref.data());
    CHECK(d0.rows == (int)kp0.size() && d0.f32 == sref);

    // full SIFT detector vs oracle/siftdet.c: keypoints and descriptors bit-exact
    {
        std::vector<KeyPoint> dk;
        Descriptors dd;
        siftDetectAndCompute(im0, dk, dd);
        std::vector<orc_kp> rk((size_t)w * h / 4);
        std::vector<float> rd(rk.size() * 128);
        const int nr = orc_sift_detect(im0.data, w, h, im0.step, rk.data(), (int)rk.size(), rd.data());
        rd.resize((size_t)nr * 128);
        CHECK((int)dk.size() == nr && nr > 50);
        CHECK(std::memcmp(dk.data(), rk.data(), sizeof(orc_kp) * std::min<size_t>(nr, dk.size())) == 0);
        CHECK(dd.rows == nr && dd.f32 == rd);
    }

    // reconstruct (two-view DLT) vs oracle/geom.c: bit-exact
    {
        const std::array<double, 9> K{1724.676, 0, 995.966, 0, 1730.482, 550.192, 0, 0, 1}, R1{1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double a = 0.05;
        const std::array<double, 9> R2{std::cos(a), 0, std::sin(a), 0, 1, 0, -std::sin(a), 0, std::cos(a)};
        const std::array<double, 3> t1{0, 0, 0}, t2{-0.2, 0.01, 0.02};
        std::vector<Point2f> q1, q2;
        for (int i = 0; i < 500; i++) {
            q1.push_back(Point2f{(float)(300 + (i * 37) % 1300), (float)(100 + (i * 53) % 800)});
            q2.push_back(Point2f{(float)(320 + (i * 37) % 1300 + (i % 7)), (float)(98 + (i * 53) % 800)});
        }
        std::vector<Point3d> X;
        reconstruct(K, R1, t1, R2, t2, q1, q2, X);
        std::vector<double> ref(q1.size() * 3);
        orc_reconstruct(K.data(), R1.data(), t1.data(), R2.data(), t2.data(), reinterpret_cast<const float*>(q1.data()),
                        reinterpret_cast<const float*>(q2.data()), (int)q1.size(), ref.data());
        CHECK(X.size() == q1.size() && std::memcmp(X.data(), ref.data(), ref.size() * sizeof(double)) == 0);
    }

    // estimateTransformation (findEssentialMat RANSAC + recoverPose) vs oracle/essential.c
    {
        const std::array<double, 9> K{1724.676, 0, 995.966, 0, 1730.482, 550.192, 0, 0, 1};
        const double a = 0.06;
        const double Rt[9] = {std::cos(a), 0, std::sin(a), 0, 1, 0, -std::sin(a), 0, std::cos(a)};
        const double tt[3] = {-0.3, 0.02, 0.05};
        std::vector<Point2f> q1, q2;
        for (int i = 0; i < 800; i++) {
            const double X[3] = {-3 + 6.0 * ((i * 37) % 101) / 101, -1.5 + 3.0 * ((i * 53) % 97) / 97, 3 + 7.0 * ((i * 17) % 89) / 89};
            double Y[3];
            for (int r = 0; r < 3; r++) Y[r] = Rt[r * 3] * X[0] + Rt[r * 3 + 1] * X[1] + Rt[r * 3 + 2] * X[2] + tt[r];
            q1.push_back(Point2f{(float)(1724.676 * X[0] / X[2] + 995.966), (float)(1730.482 * X[1] / X[2] + 550.192)});
            if (i % 5 == 0) q2.push_back(Point2f{(float)((i * 131) % 1920), (float)((i * 71) % 1080)});   // outliers
            else q2.push_back(Point2f{(float)(1724.676 * Y[0] / Y[2] + 995.966), (float)(1730.482 * Y[1] / Y[2] + 550.192)});
        }
        std::array<double, 9> R;
        std::array<double, 3> t;
        std::vector<uint8_t> cm;
        const bool ok = estimateTransformation(q1, q2, K, R, t, cm);
        double Rr[9], tr[3];
        std::vector<uint8_t> cr(q1.size()), rr(q1.size());
        int passed = 0;
        const int rok = orc_estimate_transformation(reinterpret_cast<const float*>(q1.data()),
                                                    reinterpret_cast<const float*>(q2.data()), (int)q1.size(), K.data(),
                                                    1, 0.999, 5.0, 200.0, Rr, tr, cr.data(), rr.data(), &passed);
        CHECK(ok == (rok != 0) && ok);
        CHECK(std::memcmp(R.data(), Rr, sizeof(Rr)) == 0 && std::memcmp(t.data(), tr, sizeof(tr)) == 0 && cm == cr);
    }

    // solvePnPRansac (EPnP RANSAC + LM refinement) vs oracle/pnp.c
    {
        const std::array<double, 9> K{1724.676, 0, 995.966, 0, 1730.482, 550.192, 0, 0, 1};
        const double a = 0.1;
        const double Rt[9] = {std::cos(a), -std::sin(a), 0, std::sin(a), std::cos(a), 0, 0, 0, 1};
        const double tt[3] = {0.2, -0.1, 0.4};
        std::vector<Point3f> obj;
        std::vector<Point2f> img;
        for (int i = 0; i < 700; i++) {
            const Point3f X{(float)(-3 + 6.0 * ((i * 37) % 101) / 101), (float)(-1.5 + 3.0 * ((i * 53) % 97) / 97),
                            (float)(3 + 7.0 * ((i * 17) % 89) / 89)};
            double Y[3];
            for (int r = 0; r < 3; r++) Y[r] = Rt[r * 3] * X.x + Rt[r * 3 + 1] * X.y + Rt[r * 3 + 2] * X.z + tt[r];
            obj.push_back(X);
            if (i % 4 == 0) img.push_back(Point2f{(float)((i * 131) % 1920), (float)((i * 71) % 1080)});  // outliers
            else img.push_back(Point2f{(float)(1724.676 * Y[0] / Y[2] + 995.966 + (i % 3) * 0.3),
                                       (float)(1730.482 * Y[1] / Y[2] + 550.192 - (i % 5) * 0.2)});
        }
        std::array<double, 3> rv, tv;
        std::vector<int> inl;
        const bool ok = solvePnPRansac(obj, img, K, rv, tv, 100, 8.0f, 0.99, &inl);
        double rr[3], tr[3];
        std::vector<uint8_t> mr(obj.size());
        int ni = 0;
        const int st = orc_solve_pnp_ransac(reinterpret_cast<const float*>(obj.data()),
                                            reinterpret_cast<const float*>(img.data()), (int)obj.size(), K.data(), 100,
                                            8.0f, 0.99, rr, tr, mr.data(), &ni);
        CHECK(ok && st == 1 && (int)inl.size() == ni);
        CHECK(std::memcmp(rv.data(), rr, sizeof(rr)) == 0 && std::memcmp(tv.data(), tr, sizeof(tr)) == 0);
        bool threw = false;
        std::vector<Point3f> o4(obj.begin(), obj.begin() + 4);
        std::vector<Point2f> i4(img.begin(), img.begin() + 4);
        try { solvePnPRansac(o4, i4, K, rv, tv); } catch (const std::exception&) { threw = true; }
        CHECK(threw);
    }

    // ORB: border filter in place + descriptors bit-exact
    Descriptors o0;
    std::vector<KeyPoint> ko = kp0;
    extractDescriptor(im0, ko, ORB_BF, o0);
    std::vector<orc_kp> kref(reinterpret_cast<const orc_kp*>(kp0.data()),
                             reinterpret_cast<const orc_kp*>(kp0.data()) + kp0.size());
    std::vector<uint8_t> oref(kp0.size() * 32);
    const int no = orc_orb_compute(im0.data, w, h, im0.step, kref.data(), (int)kref.size(), oref.data());
    oref.resize((size_t)no * 32);
    CHECK((int)ko.size() == no && o0.u8 == oref);
    CHECK(std::memcmp(ko.data(), kref.data(), sizeof(orc_kp) * no) == 0);

    // invalid extractor type -> throw
    {
        bool threw = false;
        try { extractDescriptor(im0, k, 7, d0); } catch (const std::exception&) { threw = true; }
        CHECK(threw);
    }

    // matchFramesPairFeatures (5-arg) vs oracle kNN + ratio (knnMatcherDistance 0.7 from the config)
    std::vector<DMatch> m;
    std::vector<KeyPoint> k1 = kp1;
    matchFramesPairFeatures(d0, im1, k1, SIFT_FLANN, m);
    std::vector<float> s1((size_t)kp1.size() * 128);
    orc_sift_compute(im1.data, w, h, im1.step, reinterpret_cast<const orc_kp*>(kp1.data()), (int)kp1.size(),
                     s1.data());
    std::vector<int> ridx(2 * kp0.size());
    std::vector<float> rdist(2 * kp0.size());
    orc_knn2(sref.data(), (int)kp0.size(), s1.data(), (int)kp1.size(), 128, ORC_NORM_L2, ridx.data(), rdist.data());
    std::vector<orc_match> rm(kp0.size());
    const int nm = orc_ratio(ridx.data(), rdist.data(), (int)kp0.size(), 0.7, rm.data());
    CHECK((int)m.size() == nm && nm > 50);
    CHECK(std::memcmp(m.data(), rm.data(), sizeof(orc_match) * std::min<size_t>(nm, m.size())) == 0);

    // 6-arg overload == extract first + 5-arg
    std::vector<DMatch> m6;
    std::vector<KeyPoint> a = kp0, b = kp1;
    matchFramesPairFeatures(im0, im1, a, b, SIFT_FLANN, m6);
    CHECK(m6.size() == m.size() && std::memcmp(m6.data(), m.data(), sizeof(DMatch) * m.size()) == 0);

    // bundleAdjustment on a small window vs the oracle (Huber 4 from the config)
    {
        std::mt19937 rng(11);
        std::normal_distribution<double> nz(0.0, 0.5);
        const int nf = 3, np = 120;
        std::array<double, 9> K{800, 0, 320, 0, 805, 240, 0, 0, 1};
        GlobalData g;
        std::vector<TemporalImageData> win(nf);
        std::uniform_real_distribution<double> u(-1.0, 1.0);
        for (int p = 0; p < np; p++) g.spatialPoints.push_back({u(rng), u(rng), 5.0 + u(rng)});
        for (int f = 0; f < nf; f++) {
            win[f].rotation = rodrigues(std::array<double, 3>{0.01 * f, -0.02 * f, 0.005 * f});
            win[f].motion = {0.1 * f, 0.0, 0.02 * f};
            for (int p = 0; p < np; p++) {
                // project with the true pose; observation noise; every 7th point unobserved
                const auto& P = g.spatialPoints[p];
                const auto& R = win[f].rotation;
                const double X = R[0] * P.x + R[1] * P.y + R[2] * P.z + win[f].motion[0];
                const double Y = R[3] * P.x + R[4] * P.y + R[5] * P.z + win[f].motion[1];
                const double Z = R[6] * P.x + R[7] * P.y + R[8] * P.z + win[f].motion[2];
                KeyPoint kp;
                kp.x = (float)(K[0] * X / Z + K[2] + nz(rng));
                kp.y = (float)(K[4] * Y / Z + K[5] + nz(rng));
                win[f].allExtractedFeatures.push_back(kp);
                win[f].correspondSpatialPointIdx.push_back((p + f) % 7 == 0 ? -1 : p);
            }
        }
        for (auto& P : g.spatialPoints) { P.x += 0.01; P.z -= 0.02; }
        // oracle on the same arrays
        double K4[4] = {K[0], K[4], K[2], K[5]};
        std::vector<double> ext(nf * 6), pts;
        std::vector<int> of, op;
        std::vector<double> oxy;
        for (int f = 0; f < nf; f++) {
            const auto r = rodrigues(win[f].rotation);
            for (int q = 0; q < 3; q++) { ext[6 * f + q] = r[q]; ext[6 * f + 3 + q] = win[f].motion[q]; }
            for (int p = 0; p < np; p++) {
                const int idx = win[f].correspondSpatialPointIdx[p];
                if (idx < 0) continue;
                of.push_back(f); op.push_back(idx);
                oxy.push_back(win[f].allExtractedFeatures[p].x); oxy.push_back(win[f].allExtractedFeatures[p].y);
            }
        }
        for (auto& P : g.spatialPoints) { pts.push_back(P.x); pts.push_back(P.y); pts.push_back(P.z); }
        orc_ba_summary rs{};
        orc_ba(K4, nf, ext.data(), np, pts.data(), (int)of.size(), of.data(), op.data(), oxy.data(), ORC_LOSS_HUBER,
               4.0, 50, &rs);
        const slam_ba_summary gs = bundleAdjustment(K, win, g);
        CHECK(gs.num_residuals == rs.num_residuals);
        CHECK(std::fabs(gs.initial_cost - rs.initial_cost) <= 1e-9 * rs.initial_cost);
        CHECK(std::fabs(gs.final_cost - rs.final_cost) <= 1e-6 * rs.final_cost + 1e-9);
        CHECK(std::fabs(std::sqrt(gs.final_cost / gs.num_residuals) - std::sqrt(rs.final_cost / rs.num_residuals)) <=
              1e-4);
        CHECK(std::fabs(K[0] - K4[0]) < 1e-3 && std::fabs(K[5] - K4[3]) < 1e-3);
    }

    // device-resident batch search: counts == oracle per candidate
    {
        const int nb = 3;
        uint8_t* d_frames = nullptr;
        CHECK(hipMalloc(&d_frames, frames.size()) == hipSuccess);
        CHECK(hipMemcpy(d_frames, frames.data(), frames.size(), hipMemcpyHostToDevice) == hipSuccess);
        Context ctx(0);
        BatchConditions cond;
        cond.featureExtractingThreshold = 12;
        cond.requiredMatchedPointsCount = 100;
        cond.matcherType = SIFT_FLANN;
        // previous frame = frame 0 (extracted alone, exported in the device format)
        std::vector<int32_t> kc(1);
        CHECK(slam_batch_extract(ctx.get(), nullptr, d_frames, 1, w, h, 12, SIFT_FLANN, kc.data()) == SLAM_OK);
        void* d_prev = nullptr;
        CHECK(hipMalloc(&d_prev, slam_batch_desc_bytes(SIFT_FLANN, kc[0])) == hipSuccess);
        int nprev = 0;
        CHECK(slam_batch_export_desc(ctx.get(), nullptr, 0, d_prev, &nprev) == SLAM_OK && nprev == kc[0]);
        const BatchResult r = findGoodFrameFromBatch(ctx, nullptr, d_frames, nb, w, h, d_prev, nprev, cond);
        CHECK((int)r.inBatch.size() == nb);
        for (int f = 0; f < nb; f++) {
            const uint8_t* fp = frames.data() + (size_t)f * w * h * 3;
            std::vector<orc_kp> kf(w * h / 4);
            const int nk = orc_fast_bgr(fp, w, h, (size_t)w * 3, 12, 1, kf.data(), (int)kf.size());
            std::vector<float> df((size_t)nk * 128);
            orc_sift_compute(fp, w, h, (size_t)w * 3, kf.data(), nk, df.data());
            std::vector<int> ii(2 * nprev);
            std::vector<float> dd(2 * nprev);
            orc_knn2(sref.data(), nprev, df.data(), nk, 128, ORC_NORM_L2, ii.data(), dd.data());
            std::vector<orc_match> mm(nprev);
            const int cnt = orc_ratio(ii.data(), dd.data(), nprev, 0.7, mm.data());
            CHECK(r.kpCounts[f] == nk);
            CHECK(r.matchCounts[f] == cnt);
        }
        CHECK(r.goodIndex == selectGoodFrame(r.matchCounts, 100, 0, true));
        CHECK(hipFree(d_prev) == hipSuccess);
        CHECK(hipFree(d_frames) == hipSuccess);
    }
}

int main(int argc, char** argv)
{
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        if (mode == "cpu") test_cpu();
        else if (mode == "gpu") test_gpu();
        else { std::fprintf(stderr, "usage: host_test cpu|gpu\n"); return 2; }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 1;
    }
    if (g_fail) { std::fprintf(stderr, "%d check(s) failed\n", g_fail); return 1; }
    std::printf("host_test %s: ok\n", mode.c_str());
    return 0;
}
