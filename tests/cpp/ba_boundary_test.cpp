// Host-layer bundleAdjustment boundary behaviour without a GPU
// (bundleAdjustment.cpp:105-128): the solver's K / extrinsics / points are
// written back whatever the summary says -- Ceres leaves its last parameter
// values in place and the reference copies them back before it checks
// IsSolutionUsable -- while a HIP / argument error (a non-zero slam status) is
// not a solver outcome and throws slamhip::Error.
//
// The device entry points are interposed by this executable (-rdynamic): the
// mock slam_ba perturbs every parameter by a known amount and reports the
// summary the test asks for, so the host layer's write-back and error paths run
// on any machine.
#include "slamhip.hpp"

#include <cmath>
#include <cstdio>
#include <string>

using namespace slamhip;

static int g_fail = 0;
#define CHECK(cond)                                                                 \
    do {                                                                            \
        if (!(cond)) {                                                              \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
            ++g_fail;                                                               \
        }                                                                           \
    } while (0)

// ---- interposed device entry points ---------------------------------------------------------

static int g_status = SLAM_OK;       // what the mock slam_ba returns
static int g_usable = 0;             // the summary it reports
static int g_loss = -1;
static double g_loss_param = 0;
static int g_nobs = -1;
static slam_ctx* const kFakeCtx = reinterpret_cast<slam_ctx*>(0x1000);

extern "C" {
slam_ctx* slam_create(int) { return kFakeCtx; }
void slam_destroy(slam_ctx*) {}
const char* slam_last_error(const slam_ctx*) { return "mock HIP failure"; }
int slam_ba(slam_ctx* c, double* K4, int nframes, double* ext6, int npoints, double* pts3, int nobs,
            const int32_t*, const int32_t*, const double*, int loss, double loss_param, int,
            slam_ba_summary* s)
{
    if (c != kFakeCtx) return SLAM_E_INVALID_ARG;
    g_loss = loss;
    g_loss_param = loss_param;
    g_nobs = nobs;
    if (g_status != SLAM_OK) return g_status;
    for (int q = 0; q < 4; q++) K4[q] += 1.0;
    for (int i = 0; i < nframes * 6; i++) ext6[i] += 0.01 * (i + 1);
    for (int i = 0; i < npoints * 3; i++) pts3[i] -= 0.5;
    s->initial_cost = 10;
    s->final_cost = 12;
    s->num_residuals = 2 * nobs;
    s->iterations = 1;
    s->successful_steps = 0;
    s->termination = g_usable ? 1 : 3;
    s->usable = g_usable;
    return SLAM_OK;
}
}

static const char* kConfig = R"({
  "onlyViz": false, "calibrate": false, "visualCalibration": true,
  "calibrationPath": "", "usePhotosCycle": false, "photosPathPattern": "", "videoSourcePath": "",
  "outputDataDir": "./data", "threadsCount": 1, "useUndistortion": false,
  "requiredExtractedPointsCount": 10, "featureExtractingThreshold": 1, "framesBatchSize": 4,
  "skipFramesFromBatchHead": 0, "useFirstFitInBatch": true, "requiredMatchedPointsCount": 5,
  "useFM-SIFT-FLANN": true, "useFM-SIFT-BF": false, "useFM-ORB": false, "knnMatcherDistance": 0.7,
  "RPUseRANSAC": true, "RPRANSACProb": 0.999, "RPRANSACThreshold": 5.0, "RPDistanceThreshold": 200.0,
  "useBundleAdjustment": true, "BAMaxFramesCnt": 2, "BAThreadsCnt": 1,
  "BAUseTrivialLossFunction": false, "BAUseHuberLossFunction": false,
  "BAHuberLossFunctionParameter": 4.0, "BAUseCauchyLossFunction": true,
  "BACauchyLossFunctionParameter": 2.5, "BAUseArctanLossFunction": false,
  "BAArctanLossFunctionParameter": 1.0, "BAUseTukeyLossFunction": false,
  "BATukeyLossFunctionParameter": 1.0, "TriangleMaxDistance": 1.0,
  "TriangleEuclidDistanceWeight": 1.0, "TriangleColorDistance": 1.0, "TriangleMinimumPoints": 3
})";

struct Problem {
    std::array<double, 9> K{500, 0, 320, 0, 510, 240, 0, 0, 1};
    std::vector<TemporalImageData> window;
    GlobalData g;
    Problem()
    {
        window.resize(2);
        for (int i = 0; i < 2; i++) {
            window[i].motion = {0.1 * i, 0, 0};
            for (int p = 0; p < 3; p++) {
                KeyPoint kp;
                kp.x = 100.f + 10 * p;
                kp.y = 50.f + i;
                window[i].allExtractedFeatures.push_back(kp);
                window[i].correspondSpatialPointIdx.push_back(p == 1 && i == 1 ? -1 : p);
            }
        }
        for (int p = 0; p < 3; p++) g.spatialPoints.push_back(Point3d{0.1 * p, 0.2, 4.0});
    }
};

static void expect_written_back(const Problem& before, const Problem& after)
{
    CHECK(after.K[0] == before.K[0] + 1 && after.K[4] == before.K[4] + 1);
    CHECK(after.K[2] == before.K[2] + 1 && after.K[5] == before.K[5] + 1);
    for (int i = 0; i < 2; i++)
        for (int q = 0; q < 3; q++)
            CHECK(std::fabs(after.window[i].motion[q] - (before.window[i].motion[q] + 0.01 * (6 * i + 3 + q + 1))) <
                  1e-12);
    // the rotations moved off identity: rotation vector (0.01, 0.02, 0.03) for frame 0
    CHECK(std::fabs(after.window[0].rotation[0] - 1.0) > 1e-6);
    for (int p = 0; p < 3; p++) CHECK(after.g.spatialPoints[p].z == before.g.spatialPoints[p].z - 0.5);
}

int main()
{
    ConfigService cfg;
    cfg.setConfigText(kConfig);

    // 1. a solve that is not usable still writes K / R / t / points back
    {
        Problem before, p;
        g_status = SLAM_OK;
        g_usable = 0;
        const slam_ba_summary s = bundleAdjustment(p.K, p.window, p.g, cfg);
        CHECK(s.usable == 0 && s.termination == 3);
        CHECK(g_nobs == 5);                                  // the -1 correspondence is skipped
        CHECK(g_loss == SLAM_LOSS_CAUCHY && g_loss_param == 2.5);
        expect_written_back(before, p);
    }
    // 2. a usable solve: same write-back
    {
        Problem before, p;
        g_usable = 1;
        const slam_ba_summary s = bundleAdjustment(p.K, p.window, p.g, cfg);
        CHECK(s.usable == 1);
        expect_written_back(before, p);
    }
    // 3. a HIP error throws and leaves the caller's data untouched
    {
        Problem before, p;
        g_status = SLAM_E_HIP;
        bool threw = false;
        try {
            bundleAdjustment(p.K, p.window, p.g, cfg);
        } catch (const Error& e) {
            threw = std::string(e.what()).find("mock HIP failure") != std::string::npos;
        }
        CHECK(threw);
        CHECK(p.K == before.K);
        CHECK(p.window[1].motion == before.window[1].motion);
        CHECK(p.g.spatialPoints[2].z == before.g.spatialPoints[2].z);
    }
    if (g_fail) { std::fprintf(stderr, "%d check(s) failed\n", g_fail); return 1; }
    std::printf("ba_boundary_test: ok\n");
    return 0;
}
