// -D USE_HIP replacement of src/mainModule/bundleAdjustment/bundleAdjustment.cpp:73-129
// (the Ceres call site).  Same problem as the reference builds: calibration
// {fx, fy, cx, cy} shared and free, extrinsics {angle-axis, t} per window frame
// with frame 0 constant, one residual block per observed keypoint in
// (frame, keypoint) order, loss from getLossFunction's config priority.  The
// solve (jets, Schur, LDS Cholesky, LM with Ceres' defaults) runs on the
// GPU behind slam_ba.  Needs OpenCV (cv::Rodrigues, cv::Mat); in this repo it is
// compiled and run against the stand-ins of tests/shim_stub (test_shim_compile.py).
#include "bundleAdjustment.h"

#include <cmath>
#include <vector>

#include "../../config/config.h"
#include "../../misc/IOmisc.h"
#include "slamhip.h"
#include "slamhip.hpp"

static int loss_from_config(double& par)
{
    par = 0;
    if (configService.getValue<bool>(ConfigFieldEnum::BA_USE_TRIVIAL_LOSS)) return SLAM_LOSS_TRIVIAL;
    if (configService.getValue<bool>(ConfigFieldEnum::BA_USE_HUBER_LOSS)) {
        par = configService.getValue<double>(ConfigFieldEnum::BA_HUBER_LOSS_PARAMETER);
        return SLAM_LOSS_HUBER;
    }
    if (configService.getValue<bool>(ConfigFieldEnum::BA_USE_CAUCHY_LOSS)) {
        par = configService.getValue<double>(ConfigFieldEnum::BA_CAUCHY_LOSS_PARAMETER);
        return SLAM_LOSS_CAUCHY;
    }
    if (configService.getValue<bool>(ConfigFieldEnum::BA_USE_ARCTAN_LOSS)) {
        par = configService.getValue<double>(ConfigFieldEnum::BA_ARCTAN_LOSS_PARAMETER);
        return SLAM_LOSS_ARCTAN;
    }
    if (configService.getValue<bool>(ConfigFieldEnum::BA_USE_TUKEY_LOSS)) {
        par = configService.getValue<double>(ConfigFieldEnum::BA_TUKEY_LOSS_PARAMETER);
        return SLAM_LOSS_TUKEY;
    }
    return SLAM_LOSS_NONE;
}

void bundleAdjustment(cv::Mat& K, std::vector<TemporalImageData>& window, GlobalData& globalData)
{
    auto& c = slamhip::Context::thread_default();
    double K4[4] = {K.at<double>(0, 0), K.at<double>(1, 1), K.at<double>(0, 2), K.at<double>(1, 2)};
    const int nf = (int)window.size();
    std::vector<double> ext((size_t)nf * 6);
    std::vector<int32_t> of, op;
    std::vector<double> oxy;
    for (int i = 0; i < nf; i++) {
        cv::Mat r;
        cv::Rodrigues(window[i].rotation, r);
        for (int q = 0; q < 3; q++) {
            ext[6 * i + q] = r.at<double>(q);
            ext[6 * i + 3 + q] = window[i].motion.at<double>(q);
        }
        const auto& kps = window[i].allExtractedFeatures;
        for (size_t p = 0; p < kps.size(); p++) {
            const int idx = window[i].correspondSpatialPointIdx.at(p);
            if (idx < 0) continue;
            of.push_back(i);
            op.push_back(idx);
            oxy.push_back(kps[p].pt.x);
            oxy.push_back(kps[p].pt.y);
        }
    }
    double par = 0;
    const int loss = loss_from_config(par);
    slam_ba_summary s{};
    // a HIP / argument error is not a solver outcome: it throws (slamhip::Error),
    // as any failure the reference's Ceres call cannot report would
    // cv::Point3d is three packed doubles: the points pass as one array (none: null)
    double* pts = globalData.spatialPoints.empty() ? nullptr : &globalData.spatialPoints[0].x;
    slamhip::check(slam_ba(c.get(), K4, nf, ext.data(), (int)globalData.spatialPoints.size(), pts, (int)of.size(),
                           of.data(), op.data(), oxy.data(), loss, par, 0, &s),
                   &c);
    // bundleAdjustment.cpp:119-128: log, then convertDataFromBA in either case --
    // the points were already updated in place by the solve, so K, R and t are
    // written back even when the solution is not usable
    if (!s.usable)
        logStreams.mainReportStream << "BA failed" << std::endl;
    else
        logStreams.mainReportStream << "Bundle Adjustment statistics (approximated RMSE):" << std::endl
                                    << " #residuals: " << s.num_residuals << std::endl
                                    << " Initial RMSE: " << std::sqrt(s.initial_cost / s.num_residuals) << std::endl
                                    << " Final RMSE: " << std::sqrt(s.final_cost / s.num_residuals) << std::endl
                                    << " Time (s): " << s.total_time_in_seconds << std::endl;
    K.at<double>(0, 0) = K4[0];
    K.at<double>(1, 1) = K4[1];
    K.at<double>(0, 2) = K4[2];
    K.at<double>(1, 2) = K4[3];
    for (int i = 0; i < nf; i++) {
        cv::Mat r(3, 1, CV_64F, &ext[6 * i]);
        cv::Rodrigues(r, window[i].rotation);
        for (int q = 0; q < 3; q++) window[i].motion.at<double>(q) = ext[6 * i + 3 + q];
    }
}
