// -D USE_HIP source set for the reference (FIT-2023-SLAM-indoor/slam-indoor-code):
// the third implementation of src/mainModule/featureMatching/featureMatching.h,
// next to featureMatchingCPU.cpp / featureMatchingCUDA.cpp (CMakeLists.txt:56-67
// picks one at compile time).  cv::KeyPoint / cv::DMatch are byte-identical to
// slam_keypoint / slam_dmatch, so buffers pass straight through the C ABI.
//
// Compiles inside the reference tree (needs OpenCV 4.8 headers and the
// reference's config/log headers).  This image has no OpenCV: the file is
// compiled and run against the stand-ins of tests/shim_stub (a working cv::Mat,
// the reference's declared signatures) by tests/test_shim_compile.py, and its
// outputs are checked against the oracle on the GPU.
#include "featureMatching.h"
#include "featureMatchingCommon.h"

#include <stdexcept>
#include <string>

#include "../../config/config.h"
#include "slamhip.h"            // include/slamhip.h (C ABI)
#include "slamhip.hpp"          // slamhip::Context::thread_default(), slamhip::check

namespace {

slam_ctx* ctx() { return slamhip::Context::thread_default().get(); }

void hip_check(int st)
{
    if (st == SLAM_E_BAD_MATCHER) throw std::exception();          // featureMatchingCPU.cpp:37,63
    slamhip::check(st, &slamhip::Context::thread_default());
}

int channels_of(const cv::Mat& m) { return m.channels(); }

}  // namespace

void extractDescriptor(Mat& frame, std::vector<KeyPoint>& features, int extractorType, Mat& desc)
{
    static_assert(sizeof(KeyPoint) == sizeof(slam_keypoint), "cv::KeyPoint layout");
    if (extractorType < 0 || extractorType > 2) throw std::exception();
    CV_Assert(frame.depth() == CV_8U);
    int n = (int)features.size();
    if (extractorType == MatcherType::ORB_BF) desc.create(n, 32, CV_8U);
    else desc.create(n, 128, CV_32F);
    hip_check(slam_describe(ctx(), frame.data, frame.cols, frame.rows, frame.step, channels_of(frame), extractorType,
                            reinterpret_cast<slam_keypoint*>(features.data()), &n, desc.data));
    features.resize(n);                                   // ORB: runByImageBorder(31) in place
    desc = desc.rowRange(0, n).clone();
}

// knnMatch(prev = query, cur = train, k = 2) + getGoodMatches (config read per call)
static void matchFeaturesHIP(const Mat& prevDesc, const Mat& curDesc, std::vector<DMatch>& matches, int type)
{
    const double ratio = configService.getValue<double>(ConfigFieldEnum::FM_KNN_DISTANCE);
    matches.resize(std::max(prevDesc.rows, 1));
    int n = 0;
    hip_check(slam_match(ctx(), prevDesc.data, prevDesc.rows, curDesc.data, curDesc.rows, type, SLAM_NORM_DEFAULT,
                         ratio, reinterpret_cast<slam_dmatch*>(matches.data()), (int)matches.size(), &n));
    matches.resize(n);
}

void matchFramesPairFeatures(Mat& firstFrame, Mat& secondFrame, std::vector<KeyPoint>& firstFeatures,
                             std::vector<KeyPoint>& secondFeatures, int matcherType, std::vector<DMatch>& matches)
{
    Mat firstDescriptor;
    extractDescriptor(firstFrame, firstFeatures, matcherType, firstDescriptor);
    matchFramesPairFeatures(firstDescriptor, secondFrame, secondFeatures, matcherType, matches);
}

void matchFramesPairFeatures(Mat& firstFrameDescriptor, Mat& secondFrame, std::vector<KeyPoint>& secondFeatures,
                             int matcherType, std::vector<DMatch>& matches)
{
    // one call: describe the candidate on the GPU and match it against the
    // previous descriptors there (no descriptor round trip through the host)
    const double ratio = configService.getValue<double>(ConfigFieldEnum::FM_KNN_DISTANCE);
    int n = (int)secondFeatures.size(), nm = 0;
    matches.resize(std::max(firstFrameDescriptor.rows, 1));
    hip_check(slam_match_frame(ctx(), firstFrameDescriptor.data, firstFrameDescriptor.rows, secondFrame.data,
                               secondFrame.cols, secondFrame.rows, secondFrame.step, secondFrame.channels(),
                               matcherType, SLAM_NORM_DEFAULT, ratio,
                               reinterpret_cast<slam_keypoint*>(secondFeatures.data()), &n,
                               reinterpret_cast<slam_dmatch*>(matches.data()), (int)matches.size(), &nm));
    secondFeatures.resize(n);
    matches.resize(nm);
    (void)matchFeaturesHIP;
}
