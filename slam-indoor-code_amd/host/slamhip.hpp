// slamhip C++ host layer: the reference's mainModule entry points over the C
// ABI of include/slamhip.h, with OpenCV-free stand-in types that are
// byte-identical to the cv ones (so the cv shim in ../shim/ only re-labels
// buffers).  Same names, argument meaning and error behaviour as the
// reference (FIT-2023-SLAM-indoor/slam-indoor-code):
//
//   fastExtractor            src/mainModule/featureExtraction/fastExtractor.h:19-21
//   extractDescriptor        src/mainModule/featureMatching/featureMatching.h:12-17
//   matchFramesPairFeatures  featureMatching.h:29-36 (6-arg), :47-53 (5-arg)
//   getMatcherTypeIndex      featureMatchingCommon.h:19 / featureMatchingCommon.cpp:13-21
//   getGoodMatches           featureMatchingCommon.h:45-48 / featureMatchingCommon.cpp:37-50
//   bundleAdjustment         src/mainModule/bundleAdjustment/bundleAdjustment.h:50-54
//   ConfigService            src/config/ConfigService.h (checkJSON semantics, config.cpp:23-51)
//   findGoodFrameFromBatch   src/mainModule/cycleProcessing/batch.cpp:59-99 (device-resident form)
//
// Errors: an invalid matcher type throws std::exception-derived slamhip::Error
// like the reference's `throw std::exception()`; a HIP/device failure throws
// slamhip::Error carrying slam_last_error().  Nothing here falls back to the CPU.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/slamhip.h"

namespace slamhip {

// ---- types (cv::KeyPoint / cv::DMatch / cv::Point3d layouts) --------------------
struct KeyPoint {
    float x = 0, y = 0, size = 0, angle = -1, response = 0;
    int32_t octave = 0, class_id = -1;
};
struct DMatch {
    int32_t queryIdx = -1, trainIdx = -1, imgIdx = 0;
    float distance = 0;
};
struct Point3d { double x = 0, y = 0, z = 0; };
struct Point3f { float x = 0, y = 0, z = 0; };
struct Point2f { float x = 0, y = 0; };   // cv::Point2f layout
static_assert(sizeof(KeyPoint) == sizeof(slam_keypoint), "KeyPoint must match cv::KeyPoint");
static_assert(sizeof(DMatch) == sizeof(slam_dmatch), "DMatch must match cv::DMatch");

enum MatcherType { SIFT_BF = 0, SIFT_FLANN = 1, ORB_BF = 2 };   // featureMatchingCommon.h:8-12
enum FastType { TYPE_5_8 = 0, TYPE_7_12 = 1, TYPE_9_16 = 2 };

// a host image: 8-bit, 1/3/4 channels (BGR order), row stride `step` bytes
struct Image {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;
    int channels = 3;
};

// descriptor matrix: SIFT rows x 128 CV_32F (integer values), ORB rows x 32 CV_8U
struct Descriptors {
    int rows = 0;
    int type = SIFT_BF;              // the extractor that produced it
    std::vector<float> f32;          // SIFT
    std::vector<uint8_t> u8;         // ORB
    bool empty() const { return rows == 0; }
    const void* data() const { return type == ORB_BF ? (const void*)u8.data() : (const void*)f32.data(); }
    int cols() const { return type == ORB_BF ? 32 : 128; }
};

class Error : public std::exception {
public:
    explicit Error(std::string m) : msg_(std::move(m)) {}
    const char* what() const noexcept override { return msg_.c_str(); }
private:
    std::string msg_;
};

// ---- context: one HIP stream + device workspace; one per thread ----------------------
class Context {
public:
    explicit Context(int device = 0);
    ~Context();
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    slam_ctx* get() const { return c_; }
    // the calling thread's context on device 0 (the reference calls
    // matchFramesPairFeatures from threadsCount std::threads, batch.cpp:181-200)
    static Context& thread_default();
private:
    slam_ctx* c_ = nullptr;
};

void check(int status, const Context* ctx = nullptr);

// ---- configuration (src/config) ------------------------------------------------------
struct ConfigValue {
    enum Kind { Null, Bool, Number, String, Other } kind = Null;
    bool b = false;
    double num = 0;
    bool is_int = false;
    std::string str;
};

class ConfigService {
public:
    void setConfigFile(const std::string& path);    // throws ConfigError (the reference exit(2)s)
    void setConfigText(const std::string& text);
    void checkJSON() const;
    bool has(const std::string& key) const { return values_.count(key) != 0; }
    template <class T> T getValue(const std::string& key) const;
    void set(const std::string& key, const ConfigValue& v) { values_[key] = v; }
private:
    std::map<std::string, ConfigValue> values_;
};

class ConfigError : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

template <> bool ConfigService::getValue<bool>(const std::string& key) const;
template <> int ConfigService::getValue<int>(const std::string& key) const;
template <> double ConfigService::getValue<double>(const std::string& key) const;
template <> std::string ConfigService::getValue<std::string>(const std::string& key) const;

// the reference's global instance (ConfigService.h: extern ConfigService configService)
extern ConfigService configService;

std::string strip_json_comments(const std::string& text);

// ---- feature extraction / matching ---------------------------------------------------
void fastExtractor(const Image& srcImage, std::vector<KeyPoint>& points, int threshold = 10,
                   bool suppression = true, FastType type = TYPE_9_16);

MatcherType getMatcherTypeIndex(const ConfigService& cfg = configService);

// features is IN/OUT: ORB removes keypoints within 31 px of the border in place
void extractDescriptor(const Image& frame, std::vector<KeyPoint>& features, int extractorType, Descriptors& desc);

// cv::SIFT::create()->detectAndCompute(frame, noArray(), kps, desc): the full
// detector (not reached by the reference's own path, which describes FAST
// keypoints); desc is n x 128 float with integer values, as SIFT::compute gives.
void siftDetectAndCompute(const Image& frame, std::vector<KeyPoint>& keypoints, Descriptors& desc);

// knnMatch(k = 2) + getGoodMatches(knnMatcherDistance from the config)
void matchFramesPairFeatures(const Descriptors& firstFrameDescriptor, const Image& secondFrame,
                             std::vector<KeyPoint>& secondFeatures, int matcherType,
                             std::vector<DMatch>& matches);
void matchFramesPairFeatures(const Image& firstFrame, const Image& secondFrame,
                             std::vector<KeyPoint>& firstFeatures, std::vector<KeyPoint>& secondFeatures,
                             int matcherType, std::vector<DMatch>& matches);

// featureMatchingCommon.cpp:37-50 over knnMatch(k = 2) rows (idx/dist nq x 2, -1 = missing)
void getGoodMatches(const std::vector<int>& idx, const std::vector<float>& dist, double knnMatcherDistance,
                    std::vector<DMatch>& goodMatches);

// selection rule of findGoodFramesFromBatch* (batch.cpp:136-146)
int selectGoodFrame(const std::vector<int32_t>& matchCounts, int requiredMatchedPointsCount,
                    int skipFramesFromBatchHead, bool useFirstFitInBatch);

// ---- bundle adjustment ---------------------------------------------------------------
struct TemporalImageData {                      // mainCycleStructures.h:38-45 (fields BA uses)
    std::vector<KeyPoint> allExtractedFeatures;
    std::vector<DMatch> allMatches;
    std::array<double, 9> rotation{1, 0, 0, 0, 1, 0, 0, 0, 1};   // row-major 3x3
    std::array<double, 3> motion{0, 0, 0};
    std::vector<int> correspondSpatialPointIdx;
};
struct GlobalData {                              // mainCycleStructures.h:49-54
    std::vector<Point3d> spatialPoints;
};

// K: row-major 3x3 (fx = K[0], fy = K[4], cx = K[2], cy = K[5]), IN/OUT.
// Loss from the config (getLossFunction priority, bundleAdjustment.cpp:131-151).
slam_ba_summary bundleAdjustment(std::array<double, 9>& calibrationMatrix,
                                 std::vector<TemporalImageData>& imagesDataForAdjustment, GlobalData& globalData,
                                 const ConfigService& cfg = configService);

// cv::Rodrigues both ways (calib3d semantics)
// reconstruct(calibration, rotation1, transition1, rotation2, transition2,
// points1, points2, spatialPoints) -- triangulate.cpp:74-100 (3 x 3 row-major)
void reconstruct(const std::array<double, 9>& K, const std::array<double, 9>& R1, const std::array<double, 3>& t1,
                 const std::array<double, 9>& R2, const std::array<double, 3>& t2, const std::vector<Point2f>& points1,
                 const std::vector<Point2f>& points2, std::vector<Point3d>& spatialPoints);

// estimateTransformation(points1, points2, calibrationMatrix, rotationMatrix,
// translationVector, chiralityMask) -- cameraTranslation.cpp:32-69; reads
// RPUseRANSAC / RPRANSACProb / RPRANSACThreshold / RPDistanceThreshold from the
// global configService as the reference does.  Returns passedPointsCount > 0.
bool estimateTransformation(const std::vector<Point2f>& points1, const std::vector<Point2f>& points2,
                            const std::array<double, 9>& K, std::array<double, 9>& R, std::array<double, 3>& t,
                            std::vector<uint8_t>& chiralityMask);

// solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs (empty),
// rvec, tvec) -- mainCycle.cpp:155-161 with OpenCV's defaults (100 iterations,
// reprojection error 8, confidence 0.99, EPnP RANSAC + iterative refinement).
// Returns the cv return value; inliers (optional) gets the inlier indices.
// Fewer than 4 points throws (OpenCV asserts); exactly 4 (P3P) throws too.
bool solvePnPRansac(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
                    const std::array<double, 9>& K, std::array<double, 3>& rvec, std::array<double, 3>& tvec,
                    int iterationsCount = 100, float reprojectionError = 8.0f, double confidence = 0.99,
                    std::vector<int>* inliers = nullptr);

std::array<double, 3> rodrigues(const std::array<double, 9>& R);
std::array<double, 9> rodrigues(const std::array<double, 3>& r);

// ---- device-resident batch search (batch.cpp:59-99) ------------------------------------
struct BatchConditions {                         // DataProcessingConditions, hot-path fields
    int featureExtractingThreshold = 10;
    int requiredExtractedPointsCount = 0;
    int skipFramesFromBatchHead = 0;
    bool useFirstFitInBatch = true;
    int requiredMatchedPointsCount = 0;
    int matcherType = SIFT_FLANN;
    double knnMatcherDistance = 0.7;
};

struct BatchResult {
    int goodIndex = SLAM_FRAME_NOT_FOUND;        // index into inBatch, or SLAM_EMPTY_BATCH / SLAM_FRAME_NOT_FOUND
    std::vector<int> inBatch;                    // frames that passed the FAST filter
    std::vector<int32_t> kpCounts, matchCounts;
};

// d_frames: nframes BGR frames (h x w x 3 u8) in device memory; d_prev: the
// previous good frame's descriptors in the internal device format
// (slam_batch_desc_bytes), also in device memory.
BatchResult findGoodFrameFromBatch(Context& ctx, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                                   const void* d_prev, int nprev, const BatchConditions& cond);

}  // namespace slamhip
