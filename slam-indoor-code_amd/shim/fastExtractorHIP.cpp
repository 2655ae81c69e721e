// -D USE_HIP replacement of src/mainModule/featureExtraction/fastExtractor.cpp:7-13
// (OpenCV FastFeatureDetector::detect) -- see featureMatchingHIP.cpp for the
// build notes.  Keypoints come back in raster order with the reference's fields
// (size 7, angle -1, response = score, octave 0, class_id -1).
#include "fastExtractor.h"

#include "slamhip.h"
#include "slamhip.hpp"

void fastExtractor(cv::Mat& srcImage, std::vector<cv::KeyPoint>& points, int threshold, bool suppression,
                   cv::FastFeatureDetector::DetectorType type)
{
    auto& c = slamhip::Context::thread_default();
    points.clear();
    if (srcImage.empty()) return;
    int cap = std::max(1024, srcImage.rows * srcImage.cols / 16), n = 0;
    for (;;) {
        points.resize(cap);
        const int st = slam_fast(c.get(), srcImage.data, srcImage.cols, srcImage.rows, srcImage.step,
                                 srcImage.channels(), threshold, suppression ? 1 : 0, (int)type,
                                 reinterpret_cast<slam_keypoint*>(points.data()), cap, &n);
        if (st == SLAM_E_CAPACITY && n > cap) { cap = n; continue; }
        slamhip::check(st, &c);
        break;
    }
    points.resize(n);
}
