// The reference's public signatures of the replaced call sites, restated
// (featureMatching.h:12-53, featureMatchingCommon.h:8-19, fastExtractor.h:19-21,
// bundleAdjustment.h:50-54); the per-file stand-ins below include this.
#pragma once
#include <vector>
#include <opencv2/opencv.hpp>
#include "cycleProcessing/mainCycleStructures.h"
using namespace cv;
enum MatcherType { SIFT_BF, SIFT_FLANN, ORB_BF };
MatcherType getMatcherTypeIndex();
void extractDescriptor(Mat& frame, std::vector<KeyPoint>& features, int extractorType, Mat& desc);
void matchFramesPairFeatures(Mat& firstFrame, Mat& secondFrame, std::vector<KeyPoint>& firstFeatures,
                             std::vector<KeyPoint>& secondFeatures, int matcherType, std::vector<DMatch>& matches);
void matchFramesPairFeatures(Mat& firstFrameDescriptor, Mat& secondFrame, std::vector<KeyPoint>& secondFeatures,
                             int matcherType, std::vector<DMatch>& matches);
void fastExtractor(cv::Mat& srcImage, std::vector<cv::KeyPoint>& points, int threshold = 10, bool suppression = true,
                   cv::FastFeatureDetector::DetectorType type = cv::FastFeatureDetector::TYPE_9_16);
void bundleAdjustment(cv::Mat& calibrationMatrix, std::vector<TemporalImageData>& imagesDataForAdjustment,
                      GlobalData& globalData);
