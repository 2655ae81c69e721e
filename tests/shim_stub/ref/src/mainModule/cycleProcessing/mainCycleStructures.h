// Stand-in for mainCycleStructures.h:38-54 (the BA window and global data types).
#pragma once
#include <vector>
#include <opencv2/opencv.hpp>
using namespace cv;
struct TemporalImageData {
    std::vector<KeyPoint> allExtractedFeatures;
    std::vector<Vec3b> colorsForAllExtractedFeatures;
    std::vector<DMatch> allMatches;
    Mat rotation;
    Mat motion;
    std::vector<int> correspondSpatialPointIdx;
};
typedef std::vector<Point3d> SpatialPointsVector;
struct GlobalData {
    SpatialPointsVector spatialPoints;
    std::vector<Vec3b> spatialPointsColors;
    std::vector<Mat> spatialCameraPositions;
    std::vector<Mat> cameraRotations;
};
