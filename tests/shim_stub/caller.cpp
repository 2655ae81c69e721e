// Calls every replaced entry point through the reference's declared signatures
// (shim_headers.h), so linking it with the shim objects proves the shim defines
// exactly those functions; plus definitions of the stand-ins' own externals.
#include "shim_headers.h"
#include "../config/config.h"
#include "../misc/IOmisc.h"

ConfigService configService;
LogFilesStreams logStreams;
template <> double ConfigService::getValue<double>(ConfigFieldEnum) { return 0.7; }
template <> bool ConfigService::getValue<bool>(ConfigFieldEnum) { return false; }
namespace cv {
Mat::Mat() : data(nullptr), rows(0), cols(0), step(0) {}
Mat::Mat(int r, int c, int, void* d) : data(static_cast<unsigned char*>(d)), rows(r), cols(c), step(0) {}
void Mat::create(int r, int c, int) { rows = r; cols = c; }
Mat Mat::rowRange(int, int) const { return *this; }
Mat Mat::clone() const { return *this; }
bool Mat::empty() const { return rows == 0; }
int Mat::channels() const { return 3; }
int Mat::depth() const { return CV_8U; }
template <> double& Mat::at<double>(int i) { return reinterpret_cast<double*>(data)[i]; }
template <> double& Mat::at<double>(int i, int j) { return reinterpret_cast<double*>(data)[i * cols + j]; }
void Rodrigues(const Mat&, Mat&) {}
}  // namespace cv

int main(int argc, char**)
{
    if (argc < 100) return 0;          // linked, never run (no GPU on the CPU suite)
    Mat a, b, d;
    std::vector<KeyPoint> k1, k2;
    std::vector<DMatch> m;
    std::vector<TemporalImageData> w;
    GlobalData g;
    fastExtractor(a, k1);
    fastExtractor(a, k1, 31, true, cv::FastFeatureDetector::TYPE_9_16);
    extractDescriptor(a, k1, SIFT_FLANN, d);
    matchFramesPairFeatures(a, b, k1, k2, ORB_BF, m);
    matchFramesPairFeatures(d, b, k2, SIFT_BF, m);
    bundleAdjustment(a, w, g);
    return 0;
}
