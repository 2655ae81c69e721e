// The stand-ins' out-of-line definitions: cv::Rodrigues over slam_rodrigues (the
// library's host restatement of cvRodrigues2), and the reference's globals the
// shim reads (configService, logStreams).  Test scaffolding.
#include <map>
#include <opencv2/opencv.hpp>

#include "ref/src/config/config.h"
#include "ref/src/misc/IOmisc.h"
#include "slamhip.h"

namespace cv {
void Rodrigues(const Mat& src, Mat& dst)
{
    CV_Assert(src.depth() == CV_64F && (src.total() == 3 || src.total() == 9));
    double in[9], out[9];
    const int n = (int)src.total();
    for (int i = 0; i < n; i++) in[i] = src.total() == 3 ? src.at<double>(i) : src.at<double>(i / 3, i % 3);
    if (slam_rodrigues(in, n, out) != SLAM_OK) throw std::runtime_error("Rodrigues");
    if (n == 3) {
        dst.create(3, 3, CV_64F);
        for (int i = 0; i < 9; i++) dst.at<double>(i / 3, i % 3) = out[i];
    } else {
        dst.create(3, 1, CV_64F);
        for (int i = 0; i < 3; i++) dst.at<double>(i) = out[i];
    }
}
}  // namespace cv

ConfigService configService;
LogFilesStreams logStreams;
std::map<int, double> g_config_values;   // set by the runner

template <> double ConfigService::getValue<double>(ConfigFieldEnum k) { return g_config_values.at((int)k); }
template <> bool ConfigService::getValue<bool>(ConfigFieldEnum k) { return g_config_values.at((int)k) != 0.0; }
