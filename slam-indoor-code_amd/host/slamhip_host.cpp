// slamhip C++ host layer (see slamhip.hpp): the reference's mainModule entry
// points over the C ABI.  Host-side bookkeeping only -- every pixel, descriptor
// and distance is computed by the HIP kernels behind include/slamhip.h.
#include "slamhip.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace slamhip {

ConfigService configService;

// ---- context ----------------------------------------------------------------------------

Context::Context(int device)
{
    c_ = slam_create(device);
    if (!c_) throw Error("slam_create: cannot open HIP device " + std::to_string(device));
}

Context::~Context() { slam_destroy(c_); }

Context& Context::thread_default()
{
    thread_local Context ctx(0);
    return ctx;
}

void check(int status, const Context* ctx)
{
    if (status == SLAM_OK) return;
    std::string msg = "slamhip status " + std::to_string(status);
    if (ctx && ctx->get()) msg += ": " + std::string(slam_last_error(ctx->get()));
    throw Error(msg);
}

// ---- configuration ------------------------------------------------------------------------

std::string strip_json_comments(const std::string& t)
{
    std::string out;
    out.reserve(t.size());
    bool in_str = false;
    for (size_t i = 0; i < t.size();) {
        const char c = t[i];
        if (in_str) {
            out += c;
            if (c == '\\' && i + 1 < t.size()) { out += t[i + 1]; i += 2; continue; }
            if (c == '"') in_str = false;
            ++i;
        } else if (c == '"') {
            in_str = true;
            out += c;
            ++i;
        } else if (t.compare(i, 2, "//") == 0) {
            const size_t j = t.find('\n', i);
            i = j == std::string::npos ? t.size() : j;
        } else if (t.compare(i, 2, "/*") == 0) {
            const size_t j = t.find("*/", i + 2);
            if (j == std::string::npos) throw ConfigError("Failed to parse JSON config");
            i = j + 2;
        } else {
            out += c;
            ++i;
        }
    }
    return out;
}

namespace {

// minimal JSON reader: the top level must be an object; nested values are
// skipped into ConfigValue::Other (the reference's keys are all scalars)
struct JsonReader {
    const std::string s;
    size_t i = 0;
    explicit JsonReader(std::string t) : s(std::move(t)) {}
    [[noreturn]] void fail() { throw ConfigError("Failed to parse JSON config"); }
    void ws() { while (i < s.size() && std::isspace((unsigned char)s[i])) ++i; }
    bool eat(char c) { ws(); if (i < s.size() && s[i] == c) { ++i; return true; } return false; }
    std::string str()
    {
        if (!eat('"')) fail();
        std::string o;
        while (i < s.size() && s[i] != '"') {
            if (s[i] == '\\') {
                if (++i >= s.size()) fail();
                const char e = s[i++];
                switch (e) {
                    case 'n': o += '\n'; break;
                    case 't': o += '\t'; break;
                    case 'r': o += '\r'; break;
                    case 'b': o += '\b'; break;
                    case 'f': o += '\f'; break;
                    case 'u': i += 4; o += '?'; break;      // non-ASCII escapes are not config material
                    default: o += e;
                }
            } else {
                o += s[i++];
            }
        }
        if (i >= s.size()) fail();
        ++i;
        return o;
    }
    ConfigValue value()
    {
        ws();
        if (i >= s.size()) fail();
        ConfigValue v;
        const char c = s[i];
        if (c == '"') { v.kind = ConfigValue::String; v.str = str(); return v; }
        if (c == '{' || c == '[') { skip_compound(); v.kind = ConfigValue::Other; return v; }
        if (s.compare(i, 4, "true") == 0) { i += 4; v.kind = ConfigValue::Bool; v.b = true; return v; }
        if (s.compare(i, 5, "false") == 0) { i += 5; v.kind = ConfigValue::Bool; v.b = false; return v; }
        if (s.compare(i, 4, "null") == 0) { i += 4; return v; }
        const size_t b = i;
        bool is_int = true;
        if (s[i] == '-' || s[i] == '+') ++i;
        while (i < s.size() && (std::isdigit((unsigned char)s[i]) || s[i] == '.' || s[i] == 'e' || s[i] == 'E' ||
                                s[i] == '-' || s[i] == '+')) {
            if (!std::isdigit((unsigned char)s[i])) is_int = false;
            ++i;
        }
        if (i == b) fail();
        char* end = nullptr;
        const std::string tok = s.substr(b, i - b);
        v.num = std::strtod(tok.c_str(), &end);
        if (!end || *end) fail();
        v.kind = ConfigValue::Number;
        v.is_int = is_int;
        return v;
    }
    void skip_compound()
    {
        int depth = 0;
        do {
            ws();
            if (i >= s.size()) fail();
            const char c = s[i];
            if (c == '"') { str(); continue; }
            if (c == '{' || c == '[') ++depth;
            if (c == '}' || c == ']') --depth;
            ++i;
        } while (depth > 0);
    }
    std::map<std::string, ConfigValue> object()
    {
        std::map<std::string, ConfigValue> m;
        if (!eat('{')) fail();
        if (eat('}')) return m;
        do {
            const std::string k = str();
            if (!eat(':')) fail();
            m[k] = value();
        } while (eat(','));
        if (!eat('}')) fail();
        ws();
        if (i != s.size()) fail();
        return m;
    }
};

enum Kind { KBool, KString, KInt, KFloat };
struct Field { const char* key; Kind kind; };
// configData.h:73-126, declaration order
const Field kFields[] = {
    {"onlyViz", KBool}, {"calibrate", KBool}, {"visualCalibration", KBool}, {"calibrationPath", KString},
    {"usePhotosCycle", KBool}, {"photosPathPattern", KString}, {"videoSourcePath", KString},
    {"outputDataDir", KString}, {"threadsCount", KInt}, {"useUndistortion", KBool},
    {"requiredExtractedPointsCount", KInt}, {"featureExtractingThreshold", KInt}, {"framesBatchSize", KInt},
    {"skipFramesFromBatchHead", KInt}, {"useFirstFitInBatch", KBool}, {"requiredMatchedPointsCount", KInt},
    {"useFM-SIFT-FLANN", KBool}, {"useFM-SIFT-BF", KBool}, {"useFM-ORB", KBool}, {"knnMatcherDistance", KFloat},
    {"RPUseRANSAC", KBool}, {"RPRANSACProb", KFloat}, {"RPRANSACThreshold", KFloat},
    {"RPDistanceThreshold", KFloat}, {"useBundleAdjustment", KBool}, {"BAMaxFramesCnt", KInt},
    {"BAThreadsCnt", KInt}, {"BAUseTrivialLossFunction", KBool}, {"BAUseHuberLossFunction", KBool},
    {"BAHuberLossFunctionParameter", KFloat}, {"BAUseCauchyLossFunction", KBool},
    {"BACauchyLossFunctionParameter", KFloat}, {"BAUseArctanLossFunction", KBool},
    {"BAArctanLossFunctionParameter", KFloat}, {"BAUseTukeyLossFunction", KBool},
    {"BATukeyLossFunctionParameter", KFloat}, {"TriangleMaxDistance", KFloat},
    {"TriangleEuclidDistanceWeight", KFloat}, {"TriangleColorDistance", KFloat}, {"TriangleMinimumPoints", KInt},
};

const char* kind_name(Kind k)
{
    switch (k) {
        case KBool: return "BOOLEAN";
        case KString: return "STRING";
        case KInt: return "INTEGER";
        default: return "FLOATING POINT NUMBER";
    }
}

bool kind_ok(const ConfigValue& v, Kind k)
{
    // nlohmann get<T>: bool needs a boolean; numbers accept numbers and booleans
    if (k == KBool) return v.kind == ConfigValue::Bool;
    if (k == KString) return v.kind == ConfigValue::String;
    return v.kind == ConfigValue::Number || v.kind == ConfigValue::Bool;
}

}  // namespace

void ConfigService::setConfigFile(const std::string& path)
{
    std::ifstream f(path);
    if (!f) throw ConfigError("Failed to open config file");
    std::stringstream ss;
    ss << f.rdbuf();
    setConfigText(ss.str());
}

void ConfigService::setConfigText(const std::string& text)
{
    try {
        JsonReader r(strip_json_comments(text));
        values_ = r.object();
    } catch (const ConfigError&) {
        throw ConfigError("Failed to parse JSON config\nMake sure you specified path to JSON with correct semantics");
    }
    checkJSON();
}

void ConfigService::checkJSON() const
{
    for (const Field& f : kFields) {
        auto it = values_.find(f.key);
        if (it == values_.end() || !kind_ok(it->second, f.kind))
            throw ConfigError(std::string("Field \"") + f.key + "\" missed or has incorrect type!\nCorrect type is " +
                              kind_name(f.kind));
    }
    auto it = values_.find("gpuCount");   // optional key of this build
    if (it != values_.end() && !kind_ok(it->second, KInt))
        throw ConfigError("Field \"gpuCount\" missed or has incorrect type!\nCorrect type is INTEGER");
}

template <> bool ConfigService::getValue<bool>(const std::string& key) const
{
    auto it = values_.find(key);
    if (it == values_.end() || it->second.kind != ConfigValue::Bool) throw ConfigError("config: no boolean " + key);
    return it->second.b;
}

template <> double ConfigService::getValue<double>(const std::string& key) const
{
    auto it = values_.find(key);
    if (it == values_.end()) throw ConfigError("config: no number " + key);
    if (it->second.kind == ConfigValue::Bool) return it->second.b ? 1.0 : 0.0;
    if (it->second.kind != ConfigValue::Number) throw ConfigError("config: no number " + key);
    return it->second.num;
}

template <> int ConfigService::getValue<int>(const std::string& key) const
{
    return (int)getValue<double>(key);
}

template <> std::string ConfigService::getValue<std::string>(const std::string& key) const
{
    auto it = values_.find(key);
    if (it == values_.end() || it->second.kind != ConfigValue::String) throw ConfigError("config: no string " + key);
    return it->second.str;
}

// ---- feature extraction / matching ------------------------------------------------------

namespace {

void check_image(const Image& im)
{
    if (im.rows > 0 && im.cols > 0 && !im.data) throw Error("null image data");
}

slam_keypoint* kp_ptr(std::vector<KeyPoint>& v) { return reinterpret_cast<slam_keypoint*>(v.data()); }

}  // namespace

void fastExtractor(const Image& src, std::vector<KeyPoint>& points, int threshold, bool suppression, FastType type)
{
    check_image(src);
    Context& ctx = Context::thread_default();
    points.clear();
    if (src.rows <= 0 || src.cols <= 0) return;
    int n = 0;
    int cap = std::max(1024, src.rows * src.cols / 16);
    for (;;) {
        points.resize(cap);
        const int st = slam_fast(ctx.get(), src.data, src.cols, src.rows, src.step, src.channels, threshold,
                                 suppression ? 1 : 0, (int)type, kp_ptr(points), cap, &n);
        if (st == SLAM_E_CAPACITY && n > cap) { cap = n; continue; }
        check(st, &ctx);
        break;
    }
    points.resize(n);
}

MatcherType getMatcherTypeIndex(const ConfigService& cfg)
{
    const int t = slam_matcher_type(cfg.getValue<bool>("useFM-SIFT-BF"), cfg.getValue<bool>("useFM-SIFT-FLANN"),
                                    cfg.getValue<bool>("useFM-ORB"));
    if (t < 0) throw Error("getMatcherTypeIndex: no feature matcher selected");   // reference: throw
    return (MatcherType)t;
}

void extractDescriptor(const Image& frame, std::vector<KeyPoint>& features, int extractorType, Descriptors& desc)
{
    if (extractorType < SIFT_BF || extractorType > ORB_BF)
        throw Error("extractDescriptor: invalid extractor type");                 // featureMatchingCPU.cpp:63
    check_image(frame);
    Context& ctx = Context::thread_default();
    desc.type = extractorType;
    int n = (int)features.size();
    if (extractorType == ORB_BF) desc.u8.assign((size_t)n * 32, 0);
    else desc.f32.assign((size_t)n * 128, 0.f);
    void* out = extractorType == ORB_BF ? (void*)desc.u8.data() : (void*)desc.f32.data();
    check(slam_describe(ctx.get(), frame.data, frame.cols, frame.rows, frame.step, frame.channels, extractorType,
                        kp_ptr(features), &n, out),
          &ctx);
    features.resize(n);                                                             // ORB border filter
    desc.rows = n;
    if (extractorType == ORB_BF) desc.u8.resize((size_t)n * 32);
    else desc.f32.resize((size_t)n * 128);
}

void siftDetectAndCompute(const Image& frame, std::vector<KeyPoint>& keypoints, Descriptors& desc)
{
    check_image(frame);
    Context& ctx = Context::thread_default();
    int cap = std::max(4096, frame.cols * frame.rows / 16), n = 0;
    for (;;) {
        keypoints.resize((size_t)cap);
        desc.f32.assign((size_t)cap * 128, 0.f);
        const int rc = slam_sift_detect(ctx.get(), frame.data, frame.cols, frame.rows, frame.step, frame.channels,
                                        kp_ptr(keypoints), cap, &n, desc.f32.data());
        if (rc == SLAM_E_CAPACITY && n > cap) { cap = n; continue; }
        check(rc, &ctx);
        break;
    }
    keypoints.resize((size_t)n);
    desc.type = SIFT_BF;
    desc.rows = n;
    desc.f32.resize((size_t)n * 128);
}

void reconstruct(const std::array<double, 9>& K, const std::array<double, 9>& R1, const std::array<double, 3>& t1,
                 const std::array<double, 9>& R2, const std::array<double, 3>& t2, const std::vector<Point2f>& points1,
                 const std::vector<Point2f>& points2, std::vector<Point3d>& spatialPoints)
{
    if (points1.size() != points2.size()) throw Error("reconstruct: point vectors differ in length");
    Context& ctx = Context::thread_default();
    spatialPoints.assign(points1.size(), Point3d{});
    check(slam_reconstruct(ctx.get(), K.data(), R1.data(), t1.data(), R2.data(), t2.data(),
                           reinterpret_cast<const float*>(points1.data()), reinterpret_cast<const float*>(points2.data()),
                           (int)points1.size(), reinterpret_cast<double*>(spatialPoints.data())),
          &ctx);
}

bool estimateTransformation(const std::vector<Point2f>& points1, const std::vector<Point2f>& points2,
                            const std::array<double, 9>& K, std::array<double, 9>& R, std::array<double, 3>& t,
                            std::vector<uint8_t>& chiralityMask)
{
    if (points1.size() != points2.size()) throw Error("estimateTransformation: point vectors differ in length");
    Context& ctx = Context::thread_default();
    const bool ransac = configService.getValue<bool>("RPUseRANSAC");
    const double prob = configService.getValue<double>("RPRANSACProb");
    const double thr = configService.getValue<double>("RPRANSACThreshold");
    const double dist = configService.getValue<double>("RPDistanceThreshold");
    chiralityMask.assign(points1.size(), 0);
    int passed = 0;
    check(slam_estimate_transformation(ctx.get(), reinterpret_cast<const float*>(points1.data()),
                                       reinterpret_cast<const float*>(points2.data()), (int)points1.size(), K.data(),
                                       ransac ? 1 : 0, prob, thr, dist, R.data(), t.data(), chiralityMask.data(),
                                       nullptr, &passed),
          &ctx);
    return passed > 0;
}

bool solvePnPRansac(const std::vector<Point3f>& objectPoints, const std::vector<Point2f>& imagePoints,
                    const std::array<double, 9>& K, std::array<double, 3>& rvec, std::array<double, 3>& tvec,
                    int iterationsCount, float reprojectionError, double confidence, std::vector<int>* inliers)
{
    if (objectPoints.size() != imagePoints.size()) throw Error("solvePnPRansac: point vectors differ in length");
    Context& ctx = Context::thread_default();
    const int n = (int)objectPoints.size();
    std::vector<uint8_t> mask((size_t)n);
    int ninl = 0, found = 0;
    check(slam_solve_pnp_ransac(ctx.get(), reinterpret_cast<const float*>(objectPoints.data()),
                                reinterpret_cast<const float*>(imagePoints.data()), n, K.data(), iterationsCount,
                                reprojectionError, confidence, rvec.data(), tvec.data(), mask.data(), &ninl, &found),
          &ctx);
    if (inliers) {
        inliers->clear();
        if (found)
            for (int i = 0; i < n; i++)
                if (mask[i]) inliers->push_back(i);
    }
    return found != 0;
}

void matchFramesPairFeatures(const Descriptors& first, const Image& second, std::vector<KeyPoint>& secondFeatures,
                             int matcherType, std::vector<DMatch>& matches)
{
    if (matcherType < SIFT_BF || matcherType > ORB_BF)
        throw Error("matchFeatures: invalid matcher type");                      // featureMatchingCPU.cpp:37
    check_image(second);
    Context& ctx = Context::thread_default();
    const double ratio = configService.getValue<double>("knnMatcherDistance");   // read per call (:42)
    int n = (int)secondFeatures.size();
    matches.assign(std::max(first.rows, 1), DMatch{});
    int nm = 0;
    check(slam_match_frame(ctx.get(), first.data(), first.rows, second.data, second.cols, second.rows, second.step,
                           second.channels, matcherType, SLAM_NORM_DEFAULT, ratio, kp_ptr(secondFeatures), &n,
                           reinterpret_cast<slam_dmatch*>(matches.data()), (int)matches.size(), &nm),
          &ctx);
    secondFeatures.resize(n);
    matches.resize(nm);
}

void matchFramesPairFeatures(const Image& firstFrame, const Image& secondFrame, std::vector<KeyPoint>& firstFeatures,
                             std::vector<KeyPoint>& secondFeatures, int matcherType, std::vector<DMatch>& matches)
{
    Descriptors firstDescriptor;
    extractDescriptor(firstFrame, firstFeatures, matcherType, firstDescriptor);
    matchFramesPairFeatures(firstDescriptor, secondFrame, secondFeatures, matcherType, matches);
}

void getGoodMatches(const std::vector<int>& idx, const std::vector<float>& dist, double knnMatcherDistance,
                    std::vector<DMatch>& goodMatches)
{
    goodMatches.clear();
    const size_t nq = idx.size() / 2;
    for (size_t q = 0; q < nq; q++) {
        if (idx[2 * q] < 0 || idx[2 * q + 1] < 0) continue;     // fewer than 2 neighbours
        if ((double)dist[2 * q] < knnMatcherDistance * (double)dist[2 * q + 1]) {
            DMatch m;
            m.queryIdx = (int)q;
            m.trainIdx = idx[2 * q];
            m.distance = dist[2 * q];
            goodMatches.push_back(m);
        }
    }
}

int selectGoodFrame(const std::vector<int32_t>& counts, int required, int skip, bool firstFit)
{
    return slam_select_good(counts.data(), (int)counts.size(), required, skip, firstFit ? 1 : 0);
}

// ---- bundle adjustment ----------------------------------------------------------------------

// cv::Rodrigues both ways: the library's cvRodrigues2 restatement (slam_rodrigues)
std::array<double, 3> rodrigues(const std::array<double, 9>& Rin)
{
    std::array<double, 3> r{0, 0, 0};
    slam_rodrigues(Rin.data(), 9, r.data());
    return r;
}

std::array<double, 9> rodrigues(const std::array<double, 3>& r)
{
    std::array<double, 9> R{};
    slam_rodrigues(r.data(), 3, R.data());
    return R;
}

slam_ba_summary bundleAdjustment(std::array<double, 9>& K, std::vector<TemporalImageData>& window, GlobalData& g,
                                 const ConfigService& cfg)
{
    Context& ctx = Context::thread_default();
    double K4[4] = {K[0], K[4], K[2], K[5]};
    const int nf = (int)window.size();
    std::vector<double> ext((size_t)nf * 6);
    std::vector<int32_t> of, op;
    std::vector<double> oxy;
    // AddResidualBlock order of bundleAdjustment.cpp:85-101: frame, then keypoint
    for (int i = 0; i < nf; i++) {
        const auto r = rodrigues(window[i].rotation);
        for (int q = 0; q < 3; q++) { ext[6 * i + q] = r[q]; ext[6 * i + 3 + q] = window[i].motion[q]; }
        const auto& kps = window[i].allExtractedFeatures;
        const auto& corr = window[i].correspondSpatialPointIdx;
        for (size_t p = 0; p < kps.size(); p++) {
            const int idx = corr.at(p);
            if (idx < 0) continue;
            if (idx >= (int)g.spatialPoints.size()) throw Error("bundleAdjustment: point index out of range");
            of.push_back(i);
            op.push_back(idx);
            oxy.push_back(kps[p].x);
            oxy.push_back(kps[p].y);
        }
    }
    // getLossFunction priority (bundleAdjustment.cpp:131-151)
    int loss = SLAM_LOSS_NONE;
    double par = 0;
    if (cfg.getValue<bool>("BAUseTrivialLossFunction")) {
        loss = SLAM_LOSS_TRIVIAL;
    } else {
        const char* flags[4] = {"BAUseHuberLossFunction", "BAUseCauchyLossFunction", "BAUseArctanLossFunction",
                                "BAUseTukeyLossFunction"};
        const char* pars[4] = {"BAHuberLossFunctionParameter", "BACauchyLossFunctionParameter",
                               "BAArctanLossFunctionParameter", "BATukeyLossFunctionParameter"};
        const int kinds[4] = {SLAM_LOSS_HUBER, SLAM_LOSS_CAUCHY, SLAM_LOSS_ARCTAN, SLAM_LOSS_TUKEY};
        for (int q = 0; q < 4; q++)
            if (cfg.getValue<bool>(flags[q])) { loss = kinds[q]; par = cfg.getValue<double>(pars[q]); break; }
    }
    static_assert(sizeof(Point3d) == 3 * sizeof(double), "Point3d layout");
    slam_ba_summary s{};
    check(slam_ba(ctx.get(), K4, nf, ext.data(), (int)g.spatialPoints.size(),
                  reinterpret_cast<double*>(g.spatialPoints.data()), (int)of.size(), of.data(), op.data(), oxy.data(),
                  loss, par, 0, &s),
          &ctx);
    K[0] = K4[0]; K[4] = K4[1]; K[2] = K4[2]; K[5] = K4[3];
    for (int i = 0; i < nf; i++) {
        window[i].rotation = rodrigues(std::array<double, 3>{ext[6 * i], ext[6 * i + 1], ext[6 * i + 2]});
        for (int q = 0; q < 3; q++) window[i].motion[q] = ext[6 * i + 3 + q];
    }
    return s;
}

// ---- device-resident batch search -------------------------------------------------------------

BatchResult findGoodFrameFromBatch(Context& ctx, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                                   const void* d_prev, int nprev, const BatchConditions& cond)
{
    BatchResult res;
    res.kpCounts.assign(nframes, 0);
    // extract + match in one call (one host sync): every candidate is matched,
    // and the batch filter below drops the ones the reference would not have
    // matched -- their counts never reach the selection
    std::vector<int32_t> counts(nframes, 0);
    check(slam_batch_extract_match(ctx.get(), stream, d_frames, nframes, w, h, cond.featureExtractingThreshold,
                                   cond.matcherType, d_prev, nprev, SLAM_NORM_DEFAULT, cond.knnMatcherDistance,
                                   res.kpCounts.data(), counts.data()),
          &ctx);
    for (int f = 0; f < nframes; f++)
        if (res.kpCounts[f] >= cond.requiredExtractedPointsCount) res.inBatch.push_back(f);   // batch.cpp:247
    if (res.inBatch.empty()) { res.goodIndex = SLAM_EMPTY_BATCH; return res; }
    res.matchCounts = counts;
    std::vector<int32_t> sel;
    for (int f : res.inBatch) sel.push_back(counts[f]);
    res.goodIndex = selectGoodFrame(sel, cond.requiredMatchedPointsCount, cond.skipFramesFromBatchHead,
                                    cond.useFirstFitInBatch);
    return res;
}

}  // namespace slamhip
