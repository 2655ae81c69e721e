// Internal declarations of libslamhip: context, device workspace, kernel launch
// entry points.  Everything here is MI355X (gfx950) HIP; nothing is a fallback.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <utility>
#include <string>
#include <vector>

#include "../../include/slamhip.h"

namespace slamhip {

// Correctly rounded f32 sqrt / divide on gfx950.  The __fsqrt_rn / __fdiv_rn
// builtins lower to the 1-ulp hardware instructions; computing in f64 (IEEE
// correctly rounded) and rounding once to f32 is exact for these ops, because
// 53 >= 2 * 24 + 2 makes the double rounding innocuous.
__device__ __forceinline__ float cr_sqrtf(float x) { return (float)sqrt((double)x); }
__device__ __forceinline__ float cr_divf(float a, float b) { return (float)((double)a / (double)b); }

// ---- numeric constants shared by kernels and host (restated from OpenCV) ----
constexpr int kSiftD = 4, kSiftN = 8;
constexpr int kSiftHist = (kSiftD + 2) * (kSiftD + 2) * (kSiftN + 2);  // 360
constexpr int kSiftDescBytes = 128;
constexpr int kOrbDescBytes = 32;
constexpr int kOrbExpBytes = 128;      // +-1 FP4 (e2m1) expansion of the 256 bits for the MFMA Hamming path
constexpr int kOrbEdge = 31;           // ORB edgeThreshold, runByImageBorder

// FAST tiles: 64 columns (one wave, one ballot per row) x 16 rows
constexpr int kFastTileW = 64, kFastTileH = 16;

struct SiftConsts {
    float gauss[16];   // 13-tap kernel of GaussianBlur(sigma = sig_diff)
    int ksize;
    float exptab[64];  // hal::exp32f table
};

// SIFT gradient map {magnitude, orientation} (sift_blur_grad): every frame is
// stored with a zero border of kGradPad pixels on each side, so a descriptor
// window of radius <= kGradPad around any in-image keypoint reads zeros (a +0
// contribution, exactly what the reference's 0 < r < rows - 1 test gives)
// instead of testing bounds per sample.  Pixel (f, y, x) lives at element
// f * grad_frame(w, h) + grad_origin(w) + y * grad_pitch(w) + x; the pitch is
// a multiple of 8 elements (64-byte rows) and grad_origin is even, so pixel
// parity is preserved (sift_tab's 16-byte pair loads).
constexpr int kGradPad = 48;
__host__ __device__ __forceinline__ int grad_pitch(int w) { return (w + 2 * kGradPad + 7) & ~7; }

// XCD-contiguous tile order for a 3-D grid of image tiles (x, y, frame):
// workgroups are dealt round-robin over the 8 XCDs by linear id, so raster-
// adjacent tiles land on different XCDs (separate L2s) and each fetches the
// halo rows it shares with its neighbours.  Here XCD k takes the k-th eighth of
// the tiles in raster order: neighbours (and the tiles in flight at once) share
// an L2.  The same tiles, each exactly once; on = false: the plain mapping.
// Measured (profiles/r5_xcd_ab.txt): FETCH_SIZE per launch 2.60 -> 1.19 GB
// (fast_detect) and 1.68 -> 0.40 GB (sift_blur_grad), but neither kernel is
// HBM-bound and both ran 2-3 % slower, so it is opt-in: SLAMHIP_XCD_TILES=1.
inline bool xcd_tiles_on()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_XCD_TILES"); return e && e[0] == '1'; }();
    return on;
}
// Timing probes that deliberately break results (SLAMHIP_FAST_DBG,
// SLAMHIP_SD_DBG) are read only in builds with -DSLAMHIP_DIAG; a normal build
// returns 0 and says once on stderr that it ignored the variable.
inline int diag_env_int(const char* name)
{
    const char* e = getenv(name);
    if (!e || !e[0]) return 0;
#ifdef SLAMHIP_DIAG
    return atoi(e);
#else
    fprintf(stderr, "slamhip: %s ignored (result-breaking timing probe; build with -DSLAMHIP_DIAG)\n", name);
    return 0;
#endif
}
#ifdef __HIPCC__
__device__ __forceinline__ void xcd_tile(bool on, int& x, int& y, int& z)
{
    x = blockIdx.x; y = blockIdx.y; z = blockIdx.z;
    if (!on) return;
    const unsigned gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
    const unsigned lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const unsigned per = n >> 3;
    if (lin >= (per << 3)) return;          // the last n % 8 tiles keep their place
    const unsigned v = (lin & 7) * per + (lin >> 3);
    x = (int)(v % gx);
    y = (int)((v / gx) % gy);
    z = (int)(v / (gx * gy));
}
#endif
__host__ __device__ __forceinline__ size_t grad_frame(int w, int h)
{
    return (size_t)grad_pitch(w) * (size_t)(h + 2 * kGradPad);
}
__host__ __device__ __forceinline__ size_t grad_origin(int w) { return (size_t)kGradPad * grad_pitch(w) + kGradPad; }

// chunked per-target SIFT sample table (sift_tab.hip)
struct SiftTabMeta {
    int len;           // table rows (entries per target, padded; a multiple of the pipeline depth)
    int radius;
    float ori_deg;
};

// band-staged SIFT tables for one (angle, size) (sift_band.hip)
struct SiftBandMeta {
    int nrec = 0, nchunks = 0;
    int pitch = 0;      // grad_pitch the table's window offsets were built for
    bool neg = false;   // floor(obin) always in [-9, -1]
    int band_first[6] = {0, 0, 0, 0, 0, 0};
    int radius = 0;
    float ori_deg = 0.f;
};

// sift_desc_cols tables (sift_cols.hip): two column passes, each band-major
struct SiftColsMeta {
    int nrec = 0, nchunks = 0;
    int band_first[2][6] = {{0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0}};
};

// sift_desc_colw tables (sift_colw.hip): one sample list per descriptor column, band-major
struct SiftColwMeta {
    int nrec = 0, nchunks = 0;
    int band_first[4][6] = {};
};

struct OrbConsts {
    float gauss[8];    // 7-tap kernel of GaussianBlur(7x7, sigma = 2)
};

// grow-only device buffer
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n);
    void release();
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// the gradient map's zero border as last written by sift_blur_grad: buffer
// (pointer + size: a reallocation changes the size), geometry, frames covered
struct SiftGradBorder {
    void* p = nullptr;
    size_t bytes = 0;
    int w = 0, h = 0, frames = 0;
    int obin = 0;          // the stored orientation form of the border (launch_sift_base)
    float ori_deg = 0.f;
    void* pp = nullptr;    // obin 2: the slot-position byte plane (gradpos) the border went to
    size_t pbytes = 0;
};

// events bracketing every launch of a kernel family (bench.py roofline timing)
struct ProfFamily {
    std::vector<hipEvent_t> ev;   // pairs
    int used = 0;
};

struct BatchState {
    int nframes = 0, w = 0, h = 0, matcher = -1, ntx = 0, nbands = 0;
    int total_kps = 0;
    std::vector<int32_t> kp_counts_raw;   // FAST counts (batch filter input)
    std::vector<int32_t> kp_counts;       // descriptor-bearing keypoints (ORB: border-filtered)
    std::vector<int32_t> kp_offsets;      // exclusive prefix of kp_counts
    int matched_nq = 0;                   // query count of the last slam_batch_match
    bool have_matches = false;
    bool have_desc = false;               // false after slam_batch_fast (keypoints only)
    int est_max_nt = 0;                   // largest per-frame count of the previous batch (fused path)
    // drop the published batch (frame count first: nothing indexes the vectors after this)
    void unpublish()
    {
        nframes = 0;
        have_matches = false;
        have_desc = false;
        total_kps = 0;
        kp_counts_raw.clear();
        kp_counts.clear();
        kp_offsets.clear();
    }
};

}  // namespace slamhip

namespace slamhip {
// slam_sift_detect_batch: frames per call (the pyramid is ~0.5 GB per 1080p
// frame; candidate / keypoint scratch is 1M entries per frame, int-indexed)
constexpr int kSiftDetectMaxFrames = 256;
}  // namespace slamhip

struct slam_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_sync = nullptr;     // stream_sync's polled event
    std::string err;
    slamhip::SiftConsts sift;
    slamhip::OrbConsts orb;
    int cu_count = 256;

    // batch workspace (device)
    slamhip::DevBuf gray, scores, masks, band_cnt, band_pref, frame_info;
    slamhip::DevBuf ftmp, grad, orbblur;   // grad: float2 {mag, ori} per pixel
    slamhip::DevBuf gradpos;               // obin 2: one slot-position byte per grad pixel
    slamhip::SiftGradBorder grad_border;
    slamhip::DevBuf kps, kp_frame, desc_u8, desc_f32, desc_norm, desc_exp;
    slamhip::DevBuf query_norm, knn_part, match_rec, match_flag, match_cnt, match_out;
    void* h_rb = nullptr;     // pinned host readback buffer (small D2H results: counts, totals)
    size_t h_rb_bytes = 0;
    void* h_up = nullptr;     // pinned host image staging (upload_image); ev_up: its last copy
    size_t h_up_bytes = 0;
    hipEvent_t ev_up = nullptr;
    // slam_batch_result_begin / _end: a winner's keypoints + matches in flight
    void* h_win = nullptr;
    size_t h_win_bytes = 0;
    hipEvent_t ev_win = nullptr;
    hipEvent_t ev_rdev = nullptr;      // slam_batch_result_dev's copies on a caller stream
    slamhip::DevBuf synth_world, synth_cams;   // slam_synth_sequence_dev: world texture, per-frame cameras
    int synth_w = 0, synth_h = 0;
    uint64_t synth_seed = 0;
    int win_pending = 0, win_nk = 0;
    size_t win_kb = 0;
    slamhip::DevBuf frames_in, qbuf, tbuf, misc;
    slamhip::BatchState batch;

    // BA workspace
    slamhip::DevBuf ba_obs, ba_par, ba_jac, ba_red, ba_S, ba_aux;

    // full SIFT detector (siftdet.hip): Gaussian + DoG pyramid, candidates, keypoints
    slamhip::DevBuf sd_pyr, sd_cand, sd_kps, sd_kpc;   // sd_kpc: the refined keypoints, frame-major
    // two-view geometry (geom.hip)
    slamhip::DevBuf geom;

    // SIFT gather table for one (angle, size) (sift_tab.hip)
    slamhip::DevBuf sift_tab;
    bool sift_tab_valid = false;
    float sift_tab_angle = 0.f, sift_tab_size = 0.f;
    int sift_tab_nrec = 0;
    slamhip::SiftTabMeta sift_meta;
    // band-staged SIFT tables (sift_band.hip)
    slamhip::DevBuf sift_band_buf;
    slamhip::DevBuf sift_split;          // sift_desc_band split tail: the halves' rows
    slamhip::DevBuf sift_split_cnt;      // ... and their arrival counters (zero between launches)
    bool sift_band_valid = false;
    float sift_band_angle = 0.f, sift_band_size = 0.f;
    slamhip::SiftBandMeta sift_band;
    // one-keypoint-per-lane two-pass tables (sift_cols.hip), built with the band tables
    slamhip::DevBuf sift_cols_buf;
    slamhip::DevBuf sift_cols_park;      // sift_desc_cols: pass 0's finished rows per lane
    bool sift_cols_valid = false;
    slamhip::SiftColsMeta sift_cols;
    // column-per-wave tables (sift_colw.hip), built with the band tables
    slamhip::DevBuf sift_colw_buf;
    bool sift_colw_valid = false;
    slamhip::SiftColwMeta sift_colw;

    bool prof_on = false;
    slamhip::ProfFamily prof[8];
    // slam_set_option: which SIFT descriptor kernel runs (all bit-identical)
    int opt_sift_kernel = SLAM_SIFT_KERNEL_AUTO;
    int opt_band_split = SLAM_BAND_SPLIT_AUTO;
    int opt_pnp_sums = SLAM_PNP_SUMS_ORDERED;
    int opt_fast_reuse = 0;               // SLAM_OPT_FAST_REUSE: off unless the caller vouches for the frames
    // FAST results left by slam_batch_fast (gray, masks, scores, band counts, the
    // emitted keypoint list and frame table): with SLAM_OPT_FAST_REUSE on when
    // slam_batch_fast ran, a batch extraction of the same frames at the same
    // threshold, border and capacity takes them instead of detecting again.  fast_gen counts every launch that rewrites any of them
    // (launch_gray*, launch_fast_detect, launch_fast_emit); the record is valid
    // while its gen is the current one.
    uint64_t fast_gen = 0;
    struct FastReuse {
        const void* frames = nullptr;
        int nframes = 0, w = 0, h = 0, thr = -1, border = -1, cap = 0;
        uint64_t gen = ~0ull;
    } fast_reuse;
    bool fast_reused = false;   // the last batch extraction took them (slam_batch_fast_reused)
    int last_sift_kernel = 0;             // SLAM_SIFT_KERNEL_* of the last descriptor launch
    hipEvent_t ev_order = nullptr;        // slam_order_after
    hipEvent_t ev_stage[2] = {nullptr, nullptr};   // the last extraction's descriptor start / end
    bool stage_recorded = false;
    // slam_batch_extract_async / _match_async / slam_batch_finish: one batch in flight
    struct Async {
        int state = 0;                    // 0 none, 1 extraction queued, 2 match queued too
        hipStream_t s = nullptr;
        int nframes = 0, w = 0, h = 0, matcher = 0, cap = 0;
        bool committed = false;           // the host batch state is already published
        int launched = 0, norm = 0, nq = 0;
        double ratio = 0;
        const void* query = nullptr;
    } async;
    void* h_async = nullptr;              // pinned: frame table + total + match counts of the batch in flight
    size_t h_async_bytes = 0;
    // slam_sift_detect_batch's host scratch, kept between calls (no fresh pages per call)
    std::vector<std::vector<slam_keypoint>> sd_per;
    std::vector<std::vector<std::pair<float, int>>> sd_ord;
};

namespace slamhip {

int set_err(slam_ctx* c, int code, const std::string& msg);
#define SLAM_HIP(ctx, call)                                                              \
    do {                                                                                 \
        hipError_t e__ = (call);                                                         \
        if (e__ != hipSuccess)                                                           \
            return ::slamhip::set_err((ctx), SLAM_E_HIP,                                 \
                                      std::string(#call) + ": " + hipGetErrorString(e__)); \
    } while (0)

// wait for everything queued on s; poll: spin on an event (short waits on the
// hot paths: batch steps, LM iterations) instead of a blocking wait
int stream_sync(slam_ctx* c, hipStream_t s, bool poll = false);
// pinned host readback space of at least n bytes (grown on demand; one per context)
void* readback(slam_ctx* c, size_t n);
// fn(0 .. n-1) on the process's persistent host thread pool (up to 16 threads,
// the caller included; siftdet.hip); items must be independent
void host_parallel_run(int n, const std::function<void(int)>& fn);
// a host copy of n bytes split over the pool (large staging copies)
void host_copy(void* dst, const void* src, size_t n);
void prof_begin(slam_ctx* c, int fam, hipStream_t s);
void prof_end(slam_ctx* c, int fam, hipStream_t s);

// host-side restatements shared with kernels (bit-identical to the oracle's)
void init_consts(slam_ctx* c);
float sift_sigma_diff();
int gauss_kernel_f32(int n, double sigma, float* k);
float host_exp32f(float x, const float* tab);

// ---- kernel launchers (fast.hip, sift.hip, orb.hip, knn.hip) ----
// gray + FAST + NMS over nframes BGR/gray frames; writes gray, masks, scores,
// per-band counts (raw and border-filtered)
hipError_t launch_fast_detect(slam_ctx* c, hipStream_t s, const uint8_t* img, size_t frame_stride,
                              size_t row_stride, int channels, int nframes, int w, int h,
                              int threshold, int nonmax, int border, int type = SLAM_FAST_TYPE_9_16);
hipError_t launch_gray(slam_ctx* c, hipStream_t s, const uint8_t* img, size_t row_stride, int channels, int w,
                       int h);
// prefix sums of band counts -> frame_info; emits keypoints in raster order
hipError_t launch_fast_emit(slam_ctx* c, hipStream_t s, int nframes, int w, int h, int cap);

// obin: store obin = (ori - ori_deg) * 8 / 360 per pixel (for sift_desc_band with
// keypoints of orientation ori_deg) instead of the orientation
hipError_t launch_sift_base(slam_ctx* c, hipStream_t s, int nframes, int w, int h, int obin = 0, float ori_deg = 0.f);
hipError_t launch_sift_desc(slam_ctx* c, hipStream_t s, int nframes, int w, int h,
                            const float* d_kp_cs, int cap, int write_f32);
bool sift_tab_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h);
hipError_t launch_sift_desc_tab(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32);
// window samples of one keypoint geometry (sift_band.hip)
struct BandSample { int i, j, r0, c0; float rf, cf, wexp; };
struct BandGeometry {
    int radius = 0, pitch = 0, pos_base = 1;
    float ori = 0.f;
    bool neg = false;                  // floor(obin) always in [-9, -1]
    std::vector<BandSample> smp;       // raster order
};
int sift_band_radius(float kp_size);
bool sift_band_geometry(slam_ctx* c, float kp_angle, float kp_size, int w, int h, BandGeometry& g);
bool sift_band_raster_ok(const BandGeometry& g, const std::vector<int>& sched);
bool sift_band_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h);
// obin: the gradient map holds obin (launch_sift_base with obin, this table's ori_deg)
hipError_t launch_sift_desc_band(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32, int obin);
int sift_band_obin_mode(const slam_ctx* c);
bool sift_band4_enabled();
bool sift_cols_enabled();
bool sift_colw_enabled();
bool sift_colw_prepare(slam_ctx* c, hipStream_t s, const BandGeometry& geo);
hipError_t launch_sift_desc_colw(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32);
bool sift_cols_prepare(slam_ctx* c, hipStream_t s, const BandGeometry& geo);
hipError_t launch_sift_desc_cols(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32);
hipError_t launch_orb_blur(slam_ctx* c, hipStream_t s, int nframes, int w, int h);
hipError_t launch_orb_desc(slam_ctx* c, hipStream_t s, int nframes, int w, int h, const float* d_kp_ab,
                           int cap);
hipError_t launch_norms_u8(hipStream_t s, const uint8_t* d, int n, int32_t* norms);
hipError_t launch_orb_expand(hipStream_t s, const uint8_t* d, int n, int8_t* out);

// kNN top-2: queries (nq, shared) vs nframes train sets described by frame_info
// (offset/count per frame); kb = 128 (SIFT u8) or 256 (ORB +-1 i8)
hipError_t launch_knn(slam_ctx* c, hipStream_t s, int kb, const void* q, const int32_t* qnorm, int nq,
                      const void* t, const int32_t* tnorm, const int32_t* t_info, int nframes,
                      int max_nt, int norm_kind, int tsplit, int4* part);
// merge partial top-2, apply the ratio test, count survivors per frame
hipError_t launch_knn_finish(slam_ctx* c, hipStream_t s, const int4* part, int nq, int nframes,
                             int tsplit, const int32_t* qnorm, int norm_kind, double ratio,
                             const int32_t* t_info, int2* top_idx, float2* top_dist,
                             slam_dmatch* rec, uint8_t* flag, int32_t* counts);
hipError_t launch_compact(slam_ctx* c, hipStream_t s, const slam_dmatch* rec, const uint8_t* flag,
                          int nq, int nframes, slam_dmatch* out, int32_t* out_counts, int stride);

// ---- full SIFT detector (siftdet.hip) ----
// img: device frame (launch_gray layout); keypoints / descriptors to host memory
int sift_detect(slam_ctx* c, const uint8_t* dimg, size_t dstep, int channels, int w, int h, slam_keypoint* out,
                int cap, int* n_out, float* desc);
int sift_detect_batch(slam_ctx* c, hipStream_t s, const uint8_t* d_frames, int nframes, int w, int h, int channels,
                      slam_keypoint* out, int cap, int* n_out, float* desc);
hipError_t launch_gray_batch(slam_ctx* c, hipStream_t s, const uint8_t* frames, int nframes, int w, int h, int channels);
// host cosf / sinf of 360 - angle per keypoint (calcSIFTDescriptor's rotation)
void sift_kp_cs(const slam_keypoint* k, int n, std::vector<float>& cs);

// ---- two-view triangulation (geom.hip) ----
int triangulate(slam_ctx* c, const double* K, const double* R1, const double* t1, const double* R2,
                const double* t2, const float* pts1, const float* pts2, int n, double* out);

// ---- relative pose: findEssentialMat (RANSAC) + recoverPose (essential.hip) ----
int relative_pose(slam_ctx* c, const float* p1, const float* p2, int n, const double* K, int use_ransac,
                  double prob, double threshold, double dist, double* R, double* t, uint8_t* chirality,
                  uint8_t* ransac_mask, int* passed);

// ---- RANSACPointSetRegistrator pieces shared by essential.hip and pnp.hip ----
// cv::RNG (multiply-with-carry, state (uint64)-1 in ptsetreg.cpp)
struct CvRng {
    uint64_t s;
    unsigned next() { s = (uint64_t)(unsigned)s * 4164903690u + (unsigned)(s >> 32); return (unsigned)s; }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};
// getSubset for callbacks whose checkSubset accepts everything: iters x 5 indices
void ransac_subsets5(int count, int iters, int* idx);
int ransac_update_iters(double p, double ep, int modelPoints, int maxIters);

// ---- solvePnPRansac: EPnP RANSAC + iterative refinement (pnp.hip) ----
int pnp_ransac(slam_ctx* c, const float* op, const float* ip, int n, const double* K, int iterations,
               float reproj, double confidence, double* rvec, double* tvec, uint8_t* mask, int* ninliers,
               int* found);

// ---- BA (ba.hip) ----
int ba_solve(slam_ctx* c, double* K4, int nframes, double* ext6, int npoints, double* pts3, int nobs,
             const int32_t* of, const int32_t* op, const double* oxy, int loss, double a,
             int max_iters, slam_ba_summary* sum);

}  // namespace slamhip

// packed keypoint-frame info: frame_info[f] = {offset, count, raw_count, 0}
