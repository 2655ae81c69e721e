/*
 * CPU ORACLE -- test infrastructure only.
 *
 * Plain-C restatement of the reference's extract -> match -> BA hot path
 * (FIT-2023-SLAM-indoor/slam-indoor-code).  The reference delegates the
 * arithmetic to OpenCV 4.8.0 and Ceres 2.2.0, neither of which is present in
 * this image, and the reference ships no tests, fixtures or golden vectors
 * (SURVEY.md section 4 / 8c).  PARITY UNPINNED against reference outputs:
 * every function here restates the upstream algorithm the reference calls
 * (cited per function), pinned only by known-answer tests derived from that
 * algorithm and by independent numpy/scipy cross-checks (tests/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * path (slam-indoor-code_amd/) never links it.
 */
#ifndef SLAM_ORACLE_H
#define SLAM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Byte-identical to cv::KeyPoint / cv::DMatch (28 B / 16 B). */
typedef struct orc_kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orc_kp;

typedef struct orc_match {
    int32_t queryIdx, trainIdx, imgIdx;
    float distance;
} orc_match;

/* MatcherType, featureMatchingCommon.h:8-12 */
enum { ORC_SIFT_BF = 0, ORC_SIFT_FLANN = 1, ORC_ORB_BF = 2 };
/* distance norms used by the reference's matchers (featureMatchingCPU.cpp:27-35,
 * featureMatchingCUDA.cpp:27-35) */
enum { ORC_NORM_L1 = 2, ORC_NORM_L2 = 4, ORC_NORM_HAMMING = 6 };

void orc_set_threads(int n);
int  orc_get_threads(void);

/* ---- gray / FAST (fastExtractor.cpp:7-13 -> FastFeatureDetector::detect) ---- */
void orc_bgr2gray(const uint8_t* bgr, int w, int h, size_t step, uint8_t* gray);
int  orc_fast_score(const uint8_t* center, const int* pixel, int threshold);
/* returns the number of keypoints found; writes min(count, cap) */
int  orc_fast(const uint8_t* gray, int w, int h, int threshold, int nms,
              orc_kp* out, int cap);
int  orc_fast_bgr(const uint8_t* bgr, int w, int h, size_t step, int threshold,
                  int nms, orc_kp* out, int cap);
/* the detector type of fastExtractor.h:19-21 (FastFeatureDetector::DetectorType):
 * FAST_t<8> / <12> / <16> */
enum { ORC_FAST_5_8 = 0, ORC_FAST_7_12 = 1, ORC_FAST_9_16 = 2 };
int  orc_fast_type(const uint8_t* gray, int w, int h, int threshold, int nms, int type,
                   orc_kp* out, int cap);
int  orc_fast_bgr_type(const uint8_t* bgr, int w, int h, size_t step, int threshold,
                       int nms, int type, orc_kp* out, int cap);

/* ---- SIFT compute on provided keypoints (featureMatchingCPU.cpp:51-65) ---- */
int   orc_gauss_kernel_f32(int n, double sigma, float* k);   /* returns n */
float orc_sift_sigma_diff(void);
float orc_fast_atan2_deg(float y, float x);
float orc_exp32f(float x);
void  orc_sift_base(const uint8_t* gray, int w, int h, float* base);
void  orc_sift_describe(const float* base, int w, int h, const orc_kp* kps,
                        int n, float* desc /* n x 128 */);
void  orc_sift_compute(const uint8_t* bgr, int w, int h, size_t step,
                       const orc_kp* kps, int n, float* desc);
void  orc_sift_one(const float* img, int cols, int rows, const orc_kp* kp, float* samples,
                   float* dst);
void  orc_sift_set_variant(int v);   /* diagnostics: 0 reference, 1 reversed, 2 fp16 inputs, 3 f64 sums */

/* siftdet.c: full SIFT detector (detectAndCompute without provided keypoints) */
int   orc_blur_ksize(double sigma);
void  orc_gauss_blur_f32(const float* src, int w, int h, double sigma, float* dst);
void  orc_resize2x_linear(const float* src, int w, int h, float* dst);
void  orc_resize_half_nearest(const float* src, int w, int h, float* dst);
int   orc_sift_octaves(int w, int h);
void  orc_sift_sigmas(double* sig);
float orc_sift_sigma_diff2x(void);
float orc_sift_ori_hist(const float* img, int cols, int rows, int px, int py, int radius,
                        float sigma, float* hist);
int   orc_sift_peaks(const float* hist, float omax, float* angles);
int   orc_kp_less(const orc_kp* a, const orc_kp* b);
int   orc_kp_dedup_sorted(orc_kp* k, int n);
int   orc_sift_detect(const uint8_t* bgr, int w, int h, size_t step, orc_kp* out, int cap,
                      float* desc);
/* geom.c: two-view DLT triangulation (reconstruct) */
double orc_hypot(double x, double y);
void orc_projection(const double K[9], const double R[9], const double t[3], double P[12]);
void orc_triangulate_point(const double P1[12], const double P2[12], double x1, double y1,
                           double x2, double y2, double X[4]);
void orc_reconstruct(const double K[9], const double R1[9], const double t1[3],
                     const double R2[9], const double t2[3], const float* pts1,
                     const float* pts2, int n, double* out);
/* essential.c: estimateTransformation (findEssentialMat RANSAC + recoverPose) */
int   orc_ep_subsets(int count, int iters, int* idx);
int   orc_ransac_update_iters(double p, double ep, int modelPoints, int maxIters);
int   orc_five_point(const double* q1, const double* q2, double* Es);
float orc_sampson(const double E[9], double x1, double y1, double x2, double y2);
int   orc_find_essential(const float* p1, const float* p2, int n, const double K[9], double prob,
                         double threshold, double E[9], uint8_t* mask, int* niters_used);
void  orc_decompose_essential(const double E[9], double R1[9], double R2[9], double t[3]);
int   orc_cheirality_bits(const double R1[9], const double R2[9], const double t[3], double dist,
                          double x1, double y1, double x2, double y2);
int   orc_recover_pose(const double E[9], const float* p1, const float* p2, int n, const double K[9],
                       double dist, double R[9], double t[3], uint8_t* mask);
int   orc_estimate_transformation(const float* p1, const float* p2, int n, const double K[9],
                                  int use_ransac, double prob, double threshold, double dist,
                                  double R[9], double t[3], uint8_t* chirality,
                                  uint8_t* ransac_mask, int* passed);
void  orc_jsvd(double* At, int n, int m, double* W, double* Vt);
/* pnp.c: solvePnPRansac (EPnP RANSAC + iterative LM refinement) */
void  orc_rodrigues_v2m(const double rv[3], double R[9], double J[27]);
void  orc_rodrigues_m2v(const double R[9], double rv[3]);
void  orc_epnp(int n, const double* op, const float* ip, const double K[9], double R[9], double t[3]);
float orc_pnp_error(const double R[9], const double t[3], const double K[9], const float* o, const float* m);
int   orc_pnp_iterative(const double* op, const double* ip, int n, const double K[9], double rvec[3],
                        double tvec[3]);
int   orc_solve_pnp_ransac(const float* op, const float* ip, int n, const double K[9], int iterationsCount,
                           float reprojectionError, double confidence, double rvec[3], double tvec[3],
                           uint8_t* mask, int* ninliers);
int   orc_sift_pyr_dims(int w, int h, int* ow, int* oh);
void  orc_sift_pyramid(const uint8_t* gray, int w, int h, float* gauss, float* dog);

/* ---- ORB compute on provided keypoints (featureMatchingCPU.cpp:59-65) ---- */
int  orc_orb_filter(const orc_kp* kps, int n, int w, int h, int border,
                    orc_kp* out);
void orc_orb_blur(const uint8_t* gray, int w, int h, uint8_t* out);
void orc_orb_describe(const uint8_t* blurred, int w, int h, const orc_kp* kps,
                      int n, uint8_t* desc /* n x 32 */);
/* filters kps in place (reference mutates the caller's vector); returns new n */
int  orc_orb_compute(const uint8_t* bgr, int w, int h, size_t step,
                     orc_kp* kps, int n, uint8_t* desc);

/* ---- k=2 brute-force kNN + Lowe ratio (featureMatchingCPU.cpp:17-43,
 *      featureMatchingCommon.cpp:37-50) ---- */
/* q/t: float rows of `dim` (L1/L2) or byte rows of `dim` bytes (Hamming).
 * idx/dist: nq x 2, idx = -1 where fewer than two train rows exist. */
void orc_knn2_l2_u8(const uint8_t* q, int nq, const uint8_t* t, int nt, int* idx, float* dist);
void orc_knn2(const void* q, int nq, const void* t, int nt, int dim, int norm,
              int* idx, float* dist);
int  orc_ratio(const int* idx, const float* dist, int nq, double ratio,
               orc_match* out);
/* FLANN-equivalent randomized KD-forest (KDTreeIndexParams(4), SearchParams(32)):
 * approximate, used only to time the reference's useFM-SIFT-FLANN CPU path. */
void orc_flann_knn2(const float* q, int nq, const float* t, int nt, int dim,
                    int trees, int checks, uint64_t seed, int* idx, float* dist);
/* batch.cpp:101-160 selection rule over per-candidate match counts (index order
 * = batch index).  Returns goodIndex or -1 (FRAME_NOT_FOUND). */
int  orc_select_good(const int* counts, int n, int required, int skip_head,
                     int first_fit);

/* ---- windowed bundle adjustment (bundleAdjustment.cpp:73-201) ---- */
enum { ORC_LOSS_NONE = 0, ORC_LOSS_TRIVIAL = 1, ORC_LOSS_HUBER = 2,
       ORC_LOSS_CAUCHY = 3, ORC_LOSS_ARCTAN = 4, ORC_LOSS_TUKEY = 5 };
typedef struct orc_ba_summary {
    double initial_cost, final_cost;
    int num_residuals, iterations, successful_steps, termination;
    int usable;
} orc_ba_summary;
void orc_aa_rotate(const double aa[3], const double p[3], double out[3]);
void orc_loss_eval(int loss, double a, double s, double rho[3]);
int  orc_ba(double K4[4], int nframes, double* ext6 /* nframes x 6 */,
            int npoints, double* pts3 /* npoints x 3 */, int nobs,
            const int* obs_frame, const int* obs_point, const double* obs_xy,
            int loss, double loss_param, int max_iters, orc_ba_summary* sum);
void orc_ba_set_trace(double* cost, int cap);
void orc_ba_set_solver(int kind /* 0 LL', 1 SimplicialLDLT */, const int* cam_perm /* nc or NULL */);
double orc_ba_cost(const double K4[4], const double* ext6, const double* pts3,
                   int nobs, const int* obs_frame, const int* obs_point,
                   const double* obs_xy, int loss, double loss_param);

#ifdef __cplusplus
}
#endif
#endif
