/*
 * slamhip -- MI355X (gfx950) implementation of the reference's extract -> match
 * -> windowed-BA hot path, exposed as a plain C ABI (no OpenCV / torch types).
 *
 * Each entry point names the reference interface it replaces (paths relative
 * to the reference repo, FIT-2023-SLAM-indoor/slam-indoor-code):
 *
 *   slam_fast            fastExtractor                 src/mainModule/featureExtraction/fastExtractor.h:19-21
 *   slam_describe        extractDescriptor             src/mainModule/featureMatching/featureMatching.h:12-17
 *   slam_match           matchFeatures + getGoodMatches featureMatchingCPU.cpp:17-43, featureMatchingCommon.cpp:37-50
 *   slam_match_frame     matchFramesPairFeatures (5-arg) featureMatching.h:47-53
 *   slam_knn2            DescriptorMatcher::knnMatch(k=2) featureMatchingCPU.cpp:40 / featureMatchingCUDA.cpp:41
 *   slam_matcher_type    getMatcherTypeIndex           featureMatchingCommon.h:19, featureMatchingCommon.cpp:13-21
 *   slam_select_good     findGoodFramesFromBatch* selection rule  batch.cpp:136-146 / :280-316
 *   slam_ba              bundleAdjustment              src/mainModule/bundleAdjustment/bundleAdjustment.h:50-54
 *   slam_batch_*         the data-parallel candidate scan around them, batch.cpp:59-226
 *
 * Conventions
 *   - Every call returns an int status (SLAM_OK = 0); no C++ exception crosses
 *     the ABI.  The reference's own error behaviour (throw std::exception on an
 *     invalid matcher type, featureMatchingCPU.cpp:37,63) is reproduced by the
 *     host mirror on top of SLAM_E_BAD_MATCHER.
 *   - slam_keypoint / slam_dmatch are byte-identical to cv::KeyPoint (28 B) and
 *     cv::DMatch (16 B), so a cv::Mat / std::vector buffer can be passed as is.
 *   - Host-pointer calls copy in, run on the context's HIP stream and copy out.
 *     slam_batch_* calls take device pointers and an optional HIP stream and
 *     keep every intermediate in HBM.
 *   - A context is NOT re-entrant across threads; the reference calls
 *     matchFramesPairFeatures from threadsCount std::threads (batch.cpp:181-200):
 *     give each thread its own context (contexts on one device share the GPU).
 */
#ifndef SLAMHIP_H
#define SLAMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLAMHIP_ABI_VERSION 3   /* 3: slam_sift_detect_batch; 2: ORB device descriptors as 128-byte FP4 (e2m1) +-1, batch async / stage / result_dev calls, synth paths */

enum slam_status {
    SLAM_OK = 0,
    SLAM_E_INVALID_ARG = -1,
    SLAM_E_BAD_MATCHER = -2,   /* reference: throw std::exception() */
    SLAM_E_HIP = -3,
    SLAM_E_CAPACITY = -4,      /* output buffer too small; *n_out holds the needed size */
    SLAM_E_NO_DEVICE = -5,
    SLAM_E_UNSUPPORTED = -6,
    SLAM_E_SOLVER = -7
};

/* MatcherType, featureMatchingCommon.h:8-12 */
enum slam_matcher { SLAM_SIFT_BF = 0, SLAM_SIFT_FLANN = 1, SLAM_ORB_BF = 2 };

/* distance norms (cv::NORM_* values).  SLAM_NORM_DEFAULT picks the reference's
 * CPU build: SIFT_BF -> L2, SIFT_FLANN -> exact BF L2 (what the reference's CUDA
 * build runs, featureMatchingCUDA.cpp:31; the CPU build's FLANN is approximate),
 * ORB -> Hamming.  SLAM_NORM_L1 gives the CUDA build's SIFT_BF (:28). */
enum slam_norm { SLAM_NORM_DEFAULT = 0, SLAM_NORM_L1 = 2, SLAM_NORM_L2 = 4, SLAM_NORM_HAMMING = 6 };

/* cv::FastFeatureDetector::DetectorType */
enum slam_fast_type { SLAM_FAST_TYPE_5_8 = 0, SLAM_FAST_TYPE_7_12 = 1, SLAM_FAST_TYPE_9_16 = 2 };

/* robust losses, getLossFunction priority bundleAdjustment.cpp:131-151 */
enum slam_loss { SLAM_LOSS_NONE = 0, SLAM_LOSS_TRIVIAL = 1, SLAM_LOSS_HUBER = 2,
                 SLAM_LOSS_CAUCHY = 3, SLAM_LOSS_ARCTAN = 4, SLAM_LOSS_TUKEY = 5 };

/* batch.h:5-6 */
#define SLAM_EMPTY_BATCH (-2)
#define SLAM_FRAME_NOT_FOUND (-1)

typedef struct slam_keypoint {      /* == cv::KeyPoint */
    float x, y, size, angle, response;
    int32_t octave, class_id;
} slam_keypoint;

typedef struct slam_dmatch {        /* == cv::DMatch */
    int32_t queryIdx, trainIdx, imgIdx;
    float distance;
} slam_dmatch;

typedef struct slam_ba_summary {    /* the ceres::Solver::Summary fields the reference logs (:119-127) */
    double initial_cost, final_cost;
    int32_t num_residuals, iterations, successful_steps;
    int32_t termination;            /* 0 no convergence, 1 convergence, 2 min radius, 3 failure */
    int32_t usable;                 /* Summary::IsSolutionUsable() */
    double total_time_in_seconds;
} slam_ba_summary;

typedef struct slam_ctx slam_ctx;

/* ---- context ---------------------------------------------------------------- */
int         slam_abi_version(void);
int         slam_device_count(void);              /* cuda::getCudaEnabledDeviceCount, main.cpp:31 */
slam_ctx*   slam_create(int device);               /* NULL if the device cannot be opened */
/* slam_create with the context stream's priority: 0 normal, > 0 the device's
 * highest (latency-critical small launches -- the pipeline's per-frame pose
 * work -- dispatched ahead of a concurrent context's large batch kernels) */
slam_ctx*   slam_create_prio(int device, int priority);
void        slam_destroy(slam_ctx* ctx);
const char* slam_last_error(const slam_ctx* ctx);
int         slam_synchronize(slam_ctx* ctx);

/* ---- reference entry points (host buffers) ------------------------------------ */
/* getMatcherTypeIndex: priority SIFT_BF > SIFT_FLANN > ORB; none -> SLAM_E_BAD_MATCHER */
int slam_matcher_type(int use_sift_bf, int use_sift_flann, int use_orb);

/* fastExtractor(src, pts, threshold, suppression, type).  img: 8-bit, 1/3/4
 * channels (3/4 = BGR/BGRA, converted as cvtColor BGR2GRAY), row stride `step`
 * bytes.  type: SLAM_FAST_TYPE_9_16 (the reference's default and every caller's),
 * _7_12 or _5_8 (FAST_t<12> / <8>); any other -> SLAM_E_INVALID_ARG.
 * *n_out = keypoints found (raster order); SLAM_E_CAPACITY if > cap. */
int slam_fast(slam_ctx* ctx, const uint8_t* img, int w, int h, size_t step, int channels,
              int threshold, int nonmax, int type,
              slam_keypoint* out, int cap, int* n_out);
/* slam_fast on a frame already in device memory (d_img, row stride `step`),
 * queued on `stream` (NULL = the context stream): the device-resident pipeline
 * uploads each frame once (fillVideoFrameBatch, batch.cpp:245 / getNextFrame +
 * fastExtractor, mainCycleInternals.cpp:107-156) and describes / matches it
 * through the slam_batch_* calls below.  Keypoints are returned to host memory. */
int slam_fast_dev(slam_ctx* ctx, void* stream, const uint8_t* d_img, int w, int h, size_t step, int channels,
                  int threshold, int nonmax, int type,
                  slam_keypoint* out, int cap, int* n_out);

/* extractDescriptor(frame, features, type, desc).  kps is IN/OUT: ORB drops
 * keypoints closer than 31 px to the border in place (*n_inout shrinks), as
 * cv::ORB::compute does to the reference's vector.  desc: SIFT n x 128 float
 * (integer values 0..255, CV_32F), ORB n x 32 uint8. */
int slam_describe(slam_ctx* ctx, const uint8_t* img, int w, int h, size_t step, int channels,
                  int matcher_type, slam_keypoint* kps, int* n_inout, void* desc);

/* Full SIFT detector -- not on the reference's own path (its SIFT descriptors
 * are computed on FAST keypoints, slam_describe); SURVEY.md 8(f) rank 2 and the
 * north star's "DoG pyramid, extrema, orientation histogram".  Replaces
 * cv::SIFT::create()->detectAndCompute(img, noArray(), kps, desc) with the
 * defaults (3 octave layers, contrast 0.04, edge 10, sigma 1.6, doubled base
 * image).  Keypoints come in OpenCV's order (KeyPointsFilter::
 * removeDuplicatedSorted), octave packed as OpenCV packs it.  *n_out = total
 * found; SLAM_E_CAPACITY if > cap (the first cap are written).  desc
 * (nullable): cap x 128 float, integer values 0..255. */
int slam_sift_detect(slam_ctx* ctx, const uint8_t* img, int w, int h, size_t step, int channels,
                     slam_keypoint* kps, int cap, int* n_out, float* desc);

/* The same detector over a device-resident batch (round 4): nframes u8 frames
 * (channels 1 or 3, rows packed at w * channels bytes, frames contiguous) in
 * device memory, e.g. decoded video in HBM; every kernel launch covers the
 * whole batch (one pyramid per frame).  Outputs stay on the device: frame f's
 * keypoints go to d_kps[f * cap ..] and its descriptors (nullable) to
 * d_desc[f * cap * 128 ..] (device pointers), each as slam_sift_detect returns
 * them; n_out (host) [f] = keypoints found in frame f, SLAM_E_CAPACITY if any
 * exceeds cap.  Runs on `stream` (NULL: the context's stream) and returns with
 * it drained.  At most 256 frames per call (SLAM_E_INVALID_ARG above; the
 * pyramid needs ~0.5 GB per 1080p frame).  The detector stages through the
 * context's batch buffers: a published slam_batch_* result is released. */
int slam_sift_detect_batch(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                           int channels, slam_keypoint* d_kps, int cap, int32_t* n_out, float* d_desc);

/* reconstruct(calibration, rotation1, transition1, rotation2, transition2,
 * points1, points2, spatialPoints) -- src/mainModule/triangulation/
 * triangulate.cpp:74-100: P_v = K [R_v | t_v], per
 * point the 4 x 4 DLT system solved by OpenCV's Jacobi SVD, X = V(3) / w.
 * K, R: 3 x 3 row-major; t: 3; pts: n x 2 float (Point2f); out: n x 3 double
 * (Point3d). */
int slam_reconstruct(slam_ctx* ctx, const double* K, const double* R1, const double* t1,
                     const double* R2, const double* t2, const float* pts1, const float* pts2,
                     int n, double* out);

/* estimateTransformation(points1, points2, calibrationMatrix, rotationMatrix,
 * translationVector, chiralityMask) -- src/mainModule/translation/
 * cameraTranslation.cpp:32-69: findEssentialMat with
 * RANSAC (RPUseRANSAC, RPRANSACProb, RPRANSACThreshold; without RANSAC the
 * reference's default call, prob 0.999 / threshold 1) then recoverPose with
 * RPDistanceThreshold.  pts: n x 2 float; K: 3 x 3 row-major; R out 3 x 3, t
 * out 3; chirality / ransac_mask (nullable): n bytes.  *passed = recoverPose's
 * count (the reference returns passed > 0). */
int slam_estimate_transformation(slam_ctx* ctx, const float* pts1, const float* pts2, int n,
                                 const double* K, int use_ransac, double prob, double threshold,
                                 double distance_threshold, double* R, double* t,
                                 uint8_t* chirality, uint8_t* ransac_mask, int* passed);

/* solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec,
 * tvec) -- src/mainModule/cycleProcessing/mainCycle.cpp:155-161 (SURVEY.md
 * 8(f) rank 3), the reference's call with an empty distortion Mat and every
 * default (iterations_count 100, reprojection_error 8, confidence 0.99): EPnP
 * RANSAC on minimal sets of 5, then SOLVEPNP_ITERATIVE (Levenberg-Marquardt)
 * on the inliers from the RANSAC model.  obj: n x 3 float (Point3f); img: n x 2
 * float (Point2f); K: 3 x 3 row-major; rvec / tvec out: 3 double each (CV_64F
 * 3 x 1); inlier_mask (nullable): n bytes.  *found = solvePnPRansac's return
 * value (0: no model, rvec / tvec zeroed).  n == 4 (OpenCV: the P3P kernel)
 * returns SLAM_E_UNSUPPORTED; n < 4 (an OpenCV assertion) SLAM_E_INVALID_ARG. */
int slam_solve_pnp_ransac(slam_ctx* ctx, const float* obj, const float* img, int n, const double* K,
                          int iterations_count, float reprojection_error, double confidence,
                          double* rvec, double* tvec, uint8_t* inlier_mask, int* n_inliers,
                          int* found);

/* cv::Rodrigues (cvRodrigues2, host code): n == 3 -> dst = 3 x 3 row-major
 * rotation of the rotation vector src; n == 9 -> dst = rotation vector of the
 * 3 x 3 matrix src (checkRange, SVD orthonormalisation).  Replaces the calls at
 * src/mainModule/cycleProcessing/mainCycle.cpp:162 (after solvePnPRansac) and
 * src/mainModule/bundleAdjustment/bundleAdjustment.cpp:167,195
 * (convertDataForBA / convertDataFromBA).  Other n: SLAM_E_INVALID_ARG. */
int slam_rodrigues(const double* src, int n, double* dst);

/* knnMatch(query, train, k = 2): idx/dist nq x 2 (idx -1 where missing). */
int slam_knn2(slam_ctx* ctx, const void* q, int nq, const void* t, int nt,
              int matcher_type, int norm, int* idx, float* dist);

/* matchFeatures: knnMatch(prevDesc = query, curDesc = train, 2) + ratio test
 * (m0.distance < ratio * m1.distance), survivors in query order. */
int slam_match(slam_ctx* ctx, const void* q, int nq, const void* t, int nt,
               int matcher_type, int norm, double ratio,
               slam_dmatch* out, int cap, int* n_out);

/* matchFramesPairFeatures(firstFrameDescriptor, secondFrame, secondFeatures,
 * type, matches): describe the frame (kps IN/OUT as above) then slam_match. */
int slam_match_frame(slam_ctx* ctx, const void* prev_desc, int nprev,
                     const uint8_t* img, int w, int h, size_t step, int channels,
                     int matcher_type, int norm, double ratio,
                     slam_keypoint* kps, int* n_inout,
                     slam_dmatch* out, int cap, int* n_out);

/* candidate selection over per-candidate match counts (batch index order):
 * scan from the tail down to skip_head, good iff count >= required and
 * count >= best so far; first_fit stops at the first good one. */
int slam_select_good(const int32_t* counts, int n, int required, int skip_head, int first_fit);

/* bundleAdjustment(K, window, global).  K4 = {fx, fy, cx, cy} (IN/OUT),
 * ext6 = nframes x {angle-axis[3], t[3]} (IN/OUT, frame 0 held constant),
 * pts3 = npoints x 3 (IN/OUT), observations (frame, point, pixel x, y).
 * Reference Ceres options (:108-114); max_iters <= 0 -> 50. */
int slam_ba(slam_ctx* ctx, double* K4, int nframes, double* ext6, int npoints, double* pts3,
            int nobs, const int32_t* obs_frame, const int32_t* obs_point, const double* obs_xy,
            int loss, double loss_param, int max_iters, slam_ba_summary* summary);

/* ---- device-resident candidate batch (batch.cpp:59-226) ------------------------ */
/* Frames are BGR u8, nframes x h x w x 3, contiguous, in device memory.  Runs
 * gray + FAST (+ORB border filter) + descriptors for every frame, on `stream`
 * (NULL = the context stream).  kp_counts (host, nframes) receives the per-frame
 * keypoint counts -- the batch filter of fillVideoFrameBatch (batch.cpp:247). */
int slam_batch_extract(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes,
                       int w, int h, int threshold, int matcher_type, int32_t* kp_counts);

/* fillVideoFrameBatch's FAST over frames already in device memory
 * (batch.cpp:245-247 with fastExtractor.cpp:7-13): gray + FAST-9 + NMS of every
 * frame in one device pass, no descriptors.  kp_counts (host, nframes)
 * receives the per-frame keypoint counts (the batch filter input); the
 * keypoints stay in the context's batch for slam_batch_get_keypoints /
 * slam_batch_counts.  Descriptor and match calls on such a batch return
 * SLAM_E_INVALID_ARG.  Only with SLAM_OPT_FAST_REUSE = 1 set when this call
 * runs (default 0): a following batch extraction (slam_batch_extract*, SIFT)
 * of the same device pointer, frame count and size at the same threshold takes
 * this pass's FAST results instead of detecting again, unless another FAST /
 * gray launch on the context came in between (the reference runs fastExtractor
 * in fillVideoFrameBatch and again for the descriptors).  Setting it is the
 * caller's promise that the frames' CONTENTS do not change in between: the
 * library compares pointers only, so a buffer refilled (or freed and
 * reallocated at the same address) in between would return the old frames'
 * keypoints and descriptors.  With the default the extraction always detects. */
int slam_batch_fast(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes, int w, int h, int threshold,
                    int32_t* kp_counts);
/* 1 when the context's last batch extraction took slam_batch_fast's results, else 0 */
int slam_batch_fast_reused(const slam_ctx* ctx);

/* match every extracted frame (train) against one query descriptor set that is
 * already in device memory in the context's internal format (see
 * slam_batch_export_desc).  match_counts (host, nframes) receives the ratio-test
 * survivor counts used by the selection rule. */
int slam_batch_match(slam_ctx* ctx, void* stream, const void* d_query, int nq,
                     int norm, double ratio, int32_t* match_counts);

/* slam_batch_extract + slam_batch_match in one call with one host sync (the
 * per-candidate work of findGoodFrameFromBatch, batch.cpp:162-226, when the
 * query set is already on the device).  The kNN launch is queued behind the
 * extraction without waiting for the keypoint counts: it is sized on the
 * previous batch's largest frame and redone at the actual size when a frame
 * outgrows it.  Same outputs as the two calls.  A context's first batch (or a
 * new frame size) takes the two-call path internally. */
int slam_batch_extract_match(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes,
                             int w, int h, int threshold, int matcher_type,
                             const void* d_query, int nq, int norm, double ratio,
                             int32_t* kp_counts, int32_t* match_counts);

/* slam_batch_extract_match whose kNN also waits on `query_ready` (a hipEvent_t,
 * nullable) recorded after the query set's producer -- e.g. the RCCL broadcast
 * of the previous good frame's descriptors.  The extraction is
 * queued ahead of the wait, so only the match is ordered behind the producer. */
int slam_batch_extract_match_ev(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes,
                                int w, int h, int threshold, int matcher_type,
                                const void* d_query, int nq, int norm, double ratio, void* query_ready,
                                int32_t* kp_counts, int32_t* match_counts);

/* slam_batch_extract_match in three halves, none of which waits on the host
 * until the last, so a caller with two contexts can queue the next search's
 * extraction (which needs no previous result) before it selects this one's
 * winner -- the host selection, the winner hand-over and the multi-rank
 * exchanges then overlap device work instead of idling it.
 *   _extract_async  queues gray + FAST + descriptors (on `stream`, NULL = the
 *                   context stream) and the frame-table read-back;
 *   _match_async    queues the kNN + ratio test against d_query behind
 *                   query_ready (a hipEvent_t, nullable), on the same stream;
 *                   for a context's first batch (or a new frame size) it
 *                   first waits for the extraction (the kNN is sized on its counts);
 *   _finish         waits, publishes the batch (the getters, export, result
 *                   calls work on it from here) and returns the counts, as
 *                   slam_batch_extract_match would (match_counts is left
 *                   untouched when no match was queued).
 * Between _extract_async and _finish the context's buffers belong to the batch
 * in flight: every other call that uses them returns SLAM_E_INVALID_ARG. */
int slam_batch_extract_async(slam_ctx* ctx, void* stream, const uint8_t* d_frames, int nframes,
                             int w, int h, int threshold, int matcher_type);
int slam_batch_match_async(slam_ctx* ctx, const void* d_query, int nq, int norm, double ratio, void* query_ready);
int slam_batch_finish(slam_ctx* ctx, int32_t* kp_counts, int32_t* match_counts);
/* the context's own HIP stream (the one NULL stands for) */
void* slam_context_stream(slam_ctx* ctx);

/* bytes per descriptor in the internal device format (SIFT: 128 u8 + i32 norm
 * side array; ORB: the 256 bits as FP4 (e2m1) +-1, 128 bytes) and the size of an exported set. */
size_t slam_batch_desc_bytes(int matcher_type, int n);
/* copy frame f's descriptors (internal format) to d_dst; returns count in *n */
int slam_batch_export_desc(slam_ctx* ctx, void* stream, int frame, void* d_dst, int* n);
/* per-frame counts of the last extract, all frames in one call: FAST keypoints
 * (the batch filter input) and descriptor-bearing keypoints (ORB: after the
 * border filter; the query size of an exported set).  Either array may be NULL.
 * Returns the frame count, or a negative status (cap < frame count).  Host-side
 * state only (no device work).  Replaces per-frame keypoints.size() reads of
 * batch.cpp:245-249 / mainCycle.cpp:99. */
int slam_batch_counts(slam_ctx* ctx, int32_t* raw_counts, int32_t* desc_counts, int cap);
/* host copies of frame f's keypoints / descriptors (reference layout) / matches */
int slam_batch_get_keypoints(slam_ctx* ctx, int frame, slam_keypoint* out, int cap, int* n);
int slam_batch_get_descriptors(slam_ctx* ctx, int frame, void* out, int cap, int* n);
int slam_batch_get_matches(slam_ctx* ctx, int frame, slam_dmatch* out, int cap, int* n);
/* frame f's keypoints and ratio-test matches (what findGoodFrameFromBatch
 * returns for its winner, batch.cpp:92-97) in one call with one host sync */
int slam_batch_get_result(slam_ctx* ctx, int frame, slam_keypoint* kps, int kcap, int* nk,
                          slam_dmatch* matches, int mcap, int* nm);
/* the same result in two halves, for a caller that overlaps the transfer with
 * its next batch: _begin queues the compaction and the copies into a pinned
 * buffer of the context and returns without waiting; _end waits for them (by
 * then usually long done) and copies out.  One result in flight per context
 * (a second _begin first waits for the first); later batch calls may run
 * between the two, on any stream (they wait on the device for the queued
 * copies before rewriting the buffers those read).  _end with a buffer that is
 * too small returns SLAM_E_CAPACITY with the needed sizes and keeps the result
 * pending, so the caller can retry. */
int slam_batch_result_begin(slam_ctx* ctx, int frame);
int slam_batch_result_end(slam_ctx* ctx, slam_keypoint* kps, int kcap, int* nk, slam_dmatch* matches, int mcap,
                          int* nm);

/* the same result into device memory, queued on `stream` (NULL = the context
 * stream) without a host sync: frame f's ratio-test matches (query order) to
 * d_matches and its keypoints to d_kps.  nm = the frame's match count as the
 * caller knows it (the batch's match_counts, or their all-gather across ranks);
 * exactly nm matches are written.  For a multi-rank scan whose winner's owner
 * broadcasts these buffers (SURVEY.md 8(e) exchange 3) with no host round trip. */
int slam_batch_result_dev(slam_ctx* ctx, void* stream, int frame, void* d_matches, int nm, void* d_kps, int kcap);

/* stream ordering at the boundary: everything queued so far on `stream` (NULL =
 * the context stream) happens before anything queued later on `waiter` (a HIP
 * stream; NULL = the legacy default stream).  A device-side wait, no host
 * block.  E.g. a descriptor export (slam_batch_export_desc on the context
 * stream) before an RCCL broadcast that torch orders behind its current stream. */
int slam_order_after(slam_ctx* ctx, void* waiter, void* stream);

/* the same for a point inside the context's last batch extraction
 * (slam_batch_extract / _extract_async / _extract_match): anything queued later
 * on `waiter` starts after that extraction's descriptor kernel has been reached
 * (SLAM_STAGE_DESC_START: gray, FAST and the blur are done) or has finished
 * (SLAM_STAGE_DESC_END).  Lets a second context's next extraction fill the
 * chip while this one's descriptor kernel drains.  SLAM_E_INVALID_ARG before
 * any extraction. */
#define SLAM_STAGE_DESC_START 0
#define SLAM_STAGE_DESC_END 1
int slam_order_after_stage(slam_ctx* ctx, void* waiter, int stage);

/* ---- options ------------------------------------------------------------------ */
/* Per-context choices; all but SLAM_OPT_PNP_SUMS (below) never change results.  SLAM_OPT_SIFT_KERNEL picks the
 * kernel for SIFT descriptors of keypoints sharing one angle and size (FAST
 * keypoints): AUTO = band-staged scatter when its schedule reproduces the raster
 * order, else the per-target gather, else the general kernel; the others force
 * one (the parity tests run each against the oracle); a forced kernel whose
 * schedule does not apply to the keypoints makes the describing call fail with
 * SLAM_E_UNSUPPORTED instead of running another.  SLAM_OPT_SIFT_BAND_SPLIT: how
 * the band kernel runs a launch's last, partial round of keypoint groups --
 * OFF = whole walks, AUTO (default) = as part-walks that each finish some of
 * the descriptor rows (two: rows 0-1 and 2-3; four: one row each) when that
 * round would leave at most one wave per CU, ALL / ALL4 = every group as two /
 * four part-walks (the tests' way to run those paths on every keypoint).
 * Unknown option or value: SLAM_E_INVALID_ARG. */
enum slam_option { SLAM_OPT_SIFT_KERNEL = 1, SLAM_OPT_SIFT_BAND_SPLIT = 2, SLAM_OPT_PNP_SUMS = 3,
                   SLAM_OPT_FAST_REUSE = 4 };
/* SLAM_OPT_FAST_REUSE: 1 = slam_batch_fast's results may be taken by the next
 * batch extraction of the same frames (see slam_batch_fast for the contract the
 * caller accepts); 0 (default) = every extraction detects. */
/* SLAM_OPT_PNP_SUMS (the one option that changes results): how solvePnPRansac's
 * refinement forms J'J, J'e and |e|^2 over the inliers each LM step --
 * ORDERED (default) = sequential sums in the oracle's order (bit-exact poses,
 * 2 m dependent f64 adds per sum: ~90 us per step at m = 1750), PAIRWISE = per-
 * thread partial sums and a fixed tree (deterministic; poses within 1e-9 of
 * the oracle's, the same inlier mask; a few us per step). */
enum slam_pnp_sums { SLAM_PNP_SUMS_ORDERED = 0, SLAM_PNP_SUMS_PAIRWISE = 1 };
enum slam_band_split { SLAM_BAND_SPLIT_OFF = 0, SLAM_BAND_SPLIT_AUTO = 1, SLAM_BAND_SPLIT_ALL = 2,
                       SLAM_BAND_SPLIT_ALL4 = 3 };
/* SLAM_SIFT_KERNEL_COLS: the one-keypoint-per-lane, two-column-pass variant of the
 * band kernel (same descriptors; an A/B kernel, never picked by AUTO).
 * SLAM_SIFT_KERNEL_COLW: one descriptor column per wave (same descriptors). */
enum slam_sift_kernel { SLAM_SIFT_KERNEL_AUTO = 0, SLAM_SIFT_KERNEL_BAND = 1, SLAM_SIFT_KERNEL_TAB = 2,
                        SLAM_SIFT_KERNEL_GENERAL = 3, SLAM_SIFT_KERNEL_COLS = 4, SLAM_SIFT_KERNEL_COLW = 5 };
int slam_set_option(slam_ctx* ctx, int option, int value);
/* the SLAM_SIFT_KERNEL_* that ran the context's last SIFT descriptor launch (0 before any) */
int slam_last_sift_kernel(const slam_ctx* ctx);

/* ---- profiling hooks (bench.py) ---------------------------------------------- */
/* average duration (ms) of the last batch's launches of one kernel family,
 * measured with HIP events on the launch stream: 0 fast, 1 sift_desc, 2 knn,
 * 3 orb_desc, 4 sift_blur, 5 ratio/compact */
int slam_profile_enable(slam_ctx* ctx, int on);
int slam_profile_read(slam_ctx* ctx, int family, double* avg_ms, int* launches);

/* ---- synthetic indoor sequence (test / bench input, host memory) ---------------- */
/* camera paths: DRIFT zooms in without bound (the texture in view thins out
 * along the sequence: the round-1..3 fixtures and tests); STEADY is a bounded
 * loop whose FAST count stays near frame 0's for any frame index (the bench's
 * configs[1] batches: every candidate at 10k +- 10 % keypoints) */
enum slam_synth_path { SLAM_SYNTH_DRIFT = 0, SLAM_SYNTH_STEADY = 1 };
int slam_synth_sequence(int w, int h, int first, int count, uint64_t seed, int path, uint8_t* out_bgr);
/* the same frames rendered on the device into d_out (count x h x w x 3, on
 * `stream`, NULL = the context stream), byte-identical to slam_synth_sequence:
 * a video "decoded" straight into HBM for the device-resident pipeline */
int slam_synth_sequence_dev(slam_ctx* ctx, void* stream, int w, int h, int first, int count, uint64_t seed, int path,
                            uint8_t* d_out);
/* slam_synth_sequence(..., SLAM_SYNTH_DRIFT, ...) */
int slam_synth_frames(int w, int h, int first, int count, uint64_t seed, uint8_t* out_bgr);

#ifdef __cplusplus
}
#endif
#endif
