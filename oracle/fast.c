/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * BGR->gray + FAST corner detection with non-max suppression.
 * Reference call: fastExtractor.cpp:10-12 (FastFeatureDetector::create(threshold,
 * suppression, type) -> detect; type defaults to TYPE_9_16, fastExtractor.h:19-21,
 * docs/FastExtractor.md:13-16 documents all three), called from batch.cpp:245-246
 * and mainCycleInternals.cpp:144-145.  Restates OpenCV 4.8 features2d/src/fast.cpp
 * FAST_t<16 / 12 / 8> + cornerScore<16 / 12 / 8> and imgproc
 * cvtColor(COLOR_BGR2GRAY) on 8U.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* cvtColor BGR2GRAY, 8U fixed point: yuv_shift 14, B2Y 1868, G2Y 9617, R2Y 4899
 * (the detector converts because the frame is CV_8UC3). */
void orc_bgr2gray(const uint8_t* bgr, int w, int h, size_t step, uint8_t* gray)
{
    for (int y = 0; y < h; y++) {
        const uint8_t* s = bgr + (size_t)y * step;
        uint8_t* d = gray + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            unsigned v = s[3 * x] * 1868u + s[3 * x + 1] * 9617u + s[3 * x + 2] * 4899u;
            d[x] = (uint8_t)((v + (1u << 13)) >> 14);
        }
    }
}

/* circles in OpenCV's makeOffsets order (fast.cpp): patternSize 16 (radius 3),
 * 12 (radius 2) and 8 (radius 1); (x, y) pairs */
static const int k_circle16[16][2] = {
    {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
static const int k_circle12[12][2] = {
    {0, 2}, {1, 2}, {2, 1}, {2, 0}, {2, -1}, {1, -2},
    {0, -2}, {-1, -2}, {-2, -1}, {-2, 0}, {-2, 1}, {-1, 2}};
static const int k_circle8[8][2] = {
    {0, 1}, {1, 1}, {1, 0}, {1, -1}, {0, -1}, {-1, -1}, {-1, 0}, {-1, 1}};

static int pattern_size(int type) { return type == ORC_FAST_5_8 ? 8 : type == ORC_FAST_7_12 ? 12 : 16; }

/* makeOffsets: pixel[k] for k < patternSize, then wrapped up to 25 */
static void make_offsets(int pixel[25], int stride, int ps)
{
    const int(*c)[2] = ps == 16 ? k_circle16 : ps == 12 ? k_circle12 : k_circle8;
    int k;
    for (k = 0; k < ps; k++) pixel[k] = c[k][0] + c[k][1] * stride;
    for (; k < 25; k++) pixel[k] = pixel[k - ps];
}

/* cornerScore<patternSize>: the largest threshold for which the pixel is still a
 * corner, - 1.  d[k] = v - p[k], k < 3 K + 1 (K = patternSize / 2); the early
 * `continue`s are OpenCV's (they never change the result) */
static int fast_score(const uint8_t* ptr, const int* pixel, int threshold, int ps)
{
    const int K = ps / 2, N = 3 * K + 1;
    int k, v = ptr[0];
    int d[25];
    for (k = 0; k < N; k++) d[k] = v - ptr[pixel[k]];
    /* the dark side: min over the K + 1 arcs starting at k and k + 1 */
    const int acheck = ps == 16 ? 3 : 2;      /* d[k+1..k+acheck] before the early test */
    int a0 = threshold;
    for (k = 0; k < ps; k += 2) {
        int a = d[k + 1];
        for (int m = 2; m <= acheck; m++) if (d[k + m] < a) a = d[k + m];
        if (a <= a0) continue;
        for (int m = acheck + 1; m <= K; m++) if (d[k + m] < a) a = d[k + m];
        int t = a < d[k] ? a : d[k];
        if (t > a0) a0 = t;
        t = a < d[k + K + 1] ? a : d[k + K + 1];
        if (t > a0) a0 = t;
    }
    const int bcheck = ps == 16 ? 5 : ps == 12 ? 4 : 3;
    int b0 = -a0;
    for (k = 0; k < ps; k += 2) {
        int b = d[k + 1];
        for (int m = 2; m <= bcheck; m++) if (d[k + m] > b) b = d[k + m];
        if (b >= b0) continue;
        for (int m = bcheck + 1; m <= K; m++) if (d[k + m] > b) b = d[k + m];
        int t = b > d[k] ? b : d[k];
        if (t < b0) b0 = t;
        t = b > d[k + K + 1] ? b : d[k + K + 1];
        if (t < b0) b0 = t;
    }
    return -b0 - 1;
}

int orc_fast_score(const uint8_t* ptr, const int* pixel, int threshold)
{
    return fast_score(ptr, pixel, threshold, 16);
}

/* FAST_t<patternSize>'s per-pixel test: OpenCV's prefilter over the circle
 * pairs (k, k + 8), k = 0..7, on pixel[0..15] (wrapped for 12 and 8, where it
 * is a filter of its own, not only a necessary condition: kept as OpenCV has
 * it), then > K contiguous of the N = patternSize + K + 1 wrapped samples all
 * darker than v - t (if every pair had a dark member) or all brighter than
 * v + t (if every pair had a bright member).  Returns 1 for a corner. */
static int fast_test(const uint8_t* ptr, const int* pixel, int t, int ps)
{
    const int K = ps / 2, N = ps + K + 1;
    const int v = ptr[0];
#define TAB(x) ((x) < v - t ? 1 : (x) > v + t ? 2 : 0)
    int d = TAB(ptr[pixel[0]]) | TAB(ptr[pixel[8]]);
    if (d == 0) return 0;
    d &= TAB(ptr[pixel[2]]) | TAB(ptr[pixel[10]]);
    d &= TAB(ptr[pixel[4]]) | TAB(ptr[pixel[12]]);
    d &= TAB(ptr[pixel[6]]) | TAB(ptr[pixel[14]]);
    if (d == 0) return 0;
    d &= TAB(ptr[pixel[1]]) | TAB(ptr[pixel[9]]);
    d &= TAB(ptr[pixel[3]]) | TAB(ptr[pixel[11]]);
    d &= TAB(ptr[pixel[5]]) | TAB(ptr[pixel[13]]);
    d &= TAB(ptr[pixel[7]]) | TAB(ptr[pixel[15]]);
#undef TAB
    if (d & 1) {
        int count = 0;
        for (int k = 0; k < N; k++) {
            if (ptr[pixel[k]] < v - t) { if (++count > K) return 1; }
            else count = 0;
        }
    }
    if (d & 2) {
        int count = 0;
        for (int k = 0; k < N; k++) {
            if (ptr[pixel[k]] > v + t) { if (++count > K) return 1; }
            else count = 0;
        }
    }
    return 0;
}

int orc_fast_type(const uint8_t* gray, int w, int h, int threshold, int nms, int type,
                  orc_kp* out, int cap)
{
    const int ps = pattern_size(type);
    int pixel[25];
    make_offsets(pixel, w, ps);
    if (threshold < 0) threshold = 0;
    if (threshold > 255) threshold = 255;
    if (w < 7 || h < 7) return 0;

    /* score map: 0 for non-corners and for everything outside rows/cols
     * [3, h-3) x [3, w-3) (OpenCV zero-fills its 3 rolling row buffers; the
     * 3-pixel border holds for every pattern size) */
    uint8_t* score = (uint8_t*)calloc((size_t)w * h, 1);
    uint8_t* corner = (uint8_t*)calloc((size_t)w * h, 1);
    for (int i = 3; i < h - 3; i++) {
        const uint8_t* row = gray + (size_t)i * w;
        for (int j = 3; j < w - 3; j++) {
            if (fast_test(row + j, pixel, threshold, ps)) {
                corner[(size_t)i * w + j] = 1;
                if (nms)
                    score[(size_t)i * w + j] = (uint8_t)fast_score(row + j, pixel, threshold, ps);
            }
        }
    }
    int count = 0;
    for (int i = 3; i < h - 3; i++) {
        for (int j = 3; j < w - 3; j++) {
            size_t o = (size_t)i * w + j;
            if (!corner[o]) continue;
            int s = score[o];
            if (nms) {
                if (!(s > score[o + 1] && s > score[o - 1] &&
                      s > score[o - w - 1] && s > score[o - w] && s > score[o - w + 1] &&
                      s > score[o + w - 1] && s > score[o + w] && s > score[o + w + 1]))
                    continue;
            }
            if (count < cap) {
                orc_kp* k = &out[count];
                k->x = (float)j; k->y = (float)i; k->size = 7.f; k->angle = -1.f;
                k->response = (float)s; k->octave = 0; k->class_id = -1;
            }
            count++;
        }
    }
    free(score);
    free(corner);
    return count;
}

int orc_fast(const uint8_t* gray, int w, int h, int threshold, int nms, orc_kp* out, int cap)
{
    return orc_fast_type(gray, w, h, threshold, nms, ORC_FAST_9_16, out, cap);
}

int orc_fast_bgr_type(const uint8_t* bgr, int w, int h, size_t step, int threshold, int nms, int type,
                      orc_kp* out, int cap)
{
    uint8_t* gray = (uint8_t*)malloc((size_t)w * h);
    orc_bgr2gray(bgr, w, h, step, gray);
    int n = orc_fast_type(gray, w, h, threshold, nms, type, out, cap);
    free(gray);
    return n;
}

int orc_fast_bgr(const uint8_t* bgr, int w, int h, size_t step, int threshold,
                 int nms, orc_kp* out, int cap)
{
    uint8_t* gray = (uint8_t*)malloc((size_t)w * h);
    orc_bgr2gray(bgr, w, h, step, gray);
    int n = orc_fast(gray, w, h, threshold, nms, out, cap);
    free(gray);
    return n;
}

/* batch.cpp:101-160 (single-thread scan; the deterministic semantics of the
 * multi-thread scan batch.cpp:270-316): scan from the tail down to
 * skipFramesFromBatchHead; good iff count >= required && count >= best. */
int orc_select_good(const int* counts, int n, int required, int skip_head, int first_fit)
{
    int good = -1, best = 0;
    for (int i = n - 1; i >= skip_head; i--) {
        if (counts[i] >= required && counts[i] >= best) {
            good = i;
            best = counts[i];
            if (first_fit) break;
        }
    }
    return good;
}
