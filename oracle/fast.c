/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * BGR->gray + FAST-9/16 corner detection with non-max suppression.
 * Reference call: fastExtractor.cpp:10-12 (FastFeatureDetector::create(threshold,
 * suppression, TYPE_9_16) -> detect), called from batch.cpp:245-246 and
 * mainCycleInternals.cpp:144-145.  Restates OpenCV 4.8 features2d/src/fast.cpp
 * FAST_t<16> + cornerScore<16> and imgproc cvtColor(COLOR_BGR2GRAY) on 8U.
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

/* Bresenham circle of radius 3, (x, y) pairs in OpenCV's makeOffsets order */
static const int k_circle16[16][2] = {
    {0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static void make_offsets(int pixel[25], int stride)
{
    int k;
    for (k = 0; k < 16; k++) pixel[k] = k_circle16[k][0] + k_circle16[k][1] * stride;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

/* cornerScore<16>: largest threshold for which the pixel is still a corner, - 1 */
int orc_fast_score(const uint8_t* ptr, const int* pixel, int threshold)
{
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    int d[25];
    for (k = 0; k < N; k++) d[k] = v - ptr[pixel[k]];

    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        if (d[k + 3] < a) a = d[k + 3];
        if (a <= a0) continue;
        for (int m = 4; m <= 8; m++) if (d[k + m] < a) a = d[k + m];
        int t = a < d[k] ? a : d[k];
        if (t > a0) a0 = t;
        t = a < d[k + 9] ? a : d[k + 9];
        if (t > a0) a0 = t;
    }

    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int m = 3; m <= 5; m++) if (d[k + m] > b) b = d[k + m];
        if (b >= b0) continue;
        for (int m = 6; m <= 8; m++) if (d[k + m] > b) b = d[k + m];
        int t = b > d[k] ? b : d[k];
        if (t < b0) b0 = t;
        t = b > d[k + 9] ? b : d[k + 9];
        if (t < b0) b0 = t;
    }
    return -b0 - 1;
}

/* segment test: >= 9 contiguous circle pixels all darker than v-t or all
 * brighter than v+t (strict), evaluated over the 25-long wrapped circle */
static int is_corner(const uint8_t* ptr, const int* pixel, int t)
{
    int v = ptr[0];
    int lo = v - t, hi = v + t;
    int cd = 0, cb = 0;
    for (int k = 0; k < 25; k++) {
        int x = ptr[pixel[k]];
        if (x < lo) { if (++cd > 8) return 1; } else cd = 0;
        if (x > hi) { if (++cb > 8) return 1; } else cb = 0;
    }
    return 0;
}

int orc_fast(const uint8_t* gray, int w, int h, int threshold, int nms,
             orc_kp* out, int cap)
{
    int pixel[25];
    make_offsets(pixel, w);
    if (threshold < 0) threshold = 0;
    if (threshold > 255) threshold = 255;
    if (w < 7 || h < 7) return 0;

    /* score map: 0 for non-corners and for everything outside rows/cols
     * [3, h-3) x [3, w-3) (OpenCV zero-fills its 3 rolling row buffers) */
    uint8_t* score = (uint8_t*)calloc((size_t)w * h, 1);
    uint8_t* corner = (uint8_t*)calloc((size_t)w * h, 1);
    for (int i = 3; i < h - 3; i++) {
        const uint8_t* row = gray + (size_t)i * w;
        for (int j = 3; j < w - 3; j++) {
            if (is_corner(row + j, pixel, threshold)) {
                corner[(size_t)i * w + j] = 1;
                if (nms)
                    score[(size_t)i * w + j] =
                        (uint8_t)orc_fast_score(row + j, pixel, threshold);
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
