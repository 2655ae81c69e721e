/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * ORB descriptor computation on provided keypoints, as reached by the reference
 * through extractDescriptor -> cv::ORB::create()->compute() (featureMatchingCPU.cpp
 * :59-65; CUDA twin featureMatchingCUDA.cpp:63-68).  Restates OpenCV 4.8
 * features2d/src/orb.cpp detectAndCompute(useProvidedKeypoints=true):
 *   - KeyPointsFilter::runByImageBorder(kps, size, edgeThreshold = 31): erases
 *     keypoints outside [31, W-31) x [31, H-31), order preserved, IN PLACE
 *     (the reference's caller vector shrinks; trainIdx indexes the filtered list);
 *   - nLevels = max octave + 1 = 1 for FAST keypoints, level 0 = gray image with
 *     a 32-px REFLECT_101 border (copyMakeBorder);
 *   - GaussianBlur(ROI, 7x7, sigma 2, REFLECT_101) on that ROI.  Because the ROI
 *     is a submatrix, GaussianBlur skips its fixed-point bit-exact 8U path and
 *     runs sepFilter2D with f32 kernels: RowVec_8u32f (fma chain from 0) then
 *     SymmColumnVec_32f8u (symmetric fma form, round-half-even, saturate u8);
 *   - computeOrbDescriptors, WTA_K = 2: the 512-point bit_pattern_31_ rotated by
 *     kp.angle (FAST: -1 degree), offsets rounded with cvRound, bit j of byte i
 *     = I(p[16i+2j]) < I(p[16i+2j+1]).
 * The ORB blur reads at most 3 px around pixels that are >= 15 px inside the
 * image for surviving keypoints, so the border treatment never reaches a bit.
 */
#include "oracle.h"
#include "orb_pattern.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

int orc_orb_filter(const orc_kp* kps, int n, int w, int h, int border, orc_kp* out)
{
    if (h <= border * 2 || w <= border * 2) return 0;
    int m = 0;
    for (int i = 0; i < n; i++) {
        /* Rect<int>::contains(Point) after Point2f -> Point (cvRound) */
        long x = lrintf(kps[i].x), y = lrintf(kps[i].y);
        if (x >= border && x < w - border && y >= border && y < h - border) out[m++] = kps[i];
    }
    return m;
}

static int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

void orc_orb_blur(const uint8_t* gray, int w, int h, uint8_t* out)
{
    float k[7];
    orc_gauss_kernel_f32(7, 2.0, k);
    float* tmp = (float*)malloc(sizeof(float) * (size_t)w * h);
    for (int y = 0; y < h; y++) {
        const uint8_t* s = gray + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            float acc = 0.f;
            for (int t = 0; t < 7; t++) acc = fmaf((float)s[reflect101(x - 3 + t, w)], k[t], acc);
            tmp[(size_t)y * w + x] = acc;
        }
    }
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            float acc = k[3] * tmp[(size_t)y * w + x];
            for (int m = 1; m <= 3; m++) {
                float a = tmp[(size_t)reflect101(y + m, h) * w + x];
                float b = tmp[(size_t)reflect101(y - m, h) * w + x];
                acc = fmaf(k[3 + m], a + b, acc);
            }
            float r = rintf(acc);
            out[(size_t)y * w + x] = (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
        }
    }
    free(tmp);
}

void orc_orb_describe(const uint8_t* img, int w, int h, const orc_kp* kps, int n, uint8_t* desc)
{
    (void)h;
#pragma omp parallel for schedule(static)
    for (int j = 0; j < n; j++) {
        float angle = kps[j].angle * (float)(M_PI / 180.f);
        float a = cosf(angle), b = sinf(angle);
        long cy = lrintf(kps[j].y), cx = lrintf(kps[j].x);
        const uint8_t* center = img + cy * w + cx;
        const int* pat = slam_orb_pattern31;
        uint8_t* d = desc + (size_t)j * 32;
        for (int i = 0; i < 32; i++, pat += 32) {
            int val = 0;
            for (int bit = 0; bit < 8; bit++) {
                int px0 = pat[4 * bit], py0 = pat[4 * bit + 1];
                int px1 = pat[4 * bit + 2], py1 = pat[4 * bit + 3];
                float x0 = (float)px0 * a - (float)py0 * b, y0 = (float)px0 * b + (float)py0 * a;
                float x1 = (float)px1 * a - (float)py1 * b, y1 = (float)px1 * b + (float)py1 * a;
                int t0 = center[lrintf(y0) * w + lrintf(x0)];
                int t1 = center[lrintf(y1) * w + lrintf(x1)];
                val |= (t0 < t1) << bit;
            }
            d[i] = (uint8_t)val;
        }
    }
}

int orc_orb_compute(const uint8_t* bgr, int w, int h, size_t step, orc_kp* kps, int n, uint8_t* desc)
{
    int m = orc_orb_filter(kps, n, w, h, 31, kps);
    if (m == 0) return 0;
    uint8_t* gray = (uint8_t*)malloc((size_t)w * h);
    uint8_t* blur = (uint8_t*)malloc((size_t)w * h);
    orc_bgr2gray(bgr, w, h, step, gray);
    orc_orb_blur(gray, w, h, blur);
    orc_orb_describe(blur, w, h, kps, m, desc);
    free(blur);
    free(gray);
    return m;
}
