/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * SIFT descriptor computation on provided (FAST) keypoints, as reached by the
 * reference through extractDescriptor -> cv::SIFT::create()->compute()
 * (featureMatchingCPU.cpp:51-65, CUDA twin featureMatchingCUDA.cpp:57-68).
 * Restates OpenCV 4.8 features2d/src/sift.dispatch.cpp (detectAndCompute with
 * useProvidedKeypoints, createInitialImage, calcDescriptors) and sift.simd.hpp
 * calcSIFTDescriptor, core hal fastAtan2 / magnitude / exp32f (SIMD forms, FMA
 * where OpenCV uses v_fma/v_muladd), imgproc getGaussianKernel + sepFilter2D.
 *
 * FAST keypoints carry octave 0 -> firstOctave 0, one octave, no upscaling;
 * only gpyr[0] (the base image) is read, with angle 360 - (-1) = 361 degrees
 * and scale 0.5 * size = 3.5.  The 361-degree angle is NOT wrapped, so samples
 * whose gradient orientation is below ~1 degree get o0 = -1 and their first
 * orientation weight lands one slot before the cell in the flat histogram;
 * that quirk is reproduced exactly (hist has a guard slot at index -1).
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SIFT_D 4
#define SIFT_N 8
#define SIFT_DESCR_SCL_FCTR 3.f
#define SIFT_DESCR_MAG_THR 0.2f
#define SIFT_INT_DESCR_FCTR 512.f
#define SIFT_INIT_SIGMA 0.5f
#define SIFT_SIGMA 1.6f

/* getGaussianKernelBitExact (smooth.dispatch.cpp) evaluated in double, then the
 * (float) cast of getGaussianKernel(n, sigma, CV_32F). */
int orc_gauss_kernel_f32(int n, double sigma, float* k)
{
    if (sigma <= 0 && (n == 1 || n == 3 || n == 5 || n == 7)) {
        static const double t1[] = {1.0};
        static const double t3[] = {0.25, 0.5, 0.25};
        static const double t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
        static const double t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
        const double* t = n == 1 ? t1 : n == 3 ? t3 : n == 5 ? t5 : t7;
        for (int i = 0; i < n; i++) k[i] = (float)t[i];
        return n;
    }
    double sigmaX = sigma > 0 ? sigma : (double)n * 0.15 + 0.35;
    double scale2X = -0.125 / (sigmaX * sigmaX);
    int n2 = (n - 1) / 2;
    double values[64];
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2.0;
    sum += 1.0;
    if ((n & 1) == 0) sum += 1.0;
    double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; i++) {
        double t = values[i] * mul1;
        k[i] = (float)t;
        k[n - 1 - i] = (float)t;
    }
    k[n2] = (float)mul1;
    if ((n & 1) == 0) k[n2 + 1] = k[n2];
    return n;
}

/* createInitialImage (no doubling): sig_diff = sqrt(max(sigma^2 - 0.5^2, 0.01)) in float */
float orc_sift_sigma_diff(void)
{
    float s = SIFT_SIGMA * SIFT_SIGMA - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA;
    return sqrtf(s > 0.01f ? s : 0.01f);
}

static int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* GaussianBlur(gray->f32, sigma = sig_diff, ksize 13, BORDER_REFLECT_101):
 * RowVec_32f: s = sum_k fma(src[x-6+k], kx[k], s) from s = 0 (k ascending);
 * SymmColumnVec_32f: s = S[0]*ky[0]; s = fma(S[m] + S[-m], ky[m], s), m = 1..6. */
void orc_sift_base(const uint8_t* gray, int w, int h, float* base)
{
    float sig = orc_sift_sigma_diff();
    int ks = (int)lrint((double)sig * 4 * 2 + 1) | 1;
    float kern[64];
    orc_gauss_kernel_f32(ks, (double)sig, kern);
    int r = ks / 2;
    float* tmp = (float*)malloc(sizeof(float) * (size_t)w * h);
    int* xo = (int*)malloc(sizeof(int) * (size_t)(w + 2 * r));
    for (int x = -r; x < w + r; x++) xo[x + r] = reflect101(x, w);
    for (int y = 0; y < h; y++) {
        const uint8_t* s = gray + (size_t)y * w;
        float* d = tmp + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            float acc = 0.f;
            for (int k = 0; k < ks; k++) acc = fmaf((float)s[xo[x + k]], kern[k], acc);
            d[x] = acc;
        }
    }
    for (int y = 0; y < h; y++) {
        float* d = base + (size_t)y * w;
        const float* c = tmp + (size_t)y * w;
        for (int x = 0; x < w; x++) d[x] = c[x] * kern[r];
        for (int m = 1; m <= r; m++) {
            const float* up = tmp + (size_t)reflect101(y - m, h) * w;
            const float* dn = tmp + (size_t)reflect101(y + m, h) * w;
            for (int x = 0; x < w; x++) d[x] = fmaf(dn[x] + up[x], kern[r + m], d[x]);
        }
    }
    free(xo);
    free(tmp);
}

/* hal::fastAtan2 (degrees), v_atan_f32 SIMD form */
static const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float orc_fast_atan2_deg(float y, float x)
{
    float ax = fabsf(x), ay = fabsf(y);
    float mn = ax < ay ? ax : ay, mx = ax < ay ? ay : ax;
    float c = mn / (mx + (float)DBL_EPSILON);
    float cc = c * c;
    float a = fmaf(fmaf(fmaf(cc, atan2_p7, atan2_p5), cc, atan2_p3), cc, atan2_p1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* hal::exp32f, SIMD form: 64-entry 2^(i/64) table + degree-4 polynomial */
#define EXPTAB_SCALE 6
#define EXPTAB_MASK 63
#define EXPPOLY_32F_A0 .9670371139572337719125840413672004409288e-2
static float g_exptab[64];
static int g_exptab_init = 0;

static void exptab_init(void)
{
    if (g_exptab_init) return;
    for (int i = 0; i < 64; i++) g_exptab[i] = (float)(exp2((double)i / 64.0) * EXPPOLY_32F_A0);
    g_exptab_init = 1;
}

float orc_exp32f(float x)
{
    exptab_init();
    const double exp_prescale = 1.4426950408889634073599246810019 * (1 << EXPTAB_SCALE);
    const double exp_postscale = 1. / (1 << EXPTAB_SCALE);
    const double exp_max_val = 3000. * (1 << EXPTAB_SCALE);
    const float A4 = (float)(1.000000000000002438532970795181890933776 / EXPPOLY_32F_A0);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / EXPPOLY_32F_A0);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / EXPPOLY_32F_A0);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / EXPPOLY_32F_A0);
    const float minval = (float)(-exp_max_val / exp_prescale);
    const float maxval = (float)(exp_max_val / exp_prescale);

    float xf = x < minval ? minval : x;
    xf = xf > maxval ? maxval : xf;
    xf = xf * (float)exp_prescale;
    int xi = (int)lrintf(xf);
    xf = (xf - (float)xi) * (float)exp_postscale;
    float yf = g_exptab[xi & EXPTAB_MASK];
    int t = (xi >> EXPTAB_SCALE) + 127;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    union { int32_t i; float f; } u;
    u.i = t << 23;
    yf = yf * u.f;
    float z = xf + A1;
    z = fmaf(z, xf, A2);
    z = fmaf(z, xf, A3);
    z = fmaf(z, xf, A4);
    return z * yf;
}

/* calcSIFTDescriptor(img, pt, ori = 360 - kp.angle, scl = size/2, d=4, n=8); img = gpyr[0] for
 * FAST keypoints, the keypoint's own octave/layer image for detected ones (siftdet.c) */
/* diagnostics (scripts/diag/sift_tolerance.py): what relaxing the reference's
 * accumulation would change.  0 = the reference (OpenCV's raster order, f32);
 * 1 = the samples added in reverse raster order (f32); 2 = mag and the three bin
 * fractions rounded to 11 significant bits (fp16 inputs, as an f16 MFMA form
 * would take them), f32 sums in raster order; 3 = the histogram summed in f64
 * (order-free up to rounding), rounded to f32 at the end. */
static int g_sift_variant;   /* process-wide: the OpenMP workers read it */
void orc_sift_set_variant(int v) { g_sift_variant = v; }

static float round_sig11(float x)
{
    if (x == 0.f || !isfinite(x)) return x;
    int e;
    frexpf(x, &e);
    const float q = ldexpf(1.f, e - 11);
    return rintf(x / q) * q;
}

void orc_sift_one(const float* img, int cols, int rows, const orc_kp* kp,
                  float* samples /* scratch, >= 5 * 75 * 75 floats */, float* dst)
{
    const int d = SIFT_D, n = SIFT_N;
    float angle = 360.f - kp->angle;
    if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    float ori = angle, scl = kp->size * 0.5f;
    int ptx = (int)lrintf(kp->x), pty = (int)lrintf(kp->y);
    float cos_t = cosf(ori * (float)(M_PI / 180));
    float sin_t = sinf(ori * (float)(M_PI / 180));
    float bins_per_rad = n / 360.f;
    float exp_scale = -1.f / (d * d * 0.5f);
    float hist_width = SIFT_DESCR_SCL_FCTR * scl;
    int radius = (int)lrintf(hist_width * 1.4142135623730951f * (d + 1) * 0.5f);
    int diag = (int)sqrt((double)cols * cols + (double)rows * rows);
    if (radius > diag) radius = diag;
    cos_t /= hist_width;
    sin_t /= hist_width;

    float hist_buf[1 + (SIFT_D + 2) * (SIFT_D + 2) * (SIFT_N + 2)];
    float* hist = hist_buf + 1; /* guard slot for the o0 == -1 quirk at cell 0 */
    memset(hist_buf, 0, sizeof(hist_buf));

    int len = (radius * 2 + 1) * (radius * 2 + 1);
    float* own = NULL;
    if (len > 75 * 75) samples = own = (float*)malloc(sizeof(float) * 5 * (size_t)len);
    float *X = samples, *Y = X + len, *RB = Y + len, *CB = RB + len, *W = CB + len;
    int k = 0;
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            float c_rot = (float)j * cos_t - (float)i * sin_t;
            float r_rot = (float)j * sin_t + (float)i * cos_t;
            float rbin = r_rot + (float)(d / 2) - 0.5f;
            float cbin = c_rot + (float)(d / 2) - 0.5f;
            int r = pty + i, c = ptx + j;
            if (rbin > -1 && rbin < d && cbin > -1 && cbin < d &&
                r > 0 && r < rows - 1 && c > 0 && c < cols - 1) {
                X[k] = img[(size_t)r * cols + c + 1] - img[(size_t)r * cols + c - 1];
                Y[k] = img[(size_t)(r - 1) * cols + c] - img[(size_t)(r + 1) * cols + c];
                RB[k] = rbin;
                CB[k] = cbin;
                W[k] = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
                k++;
            }
        }
    len = k;
    const int var = g_sift_variant;
    double hist_d[(SIFT_D + 2) * (SIFT_D + 2) * (SIFT_N + 2) + 1];
    if (var == 3) memset(hist_d, 0, sizeof(hist_d));
    for (int kk = 0; kk < len; kk++) {
        k = var == 1 ? len - 1 - kk : kk;
        float ori_k = orc_fast_atan2_deg(Y[k], X[k]);
        float mag_k = sqrtf(fmaf(X[k], X[k], Y[k] * Y[k]));
        float w_k = orc_exp32f(W[k]);
        float rbin = RB[k], cbin = CB[k];
        float obin = (ori_k - ori) * bins_per_rad;
        float mag = mag_k * w_k;
        int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin), o0 = (int)floorf(obin);
        rbin -= (float)r0;
        cbin -= (float)c0;
        obin -= (float)o0;
        if (o0 < 0) o0 += n;
        if (o0 >= n) o0 -= n;
        if (var == 2) {
            mag = round_sig11(mag);
            rbin = round_sig11(rbin);
            cbin = round_sig11(cbin);
            obin = round_sig11(obin);
        }
        float v_r1 = mag * rbin, v_r0 = mag - v_r1;
        float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
        float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
        float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
        float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
        float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
        float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
        int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
        if (var == 3) {
            double* hd = hist_d + 1;
            hd[idx] += v_rco000; hd[idx + 1] += v_rco001; hd[idx + (n + 2)] += v_rco010; hd[idx + (n + 3)] += v_rco011;
            hd[idx + (d + 2) * (n + 2)] += v_rco100; hd[idx + (d + 2) * (n + 2) + 1] += v_rco101;
            hd[idx + (d + 3) * (n + 2)] += v_rco110; hd[idx + (d + 3) * (n + 2) + 1] += v_rco111;
            continue;
        }
        hist[idx] += v_rco000;
        hist[idx + 1] += v_rco001;
        hist[idx + (n + 2)] += v_rco010;
        hist[idx + (n + 3)] += v_rco011;
        hist[idx + (d + 2) * (n + 2)] += v_rco100;
        hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
        hist[idx + (d + 3) * (n + 2)] += v_rco110;
        hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
    }

    if (var == 3)
        for (int i = 0; i < (SIFT_D + 2) * (SIFT_D + 2) * (SIFT_N + 2) + 1; i++) hist_buf[i] = (float)hist_d[i];
    float raw[SIFT_D * SIFT_D * SIFT_N];
    for (int i = 0; i < d; i++)
        for (int j = 0; j < d; j++) {
            int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
            hist[idx] += hist[idx + n];
            hist[idx + 1] += hist[idx + n + 1];
            for (int q = 0; q < n; q++) raw[(i * d + j) * n + q] = hist[idx + q];
        }
    /* first norm: 8-lane fma partials (AVX2 v_fma) + v_reduce_sum order */
    const int L = d * d * n;
    float lane[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (k = 0; k < L; k++) lane[k & 7] = fmaf(raw[k], raw[k], lane[k & 7]);
    float nrm2 = ((lane[0] + lane[4]) + (lane[1] + lane[5])) + ((lane[2] + lane[6]) + (lane[3] + lane[7]));
    float thr = sqrtf(nrm2) * SIFT_DESCR_MAG_THR;
    nrm2 = 0;
    for (k = 0; k < L; k++) {
        float val = raw[k] < thr ? raw[k] : thr;
        raw[k] = val;
        nrm2 += val * val;
    }
    float s = sqrtf(nrm2);
    nrm2 = SIFT_INT_DESCR_FCTR / (s > FLT_EPSILON ? s : FLT_EPSILON);
    for (k = 0; k < L; k++) {
        float v = rintf(raw[k] * nrm2);
        dst[k] = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
    }
    free(own);
}

void orc_sift_describe(const float* base, int w, int h, const orc_kp* kps, int n, float* desc)
{
    exptab_init();
#pragma omp parallel
    {
        float* scratch = (float*)malloc(sizeof(float) * 5 * 75 * 75 + 64);
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < n; i++) orc_sift_one(base, w, h, &kps[i], scratch, desc + (size_t)i * 128);
        free(scratch);
    }
}

void orc_sift_compute(const uint8_t* bgr, int w, int h, size_t step,
                      const orc_kp* kps, int n, float* desc)
{
    uint8_t* gray = (uint8_t*)malloc((size_t)w * h);
    float* base = (float*)malloc(sizeof(float) * (size_t)w * h);
    orc_bgr2gray(bgr, w, h, step, gray);
    orc_sift_base(gray, w, h, base);
    orc_sift_describe(base, w, h, kps, n, desc);
    free(base);
    free(gray);
}
