/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED against
 * OpenCV itself (not in this image); cross-checked piecewise in
 * tests/test_oracle.py (blur vs a float64 numpy convolution, pyramid sizes and
 * sigmas, DoG extrema vs a brute-force numpy scan, blob scale/position).
 *
 * The full SIFT detector: cv::SIFT::create() (nfeatures 0, nOctaveLayers 3,
 * contrastThreshold 0.04, edgeThreshold 10, sigma 1.6, CV_32F, no precise
 * upscale) ->detectAndCompute(image, noArray(), kps, desc) without provided
 * keypoints -- the "full SIFT detector" row of SURVEY.md 8(f) (north_star:
 * "SIFT (DoG pyramid, extrema, orientation histogram, 128-D descriptor)").  The
 * reference path itself never reaches it (its FAST keypoints take the
 * provided-keypoints branch, sift.c); the restatement follows OpenCV 4.8
 * features2d/src/sift.dispatch.cpp (createInitialImage, buildGaussianPyramid,
 * buildDoGPyramid, detectAndCompute, calcDescriptors) and sift.simd.hpp
 * (findScaleSpaceExtrema, adjustLocalExtrema, calcOrientationHist,
 * calcSIFTDescriptor), features2d/src/keypoint.cpp (removeDuplicatedSorted),
 * imgproc resize (INTER_LINEAR generic float path, INTER_NEAREST) and
 * GaussianBlur (RowVec_32f / SymmColumnVec_32f, as sift.c), core Matx 3x3
 * determinant / Cramer solve.
 *
 * Arithmetic conventions (the GPU kernels follow the same ones, so GPU and
 * oracle agree bit for bit on keypoints):
 *   - scalar C++ expressions: no contraction, left-to-right evaluation;
 *   - OpenCV SIMD v_fma / v_muladd forms: fmaf (AVX2 build), applied to every
 *     element (tail loops are not modelled);
 *   - powf(2, e) as (float)exp2((double)e) (correctly rounded save for rare
 *     double-rounding cases; glibc powf may differ in the last ulp).
 */
#include "oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define N_LAYERS 3
#define CONTRAST_THR 0.04f
#define EDGE_THR 10.f
#define SIGMA 1.6f
#define IMG_BORDER 5
#define MAX_INTERP_STEPS 5
#define ORI_HIST_BINS 36
#define ORI_SIG_FCTR 1.5f
#define ORI_RADIUS (3 * ORI_SIG_FCTR)
#define ORI_PEAK_RATIO 0.8f

static int refl101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

/* GaussianBlur(src, dst, Size(), sigma, sigma) on CV_32F, BORDER_REFLECT_101:
 * ksize = cvRound(sigma * 4 * 2 + 1) | 1; RowVec_32f fma chain from 0,
 * SymmColumnVec_32f S0 * k0 then fma(S[m] + S[-m], k[m], .) */
int orc_blur_ksize(double sigma) { return (int)lrint(sigma * 4 * 2 + 1) | 1; }

void orc_gauss_blur_f32(const float* src, int w, int h, double sigma, float* dst)
{
    const int ks = orc_blur_ksize(sigma), r = ks / 2;
    float kern[128];
    orc_gauss_kernel_f32(ks, sigma, kern);
    float* tmp = (float*)malloc(sizeof(float) * (size_t)w * h);
    int* xo = (int*)malloc(sizeof(int) * (size_t)(w + 2 * r));
    for (int x = -r; x < w + r; x++) xo[x + r] = refl101(x, w);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++) {
        const float* s = src + (size_t)y * w;
        float* d = tmp + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            float acc = 0.f;
            for (int k = 0; k < ks; k++) acc = fmaf(s[xo[x + k]], kern[k], acc);
            d[x] = acc;
        }
    }
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++) {
        float* d = dst + (size_t)y * w;
        const float* c = tmp + (size_t)y * w;
        for (int x = 0; x < w; x++) d[x] = c[x] * kern[r];
        for (int m = 1; m <= r; m++) {
            const float* up = tmp + (size_t)refl101(y - m, h) * w;
            const float* dn = tmp + (size_t)refl101(y + m, h) * w;
            for (int x = 0; x < w; x++) d[x] = fmaf(dn[x] + up[x], kern[r + m], d[x]);
        }
    }
    free(xo);
    free(tmp);
}

/* resize(src, dst, Size(2w, 2h), 0, 0, INTER_LINEAR), generic float path:
 * fx = (float)((dx + 0.5) * 0.5 - 0.5), sx = floor, columns clamp with fx = 0
 * (and a single tap S[sx] * 1 past the right edge); rows clip the source row
 * index to [0, h - 1] without touching fy.  HResizeLinear: S0 a0 + S1 a1;
 * VResizeLinear (SSE baseline v_muladd = mul + add): H0 b0 + H1 b1. */
void orc_resize2x_linear(const float* src, int w, int h, float* dst)
{
    const int W = 2 * w, H = 2 * h;
    int* xs = (int*)malloc(sizeof(int) * (size_t)W);
    float* ax = (float*)malloc(sizeof(float) * 2 * (size_t)W);
    int xmax = W;
    for (int dx = 0; dx < W; dx++) {
        float fx = (float)((dx + 0.5) * 0.5 - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= w) {
            if (xmax > dx) xmax = dx;
            if (sx >= w - 1) { fx = 0.f; sx = w - 1; }
        }
        xs[dx] = sx;
        ax[2 * dx] = 1.f - fx;
        ax[2 * dx + 1] = fx;
    }
    float* hbuf = (float*)malloc(sizeof(float) * (size_t)W * h);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < h; y++) {
        const float* S = src + (size_t)y * w;
        float* D = hbuf + (size_t)y * W;
        for (int dx = 0; dx < W; dx++) {
            const int sx = xs[dx];
            if (dx < xmax) D[dx] = S[sx] * ax[2 * dx] + S[sx + 1] * ax[2 * dx + 1];
            else D[dx] = S[sx] * 1.f;
        }
    }
#pragma omp parallel for schedule(static)
    for (int dy = 0; dy < H; dy++) {
        float fy = (float)((dy + 0.5) * 0.5 - 0.5);
        int sy = (int)floorf(fy);
        fy -= (float)sy;
        const float b0 = 1.f - fy, b1 = fy;
        int s0 = sy < 0 ? 0 : (sy > h - 1 ? h - 1 : sy);
        int s1 = sy + 1 < 0 ? 0 : (sy + 1 > h - 1 ? h - 1 : sy + 1);
        const float* S0 = hbuf + (size_t)s0 * W;
        const float* S1 = hbuf + (size_t)s1 * W;
        float* D = dst + (size_t)dy * W;
        for (int x = 0; x < W; x++) D[x] = S0[x] * b0 + S1[x] * b1;
    }
    free(hbuf);
    free(ax);
    free(xs);
}

/* resize(src, dst, Size(w / 2, h / 2), 0, 0, INTER_NEAREST): sx = floor(dx * (sw / dw)) */
void orc_resize_half_nearest(const float* src, int w, int h, float* dst)
{
    const int W = w / 2, H = h / 2;
    const double ifx = 1. / ((double)W / w), ify = 1. / ((double)H / h);
    for (int y = 0; y < H; y++) {
        int sy = (int)floor(y * ify);
        if (sy > h - 1) sy = h - 1;
        for (int x = 0; x < W; x++) {
            int sx = (int)floor(x * ifx);
            if (sx > w - 1) sx = w - 1;
            dst[(size_t)y * W + x] = src[(size_t)sy * w + sx];
        }
    }
}

/* nOctaves = cvRound(log2(min(base)) - 2) - firstOctave, firstOctave = -1 */
int orc_sift_octaves(int w, int h)
{
    int m = 2 * w < 2 * h ? 2 * w : 2 * h;
    return (int)lrint(log((double)m) / log(2.) - 2) + 1;
}

/* buildGaussianPyramid sigmas from SIFT_Impl's double sigma = 1.6 (the float
 * 1.6f reaches only createInitialImage and adjustLocalExtrema):
 * sig[0] = 1.6, sig[i] = sqrt(sig_total^2 - sig_prev^2) */
void orc_sift_sigmas(double* sig)
{
    const double sigma = 1.6;
    sig[0] = sigma;
    double k = pow(2., 1. / N_LAYERS);
    for (int i = 1; i < N_LAYERS + 3; i++) {
        double sig_prev = pow(k, (double)(i - 1)) * sigma;
        double sig_total = sig_prev * k;
        sig[i] = sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
}

/* createInitialImage(doubleImageSize = true): sig_diff = sqrtf(max(1.6^2 - 0.5^2 * 4, 0.01)) */
float orc_sift_sigma_diff2x(void)
{
    float s = SIGMA * SIGMA - 0.5f * 0.5f * 4;
    return sqrtf(s > 0.01f ? s : 0.01f);
}

typedef struct {
    int nOct, *w, *h;
    float** g;     /* nOct * 6 Gaussian layers */
    float** d;     /* nOct * 5 DoG layers */
} pyr_t;

static void build_pyramid(const uint8_t* gray, int w0, int h0, pyr_t* P)
{
    const int nL = N_LAYERS + 3, nD = N_LAYERS + 2;
    P->nOct = orc_sift_octaves(w0, h0);
    P->w = (int*)malloc(sizeof(int) * P->nOct);
    P->h = (int*)malloc(sizeof(int) * P->nOct);
    P->g = (float**)calloc((size_t)P->nOct * nL, sizeof(float*));
    P->d = (float**)calloc((size_t)P->nOct * nD, sizeof(float*));
    double sig[N_LAYERS + 3];
    orc_sift_sigmas(sig);
    float* f = (float*)malloc(sizeof(float) * (size_t)w0 * h0);
    for (size_t i = 0; i < (size_t)w0 * h0; i++) f[i] = (float)gray[i];
    const int W = 2 * w0, H = 2 * h0;
    float* dbl = (float*)malloc(sizeof(float) * (size_t)W * H);
    orc_resize2x_linear(f, w0, h0, dbl);
    free(f);
    for (int o = 0; o < P->nOct; o++) {
        const int w = o == 0 ? W : P->w[o - 1] / 2, h = o == 0 ? H : P->h[o - 1] / 2;
        P->w[o] = w;
        P->h[o] = h;
        for (int i = 0; i < nL; i++) {
            float* dst = (float*)malloc(sizeof(float) * (size_t)w * h);
            if (o == 0 && i == 0) orc_gauss_blur_f32(dbl, w, h, (double)orc_sift_sigma_diff2x(), dst);
            else if (i == 0) orc_resize_half_nearest(P->g[(o - 1) * nL + N_LAYERS], P->w[o - 1], P->h[o - 1], dst);
            else orc_gauss_blur_f32(P->g[o * nL + i - 1], w, h, sig[i], dst);
            P->g[o * nL + i] = dst;
        }
        for (int i = 0; i < nD; i++) {
            float* dd = (float*)malloc(sizeof(float) * (size_t)w * h);
            const float *a = P->g[o * nL + i + 1], *b = P->g[o * nL + i];
            for (size_t k = 0; k < (size_t)w * h; k++) dd[k] = a[k] - b[k];
            P->d[o * nD + i] = dd;
        }
    }
    free(dbl);
}

static void free_pyramid(pyr_t* P)
{
    for (int i = 0; i < P->nOct * (N_LAYERS + 3); i++) free(P->g[i]);
    for (int i = 0; i < P->nOct * (N_LAYERS + 2); i++) free(P->d[i]);
    free(P->g); free(P->d); free(P->w); free(P->h);
}

/* Matx_DetOp<float, 3> and Matx_FastSolveOp<float, 3, 1> (Cramer's rule) */
static int solve33(const float a[9], const float b[3], float x[3])
{
#define A(i, j) a[(i) * 3 + (j)]
    float d = A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) - A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
              A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1));
    if (d == 0) { x[0] = x[1] = x[2] = 0.f; return 0; }
    d = 1 / d;
    x[0] = d * (b[0] * (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) - A(0, 1) * (b[1] * A(2, 2) - A(1, 2) * b[2]) +
                A(0, 2) * (b[1] * A(2, 1) - A(1, 1) * b[2]));
    x[1] = d * (A(0, 0) * (b[1] * A(2, 2) - A(1, 2) * b[2]) - b[0] * (A(1, 0) * A(2, 2) - A(1, 2) * A(2, 0)) +
                A(0, 2) * (A(1, 0) * b[2] - b[1] * A(2, 0)));
    x[2] = d * (A(0, 0) * (A(1, 1) * b[2] - b[1] * A(2, 1)) - A(0, 1) * (A(1, 0) * b[2] - b[1] * A(2, 0)) +
                b[0] * (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)));
    return 1;
#undef A
}

/* adjustLocalExtrema: up to 5 Newton steps on the DoG scale space, contrast and
 * edge tests; fills the keypoint in doubled-image (pyramid octave o) units */
static int adjust_extremum(const pyr_t* P, int o, int* layer_io, int* r_io, int* c_io, orc_kp* kp)
{
    const float img_scale = 1.f / 255, deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale,
                cross_deriv_scale = img_scale * 0.25f;
    const int nD = N_LAYERS + 2, w = P->w[o], h = P->h[o];
    int layer = *layer_io, r = *r_io, c = *c_io, i = 0;
    float xi = 0, xr = 0, xc = 0, contr;
#define IM(R, C) img[(size_t)(R) * w + (C)]
#define PV(R, C) prv[(size_t)(R) * w + (C)]
#define NX(R, C) nxt[(size_t)(R) * w + (C)]
    for (; i < MAX_INTERP_STEPS; i++) {
        const float *img = P->d[o * nD + layer], *prv = P->d[o * nD + layer - 1], *nxt = P->d[o * nD + layer + 1];
        float dD[3] = {(IM(r, c + 1) - IM(r, c - 1)) * deriv_scale, (IM(r + 1, c) - IM(r - 1, c)) * deriv_scale,
                       (NX(r, c) - PV(r, c)) * deriv_scale};
        float v2 = IM(r, c) * 2;
        float dxx = (IM(r, c + 1) + IM(r, c - 1) - v2) * second_deriv_scale;
        float dyy = (IM(r + 1, c) + IM(r - 1, c) - v2) * second_deriv_scale;
        float dss = (NX(r, c) + PV(r, c) - v2) * second_deriv_scale;
        float dxy = (IM(r + 1, c + 1) - IM(r + 1, c - 1) - IM(r - 1, c + 1) + IM(r - 1, c - 1)) * cross_deriv_scale;
        float dxs = (NX(r, c + 1) - NX(r, c - 1) - PV(r, c + 1) + PV(r, c - 1)) * cross_deriv_scale;
        float dys = (NX(r + 1, c) - NX(r - 1, c) - PV(r + 1, c) + PV(r - 1, c)) * cross_deriv_scale;
        float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss}, X[3];
        solve33(H, dD, X);
        xi = -X[2];
        xr = -X[1];
        xc = -X[0];
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3))
            return 0;
        c += (int)lrintf(xc);
        r += (int)lrintf(xr);
        layer += (int)lrintf(xi);
        if (layer < 1 || layer > N_LAYERS || c < IMG_BORDER || c >= w - IMG_BORDER || r < IMG_BORDER ||
            r >= h - IMG_BORDER)
            return 0;
    }
    if (i >= MAX_INTERP_STEPS) return 0;
    {
        const float *img = P->d[o * nD + layer], *prv = P->d[o * nD + layer - 1], *nxt = P->d[o * nD + layer + 1];
        float dD[3] = {(IM(r, c + 1) - IM(r, c - 1)) * deriv_scale, (IM(r + 1, c) - IM(r - 1, c)) * deriv_scale,
                       (NX(r, c) - PV(r, c)) * deriv_scale};
        float t = 0;
        t += dD[0] * xc;
        t += dD[1] * xr;
        t += dD[2] * xi;
        contr = IM(r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * N_LAYERS < CONTRAST_THR) return 0;
        float v2 = IM(r, c) * 2.f;
        float dxx = (IM(r, c + 1) + IM(r, c - 1) - v2) * second_deriv_scale;
        float dyy = (IM(r + 1, c) + IM(r - 1, c) - v2) * second_deriv_scale;
        float dxy = (IM(r + 1, c + 1) - IM(r + 1, c - 1) - IM(r - 1, c + 1) + IM(r - 1, c - 1)) * cross_deriv_scale;
        float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * EDGE_THR >= (EDGE_THR + 1) * (EDGE_THR + 1) * det) return 0;
    }
#undef IM
#undef PV
#undef NX
    kp->x = ((float)c + xc) * (float)(1 << o);
    kp->y = ((float)r + xr) * (float)(1 << o);
    kp->octave = o + (layer << 8) + ((int)lrint(((double)xi + 0.5) * 255) << 16);
    kp->size = SIGMA * (float)exp2((double)(((float)layer + xi) / N_LAYERS)) * (float)(1 << o) * 2;
    kp->response = fabsf(contr);
    kp->angle = -1.f;
    kp->class_id = -1;
    *layer_io = layer;
    *r_io = r;
    *c_io = c;
    return 1;
}

/* calcOrientationHist: 36 bins, Gaussian-weighted gradient magnitudes
 * (hal::exp32f, fastAtan2, magnitude32f v_muladd form), sequential bin sums in
 * sample order, [1 4 6 4 1] / 16 circular smoothing (v_fma form) */
float orc_sift_ori_hist(const float* img, int cols, int rows, int px, int py, int radius, float sigma, float* hist)
{
    const int n = ORI_HIST_BINS;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    float th[ORI_HIST_BINS + 4];
    float* t = th + 2;
    memset(th, 0, sizeof(th));
    for (int i = -radius; i <= radius; i++) {
        const int y = py + i;
        if (y <= 0 || y >= rows - 1) continue;
        for (int j = -radius; j <= radius; j++) {
            const int x = px + j;
            if (x <= 0 || x >= cols - 1) continue;
            const float dx = img[(size_t)y * cols + x + 1] - img[(size_t)y * cols + x - 1];
            const float dy = img[(size_t)(y - 1) * cols + x] - img[(size_t)(y + 1) * cols + x];
            const float W = orc_exp32f((float)(i * i + j * j) * expf_scale);
            const float ori = orc_fast_atan2_deg(dy, dx);
            const float mag = sqrtf(fmaf(dx, dx, dy * dy));
            int bin = (int)lrintf((n / 360.f) * ori);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
            t[bin] += W * mag;
        }
    }
    t[-1] = t[n - 1];
    t[-2] = t[n - 2];
    t[n] = t[0];
    t[n + 1] = t[1];
    float maxval = 0;
    for (int i = 0; i < n; i++) {
        hist[i] = fmaf(t[i - 2] + t[i + 2], 1.f / 16.f, fmaf(t[i - 1] + t[i + 1], 4.f / 16.f, t[i] * (6.f / 16.f)));
        maxval = i == 0 ? hist[0] : (maxval > hist[i] ? maxval : hist[i]);
    }
    return maxval;
}

/* the orientation peaks of one refined extremum (findScaleSpaceExtrema) */
int orc_sift_peaks(const float* hist, float omax, float* angles /* <= 36 */)
{
    const int n = ORI_HIST_BINS;
    const float mag_thr = omax * ORI_PEAK_RATIO;
    int cnt = 0;
    for (int j = 0; j < n; j++) {
        const int l = j > 0 ? j - 1 : n - 1, r2 = j < n - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
            float bin = (float)j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
            bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
            float angle = 360.f - (360.f / n) * bin;
            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            angles[cnt++] = angle;
        }
    }
    return cnt;
}

/* KeyPointsFilter::removeDuplicatedSorted's KeypointGreater */
int orc_kp_less(const orc_kp* a, const orc_kp* b)
{
    if (a->x != b->x) return a->x < b->x;
    if (a->y != b->y) return a->y < b->y;
    if (a->size != b->size) return a->size > b->size;
    if (a->angle != b->angle) return a->angle < b->angle;
    if (a->response != b->response) return a->response > b->response;
    if (a->octave != b->octave) return a->octave > b->octave;
    return a->class_id > b->class_id;
}

static int kp_cmp(const void* pa, const void* pb)
{
    const orc_kp *a = (const orc_kp*)pa, *b = (const orc_kp*)pb;
    return orc_kp_less(a, b) ? -1 : orc_kp_less(b, a) ? 1 : 0;
}

/* sort + drop entries equal to the last kept one in (x, y, size, angle) */
int orc_kp_dedup_sorted(orc_kp* k, int n)
{
    if (n < 2) return n;
    qsort(k, (size_t)n, sizeof(orc_kp), kp_cmp);
    int i = 0;
    for (int j = 1; j < n; j++)
        if (k[i].x != k[j].x || k[i].y != k[j].y || k[i].size != k[j].size || k[i].angle != k[j].angle) k[++i] = k[j];
    return i + 1;
}

typedef struct { orc_kp* v; int n, cap; } kpvec;

static void kpvec_push(kpvec* V, const orc_kp* k)
{
    if (V->n == V->cap) {
        V->cap = V->cap ? 2 * V->cap : 1024;
        V->v = (orc_kp*)realloc(V->v, sizeof(orc_kp) * (size_t)V->cap);
    }
    V->v[V->n++] = *k;
}

/* Extremum candidates: |v| > floor(0.5 * 0.04 / 3 * 255) = 1 and >= (<=) all 26
 * neighbours; rows/cols in [5, size - 5), DoG layers 1..3 */
static int is_extremum(const float* cur, const float* prv, const float* nxt, size_t o, int w)
{
    const float val = cur[o];
    const int threshold = (int)floor(0.5 * 0.04 / N_LAYERS * 255);
    if (!(fabsf(val) > threshold)) return 0;
    const long off[9] = {-w - 1, -w, -w + 1, -1, 0, 1, w - 1, w, w + 1};
    if (val > 0) {
        for (int k = 0; k < 9; k++) {
            if (k != 4 && !(val >= cur[o + off[k]])) return 0;
            if (!(val >= nxt[o + off[k]]) || !(val >= prv[o + off[k]])) return 0;
        }
        return 1;
    }
    if (val < 0) {
        for (int k = 0; k < 9; k++) {
            if (k != 4 && !(val <= cur[o + off[k]])) return 0;
            if (!(val <= nxt[o + off[k]]) || !(val <= prv[o + off[k]])) return 0;
        }
        return 1;
    }
    return 0;
}

int orc_sift_detect(const uint8_t* bgr, int w, int h, size_t step, orc_kp* out, int cap, float* desc)
{
    uint8_t* gray = (uint8_t*)malloc((size_t)w * h);
    orc_bgr2gray(bgr, w, h, step, gray);
    pyr_t P;
    build_pyramid(gray, w, h, &P);
    free(gray);
    const int nL = N_LAYERS + 3, nD = N_LAYERS + 2;
    kpvec V = {0, 0, 0};
    float hist[ORI_HIST_BINS], angles[ORI_HIST_BINS];
    for (int o = 0; o < P.nOct; o++) {
        const int ow = P.w[o], oh = P.h[o];
        for (int i = 1; i <= N_LAYERS; i++) {
            const float *cur = P.d[o * nD + i], *prv = P.d[o * nD + i - 1], *nxt = P.d[o * nD + i + 1];
            for (int r = IMG_BORDER; r < oh - IMG_BORDER; r++)
                for (int c = IMG_BORDER; c < ow - IMG_BORDER; c++) {
                    if (!is_extremum(cur, prv, nxt, (size_t)r * ow + c, ow)) continue;
                    int r1 = r, c1 = c, layer = i;
                    orc_kp kp;
                    if (!adjust_extremum(&P, o, &layer, &r1, &c1, &kp)) continue;
                    const float scl_octv = kp.size * 0.5f / (float)(1 << o);
                    const float omax = orc_sift_ori_hist(P.g[o * nL + layer], ow, oh, c1, r1,
                                                         (int)lrintf(ORI_RADIUS * scl_octv), ORI_SIG_FCTR * scl_octv,
                                                         hist);
                    const int na = orc_sift_peaks(hist, omax, angles);
                    for (int a = 0; a < na; a++) {
                        kp.angle = angles[a];
                        kpvec_push(&V, &kp);
                    }
                }
        }
    }
    int n = orc_kp_dedup_sorted(V.v, V.n);
    /* firstOctave = -1: back to input-image units */
    for (int k = 0; k < n; k++) {
        orc_kp* kp = &V.v[k];
        kp->octave = (kp->octave & ~255) | ((kp->octave - 1) & 255);
        kp->x *= 0.5f;
        kp->y *= 0.5f;
        kp->size *= 0.5f;
    }
    const int m = n < cap ? n : cap;
    memcpy(out, V.v, sizeof(orc_kp) * (size_t)m);
    if (desc) {
        /* calcDescriptors: the keypoint's own octave / layer image, pt and size in its units */
#pragma omp parallel
        {
            float* scratch = (float*)malloc(sizeof(float) * 5 * 75 * 75 + 64);
#pragma omp for schedule(dynamic, 16)
            for (int k = 0; k < m; k++) {
                const orc_kp* kp = &V.v[k];
                int oct = kp->octave & 255, layer = (kp->octave >> 8) & 255;
                oct = oct < 128 ? oct : (-128 | oct);
                const float scale = oct >= 0 ? 1.f / (float)(1 << oct) : (float)(1 << -oct);
                orc_kp u = *kp;
                u.x = kp->x * scale;
                u.y = kp->y * scale;
                u.size = kp->size * scale;
                const int pi = oct + 1;   /* pyramid octave index (firstOctave = -1) */
                orc_sift_one(P.g[pi * nL + layer], P.w[pi], P.h[pi], &u, scratch, desc + (size_t)k * 128);
            }
            free(scratch);
        }
    }
    free(V.v);
    free_pyramid(&P);
    return n;
}

/* pieces for the tests: the whole Gaussian / DoG pyramid of a gray image,
 * concatenated octave by octave (sizes from orc_sift_pyr_dims) */
int orc_sift_pyr_dims(int w, int h, int* ow, int* oh)
{
    const int n = orc_sift_octaves(w, h);
    int W = 2 * w, H = 2 * h;
    for (int o = 0; o < n; o++) {
        ow[o] = W;
        oh[o] = H;
        W /= 2;
        H /= 2;
    }
    return n;
}

void orc_sift_pyramid(const uint8_t* gray, int w, int h, float* gauss, float* dog)
{
    pyr_t P;
    build_pyramid(gray, w, h, &P);
    const int nL = N_LAYERS + 3, nD = N_LAYERS + 2;
    size_t go = 0, dof = 0;
    for (int o = 0; o < P.nOct; o++) {
        const size_t px = (size_t)P.w[o] * P.h[o];
        for (int i = 0; i < nL; i++, go += px)
            if (gauss) memcpy(gauss + go, P.g[o * nL + i], px * sizeof(float));
        for (int i = 0; i < nD; i++, dof += px)
            if (dog) memcpy(dog + dof, P.d[o * nD + i], px * sizeof(float));
    }
    free_pyramid(&P);
}
