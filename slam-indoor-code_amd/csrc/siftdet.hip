// Full SIFT detector on gfx950: cv::SIFT::create()->detectAndCompute(image,
// noArray(), kps, desc) without provided keypoints (OpenCV 4.8
// sift.dispatch.cpp / sift.simd.hpp; restated in oracle/siftdet.c, which this
// file matches operation for operation).  SURVEY.md 8(f) rank 2: the reference
// path itself only reaches SIFT through FAST keypoints (sift.hip / sift_tab.hip).
//
// Device pipeline for one frame (HBM layout: one float plane per pyramid
// layer, octave by octave: 6 Gaussian layers, and 5 DoG planes only under
// SLAMHIP_SD_DOG=1):
//   sd_upsample   gray u8 -> 2x float image, resize INTER_LINEAR's generic
//                 float path (column clamp with fx = 0, row-index clip); by
//                 default evaluated inside the first blur's staging instead
//                 (sd_blur<5, true>: the doubled image never reaches HBM)
//   sd_blur       separable Gaussian, 64 x 32 output tile staged in LDS with a
//                 REFLECT_101 halo of up to 13; RowVec_32f fma chain from 0 and
//                 SymmColumnVec_32f symmetric fma form; writes the layer
//   sd_down       next octave's layer 0 = INTER_NEAREST half of layer 3
//   sd_extrema    26-neighbour scale-space extrema of DoG layers 1..3 with
//                 |v| > 1, appended per wavefront (one atomic per wave); the
//                 DoG values are the Gaussian layers' differences, formed
//                 while staging (the subtraction the DoG plane would hold)
//   sd_refine     one wavefront per candidate: adjustLocalExtrema on lane 0,
//                 then the 36-bin orientation histogram with all 64 lanes
//                 evaluating samples and 36 lanes summing each bin's samples
//                 in sample order (the oracle's sequential order, so the bins
//                 are bit-identical), smoothing, peaks -> keypoints
//   host          KeyPointsFilter::removeDuplicatedSorted (std::sort with the
//                 same comparator), firstOctave = -1 rescale, cosf / sinf
//   sd_desc       16 lanes per keypoint (lane = inner histogram cell): the
//                 calcSIFTDescriptor samples of each cell gathered in the
//                 reference's order into registers -- bit-identical to the
//                 oracle, no atomics -- then 0.2 clamp, x512, saturate
// Bounds: the pyramid is HBM-bound (each blur reads one plane and writes one);
// sd_refine / sd_desc are latency-bound gathers.
//
// Batches (slam_sift_detect_batch): every launch covers all frames of a
// device-resident batch (blockIdx.z = frame, one pyramid per frame, candidates
// and keypoints carry their frame), so the ~60 per-octave launches of a frame
// are paid once per batch and the small octaves fill the chip.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "kp_order.h"
#include "sift_dev.h"
#include "slamhip_internal.h"

namespace slamhip {

namespace {
using namespace sd;

constexpr int kLayers = 3;                 // nOctaveLayers
constexpr int kGL = kLayers + 3, kDL = kLayers + 2;
constexpr int kMaxOct = 16;
constexpr int kImgBorder = 5;
constexpr int kOriBins = 36;
constexpr int kOriMaxR = 16;               // cvRound(4.5 * scl_octv), scl_octv < 1.6 * 2^(3.5 / 3)
constexpr int kOriMaxS = (2 * kOriMaxR + 1) * (2 * kOriMaxR + 1);
constexpr float kSigma = 1.6f;

struct Oct {
    int w, h;
    size_t g[kGL], d[kDL];                 // float offsets into the pyramid buffer
};

struct PyrInfo {
    int n;
    Oct o[kMaxOct];
};

// ---- sd_upsample: resize(gray_f32, 2w x 2h, INTER_LINEAR) ----
// The doubled image's pixel (dx, dy) from the u8 gray w x h, separably: ups_src
// gives the four source bytes' offsets, ups_weights / ups_weights_y the column
// and row weights (sd_upsample's operations)
struct UpsTap {
    int o00, o01, o10, o11;                // byte offsets: rows s0 / s1, columns sx / sx + 1 (clamped)
};
__device__ __forceinline__ UpsTap ups_src(int w, int h, int dx, int dy)
{
    float fx = (float)((dx + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    if (sx < 0) sx = 0;
    if (sx + 1 >= w && sx >= w - 1) sx = w - 1;
    const int sy = (int)floorf((float)((dy + 0.5) * 0.5 - 0.5));
    const int s0 = min(max(sy, 0), h - 1), s1 = min(max(sy + 1, 0), h - 1);
    const int sx1 = min(sx + 1, w - 1);
    return {s0 * w + sx, s0 * w + sx1, s1 * w + sx, s1 * w + sx1};
}
// the column weights (a0, a1); in sd_upsample's single-column case (fx = 0)
// a0 = 1, a1 = 0, and g00 * 1 + g01 * 0 is g00 * 1.f exactly
__device__ __forceinline__ void ups_weights(int w, int dx, float& a0, float& a1)
{
    float fx = (float)((dx + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0.f; sx = 0; }
    if (sx + 1 >= w && sx >= w - 1) fx = 0.f;
    a0 = 1.f - fx;
    a1 = fx;
}
__device__ __forceinline__ void ups_weights_y(int dy, float& b0, float& b1)
{
    float fy = (float)((dy + 0.5) * 0.5 - 0.5);
    fy -= (float)(int)floorf(fy);
    b0 = 1.f - fy;
    b1 = fy;
}

__global__ __launch_bounds__(256) void sd_upsample(const uint8_t* __restrict__ g, int w, int h, float* __restrict__ dst,
                                                   size_t gstride, size_t dstride)
{
    const int W = 2 * w, dx = blockIdx.x * 256 + threadIdx.x, dy = blockIdx.y;
    g += blockIdx.z * gstride;
    dst += blockIdx.z * dstride;
    if (dx >= W) return;
    float fx = (float)((dx + 0.5) * 0.5 - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0.f; sx = 0; }
    const bool single = sx + 1 >= w;
    if (single && sx >= w - 1) { fx = 0.f; sx = w - 1; }
    const float a0 = 1.f - fx, a1 = fx;
    float fy = (float)((dy + 0.5) * 0.5 - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const float b0 = 1.f - fy, b1 = fy;
    const int s0 = min(max(sy, 0), h - 1), s1 = min(max(sy + 1, 0), h - 1);
    const uint8_t* r0 = g + (size_t)s0 * w;
    const uint8_t* r1 = g + (size_t)s1 * w;
    float h0, h1;
    if (single) {
        h0 = (float)r0[sx] * 1.f;
        h1 = (float)r1[sx] * 1.f;
    } else {
        h0 = (float)r0[sx] * a0 + (float)r0[sx + 1] * a1;
        h1 = (float)r1[sx] * a0 + (float)r1[sx + 1] * a1;
    }
    dst[(size_t)dy * W + dx] = h0 * b0 + h1 * b1;
}

// ---- sd_blur: GaussianBlur(src, dst, Size(), sigma) (+ dog = dst - src) ----
#ifndef SD_BLUR_TH
#define SD_BLUR_TH 32
#endif
constexpr int kTW = 64, kTH = SD_BLUR_TH, kMaxR = 13;
template <int R>
__host__ __device__ constexpr int lw_c() { return kTW + 2 * R; }   // staged columns

struct BlurParams {
    const float* src;
    const uint8_t* gray;                   // UPS: the u8 frames (gw x gh, gstride bytes apart) the source doubles
    size_t gstride;
    int gw, gh;
    float* dst;
    float* dog;                            // nullable
    size_t sstride, dstride;               // per-frame strides (floats) of src and dst / dog
    int w, h, r;
    int xcd;                               // tiles in XCD-contiguous order (xcd_tile)
    float k[2 * kMaxR + 1];
};

// Register-blocked: the row pass computes 4 adjacent outputs per task from one
// 16-B-aligned window of 2R + 4 staged floats (fma chain from 0, taps
// ascending, per output); the column pass gives each thread an 8-row strip of
// one column with its 2R + 8 inputs in registers (symmetric fma form).  Same
// per-output operations as before, ~8x fewer LDS instructions.
// UPS: the source is resize(gray, 2w x 2h, INTER_LINEAR) evaluated per staged
// pixel from the u8 frame (sd_upsample's arithmetic, separable tables), so the
// doubled base image is never written and read back.
template <int R, bool UPS = false>
__global__ __launch_bounds__(256) void sd_blur(BlurParams p)
{
    constexpr int KS = 2 * R + 1, LH = kTH + 2 * R;
    constexpr int LWP = (kTW + 2 * R + 3 + 3) & ~3;      // staged row pitch (float4 windows stay in bounds)
    constexpr int NW4 = (2 * R + 4 + 3) / 4;              // float4 loads per 4-output window
    constexpr int SR = kTH / 4;                           // column-pass rows per thread (4 strips)
    __shared__ __attribute__((aligned(16))) float in[LH * LWP];
    __shared__ __attribute__((aligned(16))) float rowp[LH * kTW];
    int bx, by, bz;
    xcd_tile(p.xcd != 0, bx, by, bz);
    const int x0 = bx * kTW, y0 = by * kTH, tid = threadIdx.x;
    p.src += bz * p.sstride;
    p.dst += bz * p.dstride;
    if (p.dog) p.dog += bz * p.dstride;
    float k[KS];
#pragma unroll
    for (int i = 0; i < KS; i++) k[i] = p.k[i];
    const int lw = kTW + 2 * R;
    // interior tiles: 16-byte loads (4-byte aligned; up to 3 floats past the
    // staged width land in the row's pad), so the tile stays clear of the right edge
    const bool interior = x0 - R >= 0 && x0 + kTW + R + 3 <= p.w && y0 - R >= 0 && y0 + kTH + R <= p.h;
    if constexpr (UPS) {
        // resize's per-column (sx, sx + 1, a0, a1) and per-row (s0, s1, b0, b1)
        // terms are separable: one table entry per staged column / row (the
        // REFLECT_101 index first), then every staged pixel's four gathers,
        // then the values -- sd_upsample's operations per pixel
        constexpr int LW = lw_c<R>(), NPX = LH * LW, NIT = (NPX + 255) / 256;
        __shared__ int4 s_col[LW], s_row[LH];
        if (tid < LW) {
            const int dx = reflect101(x0 - R + tid, p.w);
            const UpsTap tp = ups_src(p.gw, p.gh, dx, 0);
            float a0, a1;
            ups_weights(p.gw, dx, a0, a1);
            s_col[tid] = make_int4(tp.o00, tp.o01, __float_as_int(a0), __float_as_int(a1));
        } else if (tid >= 128 && tid < 128 + LH) {
            const int dy = reflect101(y0 - R + tid - 128, p.h);
            const UpsTap tp = ups_src(p.gw, p.gh, 0, dy);
            float b0, b1;
            ups_weights_y(dy, b0, b1);
            s_row[tid - 128] = make_int4(tp.o00, tp.o10, __float_as_int(b0), __float_as_int(b1));
        }
        __syncthreads();
        const uint8_t* g = p.gray + (size_t)bz * p.gstride;
        uint32_t b[NIT][4];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = min(tid + 256 * it, NPX - 1);
            const int ry = i / LW, rx = i - ry * LW;
            const int4 cx = s_col[rx], cy = s_row[ry];
            b[it][0] = g[cy.x + cx.x]; b[it][1] = g[cy.x + cx.y]; b[it][2] = g[cy.y + cx.x]; b[it][3] = g[cy.y + cx.y];
        }
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = tid + 256 * it;
            if (i < NPX) {
                const int ry = i / LW, rx = i - ry * LW;
                const int4 cx = s_col[rx], cy = s_row[ry];
                const float a0 = __int_as_float(cx.z), a1 = __int_as_float(cx.w);
                const float h0 = (float)b[it][0] * a0 + (float)b[it][1] * a1;
                const float h1 = (float)b[it][2] * a0 + (float)b[it][3] * a1;
                in[ry * LWP + rx] = h0 * __int_as_float(cy.z) + h1 * __int_as_float(cy.w);
            }
        }
    } else if (interior) {
        typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
        constexpr int NL = (kTW + 2 * R + 3) / 4;
        static_assert(4 * NL <= LWP, "16-byte row loads stay in the staged row");
        const float* src = p.src + (size_t)(y0 - R) * p.w + (x0 - R);
        // every load of the thread issued before the first LDS store: a
        // load / wait / store loop pays one memory latency per iteration.  The
        // loads are unconditional (a past-the-end index reloads the last
        // element), so no branch splits them and no wait lands between them
        constexpr int NIT = (LH * NL + 255) / 256;
        f4u v[NIT];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = min(tid + 256 * it, LH * NL - 1);
            const int ry = i / NL, j = i - ry * NL;
            v[it] = *reinterpret_cast<const f4u*>(src + (size_t)ry * p.w + 4 * j);
        }
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            // unconditional too (a past-the-end index stores the last piece's
            // values again): no branch for the compiler to sink a load into
            const int i = min(tid + 256 * it, LH * NL - 1);
            const int ry = i / NL, j = i - ry * NL;
            *reinterpret_cast<float4*>(in + ry * LWP + 4 * j) = make_float4(v[it].x, v[it].y, v[it].z, v[it].w);
        }
    } else {
        for (int i = tid; i < LH * lw; i += 256) {
            const int ry = i / lw, rx = i - ry * lw;
            const int gy = reflect101(y0 - R + ry, p.h), gx = reflect101(x0 - R + rx, p.w);
            in[ry * LWP + rx] = p.src[(size_t)gy * p.w + gx];
        }
    }
    __syncthreads();
    for (int t = tid; t < LH * (kTW / 4); t += 256) {
        const int ry = t / (kTW / 4), xq = (t - ry * (kTW / 4)) * 4;
        const float4* w4 = reinterpret_cast<const float4*>(in + ry * LWP + xq);
        float win[NW4 * 4];
#pragma unroll
        for (int m = 0; m < NW4; m++) {
            const float4 v = w4[m];
            win[4 * m] = v.x; win[4 * m + 1] = v.y; win[4 * m + 2] = v.z; win[4 * m + 3] = v.w;
        }
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < KS; tap++)
#pragma unroll
            for (int o = 0; o < 4; o++) acc[o] = fmaf(win[o + tap], k[tap], acc[o]);
        *reinterpret_cast<float4*>(rowp + ry * kTW + xq) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
    __syncthreads();
    {
        const int x = tid & (kTW - 1), y = (tid >> 6) * SR;   // 64 columns x 4 strips of 8 rows
        float col[SR + 2 * R];
#pragma unroll
        for (int m = 0; m < SR + 2 * R; m++) col[m] = rowp[(y + m) * kTW + x];
        const int gx = x0 + x;
#pragma unroll
        for (int o = 0; o < SR; o++) {
            const int gy = y0 + y + o;
            float d = col[o + R] * k[R];
#pragma unroll
            for (int m = 1; m <= R; m++) d = fmaf(col[o + R + m] + col[o + R - m], k[R + m], d);
            if (gy < p.h && gx < p.w) {
                const size_t off = (size_t)gy * p.w + gx;
                p.dst[off] = d;
                if (p.dog) p.dog[off] = d - in[(y + o + R) * LWP + x + R];
            }
        }
    }
}

// ---- sd_down: resize(src, Size(w / 2, h / 2), INTER_NEAREST) ----
__global__ __launch_bounds__(256) void sd_down(const float* __restrict__ src, int sw, int sh, float* __restrict__ dst,
                                               int W, int H, double ifx, double ify, size_t fstride)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    src += blockIdx.z * fstride;
    dst += blockIdx.z * fstride;
    if (x >= W) return;
    const int sx = min((int)floor(x * ifx), sw - 1), sy = min((int)floor(y * ify), sh - 1);
    dst[(size_t)y * W + x] = src[(size_t)sy * sw + sx];
}

// ---- sd_extrema ----
struct ExtParams {
    const float* pyr;
    PyrInfo P;
    int o;
    size_t fstride;                        // pyramid floats per frame
    int4* cand;                            // {octave | frame << 8, layer, r, c}
    int* ncand;
    int cap;
    int dogless;                           // DoG taken from the Gaussian layers (no DoG planes)
    int xcd;                               // tiles in XCD-contiguous order (xcd_tile)
};

__device__ inline bool ext_test(const float* cur, const float* prv, const float* nxt, size_t o, int w)
{
    const float val = cur[o];
    if (!(fabsf(val) > 1.f)) return false;   // threshold = floor(0.5 * 0.04 / 3 * 255) = 1
    const long off[9] = {-w - 1, -w, -w + 1, -1, 0, 1, w - 1, w, w + 1};
    if (val > 0) {
#pragma unroll
        for (int k = 0; k < 9; k++) {
            if (k != 4 && !(val >= cur[o + off[k]])) return false;
            if (!(val >= nxt[o + off[k]]) || !(val >= prv[o + off[k]])) return false;
        }
        return true;
    }
    if (val < 0) {
#pragma unroll
        for (int k = 0; k < 9; k++) {
            if (k != 4 && !(val <= cur[o + off[k]])) return false;
            if (!(val <= nxt[o + off[k]]) || !(val <= prv[o + off[k]])) return false;
        }
        return true;
    }
    return false;
}

// 64 x 16 interior pixels per workgroup, all three candidate layers: the five
// DoG planes of the tile plus a 1-pixel halo are staged in LDS once
constexpr int kEW = 64, kEH = 16, kESW = kEW + 4, kESH = kEH + 2;   // staged rows: 66 floats + 2 of pad

__global__ __launch_bounds__(256) void sd_extrema(ExtParams p)
{
    __shared__ __attribute__((aligned(16))) float t[kDL][kESH * kESW];
    const Oct& O = p.P.o[p.o];
    int bx, by, fr;
    xcd_tile(p.xcd != 0, bx, by, fr);
    const int x0 = kImgBorder + bx * kEW, y0 = kImgBorder + by * kEH, tid = threadIdx.x;
    const int xe = O.w - kImgBorder, ye = O.h - kImgBorder;     // exclusive interior bounds
    // interior tiles: 16-byte loads (4-byte aligned), 17 per staged row (the
    // last two floats land in the row's pad); edge tiles clamp per pixel
    const bool interior = x0 - 1 + kESW <= O.w && y0 - 1 + kESH <= O.h;
    if (p.dogless) {
        // DoG layer l = Gaussian layer l + 1 - layer l, the subtraction the
        // pyramid would have stored (same operands, same rounding)
        const float* fb = p.pyr + fr * p.fstride;
        if (interior) {
            typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
            constexpr int NL = kESW / 4;
            const size_t o0 = (size_t)(y0 - 1) * O.w + (x0 - 1);
            // both passes' loads first, then the differences; loads and stores
            // unconditional (a past-the-end index redoes the last piece, storing
            // the same values again), so no branch lets the compiler sink the
            // second pass's loads below the first pass's stores
            constexpr int NIT = (kESH * NL + 255) / 256;
            f4u g[NIT][kGL];
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const int i = min(tid + 256 * it, kESH * NL - 1);
                const int ry = i / NL, j = i - ry * NL;
                const size_t off = o0 + (size_t)ry * O.w + 4 * j;
#pragma unroll
                for (int l = 0; l < kGL; l++) g[it][l] = *reinterpret_cast<const f4u*>(fb + O.g[l] + off);
            }
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const int i = min(tid + 256 * it, kESH * NL - 1);
                const int ry = i / NL, j = i - ry * NL;
#pragma unroll
                for (int l = 0; l < kDL; l++) {
                    const f4u d = g[it][l + 1] - g[it][l];
                    *reinterpret_cast<float4*>(&t[l][ry * kESW + 4 * j]) = make_float4(d.x, d.y, d.z, d.w);
                }
            }
        } else {
            for (int i = tid; i < kESH * kESW; i += 256) {
                const int ry = i / kESW, rx = i - ry * kESW;
                const int gy = min(y0 - 1 + ry, O.h - 1), gx = min(x0 - 1 + rx, O.w - 1);
                const size_t off = (size_t)gy * O.w + gx;
                float g[kGL];
#pragma unroll
                for (int l = 0; l < kGL; l++) g[l] = fb[O.g[l] + off];
#pragma unroll
                for (int l = 0; l < kDL; l++) t[l][i] = g[l + 1] - g[l];
            }
        }
    } else if (interior) {
        typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
        constexpr int NL = kESW / 4;
#pragma unroll
        for (int l = 0; l < kDL; l++) {
            const float* plane = p.pyr + fr * p.fstride + O.d[l] + (size_t)(y0 - 1) * O.w + (x0 - 1);
            for (int i = tid; i < kESH * NL; i += 256) {
                const int ry = i / NL, j = i - ry * NL;
                const f4u v = *reinterpret_cast<const f4u*>(plane + (size_t)ry * O.w + 4 * j);
                *reinterpret_cast<float4*>(&t[l][ry * kESW + 4 * j]) = make_float4(v.x, v.y, v.z, v.w);
            }
        }
    } else {
#pragma unroll
        for (int l = 0; l < kDL; l++) {    // uniform plane loop: the plane base stays scalar
            const float* plane = p.pyr + fr * p.fstride + O.d[l];
            for (int i = tid; i < kESH * kESW; i += 256) {
                const int ry = i / kESW, rx = i - ry * kESW;
                const int gy = min(y0 - 1 + ry, O.h - 1), gx = min(x0 - 1 + rx, O.w - 1);
                t[l][i] = plane[(size_t)gy * O.w + gx];
            }
        }
    }
    __syncthreads();
    // Branch-free tests: thread = one column x 4 rows.  For each DoG plane and
    // staged row, the 3-wide max / min (centre included, which cannot change a
    // >= / <= test), then per candidate the 3 x 3 x 3 max / min from those;
    // val >= max26 <=> val >= every neighbour for finite DoG values.
    const int lx = tid & (kEW - 1), g = tid >> 6;         // rows 4g .. 4g + 3 of the tile
    float rmx[kDL][6], rmn[kDL][6], ctr[kLayers][4];
#pragma unroll
    for (int l = 0; l < kDL; l++)
#pragma unroll
        for (int rr = 0; rr < 6; rr++) {
            const float* row = t[l] + (4 * g + rr) * kESW + lx;
            const float a0 = row[0], a1 = row[1], a2 = row[2];
            rmx[l][rr] = fmaxf(fmaxf(a0, a1), a2);
            rmn[l][rr] = fminf(fminf(a0, a1), a2);
            if (l >= 1 && l <= kLayers && rr >= 1 && rr <= 4) ctr[l - 1][rr - 1] = a1;
        }
    unsigned hits = 0;
#pragma unroll
    for (int i = 1; i <= kLayers; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float val = ctr[i - 1][j];
            float M = rmx[i - 1][j], m = rmn[i - 1][j];
#pragma unroll
            for (int l = i - 1; l <= i + 1; l++)
#pragma unroll
                for (int rr = j; rr < j + 3; rr++) { M = fmaxf(M, rmx[l][rr]); m = fminf(m, rmn[l][rr]); }
            const bool in = y0 + 4 * g + j < ye && x0 + lx < xe;
            const bool ext = fabsf(val) > 1.f && ((val > 0 && val >= M) || (val < 0 && val <= m));
            if (in && ext) hits |= 1u << ((i - 1) * 4 + j);
        }
    __shared__ int wsum[4], gbase;
    const int lane = tid & 63, wv = tid >> 6, cnt = __popc(hits);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        gbase = tot ? atomicAdd(p.ncand, tot) : 0;
    }
    __syncthreads();
    int idx = gbase + incl - cnt;
    for (int w = 0; w < wv; w++) idx += wsum[w];
    while (hits) {
        const int bit = __ffs(hits) - 1;
        hits &= hits - 1;
        const int layer = 1 + (bit >> 2), j = bit & 3;
        if (idx < p.cap) p.cand[idx] = make_int4(p.o | (fr << 8), layer, y0 + 4 * g + j, x0 + lx);
        idx++;
    }
}

// ---- sd_refine ----
struct RefineParams {
    const float* pyr;
    PyrInfo P;
    size_t fstride;                        // pyramid floats per frame
    const int4* cand;
    const int* ncand;
    int cap;
    slam_keypoint* kps;                    // doubled-image units, octave = pyramid octave index; frame f's at f * kcap
    int* nkps;                             // per frame
    int kcap;                              // per frame
    int dbg;                               // probes (SLAMHIP_SD_REFINE_DBG, -DSLAMHIP_DIAG builds): 1 no bin sums, 2 no sample evaluation, 4 no refinement
    float exptab[64];
};

// Matx_DetOp<float, 3> + Matx_FastSolveOp<float, 3, 1> (Cramer's rule)
__device__ inline void solve33(const float* a, const float* b, float* x)
{
#define A(i, j) a[(i) * 3 + (j)]
    float d = A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) - A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
              A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1));
    if (d == 0) { x[0] = x[1] = x[2] = 0.f; return; }
    d = cr_divf(1.f, d);
    x[0] = d * (b[0] * (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) - A(0, 1) * (b[1] * A(2, 2) - A(1, 2) * b[2]) +
                A(0, 2) * (b[1] * A(2, 1) - A(1, 1) * b[2]));
    x[1] = d * (A(0, 0) * (b[1] * A(2, 2) - A(1, 2) * b[2]) - b[0] * (A(1, 0) * A(2, 2) - A(1, 2) * A(2, 0)) +
                A(0, 2) * (A(1, 0) * b[2] - b[1] * A(2, 0)));
    x[2] = d * (A(0, 0) * (A(1, 1) * b[2] - b[1] * A(2, 1)) - A(0, 1) * (A(1, 0) * b[2] - b[1] * A(2, 0)) +
                b[0] * (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)));
#undef A
}

// adjustLocalExtrema (oracle/siftdet.c adjust_extremum)
// DoG layer l at (R, C): the stored plane, or (DOGLESS) Gaussian layer l + 1
// minus layer l, the same subtraction the plane would have held
template <bool DOGLESS>
struct DogAt {
    const float* pyr;
    const Oct& O;
    __device__ float operator()(int l, int R, int C) const { return pyr[O.d[l] + (size_t)R * O.w + C]; }
};
template <>
struct DogAt<true> {
    const float* pyr;
    const Oct& O;
    __device__ float operator()(int l, int R, int C) const
    {
        const size_t off = (size_t)R * O.w + C;
        return pyr[O.g[l + 1] + off] - pyr[O.g[l] + off];
    }
};

template <bool DOGLESS>
__device__ bool adjust_extremum(const float* pyr, const Oct& O, int o, int& layer, int& r, int& c, slam_keypoint& kp)
{
    const DogAt<DOGLESS> D{pyr, O};
    const float img_scale = cr_divf(1.f, 255.f), deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale,
                cross_deriv_scale = img_scale * 0.25f;
    const int w = O.w, h = O.h;
    float xi = 0, xr = 0, xc = 0, contr;
    int i = 0;
#define IM(R, C) D(layer, R, C)
#define PV(R, C) D(layer - 1, R, C)
#define NX(R, C) D(layer + 1, R, C)
    for (; i < 5; i++) {
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
            return false;
        c += __float2int_rn(xc);
        r += __float2int_rn(xr);
        layer += __float2int_rn(xi);
        if (layer < 1 || layer > kLayers || c < kImgBorder || c >= w - kImgBorder || r < kImgBorder ||
            r >= h - kImgBorder)
            return false;
    }
    if (i >= 5) return false;
    {
        float dD[3] = {(IM(r, c + 1) - IM(r, c - 1)) * deriv_scale, (IM(r + 1, c) - IM(r - 1, c)) * deriv_scale,
                       (NX(r, c) - PV(r, c)) * deriv_scale};
        float t = 0;
        t += dD[0] * xc;
        t += dD[1] * xr;
        t += dD[2] * xi;
        contr = IM(r, c) * img_scale + t * 0.5f;
        if (fabsf(contr) * kLayers < 0.04f) return false;
        float v2 = IM(r, c) * 2.f;
        float dxx = (IM(r, c + 1) + IM(r, c - 1) - v2) * second_deriv_scale;
        float dyy = (IM(r + 1, c) + IM(r - 1, c) - v2) * second_deriv_scale;
        float dxy = (IM(r + 1, c + 1) - IM(r + 1, c - 1) - IM(r - 1, c + 1) + IM(r - 1, c - 1)) * cross_deriv_scale;
        float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * 10.f >= 11.f * 11.f * det) return false;
    }
#undef IM
#undef PV
#undef NX
    kp.x = ((float)c + xc) * (float)(1 << o);
    kp.y = ((float)r + xr) * (float)(1 << o);
    kp.octave = o + (layer << 8) + (__double2int_rn(((double)xi + 0.5) * 255) << 16);
    kp.size = kSigma * (float)exp2((double)cr_divf((float)layer + xi, (float)kLayers)) * (float)(1 << o) * 2;
    kp.response = fabsf(contr);
    kp.angle = -1.f;
    kp.class_id = -1;
    return true;
}

#ifndef SD_REFINE_U
#define SD_REFINE_U 4
#endif
template <bool DOGLESS>
__global__ __launch_bounds__(64) void sd_refine(RefineParams p)
{
    // exp32f's table in LDS: lane-divergent reads of the kernel argument
    // itself go to the kernarg segment
    __shared__ float s_exptab[64];
    s_exptab[threadIdx.x] = p.exptab[threadIdx.x];
    __shared__ __attribute__((aligned(16))) float sval[kOriMaxS + 3];
    __shared__ __attribute__((aligned(16))) unsigned char sbin[kOriMaxS + 3];
    __shared__ float th[kOriBins + 4];
    __shared__ int sh_i[4];
    __shared__ slam_keypoint sh_kp;
    const int lane = threadIdx.x;
    int n = *p.ncand;
    if (n > p.cap) n = p.cap;
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        const int4 cd = p.cand[q];
        const int o = cd.x & 255, fr = cd.x >> 8;
        const Oct& O = p.P.o[o];
        const float* pyr = p.pyr + fr * p.fstride;
        if (lane == 0) {
            int layer = cd.y, r = cd.z, c = cd.w;
            slam_keypoint kp;
            bool ok;
            if (p.dbg & 4) {
                ok = true;
                kp.x = (float)c * (float)(1 << o); kp.y = (float)r * (float)(1 << o);
                kp.octave = o + (layer << 8); kp.size = 2.f * kSigma * 1.6f * (float)(1 << o);
                kp.response = 1.f; kp.angle = -1.f;
            } else {
                ok = adjust_extremum<DOGLESS>(pyr, O, o, layer, r, c, kp);
            }
            kp.class_id = fr;              // the frame, until the host's per-frame filter (then -1)
            sh_i[0] = ok;
            sh_i[1] = layer;
            sh_i[2] = r;
            sh_i[3] = c;
            sh_kp = kp;
        }
        __syncthreads();
        const bool ok = sh_i[0];
        const int layer = sh_i[1], py = sh_i[2], px = sh_i[3];
        const slam_keypoint kp = sh_kp;
        __syncthreads();
        if (!ok) continue;
        // calcOrientationHist on gauss[o][layer]
        const float scl_octv = kp.size * 0.5f / (float)(1 << o);
        const int radius = __float2int_rn(4.5f * scl_octv);
        const float sigma = 1.5f * scl_octv;
        const float expf_scale = cr_divf(-1.f, 2.f * sigma * sigma);
        const float* img = pyr + O.g[layer];
        const int ylo = max(py - radius, 1), yhi = min(py + radius, O.h - 2);
        const int xlo = max(px - radius, 1), xhi = min(px + radius, O.w - 2);
        const int ncol = xhi - xlo + 1, nrow = yhi - ylo + 1;
        const int ns = (ncol > 0 && nrow > 0) ? ncol * nrow : 0;
        if (radius > kOriMaxR) continue;   // unreachable for nOctaveLayers = 3 (see kOriMaxR)
        // kRU samples per lane per pass, all their loads issued before any is
        // used (a load / use loop waits one memory latency per 64 samples); a
        // past-the-end sample reloads the last one and is not stored
        constexpr int kRU = SD_REFINE_U;
        for (int s0 = 0; s0 < ns; s0 += 64 * kRU) {
            float gx0[kRU], gx1[kRU], gy0[kRU], gy1[kRU];
            int si[kRU], sj[kRU];
#pragma unroll
            for (int u = 0; u < kRU; u++) {
                const int s = min(s0 + lane + 64 * u, ns - 1);
                const int yy = s / ncol, y = ylo + yy, x = xlo + (s - yy * ncol);
                si[u] = y - py;
                sj[u] = x - px;
                const float* row = img + (size_t)y * O.w + x;
                gx1[u] = row[1];
                gx0[u] = row[-1];
                gy0[u] = row[-(ptrdiff_t)O.w];
                gy1[u] = row[O.w];
            }
#pragma unroll
            for (int u = 0; u < kRU; u++) {
                const int s = s0 + lane + 64 * u;
                if (s >= ns) break;
                if (p.dbg & 2) { sval[s] = 1.f; sbin[s] = (unsigned char)(s % kOriBins); continue; }
                const int i = si[u], j = sj[u];
                const float dx = gx1[u] - gx0[u];
                const float dy = gy0[u] - gy1[u];
                const float W = exp32f((float)(i * i + j * j) * expf_scale, s_exptab);
                const float ori = fast_atan2_deg(dy, dx);
                const float mag = cr_sqrtf(fmaf(dx, dx, dy * dy));
                int bin = __float2int_rn((kOriBins / 360.f) * ori);
                if (bin >= kOriBins) bin -= kOriBins;
                if (bin < 0) bin += kOriBins;
                sval[s] = W * mag;
                sbin[s] = (unsigned char)bin;
            }
        }
        for (int s = ns + lane; s < ((ns + 3) & ~3); s += 64) sbin[s] = 0xff;   // pad to a multiple of 4
        __syncthreads();
        if (lane < kOriBins && (p.dbg & 1)) {
            th[lane + 2] = sval[lane];
        } else if (lane < kOriBins) {
            // bin `lane`'s samples in sample order: 4 (bin, value) pairs per LDS access
            float acc = 0.f;
            const uint32_t* b4 = reinterpret_cast<const uint32_t*>(sbin);
            const float4* v4 = reinterpret_cast<const float4*>(sval);
            for (int s = 0; s < (ns + 3) >> 2; s++) {
                const uint32_t b = b4[s];
                const float4 v = v4[s];
                if ((b & 0xff) == (uint32_t)lane) acc += v.x;
                if (((b >> 8) & 0xff) == (uint32_t)lane) acc += v.y;
                if (((b >> 16) & 0xff) == (uint32_t)lane) acc += v.z;
                if ((b >> 24) == (uint32_t)lane) acc += v.w;
            }
            th[lane + 2] = acc;
        }
        __syncthreads();
        if (lane == 0) {
            float* t = th + 2;
            t[-1] = t[kOriBins - 1];
            t[-2] = t[kOriBins - 2];
            t[kOriBins] = t[0];
            t[kOriBins + 1] = t[1];
            float hist[kOriBins], maxval = 0.f;
            for (int i = 0; i < kOriBins; i++) {
                hist[i] = fmaf(t[i - 2] + t[i + 2], 1.f / 16.f, fmaf(t[i - 1] + t[i + 1], 4.f / 16.f, t[i] * (6.f / 16.f)));
                maxval = i == 0 ? hist[0] : fmaxf(maxval, hist[i]);
            }
            const float mag_thr = maxval * 0.8f;
            for (int j = 0; j < kOriBins; j++) {
                const int l = j > 0 ? j - 1 : kOriBins - 1, r2 = j < kOriBins - 1 ? j + 1 : 0;
                if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                    float bin = (float)j + cr_divf(0.5f * (hist[l] - hist[r2]), hist[l] - 2 * hist[j] + hist[r2]);
                    bin = bin < 0 ? kOriBins + bin : bin >= kOriBins ? bin - kOriBins : bin;
                    float angle = 360.f - (360.f / kOriBins) * bin;
                    if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
                    const int k = atomicAdd(p.nkps + fr, 1);
                    if (k < p.kcap) {
                        slam_keypoint e = kp;
                        e.angle = angle;
                        p.kps[(size_t)fr * p.kcap + k] = e;
                    }
                }
            }
        }
        __syncthreads();
    }
}

// ---- sd_kp_compact: the frames' keypoint regions -> one frame-major list ----
// block (x, f) copies frame f's first n[f] keypoints (n[f] <= cap checked by
// the host before it reads them) to dst + (n[0] + ... + n[f - 1])
__global__ __launch_bounds__(256) void sd_kp_compact(const slam_keypoint* __restrict__ src, const int* __restrict__ n,
                                                     int cap, slam_keypoint* __restrict__ dst)
{
    const int f = blockIdx.y;
    int base = 0;
    for (int i = 0; i < f; i++) base += min(n[i], cap);
    const int cnt = min(n[f], cap);
    const uint4* s4 = reinterpret_cast<const uint4*>(src + (size_t)f * cap);
    uint4* d4 = reinterpret_cast<uint4*>(dst + base);
    static_assert(sizeof(slam_keypoint) == 28, "7 dwords per keypoint");
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(s4);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(d4);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < cnt * 7; i += gridDim.x * 256) d1[i] = s1[i];
}

// ---- sd_desc: calcSIFTDescriptor on the keypoint's own octave / layer image ----
struct DescParams {
    const float* pyr;
    PyrInfo P;
    size_t fstride;                        // pyramid floats per frame
    const int* kp_frame;                   // nullable: every keypoint in frame 0
    const slam_keypoint* kps;              // final (input-image) units
    const float* cs;                       // host cosf / sinf of the descriptor angle
    int n;
    float* desc;
    int dbg;                               // probes (SLAMHIP_SD_DBG): 1 no walk, 2 no eval (timing only), 4 no size order
    int xcd;                               // sd_desc_staged: blocks in XCD-contiguous order
    float exptab[64];
    const int* fbase;                      // nullable: keypoint g's output row g + fbase[frame] (else g)
    slam_keypoint* kout;                   // nullable: the keypoint copied to its output row too
};

// Gather form: 16 lanes per keypoint, lane q owns inner cell (q >> 2, q & 3) of
// the 4 x 4 grid and its 10 orientation slots (8 + the 2 that fold back), held
// in registers.  The cell receives the trilinear share of every sample whose
// (rbin, cbin) lies in [ci - 1, ci + 1) x [cj - 1, cj + 1); the lane walks the
// pixel bounding box of that rotated square (clipped to the window) in raster
// order -- a subsequence of calcSIFTDescriptor's sample order -- and applies the
// same per-sample arithmetic, so each slot is the oracle's sequential sum and
// the descriptor is bit-identical (no atomics).  Detected keypoints have
// ori = 360 - angle in (0, 360), so o0 is always in 0..7 (the 361-degree slot
// quirk of FAST keypoints cannot occur here).  4 keypoints per wavefront.
// The lane's 10 orientation slots live in LDS, slot-major (slot * 256 + lane:
// bank = lane, conflict-free whatever the data-dependent slot): a sample costs
// two read-add-writes at o0 and o0 + 1, in the lane's raster order, instead of
// 10 predicated adds per slot update in registers (the adds and their order
// per slot are the same, so the values are bit-identical).
__global__ __launch_bounds__(256) void sd_desc(DescParams p)
{
    __shared__ float raw_s[16][128];
    __shared__ float s_slot[10][256];
    __shared__ float s_exptab[64];
    const int tid = threadIdx.x, grp = tid >> 4, q = tid & 15, ci = q >> 2, cj = q & 3;
    float* raw = raw_s[grp];
    if (tid < 64) s_exptab[tid] = p.exptab[tid];
    // an LDS-typed pointer: a volatile generic pointer keeps flat accesses
    // (the address space is not inferred through volatile), each a full
    // vmcnt round trip -- 3x slower descriptors
    auto hs = (__attribute__((address_space(3))) volatile float*)(&s_slot[0][tid]);
    __syncthreads();
    for (int g0 = blockIdx.x * 16; g0 < p.n; g0 += gridDim.x * 16) {
        const int g = g0 + grp;
        const bool live = g < p.n;
        float h[10];
#pragma unroll
        for (int k = 0; k < 10; k++) hs[k * 256] = 0.f;
        size_t drow = (size_t)g;                 // the output row
        if (live) {
            const slam_keypoint kp = p.kps[g];
            if (p.fbase) drow = (size_t)(g + p.fbase[p.kp_frame ? p.kp_frame[g] : 0]);
            if (p.kout && q == 0) p.kout[drow] = kp;
            int oct = kp.octave & 255;
            const int layer = (kp.octave >> 8) & 255;
            oct = oct < 128 ? oct : (-128 | oct);
            const float scale = oct >= 0 ? 1.f / (float)(1 << oct) : (float)(1 << -oct);
            const Oct& O = p.P.o[oct + 1];
            const float* img = p.pyr + (p.kp_frame ? p.kp_frame[g] : 0) * p.fstride + O.g[layer];
            const float ptfx = kp.x * scale, ptfy = kp.y * scale, size = kp.size * scale;
            float angle = 360.f - kp.angle;
            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            const float ori = angle, scl = size * 0.5f;
            const int ptx = __float2int_rn(ptfx), pty = __float2int_rn(ptfy);
            const float bins_per_rad = 8 / 360.f, exp_scale = -1.f / (4 * 4 * 0.5f);
            const float hist_width = 3.f * scl;
            int radius = __float2int_rn(hist_width * 1.4142135623730951f * 5.f * 0.5f);
            const int diag = (int)sqrt((double)O.w * O.w + (double)O.h * O.h);
            radius = min(radius, diag);
            const float cos0 = p.cs[2 * g], sin0 = p.cs[2 * g + 1];
            const float cos_t = cr_divf(cos0, hist_width), sin_t = cr_divf(sin0, hist_width);
            // pixel bounding box of c_rot in [cj - 2.5, cj - 0.5), r_rot in [ci - 2.5, ci - 0.5)
            // (inverse rotation of the 4 corners, widened by 1 px, clipped to the window)
            float ilo = 1e30f, ihi = -1e30f, jlo = 1e30f, jhi = -1e30f;
#pragma unroll
            for (int cr = 0; cr < 4; cr++) {
                const float cc = (float)cj - 2.5f + 2.f * (float)(cr & 1), rr = (float)ci - 2.5f + 2.f * (float)(cr >> 1);
                const float jj = hist_width * (cc * cos0 + rr * sin0), ii = hist_width * (rr * cos0 - cc * sin0);
                ilo = fminf(ilo, ii); ihi = fmaxf(ihi, ii); jlo = fminf(jlo, jj); jhi = fmaxf(jhi, jj);
            }
            const int i0 = max(-radius, (int)floorf(ilo) - 1), i1 = min(radius, (int)ceilf(ihi) + 1);
            const int j0 = max(-radius, (int)floorf(jlo) - 1), j1 = min(radius, (int)ceilf(jhi) + 1);
            for (int i = i0; i <= i1; i++) {
                const int r = pty + i;
                if (r <= 0 || r >= O.h - 1) continue;
                // this row's part of the cell's rotated square: the j where
                // c_rot = j cos_t - i sin_t and r_rot = j sin_t + i cos_t lie in
                // [c - 2.5, c - 0.5), widened by a pixel each side (the exact test
                // below stays); the lane walks it in raster order as before
                int ja = j0, jb = j1;
                {
                    float lo = -1e30f, hi = 1e30f;
                    auto clip = [&](float a, float b, float l, float h) {
                        if (a > 0.f) { lo = fmaxf(lo, (l - b) / a); hi = fminf(hi, (h - b) / a); }
                        else if (a < 0.f) { lo = fmaxf(lo, (h - b) / a); hi = fminf(hi, (l - b) / a); }
                        else if (!(b >= l && b < h)) { lo = 1e30f; hi = -1e30f; }
                    };
                    clip(cos_t, -(float)i * sin_t, (float)cj - 2.5f, (float)cj - 0.5f);
                    clip(sin_t, (float)i * cos_t, (float)ci - 2.5f, (float)ci - 0.5f);
                    if (lo > hi) continue;
                    ja = max(ja, (int)fmaxf(floorf(lo) - 1.f, -1e9f));
                    jb = min(jb, (int)fminf(ceilf(hi) + 1.f, 1e9f));
                }
                for (int j = ja; j <= jb; j++) {
                    const int c = ptx + j;
                    const float c_rot = (float)j * cos_t - (float)i * sin_t;
                    const float r_rot = (float)j * sin_t + (float)i * cos_t;
                    float rbin = r_rot + 2.f - 0.5f, cbin = c_rot + 2.f - 0.5f;
                    if (!(rbin > -1.f && rbin < 4.f && cbin > -1.f && cbin < 4.f && c > 0 && c < O.w - 1)) continue;
                    const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                    const int dr = ci - r0, dc = cj - c0;          // 0: first corner, 1: second
                    if ((unsigned)dr > 1u || (unsigned)dc > 1u) continue;
                    const float dx = img[(size_t)r * O.w + c + 1] - img[(size_t)r * O.w + c - 1];
                    const float dy = img[(size_t)(r - 1) * O.w + c] - img[(size_t)(r + 1) * O.w + c];
                    const float wexp = exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, s_exptab);
                    const float ori_k = fast_atan2_deg(dy, dx);
                    const float mag_k = cr_sqrtf(fmaf(dx, dx, dy * dy));
                    float obin = (ori_k - ori) * bins_per_rad;
                    const float mag = mag_k * wexp;
                    int o0 = (int)floorf(obin);
                    rbin -= (float)r0;
                    cbin -= (float)c0;
                    obin -= (float)o0;
                    if (o0 < 0) o0 += 8;
                    if (o0 >= 8) o0 -= 8;
                    const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
                    const float vr = dr == 0 ? v_r0 : v_r1;           // this cell's row share
                    const float v_rc1 = vr * cbin, v_rc0 = vr - v_rc1;
                    const float vc = dc == 0 ? v_rc0 : v_rc1;
                    const float v_o1 = vc * obin, v_o0 = vc - v_o1;
                    hs[o0 * 256] = __fadd_rn(hs[o0 * 256], v_o0);
                    hs[(o0 + 1) * 256] = __fadd_rn(hs[(o0 + 1) * 256], v_o1);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 10; k++) h[k] = hs[k * 256];
        // circular fold, then the reference's norm / clamp / renorm / saturate.
        // Every barrier below is reached by all 256 threads (dead groups compute on zeros).
        h[0] += h[8];
        h[1] += h[9];
#pragma unroll
        for (int o = 0; o < 8; o++) raw[q * 8 + o] = h[o];
        __syncthreads();
        // first norm: 8 fma chains over k = l + 8 m (lanes q < 8 of the group), v_reduce_sum order
        float part = 0.f;
        if (q < 8)
            for (int m = 0; m < 16; m++) { const float t = raw[q + 8 * m]; part = fmaf(t, t, part); }
        float l[8];
#pragma unroll
        for (int t = 0; t < 8; t++) l[t] = __shfl(part, (tid & 48) + t, 64);
        const float nrm2 = ((l[0] + l[4]) + (l[1] + l[5])) + ((l[2] + l[6]) + (l[3] + l[7]));
        const float thr = cr_sqrtf(nrm2) * 0.2f;
        float v[8];
#pragma unroll
        for (int o = 0; o < 8; o++) v[o] = fminf(raw[q * 8 + o], thr);
        __syncthreads();
#pragma unroll
        for (int o = 0; o < 8; o++) raw[q * 8 + o] = v[o];
        __syncthreads();
        // second norm: sequential over k = 0..127
        float n2 = 0.f;
        for (int k = 0; k < 128; k++) { const float t = raw[k]; n2 += t * t; }
        const float sq = cr_sqrtf(n2);
        const float sc = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        if (live) {
#pragma unroll
            for (int o = 0; o < 8; o++)
                p.desc[drow * 128 + q * 8 + o] = fminf(fmaxf(rintf(v[o] * sc), 0.f), 255.f);
        }
        __syncthreads();
    }
}

// Staged form of sd_desc (the default): the same cell walks and slot
// read-add-writes, but a sample's {mag * wexp, fastAtan2} -- the four pyramid
// gathers, the square root, the arctangent and the exp -- is evaluated once per
// keypoint instead of once per cell that claims it (each sample lands in up to
// 4 cells and the cells' pixel walks overlap further).  The window is staged
// kStrip rows at a time into the keypoint's LDS strip by the keypoint's lanes
// (row clip to the union of the cells' rotated squares, the exact per-sample
// test), then the lanes walk that strip; strips go in ascending row order, so
// each slot still receives its samples in calcSIFTDescriptor's order and the
// descriptor is bit-identical.  kCpl cells per lane (16 / kCpl lanes per
// keypoint): a cell spans ~2/5 of the window's rows, so with one cell per lane
// most lanes idle in any strip; lane q of 8 takes cells q and q + 8 (rows
// ci and ci + 2 of its column), whose row spans abut.  A keypoint's lanes are
// within one wave, so a strip needs only a wave barrier.  A window wider than
// kSdW (impossible for detected keypoints: radius <= 38 at nOctaveLayers 3) is
// evaluated directly, as in sd_desc.
constexpr int kSdW = 78;   // 2 * 38 + 1 rounded up; 4 blocks per CU at kCpl 2
#ifndef SD_STAGE_U
#define SD_STAGE_U 2
#endif
constexpr int kSdU = SD_STAGE_U;   // staged positions per lane per gather pass

__device__ __forceinline__ void sd_wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

template <int kStrip, int kCpl>
__global__ __launch_bounds__(256) void sd_desc_staged(DescParams p)
{
    constexpr int L = 16 / kCpl, G = 256 / L;   // lanes per keypoint, keypoints per block
    // a staged sample: {mag * wexp, rbin, cbin, obin fractions} and {r0 + 1, c0 + 1, o0}
    // packed (r0 + 1 = 15: not a sample of any cell)
    __shared__ float4 s_rec[G][kStrip][kSdW];
    __shared__ int s_pk[G][kStrip][kSdW];
    __shared__ float s_slot[10 * kCpl][256];
    __shared__ float s_exptab[64];
    const int tid = threadIdx.x, grp = tid / L, q = tid % L;
    // the keypoint's 128 raw bins reuse its strip (own wave; after the walk)
    float* raw = reinterpret_cast<float*>(&s_rec[grp][0][0]);
    static_assert(sizeof(s_rec[0]) >= 128 * sizeof(float), "raw bins alias the strip");
    if (tid < 64) s_exptab[tid] = p.exptab[tid];
    auto hs = (__attribute__((address_space(3))) volatile float*)(&s_slot[0][tid]);
    __syncthreads();
    __shared__ float s_key[G];
    __shared__ int s_perm[G];
    // p.xcd: the blocks' keypoint ranges in XCD-contiguous order (XCD k takes
    // the k-th eighth of the list: its frames' pyramid stays in its own L2)
    int bxl = blockIdx.x;
    if (p.xcd) {
        const unsigned per = gridDim.x >> 3, lin = blockIdx.x;
        if (lin < (per << 3)) bxl = (int)((lin & 7) * per + (lin >> 3));
    }
    for (int g0 = bxl * G; g0 < p.n; g0 += gridDim.x * G) {
        // the block's keypoints dealt to its groups by window size, so a wave's
        // keypoints have similar row counts and row widths (its loops run to the
        // largest); the block keeps the same keypoints, so the gathers keep
        // their locality (a launch-wide size order lost it: r5_det_sort.txt)
        if (tid < G) {
            float key = -1.f;
            if (g0 + tid < p.n && !(p.dbg & 4)) {
                const slam_keypoint kq = p.kps[g0 + tid];
                int oct = kq.octave & 255;
                oct = oct < 128 ? oct : (-128 | oct);
                key = kq.size * (oct >= 0 ? 1.f / (float)(1 << oct) : (float)(1 << -oct));
            }
            s_key[tid] = key;
        }
        __syncthreads();
        if (tid < G) {
            const float kt = s_key[tid];
            int rank = 0;
            for (int m = 0; m < G; m++) {
                const float km = s_key[m];
                rank += (km < kt) || (km == kt && m < tid);
            }
            s_perm[rank] = tid;
        }
        __syncthreads();
        const int g = g0 + s_perm[grp];
        const bool live = g < p.n;
#pragma unroll
        for (int k = 0; k < 10 * kCpl; k++) hs[k * 256] = 0.f;
        // per-keypoint constants (identical in the keypoint's lanes)
        const float* img = nullptr;
        int ow = 0, oh = 0, ptx = 0, pty = 0, radius = 0;
        float ori = 0.f, cos_t = 0.f, sin_t = 0.f;
        int i0[kCpl], i1[kCpl], j0[kCpl], j1[kCpl];
        int ui0 = 0, nrows = 0;
        bool fits = true;
        const float bins_per_rad = 8 / 360.f, exp_scale = -1.f / (4 * 4 * 0.5f);
        int ua = INT_MAX, ub = INT_MIN;
#pragma unroll
        for (int cc = 0; cc < kCpl; cc++) { i0[cc] = 1; i1[cc] = 0; j0[cc] = 1; j1[cc] = 0; }
        size_t drow = (size_t)g;                 // the output row
        if (live) {
            const slam_keypoint kp = p.kps[g];
            if (p.fbase) drow = (size_t)(g + p.fbase[p.kp_frame ? p.kp_frame[g] : 0]);
            if (p.kout && q == 0) p.kout[drow] = kp;
            int oct = kp.octave & 255;
            const int layer = (kp.octave >> 8) & 255;
            oct = oct < 128 ? oct : (-128 | oct);
            const float scale = oct >= 0 ? 1.f / (float)(1 << oct) : (float)(1 << -oct);
            const Oct& O = p.P.o[oct + 1];
            ow = O.w; oh = O.h;
            img = p.pyr + (p.kp_frame ? p.kp_frame[g] : 0) * p.fstride + O.g[layer];
            const float ptfx = kp.x * scale, ptfy = kp.y * scale, size = kp.size * scale;
            float angle = 360.f - kp.angle;
            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            ori = angle;
            const float scl = size * 0.5f;
            ptx = __float2int_rn(ptfx); pty = __float2int_rn(ptfy);
            const float hist_width = 3.f * scl;
            radius = __float2int_rn(hist_width * 1.4142135623730951f * 5.f * 0.5f);
            const int diag = (int)sqrt((double)O.w * O.w + (double)O.h * O.h);
            radius = min(radius, diag);
            fits = 2 * radius + 1 <= kSdW;
            const float cos0 = p.cs[2 * g], sin0 = p.cs[2 * g + 1];
            cos_t = cr_divf(cos0, hist_width); sin_t = cr_divf(sin0, hist_width);
#pragma unroll
            for (int cc = 0; cc < kCpl; cc++) {
                const int cell = q + cc * L, ci = cell >> 2, cj = cell & 3;
                // pixel bounding box of c_rot in [cj - 2.5, cj - 0.5), r_rot in [ci - 2.5, ci - 0.5)
                float ilo = 1e30f, ihi = -1e30f, jlo = 1e30f, jhi = -1e30f;
#pragma unroll
                for (int cr = 0; cr < 4; cr++) {
                    const float c2 = (float)cj - 2.5f + 2.f * (float)(cr & 1), r2 = (float)ci - 2.5f + 2.f * (float)(cr >> 1);
                    const float jj = hist_width * (c2 * cos0 + r2 * sin0), ii = hist_width * (r2 * cos0 - c2 * sin0);
                    ilo = fminf(ilo, ii); ihi = fmaxf(ihi, ii); jlo = fminf(jlo, jj); jhi = fmaxf(jhi, jj);
                }
                i0[cc] = max(-radius, (int)floorf(ilo) - 1); i1[cc] = min(radius, (int)ceilf(ihi) + 1);
                j0[cc] = max(-radius, (int)floorf(jlo) - 1); j1[cc] = min(radius, (int)ceilf(jhi) + 1);
                ua = min(ua, i0[cc]); ub = max(ub, i1[cc]);
            }
        }
        // the rows any cell of the keypoint walks, and the wave's strip count
#pragma unroll
        for (int m = 1; m < L; m <<= 1) {
            ua = min(ua, __shfl_xor(ua, m, 64));
            ub = max(ub, __shfl_xor(ub, m, 64));
        }
        if (live && ub >= ua) { ui0 = ua; nrows = ub - ua + 1; }
        int nst = (nrows + kStrip - 1) / kStrip;
#pragma unroll
        for (int m = L; m < 64; m <<= 1) nst = max(nst, __shfl_xor(nst, m, 64));
        auto rowclip = [&](int i, float cl, float ch, float rl, float rh, int& ja, int& jb) -> bool {
            float lo = -1e30f, hi = 1e30f;
            auto clip = [&](float a, float b, float l, float h) {
                if (a > 0.f) { lo = fmaxf(lo, (l - b) / a); hi = fminf(hi, (h - b) / a); }
                else if (a < 0.f) { lo = fmaxf(lo, (h - b) / a); hi = fminf(hi, (l - b) / a); }
                else if (!(b >= l && b < h)) { lo = 1e30f; hi = -1e30f; }
            };
            clip(cos_t, -(float)i * sin_t, cl, ch);
            clip(sin_t, (float)i * cos_t, rl, rh);
            if (lo > hi) return false;
            ja = max(ja, (int)fmaxf(floorf(lo) - 1.f, -1e9f));
            jb = min(jb, (int)fminf(ceilf(hi) + 1.f, 1e9f));
            return true;
        };
        // the sample's weighted magnitude and angle, in calcSIFTDescriptor's arithmetic
        auto eval = [&](int r, int c, float c_rot, float r_rot) -> float2 {
            const float dx = img[(size_t)r * ow + c + 1] - img[(size_t)r * ow + c - 1];
            const float dy = img[(size_t)(r - 1) * ow + c] - img[(size_t)(r + 1) * ow + c];
            const float wexp = exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, s_exptab);
            const float ori_k = fast_atan2_deg(dy, dx);
            const float mag_k = cr_sqrtf(fmaf(dx, dx, dy * dy));
            return make_float2(mag_k * wexp, ori_k);
        };
        // the same from the sample's two differences (staged gathers)
        auto eval_g = [&](float dx, float dy, float c_rot, float r_rot) -> float2 {
            const float wexp = exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, s_exptab);
            const float ori_k = fast_atan2_deg(dy, dx);
            const float mag_k = cr_sqrtf(fmaf(dx, dx, dy * dy));
            return make_float2(mag_k * wexp, ori_k);
        };
        for (int t = 0; t < nst; t++) {
            // stage: the strip's rows of the keypoint's window, lanes strided over j;
            // every position of the row's union range is written (a sample, or the
            // no-cell mark), and the cells' walks stay inside that range
            int jaU[kStrip], jbU[kStrip];
#pragma unroll
            for (int rr = 0; rr < kStrip; rr++) {
                const int i = ui0 + t * kStrip + rr, r = pty + i;
                jaU[rr] = 1; jbU[rr] = 0;
                if (!fits || i >= ui0 + nrows || r <= 0 || r >= oh - 1) continue;
                int ja = -radius, jb = radius;
                if (!rowclip(i, -2.5f, 2.5f, -2.5f, 2.5f, ja, jb)) continue;
                jaU[rr] = ja; jbU[rr] = jb;
                // kSdU positions per lane per pass, their four gathers all issued
                // before any is used (a gather / use loop waits one memory latency
                // per position); clamped positions load in-bounds pixels that are
                // not used
                for (int jq = ja + q; jq <= jb; jq += L * kSdU) {
                    float gv[kSdU][4];
#pragma unroll
                    for (int u = 0; u < kSdU; u++) {
                        const int cq = min(max(ptx + min(jq + L * u, jb), 1), ow - 2);
                        const float* px = img + (size_t)r * ow + cq;
                        gv[u][0] = px[1];
                        gv[u][1] = px[-1];
                        gv[u][2] = px[-(ptrdiff_t)ow];
                        gv[u][3] = px[ow];
                    }
#pragma unroll
                    for (int u = 0; u < kSdU; u++) {
                    const int j = jq + L * u;
                    if (j > jb) break;
                    const int c = ptx + j;
                    const float c_rot = (float)j * cos_t - (float)i * sin_t;
                    const float r_rot = (float)j * sin_t + (float)i * cos_t;
                    float rbin = r_rot + 2.f - 0.5f, cbin = c_rot + 2.f - 0.5f;
                    int pk = 0xff;
                    float4 rec = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (rbin > -1.f && rbin < 4.f && cbin > -1.f && cbin < 4.f && c > 0 && c < ow - 1) {
                        const float2 v = (p.dbg & 2) ? make_float2(c_rot, r_rot)
                                                     : eval_g(gv[u][0] - gv[u][1], gv[u][2] - gv[u][3], c_rot, r_rot);
                        // calcSIFTDescriptor's bin split, per sample (the cell only picks its share)
                        float obin = (v.y - ori) * bins_per_rad;
                        const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                        int o0 = (int)floorf(obin);
                        rbin -= (float)r0;
                        cbin -= (float)c0;
                        obin -= (float)o0;
                        if (o0 < 0) o0 += 8;
                        if (o0 >= 8) o0 -= 8;
                        rec = make_float4(v.x, rbin, cbin, obin);
                        pk = (r0 + 1) | ((c0 + 1) << 4) | (o0 << 8);
                    }
                    s_rec[grp][rr][j + radius] = rec;
                    s_pk[grp][rr][j + radius] = pk;
                    }
                }
            }
            sd_wave_sync();
            // walk: the lane's cells over their parts of the strip, raster order.
            // One loop over the concatenated j-ranges of the lane's cells (cell
            // cc = 0's, then cc = 1's: separate slots), so a lane with one active
            // cell does not wait out an empty loop of the other
#pragma unroll
            for (int rr = 0; rr < kStrip; rr++) {
                const int i = ui0 + t * kStrip + rr, r = pty + i;
                if (r <= 0 || r >= oh - 1) continue;
                int jaC[kCpl], nC[kCpl];
#pragma unroll
                for (int cc = 0; cc < kCpl; cc++) {
                    const int cell = q + cc * L, ci = cell >> 2, cj = cell & 3;
                    int ja = max(j0[cc], 1 - ptx), jb = min(j1[cc], ow - 2 - ptx);   // c in (0, ow - 1)
                    if (fits) { ja = max(ja, jaU[rr]); jb = min(jb, jbU[rr]); }
                    const bool on = i >= i0[cc] && i <= i1[cc] &&
                                    rowclip(i, (float)cj - 2.5f, (float)cj - 0.5f, (float)ci - 2.5f, (float)ci - 0.5f, ja, jb);
                    jaC[cc] = ja;
                    nC[cc] = on ? max(0, jb - ja + 1) : 0;
                }
                int ntot = nC[0];
                if constexpr (kCpl > 1) ntot += nC[1];
                if (p.dbg & 1) ntot = 0;
                const float ic = (float)i * cos_t, is = (float)i * sin_t;
                auto jof = [&](int k) { return (kCpl > 1 && k >= nC[0]) ? jaC[kCpl - 1] + (k - nC[0]) : jaC[0] + k; };
                // one visit: the share of sample (i, j) in this cell's two slots
                auto visit = [&](int k, int j, float2 v, bool direct) {
                    const bool sel = kCpl > 1 && k >= nC[0];
                    const int ci = (q >> 2) + (sel ? L >> 2 : 0), cj = q & 3;
                    const float c_rot = (float)j * cos_t - is;
                    const float r_rot = (float)j * sin_t + ic;
                    float rbin = r_rot + 2.f - 0.5f, cbin = c_rot + 2.f - 0.5f;
                    // the reference's rbin, cbin in (-1, 4): < 4 follows from dr, dc >= 0
                    if (!(rbin > -1.f && cbin > -1.f)) return;
                    const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                    const int dr = ci - r0, dc = cj - c0;
                    if ((unsigned)dr > 1u || (unsigned)dc > 1u) return;
                    if (direct) v = eval(r, ptx + j, c_rot, r_rot);
                    const float mag = v.x;
                    float obin = (v.y - ori) * bins_per_rad;
                    int o0 = (int)floorf(obin);
                    rbin -= (float)r0;
                    cbin -= (float)c0;
                    obin -= (float)o0;
                    if (o0 < 0) o0 += 8;
                    if (o0 >= 8) o0 -= 8;
                    const float v_r1 = mag * rbin, v_r0 = mag - v_r1;
                    const float vr = dr == 0 ? v_r0 : v_r1;
                    const float v_rc1 = vr * cbin, v_rc0 = vr - v_rc1;
                    const float vc = dc == 0 ? v_rc0 : v_rc1;
                    const float v_o1 = vc * obin, v_o0 = vc - v_o1;
                    // both slots read, then both written (distinct slots): one LDS round trip
                    const int sl = ((sel ? 10 : 0) + o0) * 256;
                    const float a0 = hs[sl], a1 = hs[sl + 256];
                    hs[sl] = __fadd_rn(a0, v_o0);
                    hs[sl + 256] = __fadd_rn(a1, v_o1);
                };
                if (fits) {
                    // the staged sample of the next visit is read one visit ahead
                    const float4* rowr = &s_rec[grp][rr][0];
                    const int* rowp = &s_pk[grp][rr][0];
                    int x = min(max(jof(0) + radius, 0), kSdW - 1);
                    float4 nr = rowr[x];
                    int np = rowp[x];
                    for (int k = 0; k < ntot; k++) {
                        const float4 rec = nr;
                        const int pk = np;
                        x = min(max(jof(k + 1) + radius, 0), kSdW - 1);
                        nr = rowr[x];
                        np = rowp[x];
                        const bool sel = kCpl > 1 && k >= nC[0];
                        const int ci = (q >> 2) + (sel ? L >> 2 : 0), cj = q & 3;
                        const int dr = ci + 1 - (pk & 15), dc = cj + 1 - ((pk >> 4) & 15);
                        if ((unsigned)dr > 1u || (unsigned)dc > 1u) continue;
                        const int o0 = pk >> 8;
                        const float mag = rec.x;
                        const float v_r1 = mag * rec.y, v_r0 = mag - v_r1;
                        const float vr = dr == 0 ? v_r0 : v_r1;
                        const float v_rc1 = vr * rec.z, v_rc0 = vr - v_rc1;
                        const float vc = dc == 0 ? v_rc0 : v_rc1;
                        const float v_o1 = vc * rec.w, v_o0 = vc - v_o1;
                        const int sl = ((sel ? 10 : 0) + o0) * 256;
                        const float a0 = hs[sl], a1 = hs[sl + 256];
                        hs[sl] = __fadd_rn(a0, v_o0);
                        hs[sl + 256] = __fadd_rn(a1, v_o1);
                    }
                } else {
                    for (int k = 0; k < ntot; k++) visit(k, jof(k), make_float2(0.f, 0.f), true);
                }
            }
            sd_wave_sync();
        }
        // circular fold into the keypoint's 128 raw bins (cell * 8 + o)
#pragma unroll
        for (int cc = 0; cc < kCpl; cc++) {
            float h[10];
#pragma unroll
            for (int k = 0; k < 10; k++) h[k] = hs[(cc * 10 + k) * 256];
            h[0] += h[8];
            h[1] += h[9];
#pragma unroll
            for (int o = 0; o < 8; o++) raw[(q + cc * L) * 8 + o] = h[o];
        }
        __syncthreads();
        // first norm: 8 fma chains over k = l + 8 m (lanes q < 8 of the keypoint), v_reduce_sum order
        float part = 0.f;
        if (q < 8)
            for (int m = 0; m < 16; m++) { const float t = raw[q + 8 * m]; part = fmaf(t, t, part); }
        float l[8];
#pragma unroll
        for (int t = 0; t < 8; t++) l[t] = __shfl(part, (tid & ~(L - 1) & 63) + t, 64);
        const float nrm2 = ((l[0] + l[4]) + (l[1] + l[5])) + ((l[2] + l[6]) + (l[3] + l[7]));
        const float thr = cr_sqrtf(nrm2) * 0.2f;
        float v[kCpl][8];
#pragma unroll
        for (int cc = 0; cc < kCpl; cc++)
#pragma unroll
            for (int o = 0; o < 8; o++) v[cc][o] = fminf(raw[(q + cc * L) * 8 + o], thr);
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < kCpl; cc++)
#pragma unroll
            for (int o = 0; o < 8; o++) raw[(q + cc * L) * 8 + o] = v[cc][o];
        __syncthreads();
        // second norm: sequential over k = 0..127
        float n2 = 0.f;
        for (int k = 0; k < 128; k++) { const float t = raw[k]; n2 += t * t; }
        const float sq = cr_sqrtf(n2);
        const float sc = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        if (live) {
#pragma unroll
            for (int cc = 0; cc < kCpl; cc++)
#pragma unroll
                for (int o = 0; o < 8; o++)
                    p.desc[drow * 128 + (q + cc * L) * 8 + o] = fminf(fmaxf(rintf(v[cc][o] * sc), 0.f), 255.f);
        }
        __syncthreads();
    }
}

}  // namespace

// f(0 .. n-1) on up to 16 host threads (the GPU box's CPU share per GPU), the
// calling thread included; items are independent.  The workers persist (one
// pool per process, started on first use): spawning 15 threads per call cost
// about as much as the work it spread.
class HostPool {
public:
    explicit HostPool(int nworkers)
    {
        for (int t = 0; t < nworkers; t++) th_.emplace_back([this] { loop(); });
    }
    int size() const { return (int)th_.size() + 1; }
    void run(int n, const std::function<void(int)>& f)
    {
        std::unique_lock<std::mutex> lk(m_);
        job_ = &f;
        njobs_ = n;
        next_.store(0);
        busy_ = (int)th_.size();
        gen_++;
        lk.unlock();
        cv_.notify_all();
        work();
        lk.lock();
        done_.wait(lk, [&] { return busy_ == 0; });
        job_ = nullptr;
    }

private:
    void work()
    {
        for (int i; (i = next_.fetch_add(1)) < njobs_;) (*job_)(i);
    }
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> lk(m_);
            if (--busy_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int njobs_ = 0, busy_ = 0;
    uint64_t gen_ = 0;
    std::atomic<int> next_{0};
};

// one pool for every caller (a function-local static in a template would give
// each instantiation its own)
void host_parallel_run(int n, const std::function<void(int)>& fn)
{
    static const int hw = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    if (n <= 1 || hw <= 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    static HostPool* pool = new HostPool(hw - 1);     // never destroyed: idle workers at exit
    // one caller at a time; a second caller (another host thread, or a job of the
    // pool itself) runs its items on its own thread instead of waiting
    static std::mutex one;
    std::unique_lock<std::mutex> lk(one, std::try_to_lock);
    if (!lk.owns_lock()) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    pool->run(n, fn);
}

void host_copy(void* dst, const void* src, size_t n)
{
    constexpr size_t kPiece = 512 << 10;
    const int np = (int)std::min<size_t>(16, (n + kPiece - 1) / kPiece);
    if (np <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t per = (n + np - 1) / np;
    host_parallel_run(np, [&](int i) {
        const size_t a = (size_t)i * per, e = std::min(n, a + per);
        if (a < e) std::memcpy(static_cast<uint8_t*>(dst) + a, static_cast<const uint8_t*>(src) + a, e - a);
    });
}

namespace {

template <typename F>
void host_parallel_for(int n, F&& f)
{
    host_parallel_run(n, std::function<void(int)>([&](int i) { f(i); }));
}


}  // namespace

// pyramid geometry + sigmas (oracle/siftdet.c orc_sift_octaves / orc_sift_sigmas)
static void pyr_layout(int w, int h, PyrInfo& P, size_t& total, bool with_dog)
{
    const int m = std::min(2 * w, 2 * h);
    P.n = std::min((int)std::lrint(std::log((double)m) / std::log(2.) - 2) + 1, kMaxOct);
    size_t off = 0;
    int W = 2 * w, H = 2 * h;
    for (int o = 0; o < P.n; o++) {
        P.o[o].w = W;
        P.o[o].h = H;
        const size_t px = ((size_t)W * H + 63) & ~(size_t)63;
        for (int i = 0; i < kGL; i++, off += px) P.o[o].g[i] = off;
        for (int i = 0; i < kDL; i++) {             // DoG planes: only when the blurs write them
            P.o[o].d[i] = off;
            if (with_dog) off += px;
        }
        W /= 2;
        H /= 2;
    }
    total = off;
}

// the detector over nf gray frames (w x h, contiguous) in c->gray: pyramids,
// extrema, refinement and orientation for all frames at once, the host's
// per-frame duplicate filter, then descriptors.  out / desc: frame-major, cap
// entries per frame, in host memory (dev_out = false) or device memory (true);
// n_out[f] = keypoints found in frame f (may exceed cap).
// The pyramid blurs' tiles in XCD-contiguous order (xcd_tile: a tile's halo
// neighbours share its XCD's L2): their fetch falls 11.9 -> 4.1 GB per 16-frame
// call at the same or slightly better time (scripts/r5_sdxcd.sh, 1201 / 1199 ->
// 1212 / 1199 frames/s, bit-exact).  sd_extrema's tiles too (round 6: its
// 64-float rows start one float early, so each row touches a cache line its
// neighbour tile also fetches; 6.9 GB per 16-frame call in the plain order):
// 169 -> 152 us per launch, and sd_refine, which takes the candidates in the
// order the tiles appended them, 1.55 -> 1.34 ms (1 431-1 452 -> 1 512-1 518
// frames/s, scripts/r6_det.sh r6det10).  SLAMHIP_SD_XCD=0: the plain order.
static bool sd_xcd_on()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_SD_XCD"); return !(e && e[0] == '0'); }();
    return on;
}

// The DoG planes: not stored by default -- sd_extrema and sd_refine subtract
// the two Gaussian layers themselves (the same operands, so the same values),
// and each blur writes one plane instead of two.  SLAMHIP_SD_DOG=1: the blurs
// write the DoG planes and the later kernels read them (the round-5 form).
// The doubled base image: evaluated inside the first blur's tile staging (1,
// the default) or written by sd_upsample and read back (0, the round-5 form)
#ifndef SD_FUSED_UPS
#define SD_FUSED_UPS 1
#endif
constexpr bool kSdFusedUps = SD_FUSED_UPS != 0;

static bool sd_dog_planes()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_SD_DOG"); return e && e[0] == '1'; }();
    return on;
}

// sd_refine's grid (one wavefront per workgroup, candidates strided over it)
static int sd_refine_blocks()
{
    static const int n = [] {
        const char* e = getenv("SLAMHIP_SD_REFINE_BLOCKS");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : 4096;
    }();
    return n;
}

static int sift_detect_frames(slam_ctx* c, hipStream_t s, int nf, int w, int h, slam_keypoint* out, int cap,
                              int* n_out, float* desc, bool dev_out)
{
    const bool dogless = !sd_dog_planes();
    PyrInfo P;
    size_t total;
    pyr_layout(w, h, P, total, !dogless);
    const size_t fT = total, fD = (size_t)4 * w * h;          // pyramid / doubled-base floats per frame
    SLAM_HIP(c, c->sd_pyr.ensure((size_t)nf * fT * sizeof(float)));
    float* pyr = c->sd_pyr.as<float>();
    float* dbl = nullptr;
    if (!kSdFusedUps) {
        SLAM_HIP(c, c->ftmp.ensure((size_t)nf * fD * sizeof(float)));
        dbl = c->ftmp.as<float>();
        hipLaunchKernelGGL(sd_upsample, dim3((2 * w + 255) / 256, 2 * h, nf), dim3(256), 0, s, c->gray.as<uint8_t>(), w,
                           h, dbl, (size_t)w * h, fD);
    }
    // buildGaussianPyramid: SIFT_Impl's double sigma (1.6), not the float 1.6f
    double sig[kGL];
    sig[0] = 1.6;
    const double kk = std::pow(2., 1. / kLayers);
    for (int i = 1; i < kGL; i++) {
        const double sig_prev = std::pow(kk, (double)(i - 1)) * 1.6, sig_total = sig_prev * kk;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    auto blur = [&](const float* src, size_t sstride, float* dst, float* dog, int W, int H, double sigma,
                    const uint8_t* gray = nullptr) -> hipError_t {
        BlurParams b;
        b.gray = gray; b.gstride = (size_t)w * h; b.gw = w; b.gh = h;
        const int ks = (int)std::lrint(sigma * 4 * 2 + 1) | 1;
        if (ks > 2 * kMaxR + 1) return hipErrorInvalidValue;
        gauss_kernel_f32(ks, sigma, b.k);
        b.src = src; b.dst = dst; b.dog = dog; b.w = W; b.h = H; b.r = ks / 2;
        b.xcd = sd_xcd_on() ? 1 : 0;
        b.sstride = sstride; b.dstride = fT;
        const dim3 grid((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, nf);
        if (gray) {      // the doubled base image's blur (ksize 11), from the u8 frames
            if (b.r != 5) return hipErrorInvalidValue;
            hipLaunchKernelGGL((sd_blur<5, true>), grid, dim3(256), 0, s, b);
            return hipGetLastError();
        }
        switch (b.r) {   // ksize 11 / 13 / 17 / 21 / 27 for the default sigmas
        case 5: hipLaunchKernelGGL(sd_blur<5>, grid, dim3(256), 0, s, b); break;
        case 6: hipLaunchKernelGGL(sd_blur<6>, grid, dim3(256), 0, s, b); break;
        case 8: hipLaunchKernelGGL(sd_blur<8>, grid, dim3(256), 0, s, b); break;
        case 10: hipLaunchKernelGGL(sd_blur<10>, grid, dim3(256), 0, s, b); break;
        case 13: hipLaunchKernelGGL(sd_blur<13>, grid, dim3(256), 0, s, b); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    };
    {
        const float sd2 = std::sqrt(std::max(kSigma * kSigma - 0.5f * 0.5f * 4, 0.01f));
        SLAM_HIP(c, blur(dbl, fD, pyr + P.o[0].g[0], nullptr, P.o[0].w, P.o[0].h, (double)sd2,
                         kSdFusedUps ? c->gray.as<uint8_t>() : nullptr));
    }
    for (int o = 0; o < P.n; o++) {
        const Oct& O = P.o[o];
        if (o > 0) {
            const Oct& Q = P.o[o - 1];
            const double ifx = 1. / ((double)O.w / Q.w), ify = 1. / ((double)O.h / Q.h);
            hipLaunchKernelGGL(sd_down, dim3((O.w + 255) / 256, O.h, nf), dim3(256), 0, s, pyr + Q.g[kLayers], Q.w, Q.h,
                               pyr + O.g[0], O.w, O.h, ifx, ify, fT);
        }
        for (int i = 1; i < kGL; i++)
            SLAM_HIP(c, blur(pyr + O.g[i - 1], fT, pyr + O.g[i], dogless ? nullptr : pyr + O.d[i - 1], O.w, O.h, sig[i]));
    }
    // extrema candidates ({octave | frame << 8, layer, r, c}) of every frame
    if (nf <= 0 || nf > kSiftDetectMaxFrames) return set_err(c, SLAM_E_INVALID_ARG, "detector batch size");
    const int ccap = nf << 20, kcap_f = 1 << 20, kcap = nf * kcap_f;   // <= 2^28: int-indexed in the kernels
    SLAM_HIP(c, c->sd_cand.ensure((size_t)ccap * sizeof(int4)));
    SLAM_HIP(c, c->sd_kps.ensure((size_t)kcap * sizeof(slam_keypoint)));
    SLAM_HIP(c, c->misc.ensure((size_t)(8 + 1 + kSiftDetectMaxFrames) * sizeof(int)));
    int* cnt = c->misc.as<int>() + 8;      // [0] candidates, [1 + f] frame f's keypoints
    SLAM_HIP(c, hipMemsetAsync(cnt, 0, (size_t)(1 + nf) * sizeof(int), s));
    for (int o = 0; o < P.n; o++) {
        const Oct& O = P.o[o];
        if (O.w <= 2 * kImgBorder || O.h <= 2 * kImgBorder) continue;
        ExtParams e;
        e.pyr = pyr; e.P = P; e.o = o; e.fstride = fT; e.cand = c->sd_cand.as<int4>(); e.ncand = cnt; e.cap = ccap;
        e.dogless = dogless ? 1 : 0;
        e.xcd = sd_xcd_on() ? 1 : 0;      // as the blurs: halo lines shared in one XCD's L2
        hipLaunchKernelGGL(sd_extrema,
                           dim3((O.w - 2 * kImgBorder + kEW - 1) / kEW, (O.h - 2 * kImgBorder + kEH - 1) / kEH, nf),
                           dim3(256), 0, s, e);
    }
    SLAM_HIP(c, hipGetLastError());
    RefineParams rp;
    rp.pyr = pyr; rp.P = P; rp.fstride = fT; rp.cand = c->sd_cand.as<int4>(); rp.ncand = cnt; rp.cap = ccap;
    rp.kps = c->sd_kps.as<slam_keypoint>(); rp.nkps = cnt + 1; rp.kcap = kcap_f;
    std::memcpy(rp.exptab, c->sift.exptab, sizeof(rp.exptab));
    static const int rdbg = [] { return diag_env_int("SLAMHIP_SD_REFINE_DBG"); }();   // -DSLAMHIP_DIAG builds only
    rp.dbg = rdbg;
    if (dogless)
        hipLaunchKernelGGL(sd_refine<true>, dim3(sd_refine_blocks()), dim3(64), 0, s, rp);
    else
        hipLaunchKernelGGL(sd_refine<false>, dim3(sd_refine_blocks()), dim3(64), 0, s, rp);
    SLAM_HIP(c, hipGetLastError());
    // SLAMHIP_DET_TIMING=1: host phase times per call on stderr (diagnostics)
    static const bool timing = [] { const char* e = getenv("SLAMHIP_DET_TIMING"); return e && e[0] == '1'; }();
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_enq = now();
    // the candidate count and each frame's keypoint count
    std::vector<int> counts((size_t)nf + 1);
    SLAM_HIP(c, hipMemcpyAsync(counts.data(), cnt, counts.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    auto t_gpu1 = now();
    if (counts[0] > ccap) return set_err(c, SLAM_E_CAPACITY, "SIFT detector candidate overflow");
    // per frame (class_id): KeyPointsFilter::removeDuplicatedSorted, then firstOctave
    // = -1 back to input units.  sd_refine wrote each frame's keypoints to its
    // own region, sd_kp_compact packs the regions frame-major: frame f's are
    // rows fofs[f] .. fofs[f + 1] of the list read back
    std::vector<int> fofs((size_t)nf + 1, 0);
    int most = 0;
    for (int f = 0; f < nf; f++) {
        const int n = counts[(size_t)f + 1];
        if (n > kcap_f) return set_err(c, SLAM_E_CAPACITY, "SIFT detector keypoint overflow");
        fofs[(size_t)f + 1] = fofs[(size_t)f] + n;
        most = std::max(most, n);
    }
    // one pinned buffer: the refined keypoints come back through it, then the
    // descriptor batch (keypoints, frames, cos / sin, frame row bases) goes out
    // through it in one copy
    const size_t nall = (size_t)fofs[(size_t)nf];
    const size_t off_frame = nall * sizeof(slam_keypoint), off_cs = off_frame + nall * sizeof(int),
                 off_fb = off_cs + nall * 2 * sizeof(float), stage_bytes = off_fb + (size_t)nf * sizeof(int);
    // (host output: the descriptors come back through it too, after the kernel)
    const size_t back_bytes = (!dev_out && desc) ? nall * 128 * sizeof(float) : 0;
    uint8_t* pin = static_cast<uint8_t*>(readback(c, std::max<size_t>(std::max(stage_bytes, back_bytes), 64)));
    if (!pin) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    if (nall > 0) {
        SLAM_HIP(c, c->sd_kpc.ensure(nall * sizeof(slam_keypoint)));
        const int bx = std::min((most * 7 + 255) / 256, 64);
        hipLaunchKernelGGL(sd_kp_compact, dim3(bx, nf), dim3(256), 0, s, c->sd_kps.as<slam_keypoint>(), cnt + 1, kcap_f,
                           c->sd_kpc.as<slam_keypoint>());
        SLAM_HIP(c, hipGetLastError());
        SLAM_HIP(c, hipMemcpyAsync(pin, c->sd_kpc.p, nall * sizeof(slam_keypoint), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipStreamSynchronize(s));
    }
    auto t_d2h = now();
    const slam_keypoint* allp = reinterpret_cast<const slam_keypoint*>(pin);
    auto t_b1 = now();
    std::vector<std::vector<slam_keypoint>>& per = c->sd_per;
    if ((int)per.size() < nf) per.resize((size_t)nf);
    std::vector<std::vector<std::pair<float, int>>>& ords = c->sd_ord;
    if ((int)ords.size() < nf) ords.resize((size_t)nf);
    // the frames' filters are independent: host threads, one frame at a time each.
    // The sort orders (x, index) pairs, ties by the full KeypointGreater order:
    // the same sequence as sorting the keypoints (equal keypoints are identical
    // in every field), a third of the time
    host_parallel_for(nf, [&](int f) {
        const slam_keypoint* src = allp + fofs[(size_t)f];
        const int n0 = fofs[(size_t)f + 1] - fofs[(size_t)f];
        std::vector<std::pair<float, int>>& ord = ords[(size_t)f];
        kp_order(src, n0, ord);
        std::vector<slam_keypoint>& k = per[(size_t)f];
        k.clear();
        k.reserve((size_t)n0);
        for (int i = 0; i < n0; i++) {
            const slam_keypoint& b = src[ord[(size_t)i].second];
            if (!k.empty()) {
                const slam_keypoint& a = k.back();
                if (!(a.x != b.x || a.y != b.y || a.size != b.size || a.angle != b.angle)) continue;
            }
            k.push_back(b);
        }
        for (auto& kp : k) {
            kp.class_id = -1;
            kp.octave = (kp.octave & ~255) | ((kp.octave - 1) & 255);
            kp.x *= 0.5f;
            kp.y *= 0.5f;
            kp.size *= 0.5f;
        }
    });
    auto t_b2 = now();
    // the descriptor batch: min(n, cap) per frame, frame-major
    std::vector<int> qf((size_t)nf + 1, 0);
    for (int f = 0; f < nf; f++) {
        const std::vector<slam_keypoint>& k = per[(size_t)f];
        const int n = (int)k.size();
        n_out[f] = n;
        const int nn = std::min(n, cap);
        if (out && nn > 0 && !dev_out) std::memcpy(out + (size_t)f * cap, k.data(), (size_t)nn * sizeof(slam_keypoint));
        qf[(size_t)f + 1] = qf[(size_t)f] + nn;
    }
    const int nd = qf[(size_t)nf];
    auto t_b3 = now();
    slam_keypoint* st_kp = reinterpret_cast<slam_keypoint*>(pin);
    int* st_frame = reinterpret_cast<int*>(pin + off_frame);
    float* st_cs = reinterpret_cast<float*>(pin + off_cs);
    int* st_fb = reinterpret_cast<int*>(pin + off_fb);
    host_parallel_for(nf, [&](int f) {
        const int q = qf[(size_t)f], nn = qf[(size_t)f + 1] - q;
        st_fb[f] = f * cap - q;
        if (nn <= 0) return;
        std::memcpy(st_kp + q, per[(size_t)f].data(), (size_t)nn * sizeof(slam_keypoint));
        for (int i = 0; i < nn; i++) st_frame[q + i] = f;
        if (desc) {
            std::vector<float> part;
            sift_kp_cs(st_kp + q, nn, part);      // cosf / sinf of the descriptor angle
            std::memcpy(st_cs + (size_t)2 * q, part.data(), (size_t)2 * nn * sizeof(float));
        }
    });
    auto t_filt = now();
    // the batch to the device (the staged regions at their pinned offsets)
    SLAM_HIP(c, c->qbuf.ensure(stage_bytes));
    uint8_t* dst = c->qbuf.as<uint8_t>();
    if (nd > 0) {
        SLAM_HIP(c, hipMemcpyAsync(dst, pin, (size_t)nd * sizeof(slam_keypoint), hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(dst + off_frame, pin + off_frame, (size_t)nd * sizeof(int), hipMemcpyHostToDevice, s));
        if (desc)
            SLAM_HIP(c, hipMemcpyAsync(dst + off_cs, pin + off_cs, (size_t)nd * 2 * sizeof(float), hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(dst + off_fb, pin + off_fb, (size_t)nf * sizeof(int), hipMemcpyHostToDevice, s));
    }
    const slam_keypoint* d_kp = reinterpret_cast<const slam_keypoint*>(dst);
    if (dev_out && out && nd > 0 && !desc) {
        // the kept keypoints to the caller's device buffer, frame f at row f * cap
        for (int f = 0; f < nf; f++) {
            const int nn = qf[(size_t)f + 1] - qf[(size_t)f];
            if (nn > 0)
                SLAM_HIP(c, hipMemcpyAsync(out + (size_t)f * cap, d_kp + qf[(size_t)f], (size_t)nn * sizeof(slam_keypoint),
                                           hipMemcpyDeviceToDevice, s));
        }
    }
    if (desc && nd > 0) {
        auto t_cs = now();
        if (timing) {
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            fprintf(stderr, "[det] bucket %.0f sort %.0f serial %.0f stage %.0f h2d-enqueue %.0f us\n", us(t_d2h, t_b1), us(t_b1, t_b2),
                    us(t_b2, t_b3), us(t_b3, t_filt), us(t_filt, t_cs));
        }
        if (!dev_out) SLAM_HIP(c, c->desc_f32.ensure((size_t)nd * 128 * sizeof(float)));
        DescParams dp;
        dp.pyr = pyr; dp.P = P; dp.fstride = fT; dp.kp_frame = reinterpret_cast<const int*>(dst + off_frame);
        dp.kps = d_kp; dp.cs = reinterpret_cast<const float*>(dst + off_cs); dp.n = nd;
        // device output: descriptors and keypoints written at their frame rows by
        // the kernel (no per-frame copies); host output: compact, copied below
        dp.desc = dev_out ? desc : c->desc_f32.as<float>();
        dp.fbase = dev_out ? reinterpret_cast<const int*>(dst + off_fb) : nullptr;
        dp.kout = dev_out ? out : nullptr;
        std::memcpy(dp.exptab, c->sift.exptab, sizeof(dp.exptab));
        // SLAMHIP_SD_DESC=0: the direct form; SLAMHIP_SD_CPL: cells per lane (1 / 2)
        static const int form = [] { const char* e = getenv("SLAMHIP_SD_DESC"); return e ? atoi(e) : 1; }();
        static const int cpl = [] { const char* e = getenv("SLAMHIP_SD_CPL"); return e ? atoi(e) : 1; }();
        static const int dbg = [] { return diag_env_int("SLAMHIP_SD_DBG"); }();   // -DSLAMHIP_DIAG builds only
        dp.dbg = dbg;
        // blocks in XCD-contiguous order (scripts/r5_descxcd.sh: 15.80 -> 15.69 ms per 4 calls, 1210 / 1202 ->
        // 1215 / 1219 frames/s, bit-exact); SLAMHIP_SD_DESC_XCD=0: the plain order
        static const int dxcd = [] { const char* e = getenv("SLAMHIP_SD_DESC_XCD"); return e && e[0] == '0' ? 0 : 1; }();
        dp.xcd = dxcd;
        const int kpb = cpl == 1 ? 16 : 32;      // keypoints per block
        const dim3 dgrid(std::min((nd + kpb - 1) / kpb, 8192));
        if (form == 0)
            hipLaunchKernelGGL(sd_desc, dim3(std::min((nd + 15) / 16, 8192)), dim3(256), 0, s, dp);
        else if (cpl == 1)
            hipLaunchKernelGGL((sd_desc_staged<1, 1>), dgrid, dim3(256), 0, s, dp);
        else
            hipLaunchKernelGGL((sd_desc_staged<1, 2>), dgrid, dim3(256), 0, s, dp);
        SLAM_HIP(c, hipGetLastError());
        if (!dev_out)   // one DMA into the pinned buffer (its staged inputs were consumed before the kernel)
            SLAM_HIP(c, hipMemcpyAsync(pin, c->desc_f32.p, (size_t)nd * 128 * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    auto t_enq2 = now();
    SLAM_HIP(c, hipStreamSynchronize(s));
    if (desc && nd > 0 && !dev_out) {
        // frame-major with cap rows per frame
        for (int f = 0; f < nf; f++) {
            const int nn = qf[(size_t)f + 1] - qf[(size_t)f];
            if (nn > 0)
                host_copy(desc + (size_t)f * cap * 128, pin + (size_t)qf[(size_t)f] * 128 * sizeof(float),
                          (size_t)nn * 128 * sizeof(float));
        }
    }
    if (timing) {
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[det] nf %d nd %d enqueue %.0f gpu-wait %.0f d2h %.0f filter %.0f tail-enqueue %.0f tail-wait %.0f us\n", nf, nd,
                us(t_enq, t_enq), us(t_enq, t_gpu1), us(t_gpu1, t_d2h), us(t_d2h, t_filt), us(t_filt, t_enq2), us(t_enq2, now()));
    }
    return SLAM_OK;
}

int sift_detect(slam_ctx* c, const uint8_t* dimg, size_t dstep, int channels, int w, int h, slam_keypoint* out,
                int cap, int* n_out, float* desc)
{
    hipStream_t s = c->stream;
    SLAM_HIP(c, launch_gray(c, s, dimg, dstep, channels, w, h));
    return sift_detect_frames(c, s, 1, w, h, out, cap, n_out, desc, false);
}

int sift_detect_batch(slam_ctx* c, hipStream_t s, const uint8_t* d_frames, int nframes, int w, int h, int channels,
                      slam_keypoint* out, int cap, int* n_out, float* desc)
{
    SLAM_HIP(c, launch_gray_batch(c, s, d_frames, nframes, w, h, channels));
    return sift_detect_frames(c, s, nframes, w, h, out, cap, n_out, desc, true);
}

}  // namespace slamhip
