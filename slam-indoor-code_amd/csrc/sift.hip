// SIFT descriptors on provided (FAST) keypoints, gfx950.
//
// Replaces extractDescriptor's cv::SIFT::create()->compute(frame, kps, desc)
// (reference featureMatchingCPU.cpp:51-65 / featureMatchingCUDA.cpp:57-68).
// With octave-0 keypoints OpenCV builds one octave and reads only gpyr[0]:
// base = GaussianBlur(gray -> f32, sigma = sqrt(1.6^2 - 0.5^2), 13 taps,
// REFLECT_101), then calcSIFTDescriptor(base, pt, 360 - angle, size / 2, 4, 8).
//
//   sift_blur_grad        separable blur (same f32 operation order as OpenCV's
//                         RowVec_32f fma chain and SymmColumnVec_32f symmetric fma
//                         form -> bit-identical to the oracle) fused with the
//                         per-pixel gradient magnitude (sqrt(fma(dx,dx,dy*dy)))
//                         and fastAtan2 orientation: the per-sample transcendental
//                         work of calcSIFTDescriptor, done once per pixel instead
//                         of once per (keypoint, sample) -- every 1080p pixel is
//                         inside ~27 keypoint windows at 10k keypoints.
//   sift_desc             one wave per keypoint: the 75 x 75 window sweep with the
//                         reference's bin geometry / exp32f weights, trilinear
//                         histogram in LDS (ds_add_f32), the reference's flat
//                         histogram indexing (incl. the 361-degree o0 = -1 quirk,
//                         see oracle/sift.c), circular fold, 0.2 clamp,
//                         renormalisation x512, round-half-even, saturate u8.
// Histogram adds are commutative only up to f32 rounding, so descriptors match
// the oracle within the stated tolerance (|delta| <= 1 per element), not bitwise.
#include <cfloat>

#include "sift_dev.h"
#include "slamhip_internal.h"

namespace slamhip {

namespace {
using namespace sd;

// Fused SIFT base layer + gradient map.  One 512-thread block per 64 x 64
// output tile: the gray tile with a 7-px REFLECT_101 halo goes to LDS, the row
// pass (RowVec_32f: fma chain from 0 over the 13 taps) and the column pass
// (SymmColumnVec_32f: S0 * k0, then fma(S[m] + S[-m], k[m], .)) run out of LDS,
// and only the float2 {magnitude, orientation} map is written to HBM -- the
// f32 row-blurred and blurred planes never leave the CU.  Same operations in
// the same order as the oracle's blur, so the map is bit-identical.
#ifndef BLUR_DIAG
#define BLUR_DIAG 0             // timing-only variants (wrong results): 1 no gradient math, 2 no blur taps, 3 no stores, 4 = 1 + 2
#endif
constexpr int kBT = 64;                 // output tile (square)
constexpr int kBH = 7;                  // halo: 6 (13-tap blur) + 1 (central differences)
constexpr int kGR = kBT + 2 * kBH;      // 78 gray tile rows (y0 - 7 .. y0 + 70)
constexpr int kGL = 80;                 // gray tile columns x0 - 8 .. x0 + 71 (dword aligned)
// gray tile row stride (bytes): 24 dwords, so rows r and r + 2 are 48 = 16 (mod 32)
// dwords apart and the row pass's 32-lane groups (16 tasks of one row pair, 16
// of the next) read 32 distinct banks
#ifndef SIFT_BLUR_GS
#define SIFT_BLUR_GS 96
#endif
constexpr int kGS = SIFT_BLUR_GS;
constexpr int kTW = 68;                 // row-pass / base columns x0 - 1 .. x0 + 66 (66 used)
constexpr int kTR = kBT + 2;            // 66 base rows (y0 - 1 .. y0 + 64)
constexpr int kStrip = 6;               // column-pass outputs per task (11 strips of 6 rows)
constexpr int kBlurThreads = 512;
static_assert(kGR % 2 == 0 && kTW % 4 == 0 && kTR % kStrip == 0, "packed pass shapes");

typedef float bf2 __attribute__((ext_vector_type(2)));

struct BlurGradParams {
    const uint8_t* gray;
    float2* grad;      // {magnitude, orientation in degrees}
    int w, h;
    int tile0;         // 1: the grid starts at the first in-image tile (the border is already zero)
    int obin;          // 1: store obin = (ori - ori_deg) * 8 / 360 instead of ori (sift_desc_band's stage value);
                       // 2: store fract(obin), and (floor(obin) + 9) * 6 in the byte plane posb
                       //    (sift_desc_band's slot position, for floor(obin) in [-9, -1])
    float ori_deg;
    uint8_t* posb;     // obin 2: one byte per pixel, the map's layout
    int xcd;           // tiles in XCD-contiguous order (xcd_tile)
    SiftConsts k;
};

// a / b, correctly rounded, for 0 <= a <= b with a = 0 or a >= 2^-60 and
// 2^-60 <= b <= 2^10: the gfx950 IEEE f32 division sequence (rcp, one
// reciprocal refinement, two quotient refinements) without its v_div_scale /
// v_div_fixup steps, which are identities on this domain (no operand or
// quotient near the denormal / overflow range; 0 / b = 0 falls out of the
// sequence).  fastAtan2's c = min / (max + DBL_EPSILON) on differences of the
// blurred u8 base lies in it: a nonzero blurred value is >= ~1e-8 (the
// kernel's smallest tap squared), so a nonzero |dx| is >= its ulp, 2^-51.
__device__ __forceinline__ float div_cr_grad(float a, float b)
{
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __fmaf_rn(-b, y, 1.f);
    y = __fmaf_rn(e, y, y);
    float q = __fmul_rn(a, y);
    float r = __fmaf_rn(-b, q, a);
    q = __fmaf_rn(r, y, q);
    r = __fmaf_rn(-b, q, a);
    return __fmaf_rn(r, y, q);
}

// the same sequence on the two lanes of a packed pair (per-element IEEE fma:
// bit-identical to two div_cr_grad calls)
__device__ __forceinline__ bf2 div_cr_grad2(bf2 a, bf2 b)
{
    bf2 y = {__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    const bf2 one = {1.f, 1.f};
    const bf2 e = __builtin_elementwise_fma(-b, y, one);
    y = __builtin_elementwise_fma(e, y, y);
    bf2 q = a * y;
    bf2 r = __builtin_elementwise_fma(-b, q, a);
    q = __builtin_elementwise_fma(r, y, q);
    r = __builtin_elementwise_fma(-b, q, a);
    return __builtin_elementwise_fma(r, y, q);
}

// correctly rounded sqrt of a finite x >= 0 (no NaN / infinity here): the
// gfx950 f32 sequence (2^32 prescale below 2^-96, hardware sqrt, +-1 ulp
// residual tests) without its class check (it only returns x for 0, inf, NaN;
// 0 already comes out of the sequence as 0)
__device__ __forceinline__ float sqrt_cr_grad(float x)
{
    const bool small = x < 0x1p-96f;
    const float xs = small ? __fmul_rn(x, 0x1p32f) : x;
    const float s = __builtin_amdgcn_sqrtf(xs);
    const float sdn = __int_as_float(__float_as_int(s) - 1), sup = __int_as_float(__float_as_int(s) + 1);
    float t = __fmaf_rn(-sdn, s, xs) <= 0.f ? sdn : s;
    t = __fmaf_rn(-sup, s, xs) > 0.f ? sup : t;
    return small ? __fmul_rn(t, 0x1p-16f) : t;
}

// sqrt_cr_grad for x = 0 or x >= 2^-96 (no prescale): at x = 0 the hardware
// sqrt gives 0 and neither residual test fires (the lower neighbour is NaN,
// the upper one's residual is -0), as in the full sequence
__device__ __forceinline__ float sqrt_cr_grad_big(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __int_as_float(__float_as_int(s) - 1), sup = __int_as_float(__float_as_int(s) + 1);
    float t = __fmaf_rn(-sdn, s, x) <= 0.f ? sdn : s;
    return __fmaf_rn(-sup, s, x) > 0.f ? sup : t;
}

// {magnitude, fastAtan2 orientation} of two horizontally adjacent pixels from
// their central differences (the oracle's per-pixel expressions; the paired
// lanes of the packed operations hold the two pixels)
__device__ __forceinline__ float4 grad_pair(bf2 dx, bf2 dy)
{
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const bf2 ax = {fabsf(dx.x), fabsf(dx.y)}, ay = {fabsf(dy.x), fabsf(dy.y)};
    const bf2 mn = {ax.x < ay.x ? ax.x : ay.x, ax.y < ay.y ? ax.y : ay.y};
    const bf2 mx = {ax.x < ay.x ? ay.x : ax.x, ax.y < ay.y ? ay.y : ax.y};
    const bf2 eps = {(float)DBL_EPSILON, (float)DBL_EPSILON};
    const bf2 den = mx + eps;
    const bf2 c = div_cr_grad2(mn, den);
    const bf2 cc = c * c;
    const bf2 P7 = {p7, p7}, P5 = {p5, p5}, P3 = {p3, p3}, P1 = {p1, p1};
    bf2 a = __builtin_elementwise_fma(__builtin_elementwise_fma(__builtin_elementwise_fma(cc, P7, P5), cc, P3), cc, P1);
    a = a * c;
    const bf2 k90 = {90.f, 90.f}, k180 = {180.f, 180.f}, k360 = {360.f, 360.f};
    const bf2 a90 = k90 - a;
    a.x = ax.x >= ay.x ? a.x : a90.x;
    a.y = ax.y >= ay.y ? a.y : a90.y;
    const bf2 a180 = k180 - a;
    a.x = dx.x < 0 ? a180.x : a.x;
    a.y = dx.y < 0 ? a180.y : a.y;
    const bf2 a360 = k360 - a;
    a.x = dy.x < 0 ? a360.x : a.x;
    a.y = dy.y < 0 ? a360.y : a.y;
    const bf2 m2 = __builtin_elementwise_fma(dx, dx, dy * dy);
    // the prescaled path only when some lane of the wave has 0 < m2 < 2^-96 (a
    // gradient of one ulp of the blurred values: practically never)
    const bool tiny = (m2.x > 0.f && m2.x < 0x1p-96f) || (m2.y > 0.f && m2.y < 0x1p-96f);
    if (__builtin_amdgcn_ballot_w64(tiny) == 0)
        return make_float4(sqrt_cr_grad_big(m2.x), a.x, sqrt_cr_grad_big(m2.y), a.y);
    return make_float4(sqrt_cr_grad(m2.x), a.x, sqrt_cr_grad(m2.y), a.y);
}

// Fused SIFT base layer + gradient map.  One 512-thread block per 64 x 64
// output tile: the gray tile with a 7-px REFLECT_101 halo goes to LDS, the row
// pass (RowVec_32f: fma chain from 0 over the 13 taps) and the column pass
// (SymmColumnVec_32f: S0 * k0, then fma(S[m] + S[-m], k[m], .)) run out of LDS,
// and only the float2 {magnitude, orientation} map is written to HBM -- the
// f32 row-blurred and blurred planes never leave the CU.  Same operations in
// the same order as the oracle's blur, so the map is bit-identical.  Every
// pass runs on packed f32 (v_pk_fma_f32: two outputs per lane and
// instruction): the row pass pairs two rows, the column pass and the
// gradients two adjacent columns.
template <int kOb>
__global__ __launch_bounds__(kBlurThreads) void sift_blur_grad(BlurGradParams p)
{
    // the gray tile is dead once the row pass has read it (barrier), so the
    // blurred base rows reuse its memory: 39 KB per block, 4 blocks per CU
    constexpr int kGB = kTR * kTW * 4 > kGR * kGS ? kTR * kTW * 4 : kGR * kGS;
    __shared__ __attribute__((aligned(16))) float t[kGR * kTW];
    __shared__ __attribute__((aligned(16))) uint8_t gb_mem[kGB];
    uint8_t* const g = gb_mem;
    float* const b = reinterpret_cast<float*>(gb_mem);
    // tile (bx, by) covers pixels from ((bx - 1) * 64, (by - 1) * 64): the first
    // and last tiles of a row/column lie in the zero border of the padded map
    int bx, by, f;
    xcd_tile(p.xcd != 0, bx, by, f);
    const int x0 = (bx + p.tile0 - 1) * kBT, y0 = (by + p.tile0 - 1) * kBT;
    const int tid = threadIdx.x;
    float2* G = p.grad + (size_t)f * grad_frame(p.w, p.h) + grad_origin(p.w);
    const int pitch = grad_pitch(p.w);
    // the orientation component as stored: ori, or the band kernel's obin (the
    // same two f32 operations it would apply per keypoint-sample, once per pixel)
    const float bpr = 8 / 360.f;
    auto stored = [&](float ori) { return kOb ? __fmul_rn(__fsub_rn(ori, p.ori_deg), bpr) : ori; };
    // obin 2: the stored value is fract(obin) (v_fract_f32: exact, as the band
    // kernel's own per-sample fract), the slot position goes to the byte plane
    uint8_t* const PB = p.posb + (size_t)f * grad_frame(p.w, p.h) + grad_origin(p.w);
    auto pos_byte = [](float ob) {
        int o0;
        __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));
        return (uint32_t)((o0 + 9) * 6);
    };
    if (x0 + kBT <= 0 || y0 + kBT <= 0 || x0 >= p.w || y0 >= p.h) {
        // tile outside the image: the border only
        const float o0 = stored(0.f);
        const float ov = kOb == 2 ? __builtin_amdgcn_fractf(o0) : o0;
        const uint8_t pb = kOb == 2 ? (uint8_t)pos_byte(o0) : 0;
        for (int i = tid; i < kBT * kBT; i += kBlurThreads) {
            const int x = x0 + (i & 63), y = y0 + (i >> 6);
            if (x >= -kGradPad && x < p.w + kGradPad && y >= -kGradPad && y < p.h + kGradPad) {
                G[(ptrdiff_t)y * pitch + x] = make_float2(0.f, ov);
                if (kOb == 2) PB[(ptrdiff_t)y * pitch + x] = pb;
            }
        }
        return;
    }
    const uint8_t* src = p.gray + (size_t)f * p.w * p.h;

    // gray tile with a REFLECT_101 halo; interior tiles load dwords
    const bool wide = (p.w & 3) == 0 && x0 - 8 >= 0 && x0 + 72 <= p.w && y0 - kBH >= 0 && y0 + kBT + kBH <= p.h;
    if (wide) {
        // 16 bytes per lane (rows start 8 bytes before the tile: 4-byte aligned
        // global loads, 16-byte aligned LDS rows)
        for (int i = tid; i < kGR * (kGL / 16); i += kBlurThreads) {
            const int r = i / (kGL / 16), q = i - r * (kGL / 16);
            const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)(y0 - kBH + r) * p.w + (x0 - 8 + 16 * q));
            *reinterpret_cast<uint4*>(&g[r * kGS + 16 * q]) = v;
        }
    } else {
        for (int i = tid; i < kGR * kGL; i += kBlurThreads) {
            const int r = i / kGL, c = i - r * kGL;
            const int Y = reflect101(y0 - kBH + r, p.h), X = reflect101(x0 - 8 + c, p.w);
            g[r * kGS + c] = src[(size_t)Y * p.w + X];
        }
    }
    __syncthreads();
    bf2 kk[13];
#pragma unroll
    for (int q = 0; q < 13; q++) kk[q] = bf2{p.k.gauss[q], p.k.gauss[q]};
    // row pass (RowVec_32f: fma chain from 0 over the taps): 4 adjacent outputs
    // of two rows per task; output column c (x0 - 1 + c) reads g columns
    // c + 1 .. c + 13; the packed lanes hold rows r and r + 1
    // tasks: 16 per row pair (columns 0 .. 63), then the pairs' last task (64 .. 67)
    static_assert(kTW / 4 == 17, "row-pass task split");
    for (int i = tid; i < (kGR / 2) * (kTW / 4); i += kBlurThreads) {
        const bool tail = i >= (kGR / 2) * 16;
        const int rp = tail ? i - (kGR / 2) * 16 : i >> 4, c = tail ? 64 : 4 * (i & 15), r = 2 * rp;
        const uint32_t* g0 = reinterpret_cast<const uint32_t*>(&g[r * kGS + c]);
        const uint32_t* g1 = reinterpret_cast<const uint32_t*>(&g[(r + 1) * kGS + c]);
        uint32_t w0[5], w1[5];
#pragma unroll
        for (int q = 0; q < 5; q++) {
            w0[q] = (c + 4 * q < kGL) ? g0[q] : 0u;
            w1[q] = (c + 4 * q < kGL) ? g1[q] : 0u;
        }
        bf2 px[17];
#pragma unroll
        for (int q = 1; q <= 16; q++)
            px[q] = bf2{(float)((w0[q >> 2] >> (8 * (q & 3))) & 255u), (float)((w1[q >> 2] >> (8 * (q & 3))) & 255u)};
        bf2 acc[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
#if BLUR_DIAG == 2 || BLUR_DIAG == 4
            acc[u] = px[7 + u];                                   // timing only: no row taps
#else
            bf2 a = {0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 13; q++) a = __builtin_elementwise_fma(px[1 + u + q], kk[q], a);
            acc[u] = a;
#endif
        }
        *reinterpret_cast<float4*>(&t[r * kTW + c]) = make_float4(acc[0].x, acc[1].x, acc[2].x, acc[3].x);
        *reinterpret_cast<float4*>(&t[(r + 1) * kTW + c]) = make_float4(acc[0].y, acc[1].y, acc[2].y, acc[3].y);
    }
    __syncthreads();
    // column pass (SymmColumnVec_32f: S0 * k0, then fma(S[m] + S[-m], k[m])):
    // two adjacent columns per task (the packed lanes), a sliding window over
    // kStrip outputs; base row r (y0 - 1 + r) uses t rows r .. r + 12
    for (int i = tid; i < (kTW / 2) * (kTR / kStrip); i += kBlurThreads) {
        const int c = 2 * (i % (kTW / 2)), r0 = kStrip * (i / (kTW / 2));
        bf2 win[kStrip + 12];
#pragma unroll
        for (int q = 0; q < kStrip + 12; q++) win[q] = *reinterpret_cast<const bf2*>(&t[(r0 + q) * kTW + c]);
#pragma unroll
        for (int u = 0; u < kStrip; u++) {
            bf2 acc = win[u + 6] * kk[6];
#if !(BLUR_DIAG == 2 || BLUR_DIAG == 4)
#pragma unroll
            for (int m = 1; m <= 6; m++) acc = __builtin_elementwise_fma(win[u + 6 + m] + win[u + 6 - m], kk[6 + m], acc);
#endif
            *reinterpret_cast<bf2*>(&b[(r0 + u) * kTW + c]) = acc;
        }
    }
    __syncthreads();
    // gradients of the 64 x 64 outputs (interior pixels only, as the reference),
    // two adjacent pixels per task: output (r, c) is base (r + 1, c + 1)
    const bool inner = x0 > 0 && x0 + kBT < p.w - 1 && y0 > 0 && y0 + kBT < p.h - 1;
#pragma unroll
    for (int i = tid; i < kBT * kBT / 2; i += kBlurThreads) {
        const int r = i >> 5, c = 2 * (i & 31);
        const int x = x0 + c, y = y0 + r;
        const float* row = &b[(r + 1) * kTW];
        const bf2 lf = *reinterpret_cast<const bf2*>(&row[c]);          // base columns c, c + 1
        const bf2 rt = *reinterpret_cast<const bf2*>(&row[c + 2]);      // c + 2, c + 3
        // the rows above and below as aligned 8-byte pairs (c, c + 1), (c + 2, c + 3):
        // lane k of a 32-lane group reads dwords 2k, 2k + 1 (all 64 banks once);
        // the odd-offset pair (c + 1, c + 2) was a ds_read2_b32 on odd banks only,
        // two lanes per bank
        const bf2 u0 = *reinterpret_cast<const bf2*>(&row[c - kTW]), u1 = *reinterpret_cast<const bf2*>(&row[c + 2 - kTW]);
        const bf2 d0 = *reinterpret_cast<const bf2*>(&row[c + kTW]), d1 = *reinterpret_cast<const bf2*>(&row[c + 2 + kTW]);
        const bf2 up = {u0.y, u1.x};
        const bf2 dn = {d0.y, d1.x};
#if BLUR_DIAG == 1 || BLUR_DIAG == 4
        float4 o = make_float4(rt.x - lf.x, up.x - dn.x, rt.y - lf.y, up.y - dn.y);   // timing only: no gradient math
#else
        float4 o = grad_pair(rt - lf, up - dn);
#endif
        if (!inner) {
            if (y >= p.h + kGradPad) continue;
            const bool yin = y > 0 && y < p.h - 1;
            if (!(yin && x > 0 && x < p.w - 1)) o.x = o.y = 0.f;
            if (!(yin && x + 1 > 0 && x + 1 < p.w - 1)) o.z = o.w = 0.f;
            o.y = stored(o.y);
            o.w = stored(o.w);
            if (kOb == 2) {
                const uint32_t pb = pos_byte(o.y) | pos_byte(o.w) << 8;
                o.y = __builtin_amdgcn_fractf(o.y);
                o.w = __builtin_amdgcn_fractf(o.w);
                if (x + 1 >= p.w + kGradPad) {
                    if (x < p.w + kGradPad) PB[(size_t)y * pitch + x] = (uint8_t)pb;
                } else {
                    *reinterpret_cast<uint16_t*>(&PB[(size_t)y * pitch + x]) = (uint16_t)pb;
                }
            }
            if (x + 1 >= p.w + kGradPad) {
                if (x < p.w + kGradPad) G[(size_t)y * pitch + x] = make_float2(o.x, o.y);
                continue;
            }
        } else if (kOb) {
            o.y = stored(o.y);
            o.w = stored(o.w);
            if (kOb == 2) {
                // x even, pitch and origin even: an aligned 2-byte store
                *reinterpret_cast<uint16_t*>(&PB[(size_t)y * pitch + x]) = (uint16_t)(pos_byte(o.y) | pos_byte(o.w) << 8);
                o.y = __builtin_amdgcn_fractf(o.y);
                o.w = __builtin_amdgcn_fractf(o.w);
            }
        }
#if BLUR_DIAG == 3
        if (o.x == -1.f) *reinterpret_cast<float4*>(&G[(size_t)y * pitch + x]) = o;   // timing only: no stores
#else
        *reinterpret_cast<float4*>(&G[(size_t)y * pitch + x]) = o;
#endif
    }
}

struct DescParams {
    const float2* grad;
    int w, h;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float* kp_cs;     // optional per-keypoint {cos_t, sin_t} (host cosf/sinf); else uniform
    float cos_u, sin_u;     // uniform cos/sin of (360 - angle) for angle == -1 keypoints
    uint8_t* desc_u8;
    float* desc_f32;        // optional reference-layout output
    int* norm_i8;           // sum over k of (d_k - 128)^2 (matcher side array)
    SiftConsts k;
};

constexpr int HSTRIDE = kSiftHist + 4;   // 1 guard slot in front + padding

__global__ __launch_bounds__(64) void sift_desc(DescParams p)
{
    __shared__ float hist_s[HSTRIDE];
    __shared__ float raw[128];
    // exp32f's table in LDS: lane-divergent reads of the kernel argument itself
    // go to the kernarg segment (visible after the loop's first barrier)
    __shared__ float s_exptab[64];
    float* hist = hist_s + 1;
    const int lane = threadIdx.x;
    s_exptab[lane] = p.k.exptab[lane];
    int total = *p.total;
    if (total > p.cap) total = p.cap;
    for (int g = blockIdx.x; g < total; g += gridDim.x) {
        const slam_keypoint kp = p.kps[g];
        const int f = p.kp_frame[g];
        const float2* G = p.grad + (size_t)f * grad_frame(p.w, p.h) + grad_origin(p.w);
        const int pitch = grad_pitch(p.w);

        float angle = __fsub_rn(360.f, kp.angle);
        if (fabsf(__fsub_rn(angle, 360.f)) < FLT_EPSILON) angle = 0.f;
        const float ori = angle, scl = __fmul_rn(kp.size, 0.5f);
        const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
        float cos_t = p.kp_cs ? p.kp_cs[2 * g] : p.cos_u;
        float sin_t = p.kp_cs ? p.kp_cs[2 * g + 1] : p.sin_u;
        const float bins_per_rad = 8 / 360.f;
        const float exp_scale = -1.f / (4 * 4 * 0.5f);
        const float hist_width = __fmul_rn(3.f, scl);
        int radius = __float2int_rn(__fmul_rn(__fmul_rn(__fmul_rn(hist_width, 1.4142135623730951f), 5.f), 0.5f));
        const int diag = (int)sqrt((double)p.w * p.w + (double)p.h * p.h);
        radius = min(radius, diag);
        cos_t = cr_divf(cos_t, hist_width);
        sin_t = cr_divf(sin_t, hist_width);

        for (int i = lane; i < HSTRIDE; i += 64) hist_s[i] = 0.f;
        __syncthreads();

        const int side = 2 * radius + 1, len = side * side;
        int i = lane / side, j = lane - i * side;   // window coords (offset by radius)
        for (int s = lane; s < len; s += 64) {
            const float fi = (float)(i - radius), fj = (float)(j - radius);
            const float c_rot = __fsub_rn(__fmul_rn(fj, cos_t), __fmul_rn(fi, sin_t));
            const float r_rot = __fadd_rn(__fmul_rn(fj, sin_t), __fmul_rn(fi, cos_t));
            float rbin = __fsub_rn(__fadd_rn(r_rot, 2.f), 0.5f);
            float cbin = __fsub_rn(__fadd_rn(c_rot, 2.f), 0.5f);
            const int r = pty + i - radius, c = ptx + j - radius;
            if (rbin > -1.f && rbin < 4.f && cbin > -1.f && cbin < 4.f && r > 0 && r < p.h - 1 && c > 0 &&
                c < p.w - 1) {
                const float wexp = exp32f(__fmul_rn(__fadd_rn(__fmul_rn(c_rot, c_rot), __fmul_rn(r_rot, r_rot)),
                                                    exp_scale),
                                          s_exptab);
                const size_t o = (size_t)r * pitch + c;
                const float2 mo = G[o];
                float obin = __fmul_rn(__fsub_rn(mo.y, ori), bins_per_rad);
                const float mag = __fmul_rn(mo.x, wexp);
                const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                int o0 = (int)floorf(obin);
                rbin = __fsub_rn(rbin, (float)r0);
                cbin = __fsub_rn(cbin, (float)c0);
                obin = __fsub_rn(obin, (float)o0);
                if (o0 < 0) o0 += 8;
                if (o0 >= 8) o0 -= 8;
                const float v_r1 = __fmul_rn(mag, rbin), v_r0 = __fsub_rn(mag, v_r1);
                const float v_rc11 = __fmul_rn(v_r1, cbin), v_rc10 = __fsub_rn(v_r1, v_rc11);
                const float v_rc01 = __fmul_rn(v_r0, cbin), v_rc00 = __fsub_rn(v_r0, v_rc01);
                const float v_rco111 = __fmul_rn(v_rc11, obin), v_rco110 = __fsub_rn(v_rc11, v_rco111);
                const float v_rco101 = __fmul_rn(v_rc10, obin), v_rco100 = __fsub_rn(v_rc10, v_rco101);
                const float v_rco011 = __fmul_rn(v_rc01, obin), v_rco010 = __fsub_rn(v_rc01, v_rco011);
                const float v_rco001 = __fmul_rn(v_rc00, obin), v_rco000 = __fsub_rn(v_rc00, v_rco001);
                const int idx = ((r0 + 1) * 6 + c0 + 1) * 10 + o0;
                atomicAdd(&hist[idx], v_rco000);
                atomicAdd(&hist[idx + 1], v_rco001);
                atomicAdd(&hist[idx + 10], v_rco010);
                atomicAdd(&hist[idx + 11], v_rco011);
                atomicAdd(&hist[idx + 60], v_rco100);
                atomicAdd(&hist[idx + 61], v_rco101);
                atomicAdd(&hist[idx + 70], v_rco110);
                atomicAdd(&hist[idx + 71], v_rco111);
            }
            j += 64;
            while (j >= side) { j -= side; i++; }
        }
        __syncthreads();

        // circular fold of the 4x4 inner cells, then copy out
        for (int q = lane; q < 16; q += 64) {
            const int ci = q >> 2, cj = q & 3;
            const int idx = ((ci + 1) * 6 + (cj + 1)) * 10;
            hist[idx] = __fadd_rn(hist[idx], hist[idx + 8]);
            hist[idx + 1] = __fadd_rn(hist[idx + 1], hist[idx + 9]);
        }
        __syncthreads();
        for (int k = lane; k < 128; k += 64) {
            const int cell = k >> 3, o = k & 7;
            raw[k] = hist[(((cell >> 2) + 1) * 6 + ((cell & 3) + 1)) * 10 + o];
        }
        __syncthreads();

        // first norm: 8 fma partial sums (k mod 8) + v_reduce_sum order
        float part = 0.f;
        if (lane < 8)
            for (int m = 0; m < 16; m++) { float v = raw[lane + 8 * m]; part = __fmaf_rn(v, v, part); }
        float l[8];
#pragma unroll
        for (int q = 0; q < 8; q++) l[q] = __shfl(part, q, 64);
        float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(l[0], l[4]), __fadd_rn(l[1], l[5])),
                               __fadd_rn(__fadd_rn(l[2], l[6]), __fadd_rn(l[3], l[7])));
        const float thr = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
        // clamp, then the sequential second norm (same order as the reference)
        float v0 = fminf(raw[lane], thr), v1 = fminf(raw[lane + 64], thr);
        __syncthreads();
        raw[lane] = v0;
        raw[lane + 64] = v1;
        __syncthreads();
        float n2 = 0.f;
        for (int k = 0; k < 128; k++) { float v = raw[k]; n2 = __fadd_rn(n2, __fmul_rn(v, v)); }
        const float sq = cr_sqrtf(n2);
        const float scale = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        float q0 = rintf(__fmul_rn(v0, scale)), q1 = rintf(__fmul_rn(v1, scale));
        q0 = fminf(fmaxf(q0, 0.f), 255.f);
        q1 = fminf(fmaxf(q1, 0.f), 255.f);
        uint8_t* du = p.desc_u8 + (size_t)g * 128;
        du[lane] = (uint8_t)q0;
        du[lane + 64] = (uint8_t)q1;
        if (p.desc_f32) {
            p.desc_f32[(size_t)g * 128 + lane] = q0;
            p.desc_f32[(size_t)g * 128 + lane + 64] = q1;
        }
        int a0 = (int)q0 - 128, a1 = (int)q1 - 128;
        int nsum = a0 * a0 + a1 * a1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nsum += __shfl_xor(nsum, o, 64);
        if (lane == 0) p.norm_i8[g] = nsum;
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_sift_base(slam_ctx* c, hipStream_t s, int nframes, int w, int h, int obin, float ori_deg)
{
    hipError_t e;
    if ((e = c->grad.ensure((size_t)nframes * grad_frame(w, h) * 8)) != hipSuccess) return e;
    if (c->sift.ksize != 13) return hipErrorInvalidValue;     // the tile halo is sized for 13 taps
    BlurGradParams b;
    b.gray = c->gray.as<uint8_t>(); b.grad = c->grad.as<float2>(); b.w = w; b.h = h; b.k = c->sift;
    b.obin = obin;
    b.ori_deg = obin ? ori_deg : 0.f;
    b.posb = nullptr;
    if (obin == 2) {
        if ((e = c->gradpos.ensure((size_t)nframes * grad_frame(w, h))) != hipSuccess) return e;
        b.posb = c->gradpos.as<uint8_t>();
    }
    static_assert(kGradPad <= kBT, "one border tile on each side");
    // The zero border outside the image never changes: once a launch has written
    // it for this buffer, geometry and frame count, later launches run only the
    // tiles that meet the image (1080p: 510 of 608 tiles per frame, 12 % fewer
    // bytes written).  The tiles at the image edge still write their share of it.
    SiftGradBorder& gb = c->grad_border;
    // (the border's orientation component depends on the stored form: same form, same border)
    const bool same = gb.p == c->grad.p && gb.bytes == c->grad.bytes && gb.w == w && gb.h == h &&
                      gb.obin == b.obin && gb.ori_deg == b.ori_deg &&
                      (obin != 2 || (gb.pp == c->gradpos.p && gb.pbytes == c->gradpos.bytes));
    const bool skip = same && nframes <= gb.frames;
    b.tile0 = skip ? 1 : 0;
    b.xcd = xcd_tiles_on() ? 1 : 0;
    dim3 grid = skip ? dim3((w + kBT - 1) / kBT, (h + kBT - 1) / kBT, nframes)
                     : dim3((w + kGradPad + kBT - 1) / kBT + 1, (h + kGradPad + kBT - 1) / kBT + 1, nframes);
    prof_begin(c, 4, s);
    if (obin == 2) hipLaunchKernelGGL(sift_blur_grad<2>, grid, dim3(kBlurThreads), 0, s, b);
    else if (obin) hipLaunchKernelGGL(sift_blur_grad<1>, grid, dim3(kBlurThreads), 0, s, b);
    else hipLaunchKernelGGL(sift_blur_grad<0>, grid, dim3(kBlurThreads), 0, s, b);
    prof_end(c, 4, s);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (!skip) {
        gb.frames = same && gb.frames > nframes ? gb.frames : nframes;
        gb.p = c->grad.p;
        gb.bytes = c->grad.bytes;
        gb.w = w;
        gb.h = h;
        gb.obin = b.obin;
        gb.ori_deg = b.ori_deg;
        gb.pp = c->gradpos.p;
        gb.pbytes = c->gradpos.bytes;
    }
    return hipSuccess;
}

hipError_t launch_sift_desc(slam_ctx* c, hipStream_t s, int nframes, int w, int h, const float* d_kp_cs,
                            int cap, int write_f32)
{
    (void)nframes;
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    DescParams p;
    p.grad = c->grad.as<float2>(); p.w = w; p.h = h;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap; p.kp_cs = d_kp_cs;
    // FAST keypoints: angle -1 -> ori 361 degrees (not wrapped), host cosf/sinf
    const float ori = 361.f;
    p.cos_u = cosf(ori * (float)(M_PI / 180));
    p.sin_u = sinf(ori * (float)(M_PI / 180));
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    p.k = c->sift;
    int grid = cap < 65536 ? cap : 65536;
    if (grid < 1) grid = 1;
    prof_begin(c, 1, s);
    hipLaunchKernelGGL(sift_desc, dim3(grid), dim3(64), 0, s, p);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
