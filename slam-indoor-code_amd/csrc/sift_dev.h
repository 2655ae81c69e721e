// SIFT device helpers shared by sift.hip (descriptors on FAST keypoints) and
// siftdet.hip (the full detector): REFLECT_101 indexing, hal::fastAtan2 and
// hal::exp32f in OpenCV's SIMD operation order (oracle/sift.c restates both).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "slamhip_internal.h"

namespace slamhip {
namespace sd {

__device__ inline int reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// hal::fastAtan2, v_atan_f32 form (degrees)
__device__ inline float fast_atan2_deg(float y, float x)
{
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = fabsf(x), ay = fabsf(y);
    float mn = ax < ay ? ax : ay, mx = ax < ay ? ay : ax;
    float c = cr_divf(mn, __fadd_rn(mx, (float)DBL_EPSILON));
    float cc = __fmul_rn(c, c);
    float a = __fmul_rn(__fmaf_rn(__fmaf_rn(__fmaf_rn(cc, p7, p5), cc, p3), cc, p1), c);
    if (!(ax >= ay)) a = __fsub_rn(90.f, a);
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

// hal::exp32f, SIMD form
__device__ inline float exp32f(float x, const float* tab)
{
    const double exp_prescale = 1.4426950408889634073599246810019 * 64;
    const double exp_max_val = 3000. * 64;
    const float A4 = (float)(1.000000000000002438532970795181890933776 / .9670371139572337719125840413672004409288e-2);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / .9670371139572337719125840413672004409288e-2);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / .9670371139572337719125840413672004409288e-2);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / .9670371139572337719125840413672004409288e-2);
    const float minval = (float)(-exp_max_val / exp_prescale);
    const float maxval = (float)(exp_max_val / exp_prescale);
    float xf = x < minval ? minval : x;
    xf = xf > maxval ? maxval : xf;
    xf = __fmul_rn(xf, (float)exp_prescale);
    int xi = __float2int_rn(xf);
    xf = __fmul_rn(__fsub_rn(xf, (float)xi), (float)(1. / 64));
    float yf = tab[xi & 63];
    int t = (xi >> 6) + 127;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    yf = __fmul_rn(yf, __int_as_float(t << 23));
    float z = __fadd_rn(xf, A1);
    z = __fmaf_rn(z, xf, A2);
    z = __fmaf_rn(z, xf, A3);
    z = __fmaf_rn(z, xf, A4);
    return __fmul_rn(z, yf);
}

}  // namespace sd
}  // namespace slamhip
