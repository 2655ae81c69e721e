// SIFT descriptors, gather formulation (keypoints sharing one angle and size).
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) scatters every window sample into 8 histogram
// bins.  For FAST keypoints all angles are -1 deg and all sizes 7 px, so the
// sample geometry -- rotated bin coordinates, trilinear split, exp32f Gaussian
// weight -- is one fixed table per launch.  The table is reorganised per TARGET
// histogram cell: for each of the 20 cells that reach the descriptor (16 inner
// cells + the 4 column-5 cells whose o0 = -1 weight lands in column 4, see the
// 361-degree quirk in oracle/sift.c) it lists, in the reference's raster
// sample order, the samples that contribute and which corner of their 2 x 2
// cell footprint the target is.
//
// One lane owns one target cell (20 lanes per keypoint, 3 keypoints per
// one-wave workgroup) and accumulates into lane-private LDS slots, so every bin
// receives its contributions in exactly the reference's order and the
// descriptors are bit-identical to the oracle.  Slot layout per lane:
// position 0 = slot 9 of the cell to the left (the o0 = -1 quirk), positions
// 1..9 = slots 0..8, so a sample always adds v0 at o0 + 1 and v1 at o0 + 2
// (one ds_read2 / ds_write2 pair, no branch).  Padding entries carry weight 0:
// adding +0 to a non-negative partial sum is exact.
//
// Latency hiding: no barriers in the sample loop; the table rows (16 B per
// lane, L2-resident, identical for every keypoint) are loaded two batches
// ahead and the {mag, ori} samples one batch ahead, in registers.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kTargets = 20;            // lanes per keypoint
constexpr int kKpPerWave = 3;
constexpr int kSlotStride = 11;         // 10 positions + pad (odd stride)
constexpr int kU = 4;                   // entries per pipeline batch

struct TabEntry {                       // 16 bytes
    int8_t i, j;                        // sample offset (row, col) from the keypoint
    uint8_t pad0, pad1;
    float rf, cf, w;                    // rbin - r0 (sign bit: dr), cbin - c0 (sign bit: dc), exp32f weight
};

struct TabParams {
    const float2* grad;
    int w, h;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const TabEntry* tab;                // [len + 2 kU][kTargets]
    SiftTabMeta meta;
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

template <bool kCheck>
__device__ __forceinline__ void tab_walk(const TabParams& p, const TabEntry* e, const float2* P, int ptx,
                                         int pty, float* my)
{
    const float bins_per_rad = 8 / 360.f;
    const float ori_deg = p.meta.ori_deg;
    const int w = p.w, h = p.h;
    auto gather = [&](const TabEntry& te) -> float2 {
        int off = (int)te.i * w + (int)te.j;
        if (kCheck) {
            const int r = pty + te.i, c = ptx + te.j;
            const bool inb = (unsigned)(r - 1) < (unsigned)(h - 2) && (unsigned)(c - 1) < (unsigned)(w - 2);
            off = inb ? off : 0;
            float2 v = P[off];
            if (!inb) v.x = 0.f;           // sample outside the image: contributes +0
            return v;
        }
        return P[off];
    };
    TabEntry ec[kU], en[kU], e2[kU];
    float2 gc[kU], gn[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) ec[u] = e[u * kTargets];
#pragma unroll
    for (int u = 0; u < kU; u++) gc[u] = gather(ec[u]);
#pragma unroll
    for (int u = 0; u < kU; u++) en[u] = e[(kU + u) * kTargets];
    const int len = p.meta.len;
    for (int m = 0; m < len; m += kU) {
        const TabEntry* e_next2 = e + (size_t)(m + 2 * kU) * kTargets;   // table padded by 2 kU rows
#pragma unroll
        for (int u = 0; u < kU; u++) e2[u] = e_next2[u * kTargets];
#pragma unroll
        for (int u = 0; u < kU; u++) gn[u] = gather(en[u]);
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const TabEntry& te = ec[u];
            const float2 mo = gc[u];
            float obin = __fmul_rn(__fsub_rn(mo.y, ori_deg), bins_per_rad);
            const float mag = __fmul_rn(mo.x, te.w);
            int o0 = (int)floorf(obin);
            obin = __fsub_rn(obin, (float)o0);
            o0 += o0 < 0 ? 8 : 0;
            o0 -= o0 >= 8 ? 8 : 0;
            const float v_r1 = __fmul_rn(mag, fabsf(te.rf));
            const float br = __float_as_int(te.rf) < 0 ? v_r1 : __fsub_rn(mag, v_r1);
            const float v_c1 = __fmul_rn(br, fabsf(te.cf));
            const float v = __float_as_int(te.cf) < 0 ? v_c1 : __fsub_rn(br, v_c1);
            const float v1 = __fmul_rn(v, obin);
            const float v0 = __fsub_rn(v, v1);
            float* sp = my + o0 + 1;
            const float a0 = sp[0], a1 = sp[1];
            sp[0] = __fadd_rn(a0, v0);
            sp[1] = __fadd_rn(a1, v1);
        }
#pragma unroll
        for (int u = 0; u < kU; u++) { ec[u] = en[u]; gc[u] = gn[u]; en[u] = e2[u]; }
    }
}

__global__ __launch_bounds__(64) void sift_desc_tab(TabParams p)
{
    __shared__ float slots[64 * kSlotStride];
    __shared__ float raw[kKpPerWave][128];
    __shared__ float scal[kKpPerWave];
    __shared__ float part[kKpPerWave][8];
    __shared__ int nrm[kKpPerWave][kTargets];

    const int lane = threadIdx.x;
    const int ks = lane / kTargets, t = lane - ks * kTargets;   // keypoint slot (3 = idle lanes), target cell
    int total = *p.total;
    if (total > p.cap) total = p.cap;
    float* my = &slots[lane * kSlotStride];
    const int R = 1 + t / 5, C = 1 + t % 5;                     // target cell (R, C), C = 5: quirk only
    const int rad = p.meta.radius;
    const TabEntry* e = p.tab + t;

    for (int base = blockIdx.x * kKpPerWave; base < total; base += gridDim.x * kKpPerWave) {
        const int g = base + ks;
        const bool act = ks < kKpPerWave && g < total;
#pragma unroll
        for (int s = 0; s < 10; s++) my[s] = 0.f;
        int ptx = p.w / 2, pty = p.h / 2;
        size_t fo = 0;
        if (act) {
            const slam_keypoint kp = p.kps[g];
            ptx = __float2int_rn(kp.x);
            pty = __float2int_rn(kp.y);
            fo = (size_t)p.kp_frame[g] * p.w * p.h;
        }
        const float2* P = p.grad + fo + (size_t)pty * p.w + ptx;
        const bool interior = ptx - rad >= 1 && ptx + rad <= p.w - 2 && pty - rad >= 1 && pty + rad <= p.h - 2;
        if (__all(interior))
            tab_walk<false>(p, e, P, ptx, pty, my);
        else
            tab_walk<true>(p, e, P, ptx, pty, my);
        __syncthreads();
        // fold (slot0 += slot8, slot1 += slot9 of the same memory cell) for the 16 inner cells
        if (act && C <= 4) {
            const float* nxt = &slots[(lane + 1) * kSlotStride];   // lane of cell (R, C + 1)
            float* rw = &raw[ks][((R - 1) * 4 + (C - 1)) * 8];
            rw[0] = __fadd_rn(my[1], my[9]);
            rw[1] = __fadd_rn(my[2], nxt[0]);
#pragma unroll
            for (int q = 2; q < 8; q++) rw[q] = my[q + 1];
        }
        __syncthreads();
        // first norm: 8 fma chains over k = q + 8m (one lane each), then the
        // v_reduce_sum order; clamp + sequential second norm on one lane
        if (act && t < 8) {
            const float* rw = raw[ks];
            float a = 0.f;
#pragma unroll 4
            for (int m = 0; m < 16; m++) { const float v = rw[t + 8 * m]; a = __fmaf_rn(v, v, a); }
            part[ks][t] = a;
        }
        __syncthreads();
        if (act && t == 0) {
            float* rw = raw[ks];
            const float* l = part[ks];
            const float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(l[0], l[4]), __fadd_rn(l[1], l[5])),
                                         __fadd_rn(__fadd_rn(l[2], l[6]), __fadd_rn(l[3], l[7])));
            const float thr = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
            float n2 = 0.f;
#pragma unroll 4
            for (int k = 0; k < 128; k++) {
                const float v = fminf(rw[k], thr);
                rw[k] = v;
                n2 = __fadd_rn(n2, __fmul_rn(v, v));
            }
            const float sq = cr_sqrtf(n2);
            scal[ks] = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        }
        __syncthreads();
        if (act && C <= 4) {
            const int cell = (R - 1) * 4 + (C - 1);
            const float sc = scal[ks];
            const float* rw = &raw[ks][cell * 8];
            uint8_t* du = p.desc_u8 + (size_t)g * 128 + cell * 8;
            int ns = 0;
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                float v = rintf(__fmul_rn(rw[q], sc));
                v = fminf(fmaxf(v, 0.f), 255.f);
                const int iv = (int)v;
                if (q < 4) lo |= (uint32_t)iv << (8 * q);
                else hi |= (uint32_t)iv << (8 * (q - 4));
                ns += (iv - 128) * (iv - 128);
                if (p.desc_f32) p.desc_f32[(size_t)g * 128 + cell * 8 + q] = v;
            }
            *reinterpret_cast<uint2*>(du) = make_uint2(lo, hi);
            nrm[ks][t] = ns;
        }
        __syncthreads();
        if (act && t == 0) {
            int s = 0;
            for (int q = 0; q < kTargets; q++)
                if (q % 5 != 4) s += nrm[ks][q];
            p.norm_i8[g] = s;
        }
        __syncthreads();
    }
}

// host replica of hal::exp32f (identical operations to oracle/sift.c)
float exp32f_host(float x, const float* tab)
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
    xf = xf * (float)exp_prescale;
    int xi = (int)std::lrintf(xf);
    xf = (xf - (float)xi) * (float)(1. / 64);
    float yf = tab[xi & 63];
    int t = (xi >> 6) + 127;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    union { int32_t i; float f; } u;
    u.i = t << 23;
    yf = yf * u.f;
    float z = xf + A1;
    z = std::fma(z, xf, A2);
    z = std::fma(z, xf, A3);
    z = std::fma(z, xf, A4);
    return z * yf;
}

}  // namespace

// Build (or reuse) the per-target table for keypoints of one (angle, size);
// false when the gather path does not apply (radius clipped by a tiny image).
bool sift_tab_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h)
{
    float angle = 360.f - kp_angle;
    if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    const float ori = angle, scl = kp_size * 0.5f;
    float cos_t = cosf(ori * (float)(M_PI / 180));
    float sin_t = sinf(ori * (float)(M_PI / 180));
    const float exp_scale = -1.f / (4 * 4 * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = (int)std::lrintf(hist_width * 1.4142135623730951f * (4 + 1) * 0.5f);
    const int diag = (int)std::sqrt((double)w * w + (double)h * h);
    if (radius > diag || radius > 127) return false;
    if (c->sift_tab_valid && c->sift_tab_angle == kp_angle && c->sift_tab_size == kp_size) return true;
    cos_t /= hist_width;
    sin_t /= hist_width;
    std::vector<std::vector<TabEntry>> lists(kTargets);
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(4 / 2) - 0.5f;
            const float cbin = c_rot + (float)(4 / 2) - 0.5f;
            if (!(rbin > -1 && rbin < 4 && cbin > -1 && cbin < 4)) continue;
            const float wexp = exp32f_host((c_rot * c_rot + r_rot * r_rot) * exp_scale, c->sift.exptab);
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            const float rf = rbin - (float)r0, cf = cbin - (float)c0;
            for (int dr = 0; dr < 2; dr++)
                for (int dc = 0; dc < 2; dc++) {
                    const int R = r0 + 1 + dr, C = c0 + 1 + dc;
                    if (R < 1 || R > 4 || C < 1 || C > 5) continue;
                    TabEntry e;
                    e.i = (int8_t)i; e.j = (int8_t)j; e.pad0 = e.pad1 = 0;
                    e.rf = dr ? -rf : rf;      // sign bit carries the corner (exact: fabsf restores it)
                    e.cf = dc ? -cf : cf;
                    if (dr && rf == 0.f) e.rf = -0.f;
                    if (dc && cf == 0.f) e.cf = -0.f;
                    e.w = wexp;
                    lists[(R - 1) * 5 + (C - 1)].push_back(e);
                }
        }
    size_t mx = 0;
    for (const auto& l : lists) mx = std::max(mx, l.size());
    const int len = (int)((mx + kU - 1) / kU * kU);
    SiftTabMeta m;
    std::memset(&m, 0, sizeof(m));
    m.len = len;
    m.radius = radius;
    m.ori_deg = ori;
    // [row][target]; padding rows (and 2 kU prefetch rows) are weight-0 samples at the keypoint
    std::vector<TabEntry> flat((size_t)(len + 2 * kU) * kTargets);
    std::memset(flat.data(), 0, flat.size() * sizeof(TabEntry));
    for (int t = 0; t < kTargets; t++)
        for (size_t k = 0; k < lists[t].size(); k++) flat[k * kTargets + t] = lists[t][k];
    if (c->sift_tab.ensure(flat.size() * sizeof(TabEntry)) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_tab.p, flat.data(), flat.size() * sizeof(TabEntry), hipMemcpyHostToDevice, s) !=
        hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    c->sift_meta = m;
    c->sift_tab_valid = true;
    c->sift_tab_angle = kp_angle;
    c->sift_tab_size = kp_size;
    return true;
}

hipError_t launch_sift_desc_tab(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    TabParams p;
    p.grad = c->grad.as<float2>(); p.w = w; p.h = h;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap; p.tab = c->sift_tab.as<TabEntry>(); p.meta = c->sift_meta;
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    // one-wave workgroups, grid-stride over keypoint triples: ~10 waves per SIMD
    int grid = (cap + kKpPerWave - 1) / kKpPerWave;
    if (grid > 10240) grid = 10240;
    if (grid < 1) grid = 1;
    prof_begin(c, 1, s);
    hipLaunchKernelGGL(sift_desc_tab, dim3(grid), dim3(64), 0, s, p);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
