// SIFT descriptors, keypoint-per-lane formulation (keypoints sharing one angle
// and size -- every FAST keypoint: angle -1, size 7).
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) walks the window samples in raster order and
// adds each one's trilinear weights into up to 8 histogram bins.  Because the
// sample geometry (rotated bin coordinates, trilinear fractions, exp32f weight,
// which 2 x 2 cells a sample reaches) is the same for every keypoint of one
// (angle, size), it is a wave-uniform table built once on the host with the
// reference's float operation order, and:
//
//  - one lane owns one keypoint: a wave describes 64 keypoints, all lanes walk
//    the same sample sequence in the reference's raster order, so every
//    histogram bin receives its contributions in exactly the reference's
//    order -> bit-identical descriptors;
//  - table reads are wave-uniform (scalar loads) and the cells a sample feeds
//    are uniform (scalar branches), so no lane does another lane's work;
//  - each (keypoint, sample) gradient pair is gathered once (16-byte loads of
//    two horizontally adjacent samples where the raster run allows): about a
//    quarter of the bytes of the per-target-cell gather (sift_tab.hip), whose
//    scattered 8-16 B loads saturated the texture-data return path;
//  - the histogram lives in LDS, slot-major (position * 64 + lane), so the
//    per-lane read-modify-write at a data-dependent slot is bank-conflict free;
//    a 128-thread workgroup describes 64 keypoints: wave 0 owns histogram rows
//    R = 1, 2 and wave 1 rows R = 3, 4 (8 cells x 10 slots = 20 KB each: slots
//    0..8 + slot 9 fed by the 361-degree quirk, see oracle/sift.c), each walking
//    only the samples that reach its rows -> 8 waves per CU;
//  - a sample's kept corners (1, 2 or 4, wave-uniform) issue all their LDS
//    reads before the adds and writes (distinct bins, see lk_apply);
//  - the two normalisation passes continue across the two waves in the
//    reference's order (fma chains over k = q + 8m, then the sequential
//    clamped sum), handed over through the folded-away slots 8/9.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kBandPos = 80;            // 8 cells x 10 slots per keypoint and band
constexpr int kLkDepth = 8;             // items gathered ahead

struct LkItem {                         // 64 bytes, read with wave-uniform (scalar) loads
    float rf[2], cf[2], w[2];           // trilinear fractions and exp32f weight of the 1-2 samples
    int i, j;                           // first sample offset (row, col) from the keypoint
    uint32_t cw[2][2];                  // per sample, kept corners in order, 16 bits each:
                                        // pos (slot 0 of the band-local cell) | type << 8 | q << 10
                                        // type 0: C = 2..4, 1: C = 1, 2: C = 5; q = 2 dr + dc
    int n;                              // samples in the item (1 or 2)
    int nc[2];                          // kept corners per sample (0..4)
    int pad;
};
static_assert(sizeof(LkItem) == 64, "LkItem layout");

struct LkParams {
    const float2* grad;
    int w, h;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    int nitems[2], radius;
    float ori_deg;
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

__device__ __forceinline__ float& H(float* hb, int pos, int lane) { return hb[pos * 64 + lane]; }

template <bool kCheck>
__device__ __forceinline__ float4 lk_gather(const LkParams& p, const LkItem& it, const float2* P, int ptx, int pty)
{
    const int off = it.i * p.w + it.j;
    if (kCheck) {
        const int rr = pty + it.i, cc = ptx + it.j;
        const bool rin = (unsigned)(rr - 1) < (unsigned)(p.h - 2);
        const bool in0 = rin && (unsigned)(cc - 1) < (unsigned)(p.w - 2);
        const bool in1 = rin && (unsigned)(cc) < (unsigned)(p.w - 2);
        float2 a = P[in0 ? off : 0], b = P[in1 ? off + 1 : 0];
        if (!in0) a.x = 0.f;               // sample outside [1, w-2] x [1, h-2]: contributes +0
        if (!in1) b.x = 0.f;
        return make_float4(a.x, a.y, b.x, b.y);
    }
    const float2* q = P + off;             // interior keypoint: (i, j + 1) is inside the image
    const float2 a = q[0], b = q[1];
    return make_float4(a.x, a.y, b.x, b.y);
}

// Add one sample's kept corners.  Corner c targets cell (R, C); with pp = o0 + 1:
//   C = 2..4: v0 -> slot pp - 1 (pp = 0: slot 9 of (R, C - 1), the position
//             just before), v1 -> slot pp: one adjacent pair;
//   C = 1:    v0 is dropped when pp = 0 (it belongs to the discarded cell
//             (R, 0)): the pair becomes (slot 0, slot 1) += (v1, +0);
//   C = 5:    only v0 with pp = 0 survives, into slot 9 of (R, 4): single add.
// The pairs of one sample's corners are distinct bins, so all reads are issued
// before the writes.
template <int NC>
__device__ __forceinline__ void lk_apply(float* hb, int lane, int pp, const float cv[4], float obin, uint32_t cwa,
                                         uint32_t cwb)
{
    int a[NC];
    float x0[NC], x1[NC];
    bool single[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t code = (c < 2 ? (cwa >> (16 * c)) : (cwb >> (16 * (c - 2)))) & 0xffffu;
        const int pos = code & 127, type = (code >> 8) & 3, q = (code >> 10) & 3;
        const float v = q == 0 ? cv[0] : (q == 1 ? cv[1] : (q == 2 ? cv[2] : cv[3]));
        const float v1 = __fmul_rn(v, obin), v0 = __fsub_rn(v, v1);
        single[c] = type == 2;
        if (type == 0) {
            a[c] = pos + pp - 1; x0[c] = v0; x1[c] = v1;
        } else if (type == 1) {
            const bool z = pp == 0;
            a[c] = z ? pos : pos + pp - 1; x0[c] = z ? v1 : v0; x1[c] = z ? 0.f : v1;
        } else {
            a[c] = pos + 9; x0[c] = pp == 0 ? v0 : 0.f; x1[c] = 0.f;
        }
    }
    float r0[NC], r1[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        r0[c] = H(hb, a[c], lane);
        if (!single[c]) r1[c] = H(hb, a[c] + 1, lane);
    }
#pragma unroll
    for (int c = 0; c < NC; c++) {
        H(hb, a[c], lane) = __fadd_rn(r0[c], x0[c]);
        if (!single[c]) H(hb, a[c] + 1, lane) = __fadd_rn(r1[c], x1[c]);
    }
}

__device__ __forceinline__ void lk_sample(float* hb, int lane, float mo_m, float mo_o, float w, float rf, float cf,
                                          uint32_t cwa, uint32_t cwb, int nc, float ori_deg)
{
    if (nc == 0) return;                   // wave-uniform
    const float bins_per_rad = 8 / 360.f;
    float obin = __fmul_rn(__fsub_rn(mo_o, ori_deg), bins_per_rad);
    const float mag = __fmul_rn(mo_m, w);
    int o0 = (int)floorf(obin);
    obin = __fsub_rn(obin, (float)o0);
    o0 += o0 < 0 ? 8 : 0;
    o0 -= o0 >= 8 ? 8 : 0;
    const int pp = o0 + 1;
    const float v_r1 = __fmul_rn(mag, rf), v_r0 = __fsub_rn(mag, v_r1);
    const float v_rc11 = __fmul_rn(v_r1, cf), v_rc10 = __fsub_rn(v_r1, v_rc11);
    const float v_rc01 = __fmul_rn(v_r0, cf), v_rc00 = __fsub_rn(v_r0, v_rc01);
    const float cv[4] = {v_rc00, v_rc01, v_rc10, v_rc11};
    switch (nc) {                          // wave-uniform
        case 1: lk_apply<1>(hb, lane, pp, cv, obin, cwa, cwb); break;
        case 2: lk_apply<2>(hb, lane, pp, cv, obin, cwa, cwb); break;
        case 3: lk_apply<3>(hb, lane, pp, cv, obin, cwa, cwb); break;
        default: lk_apply<4>(hb, lane, pp, cv, obin, cwa, cwb); break;
    }
}

template <bool kCheck>
__device__ __forceinline__ void lk_walk(const LkParams& p, const LkItem* __restrict__ T, int nitems, const float2* P,
                                        int ptx, int pty, float* hb, int lane)
{
    float4 g[kLkDepth];
#pragma unroll
    for (int d = 0; d < kLkDepth; d++) g[d] = lk_gather<kCheck>(p, T[d], P, ptx, pty);
    for (int it = 0; it < nitems; it += kLkDepth) {
#pragma unroll
        for (int d = 0; d < kLkDepth; d++) {
            const float4 cur = g[d];
            g[d] = lk_gather<kCheck>(p, T[it + d + kLkDepth], P, ptx, pty);   // table padded by kLkDepth
            const LkItem& I = T[it + d];
            lk_sample(hb, lane, cur.x, cur.y, I.w[0], I.rf[0], I.cf[0], I.cw[0][0], I.cw[0][1], I.nc[0], p.ori_deg);
            if (I.n > 1)
                lk_sample(hb, lane, cur.z, cur.w, I.w[1], I.rf[1], I.cf[1], I.cw[1][0], I.cw[1][1], I.nc[1],
                          p.ori_deg);
        }
    }
}

__global__ __launch_bounds__(128) void sift_desc_lk(LkParams p, const LkItem* __restrict__ items0,
                                                   const LkItem* __restrict__ items1)
{
    __shared__ float hist[2][kBandPos * 64];
    // wave-uniform band (readfirstlane: the compiler then keeps the item table
    // pointer and trip count scalar -> s_load of the items)
    const int band = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    float* hb = hist[band];
    float* h0 = hist[0];
    float* h1 = hist[1];
    const LkItem* __restrict__ T = band ? items1 : items0;
    const int nitems = p.nitems[band];
    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int rad = p.radius;
    // XCD-aware order: groups of 64 keypoints split into 8 contiguous ranges,
    // one per XCD group (blockIdx % 8), so an XCD's L2 serves overlapping windows
    const int ngroups = (total + 63) / 64;
    const int xg = blockIdx.x & 7, nx = gridDim.x >> 3;
    const int per = (ngroups + 7) >> 3;
    const int gend = min(ngroups, (xg + 1) * per);
    for (int gi = xg * per + (blockIdx.x >> 3); gi < gend; gi += nx) {
        const int g = gi * 64 + lane;
        const bool act = g < total;
        int ptx = p.w / 2, pty = p.h / 2;
        size_t fo = 0;
        if (act) {
            const slam_keypoint kp = p.kps[g];
            ptx = __float2int_rn(kp.x);
            pty = __float2int_rn(kp.y);
            fo = (size_t)p.kp_frame[g] * p.w * p.h;
        }
        for (int q = 0; q < kBandPos; q++) H(hb, q, lane) = 0.f;
        const float2* P = p.grad + fo + (size_t)pty * p.w + ptx;
        const bool interior = ptx - rad >= 1 && ptx + rad <= p.w - 2 && pty - rad >= 1 && pty + rad <= p.h - 2;
        if (__all(interior)) lk_walk<false>(p, T, nitems, P, ptx, pty, hb, lane);
        else lk_walk<true>(p, T, nitems, P, ptx, pty, hb, lane);

        // circular fold (slot 0 += slot 8, slot 1 += slot 9) of this band's 8 cells
#pragma unroll
        for (int c = 0; c < 8; c++) {
            float& s0 = H(hb, c * 10 + 0, lane);
            float& s1 = H(hb, c * 10 + 1, lane);
            s0 = __fadd_rn(s0, H(hb, c * 10 + 8, lane));
            s1 = __fadd_rn(s1, H(hb, c * 10 + 9, lane));
        }
        // element k of this band's half: cell k >> 3, slot k & 7 (k = 0..63)
        auto raw = [&](const float* hh, int k) -> float { return H((float*)hh, (k >> 3) * 10 + (k & 7), lane); };
        // hand-over positions (slots 8 / 9 are free after the fold)
        auto xpos = [](int i) -> int { return (i >> 1) * 10 + 8 + (i & 1); };

        // first norm: 8 fma chains over k = q + 8m; wave 0 runs m = 0..7, wave 1 m = 8..15
        float l[8];
        if (band == 0) {
#pragma unroll
            for (int q = 0; q < 8; q++) l[q] = 0.f;
            for (int m = 0; m < 8; m++) {
#pragma unroll
                for (int q = 0; q < 8; q++) { const float v = raw(h0, q + 8 * m); l[q] = __fmaf_rn(v, v, l[q]); }
            }
#pragma unroll
            for (int q = 0; q < 8; q++) H(h0, xpos(q), lane) = l[q];
        }
        __syncthreads();
        if (band == 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) l[q] = H(h0, xpos(q), lane);
            for (int m = 0; m < 8; m++) {
#pragma unroll
                for (int q = 0; q < 8; q++) { const float v = raw(h1, q + 8 * m); l[q] = __fmaf_rn(v, v, l[q]); }
            }
            const float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(l[0], l[4]), __fadd_rn(l[1], l[5])),
                                         __fadd_rn(__fadd_rn(l[2], l[6]), __fadd_rn(l[3], l[7])));
            H(h1, xpos(0), lane) = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
        }
        __syncthreads();
        const float thr = H(h1, xpos(0), lane);
        // clamp + sequential second norm: wave 0 sums k = 0..63, wave 1 continues
        if (band == 0) {
            float n2 = 0.f;
            for (int k = 0; k < 64; k++) {
                const float v = fminf(raw(h0, k), thr);
                n2 = __fadd_rn(n2, __fmul_rn(v, v));
            }
            H(h0, xpos(8), lane) = n2;
        }
        __syncthreads();
        if (band == 1) {
            float n2 = H(h0, xpos(8), lane);
            for (int k = 0; k < 64; k++) {
                const float v = fminf(raw(h1, k), thr);
                n2 = __fadd_rn(n2, __fmul_rn(v, v));
            }
            const float sq = cr_sqrtf(n2);
            H(h1, xpos(1), lane) = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        }
        __syncthreads();
        const float sc = H(h1, xpos(1), lane);
        int ns = 0;
        for (int c = 0; c < 8; c++) {
            uint32_t wd[2] = {0, 0};
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                float v = rintf(__fmul_rn(fminf(raw(hb, c * 8 + kk), thr), sc));
                v = fminf(fmaxf(v, 0.f), 255.f);
                const int iv = (int)v;
                wd[kk >> 2] |= (uint32_t)iv << (8 * (kk & 3));
                ns += (iv - 128) * (iv - 128);
                if (act && p.desc_f32) p.desc_f32[(size_t)g * 128 + band * 64 + c * 8 + kk] = v;
            }
            if (act)
                *reinterpret_cast<uint2*>(p.desc_u8 + (size_t)g * 128 + band * 64 + c * 8) = make_uint2(wd[0], wd[1]);
        }
        if (band == 0) H(h0, xpos(9), lane) = __int_as_float(ns);
        __syncthreads();
        if (band == 1 && act) p.norm_i8[g] = ns + __float_as_int(H(h0, xpos(9), lane));
        __syncthreads();                    // the histograms are reset for the next group
    }
}

}  // namespace

// Build (or reuse) the two band item tables for keypoints of one (angle,
// size); false when the window does not fit the int8 offsets (the caller then
// uses another descriptor kernel).
bool sift_lk_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h)
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
    if (radius > diag || radius > 120) return false;
    if (c->sift_lk_valid && c->sift_lk_angle == kp_angle && c->sift_lk_size == kp_size) return true;
    cos_t /= hist_width;
    sin_t /= hist_width;
    struct Smp { int i, j; float rf, cf, w; uint32_t cw[2]; int nc; };
    std::vector<Smp> smp[2];
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(4 / 2) - 0.5f;
            const float cbin = c_rot + (float)(4 / 2) - 0.5f;
            if (!(rbin > -1 && rbin < 4 && cbin > -1 && cbin < 4)) continue;
            const float wexp = host_exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, c->sift.exptab);
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            for (int band = 0; band < 2; band++) {
                Smp sm;
                std::memset(&sm, 0, sizeof(sm));
                sm.i = i; sm.j = j; sm.rf = rbin - (float)r0; sm.cf = cbin - (float)c0; sm.w = wexp;
                for (int dr = 0; dr < 2; dr++)
                    for (int dc = 0; dc < 2; dc++) {
                        const int R = r0 + 1 + dr, C = c0 + 1 + dc, q = 2 * dr + dc;
                        if (R < 2 * band + 1 || R > 2 * band + 2 || C < 1 || C > 5) continue;
                        const int rl = R - 2 * band - 1;
                        const int pos = (rl * 4 + (C <= 4 ? C - 1 : 3)) * 10;
                        const int type = C == 1 ? 1 : (C == 5 ? 2 : 0);
                        const uint32_t code = (uint32_t)pos | (uint32_t)type << 8 | (uint32_t)q << 10;
                        sm.cw[sm.nc >> 1] |= code << (16 * (sm.nc & 1));
                        sm.nc++;
                    }
                if (sm.nc) smp[band].push_back(sm);
            }
        }
    // items: a sample and its right neighbour when the band's raster run continues
    std::vector<LkItem> items[2];
    for (int band = 0; band < 2; band++) {
        const auto& S = smp[band];
        for (size_t k = 0; k < S.size();) {
            LkItem it;
            std::memset(&it, 0, sizeof(it));
            const Smp& a = S[k];
            it.i = a.i; it.j = a.j; it.n = 1;
            it.rf[0] = a.rf; it.cf[0] = a.cf; it.w[0] = a.w;
            it.cw[0][0] = a.cw[0]; it.cw[0][1] = a.cw[1]; it.nc[0] = a.nc;
            if (k + 1 < S.size() && S[k + 1].i == a.i && S[k + 1].j == a.j + 1) {
                const Smp& b = S[k + 1];
                it.n = 2;
                it.rf[1] = b.rf; it.cf[1] = b.cf; it.w[1] = b.w;
                it.cw[1][0] = b.cw[0]; it.cw[1][1] = b.cw[1]; it.nc[1] = b.nc;
                k += 2;
            } else {
                k += 1;
            }
            items[band].push_back(it);
        }
    }
    // pad both tables to a common multiple of the prefetch depth, plus the
    // prefetch overrun: items with no kept corner touch nothing
    LkItem pad;
    std::memset(&pad, 0, sizeof(pad));
    pad.n = 1;
    int nit[2];
    for (int band = 0; band < 2; band++) {
        nit[band] = (int)((items[band].size() + kLkDepth - 1) / kLkDepth * kLkDepth);
        items[band].resize(nit[band] + kLkDepth, pad);
    }
    const size_t b0 = items[0].size() * sizeof(LkItem), b1 = items[1].size() * sizeof(LkItem);
    if (c->sift_lk.ensure(b0 + b1) != hipSuccess) return false;
    std::vector<uint8_t> blob(b0 + b1);
    std::memcpy(blob.data(), items[0].data(), b0);
    std::memcpy(blob.data() + b0, items[1].data(), b1);
    if (hipMemcpyAsync(c->sift_lk.p, blob.data(), blob.size(), hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    c->sift_lk_nitems = nit[0];
    c->sift_lk_nitems1 = nit[1];
    c->sift_lk_radius = radius;
    c->sift_lk_ori = ori;
    c->sift_lk_valid = true;
    c->sift_lk_angle = kp_angle;
    c->sift_lk_size = kp_size;
    return true;
}

hipError_t launch_sift_desc_lk(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    LkParams p;
    p.grad = c->grad.as<float2>(); p.w = w; p.h = h;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.nitems[0] = c->sift_lk_nitems;
    p.nitems[1] = c->sift_lk_nitems1;
    p.radius = c->sift_lk_radius;
    p.ori_deg = c->sift_lk_ori;
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    const LkItem* it0 = c->sift_lk.as<LkItem>();
    const LkItem* it1 = it0 + c->sift_lk_nitems + kLkDepth;
    // two-wave workgroups, 4 per CU (40 KB LDS each), grid-stride over groups of
    // 64 keypoints; a multiple of 8 workgroups for the XCD split
    int grid = 4 * c->cu_count;
    if (const char* ev = getenv("SLAMHIP_SIFT_LK_GRID")) grid = atoi(ev);
    const int need = (cap + 63) / 64;
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    prof_begin(c, 1, s);
    hipLaunchKernelGGL(sift_desc_lk, dim3(grid), dim3(128), 0, s, p, it0, it1);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
