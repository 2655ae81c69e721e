// SIFT descriptors of keypoints sharing one angle and size (FAST: -1 deg, 7 px):
// keypoint-per-lane scatter over LDS-staged band chunks.
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) adds every window sample into the 8 bins of
// the 2 x 2 x 2 histogram cells around it, in raster sample order; each bin's
// float additions must happen in that order for bit-exact descriptors.
//
// Here one lane owns one keypoint and walks the window samples itself, so the
// order is the reference's by construction and every sample is processed once
// (the per-target gather of sift_tab.hip evaluates each sample four times and
// gathers it with one scattered load per lane and visit).  All keypoints share
// the sample geometry, so at every step the 64 lanes of a wave visit the SAME
// window sample of 64 keypoints: its rotated bin fractions and target cells
// are wave-uniform scalar loads, only {magnitude, orientation} differ per lane.
//
//  * Stage.  Gathering one sample of 64 keypoints is 64 unrelated cache lines
//    per instruction (texture-path bound).  Instead, per chunk of 16 window
//    samples, 16 lanes load 16 consecutive samples of one keypoint (4
//    keypoints per instruction, coalesced row segments), multiply in the
//    Gaussian weight, form obin, and stage {mag * w, obin} in LDS; the walk
//    then reads its own keypoint's record (conflict-free stride).
//  * Bands.  Samples are walked band by band: band b = source cell row
//    r0 = floor(rbin) in -1..3, raster order inside a band.  A target row R
//    receives only from bands R - 2 (dr = 1) and R - 1 (dr = 0), so only two
//    target rows of 5 cells x 10 bins are live per lane (the slot sets A, B);
//    after band b row R = b + 1 is complete and moves to registers.  The band
//    order equals the raster order for every target when no row holds a later
//    band's samples left of an earlier band's (the small FAST rotation:
//    361 deg); the host checks this per target and refuses the table
//    otherwise (sift_tab then runs).
//  * Slots.  Lane-private, slot-major (bin * 64 + lane): the read-add-write
//    of a data-dependent orientation bin is bank-conflict free.
//
// The epilogue (norm, clamp, renormalise, saturate) runs per lane on the
// register copy of the histogram with the reference's operation order.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kKS = 16;                 // window samples per staged chunk
constexpr int kStride = kKS + 1;        // float2 per keypoint in the stage
constexpr int kWaves = 8;
constexpr int kKpW = 32;                // keypoints per wave; lane = keypoint + 32 * dr
constexpr int kPos = 10;                // slot positions: 0 = left cell's slot 9, 1..9 = slots 0..8
constexpr int kCols = 5;                // target columns C = 1..5 (C = 5: the 361-degree quirk column)
constexpr int kSet = kCols * kPos * kKpW;   // floats per slot set (one target row of 32 keypoints)
constexpr int kJunk = 2 * kSet;             // junk column (column 0, outside the descriptor)
constexpr int kStageOff = kJunk + kPos * kKpW;
constexpr int kKpOff = kStageOff + kKpW * kStride * 2;
constexpr int kWaveFloats = kKpOff + kKpW * 4;
constexpr int kMaxChunks = 1024;
constexpr int kRawStride = 129;          // epilogue: one keypoint per lane, odd stride = conflict-free
static_assert(kKpW * kRawStride <= kKpOff, "epilogue raw buffer must fit below the keypoint info");

struct BandParams {
    const float2* grad;
    int w, h;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float4* smp;                  // [nchunks * kKS] band-sorted {rf, cf, w, (i & 255) | (j & 255) << 8 | (c0 + 1) << 16}
    int nchunks;
    int band_first[6];                  // first chunk of band b at band_first[b + 1]
    float ori_deg;
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

typedef const __attribute__((address_space(4))) float ctabf;   // scalar-loaded sample table

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

template <bool kNeg, int kMode>
__global__ __launch_bounds__(64 * kWaves) void sift_desc_band(BandParams p)
{
    __shared__ float s_buf[kWaves][kWaveFloats];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kq = lane & 31, dr = lane >> 5;     // keypoint of the wave, target-row half (dr)
    float* buf = s_buf[wave];
    float2* stg = reinterpret_cast<float2*>(buf + kStageOff);
    int4* kpi = reinterpret_cast<int4*>(buf + kKpOff);
    float* slotk = buf + kq;                       // + set * kSet + (col * kPos + pos) * 32
    const float bins_per_rad = 8 / 360.f;
    const float ori_deg = p.ori_deg;
    const int W = p.w, H = p.h;
    ctabf* tabc = (ctabf*)p.smp;
    const float4* tabv = p.smp;

    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int ngroups = (total + kKpW - 1) / kKpW;
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so the
    // keypoint groups are split into 8 contiguous ranges, one per XCD group
    // (blockIdx % 8): each XCD walks a compact raster band whose windows overlap
    const int xg = blockIdx.x & 7;
    const int nw = (gridDim.x >> 3) * kWaves, wi = (blockIdx.x >> 3) * kWaves + wave;
    const int per = (ngroups + 7) >> 3;
    const int grp_end = min(ngroups, (xg + 1) * per);
    const int nch = p.nchunks;
    // stage mapping: lane loads sample ss of keypoint kPer * it + kl
    constexpr int kPer = 64 / kKS, kIt = kKpW / kPer;
    const int ss = lane % kKS, kl = lane / kKS;
    for (int grp = xg * per + wi; grp < grp_end; grp += nw) {
        const int g = grp * kKpW + kq;
        const bool act = g < total;
        if (dr == 0) {
            const int gg = min(g, total - 1);
            const slam_keypoint kp = p.kps[gg];
            const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
            const long long boff = (long long)p.kp_frame[gg] * W * H + (long long)pty * W + ptx;
            kpi[kq] = make_int4((int)boff, (int)(boff >> 32), ptx - 1, pty - 1);
        }
#pragma unroll 10
        for (int q = 0; q < kSet / 32; q++) buf[q * 64 + lane] = 0.f;   // both slot sets
        wave_sync();

        // ---- prefetch of one chunk: kIt x kPer keypoints x kKS consecutive window samples ----
        struct Pre { float2 v[kIt]; float w; };
        auto issue = [&](int ch, Pre& pf) __attribute__((always_inline)) {
            const float4 sm = tabv[ch * kKS + ss];
            pf.w = sm.z;
            const int bits = __float_as_int(sm.w);
            const int si = (int)(int8_t)(bits & 0xff), sj = (int)(int8_t)((bits >> 8) & 0xff);
            const long long soff = (long long)si * W + sj;
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const int4 ki = kpi[kPer * it + kl];
                const long long b = (long long)(((unsigned long long)(unsigned)ki.y << 32) | (unsigned)ki.x);
                // reference: 0 < r < rows - 1 and 0 < c < cols - 1
                const bool in = (unsigned)(ki.w + si) < (unsigned)(H - 2) && (unsigned)(ki.z + sj) < (unsigned)(W - 2);
                if (kMode == 2) pf.v[it] = make_float2((float)(ki.w & 7), (float)sj);
                else pf.v[it] = in ? p.grad[b + soff] : make_float2(0.f, 0.f);   // outside: contributes +0
            }
        };
        auto stage = [&](const Pre& pf) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const float mw = __fmul_rn(pf.v[it].x, pf.w);
                const float ob = __fmul_rn(__fsub_rn(pf.v[it].y, ori_deg), bins_per_rad);
                stg[(kPer * it + kl) * kStride + ss] = make_float2(mw, ob);
            }
        };

        float raw[4][2][8];             // this lane's half of the histogram: rows 1..4, columns 2 dr, 2 dr + 1
        int band = -1;
        bool live = dr == 1;            // band -1: the dr = 1 lanes add into row 1, the dr = 0 lanes' row 0 is outside
        float* tset = slotk + kSet;     // row (band + 1 + dr) & 1
        // ---- walk one staged chunk, then close the band when it was the band's last ----
        auto process = [&](int ch) __attribute__((always_inline)) {
            if (kMode != 1 && live) {
                // the chunk's records and wave-uniform table entries up front
                float2 r[kKS];
                float rf[kKS], cf[kKS];
                int c0[kKS];
#pragma unroll
                for (int q = 0; q < kKS; q++) {
                    r[q] = stg[kq * kStride + q];
                    rf[q] = tabc[4 * (ch * kKS + q)];
                    cf[q] = tabc[4 * (ch * kKS + q) + 1];
                    c0[q] = ((__float_as_int(tabc[4 * (ch * kKS + q) + 3]) >> 16) & 0xff) - 1;
                }
                // all values and slot addresses first (VALU only), then the kKS
                // read-add-write steps back to back: each step's chain is one LDS
                // round trip with no arithmetic waiting behind it
                float w0[kKS], w1[kKS], u0[kKS], u1[kKS];
                float* t1p[kKS];
#pragma unroll
                for (int q = 0; q < kKS; q++) {
                    const float o0f = floorf(r[q].y);
                    const float frac = __fsub_rn(r[q].y, o0f);
                    int o0 = (int)o0f;
                    int pos;
                    if (kNeg) {
                        pos = o0 + 9;                   // o0 in [-9, -1] -> wrapped o0 + 1
                    } else {
                        o0 += o0 < 0 ? 8 : 0;
                        o0 -= o0 >= 8 ? 8 : 0;
                        pos = o0 + 1;
                    }
                    const float v_r1 = __fmul_rn(r[q].x, rf[q]);
                    const float v_r0 = __fsub_rn(r[q].x, v_r1);
                    const float vr = dr ? v_r1 : v_r0;
                    const float vc1 = __fmul_rn(vr, cf[q]), vc0 = __fsub_rn(vr, vc1);
                    w1[q] = __fmul_rn(vc0, frac);
                    w0[q] = __fsub_rn(vc0, w1[q]);
                    u1[q] = __fmul_rn(vc1, frac);
                    u0[q] = __fsub_rn(vc1, u1[q]);
                    t1p[q] = tset + (c0[q] + 1) * (kPos * 32) + pos * 32;
                }
#pragma unroll
                for (int q = 0; q < kKS; q++) {
                    // dc = 1 -> column c0 + 1; dc = 0 -> column c0 (none when c0 = -1: wave-uniform)
                    float* t1 = t1p[q];
                    if (c0[q] >= 0) {
                        float* t0 = t1 - kPos * 32;
                        const float a0 = t0[0], a1 = t0[32], b0 = t1[0], b1 = t1[32];
                        t0[0] = __fadd_rn(a0, w0[q]);
                        t0[32] = __fadd_rn(a1, w1[q]);
                        t1[0] = __fadd_rn(b0, u0[q]);
                        t1[32] = __fadd_rn(b1, u1[q]);
                    } else {
                        const float b0 = t1[0], b1 = t1[32];
                        t1[0] = __fadd_rn(b0, u0[q]);
                        t1[32] = __fadd_rn(b1, u1[q]);
                    }
                }
            }
            wave_sync();
            if (ch + 1 == p.band_first[band + 2]) {
                // ---- row band + 1 complete (the dr = 0 lanes' row): fold, keep, reset ----
                if (band >= 0) {
                    const int Rd = band + 1;
                    float* a = slotk + (Rd & 1) * kSet;
                    float f[2][8];
#pragma unroll
                    for (int k2 = 0; k2 < 2; k2++) {
                        const float* c = a + (2 * dr + k2) * kPos * 32;   // column index 2 dr + k2
                        f[k2][0] = __fadd_rn(c[1 * 32], c[9 * 32]);
                        f[k2][1] = __fadd_rn(c[2 * 32], c[kPos * 32]);  // + slot 9 = position 0 of the next column
#pragma unroll
                        for (int q = 2; q < 8; q++) f[k2][q] = c[(q + 1) * 32];
                    }
                    // static register indices (a uniform select per row; an if-chain is
                    // merged by the compiler into one dynamically indexed scratch store)
#pragma unroll
                    for (int rr = 0; rr < 4; rr++)
#pragma unroll
                        for (int k2 = 0; k2 < 2; k2++)
#pragma unroll
                            for (int q = 0; q < 8; q++) raw[rr][k2][q] = Rd == rr + 1 ? f[k2][q] : raw[rr][k2][q];
                    wave_sync();
                    // reset the set: it holds row band + 3 (the dr = 1 lanes' row in band + 1)
                    float* z = buf + (Rd & 1) * kSet;
#pragma unroll 5
                    for (int q = 0; q < kSet / 64; q++) z[q * 64 + lane] = 0.f;
                    wave_sync();
                }
                band++;
                const int R = band + 1 + dr;    // this lane's target row in the new band
                live = R >= 1 && R <= 4;
                tset = slotk + (R & 1) * kSet;
            }
        };

        // the next chunk's loads are in flight while this one is walked (a second
        // chunk in flight measured slower: 3.07 vs 2.92 ms)
        Pre pf;
        issue(0, pf);
        stage(pf);
        wave_sync();
        for (int ch = 0; ch < nch; ch++) {
            if (ch + 1 < nch) issue(ch + 1, pf);
            process(ch);
            if (ch + 1 < nch) {
                stage(pf);
                wave_sync();
            }
        }

        // ---- epilogue: raw histogram to LDS, one lane per keypoint ----
        wave_sync();
        {
            float* rb = buf + kq * kRawStride;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++)
#pragma unroll
                    for (int q = 0; q < 8; q++) rb[(r * 4 + 2 * dr + k2) * 8 + q] = raw[r][k2][q];
        }
        wave_sync();
        if (dr == 0) {
            float* rb = buf + kq * kRawStride;
            float chain[8];
#pragma unroll
            for (int q = 0; q < 8; q++) chain[q] = 0.f;
#pragma unroll
            for (int k = 0; k < 128; k++) chain[k & 7] = __fmaf_rn(rb[k], rb[k], chain[k & 7]);
            const float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(chain[0], chain[4]), __fadd_rn(chain[1], chain[5])),
                                         __fadd_rn(__fadd_rn(chain[2], chain[6]), __fadd_rn(chain[3], chain[7])));
            const float thr = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
            float n2 = 0.f;
#pragma unroll 16
            for (int k = 0; k < 128; k++) {
                const float x = fminf(rb[k], thr);
                rb[k] = x;
                n2 = __fadd_rn(n2, __fmul_rn(x, x));
            }
            const float sq = cr_sqrtf(n2);
            const float sc = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
            if (act) {
                int ns = 0;
#pragma unroll 2
                for (int c = 0; c < 8; c++) {
                    uint32_t wd[4];
#pragma unroll
                    for (int wq = 0; wq < 4; wq++) {
                        uint32_t word = 0;
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            const int k = c * 16 + wq * 4 + b;
                            float x = rintf(__fmul_rn(rb[k], sc));
                            x = fminf(fmaxf(x, 0.f), 255.f);
                            const int iv = (int)x;
                            word |= (uint32_t)iv << (8 * b);
                            ns += (iv - 128) * (iv - 128);
                            rb[k] = x;
                        }
                        wd[wq] = word;
                    }
                    *reinterpret_cast<uint4*>(p.desc_u8 + (size_t)g * 128 + c * 16) =
                        make_uint4(wd[0], wd[1], wd[2], wd[3]);
                }
                p.norm_i8[g] = ns;
                if (p.desc_f32) {
                    float4* o = reinterpret_cast<float4*>(p.desc_f32 + (size_t)g * 128);
#pragma unroll 8
                    for (int c = 0; c < 32; c++) o[c] = make_float4(rb[4 * c], rb[4 * c + 1], rb[4 * c + 2], rb[4 * c + 3]);
                }
            }
        }
        wave_sync();
    }
}

}  // namespace

// Build (or reuse) the band tables for keypoints of one (angle, size); false
// when the band order does not reproduce some target's raster order or the
// tables do not fit (sift_tab / the general kernel then run).
bool sift_band_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h)
{
    if (const char* ev = getenv("SLAMHIP_SIFT_KERNEL"))
        if (std::strcmp(ev, "band") != 0) return false;
    float angle = 360.f - kp_angle;
    if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    const float ori = angle, scl = kp_size * 0.5f;
    float cos_t = cosf(ori * (float)(M_PI / 180));
    float sin_t = sinf(ori * (float)(M_PI / 180));
    const float exp_scale = -1.f / (4 * 4 * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = (int)std::lrintf(hist_width * 1.4142135623730951f * (4 + 1) * 0.5f);
    const int diag = (int)std::sqrt((double)w * w + (double)h * h);
    if (radius > diag || radius > 127 || w < 3 || h < 3) return false;
    if (c->sift_band_valid && c->sift_band_angle == kp_angle && c->sift_band_size == kp_size &&
        c->sift_band.radius == radius)
        return true;
    cos_t /= hist_width;
    sin_t /= hist_width;
    struct Smp { int i, j, r0, c0; float rf, cf, wexp; };
    std::vector<Smp> smp;   // raster order (the reference's)
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(4 / 2) - 0.5f;
            const float cbin = c_rot + (float)(4 / 2) - 0.5f;
            if (!(rbin > -1 && rbin < 4 && cbin > -1 && cbin < 4)) continue;
            const float wexp = host_exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, c->sift.exptab);
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            smp.push_back({i, j, r0, c0, rbin - (float)r0, cbin - (float)c0, wexp});
        }
    const int n = (int)smp.size();
    // band-major order (stable by r0)
    std::vector<int> ord(n);
    for (int k = 0; k < n; k++) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return smp[a].r0 < smp[b].r0; });
    // every target's visit sequence must be the same in band-major and raster order
    for (int R = 1; R <= 4; R++)
        for (int C = 1; C <= 5; C++) {
            std::vector<int> ras, bm;
            auto hits = [&](const Smp& q) {
                const int dr = R - 1 - q.r0, dc = C - 1 - q.c0;
                return dr >= 0 && dr <= 1 && dc >= 0 && dc <= 1;
            };
            for (int k = 0; k < n; k++) if (hits(smp[k])) ras.push_back(k);
            for (int k = 0; k < n; k++) if (hits(smp[ord[k]])) bm.push_back(ord[k]);
            if (ras != bm) return false;
        }
    // obin = (ori_k - ori) * 8/360 over ori_k in [0, 360] (fastAtan2's range):
    // kNeg when floor(obin) always lies in [-9, -1] (one wrap, no branch)
    const float bpr = 8 / 360.f;
    const float ob_lo = (0.f - ori) * bpr, ob_hi = (360.f - ori) * bpr;
    const bool neg = std::floor(ob_lo) >= -9.f && std::floor(ob_hi) <= -1.f;
    // chunks of kKS consecutive band-major samples of one band; each band is
    // padded to a multiple of kKS with zero-weight samples at the keypoint
    // (they add +0, which leaves every bin unchanged)
    std::vector<int2> chunks;
    std::vector<float4> tab;
    int band_first[6];
    int k = 0;
    for (int b = -1; b <= 3; b++) {
        band_first[b + 1] = (int)chunks.size();
        int end = k;
        while (end < n && smp[ord[end]].r0 == b) end++;
        for (int q = k; q < end; q++) {
            const Smp& sm = smp[ord[q]];
            union { int32_t i; float f; } u;
            u.i = (sm.i & 255) | ((sm.j & 255) << 8) | ((sm.c0 + 1) << 16);
            if ((int)(tab.size() % kKS) == 0) chunks.push_back(make_int2((int)tab.size(), kKS));
            tab.push_back(make_float4(sm.rf, sm.cf, sm.wexp, u.f));
        }
        union { int32_t i; float f; } z;
        z.i = 1 << 16;   // (i, j) = (0, 0), c0 = 0
        while (tab.size() % kKS) tab.push_back(make_float4(0.f, 0.f, 0.f, z.f));
        k = end;
    }
    band_first[5] = (int)chunks.size();
    if (k != n || (int)chunks.size() > kMaxChunks) return false;
    const size_t b_tab = tab.size() * sizeof(float4);
    if (c->sift_band_buf.ensure(b_tab) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_band_buf.p, tab.data(), b_tab, hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    SiftBandMeta& m = c->sift_band;
    m.nrec = (int)tab.size();
    m.nchunks = (int)chunks.size();
    m.neg = neg;
    for (int q = 0; q < 6; q++) m.band_first[q] = band_first[q];
    m.radius = radius;
    m.ori_deg = ori;
    c->sift_band_valid = true;
    c->sift_band_angle = kp_angle;
    c->sift_band_size = kp_size;
    return true;
}

hipError_t launch_sift_desc_band(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    const SiftBandMeta& m = c->sift_band;
    BandParams p;
    p.grad = c->grad.as<float2>(); p.w = w; p.h = h;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.smp = c->sift_band_buf.as<float4>();
    p.nchunks = m.nchunks;
    for (int q = 0; q < 6; q++) p.band_first[q] = m.band_first[q];
    p.ori_deg = m.ori_deg;
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    // persistent: one 8-wave workgroup per CU (145 KB of LDS), a multiple of 8
    // workgroups for the XCD split
    int grid = c->cu_count;
    if (const char* ev = getenv("SLAMHIP_SIFT_GRID")) grid = atoi(ev);
    const int need = (cap + kKpW * kWaves - 1) / (kKpW * kWaves);
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    prof_begin(c, 1, s);
    int mode = 0;
    if (const char* ev = getenv("SLAMHIP_SIFT_BAND_MODE")) mode = atoi(ev);   // timing experiments only
    if (mode == 1)
        hipLaunchKernelGGL((sift_desc_band<true, 1>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (mode == 2)
        hipLaunchKernelGGL((sift_desc_band<true, 2>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (m.neg)
        hipLaunchKernelGGL((sift_desc_band<true, 0>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else
        hipLaunchKernelGGL((sift_desc_band<false, 0>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
