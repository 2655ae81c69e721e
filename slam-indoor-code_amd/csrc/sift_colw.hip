// SIFT descriptors of FAST keypoints (one angle and size): one descriptor
// column per wave.
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) adds every window sample into the 8 bins of
// the 2 x 2 x 2 histogram cells around it, in raster sample order; each bin's
// float additions must happen in that order for bit-exact descriptors.
//
// sift_desc_band (sift_band.hip) walks every window sample on two lanes per
// keypoint, one per footprint column (c0, c0 + 1).  A fifth of the samples
// have c0 = -1 and a fifth c0 = 3: one of their two columns lies outside the
// descriptor (column -1; column 4, of which only position 0 -- the 361-degree
// quirk slot, column 3's slot 9 -- is read), yet its lane does the whole
// read-add-write, because the lanes of a wave must step together.  Here a wave
// owns ONE descriptor column C of 64 keypoints (lane = keypoint) and walks
// only the samples that reach it: c0 = C - 1 (its share is the right one,
// v * cbin) and c0 = C (the left one, v - v * cbin).  The share is selected
// per sample by the sign of the table's cbin: p = v * (+-cbin) (exact
// negation), cv = fma(v, km, p) with km = 0 (right: p) or 1 (left: v - v * cbin,
// one rounding as the reference's v_rc0 = v_r - v_rc1; km from the sign bit
// by two scalar instructions) -- so the walk has no branch.  Every lane step is one
// column's two read-add-write pairs, the band kernel's per-lane work, but a
// keypoint-sample costs 1.6 lane steps instead of 2.  Column 3's wave also
// keeps column 4's position 0 for its c0 = 3 samples in a register per row
// (a select and an fma by km: +0 for every other sample, exact).
//
// The four column waves of a keypoint group are in one workgroup.  After the
// walk they leave their rows in LDS (the group's own slot / stage memory, dead
// by then), and the column-0 wave folds each column's slot 9 (the next
// column's position 0, one addition as the reference's fold) and runs the
// epilogue (norm, clamp, renormalise, saturate) in the reference's order.
//
// Per wave: slots pos * 128 + 2 * lane + row (the band's row pair {r0, r0 + 1}
// as one ds_read_b64 / ds_write_b64; banks 2 * lane (+1): conflict-free for
// any data-dependent position), the stage (kKS window samples of the 64
// keypoints of this column's list), the keypoints' window offsets.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

#ifndef SIFT_COLW_KS
#define SIFT_COLW_KS 16
#endif
#ifndef SIFT_COLW_GROUPS
#define SIFT_COLW_GROUPS 2
#endif
constexpr int kKS = SIFT_COLW_KS;          // window samples per staged chunk
constexpr int kGroups = SIFT_COLW_GROUPS;  // keypoint groups per workgroup
#ifndef SIFT_COLW_BATCH
#define SIFT_COLW_BATCH SIFT_COLW_KS
#endif
constexpr int kB = SIFT_COLW_BATCH;        // samples per walk batch (values in registers)
static_assert(kKS % kB == 0 && kB % 2 == 0, "whole batches of sample pairs");
#ifndef SIFT_COLW_ONEROW
#define SIFT_COLW_ONEROW 1
#endif
constexpr bool kOneRow = SIFT_COLW_ONEROW;  // bands -1 and 3 in the one-row layout
#ifndef SIFT_COLW_PIPE
#define SIFT_COLW_PIPE 0
#endif
constexpr int kWaves = 4 * kGroups;        // wave = 4 * group + column
constexpr int kStride = 2 * kKS + 4;       // stage floats per keypoint (16-byte rows, b128 conflict-free)
constexpr int kKpW = 64;                   // keypoints per wave: lane = keypoint
constexpr int kPos = 10;                   // slot positions: 0 = the left cell's slot 9, 1..9 = slots 0..8
constexpr int kPosF = 2 * kKpW;            // floats per position: 64 lanes x 2 rows
constexpr int kSlots = kPos * kPosF;
constexpr int kStageOff = kSlots;
constexpr int kKpOff = kStageOff;         // the keypoints' window offsets: read into registers before the first stage
constexpr int kWaveFloats = kStageOff + kKpW * kStride;
constexpr int kXStride = 129;              // exchange: one keypoint's 128 bins per row, odd stride
constexpr int kX0Off = kKpW * kXStride;    // then per keypoint the 3 x 4 slot-9 values (16 floats)
constexpr int kXchFloats = kX0Off + kKpW * 16;
constexpr int kTabDw = 2 * kKS;            // per chunk: rf, signed cf (negative: the left share)
constexpr int kMaxChunks = 2048;
constexpr int kPosBase = 9;                // position = floor(obin) + 9 (floor(obin) in [-9, -1])
static_assert(kWaves * kWaveFloats * 4 <= 160 * 1024, "LDS");
static_assert(4 * kWaveFloats >= kXchFloats, "a group's exchange fits its four waves' memory");
static_assert(kStageOff % 4 == 0 && kStride % 4 == 0 && kWaveFloats % 4 == 0, "16-byte stage rows");

struct ColwParams {
    const char* grad;                      // padded gradient map (bytes), obin form
    size_t frame_bytes, origin_bytes;
    int pitch_bytes;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float2* smp;                     // [nchunks * kKS] {weight, window byte offset}
    const int* smp_s;                      // [nchunks][kTabDw]: rf, signed cf
    const int* chunk_left;                 // [nchunks]: the chunk holds a left share (cf < 0)
    int nchunks;
    int band_first[4][6];                  // column c, band b: first chunk at band_first[c][b + 1]
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) volatile f2v lds_f2v;

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

template <bool kQuirk>
__device__ __forceinline__ void colw_walk(const ColwParams& p, int C, int lane, float* buf, const unsigned* kof,
                                          float (&raw)[4][8], float (&p0)[4])
{
    float* stg = buf + kStageOff;
    constexpr int kPairs = kKS / 2, kPer = 64 / kPairs, kIt = kKpW / kPer;
    const int s2 = lane % kPairs, kl = lane / kPairs;
    char* lb = reinterpret_cast<char*>(buf + 2 * lane) + kPosBase * kPosF * 4;   // position 9 of slot pair 0
    const float4* smp4 = reinterpret_cast<const float4*>(p.smp);
    const int cbeg = p.band_first[C][0], cend = p.band_first[C][5];
    f2v quirk = {0.f, 0.f};   // column 4's position 0 for the band's row pair (column 3's wave)

#pragma unroll
    for (int q = 0; q < kSlots / 256; q++)
        *reinterpret_cast<float4*>(buf + (q * 64 + lane) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);

    struct Pre { float2 v[2 * kIt]; float wa, wb; };
    float4 smn = smp4[cbeg * kPairs + s2];
    auto issue = [&](int ch, Pre& pf) __attribute__((always_inline)) {
        const float4 sm = smn;
        pf.wa = sm.x;
        pf.wb = sm.z;
        const unsigned soa = (unsigned)__float_as_int(sm.y), sob = (unsigned)__float_as_int(sm.w);
#pragma unroll
        for (int it = 0; it < kIt; it++) {   // zero border: no bounds test
            pf.v[2 * it] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + soa));
            pf.v[2 * it + 1] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + sob));
        }
        smn = smp4[min(ch + 1, cend - 1) * kPairs + s2];
    };
    auto stage = [&](const Pre& pf) __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < kIt; it++) {
            // {mw_a, ob_a, mw_b, ob_b}: each pixel's pair stored from its own load
            // registers (a {mw_a, mw_b, ob_a, ob_b} record made the compiler copy the
            // loaded halves together right after the loads -- waiting for them there
            // and losing the prefetch)
            const float2 a = pf.v[2 * it], b = pf.v[2 * it + 1];
            float* row = stg + (kPer * it + kl) * kStride + 4 * s2;
            *reinterpret_cast<float2*>(row) = make_float2(__fmul_rn(a.x, pf.wa), a.y);
            *reinterpret_cast<float2*>(row + 2) = make_float2(__fmul_rn(b.x, pf.wb), b.y);
        }
    };
    auto walk = [&](int ch, auto Q) __attribute__((always_inline)) {
        constexpr bool kQ = decltype(Q)::value;   // a chunk of column 3 with left shares (column 4's quirk slot)
#if SIFT_COLW_KS == 16
        i16v trf, tcf;
        __asm__ volatile(
            "s_load_dwordx16 %0, %2, 0x0\n\t"
            "s_load_dwordx16 %1, %2, 0x40\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(trf), "=&s"(tcf)
            : "s"(p.smp_s + ch * kTabDw));
#else
        static_assert(kKS == 8, "chunk size");
        i8v trf, tcf;
        __asm__ volatile(
            "s_load_dwordx8 %0, %2, 0x0\n\t"
            "s_load_dwordx8 %1, %2, 0x20\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(trf), "=&s"(tcf)
            : "s"(p.smp_s + ch * kTabDw));
#endif
        // batches of kB samples (register budget): every value and slot address of
        // the batch first (VALU only), then its read-add-writes
#pragma unroll
        for (int b0 = 0; b0 < kKS; b0 += kB) {
        f4v r2[kB / 2];
#pragma unroll
        for (int q = 0; q < kB / 2; q++)
            r2[q] = *(const __attribute__((address_space(3))) volatile f4v*)(stg + lane * kStride + 2 * b0 + 4 * q);
        f2v lo[kB], hi[kB];
        char* tp[kB];
#pragma unroll
        for (int qb = 0; qb < kB; qb++) {
            const int q = b0 + qb;
            const float mw = (qb & 1) ? r2[qb >> 1].z : r2[qb >> 1].x;
            const float ob = (qb & 1) ? r2[qb >> 1].w : r2[qb >> 1].y;
            // frac = ob - floor(ob) exactly (sift_band.hip: ob never rounds up to 1)
            const float frac = __builtin_amdgcn_fractf(ob);
            int o0;
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));   // floor in [-9, -1]
            tp[qb] = lb + __mul24(o0, kPosF * 4);
            const float v_r1 = __fmul_rn(mw, __int_as_float(trf[q]));
            const f2v vr = {__fsub_rn(mw, v_r1), v_r1};                 // rows r0, r0 + 1
            const f2v cf2 = {__int_as_float(tcf[q]), __int_as_float(tcf[q])};
            // km = 1.0 for a left share (the sign bit of the table's cbin), else +0
            const float km = __int_as_float((tcf[q] >> 31) & 0x3f800000);
            const f2v km2 = {km, km};
            const f2v pc = vr * cf2;                                    // +-(v * cbin), exact sign
            // this wave's column: v * cbin (km 0) or v - v * cbin (km 1): one rounding
            const f2v cv = __builtin_elementwise_fma(vr, km2, pc);
            const f2v fr = {frac, frac};
            hi[qb] = cv * fr;                                           // bins o0 + 1
            lo[qb] = cv - hi[qb];                                       // bins o0
            if constexpr (kQ) {
                // column 4 = c0 + 1 of the c0 = 3 samples (km = 1, pc = -v * cbin): its
                // position 0 (o0 = -9, the lo share) is column 3's slot 9
                const f2v c4 = -pc;
                const f2v h4 = c4 * fr, l4 = c4 - h4;
                const f2v z = {0.f, 0.f};
                quirk = __builtin_elementwise_fma(o0 == -kPosBase ? l4 : z, km2, quirk);
            }
        }
#if SIFT_COLW_PIPE
        // two-deep read-add-write chain: sample q + 1's slots are read before q's
        // are written; where they alias (q + 1's position o' = o, o + 1, or o' + 1
        // = o) the value just computed for q replaces the stale read.  The LDS
        // applies the writes in order, so every bin still sums in raster order.
        {
            f2v A = ((lds_f2v*)(tp[0]))[0], Bv = ((lds_f2v*)(tp[0]))[kPosF / 2];
#pragma unroll
            for (int qb = 0; qb < kB; qb++) {
                auto t = (lds_f2v*)(tp[qb]);
                f2v An, Bn;
                if (qb + 1 < kB) {
                    auto tn = (lds_f2v*)(tp[qb + 1]);
                    An = tn[0];
                    Bn = tn[kPosF / 2];
                }
                const f2v a = A + lo[qb], b = Bv + hi[qb];
                t[0] = a;
                t[kPosF / 2] = b;
                if (qb + 1 < kB) {
                    const int d = (int)(tp[qb + 1] - tp[qb]);
                    An = d == 0 ? a : (d == kPosF * 4 ? b : An);
                    Bn = d == 0 ? b : (d == -kPosF * 4 ? a : Bn);
                    A = An;
                    Bv = Bn;
                }
            }
        }
#else
#pragma unroll
        for (int qb = 0; qb < kB; qb++) {
            auto t = (lds_f2v*)(tp[qb]);
            f2v a = t[0];
            f2v b = t[kPosF / 2];
            a = a + lo[qb];
            b = b + hi[qb];
            t[0] = a;
            t[kPosF / 2] = b;
        }
#endif
        }
        wave_sync();
    };
    // bands -1 and 3 keep one row of their pair (rows 0 and 3): one-row slots
    // pos * 64 + lane (ds_read_b32 / ds_write_b32), the values of two samples per
    // packed op -- the same roundings as the pair walk's row
    char* lb1 = reinterpret_cast<char*>(buf + lane) + kPosBase * kKpW * 4;
    float quirk1 = 0.f;       // column 4's position 0 of the kept row (column 3's wave)
    auto walk1 = [&](int ch, auto Upper, auto Q) __attribute__((always_inline)) {
        constexpr bool kQ = decltype(Q)::value;
        constexpr bool kUp = decltype(Upper)::value;    // band 3: row r0 = v - v_r1; band -1: row r0 + 1 = v_r1
#if SIFT_COLW_KS == 16
        i16v trf, tcf;
        __asm__ volatile(
            "s_load_dwordx16 %0, %2, 0x0\n\t"
            "s_load_dwordx16 %1, %2, 0x40\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(trf), "=&s"(tcf)
            : "s"(p.smp_s + ch * kTabDw));
#else
        i8v trf, tcf;
        __asm__ volatile(
            "s_load_dwordx8 %0, %2, 0x0\n\t"
            "s_load_dwordx8 %1, %2, 0x20\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(trf), "=&s"(tcf)
            : "s"(p.smp_s + ch * kTabDw));
#endif
#pragma unroll
        for (int b0 = 0; b0 < kKS; b0 += kB) {
        f4v r2[kB / 2];
#pragma unroll
        for (int q = 0; q < kB / 2; q++)
            r2[q] = *(const __attribute__((address_space(3))) volatile f4v*)(stg + lane * kStride + 2 * b0 + 4 * q);
        f2v lo[kB / 2], hi[kB / 2];
        char* tp[kB];
#pragma unroll
        for (int k = 0; k < kB / 2; k++) {
            const int q = b0 + 2 * k;
            const f2v mw2 = {r2[k].x, r2[k].z}, ob2 = {r2[k].y, r2[k].w};
            const f2v fr = {__builtin_amdgcn_fractf(ob2.x), __builtin_amdgcn_fractf(ob2.y)};
            int oa, ob;
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(oa) : "v"(ob2.x));
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(ob) : "v"(ob2.y));
            tp[2 * k] = lb1 + __mul24(oa, kKpW * 4);
            tp[2 * k + 1] = lb1 + __mul24(ob, kKpW * 4);
            const f2v rf2 = {__int_as_float(trf[q]), __int_as_float(trf[q + 1])};
            const f2v v_r1 = mw2 * rf2;
            const f2v c = kUp ? mw2 - v_r1 : v_r1;
            const f2v cf2 = {__int_as_float(tcf[q]), __int_as_float(tcf[q + 1])};
            const f2v km2 = {__int_as_float((tcf[q] >> 31) & 0x3f800000), __int_as_float((tcf[q + 1] >> 31) & 0x3f800000)};
            const f2v pc = c * cf2;
            const f2v cv = __builtin_elementwise_fma(c, km2, pc);
            hi[k] = cv * fr;
            lo[k] = cv - hi[k];
            if constexpr (kQ) {
                const f2v c4 = -pc;
                const f2v h4 = c4 * fr, l4 = c4 - h4;
                quirk1 = __fmaf_rn(oa == -kPosBase ? l4.x : 0.f, km2.x, quirk1);
                quirk1 = __fmaf_rn(ob == -kPosBase ? l4.y : 0.f, km2.y, quirk1);
            }
        }
#pragma unroll
        for (int qb = 0; qb < kB; qb++) {
            auto t = (__attribute__((address_space(3))) volatile float*)(tp[qb]);
            const float a = t[0], b = t[kKpW];
            t[0] = __fadd_rn(a, (qb & 1) ? lo[qb >> 1].y : lo[qb >> 1].x);
            t[kKpW] = __fadd_rn(b, (qb & 1) ? hi[qb >> 1].y : hi[qb >> 1].x);
        }
        }
        wave_sync();
    };

    // band close: row b of the column is final (the pairs' first element); the
    // second element becomes the first, the second restarts at 0.  One-row
    // bands: -1 ends by spreading its row 0 into the pair layout, 2 by
    // gathering row 3 into the one-row layout (every slot read before any is
    // written: the two layouts overlap), 3 reads its row.
    auto close_band = [&](auto B) __attribute__((always_inline)) {
        constexpr int b = decltype(B)::value;
        float e0[kPos];
        if constexpr (kOneRow && b == -1) {
#pragma unroll
            for (int pos = 0; pos < kPos; pos++) e0[pos] = ((__attribute__((address_space(3))) volatile float*)(buf + pos * kKpW + lane))[0];
#pragma unroll
            for (int pos = 0; pos < kPos; pos++) *(lds_f2v*)(buf + pos * kPosF + 2 * lane) = f2v{e0[pos], 0.f};
            if constexpr (kQuirk) quirk = f2v{quirk1, 0.f};
            wave_sync();
            return;
        } else if constexpr (kOneRow && b == 3) {
#pragma unroll
            for (int pos = 0; pos < kPos; pos++) e0[pos] = ((__attribute__((address_space(3))) volatile float*)(buf + pos * kKpW + lane))[0];
            if constexpr (kQuirk) quirk = f2v{quirk1, 0.f};
        } else if constexpr (kOneRow && b == 2) {
            float e1[kPos];
#pragma unroll
            for (int pos = 0; pos < kPos; pos++) {
                const f2v v = *(lds_f2v*)(buf + pos * kPosF + 2 * lane);
                e0[pos] = v.x;
                e1[pos] = v.y;
            }
#pragma unroll
            for (int pos = 0; pos < kPos; pos++) ((__attribute__((address_space(3))) volatile float*)(buf + pos * kKpW + lane))[0] = e1[pos];
        } else {
#pragma unroll
        for (int pos = 0; pos < kPos; pos++) {
            auto t = (lds_f2v*)(buf + pos * kPosF + 2 * lane);
            const f2v v = *t;
            e0[pos] = v.x;
            if (b < 3) *t = f2v{v.y, 0.f};
        }
        }
        if constexpr (b >= 0) {
            raw[b][0] = __fadd_rn(e0[1], e0[9]);                 // slot 0 + slot 8
            // slot 1 (+ slot 9 = the next column's position 0: column 4's for column
            // 3 here, the others' at the fold)
            raw[b][1] = kQuirk ? __fadd_rn(e0[2], quirk.x) : e0[2];
#pragma unroll
            for (int q = 2; q < 8; q++) raw[b][q] = e0[q + 1];
            p0[b] = e0[0];
        }
        if constexpr (kQuirk) {
            if constexpr (kOneRow && b == 2) quirk1 = quirk.y;
            quirk = f2v{quirk.y, 0.f};
        }
        wave_sync();
    };

    Pre pf;
    issue(cbeg, pf);
    stage(pf);
    wave_sync();
    auto run_band = [&](auto B) __attribute__((always_inline)) {
        constexpr int b = decltype(B)::value;
        const int ch_end = p.band_first[C][b + 2];
        for (int ch = p.band_first[C][b + 1]; ch < ch_end; ch++) {
            if (ch + 1 < cend) issue(ch + 1, pf);
            // column 3: only chunks holding a left share (c0 = 3) can reach column 4's
            // position 0 (a per-chunk flag from the host, wave-uniform)
            bool q = false;
            if constexpr (kQuirk) {
                // a scalar load (a vector load's vmcnt wait would also drain the prefetch)
                int fl;
                __asm__ volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(fl) : "s"(p.chunk_left + ch));
                q = fl != 0;
            }
            constexpr auto up = std::integral_constant<bool, b == 3>{};
            if constexpr (kOneRow && (b == -1 || b == 3)) {
                if (q) walk1(ch, up, std::true_type{});
                else walk1(ch, up, std::false_type{});
            } else {
                if (q) walk(ch, std::true_type{});
                else walk(ch, std::false_type{});
            }
            if (ch + 1 == ch_end) close_band(B);
            if (ch + 1 < cend) {
                stage(pf);
                wave_sync();
            }
        }
    };
    run_band(std::integral_constant<int, -1>{});
    run_band(std::integral_constant<int, 0>{});
    run_band(std::integral_constant<int, 1>{});
    run_band(std::integral_constant<int, 2>{});
    run_band(std::integral_constant<int, 3>{});
}

#ifndef SIFT_COLW_WPE
#define SIFT_COLW_WPE 0
#endif
#if SIFT_COLW_WPE
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(SIFT_COLW_WPE, SIFT_COLW_WPE)))
#else
__global__ __launch_bounds__(64 * kWaves)
#endif
void sift_desc_colw(ColwParams p)
{
    __shared__ __attribute__((aligned(16))) float s_buf[kWaves][kWaveFloats];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int C = wave & 3, gi = wave >> 2;
    float* buf = s_buf[wave];
    unsigned* kpo = reinterpret_cast<unsigned*>(buf + kKpOff);
    float* xch = s_buf[4 * gi];            // the group's exchange (its four waves' memory, contiguous)

    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int ngroups = (total + kKpW - 1) / kKpW;
    const int njobs = (ngroups + kGroups - 1) / kGroups;
    // XCD-aware job order: workgroups are dealt round-robin over the 8 XCDs, so
    // the jobs are split into 8 contiguous ranges, one per XCD group (compact
    // raster bands whose windows overlap); every wave of a workgroup runs the
    // same jobs (the exchange's barriers)
    const int xg = blockIdx.x & 7;
    const int per = (njobs + 7) >> 3;
    const int j_end = min(njobs, (xg + 1) * per);
    constexpr int kPairs = kKS / 2, kPer = 64 / kPairs, kIt = kKpW / kPer;
    const int kl = lane / kPairs;

    for (int job = xg * per + (blockIdx.x >> 3); job < j_end; job += (int)(gridDim.x >> 3)) {
        const int grp = job * kGroups + gi;
        const int g = grp * kKpW + lane;
        const bool live = grp * kKpW < total;        // wave-uniform
        const bool act = g < total;
        float raw[4][8], p0[4];
        if (live) {
            // byte offset of the keypoint's pixel in the padded map (< 4 GiB: checked on the host)
            const int gg = min(g, total - 1);
            const slam_keypoint kp = p.kps[gg];
            const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
            kpo[lane] = (unsigned)((size_t)p.kp_frame[gg] * p.frame_bytes + p.origin_bytes) +
                        (unsigned)(pty * p.pitch_bytes + ptx * 8);
            wave_sync();
            unsigned kof[kIt];
#pragma unroll
            for (int it = 0; it < kIt; it++) kof[it] = kpo[kPer * it + kl];
            if (C == 3) colw_walk<true>(p, C, lane, buf, kof, raw, p0);
            else colw_walk<false>(p, C, lane, buf, kof, raw, p0);
        }
        __syncthreads();                  // every walk of the workgroup done: slots and stages are dead
        if (live) {
            float* xr = xch + lane * kXStride;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int q = 0; q < 8; q++) xr[r * 32 + C * 8 + q] = raw[r][q];
            if (C >= 1) {
                float* x0 = xch + kX0Off + lane * 16 + (C - 1) * 4;   // column C - 1's slot 9
#pragma unroll
                for (int r = 0; r < 4; r++) x0[r] = p0[r];
            }
        }
        __syncthreads();
        if (live && C == 0) {
            float* rb = xch + lane * kXStride;
            const float* x0 = xch + kX0Off + lane * 16;
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int r = 0; r < 4; r++) rb[r * 32 + c * 8 + 1] = __fadd_rn(rb[r * 32 + c * 8 + 1], x0[c * 4 + r]);
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
                        for (int bb = 0; bb < 4; bb++) {
                            const int k = c * 16 + wq * 4 + bb;
                            float x = rintf(__fmul_rn(rb[k], sc));
                            x = fminf(fmaxf(x, 0.f), 255.f);
                            const int iv = (int)x;
                            word |= (uint32_t)iv << (8 * bb);
                            ns += (iv - 128) * (iv - 128);
                            rb[k] = x;
                        }
                        wd[wq] = word;
                    }
                    *reinterpret_cast<uint4*>(p.desc_u8 + (size_t)g * 128 + c * 16) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
                }
                p.norm_i8[g] = ns;
                if (p.desc_f32) {
                    float4* o = reinterpret_cast<float4*>(p.desc_f32 + (size_t)g * 128);
#pragma unroll 8
                    for (int c = 0; c < 32; c++) o[c] = make_float4(rb[4 * c], rb[4 * c + 1], rb[4 * c + 2], rb[4 * c + 3]);
                }
            }
        }
        __syncthreads();                  // the exchange read before the next job's walk reuses it
    }
}

}  // namespace

// SLAMHIP_SIFT_COLW=1 makes AUTO run this kernel for FAST keypoints instead of
// sift_desc_band (A/B; the two measure the same at 210 candidates since the band
// kernel's prefetch fix, and the band kernel's tail split wins at 27: DESIGN.md §4)
bool sift_colw_enabled()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_SIFT_COLW"); return e && e[0] == '1'; }();
    return on;
}

// The four columns' schedules and tables from the band geometry; false when the
// geometry is not the FAST one this kernel is written for (floor(obin) in
// [-9, -1]), a column's band is empty, or a target's order is not raster order.
bool sift_colw_prepare(slam_ctx* c, hipStream_t s, const BandGeometry& geo)
{
    c->sift_colw_valid = false;
    if (!geo.neg) return false;
    const std::vector<BandSample>& smp = geo.smp;
    const int n = (int)smp.size();
    auto f2i = [](float f) { union { float f; int32_t i; } u; u.f = f; return u.i; };
    auto i2f = [](int32_t i) { union { int32_t i; float f; } u; u.i = i; return u.f; };
    std::vector<float2> tv;
    std::vector<int32_t> ts;
    int band_first[4][6];
    auto push = [&](float w, int off, float rf, float cf, bool left) {
        if (tv.size() % kKS == 0) ts.resize(ts.size() + kTabDw, 0);
        const size_t q = tv.size() % kKS, base = ts.size() - kTabDw;
        tv.push_back(make_float2(w, i2f(off)));
        ts[base + q] = f2i(rf);
        ts[base + kKS + q] = f2i(cf) | (left ? (int32_t)0x80000000 : 0);   // -cbin (or -0) for a left share
    };
    for (int col = 0; col < 4; col++) {
        std::vector<int> sched;      // this column's samples in schedule order (< 0: padding)
        for (int b = -1; b <= 3; b++) {
            band_first[col][b + 1] = (int)(tv.size() / kKS);
            const size_t start = tv.size();
            for (int k = 0; k < n; k++) {
                const BandSample& sm = smp[k];
                if (sm.r0 != b || (sm.c0 != col - 1 && sm.c0 != col)) continue;
                const bool left = sm.c0 == col;           // this column is the sample's c0: v - v * cbin
                push(sm.wexp, (sm.i * geo.pitch + sm.j) * 8, sm.rf, sm.cf, left);
                sched.push_back(k);
            }
            if (tv.size() == start) return false;     // the band close needs a chunk
            while (tv.size() % kKS) {                  // padding: weight 0 at the keypoint (+0 everywhere)
                push(0.f, 0, 0.f, 0.f, false);
                sched.push_back(-1);
            }
        }
        band_first[col][5] = (int)(tv.size() / kKS);
        // every target cell of the column (hist rows 1..4; hist column col + 1, and
        // column 3's wave also hist column 5's quirk slot) in raster order
        for (int R = 1; R <= 4; R++)
            for (int C = col + 1; C <= (col == 3 ? 5 : col + 1); C++) {
                std::vector<int> ras, sc;
                auto hits = [&](const BandSample& q) {
                    const int dr = R - 1 - q.r0, dc = C - 1 - q.c0;
                    return dr >= 0 && dr <= 1 && dc >= 0 && dc <= 1;
                };
                for (int q = 0; q < n; q++) if (hits(smp[q])) ras.push_back(q);
                for (int q : sched) if (q >= 0 && hits(smp[q])) sc.push_back(q);
                if (ras != sc) return false;
            }
    }
    const int nchunks = (int)(tv.size() / kKS);
    if (nchunks > kMaxChunks) return false;
    std::vector<int32_t> left(nchunks, 0);
    for (int ch = 0; ch < nchunks; ch++)
        for (int q = 0; q < kKS; q++) left[ch] |= ts[(size_t)ch * kTabDw + kKS + q] < 0;
    const size_t b_v = tv.size() * sizeof(float2), b_s = ts.size() * sizeof(int32_t), b_l = left.size() * sizeof(int32_t);
    if (c->sift_colw_buf.ensure(b_v + b_s + b_l) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_colw_buf.p, tv.data(), b_v, hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_colw_buf.as<char>() + b_v, ts.data(), b_s, hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipMemcpyAsync(c->sift_colw_buf.as<char>() + b_v + b_s, left.data(), b_l, hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    SiftColwMeta& m = c->sift_colw;
    m.nrec = (int)tv.size();
    m.nchunks = nchunks;
    for (int col = 0; col < 4; col++)
        for (int q = 0; q < 6; q++) m.band_first[col][q] = band_first[col][q];
    c->sift_colw_valid = true;
    return true;
}

hipError_t launch_sift_desc_colw(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    const SiftColwMeta& m = c->sift_colw;
    ColwParams p;
    p.grad = c->grad.as<char>();
    p.frame_bytes = grad_frame(w, h) * 8;
    p.origin_bytes = grad_origin(w) * 8;
    p.pitch_bytes = grad_pitch(w) * 8;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.smp = c->sift_colw_buf.as<float2>();
    p.smp_s = reinterpret_cast<const int*>(c->sift_colw_buf.as<char>() + (size_t)m.nrec * sizeof(float2));
    p.chunk_left = reinterpret_cast<const int*>(c->sift_colw_buf.as<char>() + (size_t)m.nrec * sizeof(float2) +
                                                (size_t)m.nchunks * kTabDw * sizeof(int32_t));
    p.nchunks = m.nchunks;
    for (int col = 0; col < 4; col++)
        for (int q = 0; q < 6; q++) p.band_first[col][q] = m.band_first[col][q];
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    // persistent: as many workgroups (kGroups keypoint groups x 4 columns) per CU
    // as are resident at once, a multiple of 8 workgroups for the XCD split
#ifndef SIFT_COLW_PERCU
#define SIFT_COLW_PERCU 0   // workgroups per CU in the persistent grid; 0: as many as are resident
#endif
    static const int per_cu = [] {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sift_desc_colw, 64 * kWaves, 0) != hipSuccess || nb < 1)
            nb = 1;
        return SIFT_COLW_PERCU > 0 && SIFT_COLW_PERCU < nb ? SIFT_COLW_PERCU : nb;
    }();
    int grid = c->cu_count * per_cu;
    const int need = (cap + kKpW * kGroups - 1) / (kKpW * kGroups);
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    hipLaunchKernelGGL(sift_desc_colw, dim3(grid), dim3(64 * kWaves), 0, s, p);
    return hipGetLastError();
}

}  // namespace slamhip
