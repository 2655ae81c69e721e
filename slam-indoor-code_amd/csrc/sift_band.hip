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
//    samples, 8 lanes load 16 consecutive samples of one keypoint (two each;
//    8 keypoints per instruction pair, coalesced row segments), multiply in
//    the Gaussian weight, form obin, and stage {mw_q, mw_q+1, obin_q,
//    obin_q+1} per sample pair in LDS; the walk then reads its own keypoint's
//    records (conflict-free stride).
//  * Rows outside the descriptor.  Band -1 reaches hist rows 0 and 1, band 3
//    rows 4 and 5; hist rows 0 and 5 are discarded, so these two bands keep
//    one row in a one-row slot layout (ds_read_b32 / ds_write_b32) and pair
//    two samples per packed instruction (9 VALU per lane-sample, not 13).
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
#include <type_traits>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

#ifndef SIFT_BAND_DIAG_TAB
#define SIFT_BAND_DIAG_TAB 0
#endif
#ifndef SIFT_BAND_DIAG_KP
#define SIFT_BAND_DIAG_KP 0
#endif
#ifndef SIFT_BAND_KS
#define SIFT_BAND_KS 16
#endif
#ifndef SIFT_BAND_WAVES
#define SIFT_BAND_WAVES 8
#endif
#ifndef SIFT_BAND_SLOTCOLS
#define SIFT_BAND_SLOTCOLS 6
#endif
constexpr int kKS = SIFT_BAND_KS;       // window samples per staged chunk
constexpr int kStride = 2 * kKS + 4;    // stage floats per keypoint ({mw, obin} x kKS; 16-byte rows, b128 conflict-free)
constexpr int kWaves = SIFT_BAND_WAVES;
constexpr int kKpW = 32;                // keypoints per wave; lane = keypoint + 32 * dc
constexpr int kPos = 10;                // slot positions: 0 = left cell's slot 9, 1..9 = slots 0..8
constexpr int kCols = 5;                // histogram columns 0..4 (4: the 361-degree quirk column)
// Slots: float index pos * kPosF + col' * 64 + 2 * keypoint + row, col' = 4 - column
// (col' = 5, column -1, is a junk column: the c0 = -1 samples' column-c0 share,
// outside the descriptor), row 0 = the band's upper target row r0 + 1... i.e. the
// pair {row r0, row r0 + 1} of the two rows a band's samples reach.  A lane
// owns one column of a sample's 2 x 2 x 2 cell (dc = 0: column c0 + 1, dc = 1:
// column c0) and updates its four bins as two 8-byte pairs {row r0, row r0 + 1}
// at positions p and p + 1: ds_read_b64 / ds_write_b64 with packed f32 adds.
// Banks: 2 * keypoint (+1) whatever the column and position -- conflict-free
// for both the 32-lane read groups and the 16-lane write groups.
constexpr int kPosF = SIFT_BAND_SLOTCOLS * 64;
static_assert(SIFT_BAND_SLOTCOLS == kCols + 1, "slot columns: the junk column has its own slots");
// one-row layout of bands -1 and 3 (same memory): pos * kPos1F + col' * 32 + keypoint.
// The position stride is the pair layout's (half of each position unused): one
// slot-position byte (gradpos, (floor(obin) + 9) * 6) shifted by 8 addresses both
constexpr int kPos1F = kPosF;
constexpr int kSlots = kPos * kPosF;
constexpr int kStageOff = kSlots;
constexpr int kKpOff = kStageOff + kKpW * kStride;
constexpr int kWaveFloats = kKpOff + kKpW;
constexpr int kMaxChunks = 1024;
constexpr int kTabCols = 5;              // per chunk: rf, cf, slot offsets of the 32- and 16-keypoint layouts, weight
constexpr int kRawStride = 129;          // epilogue: one keypoint per lane, odd stride = conflict-free
static_assert(kKpW * kRawStride <= kKpOff, "epilogue raw buffer must fit below the keypoint offsets");
static_assert(kWaves * kWaveFloats * 4 <= 160 * 1024, "LDS");
static_assert(kStageOff % 4 == 0 && kStride % 4 == 0 && kWaveFloats % 4 == 0, "16-byte stage rows");

// the 16-keypoint variant (sift_desc_band4, below): four lanes per keypoint
namespace q4 {
constexpr int kKpW = 16;                 // keypoints per wave; lane = keypoint + 16 dc + 32 dp
constexpr int kColF = 2 * kKpW;          // pair layout: pos * kPosF + col' * kColF + 2 * keypoint + row
constexpr int kPosF = 6 * kColF;
constexpr int kCol1F = kKpW;             // one-row layout: pos * kPos1F + col' * kCol1F + keypoint
constexpr int kPos1F = 6 * kCol1F;
constexpr int kSlots = kPos * kPosF;
constexpr int kStageOff = kSlots;
constexpr int kKpOff = kStageOff + kKpW * kStride;
constexpr int kWaveFloats = kKpOff + kKpW;
constexpr int kWaves = 8;                // per workgroup; two workgroups per CU (4 waves per SIMD)
static_assert(kKpW * kRawStride <= kKpOff, "epilogue raw buffer must fit below the keypoint offsets");
static_assert(2 * kWaves * kWaveFloats * 4 <= 160 * 1024, "LDS: two workgroups per CU");
static_assert(kStageOff % 4 == 0 && kWaveFloats % 4 == 0, "16-byte stage rows");
}  // namespace q4

struct BandParams {
    const char* grad;                   // padded gradient map (bytes)
    size_t frame_bytes, origin_bytes;
    int pitch_bytes;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float2* smp;                  // [nchunks * kKS] scheduled {w, window offset in bytes}
    const int* smp_s;                   // [nchunks][kTabCols][kKS] {rf bits, cf bits, slot byte offsets (32 / 16 kps per wave)}
    int nchunks;
    int band_first[6];                  // first chunk of band b at band_first[b + 1]
    float ori_deg;
    const uint8_t* posb;                // kObin 2: slot-position bytes, the gradient map's layout
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
    int wave_major;                     // group order (SLAMHIP_SIFT_BAND_ORDER=0: workgroup-major, the round-4 order)
    int split;                          // SLAM_BAND_SPLIT_*: part-walks (sift_desc_band only)
    int parts_env;                      // SLAMHIP_SIFT_BAND_PARTS: 2 / 4 parts forced (timing), else 0
    float4* split_raw;                  // [slot][row][lane][4]: the parts' finished rows
    int* split_cnt;                     // [slot]: halves arrived (reset to 0 by the second)
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef int i16v __attribute__((ext_vector_type(16)));
typedef int i8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

#ifndef SIFT_BAND_ATOMIC
#define SIFT_BAND_ATOMIC 0
#endif
// a slot update as one non-returning LDS float add (ds_add_f32, round to
// nearest even like v_add_f32); no read-back into VGPRs, no dependency chain
__device__ __forceinline__ void lds_add(float* t, float v)
{
    __hip_atomic_fetch_add(t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// kObin: the gradient map's orientation form (launch_sift_base): 0 ori, 1 obin,
// 2 fract(obin) with the slot position in the byte plane p.posb (kNeg only: the
// walk then takes frac and the slot address from the stage, 2 VALU per
// lane-sample fewer)
template <bool kNeg, int kObin>
__global__ __launch_bounds__(64 * kWaves) void sift_desc_band(BandParams p)
{
    __shared__ __attribute__((aligned(16))) float s_buf[kWaves][kWaveFloats];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kq = lane & 31, dc = lane >> 5;     // keypoint of the wave, column half (dc)
#ifdef SIFT_BAND_PRIO
    // timing variant: static priority for the second-dispatched half (waves 4-7,
    // the arbitration losers: MI355X_MICROARCH.md "Two waves per SIMD" item 4)
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    float* buf = s_buf[wave];
    float* stg = buf + kStageOff;
    unsigned* kpo = reinterpret_cast<unsigned*>(buf + kKpOff);
    const float bins_per_rad = 8 / 360.f;
    const float ori_deg = p.ori_deg;

    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int ngroups = (total + kKpW - 1) / kKpW;
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so the
    // keypoint groups are split into 8 contiguous ranges, one per XCD group
    // (blockIdx % 8): each XCD walks a compact raster band whose windows overlap
    const int xg = blockIdx.x & 7;
    // wave-major within the XCD range: consecutive groups go to different
    // workgroups (CUs), so a launch's last, partial round of groups spreads over
    // all the XCD's CUs (one or two waves each) instead of filling a few CUs'
    // eight waves while the rest idle -- the strong-scaling tail of small shards
    const int nw = (gridDim.x >> 3) * kWaves;
    const int wi = p.wave_major ? wave * (gridDim.x >> 3) + (blockIdx.x >> 3) : (blockIdx.x >> 3) * kWaves + wave;
    const int per = (ngroups + 7) >> 3;
    const int grp_end = min(ngroups, (xg + 1) * per);
    // The last, partial round of an XCD range (rem groups, rem <= its CUs) runs as
    // part-walks: a part owns descriptor rows r0..r1 and walks bands r0 - 1..r1
    // only (row d receives only bands d - 1 and d, so each part sums its rows in
    // the full walk's order: bit-identical).  Two parts (rows 0-1, bands -1..1;
    // rows 2-3, bands 1..3) are ~60 % of a walk each, four (one row, two bands)
    // ~40 %; the round uses that many times the waves, so the launch's tail --
    // lone waves on otherwise idle CUs -- shrinks.  Each part leaves its rows in
    // split_raw; the last to arrive (split_cnt) takes the others' and runs the
    // epilogue.
    const int g0 = xg * per, gx = max(0, grp_end - g0);
    const int ncu = (int)(gridDim.x >> 3);                     // CUs (one workgroup each) per XCD range
    const bool split_all = p.split >= SLAM_BAND_SPLIT_ALL;    // every group in parts (tests)
    const int full = split_all ? 0 : gx / nw * nw, rem = gx - full;
    // (measured, r5tail2: two parts pay when the remainder leaves at most one lone
    // wave per CU -- rem <= CUs per XCD; at 2.75 waves per CU, batch 210, the
    // half-walks ran 0.25 ms slower than the whole ones)
    const bool split = rem > 0 && (split_all || (p.split && rem <= ncu));
    const int lg_parts = !split ? 0
                         : split_all ? (p.split == SLAM_BAND_SPLIT_ALL4 ? 2 : 1)
                         : p.parts_env ? (p.parts_env == 4 ? 2 : 1)
                         : (2 * rem > ncu ? 1 : 2);
    const int njobs = split ? full + (rem << lg_parts) : gx;
    const int nch = p.nchunks;
    // stage mapping: lane loads window samples 2 s2 and 2 s2 + 1 of keypoints kPer * it + kl
    constexpr int kPairs = kKS / 2, kPer = 64 / kPairs, kIt = kKpW / kPer;
    const int s2 = lane % kPairs, kl = lane / kPairs;
    // slot bases (bytes; the table holds byte offsets: no per-sample scaling)
    char* lb = reinterpret_cast<char*>(buf + 2 * kq + dc * 64);   // pair layout: this lane's column of a sample, col' of c0 + 1 (+ dc)
    char* lb1 = reinterpret_cast<char*>(buf + kq + dc * 32);      // one-row layout: the same column
    // kObin 2: the bases less the table's pos_base (9) positions, which the
    // position byte already counts
    char* lb2 = lb - 9 * kPosF * 4;
    char* lb12 = lb1 - 9 * kPos1F * 4;
    const f2v km2 = {dc ? 1.f : 0.f, dc ? 1.f : 0.f}, kn2 = {dc ? -1.f : 1.f, dc ? -1.f : 1.f};
    for (int job = wi; job < njobs; job += nw) {
        // rows r_lo..r_hi of the descriptor: 0..3 for a whole walk, else a part's
        int grp = g0 + job, r_lo = 0, r_hi = 3, part = -1;
        if (split && job >= full) {
            grp = g0 + full + ((job - full) >> lg_parts);
            part = (job - full) & ((1 << lg_parts) - 1);
            r_lo = part << (2 - lg_parts);
            r_hi = r_lo + (4 >> lg_parts) - 1;
        }
        const int slot = split_all ? grp : xg * ncu + ((job - full) >> lg_parts);
        const int g = grp * kKpW + kq;
        const bool act = g < total;
        if (dc == 0) {
            // byte offset of the keypoint's pixel in the padded map (< 4 GiB: checked on the host)
            const int gg = min(g, total - 1);
            const slam_keypoint kp = p.kps[gg];
            const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
#if SIFT_BAND_DIAG_KP
            // timing probe (wrong results): every keypoint reads frame 0's window at
            // (500, 500) -- the gradient loads then hit the caches
            (void)ptx; (void)pty;
            kpo[kq] = (unsigned)p.origin_bytes + (unsigned)(500 * p.pitch_bytes + 500 * 8);
#else
            kpo[kq] = (unsigned)((size_t)p.kp_frame[gg] * p.frame_bytes + p.origin_bytes) +
                      (unsigned)(pty * p.pitch_bytes + ptx * 8);
#endif
        }
#pragma unroll 10
        for (int q = 0; q < kSlots / 64; q++) buf[q * 64 + lane] = 0.f;   // both layouts
        wave_sync();
        unsigned kof[kIt];
#pragma unroll
        for (int it = 0; it < kIt; it++) kof[it] = kpo[kPer * it + kl];

        // ---- prefetch of one chunk: kIt x kPer keypoints x kKS consecutive window samples ----
        struct Pre { float2 v[2 * kIt]; float wa, wb; uint32_t pb[kIt]; };
        // the chunk's {weight, offset} entries are loaded one chunk ahead, so the
        // gradient loads never wait on them
        const float4* smp4 = reinterpret_cast<const float4*>(p.smp);
        const int ch0 = p.band_first[r_lo];                 // band r_lo - 1's first chunk
        float4 smn = smp4[ch0 * kPairs + s2];
        auto issue = [&](int ch, Pre& pf) __attribute__((always_inline)) {
            const float4 sm = smn;
            pf.wa = sm.x;
            pf.wb = sm.z;
            const unsigned soa = (unsigned)__float_as_int(sm.y), sob = (unsigned)__float_as_int(sm.w);
#pragma unroll
            for (int it = 0; it < kIt; it++) {   // zero border: no bounds test
                pf.v[2 * it] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + soa));
                pf.v[2 * it + 1] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + sob));
                // the pair's two slot-position bytes (the pair is horizontally adjacent:
                // sob = soa + 8, so one 2-byte load at the pixel offset / 8)
                if constexpr (kObin == 2)
                    pf.pb[it] = *reinterpret_cast<const uint16_t*>(p.posb + ((kof[it] + soa) >> 3));
            }
            smn = smp4[min(ch + 1, nch - 1) * kPairs + s2];
        };
        // stage record of a sample pair: {mw_q, ob_q, mw_q+1, ob_q+1} (kObin 2 / 3:
        // {mw_q, mw_q+1, fract-or-ob_q, fract-or-ob_q+1})
        auto stage = [&](const Pre& pf) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const float2 a = pf.v[2 * it], b = pf.v[2 * it + 1];
                const float mwa = __fmul_rn(a.x, pf.wa), mwb = __fmul_rn(b.x, pf.wb);
                // kObin: sift_blur_grad stored obin = (ori - ori_deg) * 8/360 per pixel already
                const float oba = kObin ? a.y : __fmul_rn(__fsub_rn(a.y, ori_deg), bins_per_rad);
                const float obb = kObin ? b.y : __fmul_rn(__fsub_rn(b.y, ori_deg), bins_per_rad);
                if constexpr (kObin == 3) {
                    // the walk's slot position, formed once per keypoint-sample here instead
                    // of on both of its walk lanes: fract(obin) in the record, the byte
                    // (floor(obin) + 9) * 6 in the row's pad (the position-plane layout)
                    int oa, ob2;
                    __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(oa) : "v"(oba));
                    __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(ob2) : "v"(obb));
                    *reinterpret_cast<float4*>(stg + (kPer * it + kl) * kStride + 4 * s2) =
                        make_float4(mwa, mwb, __builtin_amdgcn_fractf(oba), __builtin_amdgcn_fractf(obb));
                    *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(stg + (kPer * it + kl) * kStride + 2 * kKS) + 2 * s2) =
                        (uint16_t)(__mul24(oa + 9, 6) | __mul24(ob2 + 9, 6) << 8);
                    continue;
                }
                if constexpr (kObin < 2) {
                    // {mw_q, ob_q, mw_q+1, ob_q+1}: each pixel's pair stored from its own
                    // load registers (the interleaved record made the compiler copy the
                    // loaded halves together right after the loads, waiting for them
                    // there and losing the prefetch)
                    float* row = stg + (kPer * it + kl) * kStride + 4 * s2;
                    *reinterpret_cast<float2*>(row) = make_float2(mwa, oba);
                    *reinterpret_cast<float2*>(row + 2) = make_float2(mwb, obb);
                    continue;
                }
                *reinterpret_cast<float4*>(stg + (kPer * it + kl) * kStride + 4 * s2) = make_float4(mwa, mwb, oba, obb);
                // kObin 2: the position bytes go to the row's 16-byte pad (byte q = sample q)
                if constexpr (kObin == 2)
                    *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(stg + (kPer * it + kl) * kStride + 2 * kKS) + 2 * s2) =
                        (uint16_t)pf.pb[it];
            }
        };

        float raw[4][2][8];             // this lane's half of the histogram: rows 1..4, columns 2 dc, 2 dc + 1
        // the chunk's wave-uniform table {rf, cf, slot offset} in SGPRs: one
        // wait for three scalar loads, none inside the walk
#if SIFT_BAND_KS == 16
        typedef i16v tabv;
#define SIFT_BAND_TABLE_LOAD(trf, tcf, tof, sp)                 \
        __asm__ volatile(                                       \
            "s_load_dwordx16 %0, %3, 0x0\n\t"                   \
            "s_load_dwordx16 %1, %3, 0x40\n\t"                  \
            "s_load_dwordx16 %2, %3, 0x80\n\t"                  \
            "s_waitcnt lgkmcnt(0)"                              \
            : "=&s"(trf), "=&s"(tcf), "=&s"(tof)                \
            : "s"(sp))
#else
        static_assert(kKS == 8, "chunk size");
        typedef i8v tabv;
#define SIFT_BAND_TABLE_LOAD(trf, tcf, tof, sp)                 \
        __asm__ volatile(                                       \
            "s_load_dwordx8 %0, %3, 0x0\n\t"                    \
            "s_load_dwordx8 %1, %3, 0x20\n\t"                   \
            "s_load_dwordx8 %2, %3, 0x40\n\t"                   \
            "s_waitcnt lgkmcnt(0)"                              \
            : "=&s"(trf), "=&s"(tcf), "=&s"(tof)                \
            : "s"(sp))
#endif
        auto o0_of = [&](float ob) __attribute__((always_inline)) {
            int o0;
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));   // floor + convert
            if (!kNeg) {
                o0 += o0 < 0 ? 8 : 0;
                o0 -= o0 >= 8 ? 8 : 0;
            }
            return o0;
        };
        // ---- bands 0..2: both target rows live, slot pairs {row r0, row r0 + 1} ----
#if SIFT_BAND_DIAG_TAB
        // timing probe (wrong results): the table and its lgkmcnt(0) drain only
        // every other chunk, the odd chunks reuse the even one's
        tabv trf, tcf, tof;
#endif
        auto walk_pair = [&](int ch) __attribute__((always_inline)) {
#if SIFT_BAND_DIAG_TAB
            if ((ch & 1) == 0) SIFT_BAND_TABLE_LOAD(trf, tcf, tof, p.smp_s + ch * (kTabCols * kKS));
#else
            tabv trf, tcf, tof;
            SIFT_BAND_TABLE_LOAD(trf, tcf, tof, p.smp_s + ch * (kTabCols * kKS));
#endif
            float4 r2[kPairs];
#pragma unroll
            for (int q = 0; q < kPairs; q++) r2[q] = *reinterpret_cast<const float4*>(stg + kq * kStride + 4 * q);
            uint32_t pw[kKS / 4];
            if constexpr (kObin >= 2) {
#pragma unroll
                for (int q = 0; q < kKS / 4; q++) pw[q] = reinterpret_cast<const uint32_t*>(stg + kq * kStride + 2 * kKS)[q];
            }
            // every value and slot address first (VALU only), then the kKS
            // read-add-write steps back to back
            f2v lo[kKS], hi[kKS];
            char* tp[kKS];
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                const float mw = kObin < 2 ? ((q & 1) ? r2[q >> 1].z : r2[q >> 1].x) : ((q & 1) ? r2[q >> 1].y : r2[q >> 1].x);
                const float ob = kObin < 2 ? ((q & 1) ? r2[q >> 1].w : r2[q >> 1].y) : ((q & 1) ? r2[q >> 1].w : r2[q >> 1].z);
                // frac = ob - floor(ob) in one v_fract_f32 (exact here: |ob| >= 2^-24 or
                // ob = 0 -- ob is a difference of two degree values over 45 -- so
                // ob - floor(ob) never rounds up to 1.0, where fract would clamp)
                float frac;
                if constexpr (kObin >= 2) {
                    // stored fract(obin); byte (o0 + 9) * 6 moved to bits 8..15 = (o0 + 9) * 1536
                    frac = ob;
                    tp[q] = lb2 + tof[q] + __builtin_amdgcn_perm(0u, pw[q >> 2], 0x0c0c000cu | (uint32_t)(q & 3) << 8);
                } else {
                    frac = __builtin_amdgcn_fractf(ob);
                    const int o0 = o0_of(ob);
                    // the table's offset holds col' of column c0 + 1 and pos = o0 + 9 (kNeg) / o0 + 1
                    tp[q] = lb + tof[q] + __mul24(o0, kPosF * 4);
                }
                const float v_r1 = __fmul_rn(mw, __int_as_float(trf[q]));
                const f2v vr = {__fsub_rn(mw, v_r1), v_r1};            // rows r0, r0 + 1
                const f2v cf2 = {__int_as_float(tcf[q]), __int_as_float(tcf[q])};
                const f2v c1 = vr * cf2;                                 // column c0 + 1: vr * cf
                // this lane's column: dc = 0 -> c1 = fma(c1, 1, 0 * vr); dc = 1 -> vr - c1 =
                // fma(c1, -1, 1 * vr) (both products exact: one rounding, as the reference)
                const f2v cv = __builtin_elementwise_fma(c1, kn2, vr * km2);
                const f2v fr = {frac, frac};
                hi[q] = cv * fr;                                         // bins o0 + 1
                lo[q] = cv - hi[q];                                      // bins o0
            }
#if SIFT_BAND_ATOMIC
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                // four non-returning ds_add_f32: the LDS applies one lane's adds to a
                // slot in issue order, so each bin still sums in raster order
                float* t = reinterpret_cast<float*>(tp[q]);
                lds_add(t, lo[q].x);
                lds_add(t + 1, lo[q].y);
                lds_add(t + kPosF, hi[q].x);
                lds_add(t + kPosF + 1, hi[q].y);
            }
#else
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                // volatile LDS pointer: two ds_read_b64 (2 cycles each), not one ds_read2_b64 (8)
                auto t = (__attribute__((address_space(3))) volatile f2v*)(tp[q]);
                f2v a = t[0];
                f2v b = t[kPosF / 2];
                a = a + lo[q];
                b = b + hi[q];
                t[0] = a;
                t[kPosF / 2] = b;
            }
#endif
            wave_sync();
        };
        // ---- bands -1 and 3: one target row is outside the descriptor (hist row 0 /
        // 5), so only the other is kept, in a one-row layout (slot pos * kPos1F +
        // col' * 32 + keypoint: ds_read_b32 / ds_write_b32, bank = keypoint), and the
        // arithmetic pairs two consecutive samples per packed instruction ----
        auto walk_one = [&](int ch, auto upper) __attribute__((always_inline)) {
#if SIFT_BAND_DIAG_TAB
            if ((ch & 1) == 0) SIFT_BAND_TABLE_LOAD(trf, tcf, tof, p.smp_s + ch * (kTabCols * kKS));
#else
            tabv trf, tcf, tof;
            SIFT_BAND_TABLE_LOAD(trf, tcf, tof, p.smp_s + ch * (kTabCols * kKS));
#endif
            float4 r2[kPairs];
#pragma unroll
            for (int q = 0; q < kPairs; q++) r2[q] = *reinterpret_cast<const float4*>(stg + kq * kStride + 4 * q);
            uint32_t pw[kKS / 4];
            if constexpr (kObin >= 2) {
#pragma unroll
                for (int q = 0; q < kKS / 4; q++) pw[q] = reinterpret_cast<const uint32_t*>(stg + kq * kStride + 2 * kKS)[q];
            }
            float lo[kKS], hi[kKS];
            char* tp[kKS];
#pragma unroll
            for (int q2 = 0; q2 < kPairs; q2++) {
                const int qa = 2 * q2, qb = qa + 1;
                const f2v mw2 = kObin < 2 ? f2v{r2[q2].x, r2[q2].z} : f2v{r2[q2].x, r2[q2].y};   // samples qa, qb
                const float oba = kObin < 2 ? r2[q2].y : r2[q2].z, obb = r2[q2].w;
                f2v fr2;
                if constexpr (kObin >= 2) {
                    fr2 = f2v{oba, obb};
                    tp[qa] = lb12 + tof[qa] + __builtin_amdgcn_perm(0u, pw[qa >> 2], 0x0c0c000cu | (uint32_t)(qa & 3) << 8);
                    tp[qb] = lb12 + tof[qb] + __builtin_amdgcn_perm(0u, pw[qb >> 2], 0x0c0c000cu | (uint32_t)(qb & 3) << 8);
                } else {
                    fr2 = f2v{__builtin_amdgcn_fractf(oba), __builtin_amdgcn_fractf(obb)};
                    tp[qa] = lb1 + tof[qa] + __mul24(o0_of(oba), kPos1F * 4);
                    tp[qb] = lb1 + tof[qb] + __mul24(o0_of(obb), kPos1F * 4);
                }
                const f2v rf2 = {__int_as_float(trf[qa]), __int_as_float(trf[qb])};
                const f2v cf2 = {__int_as_float(tcf[qa]), __int_as_float(tcf[qb])};
                const f2v v_r1 = mw2 * rf2;
                // band -1 keeps row r0 + 1 (v_r1), band 3 row r0 (mw - v_r1)
                const f2v v = decltype(upper)::value ? v_r1 : mw2 - v_r1;
                const f2v c1 = v * cf2;
                const f2v cv = __builtin_elementwise_fma(c1, kn2, v * km2);
                const f2v h = cv * fr2;
                const f2v l = cv - h;
                lo[qa] = l.x; lo[qb] = l.y;
                hi[qa] = h.x; hi[qb] = h.y;
            }
#if SIFT_BAND_ATOMIC
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                float* t = reinterpret_cast<float*>(tp[q]);
                lds_add(t, lo[q]);
                lds_add(t + kPos1F, hi[q]);
            }
#else
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                // volatile: ds_read_b32 / ds_write_b32 pairs (read2 / write2 forms measured slower)
                auto t = (__attribute__((address_space(3))) volatile float*)(tp[q]);
                const float a = t[0];
                const float b = t[kPos1F];
                t[0] = __fadd_rn(a, lo[q]);
                t[kPos1F] = __fadd_rn(b, hi[q]);
            }
#endif
            wave_sync();
        };
#undef SIFT_BAND_TABLE_LOAD
        // the finished row of column 2 dc + k2 from slot base c (pos stride ps, next column -cs)
        auto take_row = [&](float (&f)[2][8], const float* c0p, int ps, int cs, int cstride) __attribute__((always_inline)) {
#pragma unroll
            for (int k2 = 0; k2 < 2; k2++) {
                const float* c = c0p + (4 - (2 * dc + k2)) * cstride;
                f[k2][0] = __fadd_rn(c[1 * ps], c[9 * ps]);
                f[k2][1] = __fadd_rn(c[2 * ps], c[-cs]);   // + slot 9 = position 0 of the next column
#pragma unroll
                for (int q = 2; q < 8; q++) f[k2][q] = c[(q + 1) * ps];
            }
        };
        // ---- band closes (band b: descriptor row b is complete after it) ----
        auto close_band = [&](auto B) __attribute__((always_inline)) {
            constexpr int b = decltype(B)::value;
            if constexpr (b == -1) {
                // row r0 + 1 (descriptor row 0) leaves the one-row layout for the pairs'
                // first element; the second starts at 0.  The lane moves columns 3 dc ..
                // 3 dc + 2 of its keypoint (every slot pair is written).
                float v[3][kPos];
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int ps = 0; ps < kPos; ps++) v[c][ps] = buf[ps * kPos1F + (3 * dc + c) * 32 + kq];
                wave_sync();
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int ps = 0; ps < kPos; ps++)
                        *reinterpret_cast<float2*>(buf + ps * kPosF + (3 * dc + c) * 64 + 2 * kq) = make_float2(v[c][ps], 0.f);
            } else if constexpr (b <= 2) {
                // the pairs' first element (row b) is complete
                take_row(raw[b], buf + 2 * kq, kPosF, 64, 64);
                wave_sync();
                if constexpr (b < 2) {
                    // shift: the second element becomes the first, the second restarts at 0
                    float2* z = reinterpret_cast<float2*>(buf);
#pragma unroll 6
                    for (int q = 0; q < kSlots / 128; q++) {
                        float2 vv = z[q * 64 + lane];
                        z[q * 64 + lane] = make_float2(vv.y, 0.f);
                    }
                } else {
                    // band 3 keeps only row 3: the second element moves to the one-row layout
                    float v[3][kPos];
#pragma unroll
                    for (int c = 0; c < 3; c++)
#pragma unroll
                        for (int ps = 0; ps < kPos; ps++)
                            v[c][ps] = reinterpret_cast<const float2*>(buf + ps * kPosF + (3 * dc + c) * 64 + 2 * kq)->y;
                    wave_sync();
#pragma unroll
                    for (int c = 0; c < 3; c++)
#pragma unroll
                        for (int ps = 0; ps < kPos; ps++) buf[ps * kPos1F + (3 * dc + c) * 32 + kq] = v[c][ps];
                }
            } else {
                take_row(raw[3], buf + kq, kPos1F, 32, 32);
            }
            wave_sync();
        };

        // one band: its chunks (the next chunk's loads in flight while one is
        // walked), then its close.  Unrolled over the five bands, so the walk
        // variant and the descriptor row are compile-time.
        Pre pf;
        issue(ch0, pf);
        stage(pf);
        wave_sync();
        auto run_band = [&](auto B) __attribute__((always_inline)) {
            constexpr int b = decltype(B)::value;
            // a part-walk skips the bands outside r_lo - 1..r_hi by an empty chunk
            // range (the same code path); it starts at band r_lo - 1 on zeroed
            // slots (row r_lo - 1's shares land where it discards them; row r_lo
            // starts at 0 as in the walk)
            const bool skip = b < r_lo - 1 || b > r_hi;
            // both bounds at compile-time indices (scalar kernel-argument loads), the
            // choice made wave-uniform: a select of the two addresses was a vector
            // load whose vmcnt(0) wait also drained the chunk prefetch
            const int e1 = p.band_first[b + 1], e2 = p.band_first[b + 2];
            const int ch_end = __builtin_amdgcn_readfirstlane(skip ? e1 : e2);
            for (int ch = p.band_first[b + 1]; ch < ch_end; ch++) {
                if (ch + 1 < nch) issue(ch + 1, pf);
                if constexpr (b == -1)
                    walk_one(ch, std::true_type{});
                else if constexpr (b == 3)
                    walk_one(ch, std::false_type{});
                else
                    walk_pair(ch);
                if (ch + 1 == ch_end) close_band(B);
                if (ch + 1 < nch) {
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
        // ---- epilogue: raw histogram to LDS, one lane per keypoint ----
        wave_sync();
        {
            float* rb = buf + kq * kRawStride;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++)
#pragma unroll
                    for (int q = 0; q < 8; q++) rb[(r * 4 + 2 * dc + k2) * 8 + q] = raw[r][k2][q];
        }
        if (part >= 0) {
            // a part-walk: its finished rows (this lane's columns 2 dc, 2 dc + 1; the
            // same lane of every part holds the same columns) go from the LDS copy to
            // split_raw; the last part to arrive copies the others' rows over its
            // unfinished ones and runs the epilogue (through LDS, so the walk's
            // registers stay as they are)
            float* rb = buf + kq * kRawStride + 2 * dc * 8;
            float4* sr = p.split_raw + (size_t)slot * 4 * 64 * 4 + lane * 4;   // + row * 256
            for (int r = r_lo; r <= r_hi; r++)
#pragma unroll
                for (int u = 0; u < 4; u++) {        // columns k2 x 8 bins, 4 floats each
                    const float* e = rb + r * 32 + (u >> 1) * 8 + (u & 1) * 4;
                    sr[r * 256 + u] = make_float4(e[0], e[1], e[2], e[3]);
                }
            __threadfence();                              // release: the rows before the count
            int old = 0;
            if (lane == 0) old = atomicAdd(p.split_cnt + slot, 1);
            old = __shfl(old, 0, 64);
            if (old != (1 << lg_parts) - 1) continue;    // another part finishes the group
            __threadfence();                              // acquire: the others' rows after their counts
            for (int r = 0; r < 4; r++) {
                if (r >= r_lo && r <= r_hi) continue;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    float* e = rb + r * 32 + (u >> 1) * 8 + (u & 1) * 4;
                    const float4 v = sr[r * 256 + u];
                    e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
                }
            }
            if (lane == 0) p.split_cnt[slot] = 0;         // all arrived: ready for the next launch
        }
        wave_sync();
        if (dc == 0) {
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

// ---- sift_desc_band4: 16 keypoints per wave, four lanes per keypoint ----------
// The band kernel above keeps 32 keypoints' slots per wave (19.6 KB), so the
// LDS holds 8 waves per CU, 2 per SIMD; each wave walks its samples as a chain
// of slot read-add-writes whose LDS round trips two waves per SIMD do not
// cover (the LDS array ~55 % busy).  Here a wave holds 16 keypoints (10 KB of
// LDS) and a keypoint's sample update is split over four lanes: dc picks the
// column of the 2 x 2 x 2 footprint (c0 + 1 or c0) as before, and dp the
// orientation bin (o0 or o0 + 1), so each lane does one 8-byte {row r0, row
// r0 + 1} read-add-write per sample.  The same keypoints are in flight per CU
// (two 8-wave workgroups), with twice the waves to overlap the round trips;
// the LDS bytes per keypoint-sample are unchanged.  Bin values, their order
// and the descriptors are those of sift_desc_band (the value a dp lane adds:
// fma(hi, -1, cv) = cv - hi (one rounding, the reference's v_rco000 = v_rc00 -
// v_rco001) for dp = 0, fma(hi, 1, cv * 0) = hi for dp = 1; values are >= +0).
template <bool kNeg, bool kObin, bool kDma>
__global__ __launch_bounds__(64 * q4::kWaves) __attribute__((amdgpu_waves_per_eu(4, 4))) void sift_desc_band4(BandParams p)
{
    constexpr int kKpW = q4::kKpW, kColF = q4::kColF, kPosF = q4::kPosF, kCol1F = q4::kCol1F, kPos1F = q4::kPos1F;
    constexpr int kSlots = q4::kSlots, kStageOff = q4::kStageOff, kKpOff = q4::kKpOff;
    constexpr int kWaveFloats = q4::kWaveFloats, kWaves = q4::kWaves;
    __shared__ __attribute__((aligned(16))) float s_buf[kWaves][kWaveFloats];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kq = lane & 15, dc = (lane >> 4) & 1, dp = lane >> 5;
    float* buf = s_buf[wave];
    float* stg = buf + kStageOff;
    unsigned* kpo = reinterpret_cast<unsigned*>(buf + kKpOff);
    const float bins_per_rad = 8 / 360.f;
    const float ori_deg = p.ori_deg;

    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int ngroups = (total + kKpW - 1) / kKpW;
    // XCD-aware order (see sift_desc_band)
    const int xg = blockIdx.x & 7;
    // wave-major within the XCD range: consecutive groups go to different
    // workgroups (CUs), so a launch's last, partial round of groups spreads over
    // all the XCD's CUs (one or two waves each) instead of filling a few CUs'
    // eight waves while the rest idle -- the strong-scaling tail of small shards
    const int nw = (gridDim.x >> 3) * kWaves;
    const int wi = p.wave_major ? wave * (gridDim.x >> 3) + (blockIdx.x >> 3) : (blockIdx.x >> 3) * kWaves + wave;
    const int per = (ngroups + 7) >> 3;
    const int grp_end = min(ngroups, (xg + 1) * per);
    const int nch = p.nchunks;
    constexpr int kPairs = kKS / 2, kPer = 64 / kPairs, kIt = kKpW / kPer;
    const int s2 = lane % kPairs, kl = lane / kPairs;
    char* lb = reinterpret_cast<char*>(buf + 2 * kq + dc * kColF + dp * kPosF);     // pair layout
    char* lb1 = reinterpret_cast<char*>(buf + kq + dc * kCol1F + dp * kPos1F);      // one-row layout
    // column select (dc) and bin select (dp) as exact fmas: x * k + y * m
    const f2v km2 = {dc ? 1.f : 0.f, dc ? 1.f : 0.f}, kn2 = {dc ? -1.f : 1.f, dc ? -1.f : 1.f};
    const f2v sm2 = {dp ? 0.f : 1.f, dp ? 0.f : 1.f}, sn2 = {dp ? 1.f : -1.f, dp ? 1.f : -1.f};
    for (int grp = xg * per + wi; grp < grp_end; grp += nw) {
        const int g = grp * kKpW + kq;
        const bool act = g < total;
        if (lane < kKpW) {
            const int gg = min(g, total - 1);
            const slam_keypoint kp = p.kps[gg];
            const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
            kpo[kq] = (unsigned)((size_t)p.kp_frame[gg] * p.frame_bytes + p.origin_bytes) +
                      (unsigned)(pty * p.pitch_bytes + ptx * 8);
        }
#pragma unroll 10
        for (int q = 0; q < kSlots / 64; q++) buf[q * 64 + lane] = 0.f;
        wave_sync();
        unsigned kof[kIt];
#pragma unroll
        for (int it = 0; it < kIt; it++) kof[it] = kpo[kPer * it + kl];

        // stage record (keypoint k, sample pair q): register staging {mw_q, mw_q+1, ob_q,
        // ob_q+1} at k * kStride + 4 q; LDS-DMA staging (kDma) the raw pixel pair
        // {mag, ob, mag, ob} at 4 (8 k + (q ^ (k >> 1 & 7))): a DMA writes lane-linear
        // 16-byte records, so the pair a lane fetches is XOR-swizzled by its keypoint,
        // which makes the walk's ds_read_b128 (16 keypoints per lane group) hit all
        // 64 banks once
        auto rec = [&](int k, int q) __attribute__((always_inline)) -> const float4* {
            return reinterpret_cast<const float4*>(kDma ? stg + 4 * (8 * k + (q ^ ((k >> 1) & 7))) : stg + k * kStride + 4 * q);
        };
        struct Pre { float2 v[2 * kIt]; float wa, wb; };
        const float4* smp4 = reinterpret_cast<const float4*>(p.smp);
        float4 smn = smp4[s2];
        // LDS-DMA of chunk ch: instruction it covers keypoints 8 it .. 8 it + 7, lane
        // (kl, x) fetches the 16 bytes of pair x ^ swz(keypoint) -- the schedule pairs
        // horizontally adjacent pixels (sift_band_prepare), so a pair is one load
        auto issue_dma = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const int kp = kPer * it + kl;
                const float4 sm = smp4[ch * kPairs + (s2 ^ ((kp >> 1) & 7))];
                const char* src = p.grad + (kof[it] + (unsigned)__float_as_int(sm.y));
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 (__attribute__((address_space(3))) void*)(stg + it * 256),
                                                 16, 0, 0);
            }
        };
        auto issue = [&](int ch, Pre& pf) __attribute__((always_inline)) {
            const float4 sm = smn;
            pf.wa = sm.x;
            pf.wb = sm.z;
            const unsigned soa = (unsigned)__float_as_int(sm.y), sob = (unsigned)__float_as_int(sm.w);
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                pf.v[2 * it] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + soa));
                pf.v[2 * it + 1] = *reinterpret_cast<const float2*>(p.grad + (kof[it] + sob));
            }
            smn = smp4[min(ch + 1, nch - 1) * kPairs + s2];
        };
        auto stage = [&](const Pre& pf) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const float2 a = pf.v[2 * it], b = pf.v[2 * it + 1];
                const float mwa = __fmul_rn(a.x, pf.wa), mwb = __fmul_rn(b.x, pf.wb);
                const float oba = kObin ? a.y : __fmul_rn(__fsub_rn(a.y, ori_deg), bins_per_rad);
                const float obb = kObin ? b.y : __fmul_rn(__fsub_rn(b.y, ori_deg), bins_per_rad);
                *reinterpret_cast<float4*>(stg + (kPer * it + kl) * kStride + 4 * s2) = make_float4(mwa, mwb, oba, obb);
            }
        };

        float raw[4][2][4];             // this lane's quarter of the histogram: rows 0..3, columns 2 dc + k2, bins 4 dp ..
// half a chunk's wave-uniform table in SGPRs: rf, cf, slot offset (16-keypoint
// layout) and weight of 8 samples, one wait for the four scalar loads
#define SIFT_BAND4_TABLE_LOAD(trf, tcf, tof, tw, sp)            \
        __asm__ volatile(                                       \
            "s_load_dwordx8 %0, %4, 0x0\n\t"                    \
            "s_load_dwordx8 %1, %4, 0x40\n\t"                   \
            "s_load_dwordx8 %2, %4, 0xc0\n\t"                   \
            "s_load_dwordx8 %3, %4, 0x100\n\t"                  \
            "s_waitcnt lgkmcnt(0)"                              \
            : "=&s"(trf), "=&s"(tcf), "=&s"(tof), "=&s"(tw)     \
            : "s"(sp))
        static_assert(kKS == 16 && kTabCols == 5, "table layout of SIFT_BAND4_TABLE_LOAD");
        auto o0_of = [&](float ob) __attribute__((always_inline)) {
            int o0;
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));
            if (!kNeg) {
                o0 += o0 < 0 ? 8 : 0;
                o0 -= o0 >= 8 ? 8 : 0;
            }
            return o0;
        };
        // sample qq (0..7) of half hf: its weighted magnitude and obin from the
        // staged record pair (r: records of the half's four pairs)
        auto sample = [&](const float4 (&r)[kPairs / 2], int qq, const i8v& tw, float& mw, float& ob)
            __attribute__((always_inline)) {
            const float4 x = r[qq >> 1];
            if constexpr (kDma) {
                const float mag = (qq & 1) ? x.z : x.x, o = (qq & 1) ? x.w : x.y;
                mw = __fmul_rn(mag, __int_as_float(tw[qq]));
                ob = kObin ? o : __fmul_rn(__fsub_rn(o, ori_deg), bins_per_rad);
            } else {
                mw = (qq & 1) ? x.y : x.x;
                ob = (qq & 1) ? x.w : x.z;
            }
        };
        auto load_half = [&](float4 (&r)[kPairs / 2], int hf) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < kPairs / 2; q++) r[q] = *rec(kq, hf * (kPairs / 2) + q);
        };
        // ---- bands 0..2: slot pairs {row r0, row r0 + 1}; half a chunk at a time ----
        auto walk_pair = [&](int ch, float4 (&rr)[2][kPairs / 2]) __attribute__((always_inline)) {
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                i8v trf, tcf, tof, tw;
                SIFT_BAND4_TABLE_LOAD(trf, tcf, tof, tw, p.smp_s + ch * (kTabCols * kKS) + hf * (kKS / 2));
                if constexpr (!kDma) load_half(rr[hf], hf);
#pragma unroll
              for (int qt = 0; qt < 2; qt++) {       // two batches of 4 samples (register budget)
                f2v val[kKS / 2];
                char* tp[kKS / 2];
#pragma unroll
                for (int qq = 4 * qt; qq < 4 * qt + 4; qq++) {
                    float mw, ob;
                    sample(rr[hf], qq, tw, mw, ob);
                    const float frac = __builtin_amdgcn_fractf(ob);
                    const int o0 = o0_of(ob);
                    tp[qq] = lb + tof[qq] + __mul24(o0, kPosF * 4);
                    const float v_r1 = __fmul_rn(mw, __int_as_float(trf[qq]));
                    const f2v vr = {__fsub_rn(mw, v_r1), v_r1};
                    const f2v cf2 = {__int_as_float(tcf[qq]), __int_as_float(tcf[qq])};
                    const f2v c1 = vr * cf2;
                    const f2v cv = __builtin_elementwise_fma(c1, kn2, vr * km2);
                    const f2v fr = {frac, frac};
                    const f2v hi = cv * fr;
                    val[qq] = __builtin_elementwise_fma(hi, sn2, cv * sm2);
                }
#pragma unroll
                for (int qq = 4 * qt; qq < 4 * qt + 4; qq++) {
                    auto t = (__attribute__((address_space(3))) volatile f2v*)(tp[qq]);
                    f2v a = t[0];
                    a = a + val[qq];
                    t[0] = a;
                }
              }
            }
            wave_sync();
        };
        // ---- bands -1 and 3: one kept row, one-row layout, two samples per packed op ----
        auto walk_one = [&](int ch, float4 (&rr)[2][kPairs / 2], auto upper) __attribute__((always_inline)) {
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                i8v trf, tcf, tof, tw;
                SIFT_BAND4_TABLE_LOAD(trf, tcf, tof, tw, p.smp_s + ch * (kTabCols * kKS) + hf * (kKS / 2));
                if constexpr (!kDma) load_half(rr[hf], hf);
#pragma unroll
              for (int qt = 0; qt < 2; qt++) {
                float val[kKS / 2];
                char* tp[kKS / 2];
#pragma unroll
                for (int q2 = 2 * qt; q2 < 2 * qt + 2; q2++) {
                    const int qa = 2 * q2, qb = qa + 1;
                    float mwa, mwb, oba, obb;
                    sample(rr[hf], qa, tw, mwa, oba);
                    sample(rr[hf], qb, tw, mwb, obb);
                    const f2v mw2 = {mwa, mwb};
                    const f2v fr2 = {__builtin_amdgcn_fractf(oba), __builtin_amdgcn_fractf(obb)};
                    tp[qa] = lb1 + tof[qa] + __mul24(o0_of(oba), kPos1F * 4);
                    tp[qb] = lb1 + tof[qb] + __mul24(o0_of(obb), kPos1F * 4);
                    const f2v rf2 = {__int_as_float(trf[qa]), __int_as_float(trf[qb])};
                    const f2v cf2 = {__int_as_float(tcf[qa]), __int_as_float(tcf[qb])};
                    const f2v v_r1 = mw2 * rf2;
                    const f2v v = decltype(upper)::value ? v_r1 : mw2 - v_r1;
                    const f2v c1 = v * cf2;
                    const f2v cv = __builtin_elementwise_fma(c1, kn2, v * km2);
                    const f2v h = cv * fr2;
                    const f2v vv = __builtin_elementwise_fma(h, sn2, cv * sm2);
                    val[qa] = vv.x;
                    val[qb] = vv.y;
                }
#pragma unroll
                for (int qq = 4 * qt; qq < 4 * qt + 4; qq++) {
                    auto t = (__attribute__((address_space(3))) volatile float*)(tp[qq]);
                    t[0] = __fadd_rn(t[0], val[qq]);
                }
              }
            }
            wave_sync();
        };
#undef SIFT_BAND4_TABLE_LOAD
        // the finished row: columns 2 dc + k2, bins 4 dp .. 4 dp + 3 (slot s of a
        // column at position s + 1; slot 8 (position 9) wraps into bin 0, slot 9
        // is position 0 of the next column (col' - 1) and wraps into bin 1)
        auto take_row = [&](float (&f)[2][4], const float* c0p, int ps, int cs) __attribute__((always_inline)) {
#pragma unroll
            for (int k2 = 0; k2 < 2; k2++) {
                const float* c = c0p + (4 - (2 * dc + k2)) * cs;
                const float* cb = c + 4 * dp * ps;
                const float w0 = c[9 * ps], w1 = c[-cs];
                f[k2][0] = __fadd_rn(cb[1 * ps], dp ? 0.f : w0);
                f[k2][1] = __fadd_rn(cb[2 * ps], dp ? 0.f : w1);
                f[k2][2] = cb[3 * ps];
                f[k2][3] = cb[4 * ps];
            }
        };
        // the one-row slots (or the pairs' second elements) of columns 3 dc .. 3 dc + 2,
        // positions 5 dp .. 5 dp + 4: one lane's share of a layout move
        auto close_band = [&](auto B) __attribute__((always_inline)) {
            constexpr int b = decltype(B)::value;
            if constexpr (b == -1) {
                float v[3][5];
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int ps = 0; ps < 5; ps++) v[c][ps] = buf[(5 * dp + ps) * kPos1F + (3 * dc + c) * kCol1F + kq];
                wave_sync();
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int ps = 0; ps < 5; ps++)
                        *reinterpret_cast<float2*>(buf + (5 * dp + ps) * kPosF + (3 * dc + c) * kColF + 2 * kq) =
                            make_float2(v[c][ps], 0.f);
            } else if constexpr (b <= 2) {
                take_row(raw[b], buf + 2 * kq, kPosF, kColF);
                wave_sync();
                if constexpr (b < 2) {
                    float2* z = reinterpret_cast<float2*>(buf);
#pragma unroll 5
                    for (int q = 0; q < kSlots / 128; q++) {
                        float2 vv = z[q * 64 + lane];
                        z[q * 64 + lane] = make_float2(vv.y, 0.f);
                    }
                } else {
                    float v[3][5];
#pragma unroll
                    for (int c = 0; c < 3; c++)
#pragma unroll
                        for (int ps = 0; ps < 5; ps++)
                            v[c][ps] = reinterpret_cast<const float2*>(buf + (5 * dp + ps) * kPosF + (3 * dc + c) * kColF + 2 * kq)->y;
                    wave_sync();
#pragma unroll
                    for (int c = 0; c < 3; c++)
#pragma unroll
                        for (int ps = 0; ps < 5; ps++) buf[(5 * dp + ps) * kPos1F + (3 * dc + c) * kCol1F + kq] = v[c][ps];
                }
            } else {
                take_row(raw[3], buf + kq, kPos1F, kCol1F);
            }
            wave_sync();
        };

        // register staging: chunk ch + 1's loads in flight while ch is walked, staged
        // after it.  LDS-DMA staging: chunk ch's records are read into registers first,
        // then chunk ch + 1's DMA is issued into the same buffer and lands while ch is
        // walked (waited for, vmcnt(0), before its records are read)
        Pre pf;
        float4 rr[2][kPairs / 2];
        if constexpr (kDma) {
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the stage area's earlier readers
            issue_dma(0);
        } else {
            issue(0, pf);
            stage(pf);
            wave_sync();
        }
        auto run_band = [&](auto B) __attribute__((always_inline)) {
            constexpr int b = decltype(B)::value;
            const int ch_end = p.band_first[b + 2];
            for (int ch = p.band_first[b + 1]; ch < ch_end; ch++) {
                if constexpr (kDma) {
                    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    load_half(rr[0], 0);
                    load_half(rr[1], 1);
                    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (ch + 1 < nch) issue_dma(ch + 1);
                } else {
                    if (ch + 1 < nch) issue(ch + 1, pf);
                }
                if constexpr (b == -1)
                    walk_one(ch, rr, std::true_type{});
                else if constexpr (b == 3)
                    walk_one(ch, rr, std::false_type{});
                else
                    walk_pair(ch, rr);
                if (ch + 1 == ch_end) close_band(B);
                if constexpr (!kDma) {
                    if (ch + 1 < nch) {
                        stage(pf);
                        wave_sync();
                    }
                }
            }
        };
        run_band(std::integral_constant<int, -1>{});
        run_band(std::integral_constant<int, 0>{});
        run_band(std::integral_constant<int, 1>{});
        run_band(std::integral_constant<int, 2>{});
        run_band(std::integral_constant<int, 3>{});

        // ---- epilogue: raw histogram to LDS, one lane per keypoint ----
        wave_sync();
        if constexpr (kDma) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA left in flight
        {
            float* rb = buf + kq * kRawStride;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++)
#pragma unroll
                    for (int q = 0; q < 4; q++) rb[(r * 4 + 2 * dc + k2) * 8 + 4 * dp + q] = raw[r][k2][q];
        }
        wave_sync();
        if (lane < kKpW) {
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

// SLAMHIP_SIFT_BAND4=0 (default) selects the 32-keypoint band kernel, =1 the
// 16-keypoint one with register staging, =2 with LDS-DMA staging (the same
// descriptors; r4ab on MI355X, 210 x 10.1k keypoints: 11.76 / 13.97 / 13.87 ms)
int sift_band4_mode()
{
    static const int mode = [] {
        const char* e = getenv("SLAMHIP_SIFT_BAND4");
        return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 0;
    }();
    return mode;
}

// SLAMHIP_SIFT_STAGEPOS=1: the band kernel's stage lanes form fract(obin) and the
// slot-position byte (the position-plane walk without the byte plane; A/B)
bool sift_band_stagepos()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_SIFT_STAGEPOS"); return e && e[0] == '1'; }();
    return on;
}
bool sift_band4_dma() { return sift_band4_mode() == 2; }

}  // namespace

bool sift_band4_enabled() { return sift_band4_mode() >= 1; }

// the gradient map form the band kernel takes (launch_sift_base's obin): 1
// (obin), or with SLAMHIP_SIFT_POSPLANE=1 (read per launch) 2, fract(obin) plus
// the slot-position byte plane, for the 32-keypoint kernel on a kNeg table.
// Mode 2 takes 2 VALU per lane-sample out of the walk (fract, floor, multiply
// -> one byte permute) but adds a 2-byte load and a 2-byte LDS store per
// staged sample pair: 12.20 against 11.76 ms per 210-frame launch (r4e,
// bit-exact both ways), so it is off by default
int sift_band_obin_mode(const slam_ctx* c)
{
    const char* e = getenv("SLAMHIP_SIFT_POSPLANE");
    const bool plane = e && e[0] == '1';
    return plane && c->sift_band.neg && !sift_band4_enabled() ? 2 : 1;
}

int sift_band_radius(float kp_size)
{
    const float hist_width = 3.f * (kp_size * 0.5f);
    return (int)std::lrintf(hist_width * 1.4142135623730951f * (4 + 1) * 0.5f);
}

// The window samples of a keypoint of one (angle, size), in raster order (the
// reference's calcSIFTDescriptor loop), with the host's float operation order.
bool sift_band_geometry(slam_ctx* c, float kp_angle, float kp_size, int w, int h, BandGeometry& g)
{
    float angle = 360.f - kp_angle;
    if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    const float ori = angle;
    float cos_t = cosf(ori * (float)(M_PI / 180));
    float sin_t = sinf(ori * (float)(M_PI / 180));
    const float exp_scale = -1.f / (4 * 4 * 0.5f);
    const float hist_width = 3.f * (kp_size * 0.5f);
    const int radius = sift_band_radius(kp_size);
    const int diag = (int)std::sqrt((double)w * w + (double)h * h);
    if (radius > diag || radius > kGradPad || w < 3 || h < 3) return false;   // window inside the zero border
    if (c->grad.bytes > 0xffffffffull) return false;                          // 32-bit byte offsets
    cos_t /= hist_width;
    sin_t /= hist_width;
    g.radius = radius;
    g.ori = ori;
    g.pitch = grad_pitch(w);
    g.smp.clear();
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(4 / 2) - 0.5f;
            const float cbin = c_rot + (float)(4 / 2) - 0.5f;
            if (!(rbin > -1 && rbin < 4 && cbin > -1 && cbin < 4)) continue;
            const float wexp = host_exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, c->sift.exptab);
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            g.smp.push_back({i, j, r0, c0, rbin - (float)r0, cbin - (float)c0, wexp});
        }
    // obin = (ori_k - ori) * 8/360 over ori_k in [0, 360] (fastAtan2's range):
    // neg when floor(obin) always lies in [-9, -1] (one wrap, no branch)
    const float bpr = 8 / 360.f;
    const float ob_lo = (0.f - ori) * bpr, ob_hi = (360.f - ori) * bpr;
    g.neg = std::floor(ob_lo) >= -9.f && std::floor(ob_hi) <= -1.f;
    g.pos_base = g.neg ? 9 : 1;   // slot position = floor(obin) + pos_base (wrapped when !neg)
    return true;
}

// Every target cell's visit sequence in `sched` (sample indices, < 0 = dummy)
// must be its raster-order sequence: then each bin's additions happen in the
// reference's order.
bool sift_band_raster_ok(const BandGeometry& g, const std::vector<int>& sched)
{
    const int n = (int)g.smp.size();
    for (int R = 1; R <= 4; R++)
        for (int C = 0; C <= 5; C++) {
            std::vector<int> ras, sc;
            auto hits = [&](const BandSample& q) {
                const int dr = R - 1 - q.r0, dc = C - 1 - q.c0;
                return dr >= 0 && dr <= 1 && dc >= 0 && dc <= 1;
            };
            for (int q = 0; q < n; q++) if (hits(g.smp[q])) ras.push_back(q);
            for (int q : sched) if (q >= 0 && hits(g.smp[q])) sc.push_back(q);
            if (ras != sc) return false;
        }
    return true;
}

// Build (or reuse) the band tables for keypoints of one (angle, size); false
// when the band order does not reproduce some target's raster order or the
// tables do not fit (sift_tab / the general kernel then run).
bool sift_band_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h)
{
    const bool cols = sift_cols_enabled() || c->opt_sift_kernel == SLAM_SIFT_KERNEL_COLS;
    const bool colw = (c->opt_sift_kernel == SLAM_SIFT_KERNEL_AUTO && sift_colw_enabled()) ||
                      c->opt_sift_kernel == SLAM_SIFT_KERNEL_COLW;
    if (c->opt_sift_kernel != SLAM_SIFT_KERNEL_AUTO && c->opt_sift_kernel != SLAM_SIFT_KERNEL_BAND &&
        c->opt_sift_kernel != SLAM_SIFT_KERNEL_COLS && c->opt_sift_kernel != SLAM_SIFT_KERNEL_COLW)
        return false;
    if (c->sift_band_valid && c->sift_band_angle == kp_angle && c->sift_band_size == kp_size &&
        c->sift_band.radius == sift_band_radius(kp_size) && c->sift_band.pitch == grad_pitch(w) &&
        (!cols || c->sift_cols_valid) && (!colw || c->sift_colw_valid))
        return true;
    // the tables of the column kernels follow the band tables: stale ones of an
    // earlier geometry must not survive a rebuild that does not make them
    c->sift_cols_valid = false;
    c->sift_colw_valid = false;
    BandGeometry geo;
    if (!sift_band_geometry(c, kp_angle, kp_size, w, h, geo)) return false;
    const std::vector<BandSample>& smp = geo.smp;
    const int n = (int)smp.size();
    // band-major order (stable by r0)
    std::vector<int> ord(n);
    for (int k = 0; k < n; k++) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return smp[a].r0 < smp[b].r0; });
    // schedule: band-major (stable).  Samples go in pairs (2 m, 2 m + 1) of
    // horizontally adjacent pixels (i, j), (i, j + 1) -- the LDS-DMA stage fetches a
    // pair as one 16-byte load -- so a sample whose left neighbour in its pair
    // would not be adjacent gets a zero-weight dummy at that neighbour's pixel
    // instead; each band is padded to whole chunks with dummy pairs at the
    // keypoint.  A dummy adds +0 wherever it points: every bin unchanged.
    struct Ent { int v, i, j; };      // v: sample index, or -1 for a dummy at pixel (i, j)
    std::vector<Ent> fin;
    std::vector<int> band_len(5, 0);
    {
        int k = 0;
        for (int b = -1; b <= 3; b++) {
            const size_t start = fin.size();
            while (k < n && smp[ord[k]].r0 == b) {
                const BandSample& sm = smp[ord[k]];
                if ((fin.size() - start) % 2 == 1) {
                    const Ent& a = fin.back();
                    if (!(sm.i == a.i && sm.j == a.j + 1)) fin.push_back({-1, a.i, a.j + 1});
                }
                fin.push_back({ord[k++], sm.i, sm.j});
            }
            if ((fin.size() - start) % 2 == 1) fin.push_back({-1, fin.back().i, fin.back().j + 1});
            while ((fin.size() - start) % kKS) {
                fin.push_back({-1, 0, 0});
                fin.push_back({-1, 0, 1});
            }
            band_len[b + 1] = (int)(fin.size() - start);
        }
        if (k != n) return false;
    }
    // every band must hold a chunk: the kernel closes a band (moves its finished
    // descriptor row to registers, shifts the slot rows) after the band's last
    // chunk, so an empty band (tiny keypoints: bands -1 / 3 unreached) would leave
    // its row unset -- sift_tab / the general kernel take such keypoints
    for (int b = 0; b < 5; b++)
        if (band_len[b] == 0) return false;
    {
        std::vector<int> order(fin.size());
        for (size_t q = 0; q < fin.size(); q++) order[q] = fin[q].v;
        if (!sift_band_raster_ok(geo, order)) return false;
    }
    const int radius = geo.radius;
    const float ori = geo.ori;
    const bool neg = geo.neg;
    // chunks of kKS consecutive scheduled samples of one band.  Two tables: per sample
    // {weight, window byte offset} (vector loads of the staging lanes) and per
    // chunk [rf x kKS][cf x kKS][slot byte offset x kKS] (scalar loads of the walk)
    const int pitch = geo.pitch;
    const int pos_base = geo.pos_base;
    std::vector<float2> tv;
    std::vector<int32_t> ts;
    int band_first[6];
    auto f2i = [](float f) { union { float f; int32_t i; } u; u.f = f; return u.i; };
    auto i2f = [](int32_t i) { union { int32_t i; float f; } u; u.i = i; return u.f; };
    // slot offsets: the pair layout in bands 0..2, the one-row layout in bands -1 and 3
    auto push = [&](float rf, float cf, float wexp, int i, int j, int c0, bool one_row) {
        if (tv.size() % kKS == 0) ts.resize(ts.size() + kTabCols * kKS, 0);
        const size_t q = tv.size() % kKS, base = ts.size() - kTabCols * kKS;
        tv.push_back(make_float2(wexp, i2f((i * pitch + j) * 8)));
        ts[base + q] = f2i(rf);
        ts[base + kKS + q] = f2i(cf);
        // slot byte offset of column c0 + 1 at position pos_base, in the slot layout of
        // each kernel variant (dc = 1 lanes add one column: column c0)
        ts[base + 2 * kKS + q] = 4 * (one_row ? (4 - (c0 + 1)) * 32 + pos_base * kPos1F : (4 - (c0 + 1)) * 64 + pos_base * kPosF);
        ts[base + 3 * kKS + q] = 4 * (one_row ? (4 - (c0 + 1)) * q4::kCol1F + pos_base * q4::kPos1F
                                              : (4 - (c0 + 1)) * q4::kColF + pos_base * q4::kPosF);
        ts[base + 4 * kKS + q] = f2i(wexp);           // the DMA-staged walk multiplies it in
    };
    {
        size_t q = 0;
        for (int b = -1; b <= 3; b++) {
            band_first[b + 1] = (int)(tv.size() / kKS);
            for (int e = 0; e < band_len[b + 1]; e++, q++) {
                const int v = fin[q].v;
                const bool one_row = b == -1 || b == 3;
                if (v >= 0) {
                    const BandSample& sm = smp[v];
                    push(sm.rf, sm.cf, sm.wexp, sm.i, sm.j, sm.c0, one_row);
                } else {
                    push(0.f, 0.f, 0.f, fin[q].i, fin[q].j, 0, one_row);   // weight 0: +0
                }
            }
        }
    }
    const int nchunks = (int)(tv.size() / kKS);
    band_first[5] = nchunks;
    if (nchunks > kMaxChunks) return false;
    const size_t b_v = tv.size() * sizeof(float2), b_s = ts.size() * sizeof(int32_t);
    if (c->sift_band_buf.ensure(b_v + b_s) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_band_buf.p, tv.data(), b_v, hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_band_buf.as<char>() + b_v, ts.data(), b_s, hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    SiftBandMeta& m = c->sift_band;
    m.nrec = (int)tv.size();
    m.nchunks = nchunks;
    m.pitch = pitch;
    m.neg = neg;
    for (int q = 0; q < 6; q++) m.band_first[q] = band_first[q];
    m.radius = radius;
    m.ori_deg = ori;
    if (cols) sift_cols_prepare(c, s, geo);   // the A/B kernel's tables (sift_cols.hip)
    if (colw) sift_colw_prepare(c, s, geo);   // sift_colw.hip
    c->sift_band_valid = true;
    c->sift_band_angle = kp_angle;
    c->sift_band_size = kp_size;
    return true;
}

hipError_t launch_sift_desc_band(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32, int obin)
{
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    const SiftBandMeta& m = c->sift_band;
    BandParams p;
    bool split_ok = false;
    // SLAM_OPT_SIFT_BAND_SPLIT; SLAMHIP_SIFT_BAND_SPLIT=0/1/2 overrides it (timing A/B)
    static const int env_split = [] {
        const char* e = getenv("SLAMHIP_SIFT_BAND_SPLIT");
        return e && e[0] >= '0' && e[0] <= '3' ? e[0] - '0' : -1;
    }();
    const int band_split = env_split >= 0 ? env_split : c->opt_band_split;
    p.grad = c->grad.as<char>();
    p.frame_bytes = grad_frame(w, h) * 8;
    p.origin_bytes = grad_origin(w) * 8;
    p.pitch_bytes = grad_pitch(w) * 8;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.smp = c->sift_band_buf.as<float2>();
    p.smp_s = reinterpret_cast<const int*>(c->sift_band_buf.as<char>() + (size_t)m.nrec * sizeof(float2));
    p.nchunks = m.nchunks;
    for (int q = 0; q < 6; q++) p.band_first[q] = m.band_first[q];
    p.ori_deg = m.ori_deg;
    p.posb = c->gradpos.as<uint8_t>();
    if (obin == 2 && (sift_band4_enabled() || !p.posb)) return hipErrorInvalidValue;
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    {
        static const int wm = [] { const char* e = getenv("SLAMHIP_SIFT_BAND_ORDER"); return e && e[0] == '0' ? 0 : 1; }();
        static const int pe = [] { const char* e = getenv("SLAMHIP_SIFT_BAND_PARTS"); return e ? atoi(e) : 0; }();
        p.wave_major = wm;
        p.parts_env = pe == 2 || pe == 4 ? pe : 0;
        p.split = 0;
        p.split_raw = nullptr;
        p.split_cnt = nullptr;
        split_ok = wm && band_split != SLAM_BAND_SPLIT_OFF;
    }
    // persistent: one 8-wave workgroup per CU (157 KB of LDS; band4: two of 80 KB),
    // a multiple of 8 workgroups for the XCD split
    const bool b4 = sift_band4_enabled();
    int grid = b4 ? 2 * c->cu_count : c->cu_count;
    const int kpb = b4 ? q4::kKpW * q4::kWaves : kKpW * kWaves;
    const int need = (cap + kpb - 1) / kpb;
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    if (split_ok && !b4) {
        // split slots: 8 XCD ranges x (waves per range) / 2; counters zeroed when
        // the buffer is (re)allocated, and reset by the kernel after each use
        const size_t slots = band_split >= SLAM_BAND_SPLIT_ALL ? (size_t)(cap + kKpW - 1) / kKpW + 8 : (size_t)grid;
        if ((e = c->sift_split.ensure(slots * 4 * 64 * 4 * sizeof(float4))) != hipSuccess) return e;
        const size_t before = c->sift_split_cnt.bytes;       // grows only on reallocation
        if ((e = c->sift_split_cnt.ensure(slots * sizeof(int))) != hipSuccess) return e;
        if (c->sift_split_cnt.bytes != before &&
            (e = hipMemsetAsync(c->sift_split_cnt.p, 0, c->sift_split_cnt.bytes, s)) != hipSuccess)
            return e;
        p.split = band_split;
        p.split_raw = c->sift_split.as<float4>();
        p.split_cnt = c->sift_split_cnt.as<int>();
    }
    prof_begin(c, 1, s);
    if (!b4 && obin == 1 && m.neg && c->sift_colw_valid &&
        ((c->opt_sift_kernel == SLAM_SIFT_KERNEL_AUTO && sift_colw_enabled()) ||
         c->opt_sift_kernel == SLAM_SIFT_KERNEL_COLW)) {
        // one descriptor column per wave (sift_colw.hip), the default for FAST
        // keypoints; SLAM_SIFT_KERNEL_BAND forces sift_desc_band
        e = launch_sift_desc_colw(c, s, w, h, cap, write_f32);
        prof_end(c, 1, s);
        return e;
    }
    if (!b4 && obin == 1 && m.neg && c->sift_cols_valid &&
        (sift_cols_enabled() || c->opt_sift_kernel == SLAM_SIFT_KERNEL_COLS)) {
        // SLAM_SIFT_KERNEL_COLS / SLAMHIP_SIFT_COLS=1: one keypoint per lane, two
        // column passes (A/B; measured slower)
        e = launch_sift_desc_cols(c, s, w, h, cap, write_f32);
        prof_end(c, 1, s);
        return e;
    }
    if (b4 && sift_band4_dma()) {
        if (m.neg && obin)
            hipLaunchKernelGGL((sift_desc_band4<true, true, true>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else if (m.neg)
            hipLaunchKernelGGL((sift_desc_band4<true, false, true>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else if (obin)
            hipLaunchKernelGGL((sift_desc_band4<false, true, true>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else
            hipLaunchKernelGGL((sift_desc_band4<false, false, true>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
    } else if (b4) {
        if (m.neg && obin)
            hipLaunchKernelGGL((sift_desc_band4<true, true, false>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else if (m.neg)
            hipLaunchKernelGGL((sift_desc_band4<true, false, false>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else if (obin)
            hipLaunchKernelGGL((sift_desc_band4<false, true, false>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
        else
            hipLaunchKernelGGL((sift_desc_band4<false, false, false>), dim3(grid), dim3(64 * q4::kWaves), 0, s, p);
    } else if (m.neg && obin == 2)
        hipLaunchKernelGGL((sift_desc_band<true, 2>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (m.neg && obin == 1 && sift_band_stagepos())
        hipLaunchKernelGGL((sift_desc_band<true, 3>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (obin == 2)
        return hipErrorInvalidValue;             // the position plane is built for floor(obin) in [-9, -1]
    else if (m.neg && obin)
        hipLaunchKernelGGL((sift_desc_band<true, 1>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (m.neg)
        hipLaunchKernelGGL((sift_desc_band<true, 0>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else if (obin)
        hipLaunchKernelGGL((sift_desc_band<false, 1>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    else
        hipLaunchKernelGGL((sift_desc_band<false, 0>), dim3(grid), dim3(64 * kWaves), 0, s, p);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
