// SIFT descriptors of FAST keypoints (one angle and size): one keypoint per
// lane, the histogram's columns in two passes.
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) adds every window sample into the 8 bins of
// the 2 x 2 x 2 histogram cells around it, in raster sample order; each bin's
// float additions must happen in that order for bit-exact descriptors.
//
// sift_desc_band (sift_band.hip) gives a keypoint two lanes, one per footprint
// column: every value a sample needs (the row split, the orientation fraction,
// the slot address) is formed on both lanes, 26 VALU per keypoint-sample, and
// the two lanes each do one read-add-write pair whether their column is inside
// the descriptor or not (the c0 = -1 samples' column -1 and the c0 = 3
// samples' column 4 are written and never read, except column 4's position 0,
// the quirk slot of the 361-degree angle).  Here one lane owns a keypoint
// (64 per wave) and updates both columns of its sample: 16 VALU per
// keypoint-sample, and only the columns the descriptor needs.  Both columns'
// slots of 64 keypoints would leave one wave per SIMD (30 KB), so a keypoint
// group is walked twice:
//   pass 0: descriptor columns 0, 1 -- samples with c0 in {-1, 0, 1};
//   pass 1: descriptor columns 2, 3 -- samples with c0 in {1, 2, 3}; column
//           4's position 0 (= column 3's slot 9, the o0 = -1 share) is a
//           register per row, added with a select (+0 otherwise: exact).
// A pass holds two columns' slots (10 KB per wave); the c0 = 1 samples (one
// fifth) are evaluated in both passes.  Every pass contains every sample that
// reaches its target cells, in band order, which is their raster order (the
// host checks it per target), so each bin sums in the reference's order.
// Column 1's bin 1 is slot 1 + slot 9, and its slot 9 is column 2's position
// 0: pass 0 keeps slot 1, pass 1 adds slot 9 when it takes column 2's rows
// (one addition, as the reference's fold).
//
// Per wave: slots pos * 256 + col * 128 + 2 * lane + row (row pair {r0, r0 +
// 1} of a band as one 8-byte ds_read_b64 / ds_write_b64; banks 2 * lane (+1):
// conflict-free whatever the data-dependent position), the stage (16 window
// samples of 64 keypoints, {mw, obin} pairs, the band kernel's staging), the
// keypoints' window offsets.  8 waves per CU (157.7 KB).  The finished
// histogram stays in registers: the epilogue needs no LDS round trip.
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

#ifndef SIFT_COLS_SCHED
#define SIFT_COLS_SCHED 1
#endif
#ifndef SIFT_COLS_KS
#define SIFT_COLS_KS 16
#endif
#ifndef SIFT_COLS_WAVES
#define SIFT_COLS_WAVES 8
#endif
constexpr int kKS = SIFT_COLS_KS;          // window samples per staged chunk
constexpr int kStride = 2 * kKS + 4;       // stage floats per keypoint (16-byte rows, b128 conflict-free)
constexpr int kWaves = SIFT_COLS_WAVES;
constexpr int kKpW = 64;                   // keypoints per wave: lane = keypoint
constexpr int kPos = 10;                   // slot positions: 0 = the left cell's slot 9, 1..9 = slots 0..8
constexpr int kColF = 2 * kKpW;            // floats per (position, column): 64 lanes x 2 rows
constexpr int kPosF = 2 * kColF;           // two columns per pass
constexpr int kSlots = kPos * kPosF;
constexpr int kStageOff = kSlots;
constexpr int kKpOff = kStageOff + kKpW * kStride;
constexpr int kWaveFloats = kKpOff + kKpW;
constexpr int kTabDw = 2 * kKS + 2;       // per chunk: rf[kKS], cf[kKS], classes (4 bits per sample, 2 dwords)
constexpr int kMaxChunks = 1024;
constexpr int kPosBase = 9;                // position = floor(obin) + 9 (floor(obin) in [-9, -1])
static_assert(kWaves * kWaveFloats * 4 <= 160 * 1024, "LDS");
static_assert(kStageOff % 4 == 0 && kStride % 4 == 0 && kWaveFloats % 4 == 0, "16-byte stage rows");
// sample classes (wave-uniform, from the table): which of the sample's two
// footprint columns this pass updates
constexpr int kClsLeft = 1;                // column c0 (slot pairs in LDS)
constexpr int kClsRight = 2;               // column c0 + 1 (slot pairs in LDS)
constexpr int kClsQuirk = 4;               // column c0 + 1 = 4: position 0 only, in a register

struct ColsParams {
    const char* grad;                      // padded gradient map (bytes), obin form
    size_t frame_bytes, origin_bytes;
    int pitch_bytes;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float2* smp;                     // [nchunks * kKS] {weight, window byte offset}
    const int* smp_s;                      // [nchunks][kTabDw]: rf, cf, packed classes
    float4* park;                          // pass 0's finished rows: [wave slot][16 float4][64 lanes] per row
    int nchunks;
    int band_first[2][6];                  // pass p, band b: first chunk at band_first[p][b + 1]
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef int i16v __attribute__((ext_vector_type(16)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) volatile f2v lds_f2v;

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

__global__ __launch_bounds__(64 * kWaves) void sift_desc_cols(ColsParams p)
{
    __shared__ __attribute__((aligned(16))) float s_buf[kWaves][kWaveFloats];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* buf = s_buf[wave];
    float* stg = buf + kStageOff;
    unsigned* kpo = reinterpret_cast<unsigned*>(buf + kKpOff);

    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int ngroups = (total + kKpW - 1) / kKpW;
    // XCD-aware, wave-major group order (sift_desc_band): each XCD walks a compact
    // raster range, and a launch's last partial round spreads over its CUs
    const int xg = blockIdx.x & 7;
    const int nw = (gridDim.x >> 3) * kWaves;
    const int wi = wave * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int per = (ngroups + 7) >> 3;
    const int g_end = min(ngroups, (xg + 1) * per);
    const int nch = p.nchunks;
    // stage mapping: lane loads window samples 2 s2 and 2 s2 + 1 of keypoints kPer * it + kl
    constexpr int kPairs = kKS / 2, kPer = 64 / kPairs, kIt = kKpW / kPer;
    const int s2 = lane % kPairs, kl = lane / kPairs;
    char* lb = reinterpret_cast<char*>(buf + 2 * lane);
    const float4* smp4 = reinterpret_cast<const float4*>(p.smp);

    for (int grp = xg * per + wi; grp < g_end; grp += nw) {
        const int g = grp * kKpW + lane;
        const bool act = g < total;
        {
            // byte offset of the keypoint's pixel in the padded map (< 4 GiB: checked on the host)
            const int gg = min(g, total - 1);
            const slam_keypoint kp = p.kps[gg];
            const int ptx = __float2int_rn(kp.x), pty = __float2int_rn(kp.y);
            kpo[lane] = (unsigned)((size_t)p.kp_frame[gg] * p.frame_bytes + p.origin_bytes) +
                        (unsigned)(pty * p.pitch_bytes + ptx * 8);
        }
        wave_sync();
        unsigned kof[kIt];
#pragma unroll
        for (int it = 0; it < kIt; it++) kof[it] = kpo[kPer * it + kl];

        // ---- prefetch of one chunk: kIt x kPer keypoints x kKS window samples ----
        struct Pre { float2 v[2 * kIt]; float wa, wb; };
        float4 smn = smp4[s2];
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
            smn = smp4[min(ch + 1, nch - 1) * kPairs + s2];
        };
        // stage record of a sample pair: {mw_q, mw_q+1, obin_q, obin_q+1}
        auto stage = [&](const Pre& pf) __attribute__((always_inline)) {
#pragma unroll
            for (int it = 0; it < kIt; it++) {
                const float2 a = pf.v[2 * it], b = pf.v[2 * it + 1];
                *reinterpret_cast<float4*>(stg + (kPer * it + kl) * kStride + 4 * s2) =
                    make_float4(__fmul_rn(a.x, pf.wa), __fmul_rn(b.x, pf.wb), a.y, b.y);
            }
        };

        // pass 0's finished rows go to this lane's park slot in global memory (L2),
        // pass 1's stay in registers; the epilogue takes both
        float4* park = p.park + (size_t)(blockIdx.x * kWaves + wave) * (4 * 16 * 64) + lane;
        float raw1[4][2][8];    // pass 1: descriptor row, column 2 + k, bin
        float slot9[4];         // column 1's slot 9 (column 2's position 0) per row
        f2v quirk = {0.f, 0.f}; // pass 1: column 4's position 0 for the band's row pair

        auto zero_slots = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < kSlots / 256; q++)
                *reinterpret_cast<float4*>(buf + (q * 64 + lane) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
            quirk = f2v{0.f, 0.f};
        };

        // ---- one chunk: table to SGPRs (one wait), then per sample the values and
        // the read-add-write of the columns its class names ----
        auto walk = [&](int ch) __attribute__((always_inline)) {
#if SIFT_COLS_KS == 16
            i16v trf, tcf;
            i2v tcl;
            __asm__ volatile(
                "s_load_dwordx16 %0, %3, 0x0\n\t"
                "s_load_dwordx16 %1, %3, 0x40\n\t"
                "s_load_dwordx2 %2, %3, 0x80\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&s"(trf), "=&s"(tcf), "=&s"(tcl)
                : "s"(p.smp_s + ch * kTabDw));
#else
            static_assert(kKS == 8, "chunk size");
            i8v trf, tcf;
            i2v tcl;
            __asm__ volatile(
                "s_load_dwordx8 %0, %3, 0x0\n\t"
                "s_load_dwordx8 %1, %3, 0x20\n\t"
                "s_load_dwordx2 %2, %3, 0x40\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "=&s"(trf), "=&s"(tcf), "=&s"(tcl)
                : "s"(p.smp_s + ch * kTabDw));
#endif
            f4v r2[kPairs];      // one ds_read_b128 per sample pair
#pragma unroll
            for (int q = 0; q < kPairs; q++)
                r2[q] = *(const __attribute__((address_space(3))) volatile f4v*)(stg + lane * kStride + 4 * q);
#pragma unroll
            for (int q = 0; q < kKS; q++) {
                const int cls = (tcl[q >> 3] >> (4 * (q & 7))) & 15;
                const float mw = (q & 1) ? r2[q >> 1].y : r2[q >> 1].x;
                const float ob = (q & 1) ? r2[q >> 1].w : r2[q >> 1].z;
                // frac = ob - floor(ob) exactly (sift_band.hip: ob never rounds up to 1)
                const float frac = __builtin_amdgcn_fractf(ob);
                int o0;
                __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));   // floor in [-9, -1]
                const float v_r1 = __fmul_rn(mw, __int_as_float(trf[q]));
                const f2v vr = {__fsub_rn(mw, v_r1), v_r1};                 // rows r0, r0 + 1
                const f2v cf2 = {__int_as_float(tcf[q]), __int_as_float(tcf[q])};
                const f2v cR = vr * cf2;                                    // column c0 + 1: v * cbin
                const f2v cL = vr - cR;                                     // column c0: v - v * cbin
                const f2v fr = {frac, frac};
                const f2v hR = cR * fr, lR = cR - hR;                       // bins o0 + 1, o0
                const f2v hL = cL * fr, lL = cL - hL;
                // the left column's pass-local index cl (-1: right only; 1: left only)
                // and its slot byte offset at position o0 + 9
                const int cl = (cls & kClsLeft) ? ((cls & (kClsRight | kClsQuirk)) == kClsRight ? 0 : 1) : -1;
                char* tp = lb + (kPosBase * kPosF + cl * kColF) * 4 + __mul24(o0, kPosF * 4);
                auto t = (lds_f2v*)tp;
                auto u = (lds_f2v*)(tp + kColF * 4);
                // wave-uniform branches on the class: memory effects only, no merged values
                if (cls == (kClsLeft | kClsRight)) {
                    f2v a = t[0], b = t[kPosF / 2], c = u[0], d = u[kPosF / 2];
                    t[0] = a + lL;
                    t[kPosF / 2] = b + hL;
                    u[0] = c + lR;
                    u[kPosF / 2] = d + hR;
                } else if (cls & kClsLeft) {
                    f2v a = t[0], b = t[kPosF / 2];
                    t[0] = a + lL;
                    t[kPosF / 2] = b + hL;
                } else if (cls & kClsRight) {
                    f2v c = u[0], d = u[kPosF / 2];
                    u[0] = c + lR;
                    u[kPosF / 2] = d + hR;
                }
                if constexpr (true) {
                    // column 4 (pass 1, c0 = 3): only position 0 (o0 = -9, the lo share) is
                    // ever read; +0 for every other sample (exact: values are >= +0)
                    const bool hit = (cls & kClsQuirk) && o0 == -kPosBase;
                    const f2v z = {0.f, 0.f};
                    quirk = quirk + (hit ? lR : z);
                }
#if SIFT_COLS_SCHED
                // keep each sample's values next to its read-add-writes (register pressure)
                if ((q & (SIFT_COLS_SCHED - 1)) == SIFT_COLS_SCHED - 1) __builtin_amdgcn_sched_barrier(0);
#endif
            }
            wave_sync();
        };

        // ---- band close: row b of the pass's two columns is final (the pairs' first
        // element); the second element becomes the first, the second restarts at 0 ----
        auto close_band = [&](auto P, auto B) __attribute__((always_inline)) {
            constexpr int pass = decltype(P)::value, b = decltype(B)::value;
            float e0[kPos][2];
#pragma unroll
            for (int pos = 0; pos < kPos; pos++)
#pragma unroll
                for (int cl = 0; cl < 2; cl++) {
                    auto t = (lds_f2v*)(buf + pos * kPosF + cl * kColF + 2 * lane);
                    const f2v v = *t;
                    e0[pos][cl] = v.x;
                    if (b < 3) *t = f2v{v.y, 0.f};
                }
            if constexpr (b >= 0) {
                float f[2][8];
#pragma unroll
                for (int cl = 0; cl < 2; cl++) {
                    f[cl][0] = __fadd_rn(e0[1][cl], e0[9][cl]);           // slot 0 + slot 8
                    // slot 1 + slot 9; slot 9 is the next column's position 0
                    if (cl == 0) f[cl][1] = __fadd_rn(e0[2][0], e0[0][1]);
                    else if (pass == 1) f[cl][1] = __fadd_rn(e0[2][1], quirk.x);
                    else f[cl][1] = e0[2][1];                             // + slot 9 from pass 1
#pragma unroll
                    for (int q = 2; q < 8; q++) f[cl][q] = e0[q + 1][cl];
                }
                if constexpr (pass == 0) {
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        park[(b * 4 + u) * 64] = make_float4(f[u >> 1][(u & 1) * 4], f[u >> 1][(u & 1) * 4 + 1],
                                                             f[u >> 1][(u & 1) * 4 + 2], f[u >> 1][(u & 1) * 4 + 3]);
                } else {
#pragma unroll
                    for (int cl = 0; cl < 2; cl++)
#pragma unroll
                        for (int q = 0; q < 8; q++) raw1[b][cl][q] = f[cl][q];
                    slot9[b] = e0[0][0];
                }
            }
            if constexpr (pass == 1) quirk = f2v{quirk.y, 0.f};
            wave_sync();
        };

        Pre pf;
        issue(0, pf);
        zero_slots();
        stage(pf);
        wave_sync();
        auto run_band = [&](auto P, auto B) __attribute__((always_inline)) {
            constexpr int pass = decltype(P)::value, b = decltype(B)::value;
            const int ch_end = p.band_first[pass][b + 2];
            for (int ch = p.band_first[pass][b + 1]; ch < ch_end; ch++) {
                if (ch + 1 < nch) issue(ch + 1, pf);
                walk(ch);
                if (ch + 1 == ch_end) {
                    close_band(P, B);
                    if constexpr (b == 3 && pass == 0) {
                        zero_slots();
                        wave_sync();
                    }
                }
                if (ch + 1 < nch) {
                    stage(pf);
                    wave_sync();
                }
            }
        };
        using P0 = std::integral_constant<int, 0>;
        using P1 = std::integral_constant<int, 1>;
        run_band(P0{}, std::integral_constant<int, -1>{});
        run_band(P0{}, std::integral_constant<int, 0>{});
        run_band(P0{}, std::integral_constant<int, 1>{});
        run_band(P0{}, std::integral_constant<int, 2>{});
        run_band(P0{}, std::integral_constant<int, 3>{});
        run_band(P1{}, std::integral_constant<int, -1>{});
        run_band(P1{}, std::integral_constant<int, 0>{});
        run_band(P1{}, std::integral_constant<int, 1>{});
        run_band(P1{}, std::integral_constant<int, 2>{});
        run_band(P1{}, std::integral_constant<int, 3>{});

        // ---- epilogue, from registers: the reference's norm / clamp / renormalise /
        // saturate order (the band kernel's epilogue) ----
        {
            float raw[4][4][8];
#pragma unroll
            for (int r = 0; r < 4; r++) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float4 v = park[(r * 4 + u) * 64];
                    float* f = &raw[r][u >> 1][(u & 1) * 4];
                    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
                }
                raw[r][1][1] = __fadd_rn(raw[r][1][1], slot9[r]);         // slot 1 + slot 9
#pragma unroll
                for (int cl = 0; cl < 2; cl++)
#pragma unroll
                    for (int q = 0; q < 8; q++) raw[r][2 + cl][q] = raw1[r][cl][q];
            }
            float chain[8];
#pragma unroll
            for (int q = 0; q < 8; q++) chain[q] = 0.f;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++)
#pragma unroll
                    for (int q = 0; q < 8; q++) chain[q] = __fmaf_rn(raw[r][c][q], raw[r][c][q], chain[q]);
            const float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(chain[0], chain[4]), __fadd_rn(chain[1], chain[5])),
                                         __fadd_rn(__fadd_rn(chain[2], chain[6]), __fadd_rn(chain[3], chain[7])));
            const float thr = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
            float n2 = 0.f;
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int c = 0; c < 4; c++)
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const float x = fminf(raw[r][c][q], thr);
                        raw[r][c][q] = x;
                        n2 = __fadd_rn(n2, __fmul_rn(x, x));
                    }
            const float sq = cr_sqrtf(n2);
            const float sc = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
            if (act) {
                int ns = 0;
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int c2 = 0; c2 < 2; c2++) {
                        uint32_t wd[4];
#pragma unroll
                        for (int wq = 0; wq < 4; wq++) {
                            uint32_t word = 0;
#pragma unroll
                            for (int bb = 0; bb < 4; bb++) {
                                const int c = 2 * c2 + (wq >> 1), q = (wq & 1) * 4 + bb;
                                float x = rintf(__fmul_rn(raw[r][c][q], sc));
                                x = fminf(fmaxf(x, 0.f), 255.f);
                                const int iv = (int)x;
                                word |= (uint32_t)iv << (8 * bb);
                                ns += (iv - 128) * (iv - 128);
                                raw[r][c][q] = x;
                            }
                            wd[wq] = word;
                        }
                        *reinterpret_cast<uint4*>(p.desc_u8 + (size_t)g * 128 + (r * 2 + c2) * 16) =
                            make_uint4(wd[0], wd[1], wd[2], wd[3]);
                    }
                p.norm_i8[g] = ns;
                if (p.desc_f32) {
                    float4* o = reinterpret_cast<float4*>(p.desc_f32 + (size_t)g * 128);
#pragma unroll
                    for (int r = 0; r < 4; r++)
#pragma unroll
                        for (int c = 0; c < 4; c++) {
                            o[(r * 4 + c) * 2] = make_float4(raw[r][c][0], raw[r][c][1], raw[r][c][2], raw[r][c][3]);
                            o[(r * 4 + c) * 2 + 1] = make_float4(raw[r][c][4], raw[r][c][5], raw[r][c][6], raw[r][c][7]);
                        }
                }
            }
        }
        wave_sync();
    }
}

}  // namespace

// SLAMHIP_SIFT_COLS=1: sift_desc_band launches run this kernel instead (A/B)
bool sift_cols_enabled()
{
    static const bool on = [] { const char* e = getenv("SLAMHIP_SIFT_COLS"); return e && e[0] == '1'; }();
    return on;
}

// The two passes' schedules and tables from the band geometry; false when the
// geometry is not the FAST one this kernel is written for (floor(obin) in
// [-9, -1]), a pass's band is empty, or a target's order is not raster order.
bool sift_cols_prepare(slam_ctx* c, hipStream_t s, const BandGeometry& geo)
{
    c->sift_cols_valid = false;
    if (!geo.neg) return false;
    const std::vector<BandSample>& smp = geo.smp;
    const int n = (int)smp.size();
    auto f2i = [](float f) { union { float f; int32_t i; } u; u.f = f; return u.i; };
    auto i2f = [](int32_t i) { union { int32_t i; float f; } u; u.i = i; return u.f; };
    std::vector<float2> tv;
    std::vector<int32_t> ts;
    int band_first[2][6];
    auto push = [&](float w, int off, float rf, float cf, int cls) {
        if (tv.size() % kKS == 0) ts.resize(ts.size() + kTabDw, 0);
        const size_t q = tv.size() % kKS, base = ts.size() - kTabDw;
        tv.push_back(make_float2(w, i2f(off)));
        ts[base + q] = f2i(rf);
        ts[base + kKS + q] = f2i(cf);
        ts[base + 2 * kKS + q / 8] |= cls << (4 * (q % 8));
    };
    for (int pass = 0; pass < 2; pass++) {
        std::vector<int> sched;      // this pass's samples in schedule order (< 0: padding)
        for (int b = -1; b <= 3; b++) {
            band_first[pass][b + 1] = (int)(tv.size() / kKS);
            const size_t start = tv.size();
            for (int k = 0; k < n; k++) {
                const BandSample& sm = smp[k];
                const int cl = sm.c0 - 2 * pass;           // the sample's left column in the pass
                if (sm.r0 != b || cl < -1 || cl > 1) continue;
                const int cls = (cl >= 0 ? kClsLeft : 0) | (cl + 1 <= 1 ? kClsRight : 0) |
                                (pass == 1 && cl + 1 == 2 ? kClsQuirk : 0);
                push(sm.wexp, (sm.i * geo.pitch + sm.j) * 8, sm.rf, sm.cf, cls);
                sched.push_back(k);
            }
            if (tv.size() == start) return false;     // the band close needs a chunk
            while (tv.size() % kKS) {                  // padding: weight 0 at the keypoint, no column
                push(0.f, 0, 0.f, 0.f, 0);
                sched.push_back(-1);
            }
        }
        // every target cell of the pass (hist rows 1..4; columns 1..2 / 3..5) must
        // receive its samples in raster order
        for (int R = 1; R <= 4; R++)
            for (int C = 2 * pass + 1; C <= (pass ? 5 : 2); C++) {
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
    band_first[1][5] = nchunks;
    band_first[0][5] = band_first[1][0];
    if (nchunks > kMaxChunks) return false;
    const size_t b_v = tv.size() * sizeof(float2), b_s = ts.size() * sizeof(int32_t);
    if (c->sift_cols_buf.ensure(b_v + b_s) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_cols_buf.p, tv.data(), b_v, hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (hipMemcpyAsync(c->sift_cols_buf.as<char>() + b_v, ts.data(), b_s, hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    SiftColsMeta& m = c->sift_cols;
    m.nrec = (int)tv.size();
    m.nchunks = nchunks;
    for (int pass = 0; pass < 2; pass++)
        for (int q = 0; q < 6; q++) m.band_first[pass][q] = band_first[pass][q];
    c->sift_cols_valid = true;
    return true;
}

hipError_t launch_sift_desc_cols(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    const SiftColsMeta& m = c->sift_cols;
    ColsParams p;
    p.grad = c->grad.as<char>();
    p.frame_bytes = grad_frame(w, h) * 8;
    p.origin_bytes = grad_origin(w) * 8;
    p.pitch_bytes = grad_pitch(w) * 8;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.smp = c->sift_cols_buf.as<float2>();
    p.smp_s = reinterpret_cast<const int*>(c->sift_cols_buf.as<char>() + (size_t)m.nrec * sizeof(float2));
    p.nchunks = m.nchunks;
    for (int pass = 0; pass < 2; pass++)
        for (int q = 0; q < 6; q++) p.band_first[pass][q] = m.band_first[pass][q];
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    // persistent: one 8-wave workgroup per CU, a multiple of 8 workgroups for the XCD split
    int grid = c->cu_count;
    const int need = (cap + kKpW * kWaves - 1) / (kKpW * kWaves);
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    // park: 4 rows x 16 float4 per lane of every wave of the grid
    hipError_t e;
    if ((e = c->sift_cols_park.ensure((size_t)grid * kWaves * 4 * 16 * 64 * sizeof(float4))) != hipSuccess) return e;
    p.park = c->sift_cols_park.as<float4>();
    hipLaunchKernelGGL(sift_desc_cols, dim3(grid), dim3(64 * kWaves), 0, s, p);
    return hipGetLastError();
}

}  // namespace slamhip
