// FAST-9/16 corner detection with 3x3 non-max suppression, gfx950.
//
// Replaces fastExtractor (reference src/mainModule/featureExtraction/
// fastExtractor.cpp:7-13 -> cv::FastFeatureDetector(threshold, nonmax,
// TYPE_9_16)::detect), i.e. OpenCV 4.8 FAST_t<16> + cornerScore<16> on the
// cvtColor(BGR2GRAY) image.  Output order is the reference's raster order.
//
// Kernel 1 (fast_detect): one workgroup per 64 x 64 pixel tile (256 threads).
//   BGR tile + 4 px halo -> gray in LDS (fixed point, yuv_shift 14), segment
//   test on the 16-px Bresenham circle (bit masks, 9-run test on the doubled
//   mask), cornerScore only for corners, scores of the tile + 1 px halo in LDS,
//   then one wave per 16 rows: lane = column, NMS (score strictly greater than
//   all 8 neighbours), __ballot -> one 64-bit keep mask per (row, tile).
//   Writes gray (needed by SIFT/ORB), masks, responses of kept pixels, and
//   per-16-row-band counts (raw FAST count = batch filter input; border-
//   filtered count = what ORB keeps, runByImageBorder(31)).
// Kernel 2 (fast_finalize): one workgroup: per-frame band prefix sums and the
//   frame offsets of the concatenated keypoint list.
// Kernel 3 (fast_emit): one workgroup per band: popcounts of the band's masks,
//   workgroup exclusive scan in raster order, each thread writes its row
//   segment's keypoints (x, y, 7, -1, score, 0, -1) -- order preserving.
#include "slamhip_internal.h"

namespace slamhip {

namespace {

// detect tile: kFastTileW x TH rows = TH / kFastTileH output bands (the band
// counts and fast_emit keep the 16-row band)
constexpr int TW = kFastTileW, TH = 4 * kFastTileH;
constexpr int HALO = 4;
constexpr int LW = TW + 2 * HALO;   // 72
constexpr int LH = TH + 2 * HALO;   // 72
constexpr int SW = TW + 2, SH = TH + 2;
// score row stride = the gray row's (18 dwords): prefilter task i = (row i / 18,
// group i % 18) reads gray dword 18 row + group + const = i + const, so the 32
// lanes of each ds_read_b32 lane group hit 32 distinct banks (17 groups per
// row, as the 66 score columns need, put lane 32 k + 31 of a row pair on lane
// 32 k's bank: a 2-way conflict on every prefilter read).  Group 17 of each row
// is past the score columns (valid = 0).
constexpr int SWP = LW;
constexpr int NG = SWP / 4;         // prefilter groups of 4 pixels per score row
static_assert(NG * 4 >= SW + 2, "the last group of a row is past the score columns");
constexpr int kBandsPerTile = TH / kFastTileH;
constexpr int kFastThreads = 256, kFastWaves = kFastThreads / 64;
static_assert(TH % kFastTileH == 0 && kFastWaves % kBandsPerTile == 0 && TH % kFastWaves == 0,
              "whole bands per tile, whole waves per band");
static_assert(TH * 16 % kFastThreads == 0, "whole gray store passes");

struct DetectParams {
    const uint8_t* img;
    size_t frame_stride, row_stride;
    int channels, w, h, thr, border;
    int ntx, nbands;
    int wide;        // rows and frames 4-byte aligned: 12-byte BGR loads
    int gray_wide;   // w % 4 == 0: dword gray stores
    int xcd;         // tiles in XCD-contiguous order (xcd_tile)
    int dbg;         // timing probes (SLAMHIP_FAST_DBG; wrong results): 1 no gray store, 2 no candidates, 4 no NMS
    uint8_t* gray;
    uint64_t* masks;
    uint8_t* scores;
    int* band_cnt;   // [frame][band][2] = {raw, filtered}
};

// circle offsets (dx, dy), OpenCV makeOffsets order for patternSize 16, 12, 8
__constant__ int8_t c_cdx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int8_t c_cdy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
__constant__ int8_t c_cdx12[12] = {0, 1, 2, 2, 2, 1, 0, -1, -2, -2, -2, -1};
__constant__ int8_t c_cdy12[12] = {2, 2, 1, 0, -1, -2, -2, -2, -1, 0, 1, 2};
__constant__ int8_t c_cdx8[8] = {0, 1, 1, 1, 0, -1, -1, -1};
__constant__ int8_t c_cdy8[8] = {1, 1, 0, -1, -1, -1, 0, 1};

// TYPE_7_12 / TYPE_5_8 (fastExtractor.h:19-21's `type`; every reference caller
// uses the TYPE_9_16 default): the circle test of FAST_t<PS> on a compacted
// candidate -- OpenCV's pair prefilter over the wrapped pixel[0..15] (a filter of
// its own for PS < 16), then K + 1 contiguous (K = PS / 2) all darker / brighter
__device__ inline bool run_ps(uint32_t m, int ps, int k1)
{
    const uint32_t mm = m | (m << ps);
    uint32_t r = mm;
    for (int i = 1; i < k1; i++) r &= mm >> i;
    return r != 0;
}

// cornerScore<PS> for PS = 12, 8 (d[k] = v - p[k % PS], k < 3 K + 1): the
// largest threshold that keeps the pixel a corner, - 1 (OpenCV's early
// `continue`s never change the result)
template <int PS>
__device__ inline int corner_score_small(const int* d, int threshold)
{
    constexpr int K = PS / 2;
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < PS; k += 2) {
        int a = d[k + 1];
#pragma unroll
        for (int m = 2; m <= K; m++) a = min(a, d[k + m]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + K + 1]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < PS; k += 2) {
        int b = d[k + 1];
#pragma unroll
        for (int m = 2; m <= K; m++) b = max(b, d[k + m]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + K + 1]));
    }
    return -b0 - 1;
}

// cvtColor BGR2GRAY of 4 pixels from their 12 bytes {b0 g0 r0 b1}{g1 r1 b2 g2}{r2 b3 g3 r3}:
// (1868 b + 9617 g + 4899 r + 2^13) >> 14 with each coefficient split as 256 hi + lo
// (B 7|76, G 37|145, R 19|35), both halves summed by v_dot4_u32_u8 over the pixel's
// bytes (a pixel split over two dwords chains two dot products).  Exact integer
// arithmetic: the same value as the per-channel multiply-adds.
__device__ __forceinline__ uint32_t gray4_bgr(uint32_t w0, uint32_t w1, uint32_t w2)
{
    auto dot = [](uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_udot4(a, b, c, false); };
    constexpr uint32_t R = 1u << 13;
    const uint32_t l0 = dot(w0, 76u | 145u << 8 | 35u << 16, R), h0 = dot(w0, 7u | 37u << 8 | 19u << 16, 0);
    const uint32_t l1 = dot(w1, 145u | 35u << 8, dot(w0, 76u << 24, R));
    const uint32_t h1 = dot(w1, 37u | 19u << 8, dot(w0, 7u << 24, 0));
    const uint32_t l2 = dot(w2, 35u, dot(w1, 76u << 16 | 145u << 24, R));
    const uint32_t h2 = dot(w2, 19u, dot(w1, 7u << 16 | 37u << 24, 0));
    const uint32_t l3 = dot(w2, 76u << 8 | 145u << 16 | 35u << 24, R);
    const uint32_t h3 = dot(w2, 7u << 8 | 37u << 16 | 19u << 24, 0);
    const uint32_t y0 = (h0 * 256u + l0) >> 14, y1 = (h1 * 256u + l1) >> 14;
    const uint32_t y2 = (h2 * 256u + l2) >> 14, y3 = (h3 * 256u + l3) >> 14;
    return y0 | y1 << 8 | y2 << 16 | y3 << 24;
}

__device__ inline bool run9(uint32_t m16)
{
    uint32_t m = m16 | (m16 << 16);
    uint32_t r = m;
#pragma unroll
    for (int i = 1; i < 9; i++) r &= m >> i;
    return r != 0;
}

// cornerScore<16> with d[k] = v - p[k % 16], k = 0..24
__device__ inline int corner_score(const int* d, int threshold)
{
    int a0 = threshold;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        if (a <= a0) continue;
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int b = max(d[k + 1], d[k + 2]);
        b = max(b, d[k + 3]);
        b = max(b, d[k + 4]);
        b = max(b, d[k + 5]);
        if (b >= b0) continue;
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return -b0 - 1;
}

template <int NMS, int PS>
__global__ __launch_bounds__(kFastThreads) void fast_detect(DetectParams p)
{
    __shared__ __attribute__((aligned(16))) uint8_t g[LH][LW];
    __shared__ __attribute__((aligned(4))) uint8_t sc[SH][SWP];
    __shared__ uint64_t cmask[TH];        // corners of the tile, one bit per pixel
    __shared__ uint16_t cand_list[SW * SH];
    __shared__ int ncand;

    int tx, ty, f;
    xcd_tile(p.xcd != 0, tx, ty, f);
    const int tid = threadIdx.x;
    const int x0 = tx * TW - HALO, y0 = ty * TH - HALO;
    if (tid == 0) ncand = 0;                  // published by the barrier after the tile load
    if (tid < TH) cmask[tid] = 0;
    const uint8_t* src = p.img + (size_t)f * p.frame_stride;

    // BGR -> gray tile.  Interior tiles of 3-channel frames with 4-byte aligned
    // rows: one 12-byte load (4 pixels) per lane, coalesced along the row (the
    // per-lane byte loads saturated the texture data path).  Edge tiles and
    // 1/4-channel images clamp per pixel.
    const bool wide = p.channels == 3 && p.wide && x0 >= 0 && x0 + LW <= p.w && y0 >= 0 && y0 + LH <= p.h;
    if (wide) {
        // every load of the thread first (32-bit offsets from the tile's corner),
        // then the conversions
        constexpr int G = LW / 4;                 // 18 four-pixel groups per row
        constexpr int NGR = G * LH, NIT = (NGR + kFastThreads - 1) / kFastThreads;
        const uint8_t* base = src + (size_t)y0 * p.row_stride + (size_t)x0 * 3;
        const uint32_t rs = (uint32_t)p.row_stride;
        uint32_t wv[NIT][3];
#pragma unroll
        for (int j = 0; j < NIT; j++) {
            const int i = tid + j * kFastThreads;
            if (i < NGR) {
                const int ly = i / G, gq = i - ly * G;
                const uint32_t* s32 = reinterpret_cast<const uint32_t*>(base + ((uint32_t)ly * rs + 12u * (uint32_t)gq));
                wv[j][0] = s32[0];
                wv[j][1] = s32[1];
                wv[j][2] = s32[2];
            }
        }
#pragma unroll
        for (int j = 0; j < NIT; j++) {
            const int i = tid + j * kFastThreads;
            if (i < NGR) {
                const int ly = i / G, gq = i - ly * G;
                *reinterpret_cast<uint32_t*>(&g[ly][4 * gq]) = gray4_bgr(wv[j][0], wv[j][1], wv[j][2]);
            }
        }
    } else {
        for (int i = tid; i < LW * LH; i += kFastThreads) {
            int ly = i / LW, lx = i - ly * LW;
            int gx = min(max(x0 + lx, 0), p.w - 1);
            int gy = min(max(y0 + ly, 0), p.h - 1);
            const uint8_t* s = src + (size_t)gy * p.row_stride + (size_t)gx * p.channels;
            uint32_t v;
            if (p.channels == 1) v = s[0];
            else v = ((uint32_t)s[0] * 1868u + (uint32_t)s[1] * 9617u + (uint32_t)s[2] * 4899u + (1u << 13)) >> 14;
            g[ly][lx] = (uint8_t)v;
        }
    }
    __syncthreads();

    // gray interior -> global (consumed by the SIFT / ORB blurs): one dword per lane
    if (p.dbg & 1) {
    } else if (p.gray_wide && (tx + 1) * TW <= p.w && (ty + 1) * TH <= p.h) {
#pragma unroll
        for (int k = 0; k < TH * 16 / kFastThreads; k++) {
            const int ly = (tid >> 4) + (kFastThreads / 16) * k, q = tid & 15;   // rows x 16 dwords per pass
            uint32_t* dst = reinterpret_cast<uint32_t*>(p.gray + (size_t)f * p.w * p.h +
                                                        (size_t)(ty * TH + ly) * p.w + tx * TW);
            dst[q] = *reinterpret_cast<const uint32_t*>(&g[ly + HALO][HALO + 4 * q]);
        }
    } else {
        for (int i = tid; i < TW * TH; i += kFastThreads) {
            int ly = i / TW, lx = i - ly * TW;
            int gx = tx * TW + lx, gy = ty * TH + ly;
            if (gx < p.w && gy < p.h)
                p.gray[(size_t)f * p.w * p.h + (size_t)gy * p.w + gx] = g[ly + HALO][lx + HALO];
        }
    }

    // scores of the tile + 1 px ring, in two passes.  (1) OpenCV's own
    // necessary condition (FAST_t: a 9-arc contains one pixel of each opposite
    // pair 0/8, 2/10, 4/12, 6/14, all dark or all bright) on every pixel; about
    // 4 % of the pixels of a textured frame pass.  Four horizontally adjacent
    // pixels per task: each circle row is one byte-aligned dword of the gray
    // tile (v_alignbyte over two LDS dwords), the four pixels' values are two
    // u16 pairs, and the pair min / max and the threshold tests run on packed
    // u16 (v_pk_min_u16 / v_pk_max_u16) -- the same integer comparisons as
    // per pixel.  (2) the exact segment test and cornerScore on the compacted
    // candidates only.
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 thr2 = {(unsigned short)p.thr, (unsigned short)p.thr};
    // every score pixel of the tile at least 3 px inside the image: only the
    // tile width cuts the last group of each row
    const bool inner = tx * TW - 1 >= 3 && tx * TW - 1 + SW <= p.w - 3 && ty * TH - 1 >= 3 && ty * TH - 1 + SH <= p.h - 3;
    for (int i = tid; i < SH * NG; i += kFastThreads) {
        const int ly = i / NG, lx0 = 4 * (i - ly * NG);
        const int gx0 = tx * TW - 1 + lx0, gy = ty * TH - 1 + ly;
        uint32_t valid = 0;
        if (inner) {
            valid = lx0 + 4 <= SW ? 0xfu : 0xfu >> (lx0 + 4 - SW);
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                valid |= (uint32_t)(lx0 + k < SW && gx0 + k >= 3 && gx0 + k < p.w - 3 && gy >= 3 && gy < p.h - 3) << k;
        }
        uint32_t cmask = 0;
        if (PS != 16) {
            cmask = valid;                    // TYPE_7_12 / 5_8: every pixel to the exact pass
        } else if (valid) {
            const int cy = ly + HALO - 1, cx = lx0 + HALO - 1;
            // bytes g[r][cx + dx .. cx + dx + 3] (cx + dx >= 0; bytes past the tile row
            // only reach the pixels masked out of `valid`) as two u16 pairs, each one
            // v_perm of the two LDS dwords: cx = 4 k + 3, so the byte offset
            // (cx + dx) & 3 = (3 + dx) & 3 is a compile-time selector
            struct R4 { us2 lo, hi; };
            auto row4 = [&](int r, int dx) __attribute__((always_inline)) -> R4 {
                const int b = cx + dx;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(&g[r][b & ~3]);
                const uint32_t o = (uint32_t)((3 + dx) & 3);      // == b & 3
                const uint32_t sl = 0x0c000c00u | ((o + 1) << 16) | o, sh = sl + 0x00020002u;
                return R4{__builtin_bit_cast(us2, __builtin_amdgcn_perm(w[1], w[0], sl)),
                          __builtin_bit_cast(us2, __builtin_amdgcn_perm(w[1], w[0], sh))};
            };
            auto lo = [](const R4& x) { return x.lo; };
            auto hi = [](const R4& x) { return x.hi; };
            const R4 v4 = row4(cy, 0);
            // circle pairs (0, 8), (2, 10), (4, 12), (6, 14): c_cdx / c_cdy order
            const R4 a0 = row4(cy + 3, 0), b0 = row4(cy - 3, 0);
            const R4 a1 = row4(cy + 2, 2), b1 = row4(cy - 2, -2);
            const R4 a2 = row4(cy, 3), b2 = row4(cy, -3);
            const R4 a3 = row4(cy - 2, 2), b3 = row4(cy + 2, -2);
            us2 mnl = __builtin_elementwise_min(lo(a0), lo(b0)), mnh = __builtin_elementwise_min(hi(a0), hi(b0));
            us2 mxl = __builtin_elementwise_max(lo(a0), lo(b0)), mxh = __builtin_elementwise_max(hi(a0), hi(b0));
            mnl = __builtin_elementwise_max(mnl, __builtin_elementwise_min(lo(a1), lo(b1)));
            mnh = __builtin_elementwise_max(mnh, __builtin_elementwise_min(hi(a1), hi(b1)));
            mxl = __builtin_elementwise_min(mxl, __builtin_elementwise_max(lo(a1), lo(b1)));
            mxh = __builtin_elementwise_min(mxh, __builtin_elementwise_max(hi(a1), hi(b1)));
            mnl = __builtin_elementwise_max(mnl, __builtin_elementwise_min(lo(a2), lo(b2)));
            mnh = __builtin_elementwise_max(mnh, __builtin_elementwise_min(hi(a2), hi(b2)));
            mxl = __builtin_elementwise_min(mxl, __builtin_elementwise_max(lo(a2), lo(b2)));
            mxh = __builtin_elementwise_min(mxh, __builtin_elementwise_max(hi(a2), hi(b2)));
            mnl = __builtin_elementwise_max(mnl, __builtin_elementwise_min(lo(a3), lo(b3)));
            mnh = __builtin_elementwise_max(mnh, __builtin_elementwise_min(hi(a3), hi(b3)));
            mxl = __builtin_elementwise_min(mxl, __builtin_elementwise_max(lo(a3), lo(b3)));
            mxh = __builtin_elementwise_min(mxh, __builtin_elementwise_max(hi(a3), hi(b3)));
            // mn < v - thr  <=>  v > mn + thr;  mx > v + thr (all < 2^16): the positive
            // parts max(v, t) - t are nonzero exactly where the test holds
            const us2 vl = lo(v4), vh = hi(v4);
            const us2 dl = mnl + thr2, dh = mnh + thr2, bl = vl + thr2, bh = vh + thr2;
            const us2 one = {1, 1};
            const us2 tl = __builtin_elementwise_min((__builtin_elementwise_max(vl, dl) - dl) |
                                                     (__builtin_elementwise_max(mxl, bl) - bl), one);
            const us2 th = __builtin_elementwise_min((__builtin_elementwise_max(vh, dh) - dh) |
                                                     (__builtin_elementwise_max(mxh, bh) - bh), one);
            cmask = ((uint32_t)tl.x | ((uint32_t)tl.y << 1) | ((uint32_t)th.x << 2) | ((uint32_t)th.y << 3)) & valid;
        }
        if (p.dbg & 2) cmask = 0;
        *reinterpret_cast<uint32_t*>(&sc[ly][lx0]) = 0u;
        // order-free compaction (each candidate's result lands at its own pixel):
        // a wave-wide exclusive scan of the 0..4 candidates per lane from three ballots
        const int nb = __popc(cmask);
        const uint64_t bb0 = __ballot(nb & 1), bb1 = __ballot(nb & 2), bb2 = __ballot(nb & 4);
        const int tot = __popcll(bb0) + 2 * __popcll(bb1) + 4 * __popcll(bb2);
        int wbase = 0;
        if ((tid & 63) == 0 && tot) wbase = atomicAdd(&ncand, tot);
        wbase = __shfl(wbase, 0, 64);
        const uint64_t below = (1ull << (tid & 63)) - 1;
        int o = wbase + __popcll(bb0 & below) + 2 * __popcll(bb1 & below) + 4 * __popcll(bb2 & below);
        for (uint32_t m = cmask; m; m &= m - 1) cand_list[o++] = (uint16_t)(ly * SW + lx0 + __builtin_ctz(m));
    }
    __syncthreads();
    const int nc = ncand;
    for (int k = tid; k < nc; k += kFastThreads) {
        const int i = cand_list[k];
        const int ly = i / SW, lx = i - ly * SW;
        const int cy = ly + HALO - 1, cx = lx + HALO - 1;
        const int v = g[cy][cx];
        int corner = 0, sv = 0;
        if constexpr (PS == 16) {
            int pv[16];
            uint32_t dk = 0, br = 0;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                pv[q] = g[cy + c_cdy[q]][cx + c_cdx[q]];
                dk |= (uint32_t)(pv[q] < v - p.thr) << q;
                br |= (uint32_t)(pv[q] > v + p.thr) << q;
            }
            corner = run9(dk) || run9(br);
            if (corner && NMS) {
                int d[25];
#pragma unroll
                for (int q = 0; q < 25; q++) d[q] = v - pv[q & 15];
                sv = corner_score(d, p.thr);
            }
        } else {
            const int8_t* cdx = PS == 12 ? c_cdx12 : c_cdx8;
            const int8_t* cdy = PS == 12 ? c_cdy12 : c_cdy8;
            int pv[PS];
            uint32_t dk = 0, br = 0;
#pragma unroll
            for (int q = 0; q < PS; q++) {
                pv[q] = g[cy + cdy[q]][cx + cdx[q]];
                dk |= (uint32_t)(pv[q] < v - p.thr) << q;
                br |= (uint32_t)(pv[q] > v + p.thr) << q;
            }
            // threshold_tab: 1 dark, 2 bright; pairs (k, k + 8) of the wrapped circle
            const uint32_t tb = (dk & 0xffffu) | (br << 16);
            uint32_t dd = 3;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int q0 = k % PS, q1 = (k + 8) % PS;
                const uint32_t t0 = ((tb >> q0) & 1u) | (((tb >> (16 + q0)) & 1u) << 1);
                const uint32_t t1 = ((tb >> q1) & 1u) | (((tb >> (16 + q1)) & 1u) << 1);
                dd &= t0 | t1;
            }
            corner = ((dd & 1u) && run_ps(dk, PS, PS / 2 + 1)) || ((dd & 2u) && run_ps(br, PS, PS / 2 + 1));
            if (corner && NMS) {
                int d[3 * (PS / 2) + 1];
#pragma unroll
                for (int q = 0; q < 3 * (PS / 2) + 1; q++) d[q] = v - pv[q % PS];
                sv = corner_score_small<PS>(d, p.thr);
            }
        }
        sc[ly][lx] = (uint8_t)sv;
        if (corner && ly >= 1 && ly <= TH && lx >= 1 && lx <= TW) atomicOr(&cmask[ly - 1], 1ull << (lx - 1));
    }
    __syncthreads();

    // non-max suppression on the corners only (non-corners score 0 and are never
    // kept): thread = (tile row, 16-column quarter), so a wave is one 16-row band
    static_assert(TH * 4 == kFastThreads && kFastTileH * 4 == 64, "a wave per band, four threads per row");
    const int lane = tid & 63, r = tid >> 2, qd = tid & 3;
    const int gy = ty * TH + r;
    const int bx = p.border > 3 ? p.border : 3;
    uint32_t m = gy < p.h && !(p.dbg & 4) ? (uint32_t)(cmask[r] >> (16 * qd)) & 0xffffu : 0u;
    uint32_t kraw = 0, kfil = 0;
    while (m) {
        const int c = 16 * qd + __builtin_ctz(m);
        m &= m - 1;
        const int s = sc[r + 1][c + 1];
        bool keep = true;
        if (NMS) {
            int mx = max(max(sc[r][c], sc[r][c + 1]), sc[r][c + 2]);
            mx = max(mx, max(sc[r + 1][c], sc[r + 1][c + 2]));
            mx = max(mx, max(max(sc[r + 2][c], sc[r + 2][c + 1]), sc[r + 2][c + 2]));
            keep = s > mx;
        }
        const int gx = tx * TW + c;
        keep = keep && gx < p.w;
        const bool keepf = keep && gx >= bx && gx < p.w - bx && gy >= bx && gy < p.h - bx;
        kraw |= (uint32_t)keep << (c - 16 * qd);
        kfil |= (uint32_t)keepf << (c - 16 * qd);
        if (keepf) p.scores[(size_t)f * p.w * p.h + (size_t)gy * p.w + gx] = (uint8_t)s;
    }
    // the row's four quarters -> its 64-bit keep mask (lanes 4 r' .. 4 r' + 3 of the wave)
    uint32_t lo32 = qd == 0 ? kfil : (qd == 1 ? kfil << 16 : 0u);
    uint32_t hi32 = qd == 2 ? kfil : (qd == 3 ? kfil << 16 : 0u);
    lo32 |= __shfl_xor(lo32, 1, 64);
    hi32 |= __shfl_xor(hi32, 1, 64);
    lo32 |= __shfl_xor(lo32, 2, 64);
    hi32 |= __shfl_xor(hi32, 2, 64);
    if (qd == 0 && gy < p.h) p.masks[((size_t)f * p.h + gy) * p.ntx + tx] = ((uint64_t)hi32 << 32) | lo32;
    int craw = __popc(kraw), cfil = __popc(kfil);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        craw += __shfl_xor(craw, o, 64);
        cfil += __shfl_xor(cfil, o, 64);
    }
    const int band = ty * kBandsPerTile + (tid >> 6);
    if (lane == 0 && band < p.nbands) {
        int* bc = p.band_cnt + ((size_t)f * p.nbands + band) * 2;
        if (craw) atomicAdd(&bc[0], craw);
        if (cfil) atomicAdd(&bc[1], cfil);
    }
}

// one workgroup: frame_info[f] = {offset, filtered count, raw count, 0}; band_pref
// = exclusive prefix of filtered band counts inside each frame; misc[0] = total.
// A frame's count in frame_info is clipped to the keypoint capacity (offset +
// count <= cap), so that kernels which read it before the host has checked the
// total (the fused extract + match) never index past the keypoint buffers; the
// total stays unclipped and the host reports SLAM_E_CAPACITY from it.
__global__ __launch_bounds__(1024) void fast_finalize(const int* band_cnt, int nframes, int nbands,
                                                      int* band_pref, int4* frame_info, int* total, int cap)
{
    __shared__ int cnt[1024];
    __shared__ int raw[1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int base = 0; base < nframes; base += 1024) {
        // one wave per frame: the band counts 64 at a time, a wave prefix scan
        // for band_pref (the serial per-frame loop was a chain of dependent loads)
        for (int fl = wave; fl < 1024 && base + fl < nframes; fl += 16) {
            const int f = base + fl;
            int run = 0, rsum = 0;
            for (int b0 = 0; b0 < nbands; b0 += 64) {
                const int b = b0 + lane;
                int c = 0, r = 0;
                if (b < nbands) {
                    c = band_cnt[((size_t)f * nbands + b) * 2 + 1];
                    r = band_cnt[((size_t)f * nbands + b) * 2 + 0];
                }
                int incl = c;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += v;
                }
                if (b < nbands) band_pref[(size_t)f * nbands + b] = run + incl - c;
                run += __shfl(incl, 63, 64);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
                rsum += r;
            }
            if (lane == 0) { cnt[fl] = run; raw[fl] = rsum; }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int off = base == 0 ? 0 : *total;
            for (int i = 0; i < 1024 && base + i < nframes; i++) {
                frame_info[base + i] = make_int4(off, min(cnt[i], max(cap - off, 0)), raw[i], 0);
                off += cnt[i];
            }
            *total = off;
        }
        __syncthreads();
    }
}

struct EmitParams {
    const uint64_t* masks;
    const uint8_t* scores;
    const int* band_pref;
    const int4* frame_info;
    int w, h, ntx, nbands, cap;
    slam_keypoint* kps;
    int* kp_frame;
};

__global__ __launch_bounds__(1024) void fast_emit(EmitParams p)
{
    __shared__ int wtot[16];
    const int ty = blockIdx.x, f = blockIdx.y;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int row = t / p.ntx, txi = t - row * p.ntx;
    const int gy = ty * kFastTileH + row;
    uint64_t m = 0;
    if (row < kFastTileH && gy < p.h) m = p.masks[((size_t)f * p.h + gy) * p.ntx + txi];
    const int c = __popcll(m);
    // wave inclusive scan
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int wbase = 0;
    for (int i = 0; i < wave; i++) wbase += wtot[i];
    int base = p.frame_info[f].x + p.band_pref[(size_t)f * p.nbands + ty] + wbase + incl - c;
    const uint8_t* srow = p.scores + (size_t)f * p.w * p.h + (size_t)gy * p.w;
    while (m) {
        int b = __builtin_ctzll(m);
        m &= m - 1;
        if (base < p.cap) {
            int x = txi * kFastTileW + b;
            slam_keypoint k;
            k.x = (float)x; k.y = (float)gy; k.size = 7.f; k.angle = -1.f;
            k.response = (float)srow[x]; k.octave = 0; k.class_id = -1;
            p.kps[base] = k;
            p.kp_frame[base] = f;
        }
        base++;
    }
}

// cvtColor(BGR2GRAY) alone (extractDescriptor on caller-provided keypoints; the
// SIFT detector), blockIdx.z = frame of a contiguous batch
__global__ __launch_bounds__(256) void gray_convert(const uint8_t* img, size_t row_stride, int channels, int w,
                                                    int h, uint8_t* gray)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    img += blockIdx.z * (size_t)h * row_stride;
    gray += blockIdx.z * (size_t)w * h;
    const uint8_t* s = img + (size_t)y * row_stride + (size_t)x * channels;
    uint32_t v;
    if (channels == 1) v = s[0];
    else v = ((uint32_t)s[0] * 1868u + (uint32_t)s[1] * 9617u + (uint32_t)s[2] * 4899u + (1u << 13)) >> 14;
    gray[(size_t)y * w + x] = (uint8_t)v;
}

}  // namespace

hipError_t launch_gray(slam_ctx* c, hipStream_t s, const uint8_t* img, size_t row_stride, int channels, int w, int h)
{
    c->fast_gen++;              // rewrites the gray plane (FastReuse)
    hipError_t e;
    if ((e = c->gray.ensure((size_t)w * h)) != hipSuccess) return e;
    hipLaunchKernelGGL(gray_convert, dim3((w + 255) / 256, h), dim3(256), 0, s, img, row_stride, channels, w, h,
                       c->gray.as<uint8_t>());
    return hipGetLastError();
}

hipError_t launch_gray_batch(slam_ctx* c, hipStream_t s, const uint8_t* frames, int nframes, int w, int h, int channels)
{
    c->fast_gen++;
    hipError_t e;
    if ((e = c->gray.ensure((size_t)nframes * w * h)) != hipSuccess) return e;
    hipLaunchKernelGGL(gray_convert, dim3((w + 255) / 256, h, nframes), dim3(256), 0, s, frames, (size_t)w * channels,
                       channels, w, h, c->gray.as<uint8_t>());
    return hipGetLastError();
}

hipError_t launch_fast_detect(slam_ctx* c, hipStream_t s, const uint8_t* img, size_t frame_stride,
                              size_t row_stride, int channels, int nframes, int w, int h,
                              int threshold, int nonmax, int border, int type)
{
    const int ntx = (w + TW - 1) / TW, nbands = (h + kFastTileH - 1) / kFastTileH, nty = (h + TH - 1) / TH;
    c->fast_gen++;
    hipError_t e;
    if ((e = c->gray.ensure((size_t)nframes * w * h)) != hipSuccess) return e;
    if ((e = c->scores.ensure((size_t)nframes * w * h)) != hipSuccess) return e;
    if ((e = c->masks.ensure((size_t)nframes * h * ntx * 8)) != hipSuccess) return e;
    if ((e = c->band_cnt.ensure((size_t)nframes * nbands * 2 * sizeof(int))) != hipSuccess) return e;
    if ((e = hipMemsetAsync(c->band_cnt.p, 0, (size_t)nframes * nbands * 2 * sizeof(int), s)) != hipSuccess)
        return e;
    DetectParams p;
    p.img = img; p.frame_stride = frame_stride; p.row_stride = row_stride; p.channels = channels;
    p.w = w; p.h = h; p.thr = threshold < 0 ? 0 : (threshold > 255 ? 255 : threshold);
    p.border = border; p.ntx = ntx; p.nbands = nbands;
    p.wide = (row_stride % 4 == 0) && (frame_stride % 4 == 0) && ((uintptr_t)img % 4 == 0);
    p.gray_wide = (w % 4 == 0);
    p.xcd = xcd_tiles_on() ? 1 : 0;
    // timing probes give wrong results: read only in -DSLAMHIP_DIAG builds
    // (scripts/diag/build_sift_variant.sh); a normal build ignores the variable
    static const int dbg = [] { return diag_env_int("SLAMHIP_FAST_DBG"); }();
    p.dbg = dbg;
    p.gray = c->gray.as<uint8_t>(); p.masks = c->masks.as<uint64_t>(); p.scores = c->scores.as<uint8_t>();
    p.band_cnt = c->band_cnt.as<int>();
    c->batch.ntx = ntx;
    c->batch.nbands = nbands;
    dim3 grid(ntx, nty, nframes);
    prof_begin(c, 0, s);
    if (type == SLAM_FAST_TYPE_9_16) {
        if (nonmax) hipLaunchKernelGGL((fast_detect<1, 16>), grid, dim3(kFastThreads), 0, s, p);
        else hipLaunchKernelGGL((fast_detect<0, 16>), grid, dim3(kFastThreads), 0, s, p);
    } else if (type == SLAM_FAST_TYPE_7_12) {
        if (nonmax) hipLaunchKernelGGL((fast_detect<1, 12>), grid, dim3(kFastThreads), 0, s, p);
        else hipLaunchKernelGGL((fast_detect<0, 12>), grid, dim3(kFastThreads), 0, s, p);
    } else {
        if (nonmax) hipLaunchKernelGGL((fast_detect<1, 8>), grid, dim3(kFastThreads), 0, s, p);
        else hipLaunchKernelGGL((fast_detect<0, 8>), grid, dim3(kFastThreads), 0, s, p);
    }
    prof_end(c, 0, s);
    return hipGetLastError();
}

hipError_t launch_fast_emit(slam_ctx* c, hipStream_t s, int nframes, int w, int h, int cap)
{
    const int ntx = c->batch.ntx, nbands = c->batch.nbands;
    if (ntx * kFastTileH > 1024) return hipErrorInvalidValue;   // width > 4096
    c->fast_gen++;
    hipError_t e;
    if ((e = c->band_pref.ensure((size_t)nframes * nbands * sizeof(int))) != hipSuccess) return e;
    if ((e = c->frame_info.ensure((size_t)nframes * sizeof(int4))) != hipSuccess) return e;
    if ((e = c->misc.ensure(256)) != hipSuccess) return e;
    if ((e = c->kps.ensure((size_t)cap * sizeof(slam_keypoint))) != hipSuccess) return e;
    if ((e = c->kp_frame.ensure((size_t)cap * sizeof(int))) != hipSuccess) return e;
    hipLaunchKernelGGL(fast_finalize, dim3(1), dim3(1024), 0, s, c->band_cnt.as<int>(), nframes, nbands,
                       c->band_pref.as<int>(), c->frame_info.as<int4>(), c->misc.as<int>(), cap);
    EmitParams p;
    p.masks = c->masks.as<uint64_t>(); p.scores = c->scores.as<uint8_t>();
    p.band_pref = c->band_pref.as<int>(); p.frame_info = c->frame_info.as<int4>();
    p.w = w; p.h = h; p.ntx = ntx; p.nbands = nbands; p.cap = cap;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>();
    hipLaunchKernelGGL(fast_emit, dim3(nbands, nframes), dim3(1024), 0, s, p);
    return hipGetLastError();
}

}  // namespace slamhip
