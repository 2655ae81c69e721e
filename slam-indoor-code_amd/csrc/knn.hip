// Brute-force k = 2 matcher + Lowe ratio test, gfx950 MFMA.
//
// Replaces matchFeatures (reference featureMatchingCPU.cpp:17-43:
// DescriptorMatcher BRUTEFORCE / BRUTEFORCE_HAMMING, knnMatch(query = previous
// frame, train = candidate, k = 2) at :40; CUDA twin featureMatchingCUDA.cpp:
// 19-46) and getGoodMatches (featureMatchingCommon.cpp:37-50).
//
// Distances as an int8 GEMM on the matrix cores (v_mfma_i32_32x32x32_i8):
//   SIFT: descriptors are integers 0..255 (saturate_cast<uchar>), so
//         a' = a - 128 is an exact int8 (one XOR with 0x80) and
//         |a - b|^2 = |a'|^2 + |b'|^2 - 2 <a', b'> exactly in int32.
//   ORB:  bits expanded to +-1 int8: popcount(a ^ b) = (256 - <a', b'>) / 2.
// Orientation: A = train tile (rows t), B = query tile (columns q), so the
// 32x32 accumulator puts one QUERY per lane column and 16 train rows in the
// lane's registers -> the per-query top-2 needs no cross-lane traffic until
// one final merge of lanes l and l ^ 32.  Keys are e = |t'|^2 - 2<q', t'>
// (the query norm is constant per lane), compared with strict < while train
// rows are visited in ascending index order per lane: ties keep the lower
// trainIdx exactly as OpenCV's batchDistance insertion does.  For SIFT
// descriptors with |d| <= 2048 (ours are ~512 by construction) distinct
// squared distances have distinct f32 square roots, so ranking by d^2 equals
// ranking by the reference's sqrt'ed float distance; otherwise MODE_SQRT keys
// on the float bits of sqrtf(d^2).
// Grid: x = 256-query block (4 waves x 64 queries), y = train frame, z = split
// of the train set; partial top-2s are merged by knn_finish.
#include <cfloat>
#include <climits>
#include <cstdlib>

#include <type_traits>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

enum { MODE_L2 = 0, MODE_HAM = 1, MODE_SQRT = 2, MODE_L2P = 3, MODE_HAMP = 4, MODE_L1P = 5 };

struct KnnParams {
    const uint8_t* q;
    const int* qnorm;
    int nq;
    const uint8_t* t;
    const int* tnorm;
    const int4* t_info;   // {offset, count, ...} per frame
    int tsplit;
    int4* part;           // [frame][split][nq] = {e0, i0, e1, i1}
    int keymul;           // packed-key multiplier of the dot product
    int xcd;              // knn_mfma_pk: blocks in XCD-contiguous order (xcd_tile)
};

__device__ inline bool key_lt(int ea, int ia, int eb, int ib)
{
    return ea < eb || (ea == eb && (unsigned)ia < (unsigned)ib);
}

template <int KB, int MODE, bool XOR80>
__global__ __launch_bounds__(256) void knn_mfma(KnnParams p)
{
    constexpr int KS = KB / 32;      // k-steps of 32 bytes
    constexpr int CH = KB / 16;      // 16-byte chunks per row
    __shared__ __attribute__((aligned(16))) uint8_t tile[32 * KB];
    __shared__ __attribute__((aligned(16))) int tn_s[32];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const int fr = blockIdx.y, z = blockIdx.z;
    const int4 info = p.t_info[fr];
    const int off = info.x, nt = info.y;
    const int qbase = blockIdx.x * 256 + wave * 64;
    const uint32_t xm = XOR80 ? 0x80808080u : 0u;

    // query fragments (B operand): lane holds query (lane & 31), k-chunk h
    v4i bq[2][KS];
    int qn[2] = {0, 0};
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
        const int q = qbase + qt * 32 + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            v4i v = {0, 0, 0, 0};
            if (q < p.nq) {
                uint4 u = *reinterpret_cast<const uint4*>(p.q + (size_t)q * KB + ks * 32 + h * 16);
                v = v4i{(int)(u.x ^ xm), (int)(u.y ^ xm), (int)(u.z ^ xm), (int)(u.w ^ xm)};
            }
            bq[qt][ks] = v;
        }
        if (MODE == MODE_SQRT && q < p.nq) qn[qt] = p.qnorm[q];
    }

    int chunk = (nt + p.tsplit - 1) / p.tsplit;
    chunk = (chunk + 31) & ~31;
    const int lo = z * chunk, hi = min(nt, lo + chunk);

    int b1[2] = {INT_MAX, INT_MAX}, b2[2] = {INT_MAX, INT_MAX};
    int i1[2] = {-1, -1}, i2[2] = {-1, -1};

    for (int tb = lo; tb < hi; tb += 32) {
        // stage 32 train rows (swizzled 16-byte chunks) + their keys' base term
        for (int c = tid; c < 32 * CH; c += 256) {
            const int row = c / CH, ch = c - row * CH;
            uint4 u = make_uint4(0, 0, 0, 0);
            if (tb + row < hi) {
                u = *reinterpret_cast<const uint4*>(p.t + (size_t)(off + tb + row) * KB + ch * 16);
                u.x ^= xm; u.y ^= xm; u.z ^= xm; u.w ^= xm;
            }
            *reinterpret_cast<uint4*>(tile + row * KB + ((ch ^ (row & 7)) * 16)) = u;
        }
        if (tid < 32) {
            int v = INT_MAX;
            if (tb + tid < hi) v = p.tnorm ? p.tnorm[off + tb + tid] : 0;
            tn_s[tid] = v;
        }
        __syncthreads();

        v16i acc[2];
#pragma unroll
        for (int qt = 0; qt < 2; qt++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[qt][r] = 0;
        const int arow = lane & 31;
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            const int ch = 2 * ks + h;
            v4i a = *reinterpret_cast<const v4i*>(tile + arow * KB + ((ch ^ (arow & 7)) * 16));
#pragma unroll
            for (int qt = 0; qt < 2; qt++)
                acc[qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[qt][ks], acc[qt], 0, 0, 0);
        }
        int tn[16];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            int4 v = *reinterpret_cast<const int4*>(tn_s + 8 * g + 4 * h);
            tn[4 * g + 0] = v.x; tn[4 * g + 1] = v.y; tn[4 * g + 2] = v.z; tn[4 * g + 3] = v.w;
        }
#pragma unroll
        for (int qt = 0; qt < 2; qt++) {
            int e[16];
            int m = INT_MAX;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                int ev;
                if (MODE == MODE_L2) ev = tn[j] - 2 * acc[qt][j];
                else if (MODE == MODE_HAM) ev = tn[j] - acc[qt][j];
                else ev = tn[j] == INT_MAX ? INT_MAX
                                           : __float_as_int(cr_sqrtf((float)(qn[qt] + tn[j] - 2 * acc[qt][j])));
                e[j] = ev;
                m = min(m, ev);
            }
            if (m < b2[qt]) {
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const int idx = tb + (j & 3) + 8 * (j >> 2) + 4 * h;
                    const int ev = e[j];
                    if (ev < b2[qt]) {
                        if (ev < b1[qt]) { b2[qt] = b1[qt]; i2[qt] = i1[qt]; b1[qt] = ev; i1[qt] = idx; }
                        else { b2[qt] = ev; i2[qt] = idx; }
                    }
                }
            }
        }
        __syncthreads();
    }

    // merge lanes l and l ^ 32 (same query, interleaved row subsets)
#pragma unroll
    for (int qt = 0; qt < 2; qt++) {
        const int ob1 = __shfl_xor(b1[qt], 32, 64), oi1 = __shfl_xor(i1[qt], 32, 64);
        const int ob2 = __shfl_xor(b2[qt], 32, 64), oi2 = __shfl_xor(i2[qt], 32, 64);
        int e0, x0, e1, x1;
        if (key_lt(b1[qt], i1[qt], ob1, oi1)) {
            e0 = b1[qt]; x0 = i1[qt];
            if (key_lt(b2[qt], i2[qt], ob1, oi1)) { e1 = b2[qt]; x1 = i2[qt]; } else { e1 = ob1; x1 = oi1; }
        } else {
            e0 = ob1; x0 = oi1;
            if (key_lt(b1[qt], i1[qt], ob2, oi2)) { e1 = b1[qt]; x1 = i1[qt]; } else { e1 = ob2; x1 = oi2; }
        }
        const int q = qbase + qt * 32 + (lane & 31);
        if (h == 0 && q < p.nq) p.part[((size_t)fr * p.tsplit + z) * p.nq + q] = make_int4(e0, x0, e1, x1);
    }
}

// ---- packed-key variant (the batch path and bounded host inputs) --------------
// Every candidate is one u32 key whose unsigned order is the reference's
// (distance, lower trainIdx) order:
//   L2  (d^2 < 2^21 - 1):  ((|t'|^2 - 2<q', t'> + 2^21) << 10) | row   (row < 1024 per split)
//   HAM:                   ((256 - <q', t'>)            << 22) | row   (= 2 * popcount)
// The per-row part ((|t'|^2 + 2^21) << 10 | row, or 256 << 22 | row) is staged
// once per train row, so each accumulator element costs one v_mad_i32_i24
// (acc * -2^11 or acc * -2^22 + base) and the top-2 update is branch free and
// order free: b2 = med3(b1, k, b2), b1 = min(b1, k) (b1 <= b2 always holds),
// or per two keys b1' = min3(b1, ka, kb), b2' = min(b2, med3(b1, ka, kb)) (3 VALU
// per 2 keys; the round-3 form took 5 per 3).
// -|q'|^2 <= |t'|^2 - 2<q', t'> = d^2 - |q'|^2 < 2^21 keeps the L2 field in
// [0, 2^22); padding rows carry the key 0xffffffff (never selected).
constexpr uint32_t kKeyNone = 0xffffffffu;
#ifndef KNN_QT
#define KNN_QT 2          // SIFT: 32-query tiles per wave
#endif
#ifndef KNN_MINB
#define KNN_MINB 4        // SIFT: workgroups per CU the register budget is set for
#endif
#ifndef KNN_TRACKERS
#define KNN_TRACKERS 1    // independent top-2 trackers per query tile (merged after the walk)
#endif
#ifndef KNN_NTH
#define KNN_NTH 256       // SIFT: threads per workgroup (4 waves of 64 queries sharing each train tile)
#endif
#ifndef KNN_ROWS
#define KNN_ROWS 64
#endif
constexpr int kPkRows = KNN_ROWS;      // train rows staged per iteration (32-row MFMA tiles)
#ifndef KNN_SWZ
#define KNN_SWZ 1
#endif
#ifndef KNN_PRIO
#define KNN_PRIO 0
#endif
// 16-byte chunk c of tile row r lives at chunk c ^ swz(r).  The A-fragment read
// (ds_read_b128, lane = row within a 32-row tile) is serviced in four 16-lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md, LDS):
// a row's bank window is 32 (r & 1) + 4 (c ^ swz(r)), so the 16 rows of a group
// need distinct (r & 1, swz(r)).  swz = r & 7 repeats every value twice in
// every group (rows 0 and 24, ...: 2-way conflicts on every read); swz =
// (r >> 1) & 7 is a bijection on the even and on the odd rows of each group.
__device__ __forceinline__ int knn_swz(int r) { return KNN_SWZ ? (r >> 1) & 7 : r & 7; }

// insert (e, x) into the sorted pair (e0, x0) <= (e1, x1)
__device__ __forceinline__ void top2_insert(int& e0, int& x0, int& e1, int& x1, int e, int x)
{
    if (key_lt(e, x, e1, x1)) {
        if (key_lt(e, x, e0, x0)) { e1 = e0; x1 = x0; e0 = e; x0 = x; }
        else { e1 = e; x1 = x; }
    }
}

// v_med3_u32 as inline asm (the plain min / max form is matched to the same
// instruction, but its visibility lets the scheduler hoist the epilogue and the
// kernels spill).  The asm is opaque to the MFMA -> VALU hazard checks: when an
// operand is an MFMA result register itself (Hamming keys are the accumulator's
// bits), an asm med3 placed near the MFMA can read the register before it is
// written.  `after` is a compiler-visible value computed from the same operands
// (their min3 / min): the asm cannot be scheduled before it, and the compiler
// resolves the hazard for that earlier read.
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c, uint32_t after)
{
    uint32_t r;
    __asm__("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c), "v"(after));
    return r;
}

__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c)
{
    return min(min(a, b), c);   // v_min3_u32
}

// two keys into the running pair b1 <= b2: of {b1, ka, kb} sorted x <= m <= y
// (m = med3), b2 >= b1 >= x, so the second smallest of {b1, b2, ka, kb} is
// min(b2, m) -- 3 VALU per two keys
__device__ __forceinline__ void top2_pair(uint32_t& b1, uint32_t& b2, uint32_t ka, uint32_t kb)
{
    const uint32_t n1 = min3_u32(b1, ka, kb);
    b2 = min(b2, med3_u32(b1, ka, kb, n1));
    b1 = n1;
}

template <int KB, bool HAM, int QT, int MINB, int NTH = 256>
__global__ __launch_bounds__(NTH, MINB) void knn_mfma_pk(KnnParams p)
{
    constexpr int KS = KB / 32;              // k-steps of 32 bytes (32 int8 / 64 FP4 elements)
    constexpr int CH = KB / 16;              // 16-byte chunks per row
    constexpr int PER = kPkRows * CH / NTH;  // staged chunks per thread
    static_assert(PER >= 1 && kPkRows * CH % NTH == 0, "whole staged chunks per thread");
    constexpr int SH = 10;                   // L2 index bits (Hamming keys: 10 fraction bits)
    const int keymul = p.keymul;              // -2^11 (L2)
    __shared__ __attribute__((aligned(16))) uint8_t tile2[2][kPkRows * KB];   // double-buffered train tile
    __shared__ __attribute__((aligned(16))) uint32_t tk2[2][kPkRows];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    int bx, fr, z;
    xcd_tile(p.xcd != 0, bx, fr, z);
    const int4 info = p.t_info[fr];
    const int off = info.x, nt = info.y;
    const int qbase = bx * (NTH * QT / 2) + wave * (32 * QT);
    if (KNN_PRIO == 1 && (bx & 1)) __builtin_amdgcn_s_setprio(1);
    // L2: u8 -> i8 (x ^ 0x80 on both sides).  Hamming: FP4 +-1 elements, the
    // query's signs flipped (x ^ 0x8 per nibble) so the MFMA accumulates -dot
    const uint32_t xq = HAM ? 0x88888888u : 0x80808080u, xt = HAM ? 0u : 0x80808080u;

    // query fragments (B operand): lane holds query (lane & 31), k-chunk h
    v4i bq[QT][KS];
#pragma unroll
    for (int qt = 0; qt < QT; qt++) {
        const int q = qbase + qt * 32 + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            // clamped unconditional load (all of them in flight at once), masked after
            const uint4 u = *reinterpret_cast<const uint4*>(p.q + (size_t)min(q, p.nq - 1) * KB + ks * 32 + h * 16);
            v4i v = v4i{(int)(u.x ^ xq), (int)(u.y ^ xq), (int)(u.z ^ xq), (int)(u.w ^ xq)};
            if (q >= p.nq) v = v4i{0, 0, 0, 0};
            bq[qt][ks] = v;
        }
    }

    int chunk = (nt + p.tsplit - 1) / p.tsplit;
    chunk = (chunk + kPkRows - 1) / kPkRows * kPkRows;
    const int lo = z * chunk, hi = min(nt, lo + chunk);

    // KNN_TRACKERS independent (b1, b2) pairs per query tile: the groups of a
    // tile alternate between them, so their dependent min / max chains
    // interleave; keys are distinct (row bits), so merging the pairs after the
    // walk gives the same top two
    constexpr int NT = KNN_TRACKERS;
    uint32_t b1[NT][QT], b2[NT][QT];
#pragma unroll
    for (int u = 0; u < NT; u++)
#pragma unroll
        for (int qt = 0; qt < QT; qt++) { b1[u][qt] = kKeyNone; b2[u][qt] = kKeyNone; }

    // the next tile's rows are loaded unconditionally (row clamped into the split)
    // and masked when stored: the loads stay in flight through the MFMAs instead
    // of being waited for where they are issued
    uint4 pre[PER];
    int pre_tn = 0;
    int ld_tb = lo;
    auto load = [&](int tb) {
        ld_tb = tb;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int c = tid + NTH * u, row = c / CH, ch = c - row * CH;
            pre[u] = *reinterpret_cast<const uint4*>(p.t + (size_t)(off + min(tb + row, hi - 1)) * KB + ch * 16);
        }
        if (!HAM && tid < kPkRows) pre_tn = p.tnorm[off + min(tb + tid, hi - 1)];
    };

    auto store = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int c = tid + NTH * u, row = c / CH, ch = c - row * CH;
            uint4 v = pre[u];
            if (!HAM) { v.x ^= xt; v.y ^= xt; v.z ^= xt; v.w ^= xt; }
            if (ld_tb + row >= hi) v = make_uint4(0, 0, 0, 0);
            *reinterpret_cast<uint4*>(tile2[buf] + row * KB + ((ch ^ knn_swz(row)) * 16)) = v;
        }
        if (tid < kPkRows) {
            const int row = ld_tb + tid;
            uint32_t k = HAM ? 0x7f800000u : kKeyNone;       // Hamming: +inf, never below a real key
            if (row < hi) {
                const uint32_t loc = (uint32_t)(row - lo);    // < 2^10: the host bounds the split size
                k = HAM ? __float_as_uint(768.f + (float)loc * (1.f / 1024.f))
                        : (((uint32_t)(pre_tn + (1 << 21)) << 10) | loc);
            }
            tk2[buf][tid] = k;
        }
    };
    if (lo < hi) {
        load(lo);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int tb = lo; tb < hi; tb += kPkRows, buf ^= 1) {
        const bool more = tb + kPkRows < hi;
        if (more) load(tb + kPkRows);                  // in flight during the MFMAs below
        const uint8_t* tile = tile2[buf];
        const uint32_t* tk = tk2[buf];
#pragma unroll
        for (int rt = 0; rt < kPkRows / 32; rt++) {
            // the per-row key part of the lane's 16 outputs (rows rt * 32 + 8 g + 4 h + i).
            // Hamming seeds the accumulator with it; L2 reads it after the MFMAs, one
            // pair of rows per top-2 step (live across the MFMAs, all 16 cost 42 VGPRs:
            // 126 -> 168, 4 -> 3 waves per SIMD; read up front for the pairwise update, 3
            // spills at 128)
            uint32_t kb[16];
            auto load_kb = [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const uint4 v = *reinterpret_cast<const uint4*>(tk + rt * 32 + 8 * g + 4 * h);
                    kb[4 * g + 0] = v.x; kb[4 * g + 1] = v.y; kb[4 * g + 2] = v.z; kb[4 * g + 3] = v.w;
                }
            };
            if constexpr (HAM) load_kb();
            // L2: i32 dot products.  Hamming (FP4 MFMA, the query's signs flipped):
            // the accumulator starts at the row's key 768 + row / 1024 and ends at
            // 768 - dot + row / 1024, exact in f32 (10 fraction bits below 2048);
            // positive, so its bit pattern orders like the value: it IS the key
            typedef typename std::conditional<HAM, v16f, v16i>::type AccT;
            AccT acc[QT];
#pragma unroll
            for (int qt = 0; qt < QT; qt++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    if constexpr (HAM) acc[qt][r] = __uint_as_float(kb[r]);
                    else acc[qt][r] = 0;
                }
            const int arow = rt * 32 + (lane & 31);
            if (KNN_PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const int ch = 2 * ks + h;
                v4i a = *reinterpret_cast<const v4i*>(tile + arow * KB + ((ch ^ knn_swz(arow)) * 16));
#pragma unroll
                for (int qt = 0; qt < QT; qt++) {
                    if constexpr (HAM) {
                        const v8i a8 = {a[0], a[1], a[2], a[3], 0, 0, 0, 0};
                        const v4i bb = bq[qt][ks];
                        const v8i b8 = {bb[0], bb[1], bb[2], bb[3], 0, 0, 0, 0};
                        acc[qt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[qt], 4, 4, 0, 127, 0, 127);
                    } else {
                        acc[qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[qt][ks], acc[qt], 0, 0, 0);
                    }
                }
            }
            if (KNN_PRIO == 2) __builtin_amdgcn_s_setprio(0);
#pragma unroll
            for (int qt = 0; qt < QT; qt++) {
                // compiler-visible mul24 + add (v_mad_i32_i24; the multiplier is a
                // kernel argument so it is not folded into a shift): inline asm
                // reading MFMA results would bypass the MFMA -> VALU hazard checks
                // keys in pairs (top2_pair: 3 VALU per 2 keys; keys are distinct: row bits)
#pragma unroll
                for (int j = 0; j < 16; j += 2) {
                    uint32_t ka, kc;
                    if constexpr (HAM) {
                        ka = __float_as_uint(acc[qt][j]);
                        kc = __float_as_uint(acc[qt][j + 1]);
                    } else {
                        // the pair's row parts: one ds_read_b64 (rows 8 g + 4 h + i, i + 1)
                        const uint2 kr = *reinterpret_cast<const uint2*>(tk + rt * 32 + 8 * (j >> 2) + 4 * h + (j & 3));
                        ka = (uint32_t)(__mul24(acc[qt][j], keymul) + (int)kr.x);
                        kc = (uint32_t)(__mul24(acc[qt][j + 1], keymul) + (int)kr.y);
                    }
                    top2_pair(b1[(j / 2) % NT][qt], b2[(j / 2) % NT][qt], ka, kc);
                }
            }
        }
        // the other buffer was last read before the previous barrier: refill it now
        if (more) store(buf ^ 1);
        __syncthreads();
    }

    // the trackers' pairs merged; then lanes l and l ^ 32 (same query, interleaved
    // row subsets); keys are order free
#pragma unroll
    for (int u = 1; u < NT; u++)
#pragma unroll
        for (int qt = 0; qt < QT; qt++) {
            const uint32_t c2 = min(max(b1[0][qt], b1[u][qt]), min(b2[0][qt], b2[u][qt]));
            b1[0][qt] = min(b1[0][qt], b1[u][qt]);
            b2[0][qt] = c2;
        }
#pragma unroll
    for (int qt = 0; qt < QT; qt++) {
        const uint32_t o1 = (uint32_t)__shfl_xor((int)b1[0][qt], 32, 64), o2 = (uint32_t)__shfl_xor((int)b2[0][qt], 32, 64);
        const uint32_t c1 = min(b1[0][qt], o1), c2 = min(max(b1[0][qt], o1), min(b2[0][qt], o2));
        const int q = qbase + qt * 32 + (lane & 31);
        if (h == 0 && q < p.nq) {
            int e0, x0, e1, x1;
            if constexpr (HAM) {
                // float keys: 768 - dot + row / 1024; +inf (or the initial all-ones) = none.
                // e = 256 - dot = 2 * Hamming, the code knn_finish expects
                auto dec = [&](uint32_t c, int& e, int& x) {
                    if (c >= 0x7f800000u) { e = INT_MAX; x = -1; return; }
                    const float f = __uint_as_float(c), d = floorf(f);
                    e = (int)d - 512;
                    x = lo + (int)((f - d) * 1024.f);
                };
                dec(c1, e0, x0);
                dec(c2, e1, x1);
            } else {
                const uint32_t m = (1u << SH) - 1;
                e0 = c1 == kKeyNone ? INT_MAX : (int)(c1 >> SH); x0 = c1 == kKeyNone ? -1 : lo + (int)(c1 & m);
                e1 = c2 == kKeyNone ? INT_MAX : (int)(c2 >> SH); x1 = c2 == kKeyNone ? -1 : lo + (int)(c2 & m);
            }
            p.part[((size_t)fr * p.tsplit + z) * p.nq + q] = make_int4(e0, x0, e1, x1);
        }
    }
}

// ---- packed keys with the MFMAs and the key epilogue software-pipelined ----
// knn_mfma_pk issues a 32-row tile's MFMAs and then runs the same tile's key
// epilogue (mad24 + top-2: ~3.4 VALU per key) on their results, so one wave
// alternates between the matrix pipe and the VALU and the SQ counters show the
// two busy fractions adding up (0.37 + 0.69).  Here the epilogue of tile j - 1
// runs while tile j's MFMAs execute: two accumulator sets (A / B, renamed by
// the two-tile unroll), and the scheduler is told to interleave them (one MFMA,
// then the VALU that fits in its 32 cycles).  The per-row key parts live in a
// three-slot ring, so a tile's keys are still staged when its epilogue runs in
// the next iteration (the slot is rewritten two iterations later, behind a
// barrier every wave has passed).  Keys, order and results are those of
// knn_mfma_pk.
#ifndef KNN_PIPE_MINB
#define KNN_PIPE_MINB 3       // workgroups (waves per SIMD) the register budget is set for
#endif
// L2 (int8 MFMA, keys acc * -2^11 + the row part, ring-staged) or Hamming (FP4
// MFMA on the +-1 expansion, the accumulator seeded with the row's float key
// 768 + row / 1024 and ending at 768 - dot + row / 1024, whose bits are the key:
// knn_mfma_pk's Hamming form)
template <int QT, int MINB, bool HAM>
__global__ __launch_bounds__(256, MINB) void knn_pipe(KnnParams p)
{
    constexpr int KB = HAM ? kOrbExpBytes : 128, KS = KB / 32, CH = KB / 16;
    constexpr int PER = kPkRows * CH / 256;
    constexpr int SH = 10;
    // VALU per MFMA in the interleave: the epilogue's ~3.4 (L2: mad + top-2) or
    // ~1.7 (Hamming: top-2) instructions per key over 32 keys per lane and tile
    constexpr int VPM = HAM ? 7 : 11;
    const int keymul = p.keymul;              // -2^11 (L2)
    __shared__ __attribute__((aligned(16))) uint8_t tile2[2][kPkRows * KB];
    __shared__ __attribute__((aligned(16))) uint32_t tk3[4][kPkRows];     // ring of 3 + the "no tile" slot

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    const int fr = blockIdx.y, z = blockIdx.z;
    const int4 info = p.t_info[fr];
    const int off = info.x, nt = info.y;
    const int qbase = blockIdx.x * (256 * QT / 2) + wave * (32 * QT);
    // L2: u8 -> i8 on both sides.  Hamming: the query's FP4 signs flipped
    const uint32_t xq = HAM ? 0x88888888u : 0x80808080u, xt = HAM ? 0u : 0x80808080u;

    v4i bq[QT][KS];
#pragma unroll
    for (int qt = 0; qt < QT; qt++) {
        const int q = qbase + qt * 32 + (lane & 31);
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            // clamped unconditional load (all of them in flight at once), masked after
            const uint4 u = *reinterpret_cast<const uint4*>(p.q + (size_t)min(q, p.nq - 1) * KB + ks * 32 + h * 16);
            v4i v = v4i{(int)(u.x ^ xq), (int)(u.y ^ xq), (int)(u.z ^ xq), (int)(u.w ^ xq)};
            if (q >= p.nq) v = v4i{0, 0, 0, 0};
            bq[qt][ks] = v;
        }
    }

    int chunk = (nt + p.tsplit - 1) / p.tsplit;
    chunk = (chunk + kPkRows - 1) / kPkRows * kPkRows;
    const int lo = z * chunk, hi = min(nt, lo + chunk);

    uint32_t b1[QT], b2[QT];
#pragma unroll
    for (int qt = 0; qt < QT; qt++) { b1[qt] = kKeyNone; b2[qt] = kKeyNone; }

    // unconditional (clamped) loads, masked at the store: in flight through the MFMAs
    uint4 pre[PER];
    int pre_tn = 0;
    int ld_tb = lo;
    auto load = [&](int tb) {
        ld_tb = tb;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int c = tid + 256 * u, row = c / CH, ch = c - row * CH;
            pre[u] = *reinterpret_cast<const uint4*>(p.t + (size_t)(off + min(tb + row, hi - 1)) * KB + ch * 16);
        }
        if (!HAM && tid < kPkRows) pre_tn = p.tnorm[off + min(tb + tid, hi - 1)];
    };
    auto store = [&](int buf, int slot) {
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int c = tid + 256 * u, row = c / CH, ch = c - row * CH;
            uint4 v = pre[u];
            v.x ^= xt; v.y ^= xt; v.z ^= xt; v.w ^= xt;
            if (ld_tb + row >= hi) v = make_uint4(0, 0, 0, 0);
            *reinterpret_cast<uint4*>(tile2[buf] + row * KB + ((ch ^ knn_swz(row)) * 16)) = v;
        }
        if (tid < kPkRows) {
            const int row = ld_tb + tid;
            uint32_t k = HAM ? 0x7f800000u : kKeyNone;       // Hamming: +inf, never below a real key
            if (row < hi) {
                const uint32_t loc = (uint32_t)(row - lo);    // < 2^10: the host bounds the split size
                k = HAM ? __float_as_uint(768.f + (float)loc * (1.f / 1024.f))
                        : (((uint32_t)(pre_tn + (1 << 21)) << 10) | loc);
            }
            tk3[slot][tid] = k;
        }
    };
    // the "no tile" slot: the first step's epilogue runs on kKeyNone keys (L2: zero
    // accumulators and all-ones key parts; Hamming: +inf accumulators)
    if (tid < kPkRows) tk3[3][tid] = kKeyNone;
    if (lo < hi) {
        load(lo);
        store(0, 0);
    }
    __syncthreads();

    typedef typename std::conditional<HAM, v16f, v16i>::type AccT;
    AccT accA[QT], accB[QT];
#pragma unroll
    for (int qt = 0; qt < QT; qt++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
            if constexpr (HAM) { accA[qt][r] = __uint_as_float(0x7f800000u); accB[qt][r] = __uint_as_float(0x7f800000u); }
            else { accA[qt][r] = 0; accB[qt][r] = 0; }
        }

    // the lane's 16 row key parts of a 32-row tile (rows 8 g + 4 h + i)
    auto load_kb = [&](uint32_t (&kb)[16], const uint32_t* tkp) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint4 v = *reinterpret_cast<const uint4*>(tkp + 8 * g + 4 * h);
            kb[4 * g + 0] = v.x; kb[4 * g + 1] = v.y; kb[4 * g + 2] = v.z; kb[4 * g + 3] = v.w;
        }
    };
    // the previous tile's keys, top-2 in groups of three
    auto epilogue = [&](const AccT (&acc)[QT], const uint32_t* tkp) __attribute__((always_inline)) {
        uint32_t kb[16];
        if constexpr (!HAM) load_kb(kb, tkp);
#pragma unroll
        for (int qt = 0; qt < QT; qt++) {
            uint32_t k[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if constexpr (HAM) k[j] = __float_as_uint(acc[qt][j]);
                else k[j] = (uint32_t)(__mul24(acc[qt][j], keymul) + (int)kb[j]);
            }
#pragma unroll
            for (int j = 0; j < 16; j += 2) top2_pair(b1[qt], b2[qt], k[j], k[j + 1]);
        }
    };
    // one 32-row tile: its MFMAs into acc, the previous tile's epilogue beside them
    auto step = [&](const uint8_t* tile, int rt, AccT (&acc)[QT], const AccT (&prev)[QT], const uint32_t* tk_cur,
                    const uint32_t* tk_prv) __attribute__((always_inline)) {
        const int arow = rt * 32 + (lane & 31);
        v4i a[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
            a[ks] = *reinterpret_cast<const v4i*>(tile + arow * KB + (((2 * ks + h) ^ knn_swz(arow)) * 16));
        if constexpr (HAM) {
            uint32_t kb[16];
            load_kb(kb, tk_cur + rt * 32);
#pragma unroll
            for (int qt = 0; qt < QT; qt++)
#pragma unroll
                for (int r = 0; r < 16; r++) acc[qt][r] = __uint_as_float(kb[r]);
        } else {
#pragma unroll
            for (int qt = 0; qt < QT; qt++)
#pragma unroll
                for (int r = 0; r < 16; r++) acc[qt][r] = 0;
        }
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
            for (int qt = 0; qt < QT; qt++) {
                if constexpr (HAM) {
                    const v8i a8 = {a[ks][0], a[ks][1], a[ks][2], a[ks][3], 0, 0, 0, 0};
                    const v4i bb = bq[qt][ks];
                    const v8i b8 = {bb[0], bb[1], bb[2], bb[3], 0, 0, 0, 0};
                    acc[qt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[qt], 4, 4, 0, 127, 0, 127);
                } else {
                    acc[qt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[ks], bq[qt][ks], acc[qt], 0, 0, 0);
                }
            }
        epilogue(prev, tk_prv);
        // scheduling: the tile's fragment and key reads first, then each MFMA
        // followed by the VALU that fits in its 32 cycles
        __builtin_amdgcn_sched_group_barrier(0x100, KS + 4, 0);
#pragma unroll
        for (int i = 0; i < KS * QT; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
        }
    };

    int buf = 0, slot = 0;
    const uint32_t* tk_prev = tk3[3];
    for (int tb = lo; tb < hi; tb += kPkRows) {
        const bool more = tb + kPkRows < hi;
        const int nslot = slot == 2 ? 0 : slot + 1;
        if (more) load(tb + kPkRows);
        const uint8_t* tile = tile2[buf];
        const uint32_t* tk = tk3[slot];
        step(tile, 0, accA, accB, tk, tk_prev);
        step(tile, 1, accB, accA, tk, tk);
        tk_prev = tk + 32;
        if (more) store(buf ^ 1, nslot);
        __syncthreads();
        buf ^= 1;
        slot = nslot;
    }
    epilogue(accB, tk_prev);

#pragma unroll
    for (int qt = 0; qt < QT; qt++) {
        const uint32_t o1 = (uint32_t)__shfl_xor((int)b1[qt], 32, 64), o2 = (uint32_t)__shfl_xor((int)b2[qt], 32, 64);
        const uint32_t c1 = min(b1[qt], o1), c2 = min(max(b1[qt], o1), min(b2[qt], o2));
        const int q = qbase + qt * 32 + (lane & 31);
        if (h == 0 && q < p.nq) {
            int e0, x0, e1, x1;
            if constexpr (HAM) {
                auto dec = [&](uint32_t c, int& e, int& x) {
                    if (c >= 0x7f800000u) { e = INT_MAX; x = -1; return; }
                    const float f = __uint_as_float(c), d = floorf(f);
                    e = (int)d - 512;
                    x = lo + (int)((f - d) * 1024.f);
                };
                dec(c1, e0, x0);
                dec(c2, e1, x1);
            } else {
                const uint32_t m = (1u << SH) - 1;
                e0 = c1 == kKeyNone ? INT_MAX : (int)(c1 >> SH); x0 = c1 == kKeyNone ? -1 : lo + (int)(c1 & m);
                e1 = c2 == kKeyNone ? INT_MAX : (int)(c2 >> SH); x1 = c2 == kKeyNone ? -1 : lo + (int)(c2 & m);
            }
            p.part[((size_t)fr * p.tsplit + z) * p.nq + q] = make_int4(e0, x0, e1, x1);
        }
    }
}

// ---- L1 (NORM_L1: the reference's CUDA-build SIFT_BF matcher,
// featureMatchingCUDA.cpp:28 createBFMatcher(NORM_L1)) over SIFT descriptors
// (u8 0..255) ---------------------------------------------------------------------
// |q - t|_1 is not a dot product, so no MFMA: v_sad_u8 sums the absolute
// differences of 4 bytes per instruction into an exact integer (<= 128 * 255
// < 2^15, so the reference's f32 sum is exact in any order and equal to it).
// A thread holds two queries (64 VGPRs); 64-row train tiles are staged in LDS
// (double buffered) and every row is read as a broadcast.  Keys: (L1 << 17) |
// row (< 2^17 rows per split), the top-2 as in knn_mfma_pk.
constexpr int kL1Rows = 64;

template <int QPT>
__global__ __launch_bounds__(256) void knn_l1(KnnParams p)
{
    __shared__ __attribute__((aligned(16))) uint4 tile[2][kL1Rows * 8];
    const int tid = threadIdx.x;
    const int fr = blockIdx.y, z = blockIdx.z;
    const int4 info = p.t_info[fr];
    const int off = info.x, nt = info.y;
    uint4 qv[QPT][8];
#pragma unroll
    for (int u = 0; u < QPT; u++) {
        const int q = blockIdx.x * (256 * QPT) + u * 256 + tid;
#pragma unroll
        for (int k = 0; k < 8; k++)
            qv[u][k] = q < p.nq ? reinterpret_cast<const uint4*>(p.q + (size_t)q * 128)[k] : make_uint4(0, 0, 0, 0);
    }
    int chunk = (nt + p.tsplit - 1) / p.tsplit;
    chunk = (chunk + kL1Rows - 1) / kL1Rows * kL1Rows;
    const int lo = z * chunk, hi = min(nt, lo + chunk);
    uint32_t b1[QPT], b2[QPT];
#pragma unroll
    for (int u = 0; u < QPT; u++) { b1[u] = kKeyNone; b2[u] = kKeyNone; }
    uint4 pre[2];
    auto load = [&](int tb) {
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const int e = tid + 256 * v, row = e >> 3, ch = e & 7;
            pre[v] = tb + row < hi ? reinterpret_cast<const uint4*>(p.t + (size_t)(off + tb + row) * 128)[ch]
                                   : make_uint4(0, 0, 0, 0);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int v = 0; v < 2; v++) tile[buf][tid + 256 * v] = pre[v];
    };
    if (lo < hi) {
        load(lo);
        store(0);
    }
    __syncthreads();
    int buf = 0;
    for (int tb = lo; tb < hi; tb += kL1Rows, buf ^= 1) {
        const bool more = tb + kL1Rows < hi;
        if (more) load(tb + kL1Rows);
        const int nr = min(kL1Rows, hi - tb);
        for (int r = 0; r < nr; r++) {
            const uint4* tr = tile[buf] + r * 8;   // the same row for every lane: broadcast reads
            uint32_t acc[QPT];
#pragma unroll
            for (int u = 0; u < QPT; u++) acc[u] = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint4 t = tr[k];
#pragma unroll
                for (int u = 0; u < QPT; u++) {
                    acc[u] = __builtin_amdgcn_sad_u8(qv[u][k].x, t.x, acc[u]);
                    acc[u] = __builtin_amdgcn_sad_u8(qv[u][k].y, t.y, acc[u]);
                    acc[u] = __builtin_amdgcn_sad_u8(qv[u][k].z, t.z, acc[u]);
                    acc[u] = __builtin_amdgcn_sad_u8(qv[u][k].w, t.w, acc[u]);
                }
            }
            const uint32_t loc = (uint32_t)(tb + r - lo);
#pragma unroll
            for (int u = 0; u < QPT; u++) {
                const uint32_t k = (acc[u] << 17) | loc;
                const uint32_t nb1 = min(b1[u], k);
                b2[u] = med3_u32(b1[u], k, b2[u], nb1);
                b1[u] = nb1;
            }
        }
        if (more) store(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < QPT; u++) {
        const int q = blockIdx.x * (256 * QPT) + u * 256 + tid;
        if (q < p.nq) {
            const uint32_t m = (1u << 17) - 1;
            const int e0 = b1[u] == kKeyNone ? INT_MAX : (int)(b1[u] >> 17), x0 = b1[u] == kKeyNone ? -1 : lo + (int)(b1[u] & m);
            const int e1 = b2[u] == kKeyNone ? INT_MAX : (int)(b2[u] >> 17), x1 = b2[u] == kKeyNone ? -1 : lo + (int)(b2[u] & m);
            p.part[((size_t)fr * p.tsplit + z) * p.nq + q] = make_int4(e0, x0, e1, x1);
        }
    }
}

struct FinishParams {
    const int4* part;
    int nq, nframes, tsplit, mode;
    const int* qnorm;
    double ratio;
    const int4* t_info;
    int2* top_idx;
    float2* top_dist;
    slam_dmatch* rec;
    uint8_t* flag;
    int* counts;
};

__global__ __launch_bounds__(256) void knn_finish(FinishParams p)
{
    const int q = blockIdx.x * 256 + threadIdx.x, fr = blockIdx.y;
    bool ok = false;
    if (q < p.nq) {
        int e0 = INT_MAX, x0 = -1, e1 = INT_MAX, x1 = -1;
        for (int z = 0; z < p.tsplit; z++) {
            const int4 v = p.part[((size_t)fr * p.tsplit + z) * p.nq + q];
            // insert (v.x, v.y) then (v.z, v.w) into the sorted pair
            if (key_lt(v.x, v.y, e1, x1)) {
                if (key_lt(v.x, v.y, e0, x0)) { e1 = e0; x1 = x0; e0 = v.x; x0 = v.y; }
                else { e1 = v.x; x1 = v.y; }
            }
            if (key_lt(v.z, v.w, e1, x1)) {
                if (key_lt(v.z, v.w, e0, x0)) { e1 = e0; x1 = x0; e0 = v.z; x0 = v.w; }
                else { e1 = v.z; x1 = v.w; }
            }
        }
        float d0 = FLT_MAX, d1 = FLT_MAX;
        if (p.mode == MODE_L2) {
            const int qn = p.qnorm[q];
            if (x0 >= 0) d0 = cr_sqrtf((float)(qn + e0));
            if (x1 >= 0) d1 = cr_sqrtf((float)(qn + e1));
        } else if (p.mode == MODE_HAM) {
            if (x0 >= 0) d0 = (float)((256 + e0) / 2);
            if (x1 >= 0) d1 = (float)((256 + e1) / 2);
        } else if (p.mode == MODE_L2P) {
            const int qn = p.qnorm[q];
            if (x0 >= 0) d0 = cr_sqrtf((float)(qn + e0 - (1 << 21)));
            if (x1 >= 0) d1 = cr_sqrtf((float)(qn + e1 - (1 << 21)));
        } else if (p.mode == MODE_HAMP) {
            if (x0 >= 0) d0 = (float)(e0 / 2);
            if (x1 >= 0) d1 = (float)(e1 / 2);
        } else if (p.mode == MODE_L1P) {
            if (x0 >= 0) d0 = (float)e0;
            if (x1 >= 0) d1 = (float)e1;
        } else {
            if (x0 >= 0) d0 = __int_as_float(e0);
            if (x1 >= 0) d1 = __int_as_float(e1);
        }
        const size_t o = (size_t)fr * p.nq + q;
        if (p.top_idx) { p.top_idx[o] = make_int2(x0, x1); p.top_dist[o] = make_float2(d0, d1); }
        ok = x0 >= 0 && x1 >= 0 && (double)d0 < p.ratio * (double)d1;
        slam_dmatch m;
        m.queryIdx = q; m.trainIdx = x0; m.imgIdx = 0; m.distance = d0;
        p.rec[o] = m;
        p.flag[o] = ok ? 1 : 0;
    }
    const uint64_t b = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&p.counts[fr], __popcll(b));
}

// order-preserving compaction of the ratio-test survivors, one workgroup per frame
__global__ __launch_bounds__(1024) void knn_compact(const slam_dmatch* rec, const uint8_t* flag, int nq,
                                                    slam_dmatch* out, int* out_counts, int stride)
{
    __shared__ int wtot[16];
    __shared__ int running;
    const int fr = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) running = 0;
    __syncthreads();
    for (int base = 0; base < nq; base += 1024) {
        const int q = base + t;
        const int f = (q < nq) ? flag[(size_t)fr * nq + q] : 0;
        const uint64_t b = __ballot(f != 0);
        const int below = __popcll(b & ((1ull << lane) - 1));
        if (lane == 0) wtot[wave] = __popcll(b);
        __syncthreads();
        int wb = running;
        for (int i = 0; i < wave; i++) wb += wtot[i];
        if (f) out[(size_t)fr * stride + wb + below] = rec[(size_t)fr * nq + q];
        __syncthreads();
        if (t == 0) { int s = 0; for (int i = 0; i < 16; i++) s += wtot[i]; running += s; }
        __syncthreads();
    }
    if (t == 0) out_counts[fr] = running;
}

// SLAMHIP_KNN_PIPE=1 selects knn_pipe instead of knn_mfma_pk (the same results;
// r4ab on MI355X, 210 x 10.1k x 9.6k L2: 3.16 vs 2.98 ms -- the two accumulator
// sets cost a wave per SIMD and the interleave does not win it back)
// SLAMHIP_KNN_PIPE=2 (SIFT L2 only): knn_pipe with one 32-query tile per wave
// (two 16-register accumulator sets instead of two 32-register ones), sized
// for 4 waves per SIMD
int knn_pipe_mode()
{
    static const int m = [] {
        const char* e = getenv("SLAMHIP_KNN_PIPE");
        return e ? atoi(e) : 0;
    }();
    return m;
}
bool knn_pipe_enabled() { return knn_pipe_mode() == 1; }

}  // namespace

hipError_t launch_knn(slam_ctx* c, hipStream_t s, int kb, const void* q, const int32_t* qnorm, int nq,
                      const void* t, const int32_t* tnorm, const int32_t* t_info, int nframes, int max_nt,
                      int mode, int tsplit, int4* part)
{
    if (nq <= 0 || nframes <= 0) return hipSuccess;
    // packed L2 keys carry 10 index bits: a split holds at most 1024 train rows
    if (mode == MODE_L2P && (max_nt + tsplit - 1) / tsplit > 1024) return hipErrorInvalidValue;
    // Hamming float keys carry the row in 10 fraction bits: at most 1024 rows per split
    if (mode == MODE_HAMP && (max_nt + tsplit - 1) / tsplit > 1024) return hipErrorInvalidValue;
    // L1 keys: (L1 << 17) | row, rows 0 .. 2^17 - 1 per split (the api.cpp split bound)
    if (mode == MODE_L1P && (max_nt + tsplit - 1) / tsplit > (1 << 17)) return hipErrorInvalidValue;
    KnnParams p;
    p.q = (const uint8_t*)q; p.qnorm = qnorm; p.nq = nq; p.t = (const uint8_t*)t; p.tnorm = tnorm;
    p.t_info = (const int4*)t_info; p.tsplit = tsplit; p.part = part;
    p.keymul = mode == MODE_HAMP ? -(1 << 22) : -(1 << 11);
    // SLAMHIP_KNN_XCD=1: knn_mfma_pk's blocks in XCD-contiguous order.  Its fetch
    // falls 2.25 -> 0.29 GB per launch but the launch runs 3 % longer
    // (scripts/r5_knnxcd.sh: 2.76 -> 2.83 ms at 210 candidates), so it is opt-in
    static const int kxcd = [] { const char* e = getenv("SLAMHIP_KNN_XCD"); return e && e[0] == '1' ? 1 : 0; }();
    p.xcd = kxcd;
    // SIFT packed-key launches: KNN_QT query tiles of 32 per wave (4 waves per block)
    const bool pipe1 = kb == 128 && mode == MODE_L2P && knn_pipe_mode() == 2;
    const bool qt1 = kb == 128 && mode == MODE_L2P && knn_pipe_mode() == 3;     // control: knn_mfma_pk, QT 1
    const int qblk = (pipe1 || qt1) ? 128 : (kb == 128 && mode == MODE_L2P) ? KNN_NTH / 2 * KNN_QT : 256;
    dim3 grid((nq + qblk - 1) / qblk, nframes, tsplit);
    prof_begin(c, 2, s);
    if (kb == 128 && mode == MODE_L2) hipLaunchKernelGGL((knn_mfma<128, MODE_L2, true>), grid, dim3(256), 0, s, p);
    else if (kb == 128 && mode == MODE_SQRT) hipLaunchKernelGGL((knn_mfma<128, MODE_SQRT, true>), grid, dim3(256), 0, s, p);
    else if (pipe1)
        hipLaunchKernelGGL((knn_pipe<1, 4, false>), grid, dim3(256), 0, s, p);
    else if (qt1)
        hipLaunchKernelGGL((knn_mfma_pk<128, false, 1, 4>), grid, dim3(256), 0, s, p);
    else if (kb == 128 && mode == MODE_L2P && knn_pipe_enabled())
        hipLaunchKernelGGL((knn_pipe<KNN_QT, KNN_PIPE_MINB, false>), grid, dim3(256), 0, s, p);
    else if (kb == kOrbExpBytes && mode == MODE_HAMP && knn_pipe_enabled())
        hipLaunchKernelGGL((knn_pipe<2, KNN_PIPE_MINB, true>), grid, dim3(256), 0, s, p);
    else if (kb == 128 && mode == MODE_L2P)
        hipLaunchKernelGGL((knn_mfma_pk<128, false, KNN_QT, KNN_MINB, KNN_NTH>), grid, dim3(KNN_NTH), 0, s, p);
    else if (kb == kOrbExpBytes && mode == MODE_HAMP) hipLaunchKernelGGL((knn_mfma_pk<kOrbExpBytes, true, 2, 4>), grid, dim3(256), 0, s, p);
    else if (kb == 128 && mode == MODE_L1P)
        hipLaunchKernelGGL((knn_l1<2>), dim3((nq + 511) / 512, nframes, tsplit), dim3(256), 0, s, p);
    else { prof_end(c, 2, s); return hipErrorInvalidValue; }
    prof_end(c, 2, s);
    return hipGetLastError();
}

hipError_t launch_knn_finish(slam_ctx* c, hipStream_t s, const int4* part, int nq, int nframes, int tsplit,
                             const int32_t* qnorm, int mode, double ratio, const int32_t* t_info, int2* top_idx,
                             float2* top_dist, slam_dmatch* rec, uint8_t* flag, int32_t* counts)
{
    if (nq <= 0 || nframes <= 0) return hipSuccess;
    FinishParams p;
    p.part = part; p.nq = nq; p.nframes = nframes; p.tsplit = tsplit; p.mode = mode; p.qnorm = qnorm;
    p.ratio = ratio; p.t_info = (const int4*)t_info; p.top_idx = top_idx; p.top_dist = top_dist;
    p.rec = rec; p.flag = flag; p.counts = counts;
    prof_begin(c, 5, s);
    hipLaunchKernelGGL(knn_finish, dim3((nq + 255) / 256, nframes), dim3(256), 0, s, p);
    prof_end(c, 5, s);
    return hipGetLastError();
}

hipError_t launch_compact(slam_ctx* c, hipStream_t s, const slam_dmatch* rec, const uint8_t* flag, int nq,
                          int nframes, slam_dmatch* out, int32_t* out_counts, int stride)
{
    (void)c;
    if (nq <= 0 || nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(knn_compact, dim3(nframes), dim3(1024), 0, s, rec, flag, nq, out, out_counts, stride);
    return hipGetLastError();
}

}  // namespace slamhip
