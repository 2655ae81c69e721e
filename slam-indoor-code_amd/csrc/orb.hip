// ORB (rBRIEF) descriptors on provided FAST keypoints, gfx950.
//
// Replaces extractDescriptor's cv::ORB::create()->compute(frame, kps, desc)
// (reference featureMatchingCPU.cpp:59-65 / featureMatchingCUDA.cpp:63-68):
// runByImageBorder(31) (done by fast_detect's border filter in the batch path,
// by the host API otherwise), GaussianBlur(7x7, sigma 2) on the gray level-0
// image, then the 256 rotated bit_pattern_31_ tests.
//
//   orb_blur           sepFilter2D with f32 kernels, both passes in one LDS
//                      tile: RowVec_8u32f fma chain, SymmColumnVec_32f8u
//                      symmetric fma + round-half-even + saturate ->
//                      bit-identical to the oracle.
//   orb_desc           one wave per keypoint, lane l evaluates tests l, l+64,
//                      l+128, l+192; __ballot packs 64 tests into one u64, i.e.
//                      8 descriptor bytes, little-endian; the same wave also
//                      writes the matcher's FP4 +-1 expansion (128 B).
//   orb_expand         the FP4 +-1 expansion of host-supplied descriptors for
//                      the MFMA Hamming matcher: popcount(a ^ b) = (256 - <a', b'>) / 2.
#include "orb_pattern.h"
#include "slamhip_internal.h"

namespace slamhip {

namespace {

__constant__ int c_pat[256 * 4];

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

struct BlurParams {
    const uint8_t* gray;
    float* tmp;
    uint8_t* out;
    int w, h;
    OrbConsts k;
};

// Fused 7x7 blur, one 256-thread workgroup per 64 x 64 output tile: the gray
// tile with a 3-row / 4-column REFLECT_101 halo goes to LDS (dwords for
// interior tiles), the row pass (RowVec_8u32f: fma chain from 0 over the 7
// taps) and the column pass (SymmColumnVec_32f8u: k3 * S0, then
// fma(k[3 + m], S[m] + S[-m]), round half even, saturate) run out of LDS, and
// only the u8 result is written.  The same operations in the same order as
// the oracle's sepFilter2D restatement, so the output is bit-identical; the
// f32 intermediate plane never leaves the CU.
constexpr int kOT = 64;                  // output tile (square)
constexpr int kOR = kOT + 6;             // 70 gray / row-pass rows (y0 - 3 .. y0 + 66)
constexpr int kOC = kOT + 16;            // 80 gray columns (x0 - 8 .. x0 + 71): 16-byte rows
constexpr int kORS = kOT + 1;            // row-pass row stride (floats; odd: conflict-free column reads)

__global__ __launch_bounds__(256) void orb_blur(BlurParams p)
{
    // the u8 output tile reuses the gray tile's LDS (dead after the row pass)
    __shared__ __attribute__((aligned(16))) uint8_t go[kOR * kOC];
    __shared__ float t[kOR * kORS];
    uint8_t* const g = go;
    uint8_t* const o = go;
    static_assert(kOT * kOT <= kOR * kOC, "output tile inside the gray tile's memory");
    const int x0 = blockIdx.x * kOT, y0 = blockIdx.y * kOT, f = blockIdx.z;
    const int tid = threadIdx.x;
    const uint8_t* src = p.gray + (size_t)f * p.w * p.h;
    const bool wide = (p.w & 3) == 0 && x0 - 8 >= 0 && x0 + kOT + 8 <= p.w && y0 - 3 >= 0 && y0 + kOT + 3 <= p.h;
    if (wide) {
        // 16 bytes per lane (4-byte aligned global loads, 16-byte LDS rows); both
        // passes' loads issued before the first store, loads and stores
        // unconditional (a past-the-end index redoes the last piece)
        constexpr int NP = kOR * (kOC / 16), NIT = (NP + 255) / 256;
        uint4 v[NIT];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = min(tid + 256 * it, NP - 1);
            const int r = i / (kOC / 16), q = i - r * (kOC / 16);
            v[it] = *reinterpret_cast<const uint4*>(src + (size_t)(y0 - 3 + r) * p.w + (x0 - 8 + 16 * q));
        }
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int i = min(tid + 256 * it, NP - 1);
            const int r = i / (kOC / 16), q = i - r * (kOC / 16);
            *reinterpret_cast<uint4*>(&g[r * kOC + 16 * q]) = v[it];
        }
    } else {
        for (int i = tid; i < kOR * kOC; i += 256) {
            const int r = i / kOC, c = i - r * kOC;
            g[i] = src[(size_t)reflect101(y0 - 3 + r, p.h) * p.w + reflect101(x0 - 8 + c, p.w)];
        }
    }
    __syncthreads();
    float kk[7];
#pragma unroll
    for (int q = 0; q < 7; q++) kk[q] = p.k.gauss[q];
    // row pass: 4 adjacent outputs per task; output column c (x0 + c) reads g
    // columns c + 5 .. c + 11 (x0 + c - 3 .. x0 + c + 3)
    for (int i = tid; i < kOR * (kOT / 4); i += 256) {
        const int r = i / (kOT / 4), c = 4 * (i - r * (kOT / 4));
        const uint32_t* gw = reinterpret_cast<const uint32_t*>(&g[r * kOC + c + 4]);
        const uint32_t w0 = gw[0], w1 = gw[1], w2 = gw[2];
        float px[12];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            px[q] = (float)((w0 >> (8 * q)) & 255u);
            px[4 + q] = (float)((w1 >> (8 * q)) & 255u);
            px[8 + q] = (float)((w2 >> (8 * q)) & 255u);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < 7; q++) acc = __fmaf_rn(px[1 + u + q], kk[q], acc);
            t[r * kORS + c + u] = acc;
        }
    }
    __syncthreads();
    // column pass: one column per thread, a 16-row strip (4 strips x 64 columns)
    {
        const int c = tid & 63, r0 = 16 * (tid >> 6);
        float win[16 + 6];
#pragma unroll
        for (int q = 0; q < 22; q++) win[q] = t[(r0 + q) * kORS + c];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            float acc = __fmul_rn(kk[3], win[u + 3]);
#pragma unroll
            for (int m = 1; m <= 3; m++) acc = __fmaf_rn(kk[3 + m], __fadd_rn(win[u + 3 + m], win[u + 3 - m]), acc);
            float v = rintf(acc);
            v = fminf(fmaxf(v, 0.f), 255.f);
            o[(r0 + u) * kOT + c] = (uint8_t)v;
        }
    }
    __syncthreads();
    uint8_t* dst = p.out + (size_t)f * p.w * p.h;
    if ((p.w & 15) == 0 && x0 + kOT <= p.w && y0 + kOT <= p.h) {
        // 16 bytes per thread: rows of 4 x 16-byte segments
        const int r = tid >> 2, q = tid & 3;
        *reinterpret_cast<uint4*>(dst + (size_t)(y0 + r) * p.w + x0 + 16 * q) =
            *reinterpret_cast<const uint4*>(&o[r * kOT + 16 * q]);
    } else {
        for (int i = tid; i < kOT * kOT; i += 256) {
            const int r = i >> 6, c = i & 63;
            if (x0 + c < p.w && y0 + r < p.h) dst[(size_t)(y0 + r) * p.w + x0 + c] = o[i];
        }
    }
}

struct DescParams {
    const uint8_t* img;
    int w, h;
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float* kp_ab;   // optional per-keypoint {cos, sin} of the angle (radians); else uniform
    float a_u, b_u;
    uint8_t* desc;
    uint32_t* desc_exp;   // the FP4 +-1 expansion (kOrbExpBytes per keypoint), written beside desc
};

// +-1 expansion of one descriptor byte for the FP4 MFMA matcher: nibble k (low
// nibble first) = bit k ? +1.0 (e2m1 0x2) : -1.0 (0xA)
__device__ __forceinline__ uint32_t expand_byte(uint32_t byte)
{
    uint32_t x = byte & 0xffu;                 // bit k -> bit 4 k
    x = (x | (x << 12)) & 0x000f000fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return 0xaaaaaaaau ^ (x << 3);             // 0xA ^ 0x8 = 0x2 where the bit is set
}

// One wave per keypoint.  The wave first copies the keypoint's 39 x 39 patch of
// the blurred image (pattern coordinates are within [-13, 12], so a rotation by
// any angle stays within 19 pixels of the center) into its LDS slice, coalesced,
// then the 256 tests read LDS instead of gathering bytes from scattered global
// lines.  For the uniform angle of FAST keypoints the rotated test offsets are
// the same for every keypoint and are computed once per wave.
constexpr int kOrbR = 19, kOrbPR = 2 * kOrbR + 1;    // patch rows / columns
constexpr int kOrbPD = 11;                           // dwords per patch row (39 bytes + 3 of alignment)

__global__ __launch_bounds__(256) void orb_desc(DescParams p)
{
    __shared__ uint32_t patch_mem[4][kOrbPR * kOrbPD];
    const int lane = threadIdx.x & 63;
    uint32_t* patch = patch_mem[threadIdx.x >> 6];
    const uint8_t* pb = reinterpret_cast<const uint8_t*>(patch);
    int total = *p.total;
    if (total > p.cap) total = p.cap;
    const int waves = gridDim.x * 4;
    const bool uni = p.kp_ab == nullptr;
    // rotated test points as patch offsets (dy * row + dx) for the uniform angle
    auto rot = [&](int t, float a, float b, int& o0, int& o1) __attribute__((always_inline)) {
        const int* pt = c_pat + 4 * t;
        const float x0 = __fsub_rn(__fmul_rn((float)pt[0], a), __fmul_rn((float)pt[1], b));
        const float y0 = __fadd_rn(__fmul_rn((float)pt[0], b), __fmul_rn((float)pt[1], a));
        const float x1 = __fsub_rn(__fmul_rn((float)pt[2], a), __fmul_rn((float)pt[3], b));
        const float y1 = __fadd_rn(__fmul_rn((float)pt[2], b), __fmul_rn((float)pt[3], a));
        o0 = __float2int_rn(y0) * (4 * kOrbPD) + __float2int_rn(x0);
        o1 = __float2int_rn(y1) * (4 * kOrbPD) + __float2int_rn(x1);
    };
    int u0[4], u1[4];
#pragma unroll
    for (int q = 0; q < 4; q++) rot(q * 64 + lane, p.a_u, p.b_u, u0[q], u1[q]);
    const bool aligned = (p.w & 3) == 0;
    for (int g = blockIdx.x * 4 + (threadIdx.x >> 6); g < total; g += waves) {
        const slam_keypoint kp = p.kps[g];
        const int f = p.kp_frame[g];
        const int cy = __float2int_rn(kp.y), cx = __float2int_rn(kp.x);
        // patch rows cy - 19 .. cy + 19, dwords from column (cx - 19) & ~3
        const int xb = (cx - kOrbR) & ~3;
        const uint8_t* img = p.img + (size_t)f * p.w * p.h;
        if (aligned) {
            const uint32_t* rows = reinterpret_cast<const uint32_t*>(img + (size_t)(cy - kOrbR) * p.w + xb);
            const int wd = p.w >> 2;
            // the patch's 429 dwords: every load of the lane issued before the
            // first store (a load / wait / store loop pays a memory latency per
            // 64 dwords); loads and stores unconditional, a past-the-end index
            // redoing the last dword
            constexpr int NP = kOrbPR * kOrbPD, NIT = (NP + 63) / 64;
            uint32_t v[NIT];
#pragma unroll
            for (int it = 0; it < NIT; it++) {
                const int i = min(lane + 64 * it, NP - 1);
                const int r = i / kOrbPD, k = i - r * kOrbPD;
                v[it] = rows[r * wd + k];
            }
#pragma unroll
            for (int it = 0; it < NIT; it++) patch[min(lane + 64 * it, NP - 1)] = v[it];
        } else {
            for (int i = lane; i < kOrbPR * kOrbPD; i += 64) {
                const int r = i / kOrbPD, k = i - r * kOrbPD;
                const uint8_t* src = img + (size_t)(cy - kOrbR + r) * p.w + xb + 4 * k;
                const int lim = p.w - (xb + 4 * k);      // bytes of the row left at this dword
                uint32_t v = 0;
                for (int j = 0; j < 4 && j < lim; j++) v |= (uint32_t)src[j] << (8 * j);
                patch[i] = v;
            }
        }
        // center byte of the patch
        const int c0 = kOrbR * (4 * kOrbPD) + (cx - xb);
        uint32_t* out = reinterpret_cast<uint32_t*>(p.desc + (size_t)g * 32);
        float a = 0.f, b = 0.f;
        if (!uni) { a = p.kp_ab[2 * g]; b = p.kp_ab[2 * g + 1]; }
        uint64_t m[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int o0 = u0[q], o1 = u1[q];
            if (!uni) rot(q * 64 + lane, a, b, o0, o1);
            const int t0 = pb[c0 + o0], t1 = pb[c0 + o1];
            m[q] = __ballot(t0 < t1);
        }
        // one store instruction for both outputs: lanes 32..39 write the 32
        // descriptor bytes as dwords, lane j < 32 the matcher's FP4 expansion of
        // descriptor byte j (orb_expand's format), one coalesced 128-byte row.  Each
        // lane picks its dword of the (wave-uniform) ballot masks by a 3-level select
        if (lane < 40) {
            const int idx = lane < 32 ? (lane >> 2) : (lane - 32);
            const uint32_t t0 = (idx & 1) ? (uint32_t)(m[0] >> 32) : (uint32_t)m[0];
            const uint32_t t1 = (idx & 1) ? (uint32_t)(m[1] >> 32) : (uint32_t)m[1];
            const uint32_t t2 = (idx & 1) ? (uint32_t)(m[2] >> 32) : (uint32_t)m[2];
            const uint32_t t3 = (idx & 1) ? (uint32_t)(m[3] >> 32) : (uint32_t)m[3];
            const uint32_t s0 = (idx & 2) ? t1 : t0, s1 = (idx & 2) ? t3 : t2;
            const uint32_t w32 = (idx & 4) ? s1 : s0;
            uint32_t* dst;
            uint32_t v;
            if (lane < 32) {
                dst = p.desc_exp + (size_t)g * (kOrbExpBytes / 4) + lane;
                v = expand_byte(w32 >> (8 * (lane & 3)));
            } else {
                dst = out + (lane - 32);
                v = w32;
            }
            *dst = v;
        }
    }
}

// +-1 expansion for the FP4 MFMA matcher: nibble k of the output (low nibble
// first) = bit k of the descriptor ? +1.0 (e2m1 0x2) : -1.0 (0xA); one output
// dword per descriptor byte
__global__ __launch_bounds__(256) void orb_expand(const uint8_t* d, int n, int8_t* out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;   // one output dword = one descriptor byte
    if (i >= (size_t)n * 32) return;
    reinterpret_cast<uint32_t*>(out)[i] = expand_byte(d[i]);
}

// sum over k of (d_k - 128)^2 for host-supplied u8 SIFT descriptors (one wave per row)
__global__ __launch_bounds__(256) void norms_u8(const uint8_t* d, int n, int32_t* norms)
{
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= n) return;
    int a = (int)d[(size_t)row * 128 + lane] - 128, b = (int)d[(size_t)row * 128 + lane + 64] - 128;
    int s = a * a + b * b;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) norms[row] = s;
}

bool g_pat_loaded = false;

}  // namespace

hipError_t launch_orb_blur(slam_ctx* c, hipStream_t s, int nframes, int w, int h)
{
    hipError_t e;
    const size_t px = (size_t)nframes * w * h;
    if ((e = c->orbblur.ensure(px)) != hipSuccess) return e;
    BlurParams b;
    b.gray = c->gray.as<uint8_t>(); b.tmp = nullptr; b.out = c->orbblur.as<uint8_t>();
    b.w = w; b.h = h; b.k = c->orb;
    dim3 grid((w + kOT - 1) / kOT, (h + kOT - 1) / kOT, nframes);
    prof_begin(c, 4, s);
    hipLaunchKernelGGL(orb_blur, grid, dim3(256), 0, s, b);
    prof_end(c, 4, s);
    return hipGetLastError();
}

hipError_t launch_orb_desc(slam_ctx* c, hipStream_t s, int nframes, int w, int h, const float* d_kp_ab, int cap)
{
    (void)nframes;
    hipError_t e;
    if (!g_pat_loaded) {
        if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_pat), slam_orb_pattern31, sizeof(slam_orb_pattern31))) != hipSuccess)
            return e;
        g_pat_loaded = true;
    }
    if ((e = c->desc_u8.ensure((size_t)cap * 32)) != hipSuccess) return e;
    if ((e = c->desc_exp.ensure((size_t)cap * kOrbExpBytes)) != hipSuccess) return e;
    DescParams p;
    p.img = c->orbblur.as<uint8_t>(); p.w = w; p.h = h;
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap; p.kp_ab = d_kp_ab;
    const float ang = -1.f * (float)(M_PI / 180.f);
    p.a_u = cosf(ang);
    p.b_u = sinf(ang);
    p.desc = c->desc_u8.as<uint8_t>();
    p.desc_exp = c->desc_exp.as<uint32_t>();
    int grid = (cap + 3) / 4;
    if (grid > 16384) grid = 16384;
    if (grid < 1) grid = 1;
    prof_begin(c, 3, s);
    hipLaunchKernelGGL(orb_desc, dim3(grid), dim3(256), 0, s, p);
    prof_end(c, 3, s);
    return hipGetLastError();
}

hipError_t launch_orb_expand(hipStream_t s, const uint8_t* d, int n, int8_t* out)
{
    if (n <= 0) return hipSuccess;
    const size_t dw = (size_t)n * 32;
    hipLaunchKernelGGL(orb_expand, dim3((unsigned)((dw + 255) / 256)), dim3(256), 0, s, d, n, out);
    return hipGetLastError();
}

hipError_t launch_norms_u8(hipStream_t s, const uint8_t* d, int n, int32_t* norms)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(norms_u8, dim3((n + 3) / 4), dim3(256), 0, s, d, n, norms);
    return hipGetLastError();
}

}  // namespace slamhip
