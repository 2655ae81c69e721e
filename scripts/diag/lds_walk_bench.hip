// SIFT band walk microbenchmark (gfx950): the per-sample work of the band
// kernel's walk -- a staged {mw, ob} read, the bin values, the slot address and
// the read-add-write of lane-private slots at a data-dependent orientation
// position -- in two lane mappings:
//   A: two lanes per keypoint (32 per wave, one histogram column each), 8 waves
//      per CU: 2 ds_read_b64 + 2 ds_write_b64 per lane and sample (the kernel);
//   B: one lane per keypoint (64 per wave, both columns), 4 waves per CU (the
//      slots of 64 keypoints take twice the LDS): 4 + 4 per lane and sample,
//      the shared part of the value computed once.
// Reports CU-cycles per keypoint-sample.  Timing only; not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kSteps = 4096, kPos = 10;
typedef float f2v __attribute__((ext_vector_type(2)));

template <int kLanesPerKp, int kWaves, int kVar = 0>
__global__ __launch_bounds__(64 * kWaves) void walk(float* out, uint32_t seed)
{
    constexpr int kKpW = 64 / kLanesPerKp;          // keypoints per wave
    constexpr int kColF = 2 * kKpW;                 // floats per (pos, column)
    constexpr int kPosF = 6 * kColF;
    constexpr int kStage = kKpW * 36;
    constexpr int kWaveF = kPos * kPosF + kStage;
    __shared__ __attribute__((aligned(16))) float s[kWaves * kWaveF];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* buf = s + wave * kWaveF;
    float* stg = buf + kPos * kPosF;
    for (int q = lane; q < kWaveF; q += 64) buf[q] = q < kPos * kPosF ? 0.f : (float)((q * 2654435761u) >> 8) * 1e-7f;
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
    const int kq = lane % kKpW, dc = lane / kKpW;
    char* lb = reinterpret_cast<char*>(buf + 2 * kq + (kLanesPerKp == 2 ? dc * kColF : 0));
    const f2v km2 = {dc ? 1.f : 0.f, dc ? 1.f : 0.f}, kn2 = {dc ? -1.f : 1.f, dc ? -1.f : 1.f};
    float rf = 0.37f + seed * 1e-9f, cf = 0.61f;
    uint32_t tof = (seed & 1) * 4 * kColF;
#pragma unroll 8
    for (int it = 0; it < kSteps; it += 2) {
        const float4 r = *reinterpret_cast<const float4*>(stg + kq * 36 + 4 * ((it >> 1) & 7));
        // kVar 4: a third staged word per sample, the slot byte offset (b64 beside the b128)
        uint2 so = make_uint2(0, 0);
        if constexpr (kVar == 4) so = *reinterpret_cast<const uint2*>(stg + kq * 36 + 32 + 2 * ((it >> 1) & 1));
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const float mw = h ? r.y : r.x;
            const float ob = (h ? r.w : r.z) * 64.f - 9.f;    // in [-9, -1)
            const float frac = kVar == 1 ? mw : (kVar == 4 ? (h ? r.w : r.z) : __builtin_amdgcn_fractf(ob));
            int o0;
            __asm__("v_cvt_flr_i32_f32 %0, %1" : "=v"(o0) : "v"(ob));
            // kVar 1: the slot offset staged as an integer (no fract / floor / multiply)
            char* tp = kVar == 1   ? lb + tof + (__float_as_int(ob) & 0x1e00)
                       : kVar == 4 ? lb + tof + ((h ? so.y : so.x) & 0x1e00)
                                   : lb + tof + __mul24(o0 + 9, kPosF * 4);
            const float v_r1 = __fmul_rn(mw, rf);
            const f2v vr = {__fsub_rn(mw, v_r1), v_r1};
            const f2v cf2 = {cf, cf};
            const f2v c1 = vr * cf2;
            const f2v fr = {frac, frac};
            if constexpr (kLanesPerKp == 2) {
                const f2v cv = __builtin_elementwise_fma(c1, kn2, vr * km2);
                const f2v hi = cv * fr, lo = cv - hi;
                auto t = (__attribute__((address_space(3))) volatile f2v*)(tp);
                if constexpr (kVar == 2) {          // writes only
                    t[0] = lo;
                    t[kPosF / 2] = hi;
                } else if constexpr (kVar == 3) {   // reads only (summed into the next value)
                    f2v a = t[0];
                    f2v b = t[kPosF / 2];
                    rf = __fadd_rn(rf, a.x + b.y + lo.x + hi.y);
                } else {
                    f2v a = t[0];
                    f2v b = t[kPosF / 2];
                    t[0] = a + lo;
                    t[kPosF / 2] = b + hi;
                }
            } else {
                const f2v c0 = vr - c1;
                const f2v hi1 = c1 * fr, lo1 = c1 - hi1, hi0 = c0 * fr, lo0 = c0 - hi0;
                auto t = (__attribute__((address_space(3))) volatile f2v*)(tp);
                // column c0 + 1 at col', column c0 at col' + 1 (kColF floats on)
                f2v a1 = t[0];
                f2v b1 = t[kPosF / 2];
                f2v a0 = t[kColF / 2];
                f2v b0 = t[kPosF / 2 + kColF / 2];
                t[0] = a1 + lo1;
                t[kPosF / 2] = b1 + hi1;
                t[kColF / 2] = a0 + lo0;
                t[kPosF / 2 + kColF / 2] = b0 + hi0;
            }
            rf = __fadd_rn(rf, 1e-7f);
            tof ^= 4 * kColF;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
    float acc = 0.f;
    for (int q = lane; q < kPos * kPosF; q += 64) acc += buf[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int L, int W, int V = 0>
void run(const char* name, int cus, float* out)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((walk<L, W, V>), dim3(cus), dim3(64 * W), 0, 0, out, 7u + rep);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double kps = (double)W * (64 / L) * kSteps;   // keypoint-samples per CU
        printf("%s rep %d: %.3f ms, %.3f CU-cycles per keypoint-sample @2.4GHz\n", name, rep, ms,
               ms * 1e-3 * 2.4e9 / kps);
    }
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 64 * 16 * 4);
    run<2, 8>("A: 2 lanes/kp, 8 waves/CU", cus, out);
    run<1, 4>("B: 1 lane/kp, 4 waves/CU ", cus, out);
    run<1, 2>("B: 1 lane/kp, 2 waves/CU ", cus, out);
    run<2, 8, 1>("A, 3 VALU fewer (staged slot offset)", cus, out);
    run<2, 8, 2>("A, slot writes only", cus, out);
    run<2, 8, 3>("A, slot reads only", cus, out);
    run<2, 8, 4>("A, staged {mw, frac, slot offset}", cus, out);
    return 0;
}
