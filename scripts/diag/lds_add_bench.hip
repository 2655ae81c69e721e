// LDS scatter-add microbenchmark (gfx950): the sift_desc_band slot update.
// Per step every lane adds two packed f32 pairs into lane-private slots at a
// data-dependent position (the orientation bin): (a) read-add-write with
// ds_read_b64 / ds_write_b64 (the band kernel's form), (b) four non-returning
// ds_add_f32.  Also checks that ds_add_f32 rounds as the VALU add (RNE, no
// denormal flush) on random data.  Timing only; not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

constexpr int kWaves = 8, kPosF = 384, kPos = 10, kSteps = 4096;

__device__ __forceinline__ uint32_t hsh(uint32_t x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; return x ^ (x >> 16); }

template <int kMode>
__global__ __launch_bounds__(64 * kWaves) void bench(float* out, uint32_t seed)
{
    __shared__ __attribute__((aligned(16))) float s[kWaves][kPos * kPosF];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* buf = s[wave];
    for (int q = lane; q < kPos * kPosF; q += 64) buf[q] = 0.f;
    __builtin_amdgcn_wave_barrier();
    uint32_t st = hsh(seed + blockIdx.x * 1024 + threadIdx.x);
    char* lb = reinterpret_cast<char*>(buf + 2 * (lane & 31) + (lane >> 5) * 64);
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v lo = {1.f, 2.f}, hi = {3.f, 4.f};
#pragma unroll 16
    for (int it = 0; it < kSteps; it++) {
        st = st * 1664525u + 1013904223u;
        const int o0 = (st >> 28) & 7;                      // data-dependent position 0..7
        char* tp = lb + o0 * (kPosF * 4) + ((it & 3) * 128 * 4 % (kPosF * 4));
        if constexpr (kMode >= 10) {
            // kMode - 10 independent chains (disjoint columns), reads of every chain
            // issued before the writes: the pipelining a diagonal walk would allow
            constexpr int C = kMode >= 10 ? kMode - 10 : 1;
            f2v a[C], b[C];
#pragma unroll
            for (int c = 0; c < C; c++) {
                const int o = ((st >> (4 * c)) & 7);
                auto t = (__attribute__((address_space(3))) volatile f2v*)(lb + o * (kPosF * 4) + c * 64 * 4);
                a[c] = t[0];
                b[c] = t[kPosF / 2];
            }
#pragma unroll
            for (int c = 0; c < C; c++) {
                const int o = ((st >> (4 * c)) & 7);
                auto t = (__attribute__((address_space(3))) volatile f2v*)(lb + o * (kPosF * 4) + c * 64 * 4);
                t[0] = a[c] + lo;
                t[kPosF / 2] = b[c] + hi;
            }
        } else if constexpr (kMode == 0) {
            auto t = (__attribute__((address_space(3))) volatile f2v*)(tp);
            f2v a = t[0];
            f2v b = t[kPosF / 2];
            a = a + lo;
            b = b + hi;
            t[0] = a;
            t[kPosF / 2] = b;
        } else {
            float* t = reinterpret_cast<float*>(tp);
            __hip_atomic_fetch_add(t, lo.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(t + 1, lo.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(t + kPosF, hi.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(t + kPosF + 1, hi.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __builtin_amdgcn_wave_barrier();
    float acc = 0.f;
    for (int q = lane; q < kPos * kPosF; q += 64) acc += buf[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// rounding check: lane-private running sums of random f32 values (incl. tiny
// and denormal ones) by ds_add_f32 vs by v_add_f32
__global__ void rounding(const float* vals, int n, uint32_t* mism)
{
    __shared__ float s[64];
    const int lane = threadIdx.x;
    s[lane] = 0.f;
    float r = 0.f;
    __syncthreads();
    for (int i = 0; i < n; i++) {
        const float v = vals[i * 64 + lane];
        __hip_atomic_fetch_add(&s[lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        r = __fadd_rn(r, v);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        const float a = s[lane];
        if (__float_as_uint(a) != __float_as_uint(r)) atomicAdd(mism, 1u);
        __syncthreads();
    }
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 4 * 64 * kWaves * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int modes[] = {0, 1, 12, 13, 14};
    for (int mode : modes) {
        for (int rep = 0; rep < 3; rep++) {
            const int grid = cus * 1;   // one 8-wave workgroup per CU (2 waves / SIMD), as the band kernel
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(grid), dim3(64 * kWaves), 0, 0, out, 7u + rep);
            else if (mode == 1) hipLaunchKernelGGL(bench<1>, dim3(grid), dim3(64 * kWaves), 0, 0, out, 7u + rep);
            else if (mode == 12) hipLaunchKernelGGL(bench<12>, dim3(grid), dim3(64 * kWaves), 0, 0, out, 7u + rep);
            else if (mode == 13) hipLaunchKernelGGL(bench<13>, dim3(grid), dim3(64 * kWaves), 0, 0, out, 7u + rep);
            else hipLaunchKernelGGL(bench<14>, dim3(grid), dim3(64 * kWaves), 0, 0, out, 7u + rep);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // per CU; a chained mode does C read-add-write pairs per step: report per pair-set
            const double wave_steps = (double)kWaves * kSteps * (mode >= 10 ? mode - 10 : 1);
            printf("%s%d rep %d: %.3f ms, %.2f ns per wave-step per CU (%.2f cyc @2.4GHz)\n",
                   mode == 1 ? "ds_add_f32 x4, mode " : "read-add-write b64 x2, mode ", mode, rep, ms,
                   ms * 1e6 / wave_steps, ms * 1e6 / wave_steps * 2.4);
        }
    }
    // rounding
    const int n = 4096;
    std::vector<float> v((size_t)n * 64);
    uint32_t x = 12345;
    for (auto& f : v) {
        x = x * 1664525u + 1013904223u;
        uint32_t bits = x;
        const int cls = (x >> 29);
        if (cls == 0) bits &= 0x807fffffu;                                   // denormal
        else if (cls == 1) bits = (bits & 0x80ffffffu) | (100u << 23);       // tiny normal
        else bits = (bits & 0x807fffffu) | ((120u + (x >> 24) % 16) << 23);  // ~1e-3 .. 30
        memcpy(&f, &bits, 4);
    }
    float* dv;
    uint32_t* dm;
    hipMalloc(&dv, v.size() * 4);
    hipMalloc(&dm, 4);
    hipMemcpy(dv, v.data(), v.size() * 4, hipMemcpyHostToDevice);
    hipMemset(dm, 0, 4);
    hipLaunchKernelGGL(rounding, dim3(1), dim3(64), 0, 0, dv, n, dm);
    uint32_t mism = 0;
    hipMemcpy(&mism, dm, 4, hipMemcpyDeviceToHost);
    printf("ds_add_f32 vs v_add_f32 running sums: %u mismatches of %d\n", mism, n * 64);
    return 0;
}
