// Microbenchmark: element-distributed register Cholesky variants (ba_camera_solve
// design space) on an SPD matrix in global memory.  MODE bits: 1 = reciprocal
// published with the pivot (no division on the critical path), 2 = single wave
// (wave barrier instead of s_barrier).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int kMaxNc = 136;
template <int NT, int EPT, int MODE>
__global__ __launch_bounds__(NT) void solve(const double* S, const double* rhs, int n, double* out, long long* cyc)
{
    __shared__ double col[2][kMaxNc + 2];
    __shared__ double zb[kMaxNc], dg[kMaxNc], xs[kMaxNc];
    const int tid = threadIdx.x, ne = n * (n + 1) / 2;
    long long t0 = clock64();
    double a[EPT];
    int rik[EPT];
#pragma unroll
    for (int u = 0; u < EPT; u++) {
        const int e = tid + NT * u;
        int i = -1, k = -1;
        double v = 0;
        if (e < ne) {
            i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while ((i + 1) * (i + 2) / 2 <= e) i++;
            while (i * (i + 1) / 2 > e) i--;
            k = e - i * (i + 1) / 2;
            v = S[i * n + k];
        }
        a[u] = v;
        rik[u] = e < ne ? (i << 16) | k : -1;
    }
#define RI(u) (rik[u] >> 16)
#define RK(u) (rik[u] < 0 ? -1 : (rik[u] & 0xffff))
    for (int i = tid; i < n; i += NT) zb[i] = rhs[i];
#pragma unroll
    for (int u = 0; u < EPT; u++)
        if (RK(u) == 0) { col[0][RI(u)] = a[u]; if (RI(u) == 0) { dg[0] = a[u]; col[0][kMaxNc] = 1.0 / a[u]; } }
    __syncthreads();
    long long t1 = clock64();
    for (int j = 0; j < n; j++) {
        const double* cj = col[j & 1];
        double* cn = col[(j + 1) & 1];
        const double inv = (MODE & 1) ? cj[kMaxNc] : 1.0 / cj[j];
        if (MODE & 4) {
            // branch-free: every LDS read of the step first, then selects
            double ci[EPT], ck[EPT];
#pragma unroll
            for (int u = 0; u < EPT; u++) { ci[u] = cj[rik[u] < 0 ? 0 : RI(u)]; ck[u] = cj[rik[u] < 0 ? 0 : RK(u)]; }
#pragma unroll
            for (int u = 0; u < EPT; u++) {
                const double upd = fma(-(ci[u] * ck[u]), inv, a[u]);
                a[u] = RK(u) > j ? upd : a[u];
            }
#pragma unroll
            for (int u = 0; u < EPT; u++)
                if (RK(u) == j + 1) { cn[RI(u)] = a[u]; if (RI(u) == j + 1) { dg[j + 1] = a[u]; if (MODE & 1) cn[kMaxNc] = 1.0 / a[u]; } }
        } else {
#pragma unroll
        for (int u = 0; u < EPT; u++) {
            if (RK(u) > j) {
                a[u] = fma(-(cj[RI(u)] * cj[RK(u)]), inv, a[u]);
                if (RK(u) == j + 1) { cn[RI(u)] = a[u]; if (RI(u) == j + 1) { dg[j + 1] = a[u]; if (MODE & 1) cn[kMaxNc] = 1.0 / a[u]; } }
            }
        }
        }
        for (int i = j + 1 + tid; i < n; i += NT) zb[i] = fma(-cj[i], zb[j] * inv, zb[i]);
        if (MODE & 2) { __builtin_amdgcn_wave_barrier(); __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
        else __syncthreads();
    }
    long long t2 = clock64();
    for (int i = n - 1; i >= 0; i--) {
        const double xi = zb[i] / dg[i];
        if (MODE & 4) {
            double zk[EPT];
#pragma unroll
            for (int u = 0; u < EPT; u++) zk[u] = zb[rik[u] < 0 ? 0 : RK(u)];
#pragma unroll
            for (int u = 0; u < EPT; u++)
                if (RI(u) == i && RK(u) < i) zb[RK(u)] = fma(-a[u], xi, zk[u]);
        } else {
#pragma unroll
        for (int u = 0; u < EPT; u++)
            if (RI(u) == i && RK(u) < i) zb[RK(u)] = fma(-a[u], xi, zb[RK(u)]);
        }
        if (tid == 0) xs[i] = xi;
        if (MODE & 2) { __builtin_amdgcn_wave_barrier(); __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
        else __syncthreads();
    }
    long long t3 = clock64();
    for (int i = tid; i < n; i += NT) out[i] = xs[i];
    if (tid == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; }
}
template <int NT, int EPT, int MODE>
int run(int n, const char* name)
{
    std::vector<double> S(n * n), b(n);
    for (int i = 0; i < n; i++) { b[i] = 1 + i; for (int k = 0; k < n; k++) S[i * n + k] = (i == k ? n + 1.0 : 1.0 / (1 + i + k)); }
    double *dS, *db, *dx; long long* dc;
    CK(hipMalloc(&dS, 8 * n * n)); CK(hipMalloc(&db, 8 * n)); CK(hipMalloc(&dx, 8 * n)); CK(hipMalloc(&dc, 64));
    CK(hipMemcpy(dS, S.data(), 8 * n * n, hipMemcpyHostToDevice)); CK(hipMemcpy(db, b.data(), 8 * n, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e9;
    long long c[3];
    double res = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < 50; it++) hipLaunchKernelGGL((solve<NT, EPT, MODE>), dim3(1), dim3(NT), 0, 0, dS, db, n, dx, dc);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms * 20 < best ? ms * 20 : best;
        CK(hipMemcpy(c, dc, 24, hipMemcpyDeviceToHost));
        std::vector<double> x(n); CK(hipMemcpy(x.data(), dx, 8 * n, hipMemcpyDeviceToHost));
        res = 0; for (int i = 0; i < n; i++) { double t = -b[i]; for (int k = 0; k < n; k++) t += S[i * n + k] * x[k]; res = fmax(res, fabs(t)); }
    }
    printf("%-22s n=%3d us=%7.2f cyc load=%6lld factor=%7lld back=%7lld resid=%.1e\n", name, n, best, c[0], c[1], c[2], res);
    return 0;
}
int main()
{
    run<256, 5, 1>(46, "256x5 inv");
    run<256, 5, 5>(46, "256x5 inv nobranch");
    run<64, 17, 7>(46, "64x17 wave nobranch");
    run<128, 9, 5>(46, "128x9 nobranch");
    run<512, 10, 1>(94, "512x10 inv");
    run<512, 10, 5>(94, "512x10 nobranch");
    run<256, 18, 5>(94, "256x18 nobranch");
    run<1024, 5, 5>(94, "1024x5 nobranch");
}
