// Microbenchmark: blocked (B = 8) Cholesky + solves of an SPD system held in
// LDS by one 256-thread workgroup (the candidate for ba_camera_solve).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kB = 8;
template <int NT>
__device__ bool chol_blocked(double* A, double* b, int n)   // A: n x n row-major in LDS (lower used), b: n in LDS
{
    __shared__ int s_fail;
    const int tid = threadIdx.x;
    if (tid == 0) s_fail = 0;
    for (int kb = 0; kb < n; kb += kB) {
        const int nb = min(kB, n - kb);
        // (1) diagonal block: one thread, in registers; forward-solve its rhs
        if (tid == 0) {
            double L[kB][kB], y[kB];
#pragma unroll
            for (int i = 0; i < kB; i++) {
#pragma unroll
                for (int k = 0; k < kB; k++) L[i][k] = (i < nb && k <= i) ? A[(kb + i) * n + kb + k] : (i == k ? 1.0 : 0.0);
                y[i] = i < nb ? b[kb + i] : 0.0;
            }
            bool ok = true;
#pragma unroll
            for (int j = 0; j < kB; j++) {
                double s = L[j][j];
#pragma unroll
                for (int k = 0; k < j; k++) s = fma(-L[j][k], L[j][k], s);
                if (!(s > 0.0) || !isfinite(s)) ok = false;
                const double d = sqrt(s), rd = 1.0 / d;
                L[j][j] = d;
#pragma unroll
                for (int i = j + 1; i < kB; i++) {
                    double t = L[i][j];
#pragma unroll
                    for (int k = 0; k < j; k++) t = fma(-L[i][k], L[j][k], t);
                    L[i][j] = t * rd;
                }
                double t = y[j];
#pragma unroll
                for (int k = 0; k < j; k++) t = fma(-L[j][k], y[k], t);
                y[j] = t * rd;
            }
            if (!ok) s_fail = 1;
#pragma unroll
            for (int i = 0; i < kB; i++) {
                if (i < nb) {
#pragma unroll
                    for (int k = 0; k < kB; k++) if (k <= i) A[(kb + i) * n + kb + k] = L[i][k];
                    b[kb + i] = y[i];
                }
            }
        }
        __syncthreads();
        if (s_fail) return false;
        const int r0 = kb + nb, m = n - r0;
        // (2) panel: row r solves L_r. L_diag^T = A_r. (one thread per row), and its rhs
        for (int t = tid; t < m; t += NT) {
            const int r = r0 + t;
            double l[kB];
            double br = b[r];
#pragma unroll
            for (int j = 0; j < kB; j++) {
                if (j < nb) {
                    double v = A[r * n + kb + j];
#pragma unroll
                    for (int k = 0; k < j; k++) v = fma(-l[k], A[(kb + j) * n + kb + k], v);
                    l[j] = v / A[(kb + j) * n + kb + j];
                    A[r * n + kb + j] = l[j];
                    br = fma(-l[j], b[kb + j], br);
                } else l[j] = 0.0;
            }
            b[r] = br;
        }
        __syncthreads();
        // (3) trailing update of the lower triangle: a_rc -= sum_j L_rj L_cj
        const int ne = m * (m + 1) / 2;
        for (int e = tid; e < ne; e += NT) {
            int r = (int)((sqrtf(8.f * e + 1.f) - 1.f) * 0.5f);
            while ((r + 1) * (r + 2) / 2 <= e) r++;
            while (r * (r + 1) / 2 > e) r--;
            const int c = e - r * (r + 1) / 2;
            const double* Lr = A + (r0 + r) * n + kb;
            const double* Lc = A + (r0 + c) * n + kb;
            double v = A[(r0 + r) * n + r0 + c];
#pragma unroll
            for (int j = 0; j < kB; j++) if (j < nb) v = fma(-Lr[j], Lc[j], v);
            A[(r0 + r) * n + r0 + c] = v;
        }
        __syncthreads();
    }
    // back solve L^T x = y, blocks from the bottom
    for (int kb = ((n - 1) / kB) * kB; kb >= 0; kb -= kB) {
        const int nb = min(kB, n - kb);
        if (tid == 0) {
            double x[kB];
#pragma unroll
            for (int i = kB - 1; i >= 0; i--) {
                if (i < nb) {
                    double t = b[kb + i];
#pragma unroll
                    for (int k = i + 1; k < kB; k++) if (k < nb) t = fma(-A[(kb + k) * n + kb + i], x[k], t);
                    x[i] = t / A[(kb + i) * n + kb + i];
                    b[kb + i] = x[i];
                } else x[i] = 0.0;
            }
        }
        __syncthreads();
        // rows above: y_j -= sum_{r in block} L_rj x_r
        for (int j = tid; j < kb; j += NT) {
            double v = b[j];
#pragma unroll
            for (int k = 0; k < kB; k++) if (k < nb) v = fma(-A[(kb + k) * n + j], b[kb + k], v);
            b[j] = v;
        }
        __syncthreads();
    }
    return true;
}

template <int NT>
__global__ __launch_bounds__(NT) void solve(const double* S, const double* rhs, int n, double* out, long long* cyc)
{
    extern __shared__ double sm[];
    double* A = sm;
    double* b = sm + n * n;
    long long t0 = clock64();
    for (int e = threadIdx.x; e < n * n; e += NT) A[e] = S[e];
    for (int i = threadIdx.x; i < n; i += NT) b[i] = rhs[i];
    __syncthreads();
    long long t1 = clock64();
    chol_blocked<NT>(A, b, n);
    long long t2 = clock64();
    for (int i = threadIdx.x; i < n; i += NT) out[i] = b[i];
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = 0; }
}
template <int NT>
int run(int n, const char* name)
{
    std::vector<double> S(n * n), b(n);
    for (int i = 0; i < n; i++) { b[i] = 1 + i; for (int k = 0; k < n; k++) S[i * n + k] = (i == k ? n + 1.0 : 1.0 / (1 + i + k)); }
    double *dS, *db, *dx; long long* dc;
    CK(hipMalloc(&dS, 8 * n * n)); CK(hipMalloc(&db, 8 * n)); CK(hipMalloc(&dx, 8 * n)); CK(hipMalloc(&dc, 64));
    CK(hipMemcpy(dS, S.data(), 8 * n * n, hipMemcpyHostToDevice)); CK(hipMemcpy(db, b.data(), 8 * n, hipMemcpyHostToDevice));
    const size_t lds = 8 * (n * n + n);
    CK(hipFuncSetAttribute((const void*)solve<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e9; long long c[3]; double res = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < 50; it++) hipLaunchKernelGGL((solve<NT>), dim3(1), dim3(NT), lds, 0, dS, db, n, dx, dc);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms * 20 < best ? ms * 20 : best;
        CK(hipMemcpy(c, dc, 24, hipMemcpyDeviceToHost));
        std::vector<double> x(n); CK(hipMemcpy(x.data(), dx, 8 * n, hipMemcpyDeviceToHost));
        res = 0; for (int i = 0; i < n; i++) { double t = -b[i]; for (int k = 0; k < n; k++) t += S[i * n + k] * x[k]; res = fmax(res, fabs(t)); }
    }
    printf("%-16s n=%3d us=%7.2f cyc load=%6lld solve=%7lld resid=%.1e\n", name, n, best, c[0], c[1], res);
    return 0;
}
int main()
{
    run<256>(46, "blk8 256");
    run<256>(94, "blk8 256");
    run<512>(94, "blk8 512");
    run<256>(136, "blk8 256");
}
