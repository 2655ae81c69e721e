// Microbenchmark: one-wave rows-in-registers solve of the reduced camera
// system (ba_camera_solve_rows), loaded straight from the [S | rc] layout
// ba_s_assemble writes (lower triangle + rhs, row-major, ld = n + 1).
//   V 0: pivot row published through LDS (the kernel in ba.hip)
//   V 1: column j broadcast with v_readlane (no LDS, no barriers), t = a_ij / a_jj:
//        the same operations as V 0 (bit-identical)
//   V 2: row j broadcast, t = a_ij * (1 / a_jj), reciprocal diagonal in the back solve
//   V 3 / 4: LDS look-ahead (column j + 1 published early), division / reciprocal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <cstring>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ double rl(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NP, int V>
__global__ __launch_bounds__(64) void solve(const double* Sg, int n, double* out, long long* cyc, int* okp)
{
    __shared__ __attribute__((aligned(16))) double col[2][NP + 2];
    __shared__ double xs[NP];
    const int i = threadIdx.x, ld = n + 1;
    long long t0 = clock64();
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const int r = i > k ? i : k, c = i > k ? k : i;
        a[k] = i < n && k < n ? Sg[r * ld + c] : (i == k ? 1.0 : 0.0);
    }
    double b = i < n ? Sg[i * ld + n] : 0.0;
    bool ok = true;
    long long t1 = clock64();
    if (V == 0) {
#pragma unroll
        for (int j = 0; j < NP; j++) {
            double* cj = col[j & 1];
            if (i < NP) cj[i] = a[j];
            if (i == j) cj[NP] = b;
            __builtin_amdgcn_wave_barrier();
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const double ajj = cj[j];
            if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }
            const double bj = cj[NP];
            if (i > j) {
                const double t = a[j] / ajj;
                const double2* c2 = reinterpret_cast<const double2*>(cj);
#pragma unroll
                for (int k = (j + 1) & ~1; k < NP; k += 2) {
                    const double2 v = c2[k >> 1];
                    if (k > j) a[k] = fma(-t, v.x, a[k]);
                    a[k + 1] = fma(-t, v.y, a[k + 1]);
                }
                b = fma(-t, bj, b);
            }
        }
    } else if (V == 5) {
        // V 1 with look-ahead: the next quotient right after column j + 1's update
        double ajj = rl(a[0], 0);
        ok = ajj > 0.0 && isfinite(ajj);
        double t = i > 0 ? a[0] / ajj : 0.0;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const double bj = rl(b, j);
            double tn = 0;
            if (j + 1 < NP) {
                a[j + 1] = fma(-t, rl(a[j], j + 1), a[j + 1]);
                const double pn = rl(a[j + 1], j + 1);
                ok = ok && pn > 0.0 && isfinite(pn);
                tn = i > j + 1 ? a[j + 1] / pn : 0.0;
            }
#pragma unroll
            for (int k = j + 2; k < NP; k++) a[k] = fma(-t, rl(a[j], k), a[k]);
            b = fma(-t, bj, b);
            t = tn;
        }
    } else if (V >= 3) {
        // look-ahead: column j + 1 is updated first and published while the
        // rest of step j runs; the next pivot's quotient overlaps the FMAs
        if (i < NP) col[0][i] = a[0];
        if (i == 0) col[0][NP] = b;
        double piv = col[0][0];
        ok = piv > 0.0 && isfinite(piv);
        double t = i > 0 ? (V == 3 ? a[0] / piv : a[0] * (1.0 / piv)) : 0.0;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const double* cj = col[j & 1];
            double* cn = col[(j + 1) & 1];
            const double bj = cj[NP];
            if (j + 1 < NP) {
                a[j + 1] = fma(-t, cj[j + 1], a[j + 1]);
                b = fma(-t, bj, b);
                if (i < NP) cn[i] = a[j + 1];
                if (i == j + 1) cn[NP] = b;
                const double pn = cn[j + 1];
                ok = ok && pn > 0.0 && isfinite(pn);
                const double tn = i > j + 1 ? (V == 3 ? a[j + 1] / pn : a[j + 1] * (1.0 / pn)) : 0.0;
#pragma unroll
                for (int k = j + 2; k < NP; k++) a[k] = fma(-t, cj[k], a[k]);
                t = tn;
            } else {
                b = fma(-t, bj, b);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NP; j++) {
            const double ajj = rl(a[j], j), bj = rl(b, j);
            ok = ok && ajj > 0.0 && isfinite(ajj);
            const double t = i > j ? (V == 1 ? a[j] / ajj : a[j] * (1.0 / ajj)) : 0.0;
#pragma unroll
            for (int k = j + 1; k < NP; k++) a[k] = fma(-t, V == 1 ? rl(a[j], k) : rl(a[k], j), a[k]);
            b = fma(-t, bj, b);
        }
    }
    long long t2 = clock64();
    double x = 0;
    if (V == 0) {
        double diag = 1.0;
#pragma unroll
        for (int k = 0; k < NP; k++) if (k == i) diag = a[k];
#pragma unroll
        for (int k = NP - 1; k >= 0; k--) {
            if (i == k) xs[k] = b / diag;
            __builtin_amdgcn_wave_barrier();
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (i < k) b = fma(-a[k], xs[k], b);
        }
        x = xs[i < NP ? i : 0];
    } else {
        double diag = 1.0;
#pragma unroll
        for (int k = 0; k < NP; k++) if (k == i) diag = a[k];
        const double rd = 1.0 / diag;
#pragma unroll
        for (int k = NP - 1; k >= 0; k--) {
            const double xk = V == 1 || V == 3 || V == 5 ? rl(b, k) / rl(a[k], k) : rl(b, k) * rl(rd, k);
            if (i == k) x = xk;
            b = fma(i < k ? -a[k] : 0.0, xk, b);
        }
    }
    long long t3 = clock64();
    if (i < n) out[i] = x;
    if (i == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; okp[0] = ok; }
}

template <int NP, int V>
int run(int n, const char* name)
{
    const int ld = n + 1;
    std::vector<double> S(n * n), Sg(n * ld), b(n);
    for (int i = 0; i < n; i++) { b[i] = 1 + i; for (int k = 0; k < n; k++) S[i * n + k] = (i == k ? n + 1.0 : 1.0 / (1 + i + k)); }
    for (int i = 0; i < n; i++) { for (int k = 0; k < n; k++) Sg[i * ld + k] = S[i * n + k]; Sg[i * ld + n] = b[i]; }
    double *dS, *dx; long long* dc; int* dok;
    CK(hipMalloc(&dS, 8 * n * ld)); CK(hipMalloc(&dx, 8 * n)); CK(hipMalloc(&dc, 64)); CK(hipMalloc(&dok, 4));
    CK(hipMemcpy(dS, Sg.data(), 8 * n * ld, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e9; long long c[3]; double res = 0; int ok = 0; unsigned long long xh = 0;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < 50; it++) hipLaunchKernelGGL((solve<NP, V>), dim3(1), dim3(64), 0, 0, dS, n, dx, dc, dok);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms * 20 < best ? ms * 20 : best;
        CK(hipMemcpy(c, dc, 24, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&ok, dok, 4, hipMemcpyDeviceToHost));
        std::vector<double> x(n); CK(hipMemcpy(x.data(), dx, 8 * n, hipMemcpyDeviceToHost));
        res = 0; for (int i = 0; i < n; i++) { double t = -b[i]; for (int k = 0; k < n; k++) t += S[i * n + k] * x[k]; res = fmax(res, fabs(t)); }
        xh = 0; for (int i = 0; i < n; i++) { unsigned long long u; memcpy(&u, &x[i], 8); xh = xh * 1000003ull ^ u; }
    }
    printf("%-22s n=%3d us/launch=%7.2f cyc load=%6lld factor=%7lld back=%7lld ok=%d resid=%.1e xhash=%016llx\n", name, n, best, c[0], c[1], c[2], ok, res, xh);
    return 0;
}
int main()
{
    run<48, 0>(46, "lds rows (current)");
    run<48, 1>(46, "readlane div");
    run<48, 2>(46, "readlane rcp");
    run<48, 5>(46, "readlane div lookahead");
    run<64, 0>(58, "lds rows (current)");
    run<64, 5>(58, "readlane div lookahead");
    run<64, 1>(58, "readlane div");
}
