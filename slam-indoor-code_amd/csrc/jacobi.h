// One-sided Jacobi SVD in the order of OpenCV's JacobiSVDImpl_ (core/src/
// lapack.cpp: eps = 10 DBL_EPSILON, up to max(m, 30) sweeps, descending
// selection sort), shared by host and device code of the geometry ops
// (essential.hip, pnp.hip) so every caller matches oracle/essential.c's
// orc_jsvd bit for bit.  At (n x m) holds A's columns as rows.
#pragma once
#include <cfloat>
#include <cmath>

namespace slamhip {

#define HD __host__ __device__

HD inline double ep_hypot(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { const double t = a; a = b; b = t; }
    if (a == 0.0) return 0.0;
    const double r = b / a;
    return a * sqrt(1.0 + r * r);
}

// one-sided Jacobi SVD in JacobiSVDImpl_ order: At (n x m) rows are A's columns
template <int n, int m>
HD void jsvd(double* At, double* W, double* Vt)
{
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    const int max_iter = m > 30 ? m : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += At[i * m + k] * At[j * m + k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = ep_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const double t0 = c * At[i * m + k] + s * At[j * m + k];
                    const double t1 = -s * At[i * m + k] + c * At[j * m + k];
                    At[i * m + k] = t0;
                    At[j * m + k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vt[i * n + k] + s * Vt[j * n + k];
                    const double t1 = -s * Vt[i * n + k] + c * Vt[j * n + k];
                    Vt[i * n + k] = t0;
                    Vt[j * n + k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < m; k++) { t = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = t; }
            for (int k = 0; k < n; k++) { t = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = t; }
        }
    }
}

}  // namespace slamhip
