/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED against
 * OpenCV itself (not in this image); cross-checked against numpy's LAPACK SVD
 * and noise-free synthetic scenes in tests/test_oracle.py.
 *
 * Two-view linear triangulation, the reference's reconstruct()
 * (src/mainModule/triangulation/triangulate.cpp:74-100 and
 * reconstructPointsFor3D :17-55): P_v = K [R_v | t_v] (cv::Mat products, sums
 * in k order), per point the 4 x 4 system A (rows x P_v(2) - P_v(0),
 * y P_v(2) - P_v(1)), cv::SVD::compute(A, W, U, Vt) -- OpenCV 4.8
 * core/src/lapack.cpp JacobiSVDImpl_<double> on A' with eps = 10 DBL_EPSILON,
 * descending sort -- and the homogeneous solution Vt(3, :) scaled by 1 / w
 * (convertHomogeneousPointsMatrixToSpatialPointsVector :102-119, Mat /= w is
 * convertTo with scale 1 / w).
 *
 * Conventions shared with the GPU kernel (csrc/geom.hip), so the two agree bit
 * for bit: no contraction; hypot(x, y) restated as max * sqrt(1 + (min/max)^2)
 * (std::hypot is not specified to the last ulp).
 */
#include "oracle.h"

#include <float.h>
#include <math.h>

double orc_hypot(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { double t = a; a = b; b = t; }
    if (a == 0.0) return 0.0;
    const double r = b / a;
    return a * sqrt(1.0 + r * r);
}

/* JacobiSVDImpl_(At, W, Vt, m = n = 4): rows of At are the columns of A */
static void jacobi_svd4(double At[4][4], double W[4], double Vt[4][4])
{
    const int n = 4, m = 4, max_iter = 30;
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i][k] * At[i][k];
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i][k] = 0;
        Vt[i][i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += At[i][k] * At[j][k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = orc_hypot(p, beta);
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
                    const double t0 = c * At[i][k] + s * At[j][k];
                    const double t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = t0;
                    At[j][k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vt[i][k] + s * Vt[j][k];
                    const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                    Vt[i][k] = t0;
                    Vt[j][k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < m; k++) { t = At[i][k]; At[i][k] = At[j][k]; At[j][k] = t; }
            for (int k = 0; k < n; k++) { t = Vt[i][k]; Vt[i][k] = Vt[j][k]; Vt[j][k] = t; }
        }
    }
}

/* projection = calibration * hconcat(R, t) */
void orc_projection(const double K[9], const double R[9], const double t[3], double P[12])
{
    double Rt[12];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Rt[r * 4 + c] = R[r * 3 + c];
        Rt[r * 4 + 3] = t[r];
    }
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += K[r * 3 + k] * Rt[k * 4 + c];
            P[r * 4 + c] = s;
        }
}

/* one point of reconstructPointsFor3D: homogeneous X (4) */
void orc_triangulate_point(const double P1[12], const double P2[12], double x1, double y1, double x2, double y2,
                           double X[4])
{
    const double* P[2] = {P1, P2};
    const double xs[2] = {x1, x2}, ys[2] = {y1, y2};
    double A[4][4], At[4][4], W[4], Vt[4][4];
    for (int v = 0; v < 2; v++)
        for (int c = 0; c < 4; c++) {
            A[v * 2][c] = xs[v] * P[v][8 + c] - P[v][c];
            A[v * 2 + 1][c] = ys[v] * P[v][8 + c] - P[v][4 + c];
        }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) At[c][r] = A[r][c];
    jacobi_svd4(At, W, Vt);
    for (int k = 0; k < 4; k++) X[k] = Vt[3][k];
}

/* reconstruct(K, R1, t1, R2, t2, points1, points2, spatialPoints) */
void orc_reconstruct(const double K[9], const double R1[9], const double t1[3], const double R2[9],
                     const double t2[3], const float* pts1, const float* pts2, int n, double* out)
{
    double P1[12], P2[12];
    orc_projection(K, R1, t1, P1);
    orc_projection(K, R2, t2, P2);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < n; p++) {
        double X[4];
        orc_triangulate_point(P1, P2, (double)pts1[2 * p], (double)pts1[2 * p + 1], (double)pts2[2 * p],
                              (double)pts2[2 * p + 1], X);
        const double inv = 1. / X[3];
        out[3 * p] = X[0] * inv;
        out[3 * p + 1] = X[1] * inv;
        out[3 * p + 2] = X[2] * inv;
    }
}
