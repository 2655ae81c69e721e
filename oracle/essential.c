/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED against
 * OpenCV itself (not in this image); checked in tests/test_oracle.py against
 * noise-free and noisy synthetic two-view scenes (recovered R, t, inlier sets)
 * and for internal consistency (every returned E satisfies the 5 epipolar
 * constraints, det E = 0 and 2 E E'E - tr(E E') E = 0).
 *
 * estimateTransformation (src/mainModule/translation/cameraTranslation.cpp:
 * 32-69): findEssentialMat(points1, points2, K, RANSAC, prob, threshold, mask)
 * then recoverPose(E, points1, points2, K, R, t, distanceThresh, chiralityMask)
 * with an EMPTY chiralityMask (the RANSAC mask is a different variable there),
 * so the cheirality count runs over all points.
 *
 * Restated from OpenCV 4.8 calib3d (five-point.cpp findEssentialMat /
 * EMEstimatorCallback / recoverPose / decomposeEssentialMat, ptsetreg.cpp
 * RANSACPointSetRegistrator + RANSACUpdateNumIters, triangulate.cpp) and core
 * (cv::RNG, JacobiSVDImpl_):
 *   - points normalised (x - cx) / fx, (y - cy) / fy; threshold / ((fx + fy) / 2);
 *   - RANSAC: RNG((uint64)-1), getSubset of 5 distinct indices, up to 1000
 *     iterations, a model is kept iff its inlier count (Sampson error, f32,
 *     <= thr^2) exceeds max(best, 4), then niters = RANSACUpdateNumIters(prob,
 *     outlier ratio, 5, niters);
 *   - minimal solver: Nister's five-point scheme as OpenCV lays it out -- null
 *     space of the 5 x 9 epipolar system, the 10 x 20 cubic constraint matrix in
 *     OpenCV's monomial order, A[:, :10]^-1 A[:, 10:], the 3 x 13 hidden-variable
 *     matrix B from rows 4..9, its degree-10 determinant in z, real roots
 *     (|imag| <= 1e-10), (x, y) from the null vector of B(z), E normalised.
 * Where OpenCV's internals are not reproducible here the restatement chooses
 * (and the GPU kernel shares): the null space by Householder QR of Q' (OpenCV
 * completes a full SVD with random vectors), the constraint coefficients by
 * explicit polynomial products (OpenCV: generated expressions), Gauss-Jordan
 * with partial pivoting for the 10 x 10 solve, Durand-Kerner for the roots
 * (OpenCV: solvePoly), and one-sided Jacobi SVD (as geom.c) for B(z), E and
 * the triangulations.  No contraction anywhere.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- cv::RNG (multiply-with-carry) ---- */
typedef struct { uint64_t s; } cvrng;
static unsigned rng_next(cvrng* r)
{
    r->s = (uint64_t)(unsigned)r->s * 4164903690u + (unsigned)(r->s >> 32);
    return (unsigned)r->s;
}
static int rng_uniform(cvrng* r, int a, int b) { return a == b ? a : (int)(rng_next(r) % (unsigned)(b - a) + a); }

/* RANSACPointSetRegistrator::getSubset (checkSubset always true for the EM callback) */
int orc_ep_subsets(int count, int iters, int* idx /* iters x 5 */)
{
    cvrng r = {~0ull};
    for (int it = 0; it < iters; it++) {
        int* id = idx + 5 * it;
        for (int i = 0; i < 5;) {
            int v, j;
            for (;;) {
                v = id[i] = rng_uniform(&r, 0, count);
                for (j = 0; j < i; j++)
                    if (v == id[j]) break;
                if (j == i) break;
            }
            i++;
        }
    }
    return iters;
}

/* RANSACUpdateNumIters */
int orc_ransac_update_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0 ? p : 0.;
    p = p < 1 ? p : 1.;
    ep = ep > 0 ? ep : 0.;
    ep = ep < 1 ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)lrint(num / denom);
}

/* ---- small dense linear algebra (shared operation order with csrc/essential.hip) ---- */
static double ep_hypot(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { double t = a; a = b; b = t; }
    if (a == 0.0) return 0.0;
    const double r = b / a;
    return a * sqrt(1.0 + r * r);
}

/* one-sided Jacobi SVD (JacobiSVDImpl_ order) of A (m x n, m >= n, row-major
 * copy in At as n x m), Vt n x n, W n; U columns = normalised At rows */
void orc_jsvd(double* At, int n, int m, double* W, double* Vt)
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
        int changed = 0;
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
                changed = 1;
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

/* 3 x 3 SVD: U (columns), W, Vt (JacobiSVD on A', U = At rows / W) */
static void svd33(const double A[9], double U[9], double W[3], double Vt[9])
{
    double At[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = A[r * 3 + c];
    orc_jsvd(At, 3, 3, W, Vt);
    for (int i = 0; i < 3; i++) {
        const double inv = W[i] > DBL_MIN ? 1. / W[i] : 0.;
        for (int k = 0; k < 3; k++) U[k * 3 + i] = At[i * 3 + k] * inv;
    }
}

static double det33(const double* a)
{
    return a[0] * (a[4] * a[8] - a[7] * a[5]) - a[1] * (a[3] * a[8] - a[6] * a[5]) +
           a[2] * (a[3] * a[7] - a[6] * a[4]);
}

/* ---- five-point solver ---- */
/* Polynomials in (x, y, z) by degree class, terms in OpenCV's monomial order
 * (cubic rows: 0 x^3, 1 y^3, 2 x^2y, 3 xy^2, 4 x^2z, 5 x^2, 6 y^2z, 7 y^2,
 * 8 xyz, 9 xy, 10 xz^2, 11 xz, 12 x, 13 yz^2, 14 yz, 15 y, 16 z^3, 17 z^2,
 * 18 z, 19 1).  Linear: (x, y, z, 1); quadratic: (x^2, y^2, xy, xz, x, yz, y,
 * z^2, z, 1).  Products run over the terms of a then of b, in these orders. */
static const int LQ[4][4] = {   /* linear x linear -> quadratic term */
    {0, 2, 3, 4}, {2, 1, 5, 6}, {3, 5, 7, 8}, {4, 6, 8, 9}};
static const int QL[10][4] = {  /* quadratic x linear -> cubic term */
    {0, 2, 4, 5},     /* x^2 * (x, y, z, 1) -> x^3, x^2y, x^2z, x^2 */
    {3, 1, 6, 7},     /* y^2 -> xy^2, y^3, y^2z, y^2 */
    {2, 3, 8, 9},     /* xy -> x^2y, xy^2, xyz, xy */
    {4, 8, 10, 11},   /* xz -> x^2z, xyz, xz^2, xz */
    {5, 9, 11, 12},   /* x -> x^2, xy, xz, x */
    {8, 6, 13, 14},   /* yz -> xyz, y^2z, yz^2, yz */
    {9, 7, 14, 15},   /* y -> xy, y^2, yz, y */
    {10, 13, 16, 17}, /* z^2 -> xz^2, yz^2, z^3, z^2 */
    {11, 14, 17, 18}, /* z -> xz, yz, z^2, z */
    {12, 15, 18, 19}};/* 1 -> x, y, z, 1 */

static void mul_ll(const double* a, const double* b, double* q /* += */)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) q[LQ[i][j]] += a[i] * b[j];
}
static void mul_ql(const double* a, const double* b, double s, double* c /* += s * a b */)
{
    for (int i = 0; i < 10; i++)
        for (int j = 0; j < 4; j++) c[QL[i][j]] += s * (a[i] * b[j]);
}

/* coefficient matrix (10 x 20) of 2 E E'E - tr(E E') E = 0 (9 rows) and
 * det E = 0 (row 9) with E = x E0 + y E1 + z E2 + E3 (EE: 4 basis vectors) */
static void coeff_mat(const double EE[4][9], double A[10][20])
{
    double E[9][4], EEt[9][10], tr[10], t1[10], t2[10];
    for (int k = 0; k < 9; k++)
        for (int b = 0; b < 4; b++) E[k][b] = EE[b][k];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            for (int q = 0; q < 10; q++) EEt[i * 3 + j][q] = 0;
            for (int k = 0; k < 3; k++) mul_ll(E[i * 3 + k], E[j * 3 + k], EEt[i * 3 + j]);
        }
    for (int q = 0; q < 10; q++) tr[q] = EEt[0][q] + EEt[4][q] + EEt[8][q];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double* r = A[i * 3 + j];
            for (int c = 0; c < 20; c++) r[c] = 0;
            for (int k = 0; k < 3; k++) mul_ql(EEt[i * 3 + k], E[k * 3 + j], 2.0, r);
            mul_ql(tr, E[i * 3 + j], -1.0, r);
        }
    /* det: E0 (E4 E8 - E5 E7) - E1 (E3 E8 - E5 E6) + E2 (E3 E7 - E4 E6) */
    double* d = A[9];
    for (int c = 0; c < 20; c++) d[c] = 0;
    static const int cof[3][4] = {{4, 8, 5, 7}, {3, 8, 5, 6}, {3, 7, 4, 6}};
    static const double sg[3] = {1.0, -1.0, 1.0};
    for (int e = 0; e < 3; e++) {
        for (int q = 0; q < 10; q++) t1[q] = t2[q] = 0;
        mul_ll(E[cof[e][0]], E[cof[e][1]], t1);
        mul_ll(E[cof[e][2]], E[cof[e][3]], t2);
        for (int q = 0; q < 10; q++) t1[q] -= t2[q];
        mul_ql(t1, E[e], sg[e], d);
    }
}

/* A[:, :10]^-1 A[:, 10:] by Gauss-Jordan with partial pivoting; returns 0 if singular */
static int gj_solve(double A[10][20], double R[10][10])
{
    for (int col = 0; col < 10; col++) {
        int piv = col;
        for (int r = col + 1; r < 10; r++)
            if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
        if (A[piv][col] == 0.0) return 0;
        if (piv != col)
            for (int c = 0; c < 20; c++) { double t = A[col][c]; A[col][c] = A[piv][c]; A[piv][c] = t; }
        const double inv = 1.0 / A[col][col];
        for (int c = 0; c < 20; c++) A[col][c] *= inv;
        for (int r = 0; r < 10; r++) {
            if (r == col) continue;
            const double f = A[r][col];
            if (f == 0.0) continue;
            for (int c = 0; c < 20; c++) A[r][c] -= f * A[col][c];
        }
    }
    for (int r = 0; r < 10; r++)
        for (int c = 0; c < 10; c++) R[r][c] = A[r][10 + c];
    return 1;
}

/* polynomial helpers in z (ascending coefficient arrays) */
static void zmul(const double* a, int na, const double* b, int nb, double* r /* na + nb - 1 */)
{
    for (int i = 0; i < na + nb - 1; i++) r[i] = 0;
    for (int i = 0; i < na; i++)
        for (int j = 0; j < nb; j++) r[i + j] += a[i] * b[j];
}

/* Durand-Kerner roots of sum c[k] z^k (degree n, c[n] != 0) */
static int dk_roots(const double* c, int n, double* re, double* im)
{
    double a[11];
    for (int k = 0; k <= n; k++) a[k] = c[k] / c[n];
    double zr = 0.4, zi = 0.9;
    re[0] = 1.0; im[0] = 0.0;
    for (int k = 0; k < n; k++) {
        if (k > 0) {
            const double r = re[k - 1] * zr - im[k - 1] * zi, i = re[k - 1] * zi + im[k - 1] * zr;
            re[k] = r; im[k] = i;
        } else { re[0] = zr; im[0] = zi; }
    }
    for (int iter = 0; iter < 500; iter++) {
        double maxd = 0;
        for (int k = 0; k < n; k++) {
            /* p(z_k) by Horner */
            double pr = 1.0, pi = 0.0;
            for (int d = n - 1; d >= 0; d--) {
                const double tr = pr * re[k] - pi * im[k] + a[d], ti = pr * im[k] + pi * re[k];
                pr = tr; pi = ti;
            }
            double qr = 1.0, qi = 0.0;
            for (int j = 0; j < n; j++) {
                if (j == k) continue;
                const double dr = re[k] - re[j], di = im[k] - im[j];
                const double tr = qr * dr - qi * di, ti = qr * di + qi * dr;
                qr = tr; qi = ti;
            }
            const double den = qr * qr + qi * qi;
            if (den == 0.0) continue;
            const double dr = (pr * qr + pi * qi) / den, di = (pi * qr - pr * qi) / den;
            re[k] -= dr;
            im[k] -= di;
            const double mag = fabs(dr) + fabs(di);
            if (mag > maxd) maxd = mag;
        }
        if (maxd <= 1e-14) break;
    }
    return n;
}

/* EMEstimatorCallback::runKernel: up to 10 E (row-major 3 x 3) from 5 normalised correspondences */
int orc_five_point(const double* q1 /* 5 x 2 */, const double* q2, double* Es /* 10 x 9 */)
{
    /* Q (5 x 9) rows: x1 x2, y1 x2, x2, x1 y2, y1 y2, y2, x1, y1, 1 */
    double Qt[9 * 9];
    memset(Qt, 0, sizeof(Qt));
    double Q[5][9];
    for (int i = 0; i < 5; i++) {
        const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        const double row[9] = {x1 * x2, y1 * x2, x2, x1 * y2, y1 * y2, y2, x1, y1, 1.0};
        for (int k = 0; k < 9; k++) Q[i][k] = row[k];
    }
    /* Householder QR of Q' (9 x 5): the last 4 columns of the orthogonal factor span null(Q) */
    double M[9][5], V[5][9];
    double H[9][9];
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 5; c++) M[r][c] = Q[c][r];
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 9; c++) H[r][c] = r == c ? 1.0 : 0.0;
    for (int k = 0; k < 5; k++) {
        double nrm = 0;
        for (int r = k; r < 9; r++) nrm += M[r][k] * M[r][k];
        nrm = sqrt(nrm);
        double* v = V[k];
        for (int r = 0; r < 9; r++) v[r] = r < k ? 0.0 : M[r][k];
        const double alpha = M[k][k] >= 0 ? -nrm : nrm;
        v[k] -= alpha;
        double vn = 0;
        for (int r = k; r < 9; r++) vn += v[r] * v[r];
        if (vn == 0.0) continue;
        /* M <- (I - 2 v v' / vn) M ; H <- H (I - 2 v v' / vn) */
        for (int c = 0; c < 5; c++) {
            double s = 0;
            for (int r = k; r < 9; r++) s += v[r] * M[r][c];
            s = 2 * s / vn;
            for (int r = k; r < 9; r++) M[r][c] -= s * v[r];
        }
        for (int r = 0; r < 9; r++) {
            double s = 0;
            for (int c = k; c < 9; c++) s += H[r][c] * v[c];
            s = 2 * s / vn;
            for (int c = k; c < 9; c++) H[r][c] -= s * v[c];
        }
    }
    double EE[4][9];
    for (int b = 0; b < 4; b++)
        for (int r = 0; r < 9; r++) EE[b][r] = H[r][5 + b];
    double A[10][20], R[10][10];
    coeff_mat(EE, A);
    if (!gj_solve(A, R)) return 0;
    /* B (3 x 13) from row pairs (4, 5), (6, 7), (8, 9): x [z^3 z^2 z 1], y [..], 1 [z^4 .. 1] */
    double b[3][13];
    for (int i = 0; i < 3; i++) {
        const double* r1 = R[i * 2 + 4];
        const double* r2 = R[i * 2 + 5];
        double row1[13] = {0}, row2[13] = {0};
        for (int k = 0; k < 3; k++) { row1[1 + k] = r1[k]; row1[5 + k] = r1[3 + k]; }
        for (int k = 0; k < 4; k++) row1[9 + k] = r1[6 + k];
        for (int k = 0; k < 3; k++) { row2[k] = r2[k]; row2[4 + k] = r2[3 + k]; }
        for (int k = 0; k < 4; k++) row2[8 + k] = r2[6 + k];
        for (int k = 0; k < 13; k++) b[i][k] = row1[k] - row2[k];
    }
    /* entries as ascending polynomials in z */
    double P[3][3][5];
    for (int i = 0; i < 3; i++) {
        for (int k = 0; k < 5; k++) P[i][0][k] = P[i][1][k] = P[i][2][k] = 0;
        for (int k = 0; k < 4; k++) { P[i][0][3 - k] = b[i][k]; P[i][1][3 - k] = b[i][4 + k]; }
        for (int k = 0; k < 5; k++) P[i][2][4 - k] = b[i][8 + k];
    }
    /* det of the 3 x 3 polynomial matrix (degrees 3, 3, 4 per row): degree 10 */
    const int deg[3] = {3, 3, 4};
    double cdet[11] = {0};
    {
        static const int perm[6][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 0}};
        static const double sign[6] = {1, 1, 1, -1, -1, -1};
        for (int q = 0; q < 6; q++) {
            double t1[9], t2[11];
            zmul(P[0][perm[q][0]], deg[perm[q][0]] + 1, P[1][perm[q][1]], deg[perm[q][1]] + 1, t1);
            const int n1 = deg[perm[q][0]] + deg[perm[q][1]] + 1;
            zmul(t1, n1, P[2][perm[q][2]], deg[perm[q][2]] + 1, t2);
            const int n2 = n1 + deg[perm[q][2]];
            for (int k = 0; k < n2 && k < 11; k++) cdet[k] += sign[q] * t2[k];
        }
    }
    int n = 10;
    while (n > 0 && cdet[n] == 0.0) n--;
    if (n == 0) return 0;
    double re[10], im[10];
    dk_roots(cdet, n, re, im);
    int count = 0;
    for (int r = 0; r < n; r++) {
        if (fabs(im[r]) > 1e-10) continue;
        const double z1 = re[r], z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double Bz[9];
        for (int j = 0; j < 3; j++) {
            const double* br = b[j];
            Bz[j * 3 + 0] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            Bz[j * 3 + 1] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            Bz[j * 3 + 2] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        double U[9], W[3], Vt[9];
        svd33(Bz, U, W, Vt);
        const double* xy1 = Vt + 6;       /* SVD::solveZ: the last right singular vector */
        if (fabs(xy1[2]) < 1e-10) continue;
        const double xs = xy1[0] / xy1[2], ys = xy1[1] / xy1[2];
        double Ev[9], nrm = 0;
        for (int k = 0; k < 9; k++) {
            Ev[k] = EE[0][k] * xs + EE[1][k] * ys + EE[2][k] * z1 + EE[3][k];
            nrm += Ev[k] * Ev[k];
        }
        nrm = sqrt(nrm);
        for (int k = 0; k < 9; k++) Es[count * 9 + k] = Ev[k] / nrm;
        count++;
    }
    return count;
}

/* EMEstimatorCallback::computeError: Sampson distance, stored as f32 */
float orc_sampson(const double E[9], double x1, double y1, double x2, double y2)
{
    const double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    const double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7],
                            E[2] * x2 + E[5] * y2 + E[8]};
    const double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    const double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

/* findEssentialMat(RANSAC): returns 1 with E (3 x 3) and the RANSAC mask, 0 if no model */
int orc_find_essential(const float* p1, const float* p2, int n, const double K[9], double prob, double threshold,
                       double E[9], uint8_t* mask, int* niters_used)
{
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double* q = (double*)malloc(sizeof(double) * 4 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        q[4 * i] = ((double)p1[2 * i] - cx) / fx;
        q[4 * i + 1] = ((double)p1[2 * i + 1] - cy) / fy;
        q[4 * i + 2] = ((double)p2[2 * i] - cx) / fx;
        q[4 * i + 3] = ((double)p2[2 * i + 1] - cy) / fy;
    }
    const double thr = threshold / ((fx + fy) / 2);
    const float t = (float)(thr * thr);
    const int maxIters = 1000;
    int ok = 0, maxGood = 0;
    if (n < 5) { free(q); return 0; }
    if (n == 5) {   /* count == modelPoints: the first model, every point an inlier */
        double a1[10], a2[10], Es0[90];
        for (int k = 0; k < 5; k++) {
            a1[2 * k] = q[4 * k]; a1[2 * k + 1] = q[4 * k + 1];
            a2[2 * k] = q[4 * k + 2]; a2[2 * k + 1] = q[4 * k + 3];
        }
        const int nm = orc_five_point(a1, a2, Es0);
        free(q);
        if (nm <= 0) return 0;
        memcpy(E, Es0, sizeof(double) * 9);
        memset(mask, 1, 5);
        if (niters_used) *niters_used = 1;
        return 1;
    }
    int* idx = (int*)malloc(sizeof(int) * 5 * maxIters);
    orc_ep_subsets(n, maxIters, idx);
    int niters = maxIters, iter;
    double Es[90];
    uint8_t* cur = (uint8_t*)malloc((size_t)n);
    for (iter = 0; iter < niters; iter++) {
        double a1[10], a2[10];
        for (int k = 0; k < 5; k++) {
            const int j = idx[5 * iter + k];
            a1[2 * k] = q[4 * j]; a1[2 * k + 1] = q[4 * j + 1];
            a2[2 * k] = q[4 * j + 2]; a2[2 * k + 1] = q[4 * j + 3];
        }
        const int nm = orc_five_point(a1, a2, Es);
        for (int m = 0; m < nm; m++) {
            int good = 0;
            for (int i = 0; i < n; i++) {
                cur[i] = orc_sampson(Es + 9 * m, q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]) <= t;
                good += cur[i];
            }
            if (good > (maxGood > 4 ? maxGood : 4)) {
                memcpy(mask, cur, (size_t)n);
                memcpy(E, Es + 9 * m, sizeof(double) * 9);
                maxGood = good;
                ok = 1;
                niters = orc_ransac_update_iters(prob, (double)(n - good) / n, 5, niters);
            }
        }
    }
    if (niters_used) *niters_used = iter;
    free(cur);
    free(idx);
    free(q);
    return ok;
}

/* homogeneous DLT point from two 3 x 4 projections (cv::triangulatePoints) */
static void tri_point(const double* P1, const double* P2, double x1, double y1, double x2, double y2, double X[4])
{
    const double* P[2] = {P1, P2};
    const double xs[2] = {x1, x2}, ys[2] = {y1, y2};
    double At[16], W[4], Vt[16];
    for (int v = 0; v < 2; v++)
        for (int c = 0; c < 4; c++) {
            At[c * 4 + v * 2] = xs[v] * P[v][8 + c] - P[v][c];
            At[c * 4 + v * 2 + 1] = ys[v] * P[v][8 + c] - P[v][4 + c];
        }
    orc_jsvd(At, 4, 4, W, Vt);
    for (int k = 0; k < 4; k++) X[k] = Vt[12 + k];
}

/* decomposeEssentialMat */
void orc_decompose_essential(const double E[9], double R1[9], double R2[9], double t[3])
{
    double U[9], W[3], Vt[9];
    svd33(E, U, W, Vt);
    if (det33(U) < 0)
        for (int k = 0; k < 9; k++) U[k] *= -1.;
    if (det33(Vt) < 0)
        for (int k = 0; k < 9; k++) Vt[k] *= -1.;
    static const double Wm[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
    double UW[9], UWt[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0, s2 = 0;
            for (int k = 0; k < 3; k++) { s += U[r * 3 + k] * Wm[k * 3 + c]; s2 += U[r * 3 + k] * Wm[c * 3 + k]; }
            UW[r * 3 + c] = s;
            UWt[r * 3 + c] = s2;
        }
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0, s2 = 0;
            for (int k = 0; k < 3; k++) { s += UW[r * 3 + k] * Vt[k * 3 + c]; s2 += UWt[r * 3 + k] * Vt[k * 3 + c]; }
            R1[r * 3 + c] = s;
            R2[r * 3 + c] = s2;
        }
    for (int k = 0; k < 3; k++) t[k] = U[k * 3 + 2];
}

/* the cheirality bits of one point for the 4 poses (bit k: pose k passes) */
int orc_cheirality_bits(const double R1[9], const double R2[9], const double t[3], double dist, double x1,
                        double y1, double x2, double y2)
{
    static const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int bits = 0;
    for (int pose = 0; pose < 4; pose++) {
        const double* R = (pose & 1) ? R2 : R1;
        const double sg = pose >= 2 ? -1.0 : 1.0;
        double P[12];
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) P[r * 4 + c] = R[r * 3 + c];
            P[r * 4 + 3] = t[r] * sg;
        }
        double X[4];
        tri_point(P0, P, x1, y1, x2, y2, X);
        int ok = X[2] * X[3] > 0;
        const double Xn[4] = {X[0] / X[3], X[1] / X[3], X[2] / X[3], X[3] / X[3]};
        ok = ok && Xn[2] < dist;
        double z2 = 0;
        for (int k = 0; k < 4; k++) z2 += P[8 + k] * Xn[k];
        ok = ok && z2 > 0 && z2 < dist;
        if (ok) bits |= 1 << pose;
    }
    return bits;
}

/* recoverPose(E, points1, points2, K, R, t, distanceThresh, mask (empty)): returns the good count */
int orc_recover_pose(const double E[9], const float* p1, const float* p2, int n, const double K[9], double dist,
                     double R[9], double t[3], uint8_t* mask)
{
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    double R1[9], R2[9], tt[3];
    orc_decompose_essential(E, R1, R2, tt);
    int good[4] = {0, 0, 0, 0};
    uint8_t* bits = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        const double x1 = ((double)p1[2 * i] - cx) / fx, y1 = ((double)p1[2 * i + 1] - cy) / fy;
        const double x2 = ((double)p2[2 * i] - cx) / fx, y2 = ((double)p2[2 * i + 1] - cy) / fy;
        bits[i] = (uint8_t)orc_cheirality_bits(R1, R2, tt, dist, x1, y1, x2, y2);
        for (int k = 0; k < 4; k++) good[k] += (bits[i] >> k) & 1;
    }
    int pick;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) pick = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) pick = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) pick = 2;
    else pick = 3;
    memcpy(R, (pick & 1) ? R2 : R1, sizeof(double) * 9);
    for (int k = 0; k < 3; k++) t[k] = pick >= 2 ? -tt[k] : tt[k];
    for (int i = 0; i < n; i++) mask[i] = (bits[i] >> pick) & 1;
    free(bits);
    return good[pick];
}

/* estimateTransformation: returns passedPointsCount > 0; RANSAC mask and its count too */
int orc_estimate_transformation(const float* p1, const float* p2, int n, const double K[9], int use_ransac,
                                double prob, double threshold, double dist, double R[9], double t[3],
                                uint8_t* chirality, uint8_t* ransac_mask, int* passed)
{
    double E[9];
    if (!use_ransac) { prob = 0.999; threshold = 1.0; }   /* findEssentialMat(points1, points2, K) defaults */
    if (!orc_find_essential(p1, p2, n, K, prob, threshold, E, ransac_mask, NULL)) { *passed = 0; return 0; }
    *passed = orc_recover_pose(E, p1, p2, n, K, dist, R, t, chirality);
    return *passed > 0;
}
