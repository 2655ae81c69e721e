/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED against
 * OpenCV itself (not in this image); checked in tests/test_oracle.py against
 * noise-free synthetic scenes (EPnP and the refined pose recover R, t to
 * 1e-9), scipy's rotation vectors, finite-difference Jacobians and noisy scenes
 * with outliers (inlier sets, pose error).
 *
 * solvePnPRansac as the reference calls it (src/mainModule/cycleProcessing/
 * mainCycle.cpp:155-161): solvePnPRansac(Point3f objects, Point2f image, K,
 * distortionCoeffs = empty Mat, rvec, tvec) with every default --
 * useExtrinsicGuess false, iterationsCount 100, reprojectionError 8,
 * confidence 0.99, flags SOLVEPNP_ITERATIVE.  Restated from OpenCV 4.8:
 *   - calib3d/src/solvepnp.cpp solvePnPRansac + PnPRansacCallback: minimal
 *     sets of 5 (SOLVEPNP_EPNP kernel), model = [rvec | tvec], error = f32
 *     squared distance between the image point and the f32 projection, inlier
 *     iff err <= (float)(8 * 8); RANSACPointSetRegistrator::run (ptsetreg.cpp)
 *     with RNG((uint64)-1) -- shared with essential.c (orc_ep_subsets,
 *     orc_ransac_update_iters); a model is kept iff its count exceeds
 *     max(best, 4).  Then the inliers (compressElems, in index order, as f64)
 *     are refined by solvePnP(SOLVEPNP_ITERATIVE, useExtrinsicGuess = true)
 *     from the RANSAC model.  npoints == 5 runs EPnP once on all points and
 *     returns without refinement; npoints == 4 (OpenCV: P3P) is not restated.
 *   - EPnP (calib3d/src/epnp.cpp): image points through undistortPoints (no
 *     distortion: (u - cx) * (1/fx), stored f32) and back (x fu + uc); control
 *     points from the centroid and the PCA of the object points (cvSVD of
 *     PW0' PW0); barycentric coordinates via cvInvert(CV_SVD); M (2n x 12),
 *     cvMulTransposed, cvSVD(U_T); L_6x10, rho; betas by the three
 *     approximations (cvSolve CV_SVD) each polished by 5 Gauss-Newton steps
 *     (epnp's own Householder qr_solve); R, t by the SVD of sum (pc - pc0)
 *     (pw - pw0)' with a det < 0 flip; the lowest mean reprojection error wins.
 *   - Rodrigues (calib3d/src/calibration.cpp cvRodrigues2) both ways: the
 *     matrix is orthonormalised as U Vt of its SVD, theta = acos(c) with the
 *     s < 1e-5 special cases; vector -> matrix with the 3 x 9 Jacobian.
 *   - cvFindExtrinsicCameraParams2's guess path: CvLevMarq(6, 2n, EPS + ITER,
 *     max_iter 20, FLT_EPSILON) -- lambda 10^-3, diag *= 1 + lambda, solve
 *     DECOMP_SVD, lambdaLg10 +1 on a worse error (<= 16), -1 otherwise, stop on
 *     20 iterations or ||p - p_prev|| / (||p_prev|| + DBL_EPSILON) < FLT_EPSILON;
 *     residuals and Jacobian from cvProjectPoints2 with no distortion.
 * Linear algebra is core's: JacobiSVDImpl_ (orc_jsvd, eps 10 DBL_EPSILON) with
 * left vectors = normalised A' rows, SVBkSb with threshold 2 DBL_EPSILON sum(w),
 * MulTransposedR / GEMMSingleMul sequential sums, normL2Sqr's 4-wide unroll.
 * Not restated: the random left vectors JacobiSVD draws for singular values <=
 * DBL_MIN (unreachable for rounding-perturbed inputs), any HAL/SIMD summation
 * order in cv::norm.  No contraction (Makefile: -ffp-contract=off); the GPU
 * path (csrc/pnp.hip) shares every operation order.
 */
#define _GNU_SOURCE   /* sincos */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- core linear algebra ---- */

/* JacobiSVDImpl_ with n1 = n: At rows (n x m) become the left vectors */
static void jsvd_u(double* At, int n, int m, double* W, double* Vt)
{
    orc_jsvd(At, n, m, W, Vt);
    for (int i = 0; i < n; i++) {
        const double s = W[i] > DBL_MIN ? 1 / W[i] : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* cv::solve(A (m x n, m >= n), b, x, DECOMP_SVD): a = A', JacobiSVD, SVBkSb(uT) */
static void solve_svd(const double* A, int m, int n, const double* b, double* x)
{
    double At[12 * 12], W[12], Vt[12 * 12];
    for (int r = 0; r < m; r++)
        for (int c = 0; c < n; c++) At[c * m + r] = A[r * n + c];
    jsvd_u(At, n, m, W, Vt);
    double thr = 0;
    for (int i = 0; i < n; i++) thr += W[i];
    thr *= DBL_EPSILON * 2;
    for (int j = 0; j < n; j++) x[j] = 0;
    for (int i = 0; i < n; i++) {
        double wi = W[i];
        if (fabs(wi) <= thr) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < m; j++) s += At[i * m + j] * b[j];
        s *= wi;
        for (int j = 0; j < n; j++) x[j] = x[j] + s * Vt[i * n + j];
    }
}

/* cv::invert(A (n x n), DECOMP_SVD): SVD::compute + backSubst with no rhs */
static void invert_svd(const double* A, int n, double* X)
{
    double At[9], W[3], Vt[9], buf[3];
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) At[c * n + r] = A[r * n + c];
    jsvd_u(At, n, n, W, Vt);
    double thr = 0;
    for (int i = 0; i < n; i++) thr += W[i];
    thr *= DBL_EPSILON * 2;
    for (int k = 0; k < n * n; k++) X[k] = 0;
    for (int i = 0; i < n; i++) {
        double wi = W[i];
        if (fabs(wi) <= thr) continue;
        wi = 1 / wi;
        for (int j = 0; j < n; j++) buf[j] = At[i * n + j] * wi;     /* U(j, i) / w_i */
        for (int r = 0; r < n; r++) {
            const double s = Vt[i * n + r];
            for (int j = 0; j < n; j++) X[r * n + j] = X[r * n + j] + s * buf[j];
        }
    }
}

/* cvMulTransposed(A (m x n), C, 1) = A' A: sequential sums, upper then mirrored */
static void mul_at_a(const double* A, int m, int n, double* C)
{
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            double s = 0;
            for (int k = 0; k < m; k++) s += A[k * n + i] * A[k * n + j];
            C[i * n + j] = s;
        }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) C[i * n + j] = C[j * n + i];
}

/* normL2Sqr<double, double>: 4-wide unrolled blocks, then the tail */
static double norm_l2sqr(const double* a, int n)
{
    double s = 0;
    int i = 0;
    for (; i <= n - 4; i += 4) s += a[i] * a[i] + a[i + 1] * a[i + 1] + a[i + 2] * a[i + 2] + a[i + 3] * a[i + 3];
    for (; i < n; i++) s += a[i] * a[i];
    return s;
}

/* ---- Rodrigues (cvRodrigues2) ---- */
void orc_rodrigues_v2m(const double rv[3], double R[9], double J[27])
{
    double rx = rv[0], ry = rv[1], rz = rv[2];
    const double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1 : 0;
        if (J) {
            memset(J, 0, 27 * sizeof(double));
            J[5] = J[15] = J[19] = -1;
            J[7] = J[11] = J[21] = 1;
        }
        return;
    }
    /* GCC compiles OpenCV's cos(theta) / sin(theta) pair into one glibc sincos
     * call; written out so the oracle does not depend on that optimisation */
    double s, c;
    sincos(theta, &s, &c);
    const double c1 = 1. - c, itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * r_x[k];
    if (J) {
        const double drrt[27] = {rx + rx, ry, rz, ry, 0, 0, rz, 0, 0,
                                 0, rx, 0, rx, ry + ry, rz, 0, rz, 0,
                                 0, 0, rx, 0, 0, ry, rx, ry, rz + rz};
        const double d_r_x_[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0,
                                   0, 0, 1, 0, 0, 0, -1, 0, 0,
                                   0, -1, 0, 1, 0, 0, 0, 0, 0};
        for (int i = 0; i < 3; i++) {
            const double ri = i == 0 ? rx : i == 1 ? ry : rz;
            const double a0 = -s * ri, a1 = (s - 2 * c1 * itheta) * ri, a2 = c1 * itheta;
            const double a3 = (c - s * itheta) * ri, a4 = s * itheta;
            for (int k = 0; k < 9; k++)
                J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * r_x[k] + a4 * d_r_x_[i * 9 + k];
        }
    }
}

void orc_rodrigues_m2v(const double Rin[9], double rv[3])
{
    for (int k = 0; k < 9; k++)
        if (!(Rin[k] >= -100 && Rin[k] < 100)) { rv[0] = rv[1] = rv[2] = 0; return; }   /* checkRange */
    double At[9], W[3], Vt[9], R[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = Rin[r * 3 + c];
    jsvd_u(At, 3, 3, W, Vt);                      /* U(i, k) = At[k][i] */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += At[k * 3 + i] * Vt[k * 3 + j];
            R[i * 3 + j] = s;
        }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rv[0] = rx; rv[1] = ry; rv[2] = rz;
}

/* ---- EPnP (calib3d/src/epnp.cpp) ---- */
typedef struct {
    int n;
    const double* pws;      /* n x 3 */
    const double* us;       /* n x 2 (pixels) */
    double fu, fv, uc, vc;
    double* alphas;         /* n x 4 */
    double* pcs;            /* n x 3 */
    double cws[4][3], ccs[4][3];
} epnp_t;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double dist2(const double* a, const double* b)
{
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

static void choose_control_points(epnp_t* e)
{
    const int n = e->n;
    e->cws[0][0] = e->cws[0][1] = e->cws[0][2] = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) e->cws[0][j] += e->pws[3 * i + j];
    for (int j = 0; j < 3; j++) e->cws[0][j] /= n;
    double* PW0 = (double*)malloc(sizeof(double) * 3 * (size_t)n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) PW0[3 * i + j] = e->pws[3 * i + j] - e->cws[0][j];
    double ptp[9], At[9], dc[3], Vt[9];
    mul_at_a(PW0, n, 3, ptp);
    free(PW0);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = ptp[r * 3 + c];
    jsvd_u(At, 3, 3, dc, Vt);                     /* UCt rows = At rows */
    for (int i = 1; i < 4; i++) {
        const double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; j++) e->cws[i][j] = e->cws[0][j] + k * At[3 * (i - 1) + j];
    }
}

static void compute_barycentric_coordinates(epnp_t* e)
{
    double cc[9], ci[9];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = e->cws[j][i] - e->cws[0][i];
    invert_svd(cc, 3, ci);
    for (int i = 0; i < e->n; i++) {
        const double* pi = e->pws + 3 * i;
        double* a = e->alphas + 4 * i;
        for (int j = 0; j < 3; j++)
            a[1 + j] = ci[3 * j] * (pi[0] - e->cws[0][0]) + ci[3 * j + 1] * (pi[1] - e->cws[0][1]) +
                       ci[3 * j + 2] * (pi[2] - e->cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
}

static void compute_L_6x10(const double* ut, double* l)
{
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
        int a = 0, b = 1;
        for (int j = 0; j < 6; j++) {
            dv[i][j][0] = v[i][3 * a] - v[i][3 * b];
            dv[i][j][1] = v[i][3 * a + 1] - v[i][3 * b + 1];
            dv[i][j][2] = v[i][3 * a + 2] - v[i][3 * b + 2];
            b++;
            if (b > 3) { a++; b = a + 1; }
        }
    }
    for (int i = 0; i < 6; i++) {
        double* row = l + 10 * i;
        row[0] = dot3(dv[0][i], dv[0][i]);
        row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
        row[2] = dot3(dv[1][i], dv[1][i]);
        row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
        row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
        row[5] = dot3(dv[2][i], dv[2][i]);
        row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
        row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
        row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
        row[9] = dot3(dv[3][i], dv[3][i]);
    }
}

static void find_betas_1(const double* L, const double* rho, double* betas)
{
    double l[24], b4[4];
    for (int i = 0; i < 6; i++) {
        l[4 * i] = L[10 * i]; l[4 * i + 1] = L[10 * i + 1]; l[4 * i + 2] = L[10 * i + 3]; l[4 * i + 3] = L[10 * i + 6];
    }
    solve_svd(l, 6, 4, rho, b4);
    if (b4[0] < 0) {
        betas[0] = sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0];
        betas[2] = -b4[2] / betas[0];
        betas[3] = -b4[3] / betas[0];
    } else {
        betas[0] = sqrt(b4[0]);
        betas[1] = b4[1] / betas[0];
        betas[2] = b4[2] / betas[0];
        betas[3] = b4[3] / betas[0];
    }
}

static void find_betas_2(const double* L, const double* rho, double* betas)
{
    double l[18], b3[3];
    for (int i = 0; i < 6; i++) { l[3 * i] = L[10 * i]; l[3 * i + 1] = L[10 * i + 1]; l[3 * i + 2] = L[10 * i + 2]; }
    solve_svd(l, 6, 3, rho, b3);
    if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
    } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
}

static void find_betas_3(const double* L, const double* rho, double* betas)
{
    double l[30], b5[5];
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 5; k++) l[5 * i + k] = L[10 * i + k];
    solve_svd(l, 6, 5, rho, b5);
    if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
    } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
}

/* epnp::qr_solve (6 x 4), in place on A and b */
static void qr_solve(double* A, double* b, double* X)
{
    const int nr = 6, nc = 4;
    double A1[6], A2[6];
    for (int k = 0; k < nc; k++) {
        double eta = fabs(A[k * nc + k]);
        for (int i = k + 1; i < nr; i++) {
            const double elt = fabs(A[i * nc + k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
            return;          /* X untouched, as epnp */
        }
        double sum2 = 0.0;
        const double inv_eta = 1. / eta;
        for (int i = k; i < nr; i++) {
            A[i * nc + k] *= inv_eta;
            sum2 += A[i * nc + k] * A[i * nc + k];
        }
        double sigma = sqrt(sum2);
        if (A[k * nc + k] < 0) sigma = -sigma;
        A[k * nc + k] += sigma;
        A1[k] = sigma * A[k * nc + k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double sum = 0;
            for (int i = k; i < nr; i++) sum += A[i * nc + k] * A[i * nc + j];
            const double tau = sum / A1[k];
            for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
        }
    }
    for (int j = 0; j < nc; j++) {
        double tau = 0;
        for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double sum = 0;
        for (int j = i + 1; j < nc; j++) sum += A[i * nc + j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

static void gauss_newton(const double* L, const double* rho, double betas[4])
{
    double A[24], b[6], x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
        for (int i = 0; i < 6; i++) {
            const double* rl = L + i * 10;
            double* ra = A + i * 4;
            ra[0] = 2 * rl[0] * betas[0] + rl[1] * betas[1] + rl[3] * betas[2] + rl[6] * betas[3];
            ra[1] = rl[1] * betas[0] + 2 * rl[2] * betas[1] + rl[4] * betas[2] + rl[7] * betas[3];
            ra[2] = rl[3] * betas[0] + rl[4] * betas[1] + 2 * rl[5] * betas[2] + rl[8] * betas[3];
            ra[3] = rl[6] * betas[0] + rl[7] * betas[1] + rl[8] * betas[2] + 2 * rl[9] * betas[3];
            b[i] = rho[i] - (rl[0] * betas[0] * betas[0] + rl[1] * betas[0] * betas[1] + rl[2] * betas[1] * betas[1] +
                             rl[3] * betas[0] * betas[2] + rl[4] * betas[1] * betas[2] + rl[5] * betas[2] * betas[2] +
                             rl[6] * betas[0] * betas[3] + rl[7] * betas[1] * betas[3] + rl[8] * betas[2] * betas[3] +
                             rl[9] * betas[3] * betas[3]);
        }
        qr_solve(A, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

static double compute_R_and_t(epnp_t* e, const double* ut, const double* betas, double R[9], double t[3])
{
    const int n = e->n;
    for (int i = 0; i < 4; i++) e->ccs[i][0] = e->ccs[i][1] = e->ccs[i][2] = 0.0;
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) e->ccs[j][k] += betas[i] * v[3 * j + k];
    }
    for (int i = 0; i < n; i++) {
        const double* a = e->alphas + 4 * i;
        double* pc = e->pcs + 3 * i;
        for (int j = 0; j < 3; j++)
            pc[j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
    }
    if (e->pcs[2] < 0.0) {                                   /* solve_for_sign */
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) e->ccs[i][j] = -e->ccs[i][j];
        for (int i = 0; i < 3 * n; i++) e->pcs[i] = -e->pcs[i];
    }
    /* estimate_R_and_t */
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) { pc0[j] += e->pcs[3 * i + j]; pw0[j] += e->pws[3 * i + j]; }
    for (int j = 0; j < 3; j++) { pc0[j] /= n; pw0[j] /= n; }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const double* pc = e->pcs + 3 * i;
        const double* pw = e->pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    double At[9], W[3], Vt[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = abt[r * 3 + c];
    jsvd_u(At, 3, 3, W, Vt);                  /* abt_u(i, k) = At[k][i], abt_v(j, k) = Vt[k][j] */
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[3 * i + j] = At[i] * Vt[j] + At[3 + i] * Vt[3 + j] + At[6 + i] * Vt[6 + j];
    const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                       R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
    if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
    t[0] = pc0[0] - dot3(R, pw0);
    t[1] = pc0[1] - dot3(R + 3, pw0);
    t[2] = pc0[2] - dot3(R + 6, pw0);
    /* reprojection_error */
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
        const double* pw = e->pws + 3 * i;
        const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1];
        const double inv_Zc = 1.0 / (dot3(R + 6, pw) + t[2]);
        const double ue = e->uc + e->fu * Xc * inv_Zc, ve = e->vc + e->fv * Yc * inv_Zc;
        const double u = e->us[2 * i], v = e->us[2 * i + 1];
        sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
}

/* solvePnPGeneric(SOLVEPNP_EPNP): R, t for n >= 4 correspondences (object
 * points as f64, image points f32) */
void orc_epnp(int n, const double* op, const float* ip, const double K[9], double R[9], double t[3])
{
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    epnp_t e;
    e.n = n;
    e.fu = fx; e.fv = fy; e.uc = cx; e.vc = cy;
    double* us = (double*)malloc(sizeof(double) * 2 * (size_t)n);
    double* M = (double*)malloc(sizeof(double) * 24 * (size_t)n);
    e.alphas = (double*)malloc(sizeof(double) * 4 * (size_t)n);
    e.pcs = (double*)malloc(sizeof(double) * 3 * (size_t)n);
    const double ifx = 1. / fx, ify = 1. / fy;
    for (int i = 0; i < n; i++) {
        /* undistortPoints (no distortion, R = P = I): f32 normalised points */
        const float xn = (float)(((double)ip[2 * i] - cx) * ifx), yn = (float)(((double)ip[2 * i + 1] - cy) * ify);
        us[2 * i] = xn * fx + cx;          /* epnp::init_points */
        us[2 * i + 1] = yn * fy + cy;
    }
    e.pws = op;
    e.us = us;
    choose_control_points(&e);
    compute_barycentric_coordinates(&e);
    for (int i = 0; i < n; i++) {
        const double* as = e.alphas + 4 * i;
        const double u = us[2 * i], v = us[2 * i + 1];
        double* M1 = M + 24 * i;
        double* M2 = M1 + 12;
        for (int k = 0; k < 4; k++) {
            M1[3 * k] = as[k] * e.fu;
            M1[3 * k + 1] = 0.0;
            M1[3 * k + 2] = as[k] * (e.uc - u);
            M2[3 * k] = 0.0;
            M2[3 * k + 1] = as[k] * e.fv;
            M2[3 * k + 2] = as[k] * (e.vc - v);
        }
    }
    double mtm[144], ut[144], d[12], Vt[144];
    mul_at_a(M, 2 * n, 12, mtm);
    for (int r = 0; r < 12; r++)
        for (int c = 0; c < 12; c++) ut[c * 12 + r] = mtm[r * 12 + c];
    jsvd_u(ut, 12, 12, d, Vt);                /* Ut = normalised At rows */
    double L[60], rho[6];
    compute_L_6x10(ut, L);
    rho[0] = dist2(e.cws[0], e.cws[1]);
    rho[1] = dist2(e.cws[0], e.cws[2]);
    rho[2] = dist2(e.cws[0], e.cws[3]);
    rho[3] = dist2(e.cws[1], e.cws[2]);
    rho[4] = dist2(e.cws[1], e.cws[3]);
    rho[5] = dist2(e.cws[2], e.cws[3]);
    double Betas[4][4], rep[4], Rs[4][9], ts[4][3];
    find_betas_1(L, rho, Betas[1]);
    gauss_newton(L, rho, Betas[1]);
    rep[1] = compute_R_and_t(&e, ut, Betas[1], Rs[1], ts[1]);
    find_betas_2(L, rho, Betas[2]);
    gauss_newton(L, rho, Betas[2]);
    rep[2] = compute_R_and_t(&e, ut, Betas[2], Rs[2], ts[2]);
    find_betas_3(L, rho, Betas[3]);
    gauss_newton(L, rho, Betas[3]);
    rep[3] = compute_R_and_t(&e, ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    memcpy(R, Rs[N], sizeof(double) * 9);
    memcpy(t, ts[N], sizeof(double) * 3);
    free(us); free(M); free(e.alphas); free(e.pcs);
}

/* PnPRansacCallback::computeError: f32 projection, f32 squared distance */
float orc_pnp_error(const double R[9], const double t[3], const double K[9], const float* o, const float* m)
{
    const double X = o[0], Y = o[1], Z = o[2];
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z; y *= z;
    const float px = (float)(x * K[0] + K[2]), py = (float)(y * K[4] + K[5]);
    const float dx = m[0] - px, dy = m[1] - py;
    float s = 0;
    s += dx * dx;
    s += dy * dy;
    return s;
}

/* residuals (projection - observation) and, if J, the 2n x 6 Jacobian
 * [dp/dr | dp/dt] of cvProjectPoints2 with no distortion */
static void project_jac(const double* param, const double K[9], const double* op, const double* ip, int n,
                        double* err, double* J)
{
    double R[9], dRdr[27];
    orc_rodrigues_v2m(param, R, dRdr);
    const double* t = param + 3;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    for (int i = 0; i < n; i++) {
        const double X = op[3 * i], Y = op[3 * i + 1], Z = op[3 * i + 2];
        double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        z = z ? 1. / z : 1;
        x *= z; y *= z;
        err[2 * i] = (x * fx + cx) - ip[2 * i];
        err[2 * i + 1] = (y * fy + cy) - ip[2 * i + 1];
        if (!J) continue;
        double* jx = J + 12 * i;
        double* jy = jx + 6;
        for (int j = 0; j < 3; j++) {
            const double dx0 = X * dRdr[9 * j] + Y * dRdr[9 * j + 1] + Z * dRdr[9 * j + 2];
            const double dy0 = X * dRdr[9 * j + 3] + Y * dRdr[9 * j + 4] + Z * dRdr[9 * j + 5];
            const double dz0 = X * dRdr[9 * j + 6] + Y * dRdr[9 * j + 7] + Z * dRdr[9 * j + 8];
            jx[j] = fx * (z * (dx0 - x * dz0));
            jy[j] = fy * (z * (dy0 - y * dz0));
        }
        jx[3] = fx * z; jx[4] = fx * 0.; jx[5] = fx * (-x * z);
        jy[3] = fy * 0.; jy[4] = fy * z; jy[5] = fy * (-y * z);
    }
}

/* CvLevMarq::step: param = prev - solve(JtJ (diag *= 1 + lambda), JtErr) */
static void lm_step(const double JtJ[36], const double JtErr[6], int lambdaLg10, const double prev[6], double param[6])
{
    const double LOG10 = log(10.);
    const double lambda = exp(lambdaLg10 * LOG10);
    double A[36], x[6];
    memcpy(A, JtJ, sizeof(A));
    for (int i = 0; i < 6; i++) A[i * 7] *= 1. + lambda;
    solve_svd(A, 6, 6, JtErr, x);
    for (int i = 0; i < 6; i++) param[i] = prev[i] - x[i];
}

/* cvFindExtrinsicCameraParams2(useExtrinsicGuess = 1): refines rvec / tvec in
 * place over n f64 correspondences; returns the LM iteration count */
int orc_pnp_iterative(const double* op, const double* ip, int n, const double K[9], double rvec[3], double tvec[3])
{
    const int max_iter = 20, nerr = 2 * n;
    const double eps = FLT_EPSILON;
    double param[6], prev[6], JtJ[36], JtErr[6];
    for (int k = 0; k < 3; k++) { param[k] = rvec[k]; param[3 + k] = tvec[k]; }
    double* err = (double*)malloc(sizeof(double) * (size_t)nerr);
    double* J = (double*)malloc(sizeof(double) * 6 * (size_t)nerr);
    double errNorm, prevErrNorm = DBL_MAX;
    int lambdaLg10 = -3, iters = 0;
    project_jac(param, K, op, ip, n, err, J);                /* STARTED */
    for (;;) {
        /* CALC_J */
        mul_at_a(J, nerr, 6, JtJ);
        for (int i = 0; i < 6; i++) {
            double s = 0;
            for (int k = 0; k < nerr; k++) s += J[k * 6 + i] * err[k];
            JtErr[i] = s;
        }
        memcpy(prev, param, sizeof(prev));
        lm_step(JtJ, JtErr, lambdaLg10, prev, param);
        if (iters == 0) prevErrNorm = sqrt(norm_l2sqr(err, nerr));
        /* CHECK_ERR */
        for (;;) {
            project_jac(param, K, op, ip, n, err, NULL);
            errNorm = sqrt(norm_l2sqr(err, nerr));
            if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) {
                lm_step(JtJ, JtErr, lambdaLg10, prev, param);
                continue;
            }
            break;
        }
        lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
        double d[6];
        for (int k = 0; k < 6; k++) d[k] = param[k] - prev[k];
        const double rel = sqrt(norm_l2sqr(d, 6)) / (sqrt(norm_l2sqr(prev, 6)) + DBL_EPSILON);
        if (++iters >= max_iter || rel < eps) break;
        prevErrNorm = errNorm;
        project_jac(param, K, op, ip, n, err, J);            /* CALC_J */
    }
    for (int k = 0; k < 3; k++) { rvec[k] = param[k]; tvec[k] = param[3 + k]; }
    free(err);
    free(J);
    return iters;
}

/* solvePnPRansac(op, ip, K, empty dist, rvec, tvec) with the defaults.
 * Returns 1 (pose found), 0 (RANSAC found no model: rvec / tvec zeroed), -1
 * (n < 4 or n == 4: not supported).  mask (may be NULL) = RANSAC inliers. */
int orc_solve_pnp_ransac(const float* op, const float* ip, int n, const double K[9], int iterationsCount,
                         float reprojectionError, double confidence, double rvec[3], double tvec[3], uint8_t* mask,
                         int* ninliers)
{
    *ninliers = 0;
    if (n < 5) return -1;
    double R[9], t[3];
    if (n == 5) {
        double o[15];
        for (int k = 0; k < 15; k++) o[k] = op[k];
        orc_epnp(5, o, ip, K, R, t);
        orc_rodrigues_m2v(R, rvec);
        memcpy(tvec, t, sizeof(double) * 3);
        if (mask) memset(mask, 1, 5);
        *ninliers = 5;
        return 1;
    }
    const int maxIters = iterationsCount > 1 ? iterationsCount : 1;
    int* sub = (int*)malloc(sizeof(int) * 5 * (size_t)maxIters);
    orc_ep_subsets(n, maxIters, sub);
    const float thr2 = (float)((double)reprojectionError * (double)reprojectionError);
    uint8_t* cur = (uint8_t*)malloc((size_t)n);
    uint8_t* best = (uint8_t*)calloc((size_t)n, 1);
    double bestModel[6] = {0, 0, 0, 0, 0, 0};
    int niters = maxIters, maxGood = 0;
    for (int it = 0; it < niters; it++) {
        double o[15];
        float m[10];
        for (int k = 0; k < 5; k++) {
            const int q = sub[5 * it + k];
            for (int c = 0; c < 3; c++) o[3 * k + c] = op[3 * q + c];
            m[2 * k] = ip[2 * q]; m[2 * k + 1] = ip[2 * q + 1];
        }
        double rv[3], Rp[9];
        orc_epnp(5, o, m, K, R, t);
        orc_rodrigues_m2v(R, rv);
        orc_rodrigues_v2m(rv, Rp, NULL);         /* projectPoints re-derives R from rvec */
        int good = 0;
        for (int i = 0; i < n; i++) {
            cur[i] = orc_pnp_error(Rp, t, K, op + 3 * i, ip + 2 * i) <= thr2;
            good += cur[i];
        }
        if (good > (maxGood > 4 ? maxGood : 4)) {
            uint8_t* sw = cur; cur = best; best = sw;
            for (int k = 0; k < 3; k++) { bestModel[k] = rv[k]; bestModel[3 + k] = t[k]; }
            maxGood = good;
            niters = orc_ransac_update_iters(confidence, (double)(n - good) / n, 5, niters);
        }
    }
    free(sub);
    free(cur);
    if (maxGood <= 0) {
        free(best);
        rvec[0] = rvec[1] = rvec[2] = tvec[0] = tvec[1] = tvec[2] = 0;
        if (mask) memset(mask, 0, (size_t)n);
        return 0;
    }
    double* o = (double*)malloc(sizeof(double) * 3 * (size_t)maxGood);
    double* m = (double*)malloc(sizeof(double) * 2 * (size_t)maxGood);
    int k = 0;
    for (int i = 0; i < n; i++)
        if (best[i]) {
            for (int c = 0; c < 3; c++) o[3 * k + c] = op[3 * i + c];
            m[2 * k] = ip[2 * i]; m[2 * k + 1] = ip[2 * i + 1];
            k++;
        }
    for (int c = 0; c < 3; c++) { rvec[c] = bestModel[c]; tvec[c] = bestModel[3 + c]; }
    orc_pnp_iterative(o, m, k, K, rvec, tvec);
    if (mask) memcpy(mask, best, (size_t)n);
    *ninliers = k;
    free(o); free(m); free(best);
    return 1;
}
