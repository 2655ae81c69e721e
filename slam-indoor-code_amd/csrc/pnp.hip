// solvePnPRansac on gfx950 (FP64), replacing the reference's per-frame pose
// step (src/mainModule/cycleProcessing/mainCycle.cpp:155-161: solvePnPRansac(
// Point3f objects, Point2f image, K, empty distortion, rvec, tvec) with every
// default -- 100 iterations, reprojection error 8, confidence 0.99, EPnP
// minimal sets of 5, SOLVEPNP_ITERATIVE refinement on the inliers).  Same
// restatement as oracle/pnp.c, operation for operation (no contraction), so
// rvec, tvec and the inlier mask agree bit for bit:
//   - RANSAC is speculative, as essential.hip: the host draws all subsets from
//     cv::RNG((uint64)-1) up front (the PnP callback never rejects a subset);
//     pnp_hyp solves every EPnP hypothesis -- one workgroup per hypothesis, the
//     12 x 12 Jacobi SVD of M'M with lane = column in registers and every sum
//     taken in the oracle's order through v_readlane chains, the three beta
//     approximations (6 x 4/3/5 SVD, Gauss-Newton, 3 x 3 SVDs) side by side on
//     lane 0 of three waves -- and the
//     orthonormalisation U Vt that cv::Rodrigues applies; the host finishes
//     Rodrigues (acos / cos / sin stay in glibc, as the oracle's) and
//     pnp_score counts every model's inliers (f32 error <= 64, one workgroup
//     per hypothesis); the host replays the sequential accept /
//     RANSACUpdateNumIters loop on the counts;
//   - the refinement (cvFindExtrinsicCameraParams2 + CvLevMarq) runs its state
//     machine on the host; each evaluation is pnp_eval (one thread per inlier:
//     residuals and the 2 x 6 Jacobian rows) + pnp_reduce (J'J, J'e and |e|^2 as
//     sequential sums, one lane each, in the oracle's order).
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "jacobi.h"
#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kHyp = 24;        // per hypothesis: R (9), U Vt of R (9), t (3), pad

// ---- small dense algebra, oracle/pnp.c order ----
template <int n, int m>
HD void jsvd_u(double* At, double* W, double* Vt)
{
    jsvd<n, m>(At, W, Vt);
    for (int i = 0; i < n; i++) {
        const double s = W[i] > DBL_MIN ? 1 / W[i] : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

// cv::solve(A (m x n), b, x, DECOMP_SVD)
template <int m, int n>
HD void solve_svd(const double* A, const double* b, double* x)
{
    double At[n * m], W[n], Vt[n * n];
    for (int r = 0; r < m; r++)
        for (int c = 0; c < n; c++) At[c * m + r] = A[r * n + c];
    jsvd_u<n, m>(At, W, Vt);
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

// cv::invert(3 x 3, DECOMP_SVD)
__device__ void invert_svd3(const double* A, double* X)
{
    double At[9], W[3], Vt[9], buf[3];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = A[r * 3 + c];
    jsvd_u<3, 3>(At, W, Vt);
    double thr = 0;
    for (int i = 0; i < 3; i++) thr += W[i];
    thr *= DBL_EPSILON * 2;
    for (int k = 0; k < 9; k++) X[k] = 0;
    for (int i = 0; i < 3; i++) {
        double wi = W[i];
        if (fabs(wi) <= thr) continue;
        wi = 1 / wi;
        for (int j = 0; j < 3; j++) buf[j] = At[i * 3 + j] * wi;
        for (int r = 0; r < 3; r++) {
            const double s = Vt[i * 3 + r];
            for (int j = 0; j < 3; j++) X[r * 3 + j] = X[r * 3 + j] + s * buf[j];
        }
    }
}

HD inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
HD inline double dist2(const double* a, const double* b)
{
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

// PnPRansacCallback::computeError for one point
HD inline float pnp_err(const double* R, const double* t, double fx, double fy, double cx, double cy,
                        const float* o, const float* m)
{
    const double X = o[0], Y = o[1], Z = o[2];
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z; y *= z;
    const float px = (float)(x * fx + cx), py = (float)(y * fy + cy);
    const float dx = m[0] - px, dy = m[1] - py;
    float s = 0;
    s += dx * dx;
    s += dy * dy;
    return s;
}

// ---- EPnP hypothesis kernel ----
__device__ inline double rl(double x, int k)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), k);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), k);
    return __hiloint2double(hi, lo);
}

// JacobiSVDImpl_ on the 12 x 12 At with lane i holding ROW i (x[k] = At[i][k]) and
// W[i] on its own lane.  A sweep's 66 rotations (i, j), i < j, in the cyclic
// order, grouped into dependency levels: rotation (i, j) reads and writes only
// rows i and j and W[i], W[j], so it depends only on the last earlier rotation
// on i and the last on j.  A level's rotations touch disjoint rows and follow
// every earlier rotation on their rows: run side by side -- lanes i and j each
// take the other's row (one shuffle per element), form the same p, c, s (the
// products x[k] y[k] commute) and their own new row and norm, summed over k in
// the oracle's order -- they give the sequential loop's values bit for bit, in
// 21 dependent steps per sweep instead of 66.  Only U is produced (pnp_hyp
// reads no V).  Lanes >= 12 idle.
struct JLevels {
    int8_t part[21][12];    // partner of row r at level L, -1 = idle
};
constexpr JLevels make_jlevels()
{
    JLevels t{};
    for (int L = 0; L < 21; L++)
        for (int r = 0; r < 12; r++) t.part[L][r] = -1;
    int last[12] = {};
    for (int i = 0; i < 11; i++)
        for (int j = i + 1; j < 12; j++) {
            const int l = (last[i] > last[j] ? last[i] : last[j]) + 1;
            last[i] = last[j] = l;
            t.part[l - 1][i] = (int8_t)j;
            t.part[l - 1][j] = (int8_t)i;
        }
    return t;
}
__constant__ JLevels c_jlev = make_jlevels();

__device__ inline double shfl_d(double x, int src)
{
    return __hiloint2double(__shfl(__double2hiint(x), src, 64), __shfl(__double2loint(x), src, 64));
}

// x: this lane's row of At in, its row of U' (normalised, sorted by singular
// value as JacobiSVDImpl_ leaves them) out
__device__ void wave_jsvd12_rows(double (&x)[12], int lane)
{
    const double eps = DBL_EPSILON * 10;
    const int me = lane < 12 ? lane : 0;
    double w = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) w += x[k] * x[k];
    for (int iter = 0; iter < 30; iter++) {
        bool changed = false;
        for (int L = 0; L < 21; L++) {
            const int pt = lane < 12 ? c_jlev.part[L][me] : -1;
            const int src = pt >= 0 ? pt : lane;
            double y[12];
#pragma unroll
            for (int k = 0; k < 12; k++) y[k] = shfl_d(x[k], src);
            const double wy = shfl_d(w, src);
            const bool first = lane < pt;
            double p = 0;
#pragma unroll
            for (int k = 0; k < 12; k++) p += x[k] * y[k];
            const double aa = first ? w : wy, bb = first ? wy : w;
            const bool rot = pt >= 0 && !(fabs(p) <= eps * sqrt(aa * bb));
            p *= 2;
            const double beta = aa - bb, gamma = ep_hypot(p, beta);
            double c, sn;
            if (beta < 0) {
                const double delta = (gamma - beta) * 0.5;
                sn = sqrt(delta / gamma);
                c = p / (gamma * sn * 2);
            } else {
                c = sqrt((gamma + beta) / (gamma * 2));
                sn = p / (gamma * c * 2);
            }
            double t[12];
            double wn = 0;
#pragma unroll
            for (int k = 0; k < 12; k++) {
                // row i: c a_i + s a_j; row j: -s a_i + c a_j
                t[k] = first ? c * x[k] + sn * y[k] : -sn * y[k] + c * x[k];
                wn += t[k] * t[k];
            }
            if (rot) {
#pragma unroll
                for (int k = 0; k < 12; k++) x[k] = t[k];
                w = wn;
            }
            changed |= __ballot(rot) != 0;
        }
        if (!changed) break;
    }
    // singular values, JacobiSVDImpl_'s selection sort (descending, first max),
    // then U' = At rows / W
    double sv = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) sv += x[k] * x[k];
    sv = sqrt(sv);
    double Wu[12];
    int idx[12];
#pragma unroll
    for (int q = 0; q < 12; q++) { Wu[q] = rl(sv, q); idx[q] = q; }
#pragma unroll
    for (int i = 0; i < 11; i++) {
        int j = i;
        double wj = Wu[i];
#pragma unroll
        for (int k = i + 1; k < 12; k++)
            if (wj < Wu[k]) { j = k; wj = Wu[k]; }
        if (j != i) {
            const double wi = Wu[i];
            const int ii = idx[i];
            int ij = ii;
#pragma unroll
            for (int r = i + 1; r < 12; r++)
                if (r == j) { ij = idx[r]; Wu[r] = wi; idx[r] = ii; }
            Wu[i] = wj; idx[i] = ij;
        }
    }
    int from = 0;
    double mine = 0;
#pragma unroll
    for (int q = 0; q < 12; q++)
        if (q == me) { from = idx[q]; mine = Wu[q]; }
#pragma unroll
    for (int k = 0; k < 12; k++) x[k] = shfl_d(x[k], from);
    const double sc = mine > DBL_MIN ? 1 / mine : 0.;
#pragma unroll
    for (int k = 0; k < 12; k++) x[k] *= sc;
}

struct HypParams {
    const float* op;        // n x 3
    const float* ip;        // n x 2
    const int* subsets;     // iters x 5
    double fx, fy, cx, cy;
    double* out;            // iters x kHyp
};

struct Epnp5 {
    double pws[15], us[10], alphas[20], pcs[15], cws[4][3], ccs[4][3];
    double fu, fv, uc, vc;
};

__device__ void compute_L_6x10(const double* ut, double* l)
{
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        int a = 0, b = 1;
        for (int j = 0; j < 6; j++) {
            dv[i][j][0] = v[3 * a] - v[3 * b];
            dv[i][j][1] = v[3 * a + 1] - v[3 * b + 1];
            dv[i][j][2] = v[3 * a + 2] - v[3 * b + 2];
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

__device__ void qr_solve(double* A, double* b, double* X)
{
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; k++) {
        double eta = fabs(A[k * nc + k]);
        for (int i = k + 1; i < nr; i++) {
            const double elt = fabs(A[i * nc + k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;
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

__device__ void gauss_newton(const double* L, const double* rho, double* betas)
{
    double A[24], b[6], x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
        for (int i = 0; i < 6; i++) {
            const double* rl_ = L + i * 10;
            double* ra = A + i * 4;
            ra[0] = 2 * rl_[0] * betas[0] + rl_[1] * betas[1] + rl_[3] * betas[2] + rl_[6] * betas[3];
            ra[1] = rl_[1] * betas[0] + 2 * rl_[2] * betas[1] + rl_[4] * betas[2] + rl_[7] * betas[3];
            ra[2] = rl_[3] * betas[0] + rl_[4] * betas[1] + 2 * rl_[5] * betas[2] + rl_[8] * betas[3];
            ra[3] = rl_[6] * betas[0] + rl_[7] * betas[1] + rl_[8] * betas[2] + 2 * rl_[9] * betas[3];
            b[i] = rho[i] - (rl_[0] * betas[0] * betas[0] + rl_[1] * betas[0] * betas[1] +
                             rl_[2] * betas[1] * betas[1] + rl_[3] * betas[0] * betas[2] +
                             rl_[4] * betas[1] * betas[2] + rl_[5] * betas[2] * betas[2] +
                             rl_[6] * betas[0] * betas[3] + rl_[7] * betas[1] * betas[3] +
                             rl_[8] * betas[2] * betas[3] + rl_[9] * betas[3] * betas[3]);
        }
        qr_solve(A, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

__device__ double compute_R_and_t(Epnp5& e, const double* ut, const double* betas, double* R, double* t)
{
    for (int i = 0; i < 4; i++) e.ccs[i][0] = e.ccs[i][1] = e.ccs[i][2] = 0.0;
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) e.ccs[j][k] += betas[i] * v[3 * j + k];
    }
    for (int i = 0; i < 5; i++) {
        const double* a = e.alphas + 4 * i;
        for (int j = 0; j < 3; j++)
            e.pcs[3 * i + j] = a[0] * e.ccs[0][j] + a[1] * e.ccs[1][j] + a[2] * e.ccs[2][j] + a[3] * e.ccs[3][j];
    }
    if (e.pcs[2] < 0.0) {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) e.ccs[i][j] = -e.ccs[i][j];
        for (int i = 0; i < 15; i++) e.pcs[i] = -e.pcs[i];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 3; j++) { pc0[j] += e.pcs[3 * i + j]; pw0[j] += e.pws[3 * i + j]; }
    for (int j = 0; j < 3; j++) { pc0[j] /= 5; pw0[j] /= 5; }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 5; i++) {
        const double* pc = e.pcs + 3 * i;
        const double* pw = e.pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    double At[9], W[3], Vt[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = abt[r * 3 + c];
    jsvd_u<3, 3>(At, W, Vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[3 * i + j] = At[i] * Vt[j] + At[3 + i] * Vt[3 + j] + At[6 + i] * Vt[6 + j];
    const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                       R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
    if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
    t[0] = pc0[0] - dot3(R, pw0);
    t[1] = pc0[1] - dot3(R + 3, pw0);
    t[2] = pc0[2] - dot3(R + 6, pw0);
    double sum2 = 0.0;
    for (int i = 0; i < 5; i++) {
        const double* pw = e.pws + 3 * i;
        const double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1];
        const double inv_Zc = 1.0 / (dot3(R + 6, pw) + t[2]);
        const double ue = e.uc + e.fu * Xc * inv_Zc, ve = e.vc + e.fv * Yc * inv_Zc;
        const double u = e.us[2 * i], v = e.us[2 * i + 1];
        sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / 5;
}

// A hypothesis is one workgroup of four waves: wave 0 builds M, M'M and its
// 12 x 12 SVD (lane = column) and L / rho; then waves 1..3 each run one of
// EPnP's three independent beta approximations (its SVD solve, Gauss-Newton
// and R, t, reprojection error) on their lane 0 at the same time -- on one
// lane they were three serial chains -- and wave 0 picks the oracle's choice.
__global__ __launch_bounds__(256) void pnp_hyp(HypParams p)
{
    __shared__ double s_M[120], s_mtm[144], s_ut[144];
    __shared__ double s_L[60], s_rho[6], s_R[4][9], s_t[4][3], s_rep[4];
    __shared__ Epnp5 s_e;
    const int it = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Epnp5& e = s_e;
    if (threadIdx.x == 0) {
        e.fu = p.fx; e.fv = p.fy; e.uc = p.cx; e.vc = p.cy;
        const double ifx = 1. / p.fx, ify = 1. / p.fy;
        for (int k = 0; k < 5; k++) {
            const int q = p.subsets[5 * it + k];
            for (int c = 0; c < 3; c++) e.pws[3 * k + c] = p.op[3 * q + c];
            const float xn = (float)(((double)p.ip[2 * q] - p.cx) * ifx);
            const float yn = (float)(((double)p.ip[2 * q + 1] - p.cy) * ify);
            e.us[2 * k] = xn * p.fx + p.cx;
            e.us[2 * k + 1] = yn * p.fy + p.cy;
        }
        // choose_control_points
        e.cws[0][0] = e.cws[0][1] = e.cws[0][2] = 0;
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 3; j++) e.cws[0][j] += e.pws[3 * i + j];
        for (int j = 0; j < 3; j++) e.cws[0][j] /= 5;
        double PW0[15], ptp[9], At[9], dc[3], Vt[9];
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 3; j++) PW0[3 * i + j] = e.pws[3 * i + j] - e.cws[0][j];
        for (int i = 0; i < 3; i++)
            for (int j = i; j < 3; j++) {
                double s = 0;
                for (int k = 0; k < 5; k++) s += PW0[k * 3 + i] * PW0[k * 3 + j];
                ptp[i * 3 + j] = s;
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < i; j++) ptp[i * 3 + j] = ptp[j * 3 + i];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) At[c * 3 + r] = ptp[r * 3 + c];
        jsvd_u<3, 3>(At, dc, Vt);
        for (int i = 1; i < 4; i++) {
            const double k = sqrt(dc[i - 1] / 5);
            for (int j = 0; j < 3; j++) e.cws[i][j] = e.cws[0][j] + k * At[3 * (i - 1) + j];
        }
        // compute_barycentric_coordinates
        double cc[9], ci[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = e.cws[j][i] - e.cws[0][i];
        invert_svd3(cc, ci);
        for (int i = 0; i < 5; i++) {
            const double* pi = e.pws + 3 * i;
            double* a = e.alphas + 4 * i;
            for (int j = 0; j < 3; j++)
                a[1 + j] = ci[3 * j] * (pi[0] - e.cws[0][0]) + ci[3 * j + 1] * (pi[1] - e.cws[0][1]) +
                           ci[3 * j + 2] * (pi[2] - e.cws[0][2]);
            a[0] = 1.0 - a[1] - a[2] - a[3];
        }
        // fill_M
        for (int i = 0; i < 5; i++) {
            const double* as = e.alphas + 4 * i;
            const double u = e.us[2 * i], v = e.us[2 * i + 1];
            double* M1 = s_M + 24 * i;
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
    }
    __syncthreads();
    // M'M: 78 upper entries, one thread each, sums over the 10 rows in order
    for (int q = threadIdx.x; q < 78; q += 256) {
        int i = 0, r = q;
        while (r >= 12 - i) { r -= 12 - i; i++; }
        const int j = i + r;
        double s = 0;
        for (int k = 0; k < 10; k++) s += s_M[k * 12 + i] * s_M[k * 12 + j];
        s_mtm[i * 12 + j] = s;
        s_mtm[j * 12 + i] = s;
    }
    __syncthreads();
    if (wave == 0) {
        // At = (M'M)' = M'M (symmetric): lane i takes row i
        double x[12];
        const int kc = lane < 12 ? lane : 0;
#pragma unroll
        for (int k = 0; k < 12; k++) x[k] = s_mtm[kc * 12 + k];
        wave_jsvd12_rows(x, lane);
        if (lane < 12)
#pragma unroll
            for (int k = 0; k < 12; k++) s_ut[lane * 12 + k] = x[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        compute_L_6x10(s_ut, s_L);
        s_rho[0] = dist2(e.cws[0], e.cws[1]);
        s_rho[1] = dist2(e.cws[0], e.cws[2]);
        s_rho[2] = dist2(e.cws[0], e.cws[3]);
        s_rho[3] = dist2(e.cws[1], e.cws[2]);
        s_rho[4] = dist2(e.cws[1], e.cws[3]);
        s_rho[5] = dist2(e.cws[2], e.cws[3]);
    }
    __syncthreads();
    if (lane == 0 && wave > 0) {
        // compute_R_and_t writes the camera-frame points into its Epnp5: each
        // approximation works on its own copy
        Epnp5 el = s_e;
        double L[60], rho[6], betas[4];
        for (int k = 0; k < 60; k++) L[k] = s_L[k];
        for (int k = 0; k < 6; k++) rho[k] = s_rho[k];
        if (wave == 1) {   // find_betas_approx_1
        double l[24], b4[4];
        for (int i = 0; i < 6; i++) {
            l[4 * i] = L[10 * i]; l[4 * i + 1] = L[10 * i + 1]; l[4 * i + 2] = L[10 * i + 3]; l[4 * i + 3] = L[10 * i + 6];
        }
        solve_svd<6, 4>(l, rho, b4);
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
        gauss_newton(L, rho, betas);
        s_rep[1] = compute_R_and_t(el, s_ut, betas, s_R[1], s_t[1]);
        } else if (wave == 2) {   // find_betas_approx_2
        double l[18], b3[3];
        for (int i = 0; i < 6; i++) { l[3 * i] = L[10 * i]; l[3 * i + 1] = L[10 * i + 1]; l[3 * i + 2] = L[10 * i + 2]; }
        solve_svd<6, 3>(l, rho, b3);
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
        gauss_newton(L, rho, betas);
        s_rep[2] = compute_R_and_t(el, s_ut, betas, s_R[2], s_t[2]);
        } else {   // find_betas_approx_3
        double l[30], b5[5];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < 5; k++) l[5 * i + k] = L[10 * i + k];
        solve_svd<6, 5>(l, rho, b5);
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
        gauss_newton(L, rho, betas);
        s_rep[3] = compute_R_and_t(el, s_ut, betas, s_R[3], s_t[3]);
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    int N = 1;
    if (s_rep[2] < s_rep[1]) N = 2;
    if (s_rep[3] < s_rep[N]) N = 3;
    double* o = p.out + (size_t)it * kHyp;
    const double* R = s_R[N];
    for (int k = 0; k < 9; k++) o[k] = R[k];
    for (int k = 0; k < 3; k++) o[18 + k] = s_t[N][k];
    // cv::Rodrigues' orthonormalisation R' = U Vt (the host applies checkRange)
    double At[9], W[3], Vt[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = R[r * 3 + c];
    jsvd_u<3, 3>(At, W, Vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += At[k * 3 + i] * Vt[k * 3 + j];
            o[9 + i * 3 + j] = s;
        }
}

// ---- scoring ----
struct ScoreParams {
    const float* op;
    const float* ip;
    int n;
    const double* models;   // iters x 12: R (9), t (3)
    double fx, fy, cx, cy;
    float thr2;
    int* counts;
};

__global__ __launch_bounds__(256) void pnp_score(ScoreParams p)
{
    __shared__ double m[12];
    __shared__ int red[4];
    const int it = blockIdx.x, tid = threadIdx.x;
    if (tid < 12) m[tid] = p.models[(size_t)it * 12 + tid];
    __syncthreads();
    int c = 0;
    for (int i = tid; i < p.n; i += 256)
        c += pnp_err(m, m + 9, p.fx, p.fy, p.cx, p.cy, p.op + 3 * i, p.ip + 2 * i) <= p.thr2;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) p.counts[it] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void pnp_mask(ScoreParams p, const double* model, uint8_t* mask)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p.n) return;
    mask[i] = pnp_err(model, model + 9, p.fx, p.fy, p.cx, p.cy, p.op + 3 * i, p.ip + 2 * i) <= p.thr2;
}

// ---- refinement: residuals / Jacobian and the ordered reductions ----
// up to kSpec candidate parameter vectors per launch (blockIdx.y): the LM's
// next damping values are evaluated together, each with its Jacobian, so an
// accepted step needs no second pass (one host sync per LM iteration)
constexpr int kSpec = 3;
struct EvalParams {
    double R[kSpec][9], dRdr[kSpec][27], t[kSpec][3];
    double fx, fy, cx, cy;
    const float* op;
    const float* ip;
    const int* idx;         // inlier indices, ascending
    int m;
    int withJ;
    double* err;            // [candidate] m x 2
    double* J;              // [candidate] m x 12 (rows 2k, 2k + 1 of the 2m x 6 Jacobian)
    size_t err_stride, J_stride;
};

// inlier k of candidate c: its residual (ex, ey) and, with J, its two Jacobian
// rows -- cvProjectPoints2's arithmetic as oracle/pnp.c states it
template <bool J>
__device__ __forceinline__ void pnp_row(const EvalParams& p, int c, int k, double& ex, double& ey, double* jx,
                                        double* jy)
{
    const double* R = p.R[c];
    const double* dRdr = p.dRdr[c];
    const double* t = p.t[c];
    const int i = p.idx[k];
    const double X = p.op[3 * i], Y = p.op[3 * i + 1], Z = p.op[3 * i + 2];
    const double u = p.ip[2 * i], v = p.ip[2 * i + 1];
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z; y *= z;
    ex = (x * p.fx + p.cx) - u;
    ey = (y * p.fy + p.cy) - v;
    if (!J) return;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const double dx0 = X * dRdr[9 * j] + Y * dRdr[9 * j + 1] + Z * dRdr[9 * j + 2];
        const double dy0 = X * dRdr[9 * j + 3] + Y * dRdr[9 * j + 4] + Z * dRdr[9 * j + 5];
        const double dz0 = X * dRdr[9 * j + 6] + Y * dRdr[9 * j + 7] + Z * dRdr[9 * j + 8];
        jx[j] = p.fx * (z * (dx0 - x * dz0));
        jy[j] = p.fy * (z * (dy0 - y * dz0));
    }
    jx[3] = p.fx * z; jx[4] = p.fx * 0.; jx[5] = p.fx * (-x * z);
    jy[3] = p.fy * 0.; jy[4] = p.fy * z; jy[5] = p.fy * (-y * z);
}

__global__ __launch_bounds__(256) void pnp_eval(EvalParams p)
{
    const int k = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y;
    if (k >= p.m) return;
    double* err = p.err + c * p.err_stride;
    double ex, ey, jx[6], jy[6];
    if (!p.withJ) {
        pnp_row<false>(p, c, k, ex, ey, jx, jy);
    } else {
        pnp_row<true>(p, c, k, ex, ey, jx, jy);
        double* dj = p.J + c * p.J_stride + 12 * (size_t)k;
#pragma unroll
        for (int q = 0; q < 6; q++) { dj[q] = jx[q]; dj[6 + q] = jy[q]; }
    }
    err[2 * k] = ex;
    err[2 * k + 1] = ey;
}

// SLAM_PNP_SUMS_PAIRWISE: residuals, Jacobian rows and the 28 sums of one
// candidate in one workgroup (blockIdx.x = candidate).  Each thread sums its
// strided rows, then a fixed shuffle tree and the four waves in order: the
// same result every run, not the oracle's sequential order (~1e-16 relative
// per sum).  The sequential chain of 2 m dependent f64 adds per sum is what
// pnp_reduce's time is (89 us at m = 1750); this is a few microseconds.
__global__ __launch_bounds__(256) void pnp_eval_sums(EvalParams p, double* out)
{
    const int c = blockIdx.x, t = threadIdx.x;
    double acc[28];
#pragma unroll
    for (int q = 0; q < 28; q++) acc[q] = 0.;
    for (int k = t; k < p.m; k += 256) {
        double ex, ey, jx[6], jy[6];
        pnp_row<true>(p, c, k, ex, ey, jx, jy);
        int u = 0;
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int j = i; j < 6; j++, u++) {
                acc[u] += jx[i] * jx[j];
                acc[u] += jy[i] * jy[j];
            }
#pragma unroll
        for (int i = 0; i < 6; i++) {
            acc[21 + i] += jx[i] * ex;
            acc[21 + i] += jy[i] * ey;
        }
        acc[27] += ex * ex;
        acc[27] += ey * ey;
    }
    __shared__ double part[4][28];
#pragma unroll
    for (int q = 0; q < 28; q++) {
        double v = acc[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[q] = v;
    }
    if ((t & 63) == 0)
#pragma unroll
        for (int q = 0; q < 28; q++) part[t >> 6][q] = acc[q];
    __syncthreads();
    if (t < 28) out[28 * c + t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
}

// out[0..20]: J'J upper entries, [21..26]: J'e (lanes 0..26 of wave 0), [27]:
// |e|^2 (normL2Sqr's 4-wide blocks; lane 0 of wave 1).  Each output is one sequential sum in the oracle's order, so the
// kernel time is the dependent f64 add chain (2 adds per point) plus whatever
// load latency is left exposed.  Wave 0 holds the 28 summing lanes; waves 1..3
// stream the next chunk of J rows and residuals into the other half of a
// double buffer while wave 0 walks the current one (one barrier per chunk), so
// only the first chunk's load is on the critical path.  The |e|^2 chain sits in
// wave 1 so that it does not serialise behind wave 0's divergent branch.
constexpr int kRedRows = 256;
constexpr int kRedThreads = 256;
__device__ __forceinline__ void pnp_red_load(const double* J, const double* err, int k0, int rows, int withJ,
                                             double* sJ, double* sE, int t, int nt)
{
    // 16-byte copies: J chunk (rows x 12 doubles) and residuals (rows x 2)
    if (withJ) {
        const double2* src = reinterpret_cast<const double2*>(J + 12 * (size_t)k0);
        double2* dst = reinterpret_cast<double2*>(sJ);
        for (int q = t; q < rows * 6; q += nt) dst[q] = src[q];
    }
    const double2* se = reinterpret_cast<const double2*>(err + 2 * (size_t)k0);
    double2* de = reinterpret_cast<double2*>(sE);
    for (int q = t; q < rows; q += nt) de[q] = se[q];
}

__global__ __launch_bounds__(kRedThreads) void pnp_reduce(const double* J, const double* err, int m, int withJ,
                                                          double* out, size_t err_stride, size_t J_stride)
{
    // one workgroup per candidate (blockIdx.x): its own residuals / Jacobian / sums
    J += blockIdx.x * J_stride;
    err += blockIdx.x * err_stride;
    out += 28 * blockIdx.x;
    __shared__ __attribute__((aligned(16))) double sJ[2][kRedRows * 12];
    __shared__ __attribute__((aligned(16))) double sE[2][kRedRows * 2];
    const int tid = threadIdx.x;
    int i = 0, j = 0, kind = 0;                       // kind 1: J'J (i, j), 2: J'e (i), 3: |e|^2
    if (tid < 21 && withJ) {
        int r = tid;
        while (r >= 6 - i) { r -= 6 - i; i++; }
        j = i + r;
        kind = 1;
    } else if (tid >= 21 && tid < 27 && withJ) {
        i = tid - 21;
        kind = 2;
    } else if (tid == 64) {
        kind = 3;                                     // in wave 1: its chain runs beside wave 0's
    }
    double s = 0;
    const int nch = (m + kRedRows - 1) / kRedRows;
    if (nch > 0) pnp_red_load(J, err, 0, min(kRedRows, m), withJ, sJ[0], sE[0], tid, kRedThreads);
    __syncthreads();
    for (int c = 0; c < nch; c++) {
        const int buf = c & 1, k0 = c * kRedRows;
        const int rows = min(kRedRows, m - k0);
        if (tid >= 64) {
            // waves 1..3: the next chunk into the other buffer (last read by wave 0
            // before the previous barrier)
            if (c + 1 < nch)
                pnp_red_load(J, err, k0 + kRedRows, min(kRedRows, m - k0 - kRedRows), withJ, sJ[buf ^ 1],
                             sE[buf ^ 1], tid - 64, kRedThreads - 64);
            if (kind == 3) {
                // normL2Sqr over the 2m residuals in blocks of 4 (+ a tail): full chunks
                // hold 2 * kRedRows residuals, a multiple of 4, so the blocks align
                const double* cE = sE[buf];
                const int n = 2 * rows;
                int q = 0;
                for (; q <= n - 4; q += 4)
                    s += cE[q] * cE[q] + cE[q + 1] * cE[q + 1] + cE[q + 2] * cE[q + 2] + cE[q + 3] * cE[q + 3];
                for (; q < n; q++) s += cE[q] * cE[q];
            }
        } else if (kind == 1 || kind == 2) {
            // the products do not depend on s: 8 rows' operands are read ahead, then
            // added in order (the LDS latency leaves the dependent add chain)
            const double* cJ = sJ[buf];
            const double* cE = sE[buf];
            const int ja = kind == 1 ? j : 12, jb = kind == 1 ? 6 + j : 13;   // 12 / 13: the residuals
            // software-pipelined: group g + 1's operands and products are formed
            // while group g is added, so the LDS latency leaves the add chain
            auto prod = [&](int k, double* p0, double* p1) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const double* row = cJ + 12 * (k + u);
                    const double ea = kind == 1 ? row[ja] : cE[2 * (k + u)];
                    const double eb = kind == 1 ? row[jb] : cE[2 * (k + u) + 1];
                    p0[u] = row[i] * ea;
                    p1[u] = row[6 + i] * eb;
                }
            };
            const int full = rows & ~7;
            int k = 0;
            if (full > 0) {
                double a0[8], a1[8], b0[8], b1[8];
                prod(0, a0, a1);
                for (; k + 16 <= full; k += 16) {
                    prod(k + 8, b0, b1);
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        s += a0[u];
                        s += a1[u];
                    }
                    if (k + 16 < full) prod(k + 16, a0, a1);
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        s += b0[u];
                        s += b1[u];
                    }
                }
                if (k < full) {          // one group left (already formed in a)
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        s += a0[u];
                        s += a1[u];
                    }
                    k += 8;
                }
            }
            for (; k < rows; k++) {
                const double* row = cJ + 12 * k;
                const double ea = kind == 1 ? row[ja] : cE[2 * k];
                const double eb = kind == 1 ? row[jb] : cE[2 * k + 1];
                s += row[i] * ea;
                s += row[6 + i] * eb;
            }
        }
        __syncthreads();
    }
    if (kind == 1 || kind == 2) out[tid] = s;
    else if (kind == 3) out[27] = s;
}

// ---- host: Rodrigues (cvRodrigues2) and the LM step, as oracle/pnp.c ----
void rodrigues_v2m(const double* rv, double* R, double* J)
{
    double rx = rv[0], ry = rv[1], rz = rv[2];
    const double theta = std::sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1 : 0;
        if (J) {
            std::memset(J, 0, 27 * sizeof(double));
            J[5] = J[15] = J[19] = -1;
            J[7] = J[11] = J[21] = 1;
        }
        return;
    }
    // glibc sincos: GCC turns OpenCV's cos(theta) / sin(theta) pair into one
    // sincos call (as it does for oracle/pnp.c); its results can differ from
    // separate cos / sin calls in the last bit
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

// cvRodrigues2 matrix -> vector given R (for checkRange) and R' = U Vt (device)
void rodrigues_m2v(const double* Rin, const double* R, double* rv)
{
    for (int k = 0; k < 9; k++)
        if (!(Rin[k] >= -100 && Rin[k] < 100)) { rv[0] = rv[1] = rv[2] = 0; return; }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = std::sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    rv[0] = rx; rv[1] = ry; rv[2] = rz;
}

void lm_step(const double* JtJ, const double* JtErr, int lambdaLg10, const double* prev, double* param)
{
    const double LOG10 = std::log(10.);
    const double lambda = std::exp(lambdaLg10 * LOG10);
    double A[36], x[6];
    std::memcpy(A, JtJ, sizeof(A));
    for (int i = 0; i < 6; i++) A[i * 7] *= 1. + lambda;
    solve_svd<6, 6>(A, JtErr, x);
    for (int i = 0; i < 6; i++) param[i] = prev[i] - x[i];
}

double norm_l2sqr(const double* a, int n)
{
    double s = 0;
    int i = 0;
    for (; i <= n - 4; i += 4) s += a[i] * a[i] + a[i + 1] * a[i + 1] + a[i + 2] * a[i + 2] + a[i + 3] * a[i + 3];
    for (; i < n; i++) s += a[i] * a[i];
    return s;
}

}  // namespace

int pnp_ransac(slam_ctx* c, const float* op, const float* ip, int n, const double* K, int iterations, float reproj,
               double confidence, double* rvec, double* tvec, uint8_t* mask, int* ninliers, int* found)
{
    *found = 0;
    *ninliers = 0;
    // diagnostics: SLAMHIP_PNP_TIMING=1 prints per call the points, inliers, LM
    // iterations / evaluations and the host-clock phases (RANSAC, LM) to stderr
    static const bool timing = [] { const char* e = getenv("SLAMHIP_PNP_TIMING"); return e && e[0] == '1'; }();
    const auto t_start = std::chrono::steady_clock::now();
    int n_evals = 0;
    if (n < 4) return SLAM_E_INVALID_ARG;           // solvePnPRansac asserts npoints >= 4
    if (n == 4) return SLAM_E_UNSUPPORTED;          // OpenCV switches to P3P there
    if (!(confidence > 0 && confidence < 1)) return SLAM_E_INVALID_ARG;
    hipStream_t s = c->stream;
    const int maxIters = iterations > 1 ? iterations : 1;
    const int iters = n == 5 ? 1 : maxIters;
    std::vector<int> sub((size_t)5 * iters);
    if (n == 5) for (int k = 0; k < 5; k++) sub[k] = k;
    else ransac_subsets5(n, iters, sub.data());
    size_t off = 0;
    auto carve = [&](size_t b) { const size_t o = off; off += (b + 255) & ~(size_t)255; return o; };
    const size_t o_op = carve(sizeof(float) * 3 * (size_t)n), o_ip = carve(sizeof(float) * 2 * (size_t)n),
                 o_sub = carve(sizeof(int) * 5 * (size_t)iters), o_hyp = carve(sizeof(double) * kHyp * iters),
                 o_mod = carve(sizeof(double) * 12 * (size_t)iters), o_cnt = carve(sizeof(int) * (size_t)iters),
                 o_mask = carve((size_t)n), o_idx = carve(sizeof(int) * (size_t)n),
                 o_err = carve(sizeof(double) * 2 * (size_t)n * kSpec), o_J = carve(sizeof(double) * 12 * (size_t)n * kSpec),
                 o_red = carve(sizeof(double) * 28 * kSpec);
    SLAM_HIP(c, c->geom.ensure(off));
    char* base = c->geom.as<char>();
    float* dop = reinterpret_cast<float*>(base + o_op);
    float* dip = reinterpret_cast<float*>(base + o_ip);
    SLAM_HIP(c, hipMemcpyAsync(dop, op, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(dip, ip, sizeof(float) * 2 * (size_t)n, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_sub, sub.data(), sizeof(int) * 5 * (size_t)iters, hipMemcpyHostToDevice, s));
    HypParams hp;
    hp.op = dop; hp.ip = dip;
    hp.subsets = reinterpret_cast<const int*>(base + o_sub);
    hp.fx = K[0]; hp.fy = K[4]; hp.cx = K[2]; hp.cy = K[5];
    hp.out = reinterpret_cast<double*>(base + o_hyp);
    hipLaunchKernelGGL(pnp_hyp, dim3(iters), dim3(256), 0, s, hp);
    SLAM_HIP(c, hipGetLastError());
    std::vector<double> hyp((size_t)kHyp * iters);
    SLAM_HIP(c, hipMemcpyAsync(hyp.data(), hp.out, sizeof(double) * kHyp * iters, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    // models [rvec | tvec] and the rotation projectPoints re-derives from rvec
    std::vector<double> rt((size_t)6 * iters), models((size_t)12 * iters);
    for (int it = 0; it < iters; it++) {
        const double* h = hyp.data() + (size_t)it * kHyp;
        double* m = rt.data() + 6 * (size_t)it;
        rodrigues_m2v(h, h + 9, m);
        for (int k = 0; k < 3; k++) m[3 + k] = h[18 + k];
        rodrigues_v2m(m, models.data() + 12 * (size_t)it, nullptr);
        for (int k = 0; k < 3; k++) models[12 * (size_t)it + 9 + k] = m[3 + k];
    }
    if (n == 5) {
        for (int k = 0; k < 3; k++) { rvec[k] = rt[k]; tvec[k] = rt[3 + k]; }
        if (mask) std::memset(mask, 1, 5);
        *ninliers = 5;
        *found = 1;
        return SLAM_OK;
    }
    ScoreParams sp;
    sp.op = dop; sp.ip = dip; sp.n = n;
    sp.models = reinterpret_cast<const double*>(base + o_mod);
    sp.fx = K[0]; sp.fy = K[4]; sp.cx = K[2]; sp.cy = K[5];
    sp.thr2 = (float)((double)reproj * (double)reproj);
    sp.counts = reinterpret_cast<int*>(base + o_cnt);
    SLAM_HIP(c, hipMemcpyAsync(base + o_mod, models.data(), sizeof(double) * 12 * (size_t)iters,
                               hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(pnp_score, dim3(iters), dim3(256), 0, s, sp);
    SLAM_HIP(c, hipGetLastError());
    std::vector<int> cnt(iters);
    SLAM_HIP(c, hipMemcpyAsync(cnt.data(), sp.counts, sizeof(int) * (size_t)iters, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    // RANSACPointSetRegistrator::run replayed on the speculative counts
    int best = -1, niters = maxIters, maxGood = 0;
    for (int it = 0; it < niters; it++) {
        const int good = cnt[it];
        if (good > (maxGood > 4 ? maxGood : 4)) {
            best = it;
            maxGood = good;
            niters = ransac_update_iters(confidence, (double)(n - good) / n, 5, niters);
        }
    }
    if (best < 0) {
        for (int k = 0; k < 3; k++) rvec[k] = tvec[k] = 0;
        if (mask) std::memset(mask, 0, (size_t)n);
        return SLAM_OK;
    }
    uint8_t* dmask = reinterpret_cast<uint8_t*>(base + o_mask);
    hipLaunchKernelGGL(pnp_mask, dim3((n + 255) / 256), dim3(256), 0, s, sp,
                       (const double*)(base + o_mod + sizeof(double) * 12 * (size_t)best), dmask);
    SLAM_HIP(c, hipGetLastError());
    std::vector<uint8_t> hm((size_t)n);
    SLAM_HIP(c, hipMemcpyAsync(hm.data(), dmask, (size_t)n, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    std::vector<int> idx;
    idx.reserve(maxGood);
    for (int i = 0; i < n; i++)
        if (hm[i]) idx.push_back(i);
    const int m = (int)idx.size();
    int* didx = reinterpret_cast<int*>(base + o_idx);
    SLAM_HIP(c, hipMemcpyAsync(didx, idx.data(), sizeof(int) * (size_t)m, hipMemcpyHostToDevice, s));
    // cvFindExtrinsicCameraParams2(useExtrinsicGuess = 1): CvLevMarq on the host.
    // Each LM iteration evaluates the step at the current damping and the next
    // kSpec - 1 dampings together, every candidate with its Jacobian (J'J, J'e,
    // |e|^2 as the same ordered sums); the host replays the sequential accept /
    // raise-lambda loop on the candidates' |e|^2 and takes the accepted one's
    // J'J / J'e for the next step.  Identical decisions and values to
    // evaluate-then-re-evaluate, one sync per iteration instead of two or more.
    EvalParams ev;
    ev.fx = K[0]; ev.fy = K[4]; ev.cx = K[2]; ev.cy = K[5];
    ev.op = dop; ev.ip = dip; ev.idx = didx; ev.m = m;
    ev.err = reinterpret_cast<double*>(base + o_err);
    ev.J = reinterpret_cast<double*>(base + o_J);
    ev.err_stride = 2 * (size_t)m;
    ev.J_stride = 12 * (size_t)m;
    ev.withJ = 1;
    double* dred = reinterpret_cast<double*>(base + o_red);
    double* red = static_cast<double*>(readback(c, sizeof(double) * 28 * kSpec));   // pinned: async copy + polled sync
    if (!red) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    // evaluate nc parameter vectors (6 each) with their Jacobians: red[28 c + ...]
    auto evaluate = [&](const double* params, int nc) -> int {
        for (int q = 0; q < nc; q++) {
            rodrigues_v2m(params + 6 * q, ev.R[q], ev.dRdr[q]);
            for (int k = 0; k < 3; k++) ev.t[q][k] = params[6 * q + 3 + k];
        }
        if (c->opt_pnp_sums == SLAM_PNP_SUMS_PAIRWISE) {
            hipLaunchKernelGGL(pnp_eval_sums, dim3(nc), dim3(256), 0, s, ev, dred);
        } else {
            hipLaunchKernelGGL(pnp_eval, dim3((m + 255) / 256, nc), dim3(256), 0, s, ev);
            hipLaunchKernelGGL(pnp_reduce, dim3(nc), dim3(kRedThreads), 0, s, (const double*)ev.J, (const double*)ev.err,
                               m, 1, dred, ev.err_stride, ev.J_stride);
        }
        SLAM_HIP(c, hipGetLastError());
        SLAM_HIP(c, hipMemcpyAsync(red, dred, sizeof(double) * 28 * nc, hipMemcpyDeviceToHost, s));
        n_evals++;
        return stream_sync(c, s, true);
    };
    auto take = [&](int q, double* JtJ, double* JtErr) {
        const double* r = red + 28 * q;
        int u = 0;
        for (int i = 0; i < 6; i++)
            for (int j = i; j < 6; j++, u++) JtJ[i * 6 + j] = JtJ[j * 6 + i] = r[u];
        for (int i = 0; i < 6; i++) JtErr[i] = r[21 + i];
    };
    double param[6], prev[6], JtJ[36], JtErr[6];
    std::memcpy(param, rt.data() + 6 * (size_t)best, sizeof(param));
    const int max_iter = 20;
    const double eps = FLT_EPSILON;
    double errNorm, prevErrNorm = DBL_MAX;
    int lambdaLg10 = -3, lmIters = 0;
    const auto t_lm = std::chrono::steady_clock::now();
    if (int rc = evaluate(param, 1)) return rc;
    take(0, JtJ, JtErr);
    double nrm2 = red[27];
    for (;;) {
        std::memcpy(prev, param, sizeof(prev));
        if (lmIters == 0) prevErrNorm = std::sqrt(nrm2);
        // the sequential loop: step at lambdaLg10; while it raises the error and
        // ++lambdaLg10 <= 16, step again at the raised damping
        int acc = -1;
        double cand[6 * kSpec];
        while (acc < 0) {
            int nc = 0;
            for (; nc < kSpec && lambdaLg10 + nc <= 16 + (nc == 0 ? 64 : 0); nc++)
                lm_step(JtJ, JtErr, lambdaLg10 + nc, prev, cand + 6 * nc);
            if (int rc = evaluate(cand, nc)) return rc;
            for (int q = 0; q < nc; q++) {
                errNorm = std::sqrt(red[28 * q + 27]);
                if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) continue;   // the next candidate (or batch)
                acc = q;
                break;
            }
        }
        std::memcpy(param, cand + 6 * acc, sizeof(param));
        lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
        double d[6];
        for (int k = 0; k < 6; k++) d[k] = param[k] - prev[k];
        const double rel = std::sqrt(norm_l2sqr(d, 6)) / (std::sqrt(norm_l2sqr(prev, 6)) + DBL_EPSILON);
        if (++lmIters >= max_iter || rel < eps) break;
        prevErrNorm = errNorm;
        take(acc, JtJ, JtErr);        // the accepted candidate's J'J / J'e (computed with it)
    }
    for (int k = 0; k < 3; k++) { rvec[k] = param[k]; tvec[k] = param[3 + k]; }
    if (mask) std::memcpy(mask, hm.data(), (size_t)n);
    if (timing) {
        const auto t_end = std::chrono::steady_clock::now();
        auto us = [](std::chrono::steady_clock::duration d) { return std::chrono::duration<double, std::micro>(d).count(); };
        fprintf(stderr, "pnp n %d inliers %d lm_iters %d evals %d ransac_us %.1f lm_us %.1f\n", n, m, lmIters, n_evals,
                us(t_lm - t_start), us(t_end - t_lm));
    }
    *ninliers = m;
    *found = 1;
    return SLAM_OK;
}

// cv::Rodrigues on the host (cvRodrigues2 restated as oracle/pnp.c): 3 -> 3 x 3
// (rodrigues_v2m) or 3 x 3 -> 3 (checkRange, the SVD orthonormalisation U Vt,
// rodrigues_m2v).  Used by the pipeline after solvePnPRansac (mainCycle.cpp:162)
// and by the BA parameter conversions (bundleAdjustment.cpp:153-201).
int rodrigues_host(const double* src, int n, double* dst)
{
    if (n == 3) {
        rodrigues_v2m(src, dst, nullptr);
        return SLAM_OK;
    }
    if (n != 9) return SLAM_E_INVALID_ARG;
    double At[9], W[3], Vt[9], R[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = src[r * 3 + c];
    jsvd_u<3, 3>(At, W, Vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += At[k * 3 + i] * Vt[k * 3 + j];
            R[i * 3 + j] = s;
        }
    rodrigues_m2v(src, R, dst);
    return SLAM_OK;
}

}  // namespace slamhip

extern "C" int slam_rodrigues(const double* src, int n, double* dst)
{
    if (!src || !dst) return SLAM_E_INVALID_ARG;
    return slamhip::rodrigues_host(src, n, dst);
}
