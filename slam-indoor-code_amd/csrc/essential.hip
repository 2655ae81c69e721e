// Relative pose on gfx950 (FP64), replacing the reference's estimateTransformation
// (src/mainModule/translation/cameraTranslation.cpp:32-69): findEssentialMat(
// points1, points2, K, RANSAC, prob, threshold, mask) then recoverPose(E, ...,
// distanceThresh, chiralityMask) with the reference's EMPTY chiralityMask (so
// the cheirality count runs over all points).  Same restatement as
// oracle/essential.c, operation for operation (no contraction), so E, R, t and
// both masks agree bit for bit:
//   - RANSAC is speculative: the host draws all maxIters = 1000 minimal subsets
//     from the cv::RNG((uint64)-1) stream up front (getSubset never rejects for
//     the essential-matrix callback, so the draws do not depend on results),
//     ep_hyp solves every hypothesis (one thread per iteration: the five-point
//     solver), ep_score counts every model's Sampson inliers (one workgroup per
//     iteration), and the host replays RANSACPointSetRegistrator's sequential
//     accept / RANSACUpdateNumIters loop on the counts -- the chosen model is
//     the one the sequential loop would choose;
//   - recoverPose: decomposeEssentialMat on the host (3 x 3 Jacobi SVD), the 4
//     candidate poses' triangulation + cheirality bits of every point in
//     ep_cheir (one thread per point), counts and the pose choice on the host.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "jacobi.h"
#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kMaxIters = 1000;     // findEssentialMat's maxIters
constexpr int kMaxModels = 10;

HD void svd33(const double* A, double* U, double* W, double* Vt)
{
    double At[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) At[c * 3 + r] = A[r * 3 + c];
    jsvd<3, 3>(At, W, Vt);
    for (int i = 0; i < 3; i++) {
        const double inv = W[i] > DBL_MIN ? 1. / W[i] : 0.;
        for (int k = 0; k < 3; k++) U[k * 3 + i] = At[i * 3 + k] * inv;
    }
}

HD inline double det33(const double* a)
{
    return a[0] * (a[4] * a[8] - a[7] * a[5]) - a[1] * (a[3] * a[8] - a[6] * a[5]) +
           a[2] * (a[3] * a[7] - a[6] * a[4]);
}

// ---- five-point solver (oracle/essential.c orc_five_point) ----
__constant__ int c_LQ[4][4] = {{0, 2, 3, 4}, {2, 1, 5, 6}, {3, 5, 7, 8}, {4, 6, 8, 9}};
__constant__ int c_QL[10][4] = {{0, 2, 4, 5},   {3, 1, 6, 7},   {2, 3, 8, 9},     {4, 8, 10, 11},  {5, 9, 11, 12},
                                {8, 6, 13, 14}, {9, 7, 14, 15}, {10, 13, 16, 17}, {11, 14, 17, 18}, {12, 15, 18, 19}};

__device__ inline void mul_ll(const double* a, const double* b, double* q)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) q[c_LQ[i][j]] += a[i] * b[j];
}
__device__ inline void mul_ql(const double* a, const double* b, double s, double* c)
{
    for (int i = 0; i < 10; i++)
        for (int j = 0; j < 4; j++) c[c_QL[i][j]] += s * (a[i] * b[j]);
}

__device__ void coeff_mat(const double (*EE)[9], double (*A)[20])
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
    double* d = A[9];
    for (int c = 0; c < 20; c++) d[c] = 0;
    const int cof[3][4] = {{4, 8, 5, 7}, {3, 8, 5, 6}, {3, 7, 4, 6}};
    const double sg[3] = {1.0, -1.0, 1.0};
    for (int e = 0; e < 3; e++) {
        for (int q = 0; q < 10; q++) t1[q] = t2[q] = 0;
        mul_ll(E[cof[e][0]], E[cof[e][1]], t1);
        mul_ll(E[cof[e][2]], E[cof[e][3]], t2);
        for (int q = 0; q < 10; q++) t1[q] -= t2[q];
        mul_ql(t1, E[e], sg[e], d);
    }
}

__device__ bool gj_solve(double (*A)[20], double (*R)[10])
{
    for (int col = 0; col < 10; col++) {
        int piv = col;
        for (int r = col + 1; r < 10; r++)
            if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
        if (A[piv][col] == 0.0) return false;
        if (piv != col)
            for (int c = 0; c < 20; c++) { const double t = A[col][c]; A[col][c] = A[piv][c]; A[piv][c] = t; }
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
    return true;
}

__device__ inline void zmul(const double* a, int na, const double* b, int nb, double* r)
{
    for (int i = 0; i < na + nb - 1; i++) r[i] = 0;
    for (int i = 0; i < na; i++)
        for (int j = 0; j < nb; j++) r[i + j] += a[i] * b[j];
}

// Durand-Kerner with the degree as a template parameter: every array index is
// a compile-time constant, so a[], re[], im[] live in registers (the runtime-n
// form kept them in scratch memory and dominated ep_hyp).  Same operations in
// the same order as oracle/essential.c.
template <int N>
__device__ void dk_roots_n(const double* c, double* re_out, double* im_out)
{
    double a[N + 1], re[N], im[N];
#pragma unroll
    for (int k = 0; k <= N; k++) a[k] = c[k] / c[N];
    const double zr = 0.4, zi = 0.9;
    re[0] = zr; im[0] = zi;
#pragma unroll
    for (int k = 1; k < N; k++) {
        const double r = re[k - 1] * zr - im[k - 1] * zi, i = re[k - 1] * zi + im[k - 1] * zr;
        re[k] = r; im[k] = i;
    }
    for (int iter = 0; iter < 500; iter++) {
        double maxd = 0;
#pragma unroll
        for (int k = 0; k < N; k++) {
            double pr = 1.0, pi = 0.0;
#pragma unroll
            for (int d = N - 1; d >= 0; d--) {
                const double tr = pr * re[k] - pi * im[k] + a[d], ti = pr * im[k] + pi * re[k];
                pr = tr; pi = ti;
            }
            double qr = 1.0, qi = 0.0;
#pragma unroll
            for (int j = 0; j < N; j++) {
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
#pragma unroll
    for (int k = 0; k < N; k++) { re_out[k] = re[k]; im_out[k] = im[k]; }
}

__device__ void dk_roots(const double* c, int n, double* re, double* im)
{
    switch (n) {
    case 1: dk_roots_n<1>(c, re, im); break;
    case 2: dk_roots_n<2>(c, re, im); break;
    case 3: dk_roots_n<3>(c, re, im); break;
    case 4: dk_roots_n<4>(c, re, im); break;
    case 5: dk_roots_n<5>(c, re, im); break;
    case 6: dk_roots_n<6>(c, re, im); break;
    case 7: dk_roots_n<7>(c, re, im); break;
    case 8: dk_roots_n<8>(c, re, im); break;
    case 9: dk_roots_n<9>(c, re, im); break;
    default: dk_roots_n<10>(c, re, im); break;
    }
}

__device__ int five_point(const double* q1, const double* q2, double* Es)
{
    double Q[5][9];
    for (int i = 0; i < 5; i++) {
        const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        Q[i][0] = x1 * x2; Q[i][1] = y1 * x2; Q[i][2] = x2; Q[i][3] = x1 * y2; Q[i][4] = y1 * y2;
        Q[i][5] = y2; Q[i][6] = x1; Q[i][7] = y1; Q[i][8] = 1.0;
    }
    double M[9][5], v[9], H[9][9];
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 5; c++) M[r][c] = Q[c][r];
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 9; c++) H[r][c] = r == c ? 1.0 : 0.0;
    for (int k = 0; k < 5; k++) {
        double nrm = 0;
        for (int r = k; r < 9; r++) nrm += M[r][k] * M[r][k];
        nrm = sqrt(nrm);
        for (int r = 0; r < 9; r++) v[r] = r < k ? 0.0 : M[r][k];
        const double alpha = M[k][k] >= 0 ? -nrm : nrm;
        v[k] -= alpha;
        double vn = 0;
        for (int r = k; r < 9; r++) vn += v[r] * v[r];
        if (vn == 0.0) continue;
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
    double b[3][13];
    for (int i = 0; i < 3; i++) {
        const double* r1 = R[i * 2 + 4];
        const double* r2 = R[i * 2 + 5];
        double row1[13], row2[13];
        for (int k = 0; k < 13; k++) row1[k] = row2[k] = 0;
        for (int k = 0; k < 3; k++) { row1[1 + k] = r1[k]; row1[5 + k] = r1[3 + k]; }
        for (int k = 0; k < 4; k++) row1[9 + k] = r1[6 + k];
        for (int k = 0; k < 3; k++) { row2[k] = r2[k]; row2[4 + k] = r2[3 + k]; }
        for (int k = 0; k < 4; k++) row2[8 + k] = r2[6 + k];
        for (int k = 0; k < 13; k++) b[i][k] = row1[k] - row2[k];
    }
    double P[3][3][5];
    for (int i = 0; i < 3; i++) {
        for (int k = 0; k < 5; k++) P[i][0][k] = P[i][1][k] = P[i][2][k] = 0;
        for (int k = 0; k < 4; k++) { P[i][0][3 - k] = b[i][k]; P[i][1][3 - k] = b[i][4 + k]; }
        for (int k = 0; k < 5; k++) P[i][2][4 - k] = b[i][8 + k];
    }
    const int deg[3] = {3, 3, 4};
    const int perm[6][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 0}};
    const double sign[6] = {1, 1, 1, -1, -1, -1};
    double cdet[11];
    for (int k = 0; k < 11; k++) cdet[k] = 0;
    for (int q = 0; q < 6; q++) {
        double t1[9], t2[11];
        zmul(P[0][perm[q][0]], deg[perm[q][0]] + 1, P[1][perm[q][1]], deg[perm[q][1]] + 1, t1);
        const int n1 = deg[perm[q][0]] + deg[perm[q][1]] + 1;
        zmul(t1, n1, P[2][perm[q][2]], deg[perm[q][2]] + 1, t2);
        const int n2 = n1 + deg[perm[q][2]];
        for (int k = 0; k < n2 && k < 11; k++) cdet[k] += sign[q] * t2[k];
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
        const double* xy1 = Vt + 6;
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

HD inline float sampson(const double* E, double x1, double y1, double x2, double y2)
{
    const double Ex1[3] = {E[0] * x1 + E[1] * y1 + E[2], E[3] * x1 + E[4] * y1 + E[5], E[6] * x1 + E[7] * y1 + E[8]};
    const double Etx2[3] = {E[0] * x2 + E[3] * y2 + E[6], E[1] * x2 + E[4] * y2 + E[7],
                            E[2] * x2 + E[5] * y2 + E[8]};
    const double x2tEx1 = x2 * Ex1[0] + y2 * Ex1[1] + Ex1[2];
    const double a = Ex1[0] * Ex1[0], b = Ex1[1] * Ex1[1], c = Etx2[0] * Etx2[0], d = Etx2[1] * Etx2[1];
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

// ---- kernels ----
struct EpParams {
    const double4* q;          // normalised (x1, y1, x2, y2) per point
    int n;
    const int* subsets;        // kMaxIters x 5
    double* Es;                // kMaxIters x 10 x 9
    int* nmodels;              // kMaxIters
    int* counts;               // kMaxIters x 10
    float thr2;
    int it0, it1;              // the hypotheses of this launch: [it0, it1)
};

__global__ __launch_bounds__(64) void ep_hyp(EpParams p)
{
    const int it = p.it0 + blockIdx.x * 64 + threadIdx.x;
    if (it >= p.it1) return;
    double a1[10], a2[10];
    for (int k = 0; k < 5; k++) {
        const double4 v = p.q[p.subsets[5 * it + k]];
        a1[2 * k] = v.x; a1[2 * k + 1] = v.y;
        a2[2 * k] = v.z; a2[2 * k + 1] = v.w;
    }
    p.nmodels[it] = five_point(a1, a2, p.Es + (size_t)it * kMaxModels * 9);
}

__global__ __launch_bounds__(256) void ep_score(EpParams p)
{
    __shared__ int red[4];
    __shared__ double Esh[kMaxModels * 9];
    const int it = p.it0 + blockIdx.x, tid = threadIdx.x;
    const int nm = p.nmodels[it];
    for (int e = tid; e < nm * 9; e += 256) Esh[e] = p.Es[(size_t)it * kMaxModels * 9 + e];
    __syncthreads();
    for (int m = 0; m < nm; m++) {
        int c = 0;
        for (int i = tid; i < p.n; i += 256) {
            const double4 v = p.q[i];
            c += sampson(Esh + 9 * m, v.x, v.y, v.z, v.w) <= p.thr2;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((tid & 63) == 0) red[tid >> 6] = c;
        __syncthreads();
        if (tid == 0) p.counts[it * kMaxModels + m] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void ep_mask(const double4* q, int n, const double* E, float thr2, uint8_t* mask)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double4 v = q[i];
    mask[i] = sampson(E, v.x, v.y, v.z, v.w) <= thr2;
}

struct CheirParams {
    const double4* q;
    int n;
    double R1[9], R2[9], t[3], dist;
    uint8_t* bits;
};

__device__ void tri_point(const double* P1, const double* P2, double x1, double y1, double x2, double y2, double* X)
{
    const double* P[2] = {P1, P2};
    const double xs[2] = {x1, x2}, ys[2] = {y1, y2};
    double At[16], W[4], Vt[16];
    for (int v = 0; v < 2; v++)
        for (int c = 0; c < 4; c++) {
            At[c * 4 + v * 2] = xs[v] * P[v][8 + c] - P[v][c];
            At[c * 4 + v * 2 + 1] = ys[v] * P[v][8 + c] - P[v][4 + c];
        }
    jsvd<4, 4>(At, W, Vt);
    for (int k = 0; k < 4; k++) X[k] = Vt[12 + k];
}

__global__ __launch_bounds__(128) void ep_cheir(CheirParams p)
{
    const int i = blockIdx.x * 128 + threadIdx.x;
    if (i >= p.n) return;
    const double4 v = p.q[i];
    const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int bits = 0;
    for (int pose = 0; pose < 4; pose++) {
        const double* R = (pose & 1) ? p.R2 : p.R1;
        const double sg = pose >= 2 ? -1.0 : 1.0;
        double P[12];
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) P[r * 4 + c] = R[r * 3 + c];
            P[r * 4 + 3] = p.t[r] * sg;
        }
        double X[4];
        tri_point(P0, P, v.x, v.y, v.z, v.w, X);
        bool ok = X[2] * X[3] > 0;
        const double Xn[4] = {X[0] / X[3], X[1] / X[3], X[2] / X[3], X[3] / X[3]};
        ok = ok && Xn[2] < p.dist;
        double z2 = 0;
        for (int k = 0; k < 4; k++) z2 += P[8 + k] * Xn[k];
        ok = ok && z2 > 0 && z2 < p.dist;
        if (ok) bits |= 1 << pose;
    }
    p.bits[i] = (uint8_t)bits;
}

// ---- host side ----
}  // namespace

int ransac_update_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0 ? p : 0.;
    p = p < 1 ? p : 1.;
    ep = ep > 0 ? ep : 0.;
    ep = ep < 1 ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - std::pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)std::lrint(num / denom);
}

void ransac_subsets5(int count, int iters, int* idx)
{
    CvRng rng{~0ull};
    for (int it = 0; it < iters; it++) {
        int* id = idx + 5 * it;
        for (int i = 0; i < 5; i++) {
            int v, j;
            for (;;) {
                v = id[i] = rng.uniform(0, count);
                for (j = 0; j < i; j++)
                    if (v == id[j]) break;
                if (j == i) break;
            }
        }
    }
}

namespace {

void decompose_essential(const double* E, double* R1, double* R2, double* t)
{
    double U[9], W[3], Vt[9];
    svd33(E, U, W, Vt);
    if (det33(U) < 0)
        for (int k = 0; k < 9; k++) U[k] *= -1.;
    if (det33(Vt) < 0)
        for (int k = 0; k < 9; k++) Vt[k] *= -1.;
    const double Wm[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
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

}  // namespace

int relative_pose(slam_ctx* c, const float* p1, const float* p2, int n, const double* K, int use_ransac,
                  double prob, double threshold, double dist, double* R, double* t, uint8_t* chirality,
                  uint8_t* ransac_mask, int* passed)
{
    *passed = 0;
    if (!use_ransac) { prob = 0.999; threshold = 1.0; }      // findEssentialMat(points1, points2, K) defaults
    if (n < 5) return SLAM_OK;
    hipStream_t s = c->stream;
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    std::vector<double> q((size_t)4 * n);
    for (int i = 0; i < n; i++) {
        q[4 * i] = ((double)p1[2 * i] - cx) / fx;
        q[4 * i + 1] = ((double)p1[2 * i + 1] - cy) / fy;
        q[4 * i + 2] = ((double)p2[2 * i] - cx) / fx;
        q[4 * i + 3] = ((double)p2[2 * i + 1] - cy) / fy;
    }
    const double thr = threshold / ((fx + fy) / 2);
    const float thr2 = (float)(thr * thr);
    const int iters = n == 5 ? 1 : kMaxIters;
    std::vector<int> sub((size_t)5 * kMaxIters, 0);
    if (n == 5) {
        for (int k = 0; k < 5; k++) sub[k] = k;
    } else {
        ransac_subsets5(n, kMaxIters, sub.data());
    }
    // device layout
    size_t off = 0;
    auto carve = [&](size_t b) { const size_t o = off; off += (b + 255) & ~(size_t)255; return o; };
    const size_t o_q = carve(sizeof(double4) * (size_t)n), o_sub = carve(sizeof(int) * 5 * kMaxIters),
                 o_es = carve(sizeof(double) * 9 * kMaxModels * kMaxIters), o_nm = carve(sizeof(int) * kMaxIters),
                 o_ct = carve(sizeof(int) * kMaxModels * kMaxIters), o_e = carve(sizeof(double) * 9),
                 o_mask = carve((size_t)n), o_bits = carve((size_t)n);
    SLAM_HIP(c, c->geom.ensure(off));
    char* base = c->geom.as<char>();
    EpParams ep;
    ep.q = reinterpret_cast<const double4*>(base + o_q);
    ep.n = n;
    ep.subsets = reinterpret_cast<const int*>(base + o_sub);
    ep.Es = reinterpret_cast<double*>(base + o_es);
    ep.nmodels = reinterpret_cast<int*>(base + o_nm);
    ep.counts = reinterpret_cast<int*>(base + o_ct);
    ep.thr2 = thr2;
    SLAM_HIP(c, hipMemcpyAsync(base + o_q, q.data(), sizeof(double) * 4 * (size_t)n, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_sub, sub.data(), sizeof(int) * 5 * kMaxIters, hipMemcpyHostToDevice, s));
    std::vector<int> nm(kMaxIters, 0), ct((size_t)kMaxModels * kMaxIters, 0);
    // The hypotheses in chunks (64, 256, then the rest), each replayed before the
    // next is launched: RANSACUpdateNumIters only lowers niters, so the loop
    // needs hypotheses [0, niters) and a chunk past the last one is never run.
    // A launch lasts as long as its slowest five-point solve (Durand-Kerner runs
    // up to 500 iterations), so small first chunks cut the wait when the model
    // is found early; the decisions are those of one launch over all of them.
    // RANSACPointSetRegistrator::run replayed on the speculative counts
    int best_it = -1, best_m = -1;
    int niters = iters, maxGood = 0, done = 0;
    static const int kChunks[3] = {64, 256, kMaxIters};
    for (int ci = 0; done < niters; ci++) {
        const int end = std::min(niters, ci < 2 ? done + kChunks[ci] : kMaxIters);
        ep.it0 = done;
        ep.it1 = end;
        hipLaunchKernelGGL(ep_hyp, dim3((end - done + 63) / 64), dim3(64), 0, s, ep);
        hipLaunchKernelGGL(ep_score, dim3(end - done), dim3(256), 0, s, ep);
        SLAM_HIP(c, hipGetLastError());
        SLAM_HIP(c, hipMemcpyAsync(nm.data() + done, ep.nmodels + done, sizeof(int) * (end - done), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipMemcpyAsync(ct.data() + (size_t)done * kMaxModels, ep.counts + (size_t)done * kMaxModels,
                                   sizeof(int) * kMaxModels * (end - done), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipStreamSynchronize(s));
        if (n == 5) {
            if (nm[0] > 0) { best_it = 0; best_m = 0; }
            break;
        }
        for (int it = done; it < end && it < niters; it++)
            for (int m = 0; m < nm[it]; m++) {
                const int good = ct[(size_t)it * kMaxModels + m];
                if (good > (maxGood > 4 ? maxGood : 4)) {
                    best_it = it;
                    best_m = m;
                    maxGood = good;
                    niters = ransac_update_iters(prob, (double)(n - good) / n, 5, niters);
                }
            }
        done = end;
    }
    if (best_it < 0) return SLAM_OK;
    double E[9];
    SLAM_HIP(c, hipMemcpy(E, ep.Es + ((size_t)best_it * kMaxModels + best_m) * 9, sizeof(E), hipMemcpyDeviceToHost));
    double* dE = reinterpret_cast<double*>(base + o_e);
    uint8_t* dmask = reinterpret_cast<uint8_t*>(base + o_mask);
    uint8_t* dbits = reinterpret_cast<uint8_t*>(base + o_bits);
    SLAM_HIP(c, hipMemcpyAsync(dE, E, sizeof(E), hipMemcpyHostToDevice, s));
    if (n == 5) SLAM_HIP(c, hipMemsetAsync(dmask, 1, 5, s));
    else hipLaunchKernelGGL(ep_mask, dim3((n + 255) / 256), dim3(256), 0, s, ep.q, n, (const double*)dE, thr2, dmask);
    // recoverPose
    CheirParams cp;
    decompose_essential(E, cp.R1, cp.R2, cp.t);
    cp.q = ep.q; cp.n = n; cp.dist = dist; cp.bits = dbits;
    hipLaunchKernelGGL(ep_cheir, dim3((n + 127) / 128), dim3(128), 0, s, cp);
    SLAM_HIP(c, hipGetLastError());
    std::vector<uint8_t> bits((size_t)n);
    if (ransac_mask) SLAM_HIP(c, hipMemcpyAsync(ransac_mask, dmask, (size_t)n, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(bits.data(), dbits, (size_t)n, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    int good[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 4; k++) good[k] += (bits[i] >> k) & 1;
    int pick;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3]) pick = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3]) pick = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3]) pick = 2;
    else pick = 3;
    std::memcpy(R, (pick & 1) ? cp.R2 : cp.R1, sizeof(double) * 9);
    for (int k = 0; k < 3; k++) t[k] = pick >= 2 ? -cp.t[k] : cp.t[k];
    if (chirality)
        for (int i = 0; i < n; i++) chirality[i] = (bits[i] >> pick) & 1;
    *passed = good[pick];
    return SLAM_OK;
}

}  // namespace slamhip
