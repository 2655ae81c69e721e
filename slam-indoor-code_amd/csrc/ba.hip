// Windowed bundle adjustment on gfx950 (FP64), replacing the reference's Ceres
// call site bundleAdjustment (src/mainModule/bundleAdjustment/
// bundleAdjustment.cpp:73-129): same parameter blocks (shared free intrinsics
// {fx, fy, cx, cy}, per-frame angle-axis + t with frame 0 constant, points),
// same residual (ProjectionCostFunctor :15-41), same losses (getLossFunction
// :131-151, Ceres Corrector), same Levenberg-Marquardt trust region with
// Jacobi scaling and Schur elimination of the points (Options :108-114).
//
// Device side, per LM iteration:
//   ba_eval      one thread per observation: residual + 2 x 13 Jacobian by
//                forward-mode jets (ceres/jet.h arithmetic), loss correction,
//                cost reduced per workgroup.
//   ba_point     one thread per point (observations grouped by point, CSR):
//                scaled J'J blocks, V_p + D_p inverse (3x3 Cholesky), and the
//                point's whole contribution to the reduced camera system
//                S = U + D_c - sum_p W_p V_p^-1 W_p' and rhs, accumulated in an
//                LDS copy of S (ds_add_f64) and flushed once per workgroup.
//   rocSOLVER    dpotrf / dpotrs on S (nc = 4 + 6 (W - 1): 46 at W = 8).
//   ba_backsub   one thread per point: y_p = V_p^-1 (g_p - W_p' y_c); model cost
//                change J_s step; candidate x + step .* scale.
// The host keeps the scalar LM state (radius, decrease factor, tolerances) and
// makes exactly the oracle's accept / reject decisions (oracle/ba.c).
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int NJ = 13;

struct Jet {
    double a;
    double v[NJ];
};

__device__ inline Jet jc(double a) { Jet r; r.a = a;
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = 0; return r; }
__device__ inline Jet jv(double a, int k) { Jet r = jc(a); r.v[k] = 1.0; return r; }
__device__ inline Jet jadd(const Jet& x, const Jet& y) { Jet r; r.a = __dadd_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dadd_rn(x.v[i], y.v[i]); return r; }
__device__ inline Jet jsub(const Jet& x, const Jet& y) { Jet r; r.a = __dsub_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dsub_rn(x.v[i], y.v[i]); return r; }
__device__ inline Jet jmul(const Jet& x, const Jet& y) { Jet r; r.a = __dmul_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dadd_rn(__dmul_rn(x.a, y.v[i]), __dmul_rn(x.v[i], y.a)); return r; }
__device__ inline Jet jdiv(const Jet& f, const Jet& g)
{
    const double gi = __ddiv_rn(1.0, g.a), fg = __dmul_rn(f.a, gi);
    Jet r; r.a = fg;
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dmul_rn(__dsub_rn(f.v[i], __dmul_rn(fg, g.v[i])), gi);
    return r;
}
__device__ inline Jet jsqrt(const Jet& f)
{
    const double t = __dsqrt_rn(f.a), tw = __ddiv_rn(1.0, __dmul_rn(2.0, t));
    Jet r; r.a = t;
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dmul_rn(f.v[i], tw);
    return r;
}
__device__ inline Jet jcos(const Jet& f) { Jet r; r.a = cos(f.a); const double s = -sin(f.a);
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dmul_rn(s, f.v[i]); return r; }
__device__ inline Jet jsin(const Jet& f) { Jet r; r.a = sin(f.a); const double c = cos(f.a);
#pragma unroll
    for (int i = 0; i < NJ; i++) r.v[i] = __dmul_rn(c, f.v[i]); return r; }

// ceres AngleAxisRotatePoint + t, pinhole, minus the observation
__device__ void project(const double* K, const double* e, const double* X, double ox, double oy, double r[2],
                        double J[2][NJ])
{
    Jet aa[3] = {jv(e[0], 4), jv(e[1], 5), jv(e[2], 6)};
    Jet pt[3] = {jv(X[0], 10), jv(X[1], 11), jv(X[2], 12)};
    Jet p[3];
    Jet th2 = jadd(jadd(jmul(aa[0], aa[0]), jmul(aa[1], aa[1])), jmul(aa[2], aa[2]));
    if (th2.a > DBL_EPSILON) {
        Jet th = jsqrt(th2);
        Jet ct = jcos(th), st = jsin(th);
        Jet ti = jdiv(jc(1.0), th);
        Jet w[3] = {jmul(aa[0], ti), jmul(aa[1], ti), jmul(aa[2], ti)};
        Jet wx[3] = {jsub(jmul(w[1], pt[2]), jmul(w[2], pt[1])), jsub(jmul(w[2], pt[0]), jmul(w[0], pt[2])),
                     jsub(jmul(w[0], pt[1]), jmul(w[1], pt[0]))};
        Jet tmp = jmul(jadd(jadd(jmul(w[0], pt[0]), jmul(w[1], pt[1])), jmul(w[2], pt[2])), jsub(jc(1.0), ct));
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = jadd(jadd(jmul(pt[k], ct), jmul(wx[k], st)), jmul(w[k], tmp));
    } else {
        Jet wx[3] = {jsub(jmul(aa[1], pt[2]), jmul(aa[2], pt[1])), jsub(jmul(aa[2], pt[0]), jmul(aa[0], pt[2])),
                     jsub(jmul(aa[0], pt[1]), jmul(aa[1], pt[0]))};
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = jadd(pt[k], wx[k]);
    }
    p[0] = jadd(p[0], jv(e[3], 7));
    p[1] = jadd(p[1], jv(e[4], 8));
    p[2] = jadd(p[2], jv(e[5], 9));
    Jet x2 = jdiv(p[0], p[2]), y2 = jdiv(p[1], p[2]);
    Jet u = jsub(jadd(jmul(jv(K[0], 0), x2), jv(K[2], 2)), jc(ox));
    Jet v = jsub(jadd(jmul(jv(K[1], 1), y2), jv(K[3], 3)), jc(oy));
    r[0] = u.a;
    r[1] = v.a;
    if (J) {
#pragma unroll
        for (int i = 0; i < NJ; i++) { J[0][i] = u.v[i]; J[1][i] = v.v[i]; }
    }
}

__device__ inline void loss_eval(int loss, double a, double s, double rho[3])
{
    switch (loss) {
    case SLAM_LOSS_HUBER: {
        const double b = a * a;
        if (s > b) {
            const double r = sqrt(s);
            rho[0] = 2.0 * a * r - b;
            rho[1] = fmax(DBL_MIN, a / r);
            rho[2] = -rho[1] / (2.0 * s);
        } else { rho[0] = s; rho[1] = 1.0; rho[2] = 0.0; }
        return;
    }
    case SLAM_LOSS_CAUCHY: {
        const double b = a * a, c = 1.0 / b;
        const double sum = 1.0 + s * c, inv = 1.0 / sum;
        rho[0] = b * log(sum);
        rho[1] = fmax(DBL_MIN, inv);
        rho[2] = -c * (inv * inv);
        return;
    }
    case SLAM_LOSS_ARCTAN: {
        const double b = 1.0 / (a * a);
        const double sum = 1 + s * s * b, inv = 1 / sum;
        rho[0] = a * atan2(s, a);
        rho[1] = fmax(DBL_MIN, inv);
        rho[2] = -2.0 * s * b * (inv * inv);
        return;
    }
    case SLAM_LOSS_TUKEY: {
        const double a2 = a * a;
        if (s <= a2) {
            const double value = 1.0 - s / a2, vs = value * value;
            rho[0] = a2 / 3.0 * (1.0 - vs * value);
            rho[1] = vs;
            rho[2] = -2.0 / a2 * value;
        } else { rho[0] = a2 / 3.0; rho[1] = 0.0; rho[2] = 0.0; }
        return;
    }
    default:
        rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
        return;
    }
}

struct BaDev {
    int nf, np, no, nc, loss;
    double a;
    const int* of;
    const int* op;
    const double* oxy;
    const int* pstart;      // CSR obs per point
    const int* plist;
    double* x;              // parameters: K[4], ext[nf * 6] (incl. frame 0), pts[np * 3]
    double* xc;             // candidate
    double* r;              // [no][2]
    double* J;              // [no][2][13]
    double* scale;          // [4 + 6 (nf - 1) + 3 np]
    double* g;              // scaled gradient (camera part reduced in place)
    double* S;              // nc x nc (column-major == row-major, symmetric)
    double* rc;             // nc
    double* Vinv;           // [np][9]
    double* wobs;           // [no][10][3] scaled J_c' J_p per observation
    double* step;           // N
    double* red;            // reduction slots: 0 cost, 1 cand cost, 2 mcc, 3 gmax(unscaled), 4 snorm^2, 5 flag
    double radius;
};

__device__ inline double* ext_of(const BaDev& d, double* x, int f) { return x + 4 + 6 * f; }

// column of partial i (0..12) for observation o; -1 for constant frame 0
__device__ inline int col_of(const BaDev& d, int f, int p, int i)
{
    if (i < 4) return i;
    if (i < 10) return f == 0 ? -1 : 4 + 6 * (f - 1) + (i - 4);
    return d.nc + 3 * p + (i - 10);
}

__device__ inline void block_add_double(double v, double* slot)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(slot, v);
}

__device__ inline void block_max_double(double v, double* slot)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* s = reinterpret_cast<unsigned long long*>(slot);
        unsigned long long old = *s, assumed;
        do {
            assumed = old;
            if (__longlong_as_double(assumed) >= v) break;
            old = atomicCAS(s, assumed, __double_as_longlong(v));
        } while (old != assumed);
    }
}

// residuals + Jacobians (jac = 1) or cost only, at parameters xs
__global__ __launch_bounds__(128) void ba_eval(BaDev d, const double* xs, int jac, double* cost_slot)
{
    const int o = blockIdx.x * 128 + threadIdx.x;
    double c = 0;
    if (o < d.no) {
        const int f = d.of[o], p = d.op[o];
        double r[2], J[2][NJ];
        project(xs, xs + 4 + 6 * f, xs + 4 + 6 * d.nf + 3 * p, d.oxy[2 * o], d.oxy[2 * o + 1], r, jac ? J : nullptr);
        const double sq = r[0] * r[0] + r[1] * r[1];
        if (d.loss == SLAM_LOSS_NONE) {
            c = 0.5 * sq;
        } else {
            double rho[3];
            loss_eval(d.loss, d.a, sq, rho);
            c = 0.5 * rho[0];
            if (jac) {
                const double sqrt_rho1 = sqrt(rho[1]);
                double residual_scaling, alpha_sq_norm;
                if (sq == 0.0 || rho[2] <= 0.0) { residual_scaling = sqrt_rho1; alpha_sq_norm = 0.0; }
                else {
                    const double D = 1.0 + 2.0 * sq * rho[2] / rho[1];
                    const double alpha = 1.0 - sqrt(D);
                    residual_scaling = sqrt_rho1 / (1 - alpha);
                    alpha_sq_norm = alpha / sq;
                }
                if (alpha_sq_norm == 0.0) {
                    for (int i = 0; i < NJ; i++) { J[0][i] *= sqrt_rho1; J[1][i] *= sqrt_rho1; }
                } else {
                    for (int i = 0; i < NJ; i++) {
                        const double rtj = J[0][i] * r[0] + J[1][i] * r[1];
                        J[0][i] = sqrt_rho1 * (J[0][i] - alpha_sq_norm * r[0] * rtj);
                        J[1][i] = sqrt_rho1 * (J[1][i] - alpha_sq_norm * r[1] * rtj);
                    }
                }
                r[0] *= residual_scaling;
                r[1] *= residual_scaling;
            }
        }
        if (jac) {
            d.r[2 * o] = r[0];
            d.r[2 * o + 1] = r[1];
            double* Jo = d.J + (size_t)o * 2 * NJ;
            for (int i = 0; i < NJ; i++) { Jo[i] = J[0][i]; Jo[NJ + i] = J[1][i]; }
        }
    }
    if (!isfinite(c)) c = INFINITY;
    block_add_double(c, cost_slot);
}

// unscaled column norms^2 (iteration 0) or unscaled gradient J'f (accumulated into out)
__global__ __launch_bounds__(128) void ba_colsum(BaDev d, int what, double* out)
{
    const int o = blockIdx.x * 128 + threadIdx.x;
    if (o >= d.no) return;
    const int f = d.of[o], p = d.op[o];
    const double* Jo = d.J + (size_t)o * 2 * NJ;
    for (int i = 0; i < NJ; i++) {
        const int cidx = col_of(d, f, p, i);
        if (cidx < 0) continue;
        const double v = what == 0 ? Jo[i] * Jo[i] + Jo[NJ + i] * Jo[NJ + i]
                                   : Jo[i] * d.r[2 * o] + Jo[NJ + i] * d.r[2 * o + 1];
        atomicAdd(&out[cidx], v);
    }
}

__global__ __launch_bounds__(256) void ba_finish_scale(double* s, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) s[i] = 1.0 / (1.0 + sqrt(s[i]));
}

// g <- g .* scale ; gmax(unscaled) into red[3]
__global__ __launch_bounds__(256) void ba_scale_grad(BaDev d, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    double m = 0;
    if (i < n) {
        m = fabs(d.g[i]);
        d.g[i] *= d.scale[i];
    }
    block_max_double(m, &d.red[3]);
}

// the point pass: build S (camera block + damping is added by ba_cam_diag),
// rc, Vinv, per-observation W blocks.  One thread per point, S in LDS.
__global__ __launch_bounds__(256) void ba_point(BaDev d)
{
    extern __shared__ double Sl[];   // nc * nc + nc
    const int nc = d.nc;
    for (int i = threadIdx.x; i < nc * nc + nc; i += 256) Sl[i] = 0;
    __syncthreads();
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < d.np) {
        const int o0 = d.pstart[p], o1 = d.pstart[p + 1];
        double V[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        double dg[3] = {0, 0, 0};
        for (int q = o0; q < o1; q++) {
            const int o = d.plist[q], f = d.of[o];
            const double* Jo = d.J + (size_t)o * 2 * NJ;
            double js[2][NJ];
            int cols[NJ];
            for (int i = 0; i < NJ; i++) {
                cols[i] = col_of(d, f, p, i);
                const double s = cols[i] >= 0 ? d.scale[cols[i]] : 0.0;
                js[0][i] = Jo[i] * s;
                js[1][i] = Jo[NJ + i] * s;
            }
            // U (camera x camera) contribution of this observation
            for (int i = 0; i < 10; i++) {
                if (cols[i] < 0) continue;
                for (int j = 0; j < 10; j++) {
                    if (cols[j] < 0) continue;
                    atomicAdd(&Sl[cols[i] * nc + cols[j]], js[0][i] * js[0][j] + js[1][i] * js[1][j]);
                }
            }
            for (int i = 0; i < 3; i++) {
                for (int j = 0; j < 3; j++)
                    V[i * 3 + j] += js[0][10 + i] * js[0][10 + j] + js[1][10 + i] * js[1][10 + j];
                dg[i] += js[0][10 + i] * js[0][10 + i] + js[1][10 + i] * js[1][10 + i];
            }
            double* w = d.wobs + (size_t)o * 30;
            for (int i = 0; i < 10; i++)
                for (int k = 0; k < 3; k++)
                    w[i * 3 + k] = cols[i] < 0 ? 0.0 : js[0][i] * js[0][10 + k] + js[1][i] * js[1][10 + k];
        }
        // LM damping on the point block: clamp(diag) / radius
        for (int k = 0; k < 3; k++) V[k * 4] += fmin(fmax(dg[k], 1e-6), 1e32) / d.radius;
        // 3x3 Cholesky inverse
        double L[9];
        for (int i = 0; i < 9; i++) L[i] = V[i];
        bool ok = true;
        for (int j = 0; j < 3 && ok; j++) {
            double s = L[j * 3 + j];
            for (int k = 0; k < j; k++) s -= L[j * 3 + k] * L[j * 3 + k];
            if (!(s > 0.0) || !isfinite(s)) { ok = false; break; }
            const double dd = sqrt(s);
            L[j * 3 + j] = dd;
            for (int i = j + 1; i < 3; i++) {
                double t = L[i * 3 + j];
                for (int k = 0; k < j; k++) t -= L[i * 3 + k] * L[j * 3 + k];
                L[i * 3 + j] = t / dd;
            }
        }
        double Vi[9];
        if (ok) {
            for (int cc = 0; cc < 3; cc++) {
                double e[3] = {0, 0, 0};
                e[cc] = 1;
                for (int i = 0; i < 3; i++) { double t = e[i]; for (int k = 0; k < i; k++) t -= L[i * 3 + k] * e[k]; e[i] = t / L[i * 3 + i]; }
                for (int i = 2; i >= 0; i--) { double t = e[i]; for (int k = i + 1; k < 3; k++) t -= L[k * 3 + i] * e[k]; e[i] = t / L[i * 3 + i]; }
                for (int rr = 0; rr < 3; rr++) Vi[rr * 3 + cc] = e[rr];
            }
        } else {
            for (int i = 0; i < 9; i++) Vi[i] = NAN;
            d.red[5] = 1.0;   // signals a failed linear solve
        }
        for (int i = 0; i < 9; i++) d.Vinv[(size_t)p * 9 + i] = Vi[i];
        const double* gp = d.g + nc + 3 * p;
        // Schur: S -= W_p Vinv W_p' ; rc -= W_p Vinv g_p  (W_p = sum of the obs blocks)
        for (int q1 = o0; q1 < o1; q1++) {
            const int oa = d.plist[q1], fa = d.of[oa];
            const double* wa = d.wobs + (size_t)oa * 30;
            for (int i = 0; i < 10; i++) {
                const int ci = col_of(d, fa, p, i);
                if (ci < 0) continue;
                double WV[3];
                for (int k = 0; k < 3; k++)
                    WV[k] = wa[i * 3 + 0] * Vi[0 * 3 + k] + wa[i * 3 + 1] * Vi[1 * 3 + k] + wa[i * 3 + 2] * Vi[2 * 3 + k];
                atomicAdd(&Sl[nc * nc + ci], -(WV[0] * gp[0] + WV[1] * gp[1] + WV[2] * gp[2]));
                for (int q2 = o0; q2 < o1; q2++) {
                    const int ob = d.plist[q2], fb = d.of[ob];
                    const double* wb = d.wobs + (size_t)ob * 30;
                    for (int j = 0; j < 10; j++) {
                        const int cj = col_of(d, fb, p, j);
                        if (cj < 0) continue;
                        atomicAdd(&Sl[ci * nc + cj], -(WV[0] * wb[j * 3] + WV[1] * wb[j * 3 + 1] + WV[2] * wb[j * 3 + 2]));
                    }
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nc * nc; i += 256)
        if (Sl[i] != 0.0) atomicAdd(&d.S[i], Sl[i]);
    for (int i = threadIdx.x; i < nc; i += 256)
        if (Sl[nc * nc + i] != 0.0) atomicAdd(&d.rc[i], Sl[nc * nc + i]);
}

// camera damping: diag(U) (the scaled column norms of the camera columns,
// clamped) / radius, and rc += g_c.  Runs after ba_point; U's diagonal is read
// from the accumulated camera-only column norms in `cdiag`.
__global__ __launch_bounds__(64) void ba_cam_diag(BaDev d, const double* cdiag)
{
    const int i = threadIdx.x + blockIdx.x * 64;
    if (i >= d.nc) return;
    d.S[i * d.nc + i] += fmin(fmax(cdiag[i], 1e-6), 1e32) / d.radius;
    d.rc[i] += d.g[i];
}

// scaled camera column norms (diag of U) from the per-observation Jacobians
__global__ __launch_bounds__(128) void ba_cam_colnorm(BaDev d, double* cdiag)
{
    const int o = blockIdx.x * 128 + threadIdx.x;
    if (o >= d.no) return;
    const int f = d.of[o], p = d.op[o];
    const double* Jo = d.J + (size_t)o * 2 * NJ;
    for (int i = 0; i < 10; i++) {
        const int cidx = col_of(d, f, p, i);
        if (cidx < 0) continue;
        const double s = d.scale[cidx];
        const double a = Jo[i] * s, b = Jo[NJ + i] * s;
        atomicAdd(&cdiag[cidx], a * a + b * b);
    }
}

// back substitution per point + negation + finiteness flag
__global__ __launch_bounds__(256) void ba_backsub(BaDev d, const double* yc)
{
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < d.np) {
        const int o0 = d.pstart[p], o1 = d.pstart[p + 1];
        double t[3] = {d.g[d.nc + 3 * p], d.g[d.nc + 3 * p + 1], d.g[d.nc + 3 * p + 2]};
        for (int q = o0; q < o1; q++) {
            const int o = d.plist[q], f = d.of[o];
            const double* w = d.wobs + (size_t)o * 30;
            for (int i = 0; i < 10; i++) {
                const int ci = col_of(d, f, p, i);
                if (ci < 0) continue;
                for (int k = 0; k < 3; k++) t[k] -= w[i * 3 + k] * yc[ci];
            }
        }
        const double* Vi = d.Vinv + (size_t)p * 9;
        for (int k = 0; k < 3; k++) {
            const double y = Vi[3 * k] * t[0] + Vi[3 * k + 1] * t[1] + Vi[3 * k + 2] * t[2];
            if (!isfinite(y)) d.red[5] = 1.0;
            d.step[d.nc + 3 * p + k] = -y;
        }
    }
    if (p < d.nc) {
        const double y = yc[p];
        if (!isfinite(y)) d.red[5] = 1.0;
        d.step[p] = -y;
    }
}

// model cost change -(J_s step).(f + J_s step / 2), candidate x + step .* scale,
// squared step norm
__global__ __launch_bounds__(128) void ba_model(BaDev d)
{
    const int o = blockIdx.x * 128 + threadIdx.x;
    double m = 0;
    if (o < d.no) {
        const int f = d.of[o], p = d.op[o];
        const double* Jo = d.J + (size_t)o * 2 * NJ;
        double mr0 = 0, mr1 = 0;
        for (int i = 0; i < NJ; i++) {
            const int c = col_of(d, f, p, i);
            if (c < 0) continue;
            const double s = d.scale[c] * d.step[c];
            mr0 += Jo[i] * s;
            mr1 += Jo[NJ + i] * s;
        }
        m = -(mr0 * (d.r[2 * o] + mr0 / 2.0) + mr1 * (d.r[2 * o + 1] + mr1 / 2.0));
    }
    block_add_double(m, &d.red[2]);
}

// candidate parameters in the full layout (frame 0 copied), step norm^2
__global__ __launch_bounds__(256) void ba_candidate(BaDev d, int N)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    double sn = 0;
    if (i < N) {
        // tangent index i -> full layout index
        int full;
        if (i < 4) full = i;
        else if (i < d.nc) full = i + 6;          // skip frame 0's 6 entries
        else full = 4 + 6 * d.nf + (i - d.nc);
        const double delta = d.step[i] * d.scale[i];
        d.xc[full] = d.x[full] + delta;
        sn = delta * delta;
    }
    if (i < 6) d.xc[4 + i] = d.x[4 + i];
    block_add_double(sn, &d.red[4]);
}

}  // namespace

int ba_solve(slam_ctx* c, double* K4, int nf, double* ext6, int np, double* pts3, int no, const int32_t* of,
             const int32_t* op, const double* oxy, int loss, double a, int max_iters, slam_ba_summary* sum)
{
    if (max_iters <= 0) max_iters = 50;
    const int nc = 4 + 6 * (nf - 1), N = nc + 3 * np, NX = 4 + 6 * nf + 3 * np;
    std::memset(sum, 0, sizeof(*sum));
    sum->num_residuals = 2 * no;
    sum->usable = 1;
    if ((size_t)(nc * nc + nc) * 8 > 150 * 1024) return set_err(c, SLAM_E_UNSUPPORTED, "BA window too large for LDS");
    hipStream_t s = c->stream;

    // observations grouped by point (CSR), host side
    std::vector<int> pstart(np + 1, 0), plist(no > 0 ? no : 1);
    for (int o = 0; o < no; o++) pstart[op[o] + 1]++;
    for (int p = 0; p < np; p++) pstart[p + 1] += pstart[p];
    {
        std::vector<int> fill(np, 0);
        for (int o = 0; o < no; o++) plist[pstart[op[o]] + fill[op[o]]++] = o;
    }
    std::vector<double> x(NX);
    std::memcpy(x.data(), K4, 32);
    std::memcpy(x.data() + 4, ext6, sizeof(double) * 6 * nf);
    std::memcpy(x.data() + 4 + 6 * nf, pts3, sizeof(double) * 3 * np);

    // device layout
    size_t off = 0;
    auto carve = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_of = carve(4 * (size_t)no), o_op = carve(4 * (size_t)no), o_oxy = carve(16 * (size_t)no),
                 o_ps = carve(4 * (size_t)(np + 1)), o_pl = carve(4 * (size_t)(no > 0 ? no : 1)),
                 o_x = carve(8 * (size_t)NX), o_xc = carve(8 * (size_t)NX), o_r = carve(16 * (size_t)no),
                 o_J = carve(8 * 2 * NJ * (size_t)no), o_sc = carve(8 * (size_t)N), o_g = carve(8 * (size_t)N),
                 o_S = carve(8 * (size_t)nc * nc), o_rc = carve(8 * (size_t)nc), o_Vi = carve(72 * (size_t)np),
                 o_w = carve(240 * (size_t)no), o_st = carve(8 * (size_t)N), o_red = carve(8 * 16),
                 o_cd = carve(8 * (size_t)nc), o_info = carve(16);
    SLAM_HIP(c, c->ba_par.ensure(off));
    char* base = c->ba_par.as<char>();
    BaDev d;
    d.nf = nf; d.np = np; d.no = no; d.nc = nc; d.loss = loss; d.a = a;
    d.of = (const int*)(base + o_of); d.op = (const int*)(base + o_op); d.oxy = (const double*)(base + o_oxy);
    d.pstart = (const int*)(base + o_ps); d.plist = (const int*)(base + o_pl);
    d.x = (double*)(base + o_x); d.xc = (double*)(base + o_xc); d.r = (double*)(base + o_r); d.J = (double*)(base + o_J);
    d.scale = (double*)(base + o_sc); d.g = (double*)(base + o_g); d.S = (double*)(base + o_S);
    d.rc = (double*)(base + o_rc); d.Vinv = (double*)(base + o_Vi); d.wobs = (double*)(base + o_w);
    d.step = (double*)(base + o_st); d.red = (double*)(base + o_red);
    double* cdiag = (double*)(base + o_cd);
    int* dinfo = (int*)(base + o_info);
    d.radius = 1e4;
    if (no > 0) {
        SLAM_HIP(c, hipMemcpyAsync(base + o_of, of, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_op, op, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_oxy, oxy, 16 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_pl, plist.data(), 4 * (size_t)no, hipMemcpyHostToDevice, s));
    }
    SLAM_HIP(c, hipMemcpyAsync(base + o_ps, pstart.data(), 4 * (size_t)(np + 1), hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(d.x, x.data(), 8 * (size_t)NX, hipMemcpyHostToDevice, s));

    rocblas_handle hb;
    if (rocblas_create_handle(&hb) != rocblas_status_success) return set_err(c, SLAM_E_SOLVER, "rocblas_create_handle");
    rocblas_set_stream(hb, s);

    const unsigned gobs = (unsigned)((no + 127) / 128 > 0 ? (no + 127) / 128 : 1);
    const unsigned gpts = (unsigned)((np + 255) / 256 > 0 ? (np + 255) / 256 : 1);
    const unsigned gN = (unsigned)((N + 255) / 256);
    double red[8];
    auto read_red = [&]() -> int {
        SLAM_HIP(c, hipMemcpyAsync(red, d.red, sizeof(red), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipStreamSynchronize(s));
        return SLAM_OK;
    };
    int rc = SLAM_OK;
    auto evaluate_jac = [&]() -> int {
        SLAM_HIP(c, hipMemsetAsync(d.red, 0, sizeof(double) * 16, s));
        hipLaunchKernelGGL(ba_eval, dim3(gobs), dim3(128), 0, s, d, (const double*)d.x, 1, d.red + 0);
        SLAM_HIP(c, hipGetLastError());
        return SLAM_OK;
    };

    // iteration 0: cost, Jacobian, Jacobi scaling, gradient
    if ((rc = evaluate_jac())) goto done;
    SLAM_HIP(c, hipMemsetAsync(d.scale, 0, 8 * (size_t)N, s));
    if (no > 0) hipLaunchKernelGGL(ba_colsum, dim3(gobs), dim3(128), 0, s, d, 0, d.scale);
    hipLaunchKernelGGL(ba_finish_scale, dim3(gN), dim3(256), 0, s, d.scale, N);
    {
        double cost, xnorm = 0;
        for (int i = 0; i < 4; i++) xnorm += x[i] * x[i];
        for (int i = 4 + 6; i < NX; i++) xnorm += x[i] * x[i];
        xnorm = std::sqrt(xnorm);
        if ((rc = read_red())) goto done;
        cost = red[0];
        sum->initial_cost = cost;
        double radius = 1e4, decrease_factor = 2.0;
        int consecutive_invalid = 0, iter = 0;
        bool have_jac = true;
        for (;;) {
            if (have_jac) {
                SLAM_HIP(c, hipMemsetAsync(d.g, 0, 8 * (size_t)N, s));
                SLAM_HIP(c, hipMemsetAsync(d.red + 3, 0, 8, s));
                if (no > 0) hipLaunchKernelGGL(ba_colsum, dim3(gobs), dim3(128), 0, s, d, 1, d.g);
                hipLaunchKernelGGL(ba_scale_grad, dim3(gN), dim3(256), 0, s, d, N);
                if ((rc = read_red())) goto done;
                have_jac = false;
                if (red[3] <= 1e-10) { sum->termination = 1; break; }
            }
            if (iter >= max_iters) { sum->termination = 0; break; }
            iter++;
            d.radius = radius;
            SLAM_HIP(c, hipMemsetAsync(d.S, 0, 8 * (size_t)nc * nc, s));
            SLAM_HIP(c, hipMemsetAsync(d.rc, 0, 8 * (size_t)nc, s));
            SLAM_HIP(c, hipMemsetAsync(cdiag, 0, 8 * (size_t)nc, s));
            SLAM_HIP(c, hipMemsetAsync(d.red, 0, sizeof(double) * 16, s));
            if (no > 0) hipLaunchKernelGGL(ba_cam_colnorm, dim3(gobs), dim3(128), 0, s, d, cdiag);
            hipLaunchKernelGGL(ba_point, dim3(gpts), dim3(256), (size_t)(nc * nc + nc) * 8, s, d);
            hipLaunchKernelGGL(ba_cam_diag, dim3((nc + 63) / 64), dim3(64), 0, s, d, (const double*)cdiag);
            SLAM_HIP(c, hipGetLastError());
            // reduced camera system: S y_c = rc  (rocSOLVER Cholesky)
            rocsolver_dpotrf(hb, rocblas_fill_lower, nc, d.S, nc, dinfo);
            rocsolver_dpotrs(hb, rocblas_fill_lower, nc, 1, d.S, nc, d.rc, nc);
            int info = 0;
            SLAM_HIP(c, hipMemcpyAsync(&info, dinfo, 4, hipMemcpyDeviceToHost, s));
            hipLaunchKernelGGL(ba_backsub, dim3((unsigned)std::max((np + 255) / 256, (nc + 255) / 256)), dim3(256), 0,
                               s, d, (const double*)d.rc);
            if (no > 0) hipLaunchKernelGGL(ba_model, dim3(gobs), dim3(128), 0, s, d);
            hipLaunchKernelGGL(ba_candidate, dim3(gN), dim3(256), 0, s, d, N);
            hipLaunchKernelGGL(ba_eval, dim3(gobs), dim3(128), 0, s, d, (const double*)d.xc, 0, d.red + 1);
            SLAM_HIP(c, hipGetLastError());
            if ((rc = read_red())) goto done;
            const bool solved = info == 0 && red[5] == 0.0;
            const double mcc = red[2];
            const bool valid = solved && mcc > 0.0;
            if (!valid) {
                if (++consecutive_invalid >= 5) { sum->termination = 3; sum->usable = 0; break; }
                radius /= decrease_factor;
                decrease_factor *= 2.0;
                if (radius <= 1e-32) { sum->termination = 2; break; }
                continue;
            }
            consecutive_invalid = 0;
            double cand = red[1];
            if (!std::isfinite(cand)) cand = DBL_MAX;
            const double snorm = std::sqrt(red[4]);
            if (snorm <= 1e-8 * (xnorm + 1e-8)) { sum->termination = 1; break; }
            if (std::fabs(cost - cand) <= 1e-6 * cost) { sum->termination = 1; break; }
            const double rel = (cost - cand) / mcc;
            if (rel > 1e-3) {
                SLAM_HIP(c, hipMemcpyAsync(d.x, d.xc, 8 * (size_t)NX, hipMemcpyDeviceToDevice, s));
                SLAM_HIP(c, hipMemcpyAsync(x.data(), d.xc, 8 * (size_t)NX, hipMemcpyDeviceToHost, s));
                if ((rc = evaluate_jac())) goto done;
                if ((rc = read_red())) goto done;
                cost = red[0];
                xnorm = 0;
                for (int i = 0; i < 4; i++) xnorm += x[i] * x[i];
                for (int i = 4 + 6; i < NX; i++) xnorm += x[i] * x[i];
                xnorm = std::sqrt(xnorm);
                have_jac = true;
                const double qq = 2.0 * rel - 1.0;
                radius = radius / std::fmax(1.0 / 3.0, 1.0 - qq * qq * qq);
                radius = std::fmin(1e16, radius);
                decrease_factor = 2.0;
                sum->successful_steps++;
            } else {
                radius /= decrease_factor;
                decrease_factor *= 2.0;
                if (radius <= 1e-32) { sum->termination = 2; break; }
            }
        }
        sum->iterations = iter;
        sum->final_cost = cost;
    }
    SLAM_HIP(c, hipMemcpyAsync(x.data(), d.x, 8 * (size_t)NX, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    std::memcpy(K4, x.data(), 32);
    std::memcpy(ext6 + 6, x.data() + 4 + 6, sizeof(double) * 6 * (nf - 1));
    std::memcpy(pts3, x.data() + 4 + 6 * nf, sizeof(double) * 3 * np);
done:
    rocblas_destroy_handle(hb);
    return rc;
}

}  // namespace slamhip
