// Windowed bundle adjustment on gfx950 (FP64), replacing the reference's Ceres
// call site bundleAdjustment (src/mainModule/bundleAdjustment/
// bundleAdjustment.cpp:73-129): same parameter blocks (shared free intrinsics
// {fx, fy, cx, cy}, per-frame angle-axis + t with frame 0 constant, points),
// same residual (ProjectionCostFunctor :15-41), same losses (getLossFunction
// :131-151, Ceres Corrector), same Levenberg-Marquardt trust region with
// Jacobi scaling and Schur elimination of the points (Options :108-114).
//
// Device side:
//   ba_eval      one thread per observation: residual + 2 x 13 Jacobian by
//                forward-mode jets (ceres/jet.h arithmetic), loss correction,
//                cost reduced per workgroup.
//   ba_cam_gram  per new Jacobian: [U | g_c] = sum_o J_c' [J_c | f] over the
//                camera columns, register-tiled in workgroup-private slices
//                (no atomics), summed by ba_sum_parts.
//   per LM iteration:
//   ba_point     one thread per point (observations grouped by point, CSR):
//                scaled V_p + D_p / radius, its 3x3 Cholesky inverse, the
//                per-observation W blocks J_c' J_p.
//   ba_schur     [-sum_p W_p V_p^-1 W_p' | -sum_p W_p V_p^-1 g_p], same tiling;
//                ba_schur_reduce adds U, the camera damping and g_c: the
//                reduced camera system S y_c = rc.
//   ba_chol_solve  Cholesky + both triangular solves of S in one workgroup's
//                LDS (nc = 4 + 6 (W - 1): 46 at W = 8).
//   ba_backsub   one thread per point: y_p = V_p^-1 (g_p - W_p' y_c); model cost
//                change J_s step; candidate x + step .* scale.
// The host keeps the scalar LM state (radius, decrease factor, tolerances) and
// makes exactly the oracle's accept / reject decisions (oracle/ba.c).
#include <cfloat>
#include <cstdlib>
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

// workgroup reductions into one global slot: wave shuffles, then the waves'
// partials through LDS, then one atomic per workgroup (every thread calls)
__device__ inline double block_reduce(double v, bool is_max)
{
    __shared__ double wpart[16];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double w = __shfl_xor(v, o, 64);
        v = is_max ? fmax(v, w) : v + w;
    }
    __syncthreads();   // wpart may still be read by a previous call
    if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = wpart[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) t = is_max ? fmax(t, wpart[w]) : t + wpart[w];
    return t;
}

__device__ inline void block_add_double(double v, double* slot)
{
    const double t = block_reduce(v, false);
    if (threadIdx.x == 0) atomicAdd(slot, t);
}

__device__ inline void block_max_double(double v, double* slot)
{
    const double t = block_reduce(v, true);
    if (threadIdx.x == 0) {
        unsigned long long* s = reinterpret_cast<unsigned long long*>(slot);
        unsigned long long old = *s, assumed;
        do {
            assumed = old;
            if (__longlong_as_double(assumed) >= t) break;
            old = atomicCAS(s, assumed, __double_as_longlong(t));
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

// Camera-block reductions.  The camera part of the normal equations is small
// and dense (nc = 4 + 6 (W - 1) columns, 46 at W = 8) while the sums run over
// tens of thousands of observations / points, so every camera reduction is
// one shape: out[i][j] = sum_r A[r][i] * B[r][j] over rank-1 terms r, i < nc,
// j <= nc (column nc carries the right-hand side).  Each workgroup stages
// kVec rank-1 vectors at a time in LDS (dense, zero-filled to 16 T), each of
// its 16 x 16 threads owns a T x T register tile of the output (rows ty + 16 a,
// columns tx + 16 b), and the workgroup's tile goes to a private slice of
// `part`; ba_sum_parts adds the slices in a fixed order.  No atomics, so the
// camera system is bit-for-bit reproducible run to run.
constexpr int kVec = 48;
constexpr int kGramBlocks = 1024;   // upper bound on workgroup slices

template <int T>
__device__ inline void gram_accumulate(const double* A, const double* B, double (&acc)[T][T], int ty, int tx)
{
    constexpr int NCP = 16 * T;
    for (int r = 0; r < kVec; r++) {
        double a[T], b[T];
#pragma unroll
        for (int u = 0; u < T; u++) { a[u] = A[r * NCP + ty + 16 * u]; b[u] = B[r * NCP + tx + 16 * u]; }
#pragma unroll
        for (int u = 0; u < T; u++)
#pragma unroll
            for (int v = 0; v < T; v++) acc[u][v] = fma(a[u], b[v], acc[u][v]);
    }
}

template <int T>
__device__ inline void gram_store(const BaDev& d, const double (&acc)[T][T], int ty, int tx, double* out)
{
    const int ld = d.nc + 1;
#pragma unroll
    for (int u = 0; u < T; u++)
#pragma unroll
        for (int v = 0; v < T; v++) {
            const int i = ty + 16 * u, j = tx + 16 * v;
            if (i < d.nc && j < ld) out[i * ld + j] = acc[u][v];
        }
}

// camera column of partial ii (0..9) of an observation in frame f (frame 0: -1)
__device__ inline int cam_col(int f, int ii) { return ii < 4 ? ii : f == 0 ? -1 : 4 + 6 * (f - 1) + (ii - 4); }

// [U | g_c] partials: rank-1 terms are the (scaled) camera rows of each
// observation's Jacobian, augmented with the residual.  scl == nullptr gives
// the unscaled Gram matrix (iteration 0: its diagonal is the Jacobi column norm).
// Staging: zero the tile, then one thread per (observation, row, partial)
// scatters J into its column (coalesced J reads, one writer per LDS cell).
template <int T>
__global__ __launch_bounds__(256) void ba_cam_gram(BaDev d, const double* scl, double* part)
{
    constexpr int NCP = 16 * T, kObs = kVec / 2;
    __shared__ double B[kVec * NCP];
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15, nc = d.nc;
    double acc[T][T];
#pragma unroll
    for (int u = 0; u < T; u++)
#pragma unroll
        for (int v = 0; v < T; v++) acc[u][v] = 0;
    const int nchunk = (d.no + kObs - 1) / kObs;
    for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        for (int e = tid; e < kVec * NCP; e += 256) B[e] = 0;
        __syncthreads();
        for (int e = tid; e < kObs * 2 * 11; e += 256) {
            const int lo = e / 22, rr = e - 22 * lo, row = rr / 11, ii = rr - 11 * row;
            const int o = ch * kObs + lo;
            if (o >= d.no) continue;
            double* Bt = B + (2 * lo + row) * NCP;
            if (ii == 10) { Bt[nc] = d.r[2 * o + row]; continue; }
            const int col = cam_col(d.of[o], ii);
            if (col < 0) continue;
            Bt[col] = d.J[(size_t)o * 2 * NJ + row * NJ + ii] * (scl ? scl[col] : 1.0);
        }
        __syncthreads();
        gram_accumulate<T>(B, B, acc, ty, tx);
        __syncthreads();
    }
    gram_store<T>(d, acc, ty, tx, part + (size_t)blockIdx.x * nc * (nc + 1));
}

// Schur partials: per point the three columns of W_p = sum_o J_c' J_p (scaled,
// from wobs) augmented with g_p, against -Y_p = -W_p V_p^-1; the sum is
// [-sum W V^-1 W' | -sum W V^-1 g_p].  16 points (48 rank-1 terms) per chunk.
// A chunk's observations are one contiguous CSR range: their ids, frames and
// the points' V^-1 go to LDS first, then one thread per (point, partial, k)
// sums its point's observations into W (deterministic order, one writer per
// LDS cell except the frame columns, which differ per observation frame).
constexpr int kSchurObs = 512;   // LDS capacity for a chunk's observation list

template <int T>
__global__ __launch_bounds__(256) void ba_schur(BaDev d, double* part)
{
    constexpr int NCP = 16 * T, kPts = kVec / 3;
    __shared__ double A[kVec * NCP];
    __shared__ double B[kVec * NCP];
    __shared__ double Vi[kPts * 9];
    __shared__ int qs[kPts + 1];
    __shared__ int lobs[kSchurObs], lf[kSchurObs];
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15, nc = d.nc;
    double acc[T][T];
#pragma unroll
    for (int u = 0; u < T; u++)
#pragma unroll
        for (int v = 0; v < T; v++) acc[u][v] = 0;
    const int nchunk = (d.np + kPts - 1) / kPts;
    for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int p0 = ch * kPts, npts = min(kPts, d.np - p0);
        for (int e = tid; e < kVec * NCP; e += 256) B[e] = 0;
        if (tid <= kPts) qs[tid] = d.pstart[p0 + min(tid, npts)];
        for (int e = tid; e < kPts * 9; e += 256) Vi[e] = e < npts * 9 ? d.Vinv[(size_t)p0 * 9 + e] : 0.0;
        __syncthreads();
        const int q0 = qs[0], nq = qs[npts] - q0;
        const bool staged = nq <= kSchurObs;
        if (staged)
            for (int e = tid; e < nq; e += 256) {
                const int o = d.plist[q0 + e];
                lobs[e] = o;
                lf[e] = d.of[o];
            }
        __syncthreads();
        for (int e = tid; e < kPts * 31; e += 256) {
            const int lp = e / 31, rr = e - 31 * lp;
            if (lp >= npts) continue;
            if (rr == 30) {
                for (int k = 0; k < 3; k++) B[(3 * lp + k) * NCP + nc] = d.g[nc + 3 * (p0 + lp) + k];
                continue;
            }
            const int ii = rr / 3, k = rr - 3 * ii;
            double* Bt = B + (3 * lp + k) * NCP;
            double ks = 0;   // intrinsics columns: summed over all observations
            for (int q = qs[lp]; q < qs[lp + 1]; q++) {
                const int o = staged ? lobs[q - q0] : d.plist[q];
                const double w = d.wobs[(size_t)o * 30 + ii * 3 + k];
                if (ii < 4) ks += w;
                else {
                    const int col = cam_col(staged ? lf[q - q0] : d.of[o], ii);
                    if (col >= 0) Bt[col] += w;
                }
            }
            if (ii < 4) Bt[ii] = ks;
        }
        __syncthreads();
        for (int e = tid; e < kVec * NCP; e += 256) {
            const int r = e / NCP, i = e - r * NCP;
            const int lp = r / 3, k = r - 3 * lp;
            double v = 0;
            if (lp < npts && i < nc) {
                const double* w = B + 3 * lp * NCP + i;
                const double* vi = Vi + 9 * lp;
                v = -(w[0] * vi[k] + w[NCP] * vi[3 + k] + w[2 * NCP] * vi[6 + k]);
            }
            A[e] = v;
        }
        __syncthreads();
        gram_accumulate<T>(A, B, acc, ty, tx);
        __syncthreads();
    }
    gram_store<T>(d, acc, ty, tx, part + (size_t)blockIdx.x * nc * (nc + 1));
}

// sum of the nblk workgroup slices per entry: 16 entries x 16 partial sums per
// workgroup (coalesced rows of 16 entries), then a fixed-order LDS tree
__device__ inline double sum_slices(const double* part, int nblk, int E, int e, bool valid)
{
    __shared__ double red[256];
    const int g = threadIdx.x >> 4;
    double s = 0;
    if (valid)
        for (int b = g; b < nblk; b += 16) s += part[(size_t)b * E + e];
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int w = 8; w > 0; w >>= 1) {
        if (g < w) red[threadIdx.x] += red[threadIdx.x + 16 * w];
        __syncthreads();
    }
    return red[threadIdx.x & 15];
}

__global__ __launch_bounds__(256) void ba_sum_parts(const double* part, int nblk, int E, double* out)
{
    const int e = blockIdx.x * 16 + (threadIdx.x & 15);
    const double s = sum_slices(part, nblk, E, e, e < E);
    if (threadIdx.x < 16 && e < E) out[e] = s;
}

// reduced camera system from the Schur slices and [U | g_c]:
// S = U + diag(clamp(diag U)) / radius - sum W V^-1 W',  rc = g_c - sum W V^-1 g_p
__global__ __launch_bounds__(256) void ba_schur_reduce(BaDev d, const double* part, int nblk, const double* Ua)
{
    const int nc = d.nc, ld = nc + 1, E = nc * ld;
    const int e = blockIdx.x * 16 + (threadIdx.x & 15);
    const double s = sum_slices(part, nblk, E, e, e < E);
    if (threadIdx.x >= 16 || e >= E) return;
    const int i = e / ld, j = e - i * ld;
    if (j < nc) {
        double u = Ua[e];
        if (i == j) u += fmin(fmax(Ua[e], 1e-6), 1e32) / d.radius;
        d.S[i * nc + j] = u + s;
    } else {
        d.rc[i] = d.g[i] + s;
    }
}

// Jacobi scaling 1 / (1 + |column|): camera columns from diag of the unscaled
// Gram matrix, point columns summed over the point's observations (CSR).
__global__ __launch_bounds__(256) void ba_scale_init(BaDev d, const double* Ua, int N)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    double s = 0;
    if (i < d.nc) s = Ua[i * (d.nc + 1) + i];
    else {
        const int p = (i - d.nc) / 3, k = (i - d.nc) % 3;
        for (int q = d.pstart[p]; q < d.pstart[p + 1]; q++) {
            const double* Jo = d.J + (size_t)d.plist[q] * 2 * NJ;
            s += Jo[10 + k] * Jo[10 + k] + Jo[NJ + 10 + k] * Jo[NJ + 10 + k];
        }
    }
    d.scale[i] = 1.0 / (1.0 + sqrt(s));
}

// scaled gradient g = scale .* J'f; max |unscaled g| into red[3].  The camera
// part comes scaled from the Gram pass (column nc of [U | g_c]).
__global__ __launch_bounds__(256) void ba_grad(BaDev d, const double* Ua, int N)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    double m = 0;
    if (i < N) {
        if (i < d.nc) {
            const double gs = Ua[i * (d.nc + 1) + d.nc];
            d.g[i] = gs;
            m = fabs(gs / d.scale[i]);
        } else {
            const int p = (i - d.nc) / 3, k = (i - d.nc) % 3;
            double u = 0;
            for (int q = d.pstart[p]; q < d.pstart[p + 1]; q++) {
                const int o = d.plist[q];
                const double* Jo = d.J + (size_t)o * 2 * NJ;
                u += Jo[10 + k] * d.r[2 * o] + Jo[NJ + 10 + k] * d.r[2 * o + 1];
            }
            m = fabs(u);
            d.g[i] = u * d.scale[i];
        }
    }
    block_max_double(m, &d.red[3]);
}

// the point pass: scaled V_p + D_p / radius, its inverse, and the scaled
// per-observation W blocks J_c' J_p.  One thread per point.
__global__ __launch_bounds__(64) void ba_point(BaDev d)
{
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= d.np) return;
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
    double sn = 0, xx = 0;
    if (i < N) {
        // tangent index i -> full layout index
        int full;
        if (i < 4) full = i;
        else if (i < d.nc) full = i + 6;          // skip frame 0's 6 entries
        else full = 4 + 6 * d.nf + (i - d.nc);
        const double delta = d.step[i] * d.scale[i];
        const double v = d.x[full] + delta;
        d.xc[full] = v;
        sn = delta * delta;
        xx = v * v;
    }
    if (i < 6) d.xc[4 + i] = d.x[4 + i];
    block_add_double(sn, &d.red[4]);
    block_add_double(xx, &d.red[7]);
}

__device__ inline double readlane_f64(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// S y = rc for nc <= NP (48 or 64) in ONE wavefront, no LDS: lane i holds row i
// of S (padded with the identity to NP) and b_i.  Step j of the symmetric
// right-looking Cholesky updates, on lanes i > j, a_ik -= (a_ij a_kj) / a_jj for
// k > j with a_kj read from lane k (v_readlane, compile-time lane): the product
// is formed the same way on both sides of the diagonal, so the matrix stays
// exactly symmetric and lane i ends up holding both row i and column i of the
// unscaled factor (L_ik = a_ik / sqrt(a_kk)).  Forward solve rides along; the
// back solve is lane-local plus one broadcast per column.
template <int NP>
__global__ __launch_bounds__(64) void ba_chol_wave(BaDev d)
{
    const int n = d.nc, i = threadIdx.x;
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) a[k] = i < n && k < n ? d.S[i * n + k] : (i == k ? 1.0 : 0.0);
    double b = i < n ? d.rc[i] : 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const double ajj = readlane_f64(a[j], j);
        if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }
        const double inv = 1.0 / ajj;
        const double bj = readlane_f64(b, j);
        if (i > j) {
            const double aij = a[j];
#pragma unroll
            for (int k = j + 1; k < NP; k++) {
                const double akj = readlane_f64(a[j], k);
                a[k] = fma(-(aij * akj), inv, a[k]);
            }
            b = fma(-aij, bj * inv, b);
        } else {
#pragma unroll
            for (int k = j + 1; k < NP; k++) (void)readlane_f64(a[j], k);
        }
    }
    if (!ok) {
        if (i == 0) d.red[5] = 1.0;
        return;
    }
    double diag = 0;
#pragma unroll
    for (int k = 0; k < NP; k++) if (k == i) diag = a[k];
    const double rdi = 1.0 / sqrt(diag);
    b *= rdi;   // y_i
#pragma unroll
    for (int j = NP - 1; j >= 0; j--) {
        const double xj = readlane_f64(b, j) * readlane_f64(rdi, j);
        if (i < j) b = fma(-a[j] * rdi, xj, b);
        if (i == j) b = xj;
    }
    if (i < n) d.rc[i] = b;
}

// S y = rc for 64 < nc <= NP (96): thread i keeps row i in registers as in
// ba_chol_wave, but rows span two wavefronts, so column j (= row j, the matrix
// stays symmetric) and b_j are published by thread j into a double-buffered
// LDS row: one barrier per column; the back solve broadcasts x_j the same way.
template <int NP>
__global__ __launch_bounds__(128) void ba_chol_rows(BaDev d)
{
    __shared__ double rowbuf[2][NP + 1];
    __shared__ double xs[NP];
    const int n = d.nc, i = threadIdx.x;
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) a[k] = i < n && k < n ? d.S[i * n + k] : (i == k ? 1.0 : 0.0);
    double b = i < n ? d.rc[i] : 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        double* rb = rowbuf[j & 1];
        if (i == j) {
#pragma unroll
            for (int k = j; k < NP; k++) rb[k] = a[k];
            rb[NP] = b;
        }
        __syncthreads();
        const double ajj = rb[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }   // uniform: one pivot for all threads
        const double inv = 1.0 / ajj, bj = rb[NP];
        if (i > j && i < NP) {
            const double aij = a[j];
#pragma unroll
            for (int k = j + 1; k < NP; k++) a[k] = fma(-(aij * rb[k]), inv, a[k]);
            b = fma(-aij, bj * inv, b);
        }
    }
    if (!ok) {
        if (i == 0) d.red[5] = 1.0;
        return;
    }
    double diag = 1.0;
#pragma unroll
    for (int k = 0; k < NP; k++) if (k == i) diag = a[k];
    const double rdi = 1.0 / sqrt(diag);
    b *= rdi;   // y_i
#pragma unroll
    for (int j = NP - 1; j >= 0; j--) {
        if (i == j) xs[j] = b * rdi;
        __syncthreads();
        const double xj = xs[j];
        if (i < j) b = fma(-a[j] * rdi, xj, b);
        if (i == j) b = xj;
    }
    if (i < n) d.rc[i] = b;
}

// S y = rc in place on the reduced camera system, one workgroup of 16 x 16
// threads.  Factorisation: each thread keeps its T x T tile of S (rows
// ty + 16 u, columns tx + 16 v) in registers; step j updates the trailing
// lower triangle with a_ij a_kj / a_jj from column j, which the column's
// owners publish into a double-buffered LDS vector, so one barrier per column.
// L_ij = a_ij / sqrt(a_jj).  The forward solve rides along (thread per row);
// the back solve L' x = y is thread-per-row with one barrier per column, on
// L dumped to LDS.  A non-positive pivot sets red[5] (failed linear solve).
template <int T>
__global__ __launch_bounds__(256) void ba_chol_solve(BaDev d)
{
    constexpr int NCP = 16 * T;
    extern __shared__ double Al[];   // n * n (lower triangle of the unscaled factor)
    __shared__ double col[2][NCP];
    __shared__ double b[NCP], rd[NCP];
    const int n = d.nc, tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    double a[T][T];
#pragma unroll
    for (int u = 0; u < T; u++)
#pragma unroll
        for (int v = 0; v < T; v++) {
            const int i = ty + 16 * u, k = tx + 16 * v;
            a[u][v] = i < n && k < n ? d.S[i * n + k] : 0.0;
        }
    if (tid < n) b[tid] = d.rc[tid];
    // publish column 0
    if (tx == 0)
#pragma unroll
        for (int u = 0; u < T; u++) col[0][ty + 16 * u] = a[u][0];
    __syncthreads();
    bool ok = true;
    for (int j = 0; j < n; j++) {
        const double* cj = col[j & 1];
        const double ajj = cj[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }   // uniform: one pivot for all threads
        const double inv = 1.0 / ajj;
        if (tid == 0) rd[j] = 1.0 / sqrt(ajj);
        double ci[T], ck[T];
#pragma unroll
        for (int u = 0; u < T; u++) { ci[u] = cj[ty + 16 * u] * inv; ck[u] = cj[tx + 16 * u]; }
#pragma unroll
        for (int u = 0; u < T; u++)
#pragma unroll
            for (int v = 0; v < T; v++) {
                const int i = ty + 16 * u, k = tx + 16 * v;
                if (k > j && k <= i) a[u][v] = fma(-ci[u], ck[v], a[u][v]);
            }
        // forward solve: b_i -= a_ij b_j / a_jj, thread per row
        if (tid > j && tid < n) b[tid] = fma(-cj[tid], b[j] * inv, b[tid]);
        // publish column j + 1 (already updated by step j) into the other buffer
        const int jn = j + 1;
        if (jn < n && tx == (jn & 15)) {
            const int v = jn >> 4;
#pragma unroll
            for (int u = 0; u < T; u++)
#pragma unroll
                for (int vv = 0; vv < T; vv++)
                    if (vv == v) col[jn & 1][ty + 16 * u] = a[u][vv];
        }
        // keep the final column j (lower part) for the back solve
        if (tx == (j & 15)) {
            const int v = j >> 4;
#pragma unroll
            for (int u = 0; u < T; u++)
#pragma unroll
                for (int vv = 0; vv < T; vv++) {
                    const int i = ty + 16 * u;
                    if (vv == v && i >= j && i < n) Al[i * n + j] = a[u][vv];
                }
        }
        __syncthreads();
    }
    if (!ok) {
        if (tid == 0) d.red[5] = 1.0;
        return;
    }
    // y = D^-1/2 (forward-solved b); back solve L' x = y, x_j = y_j / d_j,
    // y_i -= L_ji x_j = a_ji rd_i x_j (i < j)
    if (tid < n) b[tid] *= rd[tid];
    __syncthreads();
    for (int j = n - 1; j >= 0; j--) {
        const double xj = b[j] * rd[j];
        if (tid < j) b[tid] = fma(-Al[j * n + tid] * rd[tid], xj, b[tid]);
        if (tid == j) d.rc[j] = xj;
        __syncthreads();
    }
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
    // reduced camera system in one workgroup's LDS: nc <= 136 (148 KB of 160)
    if (nc > 136) return set_err(c, SLAM_E_UNSUPPORTED, "BA window too large (more than 23 frames)");
    const int E = nc * (nc + 1);
    const int gT = nc + 1 <= 48 ? 3 : nc + 1 <= 64 ? 4 : nc + 1 <= 96 ? 6 : 9;
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
                 o_ua = carve(8 * (size_t)E), o_part = carve(8 * (size_t)E * kGramBlocks);
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
    double* Ua = (double*)(base + o_ua);      // [U | g_c], nc x (nc + 1)
    double* part = (double*)(base + o_part);  // per-workgroup slices of the camera reductions
    d.radius = 1e4;
    if (no > 0) {
        SLAM_HIP(c, hipMemcpyAsync(base + o_of, of, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_op, op, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_oxy, oxy, 16 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_pl, plist.data(), 4 * (size_t)no, hipMemcpyHostToDevice, s));
    }
    SLAM_HIP(c, hipMemcpyAsync(base + o_ps, pstart.data(), 4 * (size_t)(np + 1), hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(d.x, x.data(), 8 * (size_t)NX, hipMemcpyHostToDevice, s));

    const size_t chol_lds = (size_t)nc * nc * 8;
    const void* chol_fn = gT == 3 ? (const void*)ba_chol_solve<3> : gT == 4 ? (const void*)ba_chol_solve<4>
                        : gT == 6 ? (const void*)ba_chol_solve<6> : (const void*)ba_chol_solve<9>;
    if (chol_lds > 60 * 1024)
        SLAM_HIP(c, hipFuncSetAttribute(chol_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chol_lds));

    // camera reductions: workgroups in flight and the launch helpers
    int gblocks = 256;
    if (const char* ev = std::getenv("SLAMHIP_BA_BLOCKS")) gblocks = std::max(1, std::min(kGramBlocks, std::atoi(ev)));
    const int nbg = std::max(1, std::min(gblocks, (no + kVec / 2 - 1) / (kVec / 2)));
    const int nbs = std::max(1, std::min(gblocks, (np + kVec / 3 - 1) / (kVec / 3)));
    auto cam_gram = [&](const double* scl) {
        switch (gT) {
        case 3: hipLaunchKernelGGL(ba_cam_gram<3>, dim3(nbg), dim3(256), 0, s, d, scl, part); break;
        case 4: hipLaunchKernelGGL(ba_cam_gram<4>, dim3(nbg), dim3(256), 0, s, d, scl, part); break;
        case 6: hipLaunchKernelGGL(ba_cam_gram<6>, dim3(nbg), dim3(256), 0, s, d, scl, part); break;
        default: hipLaunchKernelGGL(ba_cam_gram<9>, dim3(nbg), dim3(256), 0, s, d, scl, part); break;
        }
        hipLaunchKernelGGL(ba_sum_parts, dim3((E + 15) / 16), dim3(256), 0, s, (const double*)part, nbg, E, Ua);
    };
    auto schur = [&]() {
        switch (gT) {
        case 3: hipLaunchKernelGGL(ba_schur<3>, dim3(nbs), dim3(256), 0, s, d, part); break;
        case 4: hipLaunchKernelGGL(ba_schur<4>, dim3(nbs), dim3(256), 0, s, d, part); break;
        case 6: hipLaunchKernelGGL(ba_schur<6>, dim3(nbs), dim3(256), 0, s, d, part); break;
        default: hipLaunchKernelGGL(ba_schur<9>, dim3(nbs), dim3(256), 0, s, d, part); break;
        }
        hipLaunchKernelGGL(ba_schur_reduce, dim3((E + 15) / 16), dim3(256), 0, s, d, (const double*)part, nbs,
                           (const double*)Ua);
    };
    auto chol = [&]() {
        if (nc <= 48) { hipLaunchKernelGGL(ba_chol_wave<48>, dim3(1), dim3(64), 0, s, d); return; }
        if (nc <= 64) { hipLaunchKernelGGL(ba_chol_wave<64>, dim3(1), dim3(64), 0, s, d); return; }
        if (nc <= 96) { hipLaunchKernelGGL(ba_chol_rows<96>, dim3(1), dim3(128), 0, s, d); return; }
        switch (gT) {
        case 3: hipLaunchKernelGGL(ba_chol_solve<3>, dim3(1), dim3(256), chol_lds, s, d); break;
        case 4: hipLaunchKernelGGL(ba_chol_solve<4>, dim3(1), dim3(256), chol_lds, s, d); break;
        case 6: hipLaunchKernelGGL(ba_chol_solve<6>, dim3(1), dim3(256), chol_lds, s, d); break;
        default: hipLaunchKernelGGL(ba_chol_solve<9>, dim3(1), dim3(256), chol_lds, s, d); break;
        }
    };
    const unsigned gobs = (unsigned)((no + 127) / 128 > 0 ? (no + 127) / 128 : 1);
    const unsigned gpts = (unsigned)((np + 63) / 64 > 0 ? (np + 63) / 64 : 1);
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

    // iteration 0: cost, Jacobian, Jacobi scaling
    if ((rc = evaluate_jac())) goto done;
    cam_gram(nullptr);
    hipLaunchKernelGGL(ba_scale_init, dim3(gN), dim3(256), 0, s, d, (const double*)Ua, N);
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
        // One host sync per LM iteration: the gradient of a new Jacobian, the
        // step, the candidate and its cost are queued together, then read back
        // in one copy.  A step computed alongside a gradient that turns out to
        // satisfy the gradient tolerance is simply discarded.
        for (;;) {
            SLAM_HIP(c, hipMemsetAsync(d.red, 0, sizeof(double) * 16, s));
            if (have_jac) {
                cam_gram(d.scale);
                hipLaunchKernelGGL(ba_grad, dim3(gN), dim3(256), 0, s, d, (const double*)Ua, N);
            }
            const bool stepping = iter < max_iters;
            if (stepping) {
                d.radius = radius;
                hipLaunchKernelGGL(ba_point, dim3(gpts), dim3(64), 0, s, d);
                schur();
                chol();
                hipLaunchKernelGGL(ba_backsub, dim3((unsigned)std::max((np + 255) / 256, (nc + 255) / 256)),
                                   dim3(256), 0, s, d, (const double*)d.rc);
                if (no > 0) hipLaunchKernelGGL(ba_model, dim3(gobs), dim3(128), 0, s, d);
                hipLaunchKernelGGL(ba_candidate, dim3(gN), dim3(256), 0, s, d, N);
                hipLaunchKernelGGL(ba_eval, dim3(gobs), dim3(128), 0, s, d, (const double*)d.xc, 0, d.red + 1);
            }
            SLAM_HIP(c, hipGetLastError());
            if ((rc = read_red())) goto done;
            if (have_jac) {
                have_jac = false;
                if (red[3] <= 1e-10) { sum->termination = 1; break; }
            }
            if (!stepping) { sum->termination = 0; break; }
            iter++;
            const bool solved = red[5] == 0.0;
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
                // accept: the candidate becomes x (pointer swap), its cost and
                // norm were reduced alongside it; re-linearise there
                std::swap(d.x, d.xc);
                cost = cand;
                xnorm = std::sqrt(red[7]);
                hipLaunchKernelGGL(ba_eval, dim3(gobs), dim3(128), 0, s, d, (const double*)d.x, 1, d.red + 0);
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
    return rc;
}

}  // namespace slamhip
