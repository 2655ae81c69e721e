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
//   ba_frame_gram per new Jacobian: [U | g_c] as per-frame 10 x 11 blocks
//                (K + the frame's extrinsics, residual column), chunked,
//                reduced per frame in order, assembled by ba_u_assemble.
//   per LM iteration:
//   ba_point     one thread per point (observations grouped by point, CSR):
//                scaled V_p + D_p / radius, its 3x3 Cholesky inverse, the
//                per-observation W blocks J_c' J_p and Y = W V_p^-1.
//   ba_pair_schur  per-frame-pair 10 x 11 blocks of sum Y_a W_b' over the
//                ordered observation pairs of each point (+ Y_a g_p on self
//                pairs); ba_s_assemble adds U, the camera damping and g_c:
//                the reduced camera system S y_c = rc.
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
    double* yobs;           // [no][10][3] wobs . V_p^-1
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

// Camera-block reductions, frame-structured.  An observation in frame f
// touches only the 10 camera columns K (4) + ext_f (6) (frame 0: K only), so
// every camera sum is a sum of 10 x 11 blocks:
//   [U | g_c]  = sum_f  B_f,      B_f  = sum_{o in f} J_c(o)' [J_c(o) | f_o]
//   S_schur    = sum_{fa,fb} C_fa,fb, C = sum over ordered observation pairs
//                (a, b) of one point, a in fa, b in fb, of Y_a W_b'
//                (W_o = J_c(o)' J_p(o), Y_o = W_o V_p^-1), rhs column Y_a g_p on
//                the self pairs a == b
// (camera rows / columns in local order K0..K3, ext0..ext5).  Observations
// (gram) and observation pairs (Schur) are bucketed on the host by frame /
// frame pair and cut into chunks of <= 64; one workgroup per chunk sums its
// 10 x 11 block (thread = entry, terms in chunk order), a segmented pass adds
// each bucket's chunks in order, and an assembly pass maps the blocks onto the
// dense nc x (nc + 1) systems.  Fixed order throughout: the camera system is
// bit-reproducible, with no atomics and no work on the ~90 % structural zeros
// that dense nc-wide tiles would multiply.
constexpr int kChunk = 64;
constexpr int kBlk = 110;    // 10 x 11 block entries

struct Chunk {
    int bucket;              // frame (gram) or fa * nf + fb (Schur)
    int start, len;          // range in the bucketed observation / pair list
};

// camera column of local partial ii (0..9) of an observation in frame f (frame 0 ext: -1)
__device__ inline int cam_col(int f, int ii) { return ii < 4 ? ii : f == 0 ? -1 : 4 + 6 * (f - 1) + (ii - 4); }

// B_f chunk: rows = (observation, residual row) of one frame, A[row] = scaled
// J_c row (scl == nullptr: unscaled, iteration 0's column norms) | residual
__global__ __launch_bounds__(128) void ba_frame_gram(BaDev d, const Chunk* __restrict__ ch,
                                                      const int* __restrict__ flist, const double* scl,
                                                      double* part)
{
    __shared__ double A[2 * kChunk][11];
    __shared__ int ob[kChunk];
    const Chunk c = ch[blockIdx.x];
    const int tid = threadIdx.x, f = c.bucket;
    if (tid < kChunk) ob[tid] = tid < c.len ? flist[c.start + tid] : 0;
    __syncthreads();
#pragma unroll 4
    for (int e = tid; e < 2 * kChunk * 11; e += 128) {
        const int row = e / 11, ii = e - 11 * row, q = row >> 1, rr = row & 1;
        double v = 0;
        if (q < c.len) {
            const int o = ob[q];
            if (ii == 10) v = d.r[2 * o + rr];
            else {
                const int col = cam_col(f, ii);
                if (col >= 0) v = d.J[(size_t)o * 2 * NJ + rr * NJ + ii] * (scl ? scl[col] : 1.0);
            }
        }
        A[row][ii] = v;
    }
    __syncthreads();
    if (tid < kBlk) {
        const int ii = tid / 11, jj = tid - 11 * ii;
        double acc = 0;
        for (int row = 0; row < 2 * c.len; row++) acc = fma(A[row][ii], A[row][jj], acc);
        part[(size_t)blockIdx.x * kBlk + tid] = acc;
    }
}

// C_fa,fb chunk: pairs (a, b) with a in fa, b in fb; Y_a . W_b' (+ Y_a g_p on self pairs)
__global__ __launch_bounds__(128) void ba_pair_schur(BaDev d, const Chunk* __restrict__ ch,
                                                      const int2* __restrict__ pairs, double* part)
{
    __shared__ double Y[kChunk][30];
    __shared__ double Wb[kChunk][33];      // W_b (30) + g_p (3, zero unless a self pair)
    __shared__ int2 pq[kChunk];
    const Chunk c = ch[blockIdx.x];
    const int tid = threadIdx.x;
    if (tid < kChunk) pq[tid] = tid < c.len ? pairs[c.start + tid] : make_int2(0, 0);
    __syncthreads();
#pragma unroll 4
    for (int e = tid; e < kChunk * 30; e += 128) {
        const int q = e / 30, k = e - 30 * q;
        Y[q][k] = q < c.len ? d.yobs[(size_t)pq[q].x * 30 + k] : 0.0;
    }
#pragma unroll 4
    for (int e = tid; e < kChunk * 33; e += 128) {
        const int q = e / 33, k = e - 33 * q;
        double v = 0;
        if (q < c.len) {
            const int2 pr = pq[q];
            if (k < 30) v = d.wobs[(size_t)pr.y * 30 + k];
            else if (pr.x == pr.y) v = d.g[d.nc + 3 * d.op[pr.x] + (k - 30)];
        }
        Wb[q][k] = v;
    }
    __syncthreads();
    if (tid < kBlk) {
        const int ii = tid / 11, jj = tid - 11 * ii;
        const int jo = jj < 10 ? 3 * jj : 30;
        double acc = 0;
        for (int q = 0; q < c.len; q++) {
            acc = fma(Y[q][3 * ii], Wb[q][jo], acc);
            acc = fma(Y[q][3 * ii + 1], Wb[q][jo + 1], acc);
            acc = fma(Y[q][3 * ii + 2], Wb[q][jo + 2], acc);
        }
        part[(size_t)blockIdx.x * kBlk + tid] = acc;
    }
}

// per bucket: the sum of its chunks' blocks, in chunk order
__global__ __launch_bounds__(128) void ba_bucket_reduce(const double* __restrict__ part,
                                                         const int* __restrict__ cstart, int nbucket,
                                                         double* __restrict__ blk)
{
    const int e = blockIdx.x * 128 + threadIdx.x;
    if (e >= nbucket * kBlk) return;
    const int bk = e / kBlk, k = e - bk * kBlk;
    const int c0 = cstart[bk], c1 = cstart[bk + 1];
    double s = 0;
    int c = c0;
    for (; c + 8 <= c1; c += 8) {           // 8 loads in flight, adds still in chunk order
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = part[(size_t)(c + u) * kBlk + k];
#pragma unroll
        for (int u = 0; u < 8; u++) s += v[u];
    }
    for (; c < c1; c++) s += part[(size_t)c * kBlk + k];
    blk[e] = s;
}

// global camera index -> (frame or -1 for K, local index)
__device__ inline void cam_local(int i, int& f, int& ii)
{
    if (i < 4) { f = -1; ii = i; }
    else { f = (i - 4) / 6 + 1; ii = 4 + (i - 4) % 6; }
}

// in-order sum of n strided block entries with 8 loads in flight
__device__ inline double blk_sum(const double* p, int n, size_t stride)
{
    double s = 0;
    int k = 0;
    for (; k + 8 <= n; k += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; u++) s += v[u];
    }
    for (; k < n; k++) s += p[(size_t)k * stride];
    return s;
}

// sum of the blocks mapping onto camera entry (i, j) (j == nc: rhs column).
// U blocks are per frame, Schur blocks per frame pair (fa, fb); only the
// K / rhs sides sum over a free frame index (the rhs of the Schur blocks lives
// on the self pairs, fa == fb).
__device__ inline double cam_entry(const double* blk, int nf, bool pairs, int nc, int i, int j)
{
    int fi, ii, fj, jj;
    cam_local(i, fi, ii);
    const bool rhs = j == nc;
    if (rhs) { fj = -1; jj = 10; }
    else cam_local(j, fj, jj);
    const int e = ii * 11 + jj;
    if (!pairs) {
        if (fi >= 0 && fj >= 0) return fi == fj ? blk[(size_t)fi * kBlk + e] : 0.0;
        if (fi >= 0) return blk[(size_t)fi * kBlk + e];
        if (fj >= 0) return blk[(size_t)fj * kBlk + e];
        return blk_sum(blk + e, nf, kBlk);
    }
    if (fi >= 0 && fj >= 0) return blk[(size_t)(fi * nf + fj) * kBlk + e];
    if (rhs) {
        if (fi >= 0) return blk[(size_t)(fi * nf + fi) * kBlk + e];
        return blk_sum(blk + e, nf, (size_t)(nf + 1) * kBlk);
    }
    if (fi >= 0) return blk_sum(blk + (size_t)fi * nf * kBlk + e, nf, kBlk);
    if (fj >= 0) return blk_sum(blk + (size_t)fj * kBlk + e, nf, (size_t)nf * kBlk);
    return blk_sum(blk + e, nf * nf, kBlk);
}

// [U | g_c] (nc x (nc + 1)) from the frame blocks
__global__ __launch_bounds__(256) void ba_u_assemble(BaDev d, const double* __restrict__ blk, double* Ua)
{
    const int nc = d.nc, ld = nc + 1, e = blockIdx.x * 256 + threadIdx.x;
    if (e >= nc * ld) return;
    const int i = e / ld, j = e - i * ld;
    Ua[e] = cam_entry(blk, d.nf, false, nc, i, j);
}

// reduced camera system: S = U + diag(clamp(diag U)) / radius - sum C,
// rc = g_c - sum (self-pair rhs)
__global__ __launch_bounds__(256) void ba_s_assemble(BaDev d, const double* __restrict__ blk, const double* Ua)
{
    const int nc = d.nc, ld = nc + 1, e = blockIdx.x * 256 + threadIdx.x;
    if (e >= nc * ld) return;
    const int i = e / ld, j = e - i * ld;
    const double sc = cam_entry(blk, d.nf, true, nc, i, j);
    if (j < nc) {
        double u = Ua[e];
        if (i == j) u += fmin(fmax(Ua[e], 1e-6), 1e32) / d.radius;
        d.S[i * nc + j] = u - sc;
    } else {
        d.rc[i] = d.g[i] - sc;
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

// per observation: W_o = scaled J_c' J_p (10 x 3) and Y_o = W_o V_p^-1, one
// thread per (observation, camera partial)
__global__ __launch_bounds__(256) void ba_obs_wy(BaDev d)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.no * 10) return;
    const int o = e / 10, i = e - 10 * o, f = d.of[o], p = d.op[o];
    const double* Jo = d.J + (size_t)o * 2 * NJ;
    const int ci = col_of(d, f, p, i);
    double w[3] = {0, 0, 0};
    if (ci >= 0) {
        const double si = d.scale[ci];
        const double a0 = Jo[i] * si, a1 = Jo[NJ + i] * si;
        for (int k = 0; k < 3; k++) {
            const double sp = d.scale[d.nc + 3 * p + k];
            w[k] = a0 * (Jo[10 + k] * sp) + a1 * (Jo[NJ + 10 + k] * sp);
        }
    }
    const double* Vi = d.Vinv + (size_t)p * 9;
    double* wo = d.wobs + (size_t)o * 30 + 3 * i;
    double* yo = d.yobs + (size_t)o * 30 + 3 * i;
    for (int k = 0; k < 3; k++) {
        wo[k] = w[k];
        yo[k] = w[0] * Vi[0 * 3 + k] + w[1] * Vi[1 * 3 + k] + w[2] * Vi[2 * 3 + k];
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

// S y = rc for nc <= NP with NT = 64 * ceil(NP / 64) threads: thread i keeps
// row i of S in registers (as ba_chol_wave).  At step j every thread k writes
// its a_kj into a double-buffered LDS column (the matrix stays exactly
// symmetric, so this is row j too) and thread j adds b_j: one parallel store
// per thread and one barrier per column; the back solve broadcasts x_j the
// same way.
template <int NP, int NT>
__global__ __launch_bounds__(NT) void ba_chol_rows(BaDev d)
{
    __shared__ double colbuf[2][NP + 1];
    __shared__ double xs[NP];
    const int n = d.nc, i = threadIdx.x;
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) a[k] = i < n && k < n ? d.S[i * n + k] : (i == k ? 1.0 : 0.0);
    double b = i < n ? d.rc[i] : 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        double* cb = colbuf[j & 1];
        if (i < NP) cb[i] = a[j];
        if (i == j) cb[NP] = b;
        __syncthreads();
        const double ajj = cb[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }   // uniform: one pivot for all threads
        const double inv = 1.0 / ajj, bj = cb[NP];
        if (i > j && i < NP) {
            const double aij = a[j];
#pragma unroll
            for (int k = j + 1; k < NP; k++) a[k] = fma(-(aij * cb[k]), inv, a[k]);
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
    // frame buckets of observations (gram) and frame-pair buckets of ordered
    // observation pairs of one point (Schur), cut into chunks of <= kChunk
    std::vector<int> flist(no > 0 ? no : 1);
    std::vector<Chunk> gch;
    std::vector<int> gcs(nf + 1, 0);
    {
        std::vector<int> fstart(nf + 1, 0), fill(nf, 0);
        for (int o = 0; o < no; o++) fstart[of[o] + 1]++;
        for (int f = 0; f < nf; f++) fstart[f + 1] += fstart[f];
        for (int o = 0; o < no; o++) flist[fstart[of[o]] + fill[of[o]]++] = o;
        for (int f = 0; f < nf; f++) {
            gcs[f] = (int)gch.size();
            for (int st = fstart[f]; st < fstart[f + 1]; st += kChunk)
                gch.push_back(Chunk{f, st, std::min(kChunk, fstart[f + 1] - st)});
        }
        gcs[nf] = (int)gch.size();
    }
    const int nb2 = nf * nf;
    std::vector<int2> pairs;
    std::vector<Chunk> sch;
    std::vector<int> scs(nb2 + 1, 0);
    {
        std::vector<size_t> pos(nb2 + 1, 0);
        for (int p = 0; p < np; p++)
            for (int qa = pstart[p]; qa < pstart[p + 1]; qa++)
                for (int qb = pstart[p]; qb < pstart[p + 1]; qb++) pos[of[plist[qa]] * nf + of[plist[qb]] + 1]++;
        for (int b = 0; b < nb2; b++) pos[b + 1] += pos[b];
        pairs.resize(std::max<size_t>(pos[nb2], 1));
        std::vector<size_t> st(pos.begin(), pos.end() - 1);
        for (int p = 0; p < np; p++)
            for (int qa = pstart[p]; qa < pstart[p + 1]; qa++)
                for (int qb = pstart[p]; qb < pstart[p + 1]; qb++) {
                    const int a = plist[qa], b = plist[qb];
                    pairs[st[of[a] * nf + of[b]]++] = make_int2(a, b);
                }
        for (int b = 0; b < nb2; b++) {
            scs[b] = (int)sch.size();
            for (size_t q = pos[b]; q < pos[b + 1]; q += kChunk)
                sch.push_back(Chunk{b, (int)q, (int)std::min<size_t>(kChunk, pos[b + 1] - q)});
        }
        scs[nb2] = (int)sch.size();
    }
    const int ngch = (int)gch.size(), nsch = (int)sch.size();

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
                 o_w = carve(240 * (size_t)no), o_y = carve(240 * (size_t)no), o_st = carve(8 * (size_t)N),
                 o_red = carve(8 * 16), o_ua = carve(8 * (size_t)E),
                 o_part = carve(8 * (size_t)kBlk * std::max(1, std::max(ngch, nsch))),
                 o_bu = carve(8 * (size_t)kBlk * nf), o_bs = carve(8 * (size_t)kBlk * nb2),
                 o_fl = carve(4 * flist.size()), o_gch = carve(sizeof(Chunk) * std::max(1, ngch)),
                 o_gcs = carve(4 * gcs.size()), o_pr = carve(sizeof(int2) * pairs.size()),
                 o_sch = carve(sizeof(Chunk) * std::max(1, nsch)), o_scs = carve(4 * scs.size());
    SLAM_HIP(c, c->ba_par.ensure(off));
    char* base = c->ba_par.as<char>();
    BaDev d;
    d.nf = nf; d.np = np; d.no = no; d.nc = nc; d.loss = loss; d.a = a;
    d.of = (const int*)(base + o_of); d.op = (const int*)(base + o_op); d.oxy = (const double*)(base + o_oxy);
    d.pstart = (const int*)(base + o_ps); d.plist = (const int*)(base + o_pl);
    d.x = (double*)(base + o_x); d.xc = (double*)(base + o_xc); d.r = (double*)(base + o_r); d.J = (double*)(base + o_J);
    d.scale = (double*)(base + o_sc); d.g = (double*)(base + o_g); d.S = (double*)(base + o_S);
    d.rc = (double*)(base + o_rc); d.Vinv = (double*)(base + o_Vi); d.wobs = (double*)(base + o_w);
    d.step = (double*)(base + o_st); d.red = (double*)(base + o_red); d.yobs = (double*)(base + o_y);
    double* Ua = (double*)(base + o_ua);      // [U | g_c], nc x (nc + 1)
    double* part = (double*)(base + o_part);  // per-chunk 10 x 11 blocks
    double* blkU = (double*)(base + o_bu);    // per-frame B_f
    double* blkS = (double*)(base + o_bs);    // per-frame-pair C_fa,fb
    const int* dflist = (const int*)(base + o_fl);
    const Chunk* dgch = (const Chunk*)(base + o_gch);
    const int* dgcs = (const int*)(base + o_gcs);
    const int2* dpairs = (const int2*)(base + o_pr);
    const Chunk* dsch = (const Chunk*)(base + o_sch);
    const int* dscs = (const int*)(base + o_scs);
    d.radius = 1e4;
    if (no > 0) {
        SLAM_HIP(c, hipMemcpyAsync(base + o_of, of, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_op, op, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_oxy, oxy, 16 * (size_t)no, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(base + o_pl, plist.data(), 4 * (size_t)no, hipMemcpyHostToDevice, s));
    }
    SLAM_HIP(c, hipMemcpyAsync(base + o_ps, pstart.data(), 4 * (size_t)(np + 1), hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(d.x, x.data(), 8 * (size_t)NX, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_fl, flist.data(), 4 * flist.size(), hipMemcpyHostToDevice, s));
    if (ngch) SLAM_HIP(c, hipMemcpyAsync(base + o_gch, gch.data(), sizeof(Chunk) * ngch, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_gcs, gcs.data(), 4 * gcs.size(), hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_pr, pairs.data(), sizeof(int2) * pairs.size(), hipMemcpyHostToDevice, s));
    if (nsch) SLAM_HIP(c, hipMemcpyAsync(base + o_sch, sch.data(), sizeof(Chunk) * nsch, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(base + o_scs, scs.data(), 4 * scs.size(), hipMemcpyHostToDevice, s));

    const size_t chol_lds = (size_t)nc * nc * 8;
    const void* chol_fn = gT == 3 ? (const void*)ba_chol_solve<3> : gT == 4 ? (const void*)ba_chol_solve<4>
                        : gT == 6 ? (const void*)ba_chol_solve<6> : (const void*)ba_chol_solve<9>;
    if (chol_lds > 60 * 1024)
        SLAM_HIP(c, hipFuncSetAttribute(chol_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chol_lds));

    // camera reductions (frame-structured blocks) and the reduced system
    auto cam_gram = [&](const double* scl) {
        if (ngch) hipLaunchKernelGGL(ba_frame_gram, dim3(ngch), dim3(128), 0, s, d, dgch, dflist, scl, part);
        hipLaunchKernelGGL(ba_bucket_reduce, dim3((nf * kBlk + 127) / 128), dim3(128), 0, s, (const double*)part,
                           dgcs, nf, blkU);
        hipLaunchKernelGGL(ba_u_assemble, dim3((E + 255) / 256), dim3(256), 0, s, d, (const double*)blkU, Ua);
    };
    auto schur = [&]() {
        if (nsch) hipLaunchKernelGGL(ba_pair_schur, dim3(nsch), dim3(128), 0, s, d, dsch, dpairs, part);
        hipLaunchKernelGGL(ba_bucket_reduce, dim3((nb2 * kBlk + 127) / 128), dim3(128), 0, s, (const double*)part,
                           dscs, nb2, blkS);
        hipLaunchKernelGGL(ba_s_assemble, dim3((E + 255) / 256), dim3(256), 0, s, d, (const double*)blkS,
                           (const double*)Ua);
    };
    auto chol = [&]() {
        if (nc <= 48) { hipLaunchKernelGGL(ba_chol_wave<48>, dim3(1), dim3(64), 0, s, d); return; }
        if (nc <= 64) { hipLaunchKernelGGL(ba_chol_wave<64>, dim3(1), dim3(64), 0, s, d); return; }
        if (nc <= 96) { hipLaunchKernelGGL((ba_chol_rows<96, 128>), dim3(1), dim3(128), 0, s, d); return; }
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
    // the per-iteration scalars come back through pinned memory: an async copy
    // plus a polled sync (a pageable destination makes the copy itself block)
    double* red = static_cast<double*>(readback(c, sizeof(double) * 8));
    if (!red) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    auto read_red = [&]() -> int {
        SLAM_HIP(c, hipMemcpyAsync(red, d.red, sizeof(double) * 8, hipMemcpyDeviceToHost, s));
        return stream_sync(c, s, true);
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
                if (no > 0) hipLaunchKernelGGL(ba_obs_wy, dim3((no * 10 + 255) / 256), dim3(256), 0, s, d);
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
