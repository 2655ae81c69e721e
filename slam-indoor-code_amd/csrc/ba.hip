// Windowed bundle adjustment on gfx950 (FP64), replacing the reference's Ceres
// call site bundleAdjustment (src/mainModule/bundleAdjustment/
// bundleAdjustment.cpp:73-129): same parameter blocks (shared free intrinsics
// {fx, fy, cx, cy}, per-frame angle-axis + t with frame 0 constant, points),
// same residual (ProjectionCostFunctor :15-41), same losses (getLossFunction
// :131-151, Ceres Corrector), same Levenberg-Marquardt trust region with
// Jacobi scaling and Schur elimination of the points (Options :108-114).
//
// The whole Levenberg-Marquardt loop runs on the device (the per-iteration
// launches and the device state are described below, before BaState); the
// host builds the index structures once per solve, queues the iterations and
// reads the state back once at the end, making exactly the oracle's accept /
// reject decisions (oracle/ba.c) on the device.
#include <cfloat>
#include <cstdlib>
#ifdef BA_HOST_TIMING
#include <chrono>
#include <cstdio>
#define BA_T(i) ht[i] = std::chrono::steady_clock::now()
#else
#define BA_T(i) (void)0
#endif
#include <cmath>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int NJ = 13;

#ifdef BA_DIAG
// diagnostic build only: per-workgroup wall-clock stamps of schur / update phases
__device__ long long g_dt[2][16384][4];
#define BA_DT(k, i) do { if (threadIdx.x == 0 && blockIdx.x < 16384) g_dt[k][blockIdx.x][i] = wall_clock64(); } while (0)
#else
#define BA_DT(k, i) (void)0
#endif

// forward-mode jets (ceres/jet.h arithmetic) over W of the 13 residual-block
// parameters, columns [OFF, OFF + W): K 0..3, extrinsics 4..9, point 10..12.
// The full block (W = 13) serves the initial evaluation; an iteration splits
// the Jacobian over three lanes per observation (K, extrinsics, point), each
// carrying the value path and its own columns.
template <int W>
struct JetT {
    double a;
    double v[W];
};

template <int W> __device__ inline JetT<W> jc(double a) { JetT<W> r; r.a = a;
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = 0; return r; }
// seeded variable for global column c (a constant when inlined)
template <int W, int OFF> __device__ inline JetT<W> jv(double a, int c)
{
    JetT<W> r = jc<W>(a);
    if (c >= OFF && c < OFF + W) r.v[c - OFF] = 1.0;
    return r;
}
template <int W> __device__ inline JetT<W> jadd(const JetT<W>& x, const JetT<W>& y) { JetT<W> r; r.a = __dadd_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dadd_rn(x.v[i], y.v[i]); return r; }
template <int W> __device__ inline JetT<W> jsub(const JetT<W>& x, const JetT<W>& y) { JetT<W> r; r.a = __dsub_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dsub_rn(x.v[i], y.v[i]); return r; }
template <int W> __device__ inline JetT<W> jmul(const JetT<W>& x, const JetT<W>& y) { JetT<W> r; r.a = __dmul_rn(x.a, y.a);
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dadd_rn(__dmul_rn(x.a, y.v[i]), __dmul_rn(x.v[i], y.a)); return r; }
template <int W> __device__ inline JetT<W> jdiv(const JetT<W>& f, const JetT<W>& g)
{
    const double gi = __ddiv_rn(1.0, g.a), fg = __dmul_rn(f.a, gi);
    JetT<W> r; r.a = fg;
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dmul_rn(__dsub_rn(f.v[i], __dmul_rn(fg, g.v[i])), gi);
    return r;
}
template <int W> __device__ inline JetT<W> jsqrt(const JetT<W>& f)
{
    const double t = __dsqrt_rn(f.a), tw = __ddiv_rn(1.0, __dmul_rn(2.0, t));
    JetT<W> r; r.a = t;
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dmul_rn(f.v[i], tw);
    return r;
}
template <int W> __device__ inline JetT<W> jcos(const JetT<W>& f) { JetT<W> r; r.a = cos(f.a); const double s = -sin(f.a);
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dmul_rn(s, f.v[i]); return r; }
template <int W> __device__ inline JetT<W> jsin(const JetT<W>& f) { JetT<W> r; r.a = sin(f.a); const double c = cos(f.a);
#pragma unroll
    for (int i = 0; i < W; i++) r.v[i] = __dmul_rn(c, f.v[i]); return r; }

// ceres AngleAxisRotatePoint + t, pinhole, minus the observation; J: the
// columns [OFF, OFF + W) of the 2 x 13 block Jacobian
template <int W, int OFF>
__device__ __forceinline__ void project(const double* K, const double* e, const double* X, double ox, double oy,
                                        double r[2], double J[2][W])
{
    typedef JetT<W> Jet;
    Jet aa[3] = {jv<W, OFF>(e[0], 4), jv<W, OFF>(e[1], 5), jv<W, OFF>(e[2], 6)};
    Jet pt[3] = {jv<W, OFF>(X[0], 10), jv<W, OFF>(X[1], 11), jv<W, OFF>(X[2], 12)};
    Jet p[3];
    Jet th2 = jadd(jadd(jmul(aa[0], aa[0]), jmul(aa[1], aa[1])), jmul(aa[2], aa[2]));
    if (th2.a > DBL_EPSILON) {
        Jet th = jsqrt(th2);
        Jet ct = jcos(th), st = jsin(th);
        Jet ti = jdiv(jc<W>(1.0), th);
        Jet w[3] = {jmul(aa[0], ti), jmul(aa[1], ti), jmul(aa[2], ti)};
        Jet wx[3] = {jsub(jmul(w[1], pt[2]), jmul(w[2], pt[1])), jsub(jmul(w[2], pt[0]), jmul(w[0], pt[2])),
                     jsub(jmul(w[0], pt[1]), jmul(w[1], pt[0]))};
        Jet tmp = jmul(jadd(jadd(jmul(w[0], pt[0]), jmul(w[1], pt[1])), jmul(w[2], pt[2])), jsub(jc<W>(1.0), ct));
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = jadd(jadd(jmul(pt[k], ct), jmul(wx[k], st)), jmul(w[k], tmp));
    } else {
        Jet wx[3] = {jsub(jmul(aa[1], pt[2]), jmul(aa[2], pt[1])), jsub(jmul(aa[2], pt[0]), jmul(aa[0], pt[2])),
                     jsub(jmul(aa[0], pt[1]), jmul(aa[1], pt[0]))};
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = jadd(pt[k], wx[k]);
    }
    p[0] = jadd(p[0], jv<W, OFF>(e[3], 7));
    p[1] = jadd(p[1], jv<W, OFF>(e[4], 8));
    p[2] = jadd(p[2], jv<W, OFF>(e[5], 9));
    Jet x2 = jdiv(p[0], p[2]), y2 = jdiv(p[1], p[2]);
    Jet u = jsub(jadd(jmul(jv<W, OFF>(K[0], 0), x2), jv<W, OFF>(K[2], 2)), jc<W>(ox));
    Jet v = jsub(jadd(jmul(jv<W, OFF>(K[1], 1), y2), jv<W, OFF>(K[3], 3)), jc<W>(oy));
    r[0] = u.a;
    r[1] = v.a;
#pragma unroll
    for (int i = 0; i < W; i++) { J[0][i] = u.v[i]; J[1][i] = v.v[i]; }
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

// ---------------------------------------------------------------------------
// Device-resident LM.  Every decision of the oracle's loop (oracle/ba.c) is
// taken on the device: the host queues iterations without waiting on any of
// them and reads the state once at the end (plus one early-exit poll per
// chunk of iterations).  Buffers that change on an accepted step come in two
// copies, indexed by the state's `cur`: the candidate is always 1 - cur, and
// accepting is cur ^= 1.  The candidate's residuals, Jacobian and gradient are
// computed speculatively alongside its cost, so an accepted step needs no
// further pass.  Per iteration seven launches (a launch boundary, ~2 us, is
// the cheapest cross-workgroup sum point here):
//   A  ba_schur_pts    point chunks (points grouped by the frames of their
//                      observations): V_p + D_p / radius and its inverse, the
//                      W / Y blocks in LDS, per chunk the frame-pair blocks of
//                      sum Y_a W_b' (+ the rhs Y_a g_p)
//   A' ba_blk_reduce   each frame-pair bucket summed over its chunks in order
//   B  ba_s_assemble   the reduced camera system S from [U | g_c] and the
//                      buckets, damping
//   B' ba_camera_solve_lane  one wave: register Cholesky, both solves
//   C  ba_update       back substitution, candidate, model cost change, the
//                      candidate's residuals + Jacobian (jets) + cost + point
//                      gradient, and the chunk's shares of the candidate's
//                      per-frame [J_c | r] Gram blocks (f64 MFMA; workgroup =
//                      a Schur point chunk)
//   D  ba_frame_reduce each frame's chunk partials summed in order
//   E  ba_decide       one workgroup: the candidate's [U | g_c], the reduced
//                      scalars, and the accept / reject logic (Ceres
//                      LevenbergMarquardtStrategy as oracle/ba.c restates it)
// Every kernel returns at entry once the state says done.
// ---------------------------------------------------------------------------

// camera-block geometry shared by the reductions: an observation in frame f
// touches only the 10 camera columns K (4) + ext_f (6) (frame 0: K only), so
// [U | g_c] is a sum of per-frame 10 x 11 blocks and the Schur term a sum of
// per-frame-pair blocks
constexpr int kChunk = 64;   // observation slots per Schur point chunk
constexpr int kGChunk = 32;  // observations per gram chunk
constexpr int kBlk = 110;    // 10 x 11 block entries

struct Chunk {
    int bucket;              // frame (gram)
    int start, len;          // range in the frame-bucketed observation list
};

struct PtChunk {             // Schur point chunk: points [start, start + len) of the grouped point order
    int start, len, nobs;    // nobs: observations per point (same for the whole group)
    int part;                // first partial block; n * n follow (pair a * n + b)
    int group;               // frame tuple id
    int fpart;               // first frame Gram partial (ba_update); n follow (tuple position a)
    int qstart;              // first observation slot: point start + lp has slots qstart + lp * nobs + a
};

struct BaState {
    double radius, decrease_factor, cost, xnorm, initial_cost;
    double cand_cost, mcc, snorm2, xcnorm2, gmax_pts;   // C's reduced scalars (candidate)
    int iter, max_iters, consecutive_invalid, successful, termination, usable, done, cur;
    int fail;                // A / B / C: failed linear solve or non-finite step (this iteration)
    int pad[3];
};

struct BaDev {
    int nf, np, no, nc, N, NX, loss;
    double a;
    const int* of;
    const int* op;
    const double* oxy;
    const int* pstart;       // observations of point p: [pstart[p], pstart[p + 1]) (device numbering)
    const int* flist;        // observations bucketed by frame
    const Chunk* gch;        // gram chunks
    const int* gcs;          // first gram chunk of frame f (nf + 1)
    const PtChunk* pch;      // Schur point chunks
    const int* gframes;      // frames of a group's tuple: [group * 64 + a]
    const int* fpstart;      // ba_update's frame Gram partials of frame f: [fpstart[f], fpstart[f + 1])
    const int* fppos;        // where chunk partial fpart + a is stored (frame-major, chunk order)
    const int* bstart;       // partials of bucket fa * nf + fb (CSR, fixed order)
    const int* bpos;         // where Schur partial part + pr is stored (bucket-major, chunk order)
    double* x[2];            // full layout: K[4], ext[nf * 6] (frame 0 incl.), pts[np * 3]
    double* r[2];            // [no][2]
    double* J[2];            // [no][2][13]
    double* g[2];            // scaled gradient (tangent layout, N)
    double* blkU[2];         // per-frame [J_c | r] Gram blocks of J[b] ([nf][110]; [U | g_c] = their sum)
    double* scale;           // N
    double* Vinv;            // [np][9]
    double* yc;              // nc: reduced-system solution
    double* Sg;              // [S | rc], nc x (nc + 1) (lower triangle + rhs)
    double* spart;           // Schur partial blocks
    double* blkS;            // [nf * nf][110]
    double* gpart;           // frame Gram partial blocks (ba_gram chunks at init, ba_update chunks per iteration)
    double* wpart;           // per-workgroup scalar partials (8 per workgroup)
    BaState* st;
};

__device__ inline int col_of(const BaDev& d, int f, int p, int i)
{
    if (i < 4) return i;
    if (i < 10) return f == 0 ? -1 : 4 + 6 * (f - 1) + (i - 4);
    return d.nc + 3 * p + (i - 10);
}

// tangent index -> full layout index (frame 0's extrinsics are constant)
__device__ inline int full_of(const BaDev& d, int i)
{
    if (i < 4) return i;
    if (i < d.nc) return i + 6;
    return 4 + 6 * d.nf + (i - d.nc);
}

// Cross-workgroup sums go through kernel boundaries: every launch writes its
// per-workgroup (or per-chunk) partials with plain stores, and the next launch
// sums them in a fixed order.  An in-launch "last workgroup finishes the sum"
// protocol (write-through stores + an arrival counter) was tried and cost
// 20-65 us per launch here -- contended counter atomics and the serial tail --
// against ~2 us for a launch boundary.

// workgroup sum / max of one value per thread (every thread calls; result in thread 0)
template <int NT>
__device__ inline double wg_reduce(double v, bool is_max)
{
    __shared__ double wp[NT / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double w = __shfl_xor(v, o, 64);
        v = is_max ? fmax(v, w) : v + w;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) wp[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = wp[0];
    for (int w = 1; w < NT / 64; w++) t = is_max ? fmax(t, wp[w]) : t + wp[w];
    return t;
}

// sum / max of n per-workgroup partial slots (stride 8) by the whole
// (last) workgroup: strided per-thread partials, then the fixed tree of
// wg_reduce -- deterministic.  Every thread calls; the result is in thread 0.
template <int NT>
__device__ inline double wg_sum_parts(const double* p, int n, int k, bool is_max)
{
    double s = 0;
    for (int w = threadIdx.x; w < n; w += NT) {
        const double v = p[(size_t)w * 8 + k];
        s = is_max ? fmax(s, v) : s + v;
    }
    return wg_reduce<NT>(s, is_max);
}

// residual + loss-corrected Jacobian columns [OFF, OFF + W) of observation o at
// parameters (K, e, X); returns the cost term 0.5 rho (Ceres Corrector,
// loss_function.cc: every column is corrected on its own)
template <int W, int OFF>
__device__ __forceinline__ double eval_obs(const BaDev& d, const double* K, const double* e, const double* X, int o,
                                           double r[2], double J[2][W])
{
    project<W, OFF>(K, e, X, d.oxy[2 * o], d.oxy[2 * o + 1], r, J);
    const double sq = r[0] * r[0] + r[1] * r[1];
    double c;
    if (d.loss == SLAM_LOSS_NONE) {
        c = 0.5 * sq;
    } else {
        double rho[3];
        loss_eval(d.loss, d.a, sq, rho);
        c = 0.5 * rho[0];
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
#pragma unroll
            for (int i = 0; i < W; i++) { J[0][i] *= sqrt_rho1; J[1][i] *= sqrt_rho1; }
        } else {
#pragma unroll
            for (int i = 0; i < W; i++) {
                const double rtj = J[0][i] * r[0] + J[1][i] * r[1];
                J[0][i] = sqrt_rho1 * (J[0][i] - alpha_sq_norm * r[0] * rtj);
                J[1][i] = sqrt_rho1 * (J[1][i] - alpha_sq_norm * r[1] * rtj);
            }
        }
        r[0] *= residual_scaling;
        r[1] *= residual_scaling;
    }
    return c;
}

// ---- init I0: the device numbering (one thread per device point p'): its
// observations gathered from the caller's arrays (q -> qsrc[q]), its position
// from the caller's point por[p'], the cameras copied ----
__global__ __launch_bounds__(128) void ba_import(BaDev d, const int* __restrict__ rof, const double* __restrict__ roxy,
                                                 const int* __restrict__ qsrc, const int* __restrict__ por,
                                                 const double* __restrict__ xin)
{
    const int pp = blockIdx.x * 128 + threadIdx.x, xp = 4 + 6 * d.nf;
    if (pp < d.np) {
        const int p = por[pp];
#pragma unroll
        for (int k = 0; k < 3; k++) d.x[0][xp + 3 * pp + k] = xin[xp + 3 * p + k];
        int* of = const_cast<int*>(d.of);
        int* op = const_cast<int*>(d.op);
        double* oxy = const_cast<double*>(d.oxy);
        for (int q = d.pstart[pp]; q < d.pstart[pp + 1]; q++) {
            const int o = qsrc[q];
            of[q] = rof[o];
            op[q] = pp;
            oxy[2 * q] = roxy[2 * o];
            oxy[2 * q + 1] = roxy[2 * o + 1];
        }
    }
    if (pp < xp) d.x[0][pp] = xin[pp];
}

// ---- the solution x[cur] back in the caller's point order ----
__global__ __launch_bounds__(128) void ba_export(BaDev d, const int* __restrict__ por, double* __restrict__ xout)
{
    const int pp = blockIdx.x * 128 + threadIdx.x, xp = 4 + 6 * d.nf;
    const double* x = d.x[d.st->cur];
    if (pp < d.np) {
        const int p = por[pp];
#pragma unroll
        for (int k = 0; k < 3; k++) xout[xp + 3 * p + k] = x[xp + 3 * pp + k];
    }
    if (pp < xp) xout[pp] = x[pp];
}

// ---- init I1: residuals, Jacobian and cost at x[0] (one thread per observation) ----
__global__ __launch_bounds__(128) void ba_eval_init(BaDev d)
{
    const int o = blockIdx.x * 128 + threadIdx.x;
    double c = 0;
    if (o < d.no) {
        const double* xs = d.x[0];
        const int f = d.of[o], p = d.op[o];
        double r[2], J[2][NJ];
        c = eval_obs<NJ, 0>(d, xs, xs + 4 + 6 * f, xs + 4 + 6 * d.nf + 3 * p, o, r, J);
        d.r[0][2 * o] = r[0];
        d.r[0][2 * o + 1] = r[1];
        double* Jo = d.J[0] + (size_t)o * 2 * NJ;
#pragma unroll
        for (int i = 0; i < NJ; i++) { Jo[i] = J[0][i]; Jo[NJ + i] = J[1][i]; }
    }
    if (!isfinite(c)) c = INFINITY;
    const double t = wg_reduce<128>(c, false);
    if (threadIdx.x == 0) d.wpart[(size_t)blockIdx.x * 8] = t;
}

// ---- init I3: point Jacobi scaling, scaled point gradient, its max (one thread per point) ----
__global__ __launch_bounds__(128) void ba_point_init(BaDev d)
{
    const int p = blockIdx.x * 128 + threadIdx.x;
    double m = 0;
    if (p < d.np) {
        double s2[3] = {0, 0, 0}, u[3] = {0, 0, 0};
        for (int o = d.pstart[p]; o < d.pstart[p + 1]; o++) {
            const double* Jo = d.J[0] + (size_t)o * 2 * NJ;
            for (int k = 0; k < 3; k++) {
                s2[k] += Jo[10 + k] * Jo[10 + k] + Jo[NJ + 10 + k] * Jo[NJ + 10 + k];
                u[k] += Jo[10 + k] * d.r[0][2 * o] + Jo[NJ + 10 + k] * d.r[0][2 * o + 1];
            }
        }
        for (int k = 0; k < 3; k++) {
            const double sc = 1.0 / (1.0 + sqrt(s2[k]));
            d.scale[d.nc + 3 * p + k] = sc;
            d.g[0][d.nc + 3 * p + k] = u[k] * sc;
            m = fmax(m, fabs(u[k]));
        }
    }
    const double t = wg_reduce<128>(m, true);
    if (threadIdx.x == 0) d.wpart[(size_t)blockIdx.x * 8 + 4] = t;
}

// global camera index -> (frame or -1 for K, local index)
__device__ inline void cam_local(int i, int& f, int& ii)
{
    if (i < 4) { f = -1; ii = i; }
    else { f = (i - 4) / 6 + 1; ii = 4 + (i - 4) % 6; }
}

// sum of the blocks mapping onto camera entry (i, j) (j == nc: rhs column).
// U blocks are per frame, Schur blocks per frame pair (fa, fb); only the
// K / rhs sides sum over a free frame index (the rhs of the Schur blocks lives
// on the self pairs, fa == fb).  Fixed order.
__device__ inline double blk_sum(const double* p, int n, size_t stride)
{
    double s = 0;
    int k = 0;
    for (; k + 32 <= n; k += 32) {         // 32 loads in flight, adds in order
        double v[32];
#pragma unroll
        for (int u = 0; u < 32; u++) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
        for (int u = 0; u < 32; u++) s += v[u];
    }
    for (; k + 8 <= n; k += 8) {           // 8 loads in flight, adds in order
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = p[(size_t)(k + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; u++) s += v[u];
    }
    for (; k < n; k++) s += p[(size_t)k * stride];
    return s;
}
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

// camera column of local partial ii (0..9) of an observation in frame f (frame 0 ext: -1)
__device__ inline int cam_col(int f, int ii) { return ii < 4 ? ii : f == 0 ? -1 : 4 + 6 * (f - 1) + (ii - 4); }

// ---- D / init: frame chunks of [J_c | r] Gram blocks, per-frame ordered sums,
// then the last workgroup ----
//   mode 0: unscaled J[0] (init: camera Jacobi scaling from the diagonal)
//   mode 1: scaled J[0] (init: [U | g_c] of the initial Jacobian, gradient check)
//   mode 2: (iterations: the partials come from ba_update, ba_frame_reduce sums them)
enum { kGramUnscaled = 0, kGramInit = 1, kGramStep = 2 };

__device__ void lm_decide(const BaDev& d, BaState& st, int cand, double gmax_cam);

template <int MODE>
__global__ __launch_bounds__(128) void ba_gram(BaDev d)
{
    __shared__ double A[2 * kGChunk][11];
    __shared__ int ob[kGChunk];
    if (MODE == kGramStep && d.st->done) return;
    const int b = MODE == kGramStep ? 1 - d.st->cur : 0;     // which J / r
    const Chunk c = d.gch[blockIdx.x];
    const int tid = threadIdx.x, f = c.bucket;
    if (tid < kGChunk) ob[tid] = tid < c.len ? d.flist[c.start + tid] : 0;
    __syncthreads();
    const double* Jb = d.J[b];
    const double* rb = d.r[b];
    for (int e = tid; e < 2 * kGChunk * 11; e += 128) {
        const int row = e / 11, ii = e - 11 * row, q = row >> 1, rr = row & 1;
        double v = 0;
        if (q < c.len) {
            const int o = ob[q];
            if (ii == 10) v = rb[2 * o + rr];
            else {
                const int col = cam_col(f, ii);
                if (col >= 0) v = Jb[(size_t)o * 2 * NJ + rr * NJ + ii] * (MODE == kGramUnscaled ? 1.0 : d.scale[col]);
            }
        }
        A[row][ii] = v;
    }
    __syncthreads();
    if (tid < kBlk) {
        const int ii = tid / 11, jj = tid - 11 * ii;
        double acc = 0;
        for (int row = 0; row < 2 * c.len; row++) acc = fma(A[row][ii], A[row][jj], acc);
        d.gpart[(size_t)blockIdx.x * kBlk + tid] = acc;
    }
}

// per bucket (frame pair; its partials stored contiguously): the sum of its
// partial 10 x 11 blocks.  One workgroup per bucket: the range is cut into
// kRedSeg contiguous segments, each summed in order by its own thread per
// entry (8 loads in flight), then the segment sums are added in segment
// order -- a fixed two-level order, with ~kRedSeg x shorter dependent chains.
constexpr int kRedSeg = 9;                  // 9 x 110 = 990 of 1024 threads

__global__ __launch_bounds__(1024) void ba_blk_reduce(const BaState* __restrict__ st, int check_done,
                                                       const double* __restrict__ part, const int* __restrict__ start,
                                                       double* __restrict__ out)
{
    __shared__ double seg[kRedSeg][kBlk];
    if (check_done && st->done) return;
    const int bk = blockIdx.x, t = threadIdx.x, sg = t / kBlk, k = t - sg * kBlk;
    const int p0 = start[bk], p1 = start[bk + 1], len = p1 - p0;
    if (sg < kRedSeg) {
        const int per = (len + kRedSeg - 1) / kRedSeg;
        const int q0 = p0 + min(len, sg * per), q1 = p0 + min(len, (sg + 1) * per);
        double s = 0;
        int q = q0;
        for (; q + 8 <= q1; q += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = part[(size_t)(q + u) * kBlk + k];
#pragma unroll
            for (int u = 0; u < 8; u++) s += v[u];
        }
        for (; q < q1; q++) s += part[(size_t)q * kBlk + k];
        seg[sg][k] = s;
    }
    __syncthreads();
    if (t < kBlk) {
        double s = 0;
#pragma unroll
        for (int g = 0; g < kRedSeg; g++) s += seg[g][t];
        out[(size_t)bk * kBlk + t] = s;
    }
}

// the frame blocks of a Jacobian: ba_blk_reduce into blkU[b], b chosen on
// the device (the candidate's buffer in an iteration)
template <int MODE>
__global__ __launch_bounds__(1024) void ba_frame_reduce(BaDev d)
{
    __shared__ double seg[kRedSeg][kBlk];
    if (MODE == kGramStep && d.st->done) return;
    const int b = MODE == kGramStep ? 1 - d.st->cur : MODE == kGramUnscaled ? 1 : 0;
    const int bk = blockIdx.x, t = threadIdx.x, sg = t / kBlk, k = t - sg * kBlk;
    // step: ba_update's chunk partials of frame bk; init: ba_gram's chunks
    const int p0 = MODE == kGramStep ? d.fpstart[bk] : d.gcs[bk];
    const int p1 = MODE == kGramStep ? d.fpstart[bk + 1] : d.gcs[bk + 1], len = p1 - p0;
    if (sg < kRedSeg) {
        const int per = (len + kRedSeg - 1) / kRedSeg;
        const int q0 = p0 + min(len, sg * per), q1 = p0 + min(len, (sg + 1) * per);
        double s = 0;
        int q = q0;
        for (; q + 8 <= q1; q += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = d.gpart[(size_t)(q + u) * kBlk + k];
#pragma unroll
            for (int u = 0; u < 8; u++) s += v[u];
        }
        for (; q < q1; q++) s += d.gpart[(size_t)q * kBlk + k];
        seg[sg][k] = s;
    }
    __syncthreads();
    if (t < kBlk) {
        double s = 0;
#pragma unroll
        for (int g = 0; g < kRedSeg; g++) s += seg[g][t];
        d.blkU[b][(size_t)bk * kBlk + t] = s;
    }
}

// one workgroup after the frame blocks of a Jacobian are summed: [U | g_c],
// then by mode
//   unscaled: the initial cost (eval partials) and the camera Jacobi scaling
//   init:     the camera gradient and the oracle's first gradient check
//   step:     the candidate's reduced scalars (update partials), its camera
//             gradient, and the LM decision
constexpr int kDecideThreads = 256;

template <int MODE>
__global__ __launch_bounds__(kDecideThreads) void ba_decide(BaDev d, int nwp)
{
    if (MODE == kGramStep && d.st->done) return;
    const int b = MODE == kGramStep ? 1 - d.st->cur : MODE == kGramUnscaled ? 1 : 0;
    const int tid = threadIdx.x, nc = d.nc;
    const double* blk = d.blkU[b];
    if (MODE == kGramUnscaled) {
        for (int i = tid; i < nc; i += kDecideThreads)
            d.scale[i] = 1.0 / (1.0 + sqrt(cam_entry(blk, d.nf, false, nc, i, i)));
        const double cost = wg_sum_parts<kDecideThreads>(d.wpart, nwp, 0, false);
        if (tid == 0) {
            d.st->cost = cost;
            d.st->initial_cost = cost;
        }
        return;
    }
    // step: the update partials' per-thread strided sums first (their loads
    // in flight alongside the gradient's), reduced below with wg_sum_parts's
    // tree in one pass
    double v5[5] = {0, 0, 0, 0, 0};
    if (MODE == kGramStep)
        for (int w = tid; w < nwp; w += kDecideThreads) {
            const double* pw = d.wpart + (size_t)w * 8;
#pragma unroll
            for (int k = 0; k < 5; k++) v5[k] = k == 4 ? fmax(v5[k], pw[k]) : v5[k] + pw[k];
        }
    // camera gradient (scaled: the rhs column of [U | g_c]) and its unscaled max
    double m = 0;
    for (int i = tid; i < nc; i += kDecideThreads) {
        const double gs = cam_entry(blk, d.nf, false, nc, i, nc);
        d.g[b][i] = gs;
        m = fmax(m, fabs(gs / d.scale[i]));
    }
    const double gmax_cam = wg_reduce<kDecideThreads>(m, true);
    if (MODE == kGramStep) {
        __shared__ double sred[kDecideThreads / 64][5];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const double w = __shfl_xor(v5[k], o, 64);
                v5[k] = k == 4 ? fmax(v5[k], w) : v5[k] + w;
            }
        if ((tid & 63) == 0)
#pragma unroll
            for (int k = 0; k < 5; k++) sred[tid >> 6][k] = v5[k];
        __syncthreads();
        if (tid == 0) {
            double r[5];
#pragma unroll
            for (int k = 0; k < 5; k++) {
                r[k] = sred[0][k];
                for (int w = 1; w < kDecideThreads / 64; w++) r[k] = k == 4 ? fmax(r[k], sred[w][k]) : r[k] + sred[w][k];
            }
            BaState& st = *d.st;
            st.cand_cost = r[0]; st.mcc = r[1]; st.snorm2 = r[2]; st.xcnorm2 = r[3]; st.gmax_pts = r[4];
            lm_decide(d, st, b, gmax_cam);
        }
        return;
    }
    if (MODE == kGramInit) {
        const double gmp = wg_sum_parts<kDecideThreads>(d.wpart, nwp, 4, true);
        if (tid == 0) {
            BaState& st = *d.st;
            st.gmax_pts = gmp;
            // the oracle's first gradient check (have_jac at iteration 0)
            if (fmax(gmax_cam, gmp) <= 1e-10) { st.termination = 1; st.done = 1; }
            else if (st.max_iters <= 0) { st.termination = 0; st.done = 1; }
        }
        return;
    }
}

// the oracle's accept / reject step (oracle/ba.c, the loop after the solve)
__device__ void lm_decide(const BaDev& d, BaState& st, int cand, double gmax_cam)
{
    st.iter++;
    const bool valid = !st.fail && st.mcc > 0.0;
    st.fail = 0;
    if (!valid) {
        if (++st.consecutive_invalid >= 5) { st.termination = 3; st.usable = 0; st.done = 1; return; }
        st.radius /= st.decrease_factor;
        st.decrease_factor *= 2.0;
        if (st.radius <= 1e-32) { st.termination = 2; st.done = 1; return; }
    } else {
        st.consecutive_invalid = 0;
        double cc = st.cand_cost;
        if (!isfinite(cc)) cc = DBL_MAX;
        const double snorm = sqrt(st.snorm2);
        if (snorm <= 1e-8 * (st.xnorm + 1e-8)) { st.termination = 1; st.done = 1; return; }
        if (fabs(st.cost - cc) <= 1e-6 * st.cost) { st.termination = 1; st.done = 1; return; }
        const double rel = (st.cost - cc) / st.mcc;
        if (rel > 1e-3) {
            st.cur = cand;                        // x, r, J, g, [U | g_c] of the candidate
            st.cost = cc;
            st.xnorm = sqrt(st.xcnorm2);
            const double q = 2.0 * rel - 1.0;
            st.radius = fmin(1e16, st.radius / fmax(1.0 / 3.0, 1.0 - q * q * q));
            st.decrease_factor = 2.0;
            st.successful++;
            // the new Jacobian's gradient check (the oracle's next loop top)
            if (fmax(gmax_cam, st.gmax_pts) <= 1e-10) { st.termination = 1; st.done = 1; return; }
        } else {
            st.radius /= st.decrease_factor;
            st.decrease_factor *= 2.0;
            if (st.radius <= 1e-32) { st.termination = 2; st.done = 1; return; }
        }
    }
    if (st.iter >= st.max_iters) { st.termination = 0; st.done = 1; }
}

// ---- A: point chunks -> V_p^-1, W / Y in LDS, frame-pair Schur partials ----
constexpr int kSchurThreads = 128;

__global__ __launch_bounds__(kSchurThreads) void ba_schur_pts(BaDev d)
{
    __shared__ double sW[kChunk][30];     // per observation slot: W (10 x 3)
    __shared__ double sY[kChunk][30];     // Y = W V^-1
    __shared__ double sG[kChunk][3];      // point gradient (scaled), per point slot
    __shared__ double sZero[3];
    __shared__ int s_fail;
    const BaState& st = *d.st;
    if (st.done) return;
    const int cur = st.cur;
    const double radius = st.radius;
    const PtChunk ch = d.pch[blockIdx.x];
    const int n = ch.nobs, npts = ch.len, tid = threadIdx.x;
    if (tid == 0) s_fail = 0;
    if (tid < 3) sZero[tid] = 0.0;
    __syncthreads();
    const double* J = d.J[cur];
    const double* g = d.g[cur];
    // phase 1: one thread per observation slot (point q / n, slot q % n): the
    // point's V_p + D_p / radius and its inverse (every slot of the point
    // computes the same values), then the slot's W = J_c' J_p and Y = W V_p^-1
    BA_DT(0, 0);
    if (tid < npts * n || (n == 0 && tid < npts)) {
        const int lp = n ? tid / n : tid, a = n ? tid - lp * n : 0;
        const int p = ch.start + lp;
        const int q0 = ch.qstart + lp * n;
        double V[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        const double sp[3] = {d.scale[d.nc + 3 * p], d.scale[d.nc + 3 * p + 1], d.scale[d.nc + 3 * p + 2]};
        for (int aa = 0; aa < n; aa++) {
            const double* Jo = J + (size_t)(q0 + aa) * 2 * NJ;
            const double jp0[3] = {Jo[10] * sp[0], Jo[11] * sp[1], Jo[12] * sp[2]};
            const double jp1[3] = {Jo[NJ + 10] * sp[0], Jo[NJ + 11] * sp[1], Jo[NJ + 12] * sp[2]};
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) V[i * 3 + j] += jp0[i] * jp0[j] + jp1[i] * jp1[j];
        }
        // LM damping: clamp(diag) / radius (the diagonal is V's own)
#pragma unroll
        for (int k = 0; k < 3; k++) V[k * 4] += fmin(fmax(V[k * 4], 1e-6), 1e32) / radius;
        double L[9];
#pragma unroll
        for (int i = 0; i < 9; i++) L[i] = V[i];
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = L[j * 3 + j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= L[j * 3 + k] * L[j * 3 + k];
            if (!(s > 0.0) || !isfinite(s)) ok = false;
            const double dd = sqrt(s);
            L[j * 3 + j] = dd;
#pragma unroll
            for (int i = j + 1; i < 3; i++) {
                double t = L[i * 3 + j];
#pragma unroll
                for (int k = 0; k < j; k++) t -= L[i * 3 + k] * L[j * 3 + k];
                L[i * 3 + j] = t / dd;
            }
        }
        double Vi[9];
        if (ok) {
#pragma unroll
            for (int cc = 0; cc < 3; cc++) {
                double e[3] = {0, 0, 0};
                e[cc] = 1;
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    double t = e[i];
#pragma unroll
                    for (int k = 0; k < i; k++) t -= L[i * 3 + k] * e[k];
                    e[i] = t / L[i * 3 + i];
                }
#pragma unroll
                for (int i = 2; i >= 0; i--) {
                    double t = e[i];
#pragma unroll
                    for (int k = i + 1; k < 3; k++) t -= L[k * 3 + i] * e[k];
                    e[i] = t / L[i * 3 + i];
                }
#pragma unroll
                for (int rr = 0; rr < 3; rr++) Vi[rr * 3 + cc] = e[rr];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 9; i++) Vi[i] = NAN;
            s_fail = 1;
        }
        if (a == 0) {
#pragma unroll
            for (int i = 0; i < 9; i++) d.Vinv[(size_t)p * 9 + i] = Vi[i];
#pragma unroll
            for (int k = 0; k < 3; k++) sG[lp][k] = g[d.nc + 3 * p + k];
        }
        if (n) {
            const int o = q0 + a, f = d.of[o];
            const double* Jo = J + (size_t)o * 2 * NJ;
            const double jp0[3] = {Jo[10] * sp[0], Jo[11] * sp[1], Jo[12] * sp[2]};
            const double jp1[3] = {Jo[NJ + 10] * sp[0], Jo[NJ + 11] * sp[1], Jo[NJ + 12] * sp[2]};
            const int slot = tid;
#pragma unroll
            for (int i = 0; i < 10; i++) {
                const int ci = cam_col(f, i);
                double w[3] = {0, 0, 0};
                if (ci >= 0) {
                    const double si = d.scale[ci];
                    const double a0 = Jo[i] * si, a1 = Jo[NJ + i] * si;
#pragma unroll
                    for (int k = 0; k < 3; k++) w[k] = a0 * jp0[k] + a1 * jp1[k];
                }
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    sW[slot][3 * i + k] = w[k];
                    sY[slot][3 * i + k] = w[0] * Vi[0 * 3 + k] + w[1] * Vi[1 * 3 + k] + w[2] * Vi[2 * 3 + k];
                }
            }
        }
    }
    __syncthreads();
    BA_DT(0, 1);
    // phase 2: per tuple pair (a, b) the 10 x 11 block sum_q Y_a W_b' (+ Y_a g_p in
    // column 10 on self pairs), each entry summed over the chunk's points in
    // order; a work item is a 2 x 2 register block of entries (four
    // independent FMA chains, two Y and two W triples per point)
    const int items = n * n * 30;
    for (int it = tid; it < items; it += kSchurThreads) {
        const int pr = it / 30, blk = it - pr * 30, a = pr / n, bb = pr - a * n;
        const int ii0 = 2 * (blk / 6), jj0 = 2 * (blk - 6 * (blk / 6));
        const double* y0 = sY[a] + 3 * ii0;                   // + q * n * 30
        const double* w[2];
        int ws[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int jj = jj0 + u;
            if (jj < 10) { w[u] = sW[bb] + 3 * jj; ws[u] = n * 30; }
            else if (jj == 10 && a == bb) { w[u] = sG[0]; ws[u] = 3; }
            else { w[u] = sZero; ws[u] = 0; }
        }
        double acc[2][2] = {{0, 0}, {0, 0}};
#pragma unroll 4
        for (int q = 0; q < npts; q++) {
            const double* ya = y0 + q * n * 30;
            const double* yb = ya + 3;
            const double* wa = w[0] + q * ws[0];
            const double* wb = w[1] + q * ws[1];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                acc[0][0] = fma(ya[k], wa[k], acc[0][0]);
                acc[0][1] = fma(ya[k], wb[k], acc[0][1]);
                acc[1][0] = fma(yb[k], wa[k], acc[1][0]);
                acc[1][1] = fma(yb[k], wb[k], acc[1][1]);
            }
        }
        double* out = d.spart + (size_t)d.bpos[ch.part + pr] * kBlk;
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int u = 0; u < 2; u++)
                if (jj0 + u < 11) out[(ii0 + r) * 11 + jj0 + u] = acc[r][u];
    }
    if (s_fail && tid == 0) atomicOr(&d.st->fail, 1);
#ifdef BA_DIAG
    __syncthreads();
    BA_DT(0, 2);
    if (tid == 0) g_dt[0][blockIdx.x][3] = n;
#endif
}

// ---- B: one workgroup: S y_c = rc ----
// The lower triangle of S is spread over the 256 threads, EPT elements each in
// registers (element e = tid + 256 u, row-major over the triangle).  Right-
// looking elimination on the unscaled factor: step j updates every element
// (i, k), k > j, by a_ik -= a_ij a_kj / a_jj from column j, which the owners of
// column j published into a double-buffered LDS vector at the end of step
// j - 1, and the rhs rides along (b_i -= a_ij b_j / a_jj): one barrier per
// column.  Back solve x_i = (z_i - sum_{k > i} a_ki x_k) / a_ii, column by
// column: the owners of row i update z, one barrier per column.
constexpr int kMaxNc = 136;

// the reduced camera system [S | rc] (nc x (nc + 1), row-major) from the
// scaled [U | g_c], the damping and the Schur buckets: one thread per entry
__global__ __launch_bounds__(256) void ba_s_assemble(BaDev d)
{
    const BaState& st = *d.st;
    if (st.done) return;
    const int n = d.nc, ld = n + 1, e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n * ld) return;
    const int i = e / ld, j = e - i * ld;
    if (j > i && j < n) return;                       // lower triangle + rhs only
    double u = cam_entry(d.blkU[st.cur], d.nf, false, n, i, j);
    if (i == j) u += fmin(fmax(u, 1e-6), 1e32) / st.radius;
    d.Sg[e] = u - cam_entry(d.blkS, d.nf, true, n, i, j);
}

// Rows in registers (nc <= 128): thread i keeps row i of S (NP doubles,
// compile-time indices).  Step j: every thread publishes its a_ij (column j =
// row j: the trailing matrix is updated on both sides of the diagonal), then
// threads i > j update their entries k > j by a_ik -= t_i a_kj, t_i = a_ij /
// a_jj, with a_kj read from LDS in pairs (uniform addresses: broadcasts).
// Thread i stops at step i, so after the elimination it holds row i (k <= i)
// and column i (k > i) of the unscaled factor: the forward solve rides along,
// and the back solve x_i = (z_i - sum_{k > i} a_ki x_k) / a_ii needs only its
// own column and the published x_k.  One wave: no barrier (a wave's LDS
// operations complete in order); two waves: one barrier per column.
template <int NP, int NW>
__global__ __launch_bounds__(64 * NW) void ba_camera_solve_rows(BaDev d)
{
    __shared__ __attribute__((aligned(16))) double col[2][NP + 2];   // published column j, b_j
    __shared__ double xs[NP];
    const BaState& st = *d.st;
    if (st.done) return;
    const int n = d.nc, ld = n + 1, i = threadIdx.x;
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const int r = i > k ? i : k, c = i > k ? k : i;   // the lower triangle, mirrored
        a[k] = i < n && k < n ? d.Sg[r * ld + c] : (i == k ? 1.0 : 0.0);
    }
    double b = i < n ? d.Sg[i * ld + n] : 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        double* cj = col[j & 1];
        if (i < NP) cj[i] = a[j];
        if (i == j) cj[NP] = b;
        if (NW > 1) __syncthreads();
        else { __builtin_amdgcn_wave_barrier(); __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
        const double ajj = cj[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) { ok = false; break; }   // uniform: one LDS value
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
    if (!ok) {
        if (i == 0) atomicOr(&d.st->fail, 1);
        return;
    }
    double diag = 1.0;
#pragma unroll
    for (int k = 0; k < NP; k++) if (k == i) diag = a[k];
#pragma unroll
    for (int k = NP - 1; k >= 0; k--) {
        if (i == k) xs[k] = b / diag;
        if (NW > 1) __syncthreads();
        else { __builtin_amdgcn_wave_barrier(); __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
        if (i < k) b = fma(-a[k], xs[k], b);
    }
    if (NW > 1) __syncthreads();
    if (i < n) {
        const double y = xs[i];
        d.yc[i] = y;
        if (!isfinite(y)) atomicOr(&d.st->fail, 1);
    }
}

// One wave: the same elimination as ba_camera_solve_rows (bit-identical
// operations), with column j's entries a_kj broadcast by v_readlane from lane
// k (k and j are compile-time constants of the unrolled loops) instead of a
// published LDS column: no LDS round trip or wave barrier per column.  The
// back solve broadcasts b_k and a_kk the same way.  nc <= 64
// (scripts/diag/chol_lane.hip: 22.9 -> 18.0 us at nc = 46; reciprocal pivots
// measured slower in the kernel, 30.9 us).
__device__ __forceinline__ double lane_bcast(double v, int lane)
{
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)u, lane), hi = __builtin_amdgcn_readlane((int)(u >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NP>
__global__ __launch_bounds__(64) void ba_camera_solve_lane(BaDev d)
{
    const BaState& st = *d.st;
    if (st.done) return;
    const int n = d.nc, ld = n + 1, i = threadIdx.x;
    double a[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const int r = i > k ? i : k, c = i > k ? k : i;   // the lower triangle, mirrored
        a[k] = i < n && k < n ? d.Sg[r * ld + c] : (i == k ? 1.0 : 0.0);
    }
    double b = i < n ? d.Sg[i * ld + n] : 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const double ajj = lane_bcast(a[j], j), bj = lane_bcast(b, j);
        ok = ok && ajj > 0.0 && isfinite(ajj);
        const double t = i > j ? a[j] / ajj : 0.0;
#pragma unroll
        for (int k = j + 1; k < NP; k++) a[k] = fma(-t, lane_bcast(a[j], k), a[k]);
        b = fma(-t, bj, b);
    }
    if (!ok) {
        if (i == 0) atomicOr(&d.st->fail, 1);
        return;
    }
    double x = 0;
#pragma unroll
    for (int k = NP - 1; k >= 0; k--) {
        const double xk = lane_bcast(b, k) / lane_bcast(a[k], k);
        if (i == k) x = xk;
        b = fma(i < k ? -a[k] : 0.0, xk, b);
    }
    if (i < n) {
        d.yc[i] = x;
        if (!isfinite(x)) atomicOr(&d.st->fail, 1);
    }
}

template <int kSolveThreads, int EPT>
__global__ __launch_bounds__(kSolveThreads) void ba_camera_solve(BaDev d)
{
    __shared__ double col[2][kMaxNc];
    __shared__ double zb[kMaxNc], dg[kMaxNc], xs[kMaxNc];
    const BaState& st = *d.st;
    if (st.done) return;
    const int n = d.nc, ld = n + 1, tid = threadIdx.x;
    const int ne = n * (n + 1) / 2;
    double a[EPT];
    int rik[EPT];                 // row << 16 | column; -1 for no element
#pragma unroll
    for (int u = 0; u < EPT; u++) {
        const int e = tid + kSolveThreads * u;
        int i = -1, k = -1;
        double v = 0;
        if (e < ne) {
            i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while ((i + 1) * (i + 2) / 2 <= e) i++;
            while (i * (i + 1) / 2 > e) i--;
            k = e - i * (i + 1) / 2;
            v = d.Sg[i * ld + k];              // ba_s_assemble: lower triangle + rhs
        }
        a[u] = v;
        rik[u] = e < ne ? (i << 16) | k : -1;
    }
#define RI(u) (rik[u] >> 16)
#define RK(u) (rik[u] < 0 ? -1 : (rik[u] & 0xffff))
    if (tid < n) zb[tid] = d.Sg[tid * ld + n];
#pragma unroll
    for (int u = 0; u < EPT; u++)
        if (RK(u) == 0) {
            col[0][RI(u)] = a[u];
            if (RI(u) == 0) dg[0] = a[u];
        }
    __syncthreads();
    bool fail = false;
    for (int j = 0; j < n; j++) {
        const double* cj = col[j & 1];
        double* cn = col[(j + 1) & 1];
        const double ajj = cj[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) { fail = true; break; }   // uniform: one LDS value
        const double inv = 1.0 / ajj;
#pragma unroll
        for (int u = 0; u < EPT; u++) {
            if (RK(u) > j) {
                a[u] = fma(-(cj[RI(u)] * cj[RK(u)]), inv, a[u]);
                if (RK(u) == j + 1) {
                    cn[RI(u)] = a[u];
                    if (RI(u) == j + 1) dg[j + 1] = a[u];
                }
            }
        }
        if (tid > j && tid < n) zb[tid] = fma(-cj[tid], zb[j] * inv, zb[tid]);
        __syncthreads();
    }
    if (fail) {
        if (tid == 0) atomicOr(&d.st->fail, 1);
        return;
    }
    for (int i = n - 1; i >= 0; i--) {
        const double xi = zb[i] / dg[i];
#pragma unroll
        for (int u = 0; u < EPT; u++)
            if (RI(u) == i && RK(u) < i) zb[RK(u)] = fma(-a[u], xi, zb[RK(u)]);
        if (tid == 0) xs[i] = xi;
        __syncthreads();
    }
    for (int i = tid; i < n; i += kSolveThreads) {
        const double y = xs[i];
        d.yc[i] = y;
        if (!isfinite(y)) atomicOr(&d.st->fail, 1);
    }
#undef RI
#undef RK
}

// ---- C: back substitution, candidate, model cost change, the speculative
// residuals / Jacobian / cost / point gradient at the candidate, and the
// candidate's frame Gram partials.  A workgroup owns one Schur point chunk
// (points of one frame tuple, <= 64 observation slots, slot = point * n + a
// with a the tuple position) and has three waves: phase 1 one thread per point
// (back substitution, candidate point), phase 2 one observation slot per lane
// in every wave, wave w computing the Jacobian columns of its parameter block
// (K, extrinsics, point) along the shared value path, phase 3 one thread per
// point (its slots' gradient terms, in slot order) and, per tuple position a
// (frame f_a), the chunk's share of f_a's [J_c | r]' [J_c | r] block on the
// f64 matrix cores: v_mfma_f64_16x16x4 with the 4 rows of two points' a-slots
// as k and the 11 columns (10 scaled camera partials + the residual) on both
// sides (lane l holds M[k = l >> 4][c = l & 15] as A and as B). ----
constexpr int kUpdSlots = 64;
constexpr int kUpdThreads = 3 * kUpdSlots;
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kUpdThreads) void ba_update(BaDev d)
{
    __shared__ double sXc[kUpdSlots][3], sStep[kUpdSlots][3], sU[kUpdSlots][3];
    __shared__ double sG[kUpdSlots][2][11];     // the candidate's scaled [J_c | r] rows per slot
    __shared__ int s_fail;
    const BaState& st = *d.st;
    if (st.done) return;
    const int cur = st.cur, cand = 1 - cur, nc = d.nc, tid = threadIdx.x;
    const PtChunk ch = d.pch[blockIdx.x];
    const int n = ch.nobs, npts = ch.len, nslot = npts * n;
    const double* x = d.x[cur];
    double* xc = d.x[cand];
    const double* J = d.J[cur];
    const double* r = d.r[cur];
    double cc = 0, mcc = 0, sn = 0, xx = 0, gm = 0;
    if (tid == 0) s_fail = 0;
    __syncthreads();
    BA_DT(1, 0);
    // phase 1: y_p = V_p^-1 (g_p - W_p' y_c); step = -y; candidate point
    if (tid < npts) {
        const int p = ch.start + tid, q0 = ch.qstart + tid * n;
        const double* sp = d.scale + nc + 3 * p;
        double t[3] = {d.g[cur][nc + 3 * p], d.g[cur][nc + 3 * p + 1], d.g[cur][nc + 3 * p + 2]};
        for (int o = q0; o < q0 + n; o++) {
            const int f = d.of[o];
            const double* Jo = J + (size_t)o * 2 * NJ;
            double jy0 = 0, jy1 = 0;
#pragma unroll
            for (int i = 0; i < 10; i++) {
                const int ci = cam_col(f, i);
                if (ci < 0) continue;
                const double s = d.scale[ci] * d.yc[ci];
                jy0 += Jo[i] * s;
                jy1 += Jo[NJ + i] * s;
            }
#pragma unroll
            for (int k = 0; k < 3; k++) t[k] -= Jo[10 + k] * sp[k] * jy0 + Jo[NJ + 10 + k] * sp[k] * jy1;
        }
        const double* Vi = d.Vinv + (size_t)p * 9;
        const double* X = x + 4 + 6 * d.nf + 3 * p;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const double y = Vi[3 * k] * t[0] + Vi[3 * k + 1] * t[1] + Vi[3 * k + 2] * t[2];
            if (!isfinite(y)) s_fail = 1;
            const double stp = -y;
            const double delta = stp * sp[k];
            const double v = X[k] + delta;
            sStep[tid][k] = stp;
            sXc[tid][k] = v;
            xc[4 + 6 * d.nf + 3 * p + k] = v;
            sn += delta * delta;
            if (n > 0) xx += v * v;           // unobserved points: not in Ceres's program
        }
    }
    __syncthreads();
    BA_DT(1, 1);
    // phase 2: slot = lane, parameter block = wave
    const int slot = tid & (kUpdSlots - 1), part = tid / kUpdSlots;
    if (slot < nslot) {
        const int lp = slot / n;
        const int p = ch.start + lp, o = ch.qstart + slot, f = d.of[o];
        const double* sp = d.scale + nc + 3 * p;
        double Kc[4], Ec[6], Xc[3];
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int ci = cam_col(f, i);
            const double xv = x[i < 4 ? i : 4 + 6 * f + (i - 4)];
            const double v = ci < 0 ? xv : xv + d.scale[ci] * -d.yc[ci];   // frame 0's extrinsics: constant
            if (i < 4) Kc[i] = v;
            else Ec[i - 4] = v;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) Xc[k] = sXc[lp][k];
        double rc[2];
        double* Jw = d.J[cand] + (size_t)o * 2 * NJ;
        if (part == 0) {
            double Jc[2][4];
            eval_obs<4, 0>(d, Kc, Ec, Xc, o, rc, Jc);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                Jw[i] = Jc[0][i]; Jw[NJ + i] = Jc[1][i];
                sG[slot][0][i] = Jc[0][i] * d.scale[i];
                sG[slot][1][i] = Jc[1][i] * d.scale[i];
            }
        } else if (part == 1) {
            double Jc[2][6];
            eval_obs<6, 4>(d, Kc, Ec, Xc, o, rc, Jc);
#pragma unroll
            for (int i = 0; i < 6; i++) {
                Jw[4 + i] = Jc[0][i]; Jw[NJ + 4 + i] = Jc[1][i];
                const int ci = cam_col(f, 4 + i);     // frame 0's extrinsics: constant, zero columns
                sG[slot][0][4 + i] = ci < 0 ? 0.0 : Jc[0][i] * d.scale[ci];
                sG[slot][1][4 + i] = ci < 0 ? 0.0 : Jc[1][i] * d.scale[ci];
            }
        } else {
            double Jc[2][3];
            double c = eval_obs<3, 10>(d, Kc, Ec, Xc, o, rc, Jc);
            if (!isfinite(c)) c = INFINITY;
            cc = c;
#pragma unroll
            for (int i = 0; i < 3; i++) { Jw[10 + i] = Jc[0][i]; Jw[NJ + 10 + i] = Jc[1][i]; }
            d.r[cand][2 * o] = rc[0];
            d.r[cand][2 * o + 1] = rc[1];
            sG[slot][0][10] = rc[0];
            sG[slot][1][10] = rc[1];
#pragma unroll
            for (int k = 0; k < 3; k++) sU[slot][k] = Jc[0][k] * rc[0] + Jc[1][k] * rc[1];
            // model cost change -(J_s step) . (f + J_s step / 2), current Jacobian
            const double* Jo = J + (size_t)o * 2 * NJ;
            double mr0 = 0, mr1 = 0;
#pragma unroll
            for (int i = 0; i < 10; i++) {
                const int ci = cam_col(f, i);
                if (ci < 0) continue;
                const double s = d.scale[ci] * -d.yc[ci];
                mr0 += Jo[i] * s;
                mr1 += Jo[NJ + i] * s;
            }
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const double s = sp[k] * sStep[lp][k];
                mr0 += Jo[10 + k] * s;
                mr1 += Jo[NJ + 10 + k] * s;
            }
            mcc = -(mr0 * (r[2 * o] + mr0 / 2.0) + mr1 * (r[2 * o + 1] + mr1 / 2.0));
        }
    }
    __syncthreads();
    BA_DT(1, 2);
    // phase 3: the point gradient at the candidate, its slots in order
    if (tid < npts) {
        const int p = ch.start + tid;
        double u[3] = {0, 0, 0};
        for (int a = 0; a < n; a++)
#pragma unroll
            for (int k = 0; k < 3; k++) u[k] += sU[tid * n + a][k];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gm = fmax(gm, fabs(u[k]));
            d.g[cand][nc + 3 * p + k] = u[k] * d.scale[nc + 3 * p + k];
        }
    }
    // the chunk's frame Gram partials: tuple position a on wave a % 3
    {
        const int lane = tid & 63, c = lane & 15, k = lane >> 4, rr = k & 1, half = k >> 1;
        for (int a = part; a < n; a += 3) {
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int m = 0; 2 * m < npts; m++) {
                const int lp = 2 * m + half;
                const double v = lp < npts && c < 11 ? sG[lp * n + a][rr][c] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
            }
            double* out = d.gpart + (size_t)d.fppos[ch.fpart + a] * kBlk;   // D: col = lane & 15, row = (lane >> 4) + 4 reg
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int row = k + 4 * q;
                if (row < 10 && c < 11) out[row * 11 + c] = acc[q];
            }
        }
    }
    // the camera part of the candidate (tangent entries 0 .. nc) and frame 0's
    // constant extrinsics: workgroup 0
    if (blockIdx.x == 0) {
        for (int i = tid; i < nc; i += kUpdThreads) {
            const int full = full_of(d, i);
            const double delta = -d.yc[i] * d.scale[i];
            const double v = x[full] + delta;
            xc[full] = v;
            sn += delta * delta;
            const int fr = i < 4 ? -1 : 1 + (i - 4) / 6;    // a frame without observations: not in the program
            if (fr < 0 || d.gcs[fr + 1] > d.gcs[fr]) xx += v * v;
        }
        for (int i = tid; i < 6; i += kUpdThreads) xc[4 + i] = x[4 + i];
    }
    // the five workgroup partials in one pass (same tree as wg_reduce: lanes by
    // xor shuffles, then the waves in order)
    __shared__ double sred[kUpdThreads / 64][5];
    double v5[5] = {cc, mcc, sn, xx, gm};
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const double w = __shfl_xor(v5[k], o, 64);
            v5[k] = k == 4 ? fmax(v5[k], w) : v5[k] + w;
        }
    if ((tid & 63) == 0)
#pragma unroll
        for (int k = 0; k < 5; k++) sred[tid >> 6][k] = v5[k];
    __syncthreads();
    if (tid == 0) {
        double t[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            t[k] = sred[0][k];
            for (int w = 1; w < kUpdThreads / 64; w++) t[k] = k == 4 ? fmax(t[k], sred[w][k]) : t[k] + sred[w][k];
        }
        double* w = d.wpart + (size_t)blockIdx.x * 8;
        w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3]; w[4] = t[4];
        if (s_fail) atomicOr(&d.st->fail, 1);
    }
    BA_DT(1, 3);
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
    if (no == 0) {
        // zero cost and gradient: the oracle's first gradient check ends the solve
        sum->termination = 1;
        return SLAM_OK;
    }
    const int E = nc * (nc + 1);
    hipStream_t s = c->stream;
#ifdef BA_HOST_TIMING
    std::chrono::steady_clock::time_point ht[16];
#endif
    BA_T(0);

    // ---- host bookkeeping (once per solve) ----
    // observations grouped by point (CSR, observation order within a point)
    std::vector<int> pstart(np + 1, 0), plist(no);
    for (int o = 0; o < no; o++) pstart[op[o] + 1]++;
    for (int p = 0; p < np; p++) pstart[p + 1] += pstart[p];
    {
        std::vector<int> fill(np, 0);
        for (int o = 0; o < no; o++) plist[pstart[op[o]] + fill[op[o]]++] = o;
    }
    BA_T(6);
    // points grouped by the frame tuple of their observations (CSR order): a
    // group's points feed the same frame-pair buckets, so one chunk's pair
    // blocks are sums over its points with no scatter
    std::vector<int> porder(np);
    std::vector<PtChunk> pch;
    std::vector<int> gframes;
    int nparts = 0, nfp = 0;
    {
        // tuples hashed (FNV-1a over the frame sequence) into an open-addressing
        // table, the stored tuple compared on a hit; groups numbered by first
        // appearance
        uint32_t tmask = 1023;
        std::vector<int> table((size_t)tmask + 1, -1), pg(np), tstart(1, 0), tfr;
        std::vector<uint64_t> thash;
        auto bucket = [&](uint64_t h) { return (uint32_t)(h ^ (h >> 29)) & tmask; };
        // the common tuple (consecutive frames f0, f0 + 1, ...: a track) by direct
        // index (f0, n); any other tuple through the hash
        std::vector<int> track((size_t)(nf + 1) * (kChunk + 1), -1);
        for (int p = 0; p < np; p++) {
            const int q0 = pstart[p], n = pstart[p + 1] - q0;
            if (n > kChunk) return set_err(c, SLAM_E_UNSUPPORTED, "BA point with more than 64 observations");
            int f0 = n ? of[plist[q0]] : nf;
            for (int k = 1; k < n && f0 >= 0; k++)
                if (of[plist[q0 + k]] != f0 + k) f0 = -1;
            int* tslot = f0 >= 0 ? &track[(size_t)f0 * (kChunk + 1) + n] : nullptr;
            if (tslot && *tslot >= 0) { pg[p] = *tslot; continue; }
            uint64_t h = 1469598103934665603ull ^ (uint64_t)n;
            for (int q = q0; q < q0 + n; q++) h = (h ^ (uint64_t)of[plist[q]]) * 1099511628211ull;
            uint32_t slot = bucket(h);
            int g = -1;
            for (;; slot = (slot + 1) & tmask) {
                const int e = table[slot];
                if (e < 0) break;
                if (thash[e] != h || tstart[e + 1] - tstart[e] != n) continue;
                bool same = true;
                for (int k = 0; same && k < n; k++) same = tfr[tstart[e] + k] == of[plist[q0 + k]];
                if (same) { g = e; break; }
            }
            if (g < 0) {
                g = (int)thash.size();
                table[slot] = g;
                thash.push_back(h);
                for (int q = q0; q < q0 + n; q++) tfr.push_back(of[plist[q]]);
                tstart.push_back((int)tfr.size());
                if (tslot) *tslot = g;
                if (2 * thash.size() > tmask) {           // keep the load under 1/2
                    tmask = 2 * tmask + 1;
                    table.assign((size_t)tmask + 1, -1);
                    for (int e = 0; e < (int)thash.size(); e++) {
                        uint32_t t = bucket(thash[e]);
                        while (table[t] >= 0) t = (t + 1) & tmask;
                        table[t] = e;
                    }
                }
            }
            pg[p] = g;
        }
        const int ng = (int)thash.size();
        std::vector<int> gcount(ng + 1, 0), fill(ng, 0);
        for (int p = 0; p < np; p++) gcount[pg[p] + 1]++;
        for (int g = 0; g < ng; g++) gcount[g + 1] += gcount[g];
        for (int p = 0; p < np; p++) porder[gcount[pg[p]] + fill[pg[p]]++] = p;
        gframes.assign((size_t)std::max(ng, 1) * 64, 0);
        for (int g = 0; g < ng; g++) {
            const int n = tstart[g + 1] - tstart[g];
            for (int k = 0; k < n; k++) gframes[(size_t)g * 64 + k] = tfr[tstart[g] + k];
            const int per = std::max(1, kChunk / std::max(n, 1));
            for (int st = gcount[g]; st < gcount[g + 1]; st += per) {
                const int len = std::min(per, gcount[g + 1] - st);
                pch.push_back(PtChunk{st, len, n, nparts, g, nfp, 0});
                nparts += n * n;
                nfp += n;
            }
        }
    }
    BA_T(7);
    // device numbering: points in group order (p' = rank in porder), their
    // observations consecutive in CSR order (q), so a chunk's points and
    // observation slots are contiguous ranges (no index lists on the device).
    // The host builds the maps (q -> caller's observation, p' -> caller's
    // point); ba_import gathers the arrays on the device, ba_export scatters
    // the solution back.
    std::vector<int> qstart(np + 1, 0), qsrc(std::max(no, 1));
    {
        int q = 0;
        for (int pp = 0; pp < np; pp++) {
            const int p = porder[pp];
            qstart[pp] = q;
            for (int k = pstart[p]; k < pstart[p + 1]; k++) qsrc[q++] = plist[k];
        }
        qstart[np] = q;
        for (PtChunk& ch : pch) ch.qstart = qstart[ch.start];
    }
    BA_T(8);
    // observations (q) bucketed by frame, cut into gram chunks (initial Jacobian)
    std::vector<int> flist(no);
    std::vector<Chunk> gch;
    std::vector<int> gcs(nf + 1, 0);
    {
        std::vector<int> fstart(nf + 1, 0), fill(nf, 0);
        for (int o = 0; o < no; o++) fstart[of[o] + 1]++;
        for (int f = 0; f < nf; f++) fstart[f + 1] += fstart[f];
        for (int q = 0; q < no; q++) {
            const int f = of[qsrc[q]];
            flist[fstart[f] + fill[f]++] = q;
        }
        for (int f = 0; f < nf; f++) {
            gcs[f] = (int)gch.size();
            for (int st = fstart[f]; st < fstart[f + 1]; st += kGChunk)
                gch.push_back(Chunk{f, st, std::min(kGChunk, fstart[f + 1] - st)});
        }
        gcs[nf] = (int)gch.size();
    }
    BA_T(9);
    const int nb2 = nf * nf;
    std::vector<int> bstart(nb2 + 1, 0), bpos(std::max(nparts, 1));
    {
        for (const PtChunk& ch : pch)
            for (int pr = 0; pr < ch.nobs * ch.nobs; pr++) {
                const int* fr = &gframes[(size_t)ch.group * 64];
                bstart[fr[pr / ch.nobs] * nf + fr[pr % ch.nobs] + 1]++;
            }
        for (int b = 0; b < nb2; b++) bstart[b + 1] += bstart[b];
        std::vector<int> fill(nb2, 0);
        for (const PtChunk& ch : pch)
            for (int pr = 0; pr < ch.nobs * ch.nobs; pr++) {
                const int* fr = &gframes[(size_t)ch.group * 64];
                const int bk = fr[pr / ch.nobs] * nf + fr[pr % ch.nobs];
                bpos[ch.part + pr] = bstart[bk] + fill[bk]++;
            }
    }
    // ba_update's frame Gram partials per frame, in chunk order
    std::vector<int> fpstart(nf + 1, 0), fppos(std::max(nfp, 1));
    {
        for (const PtChunk& ch : pch)
            for (int a = 0; a < ch.nobs; a++) fpstart[gframes[(size_t)ch.group * 64 + a] + 1]++;
        for (int f = 0; f < nf; f++) fpstart[f + 1] += fpstart[f];
        std::vector<int> fill(nf, 0);
        for (const PtChunk& ch : pch)
            for (int a = 0; a < ch.nobs; a++) {
                const int f = gframes[(size_t)ch.group * 64 + a];
                fppos[ch.fpart + a] = fpstart[f] + fill[f]++;
            }
    }
    const int ngch = (int)gch.size(), npch = (int)pch.size();

    BA_T(1);
    // tangent vector norm over Ceres's reduced program (Program::RemoveFixedBlocks:
    // frame 0's constant extrinsics and every block no residual uses are
    // dropped), caller's order
    double xnorm = 0;
    {
        std::vector<unsigned char> fused(nf, 0), pused(np, 0);
        for (int o = 0; o < no; o++) { fused[of[o]] = 1; pused[op[o]] = 1; }
        for (int i = 0; i < 4; i++) xnorm += K4[i] * K4[i];
        for (int i = 6; i < 6 * nf; i++) if (fused[i / 6]) xnorm += ext6[i] * ext6[i];
        for (int i = 0; i < 3 * np; i++) if (pused[i / 3]) xnorm += pts3[i] * pts3[i];
    }
    xnorm = std::sqrt(xnorm);

    const unsigned gobs = (unsigned)((no + 127) / 128);
    const unsigned gpt128 = (unsigned)std::max(1, (np + 127) / 128);
    const unsigned gupd = (unsigned)std::max(1, npch);
    const int nwp = (int)std::max({gobs, gpt128, gupd});

    // ---- device layout ----
    size_t off = 0;
    auto carve = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    // the uploaded arrays first: one pinned image, one copy
    const size_t o_rof = carve(4 * (size_t)no), o_roxy = carve(16 * (size_t)no), o_qsrc = carve(4 * (size_t)no),
                 o_por = carve(4 * (size_t)std::max(np, 1)), o_xin = carve(8 * (size_t)NX),
                 o_ps = carve(4 * (size_t)(np + 1)), o_fl = carve(4 * (size_t)no),
                 o_gch = carve(sizeof(Chunk) * std::max(1, ngch)), o_gcs = carve(4 * gcs.size()),
                 o_pch = carve(sizeof(PtChunk) * std::max(1, npch)),
                 o_gf = carve(4 * gframes.size()), o_bs = carve(4 * bstart.size()), o_bl = carve(4 * bpos.size()),
                 o_fps = carve(4 * fpstart.size()), o_fpl = carve(4 * fppos.size()),
                 o_st = carve(sizeof(BaState));
    const size_t up_bytes = off;
    const size_t o_of = carve(4 * (size_t)no), o_op = carve(4 * (size_t)no), o_oxy = carve(16 * (size_t)no),
                 o_x0 = carve(8 * (size_t)NX), o_xout = carve(8 * (size_t)NX),
                 o_x1 = carve(8 * (size_t)NX), o_r0 = carve(16 * (size_t)no),
                 o_r1 = carve(16 * (size_t)no), o_J0 = carve(8 * 2 * NJ * (size_t)no),
                 o_J1 = carve(8 * 2 * NJ * (size_t)no), o_g0 = carve(8 * (size_t)N), o_g1 = carve(8 * (size_t)N),
                 o_u0 = carve(8 * (size_t)kBlk * nf), o_u1 = carve(8 * (size_t)kBlk * nf), o_sc = carve(8 * (size_t)N),
                 o_vi = carve(72 * (size_t)std::max(np, 1)), o_yc = carve(8 * (size_t)nc),
                 o_sg = carve(8 * (size_t)E),
                 o_sp = carve(8 * (size_t)kBlk * std::max(nparts, 1)), o_bk = carve(8 * (size_t)kBlk * nb2),
                 o_gp = carve(8 * (size_t)kBlk * std::max({ngch, nfp, 1})),
                 o_wp = carve(64 * (size_t)nwp);
    // pinned host space: the upload image, then the state readbacks and the final x
    char* pin = static_cast<char*>(readback(c, up_bytes + 2 * sizeof(BaState) + 8 * (size_t)NX));
    if (!pin) return set_err(c, SLAM_E_HIP, "pinned staging allocation failed");
    BaState* hst = reinterpret_cast<BaState*>(pin + up_bytes);
    double* hx = reinterpret_cast<double*>(pin + up_bytes + 2 * sizeof(BaState));
    SLAM_HIP(c, c->ba_par.ensure(off));
    char* base = c->ba_par.as<char>();
    BaDev d;
    d.nf = nf; d.np = np; d.no = no; d.nc = nc; d.N = N; d.NX = NX; d.loss = loss; d.a = a;
    d.of = (const int*)(base + o_of); d.op = (const int*)(base + o_op); d.oxy = (const double*)(base + o_oxy);
    d.pstart = (const int*)(base + o_ps); d.flist = (const int*)(base + o_fl);
    d.gch = (const Chunk*)(base + o_gch); d.gcs = (const int*)(base + o_gcs);
    d.pch = (const PtChunk*)(base + o_pch);
    d.gframes = (const int*)(base + o_gf); d.bstart = (const int*)(base + o_bs); d.bpos = (const int*)(base + o_bl);
    d.fpstart = (const int*)(base + o_fps); d.fppos = (const int*)(base + o_fpl);
    d.x[0] = (double*)(base + o_x0); d.x[1] = (double*)(base + o_x1);
    d.r[0] = (double*)(base + o_r0); d.r[1] = (double*)(base + o_r1);
    d.J[0] = (double*)(base + o_J0); d.J[1] = (double*)(base + o_J1);
    d.g[0] = (double*)(base + o_g0); d.g[1] = (double*)(base + o_g1);
    d.blkU[0] = (double*)(base + o_u0); d.blkU[1] = (double*)(base + o_u1);
    d.scale = (double*)(base + o_sc); d.Vinv = (double*)(base + o_vi); d.yc = (double*)(base + o_yc);
    d.Sg = (double*)(base + o_sg);
    d.spart = (double*)(base + o_sp); d.blkS = (double*)(base + o_bk); d.gpart = (double*)(base + o_gp);
    d.wpart = (double*)(base + o_wp);
    d.st = (BaState*)(base + o_st);

    BaState st0;
    std::memset(&st0, 0, sizeof(st0));
    st0.radius = 1e4;
    st0.decrease_factor = 2.0;
    st0.xnorm = xnorm;
    st0.max_iters = max_iters;
    st0.usable = 1;
    auto put = [&](size_t o, const void* src, size_t bytes) { if (bytes) std::memcpy(pin + o, src, bytes); };
    put(o_rof, of, 4 * (size_t)no);
    put(o_roxy, oxy, 16 * (size_t)no);
    put(o_qsrc, qsrc.data(), 4 * (size_t)no);
    put(o_por, porder.data(), 4 * (size_t)np);
    put(o_xin, K4, 32);
    put(o_xin + 32, ext6, sizeof(double) * 6 * nf);
    put(o_xin + 32 + sizeof(double) * 6 * nf, pts3, sizeof(double) * 3 * np);
    put(o_ps, qstart.data(), 4 * (size_t)(np + 1));
    put(o_fl, flist.data(), 4 * (size_t)no);
    put(o_gch, gch.data(), sizeof(Chunk) * ngch);
    put(o_gcs, gcs.data(), 4 * gcs.size());
    put(o_pch, pch.data(), sizeof(PtChunk) * npch);
    put(o_gf, gframes.data(), 4 * gframes.size());
    put(o_bs, bstart.data(), 4 * bstart.size());
    put(o_bl, bpos.data(), 4 * bpos.size());
    put(o_fps, fpstart.data(), 4 * fpstart.size());
    put(o_fpl, fppos.data(), 4 * fppos.size());
    put(o_st, &st0, sizeof(st0));
    SLAM_HIP(c, hipMemcpyAsync(base, pin, up_bytes, hipMemcpyHostToDevice, s));
    // (every bucket / frame block is written by its reduction, empty ones as 0)
    BA_T(2);

    auto camera_solve = [&]() {
        hipLaunchKernelGGL(ba_s_assemble, dim3((E + 255) / 256), dim3(256), 0, s, d);
        if (nc <= 16) hipLaunchKernelGGL((ba_camera_solve_lane<16>), dim3(1), dim3(64), 0, s, d);
        else if (nc <= 28) hipLaunchKernelGGL((ba_camera_solve_lane<28>), dim3(1), dim3(64), 0, s, d);
        else if (nc <= 48) hipLaunchKernelGGL((ba_camera_solve_lane<48>), dim3(1), dim3(64), 0, s, d);
        else if (nc <= 64) hipLaunchKernelGGL((ba_camera_solve_lane<64>), dim3(1), dim3(64), 0, s, d);
        else if (nc <= 96) hipLaunchKernelGGL((ba_camera_solve_rows<96, 2>), dim3(1), dim3(128), 0, s, d);
        else if (nc <= 128) hipLaunchKernelGGL((ba_camera_solve_rows<128, 2>), dim3(1), dim3(128), 0, s, d);
        else hipLaunchKernelGGL((ba_camera_solve<1024, 10>), dim3(1), dim3(1024), 0, s, d);
    };

    // ---- iteration 0: cost + Jacobian, Jacobi scaling, gradient check ----
    const int* dgcs = (const int*)(base + o_gcs);
    const int* dbs = (const int*)(base + o_bs);
    (void)dgcs;
    const int* dpor = (const int*)(base + o_por);
    double* dxout = (double*)(base + o_xout);
    hipLaunchKernelGGL(ba_import, dim3((std::max(np, 4 + 6 * nf) + 127) / 128), dim3(128), 0, s, d,
                       (const int*)(base + o_rof), (const double*)(base + o_roxy), (const int*)(base + o_qsrc), dpor,
                       (const double*)(base + o_xin));
    hipLaunchKernelGGL(ba_eval_init, dim3(gobs), dim3(128), 0, s, d);
    hipLaunchKernelGGL(ba_gram<kGramUnscaled>, dim3(ngch), dim3(128), 0, s, d);
    hipLaunchKernelGGL(ba_frame_reduce<kGramUnscaled>, dim3(nf), dim3(1024), 0, s, d);
    hipLaunchKernelGGL(ba_decide<kGramUnscaled>, dim3(1), dim3(kDecideThreads), 0, s, d, (int)gobs);
    hipLaunchKernelGGL(ba_point_init, dim3(gpt128), dim3(128), 0, s, d);
    hipLaunchKernelGGL(ba_gram<kGramInit>, dim3(ngch), dim3(128), 0, s, d);
    hipLaunchKernelGGL(ba_frame_reduce<kGramInit>, dim3(nf), dim3(1024), 0, s, d);
    hipLaunchKernelGGL(ba_decide<kGramInit>, dim3(1), dim3(kDecideThreads), 0, s, d, (int)gpt128);
    SLAM_HIP(c, hipGetLastError());
    BA_T(3);

    // ---- LM iterations, queued in chunks; the host only polls for early exit ----
    if (!c->ev_sync) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
    constexpr int kIterChunk = 4;
    int queued = 0;
    bool pending = false;
    for (;;) {
        const int k = std::min(kIterChunk, max_iters - queued);
        for (int it = 0; it < k; it++) {
            hipLaunchKernelGGL(ba_schur_pts, dim3(npch), dim3(kSchurThreads), 0, s, d);
            hipLaunchKernelGGL(ba_blk_reduce, dim3(nb2), dim3(1024), 0, s, (const BaState*)d.st, 1,
                               (const double*)d.spart, dbs, d.blkS);
            camera_solve();
            hipLaunchKernelGGL(ba_update, dim3(gupd), dim3(kUpdThreads), 0, s, d);
            hipLaunchKernelGGL(ba_frame_reduce<kGramStep>, dim3(nf), dim3(1024), 0, s, d);
            hipLaunchKernelGGL(ba_decide<kGramStep>, dim3(1), dim3(kDecideThreads), 0, s, d, (int)gupd);
        }
        SLAM_HIP(c, hipGetLastError());
        queued += k;
        if (queued >= max_iters) break;
        // the previous chunk's state (polled without blocking the queue): the
        // chunk just queued runs while the host waits
        if (pending) {
            for (;;) {
                const hipError_t e = hipEventQuery(c->ev_sync);
                if (e == hipSuccess) break;
                if (e != hipErrorNotReady) return set_err(c, SLAM_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
            }
            if (hst->done) break;
        }
        SLAM_HIP(c, hipMemcpyAsync(hst, d.st, sizeof(BaState), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipEventRecord(c->ev_sync, s));
        pending = true;
    }
    // the solution in the caller's order and the final state: one sync
    hipLaunchKernelGGL(ba_export, dim3((std::max(np, 4 + 6 * nf) + 127) / 128), dim3(128), 0, s, d, dpor, dxout);
    SLAM_HIP(c, hipGetLastError());
    SLAM_HIP(c, hipMemcpyAsync(hst + 1, d.st, sizeof(BaState), hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(hx, dxout, 8 * (size_t)NX, hipMemcpyDeviceToHost, s));
    {
        int rc = stream_sync(c, s, true);
        if (rc) return rc;
    }
    BA_T(4);
    const BaState& fs = hst[1];
    sum->initial_cost = fs.initial_cost;
    sum->final_cost = fs.cost;
    sum->iterations = fs.iter;
    sum->successful_steps = fs.successful;
    sum->termination = fs.termination;
    sum->usable = fs.usable;
    std::memcpy(K4, hx, 32);
    std::memcpy(ext6 + 6, hx + 4 + 6, sizeof(double) * 6 * (nf - 1));
    std::memcpy(pts3, hx + 4 + 6 * nf, sizeof(double) * 3 * np);
#ifdef BA_DIAG
    {
        static long long h[2][16384][4];
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dt), sizeof(h));
        const int nwg[2] = {npch, npch};
        for (int k = 0; k < 2; k++) {
            long long t0 = h[k][0][0], tend = 0;
            double ph[3] = {0, 0, 0}, phmax[3] = {0, 0, 0};
            const int last = k == 0 ? 2 : 3;
            for (int w = 0; w < nwg[k]; w++) { t0 = std::min(t0, h[k][w][0]); tend = std::max(tend, h[k][w][last]); }
            double skew = 0;
            for (int w = 0; w < nwg[k]; w++) {
                skew = std::max(skew, (double)(h[k][w][0] - t0));
                for (int i = 0; i < last; i++) {
                    const double v = (double)(h[k][w][i + 1] - h[k][w][i]);
                    ph[i] += v / nwg[k];
                    phmax[i] = std::max(phmax[i], v);
                }
            }
            fprintf(stderr, "ba_diag %s wgs %d span_us %.2f start_skew_us %.2f phase_avg_us %.2f %.2f %.2f phase_max_us %.2f %.2f %.2f\n",
                    k ? "update" : "schur", nwg[k], (tend - t0) / 100.0, skew / 100.0, ph[0] / 100.0, ph[1] / 100.0,
                    ph[2] / 100.0, phmax[0] / 100.0, phmax[1] / 100.0, phmax[2] / 100.0);
            if (k == 0) {
                double byn[8] = {0}; int cn[8] = {0};
                for (int w = 0; w < nwg[k]; w++) { int nn = (int)h[k][w][3]; if (nn < 8) { byn[nn] += (h[k][w][2] - h[k][w][0]) / 100.0; cn[nn]++; } }
                for (int nn = 0; nn < 8; nn++) if (cn[nn]) fprintf(stderr, "   schur n=%d wgs %d avg_total_us %.2f\n", nn, cn[nn], byn[nn] / cn[nn]);
            }
        }
    }
#endif
#ifdef BA_HOST_TIMING
    BA_T(5);
    auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(ht[b] - ht[a]).count(); };
    fprintf(stderr, "ba_host_us bookkeeping %.1f (csr %.1f group %.1f renumber %.1f frames %.1f parts %.1f) uploads %.1f init_queue %.1f loop %.1f readback %.1f total %.1f\n",
            us(0, 1), us(0, 6), us(6, 7), us(7, 8), us(8, 9), us(9, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(0, 5));
#endif
    return SLAM_OK;
}

}  // namespace slamhip
