// Two-view linear triangulation on gfx950 (FP64), replacing the reference's
// reconstruct() (src/mainModule/triangulation/triangulate.cpp:74-100) and its
// reconstructPointsFor3D (:17-55): per matched point the 4 x 4 DLT system
// A = [x P(2) - P(0); y P(2) - P(1)] of both views, cv::SVD::compute(A) -- the
// one-sided Jacobi SVD of OpenCV's lapack.cpp (JacobiSVDImpl_<double> on A',
// eps = 10 DBL_EPSILON, descending sort) -- and X = Vt(3, 0..2) / Vt(3, 3)
// (convertHomogeneousPointsMatrixToSpatialPointsVector, :102-119).
//
// One thread per point: the whole 4 x 4 problem (A', Vt, W: 36 doubles) lives
// in registers with fully unrolled sweeps, so the kernel is bound by the FP64
// pipe on ~2k flop per point (a few sweeps) -- at 10k points a few microseconds.
// The operation order is oracle/geom.c's (no contraction, restated hypot), so
// the points agree bit for bit.
#include <cfloat>
#include <cmath>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

__device__ inline double hypot_r(double x, double y)
{
    double a = fabs(x), b = fabs(y);
    if (a < b) { const double t = a; a = b; b = t; }
    if (a == 0.0) return 0.0;
    const double r = b / a;
    return a * sqrt(1.0 + r * r);
}

struct TriParams {
    double P1[12], P2[12];
    const float2* pts1;
    const float2* pts2;
    int n;
    double* out;       // n x 3
};

__global__ __launch_bounds__(128) void tri_dlt(TriParams p)
{
    const int q = blockIdx.x * 128 + threadIdx.x;
    if (q >= p.n) return;
    const float2 u1 = p.pts1[q], u2 = p.pts2[q];
    const double xs[2] = {(double)u1.x, (double)u2.x}, ys[2] = {(double)u1.y, (double)u2.y};
    double At[4][4], Vt[4][4], W[4];
#pragma unroll
    for (int v = 0; v < 2; v++) {
        const double* P = v == 0 ? p.P1 : p.P2;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            At[c][v * 2] = xs[v] * P[8 + c] - P[c];
            At[c][v * 2 + 1] = ys[v] * P[8 + c] - P[4 + c];
        }
    }
    const double eps = DBL_EPSILON * 10;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) sd += At[i][k] * At[i][k];
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < 4; k++) Vt[i][k] = i == k ? 1.0 : 0.0;
    }
    for (int iter = 0; iter < 30; iter++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = i + 1; j < 4; j++) {
                double a = W[i], pp = 0, b = W[j];
#pragma unroll
                for (int k = 0; k < 4; k++) pp += At[i][k] * At[j][k];
                if (fabs(pp) <= eps * sqrt(a * b)) continue;
                pp *= 2;
                const double beta = a - b, gamma = hypot_r(pp, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = pp / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = pp / (gamma * c * 2);
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double t0 = c * At[i][k] + s * At[j][k];
                    const double t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = t0;
                    At[j][k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double t0 = c * Vt[i][k] + s * Vt[j][k];
                    const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                    Vt[i][k] = t0;
                    Vt[j][k] = t1;
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) sd += At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
    // descending selection sort, as JacobiSVDImpl_ (swaps W and Vt rows); the
    // smallest singular value's row ends at index 3
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int j = i;
#pragma unroll
        for (int k = i + 1; k < 4; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double wi = W[i], wj = 0;
            double vi[4], vj[4];
#pragma unroll
            for (int k = 0; k < 4; k++) { vi[k] = Vt[i][k]; vj[k] = 0; }
#pragma unroll
            for (int r = i + 1; r < 4; r++)
                if (r == j) {
                    wj = W[r];
#pragma unroll
                    for (int k = 0; k < 4; k++) vj[k] = Vt[r][k];
                    W[r] = wi;
#pragma unroll
                    for (int k = 0; k < 4; k++) Vt[r][k] = vi[k];
                }
            W[i] = wj;
#pragma unroll
            for (int k = 0; k < 4; k++) Vt[i][k] = vj[k];
        }
    }
    const double inv = 1. / Vt[3][3];
    p.out[3 * q] = Vt[3][0] * inv;
    p.out[3 * q + 1] = Vt[3][1] * inv;
    p.out[3 * q + 2] = Vt[3][2] * inv;
}

// projection = calibration * hconcat(R, t), sums in k order (cv::Mat product)
void projection(const double* K, const double* R, const double* t, double* P)
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

}  // namespace

int triangulate(slam_ctx* c, const double* K, const double* R1, const double* t1, const double* R2,
                const double* t2, const float* pts1, const float* pts2, int n, double* out)
{
    hipStream_t s = c->stream;
    TriParams p;
    projection(K, R1, t1, p.P1);
    projection(K, R2, t2, p.P2);
    const size_t pb = (size_t)n * sizeof(float2), ob = (size_t)n * 3 * sizeof(double);
    SLAM_HIP(c, c->geom.ensure(2 * pb + ob + 256));
    char* base = c->geom.as<char>();
    float2* d1 = reinterpret_cast<float2*>(base);
    float2* d2 = reinterpret_cast<float2*>(base + pb);
    double* dout = reinterpret_cast<double*>(base + ((2 * pb + 255) & ~(size_t)255));
    SLAM_HIP(c, hipMemcpyAsync(d1, pts1, pb, hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemcpyAsync(d2, pts2, pb, hipMemcpyHostToDevice, s));
    p.pts1 = d1; p.pts2 = d2; p.n = n; p.out = dout;
    hipLaunchKernelGGL(tri_dlt, dim3((n + 127) / 128), dim3(128), 0, s, p);
    SLAM_HIP(c, hipGetLastError());
    SLAM_HIP(c, hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipStreamSynchronize(s));
    return SLAM_OK;
}

}  // namespace slamhip
