/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * Windowed bundle adjustment as the reference sets it up in Ceres 2.2:
 * bundleAdjustment.cpp:73-129 --
 *   - parameter blocks: calibration {fx, fy, cx, cy} (:157-161, free, shared by
 *     every residual), one {angle-axis, t} block per window frame (:163-175,
 *     :84-85) with the first one constant (:86), one 3-vector per point;
 *   - residual ProjectionCostFunctor (:15-41): AngleAxisRotatePoint + t, pinhole
 *     without distortion, r = (fx x/z + cx - u, fy y/z + cy - v), AutoDiff
 *     <2, 4, 6, 3> (:43-45);
 *   - loss from getLossFunction (:131-151, priority Trivial > Huber > Cauchy >
 *     Arctan > Tukey > none), applied through Ceres's Corrector;
 *   - Solver::Options (:108-114): LEVENBERG_MARQUARDT trust region (Ceres
 *     defaults: 50 iterations, function_tolerance 1e-6, gradient_tolerance 1e-10,
 *     parameter_tolerance 1e-8, initial radius 1e4, max radius 1e16,
 *     min_relative_decrease 1e-3, Jacobi column scaling computed once from the
 *     initial Jacobian), SPARSE_SCHUR (points eliminated, reduced camera system
 *     factorised by Cholesky).
 * Jacobians use forward-mode jets with Ceres jet.h arithmetic (13 partials).
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NJ 13
typedef struct { double a; double v[NJ]; } jet;

static jet jconst(double a) { jet r; r.a = a; memset(r.v, 0, sizeof(r.v)); return r; }
static jet jvar(double a, int i) { jet r = jconst(a); r.v[i] = 1.0; return r; }
static jet jadd(jet x, jet y) { jet r; r.a = x.a + y.a; for (int i = 0; i < NJ; i++) r.v[i] = x.v[i] + y.v[i]; return r; }
static jet jsub(jet x, jet y) { jet r; r.a = x.a - y.a; for (int i = 0; i < NJ; i++) r.v[i] = x.v[i] - y.v[i]; return r; }
static jet jmul(jet x, jet y) { jet r; r.a = x.a * y.a; for (int i = 0; i < NJ; i++) r.v[i] = x.a * y.v[i] + x.v[i] * y.a; return r; }
static jet jdiv(jet f, jet g)
{
    double gi = 1.0 / g.a, fg = f.a * gi;
    jet r; r.a = fg;
    for (int i = 0; i < NJ; i++) r.v[i] = (f.v[i] - fg * g.v[i]) * gi;
    return r;
}
static jet jsqrt(jet f)
{
    double t = sqrt(f.a), tw = 1.0 / (2.0 * t);
    jet r; r.a = t;
    for (int i = 0; i < NJ; i++) r.v[i] = f.v[i] * tw;
    return r;
}
static jet jcos(jet f) { jet r; r.a = cos(f.a); double s = -sin(f.a); for (int i = 0; i < NJ; i++) r.v[i] = s * f.v[i]; return r; }
static jet jsin(jet f) { jet r; r.a = sin(f.a); double c = cos(f.a); for (int i = 0; i < NJ; i++) r.v[i] = c * f.v[i]; return r; }

/* ceres/rotation.h AngleAxisRotatePoint */
static void aa_rotate_jet(const jet aa[3], const jet pt[3], jet res[3])
{
    jet theta2 = jadd(jadd(jmul(aa[0], aa[0]), jmul(aa[1], aa[1])), jmul(aa[2], aa[2]));
    if (theta2.a > DBL_EPSILON) {
        jet theta = jsqrt(theta2);
        jet ct = jcos(theta), st = jsin(theta);
        jet ti = jdiv(jconst(1.0), theta);
        jet w[3] = {jmul(aa[0], ti), jmul(aa[1], ti), jmul(aa[2], ti)};
        jet wx[3] = {jsub(jmul(w[1], pt[2]), jmul(w[2], pt[1])),
                     jsub(jmul(w[2], pt[0]), jmul(w[0], pt[2])),
                     jsub(jmul(w[0], pt[1]), jmul(w[1], pt[0]))};
        jet tmp = jmul(jadd(jadd(jmul(w[0], pt[0]), jmul(w[1], pt[1])), jmul(w[2], pt[2])),
                       jsub(jconst(1.0), ct));
        for (int k = 0; k < 3; k++)
            res[k] = jadd(jadd(jmul(pt[k], ct), jmul(wx[k], st)), jmul(w[k], tmp));
    } else {
        jet wx[3] = {jsub(jmul(aa[1], pt[2]), jmul(aa[2], pt[1])),
                     jsub(jmul(aa[2], pt[0]), jmul(aa[0], pt[2])),
                     jsub(jmul(aa[0], pt[1]), jmul(aa[1], pt[0]))};
        for (int k = 0; k < 3; k++) res[k] = jadd(pt[k], wx[k]);
    }
}

void orc_aa_rotate(const double aa[3], const double p[3], double out[3])
{
    jet a[3] = {jconst(aa[0]), jconst(aa[1]), jconst(aa[2])};
    jet q[3] = {jconst(p[0]), jconst(p[1]), jconst(p[2])};
    jet r[3];
    aa_rotate_jet(a, q, r);
    for (int k = 0; k < 3; k++) out[k] = r[k].a;
}

/* ProjectionCostFunctor::operator() with jets: partials ordered
 * [calib 0..3][ext 4..9][point 10..12] */
static void project_jet(const double* K, const double* e, const double* X, const double* obs,
                        double r[2], double J[2][NJ])
{
    jet cal[4], ext[6], pt[3];
    for (int i = 0; i < 4; i++) cal[i] = jvar(K[i], i);
    for (int i = 0; i < 6; i++) ext[i] = jvar(e[i], 4 + i);
    for (int i = 0; i < 3; i++) pt[i] = jvar(X[i], 10 + i);
    jet p[3];
    aa_rotate_jet(ext, pt, p);
    p[0] = jadd(p[0], ext[3]);
    p[1] = jadd(p[1], ext[4]);
    p[2] = jadd(p[2], ext[5]);
    jet x2 = jdiv(p[0], p[2]), y2 = jdiv(p[1], p[2]);
    jet u = jadd(jmul(cal[0], x2), cal[2]);
    jet v = jadd(jmul(cal[1], y2), cal[3]);
    u = jsub(u, jconst(obs[0]));
    v = jsub(v, jconst(obs[1]));
    r[0] = u.a; r[1] = v.a;
    if (J) for (int i = 0; i < NJ; i++) { J[0][i] = u.v[i]; J[1][i] = v.v[i]; }
}

/* ceres/loss_function.cc, rho = [rho(s), rho'(s), rho''(s)] */
void orc_loss_eval(int loss, double a, double s, double rho[3])
{
    switch (loss) {
    case ORC_LOSS_HUBER: {
        double b = a * a;
        if (s > b) {
            double r = sqrt(s);
            rho[0] = 2.0 * a * r - b;
            rho[1] = fmax(DBL_MIN, a / r);
            rho[2] = -rho[1] / (2.0 * s);
        } else { rho[0] = s; rho[1] = 1.0; rho[2] = 0.0; }
        return;
    }
    case ORC_LOSS_CAUCHY: {
        double b = a * a, c = 1.0 / b;
        double sum = 1.0 + s * c, inv = 1.0 / sum;
        rho[0] = b * log(sum);
        rho[1] = fmax(DBL_MIN, inv);
        rho[2] = -c * (inv * inv);
        return;
    }
    case ORC_LOSS_ARCTAN: {
        double b = 1.0 / (a * a);
        double sum = 1 + s * s * b, inv = 1 / sum;
        rho[0] = a * atan2(s, a);
        rho[1] = fmax(DBL_MIN, inv);
        rho[2] = -2.0 * s * b * (inv * inv);
        return;
    }
    case ORC_LOSS_TUKEY: {
        double a2 = a * a;
        if (s <= a2) {
            double value = 1.0 - s / a2, vs = value * value;
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

/* residual_block.cc + corrector.cc: cost = 0.5 rho(|r|^2); Jacobian corrected with
 * the uncorrected residual, then the residual scaled. */
static double eval_obs(const double* K, const double* e, const double* X, const double* obs,
                       int loss, double a, double r[2], double J[2][NJ])
{
    project_jet(K, e, X, obs, r, J);
    double sq = r[0] * r[0] + r[1] * r[1];
    if (loss == ORC_LOSS_NONE) return 0.5 * sq;
    double rho[3];
    orc_loss_eval(loss, a, sq, rho);
    if (!J) return 0.5 * rho[0];
    double sqrt_rho1 = sqrt(rho[1]);
    double residual_scaling, alpha_sq_norm;
    if (sq == 0.0 || rho[2] <= 0.0) {
        residual_scaling = sqrt_rho1;
        alpha_sq_norm = 0.0;
    } else {
        double D = 1.0 + 2.0 * sq * rho[2] / rho[1];
        double alpha = 1.0 - sqrt(D);
        residual_scaling = sqrt_rho1 / (1 - alpha);
        alpha_sq_norm = alpha / sq;
    }
    if (alpha_sq_norm == 0.0) {
        for (int i = 0; i < NJ; i++) { J[0][i] *= sqrt_rho1; J[1][i] *= sqrt_rho1; }
    } else {
        for (int c = 0; c < NJ; c++) {
            double rtj = J[0][c] * r[0] + J[1][c] * r[1];
            J[0][c] = sqrt_rho1 * (J[0][c] - alpha_sq_norm * r[0] * rtj);
            J[1][c] = sqrt_rho1 * (J[1][c] - alpha_sq_norm * r[1] * rtj);
        }
    }
    r[0] *= residual_scaling;
    r[1] *= residual_scaling;
    return 0.5 * rho[0];
}

double orc_ba_cost(const double K4[4], const double* ext6, const double* pts3, int nobs,
                   const int* of, const int* op, const double* oxy, int loss, double a)
{
    double c = 0;
    for (int o = 0; o < nobs; o++) {
        double r[2];
        c += eval_obs(K4, ext6 + 6 * of[o], pts3 + 3 * op[o], oxy + 2 * o, loss, a, r, NULL);
    }
    return c;
}

/* dense Cholesky, lower; returns 0 on failure */
static int cholesky(double* A, int n)
{
    for (int j = 0; j < n; j++) {
        double s = A[j * n + j];
        for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
        if (!(s > 0.0) || !isfinite(s)) return 0;
        double d = sqrt(s);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double t = A[i * n + j];
            for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / d;
        }
    }
    return 1;
}

static void chol_solve(const double* L, int n, double* b)
{
    for (int i = 0; i < n; i++) {
        double t = b[i];
        for (int k = 0; k < i; k++) t -= L[i * n + k] * b[k];
        b[i] = t / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double t = b[i];
        for (int k = i + 1; k < n; k++) t -= L[k * n + i] * b[k];
        b[i] = t / L[i * n + i];
    }
}

/* (V + D) inverse for a 3x3 SPD block via LLT (InvertPSDMatrix, full rank) */
static int inv3(const double* M, double* Minv)
{
    double L[9];
    memcpy(L, M, sizeof(L));
    if (!cholesky(L, 3)) return 0;
    for (int c = 0; c < 3; c++) {
        double e[3] = {0, 0, 0};
        e[c] = 1;
        chol_solve(L, 3, e);
        for (int r = 0; r < 3; r++) Minv[r * 3 + c] = e[r];
    }
    return 1;
}

/* The reduced camera system's factorisation.  The reference's Solver::Options
 * (bundleAdjustment.cpp:108-114) pick SPARSE_SCHUR on EIGEN_SPARSE: Ceres 2.2
 * factorises S with Eigen's SimplicialLDLT (up-looking LDL', AMD ordering).  AMD
 * on S's nearly dense pattern cannot be restated without Eigen's source, so the
 * default here is a dense Cholesky LL' in natural order (ORC_BA_LLT); the
 * envelope checker (tests/ba_envelope.py) also samples SimplicialLDLT's own
 * arithmetic (ORC_BA_LDLT) under random symmetric orderings of the camera
 * columns, the variety the reference's factorisation spans.  Per calling thread. */
enum { ORC_BA_LLT = 0, ORC_BA_LDLT = 1, ORC_BA_GAUSS_FMA = 2 };
static __thread int g_solver;
static __thread const int* g_perm;
void orc_ba_set_solver(int kind, const int* perm) { g_solver = kind; g_perm = perm; }
/* The reduced camera matrix's accumulation order.  ORC_BA_SCHUR_CERES (default)
 * follows Ceres's SchurEliminator::Eliminate (schur_eliminator_impl.h, upstream):
 * S starts from the camera damping; then per point chunk, in chunk order, every
 * observation row adds its F'F (ChunkDiagonalBlockAndGradient ->
 * EBlockRowOuterProduct) and the chunk subtracts F'E (E'E)^-1 E'F
 * (ChunkOuterProduct).  ORC_BA_SCHUR_GRAM_FIRST is the round-1..4 order (the
 * whole camera Gram first, then every point's Schur term subtracted): S is a
 * small difference of large sums (born-once points cancel most of the camera
 * information), and this order's rounding moves the first LM step ~1e-9
 * relative from Ceres's order on the framesBatchSize-210 windows
 * (scripts/diag/ba_perk.py). */
enum { ORC_BA_SCHUR_CERES = 0, ORC_BA_SCHUR_GRAM_FIRST = 1 };
static __thread int g_assembly;
void orc_ba_set_assembly(int kind) { g_assembly = kind; }

/* Eigen SimplicialLDLT (SimplicialCholesky_impl.h, factorize_preordered, from
 * Davis's LDL) on a dense pattern: row k of L from the upper triangle's column
 * k (pattern in ascending order), y_r -= L_ri y_i, l_ki = y_i / d_i,
 * d_k -= l_ki y_i; a zero pivot fails.  Then x = L^-T D^-1 L^-1 b
 * (SparseTriangularSolver: column-oriented forward sweep, D^-1 applied as the
 * reciprocal times x, row-oriented back sweep). */
static int ldlt_solve(const double* A, int n, double* b)
{
    double* L = (double*)calloc((size_t)n * n, sizeof(double));
    double* D = (double*)malloc(sizeof(double) * n);
    double* y = (double*)calloc((size_t)n, sizeof(double));
    int ok = 1;
    for (int k = 0; k < n && ok; k++) {
        for (int i = 0; i <= k; i++) y[i] = A[i * n + k];
        double d = y[k];
        y[k] = 0.0;
        for (int i = 0; i < k; i++) {
            const double yi = y[i];
            y[i] = 0.0;
            const double lki = yi / D[i];
            for (int r = i + 1; r < k; r++) y[r] -= L[r * n + i] * yi;
            d -= lki * yi;
            L[k * n + i] = lki;
        }
        if (d == 0.0) ok = 0;
        D[k] = d;
    }
    if (ok) {
        for (int i = 0; i < n; i++) {
            const double t = b[i];
            if (t != 0.0)
                for (int r = i + 1; r < n; r++) b[r] -= t * L[r * n + i];
        }
        for (int i = 0; i < n; i++) b[i] = (1.0 / D[i]) * b[i];
        for (int i = n - 1; i >= 0; i--) {
            double t = b[i];
            for (int r = i + 1; r < n; r++) t -= L[r * n + i] * b[r];
            b[i] = t;
        }
    }
    free(L); free(D); free(y);
    return ok;
}

static int cholesky(double* A, int n);
static void chol_solve(const double* L, int n, double* b);

/* Diagnostics (ORC_BA_GAUSS_FMA): the arithmetic of the GPU's one-wave camera
 * solve (csrc/ba.hip ba_camera_solve_lane): symmetric Gaussian elimination on
 * the full rows, row i -= (a_ij / a_jj) row j with fused multiply-adds, then
 * the back substitution x_k = b_k / a_kk, b_i -= a_ik x_k (k descending). */
static int gauss_fma_solve(double* A, int n, double* b)
{
    for (int i = 0; i < n; i++)
        for (int k = 0; k < i; k++) A[i * n + k] = A[k * n + i];   /* mirrored lower triangle */
    for (int j = 0; j < n; j++) {
        const double ajj = A[j * n + j], bj = b[j];
        if (!(ajj > 0.0) || !isfinite(ajj)) return 0;
        for (int i = j + 1; i < n; i++) {
            const double t = A[i * n + j] / ajj;
            /* column j as the rows below hold it (the GPU broadcasts lane k's a_kj) */
            for (int k = j + 1; k < n; k++) A[i * n + k] = fma(-t, A[k * n + j], A[i * n + k]);
            b[i] = fma(-t, bj, b[i]);
        }
    }
    for (int k = n - 1; k >= 0; k--) {
        const double xk = b[k] / A[k * n + k];
        for (int i = 0; i < k; i++) b[i] = fma(-A[i * n + k], xk, b[i]);
        b[k] = xk;
    }
    return 1;
}

/* S y = rc (S overwritten), under the calling thread's solver and ordering */
static int solve_reduced(double* S, int nc, double* rc)
{
    double* A = S;
    double* b = rc;
    double *Ap = NULL, *bp = NULL;
    if (g_perm) {
        Ap = (double*)malloc(sizeof(double) * nc * nc);
        bp = (double*)malloc(sizeof(double) * nc);
        for (int i = 0; i < nc; i++) {
            bp[i] = rc[g_perm[i]];
            for (int j = 0; j < nc; j++) Ap[i * nc + j] = S[g_perm[i] * nc + g_perm[j]];
        }
        A = Ap; b = bp;
    }
    int ok;
    if (g_solver == ORC_BA_LDLT) ok = ldlt_solve(A, nc, b);
    else if (g_solver == ORC_BA_GAUSS_FMA) ok = gauss_fma_solve(A, nc, b);
    else {
        ok = cholesky(A, nc);
        if (ok) chol_solve(A, nc, b);
    }
    if (g_perm) {
        if (ok) for (int i = 0; i < nc; i++) rc[g_perm[i]] = bp[i];
        free(Ap); free(bp);
    }
    return ok;
}

typedef struct {
    int nf, np, no, nc, nparam;
    const int *of, *op;
    const double* oxy;
    int loss;
    double a;
    /* per observation corrected residuals and Jacobian rows */
    double *r, *J;
    /* CSR obs per point */
    int *pstart, *plist;
} ba_problem;

/* column index of a partial for obs o: calib 0..3, ext of frame f (f >= 1) at
 * 4 + 6 (f - 1), point p at nc + 3 p; -1 for the constant frame 0 */
static int col_of(const ba_problem* P, int o, int i)
{
    if (i < 4) return i;
    if (i < 10) return P->of[o] == 0 ? -1 : 4 + 6 * (P->of[o] - 1) + (i - 4);
    return P->nc + 3 * P->op[o] + (i - 10);
}

static double evaluate(ba_problem* P, const double* K, const double* E, const double* X, int jac)
{
    double cost = 0;
    for (int o = 0; o < P->no; o++) {
        double r[2], J[2][NJ];
        cost += eval_obs(K, E + 6 * P->of[o], X + 3 * P->op[o], P->oxy + 2 * o, P->loss, P->a, r,
                         jac ? J : NULL);
        if (jac) {
            P->r[2 * o] = r[0]; P->r[2 * o + 1] = r[1];
            memcpy(P->J + (size_t)o * 2 * NJ, J, sizeof(J));
        }
    }
    return cost;
}

static void unpack_x(const ba_problem* P, const double* x, double* K, double* E, double* X,
                     const double* E0)
{
    memcpy(K, x, 4 * sizeof(double));
    memcpy(E, E0, 6 * sizeof(double));
    memcpy(E + 6, x + 4, (size_t)6 * (P->nf - 1) * sizeof(double));
    memcpy(X, x + P->nc, (size_t)3 * P->np * sizeof(double));
}

/* diagnostics: the cost after each LM iteration (cost[k - 1] = the final cost a
 * run capped at k iterations reports), per calling thread */
static __thread double* g_trace;
static __thread int g_trace_cap;
void orc_ba_set_trace(double* cost, int cap) { g_trace = cost; g_trace_cap = cost ? cap : 0; }

int orc_ba(double K4[4], int nf, double* ext6, int np, double* pts3, int no,
           const int* of, const int* op, const double* oxy, int loss, double a,
           int max_iters, orc_ba_summary* sum)
{
    ba_problem P;
    memset(&P, 0, sizeof(P));
    P.nf = nf; P.np = np; P.no = no; P.of = of; P.op = op; P.oxy = oxy; P.loss = loss; P.a = a;
    P.nc = 4 + 6 * (nf - 1);
    P.nparam = P.nc + 3 * np;
    const int nc = P.nc, N = P.nparam;
    if (max_iters <= 0) max_iters = 50;
    P.r = (double*)calloc((size_t)2 * no, sizeof(double));
    P.J = (double*)calloc((size_t)2 * NJ * no, sizeof(double));
    P.pstart = (int*)calloc((size_t)np + 1, sizeof(int));
    P.plist = (int*)malloc(sizeof(int) * (size_t)(no > 0 ? no : 1));
    for (int o = 0; o < no; o++) P.pstart[op[o] + 1]++;
    for (int p = 0; p < np; p++) P.pstart[p + 1] += P.pstart[p];
    {
        int* fill = (int*)calloc((size_t)np, sizeof(int));
        for (int o = 0; o < no; o++) P.plist[P.pstart[op[o]] + fill[op[o]]++] = o;
        free(fill);
    }

    double* x = (double*)malloc(sizeof(double) * N);
    double* xc = (double*)malloc(sizeof(double) * N);
    double *K = (double*)malloc(sizeof(double) * 4), *E = (double*)malloc(sizeof(double) * 6 * nf),
           *X = (double*)malloc(sizeof(double) * 3 * (np > 0 ? np : 1));
    memcpy(x, K4, 4 * sizeof(double));
    memcpy(x + 4, ext6 + 6, (size_t)6 * (nf - 1) * sizeof(double));
    memcpy(x + nc, pts3, (size_t)3 * np * sizeof(double));
    const double* E0 = ext6;

    double* scale = (double*)malloc(sizeof(double) * N);
    double* g = (double*)malloc(sizeof(double) * N);      /* scaled gradient J_s' f */
    double* diag = (double*)malloc(sizeof(double) * N);
    double* step = (double*)malloc(sizeof(double) * N);
    double* S = (double*)malloc(sizeof(double) * nc * nc);
    double* Vinv = (double*)malloc(sizeof(double) * 9 * (np > 0 ? np : 1));
    double* V = (double*)malloc(sizeof(double) * 9 * (np > 0 ? np : 1));
    double* Wp = (double*)malloc(sizeof(double) * nc * 3);
    double* rc = (double*)malloc(sizeof(double) * nc);

    unpack_x(&P, x, K, E, X, E0);
    double cost = evaluate(&P, K, E, X, 1);
    sum->initial_cost = cost;
    sum->num_residuals = 2 * no;
    sum->iterations = 0;
    sum->successful_steps = 0;
    sum->termination = 0;
    sum->usable = 1;

    /* Jacobi scaling from the initial Jacobian: 1 / (1 + sqrt(|col|^2)) */
    for (int i = 0; i < N; i++) scale[i] = 0;
    for (int o = 0; o < no; o++) {
        const double* Jo = P.J + (size_t)o * 2 * NJ;
        for (int i = 0; i < NJ; i++) {
            int c = col_of(&P, o, i);
            if (c >= 0) scale[c] += Jo[i] * Jo[i] + Jo[NJ + i] * Jo[NJ + i];
        }
    }
    for (int i = 0; i < N; i++) scale[i] = 1.0 / (1.0 + sqrt(scale[i]));

    double radius = 1e4, decrease_factor = 2.0;
    const double min_diag = 1e-6, max_diag = 1e32;
    /* Ceres's x_norm covers the reduced program only (Program::RemoveFixedBlocks:
     * constant blocks and blocks no residual uses are dropped): calib, the
     * extrinsics of frames >= 1 with an observation, the observed points */
    unsigned char* used = (unsigned char*)calloc((size_t)N, 1);
    for (int i = 0; i < 4; i++) used[i] = 1;
    for (int o = 0; o < no; o++) {
        if (of[o] > 0) memset(used + 4 + 6 * (of[o] - 1), 1, 6);
        memset(used + nc + 3 * op[o], 1, 3);
    }
    double xnorm = 0;
    for (int i = 0; i < N; i++) if (used[i]) xnorm += x[i] * x[i];
    xnorm = sqrt(xnorm);
    int reuse_diag = 0, consecutive_invalid = 0, iter = 0;
    int have_jac = 1;
    double gmax;

    for (;;) {
        if (have_jac) {
            /* gradient (unscaled J'f) max norm check; scaled quantities for the solve */
            for (int i = 0; i < N; i++) g[i] = 0;
            for (int o = 0; o < no; o++) {
                const double* Jo = P.J + (size_t)o * 2 * NJ;
                for (int i = 0; i < NJ; i++) {
                    int c = col_of(&P, o, i);
                    if (c >= 0) g[c] += Jo[i] * P.r[2 * o] + Jo[NJ + i] * P.r[2 * o + 1];
                }
            }
            gmax = 0;
            for (int i = 0; i < N; i++) if (fabs(g[i]) > gmax) gmax = fabs(g[i]);
            for (int i = 0; i < N; i++) g[i] *= scale[i];
            have_jac = 0;
            if (gmax <= 1e-10) { sum->termination = 1; break; }
        }
        if (iter > 0 && iter <= g_trace_cap) g_trace[iter - 1] = cost;
        if (iter >= max_iters) { sum->termination = 0; break; }
        iter++;

        /* normal equations in the scaled space: H = J_s' J_s */
        memset(S, 0, sizeof(double) * nc * nc);
        memset(V, 0, sizeof(double) * 9 * np);
        if (!reuse_diag) for (int i = 0; i < N; i++) diag[i] = 0;
        for (int o = 0; o < no; o++) {
            const double* Jo = P.J + (size_t)o * 2 * NJ;
            double js[2][NJ];
            int cols[NJ];
            for (int i = 0; i < NJ; i++) {
                cols[i] = col_of(&P, o, i);
                double s = cols[i] >= 0 ? scale[cols[i]] : 0.0;
                js[0][i] = Jo[i] * s;
                js[1][i] = Jo[NJ + i] * s;
            }
            if (!reuse_diag)
                for (int i = 0; i < NJ; i++)
                    if (cols[i] >= 0) diag[cols[i]] += js[0][i] * js[0][i] + js[1][i] * js[1][i];
            /* camera-camera block */
            if (g_assembly == ORC_BA_SCHUR_GRAM_FIRST)
            for (int i = 0; i < 10; i++) {
                if (cols[i] < 0) continue;
                for (int j = 0; j < 10; j++) {
                    if (cols[j] < 0) continue;
                    S[cols[i] * nc + cols[j]] += js[0][i] * js[0][j] + js[1][i] * js[1][j];
                }
            }
            double* Vp = V + 9 * op[o];
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++)
                    Vp[i * 3 + j] += js[0][10 + i] * js[0][10 + j] + js[1][10 + i] * js[1][10 + j];
        }
        if (!reuse_diag)
            for (int i = 0; i < N; i++) diag[i] = fmin(fmax(diag[i], min_diag), max_diag);
        /* LM damping D^2 = diag / radius on every diagonal entry */
        for (int i = 0; i < nc; i++) S[i * nc + i] += diag[i] / radius;
        int ok = 1;
        for (int c = 0; c < nc; c++) rc[c] = g[c];
        for (int p = 0; p < np && ok; p++) {
            double Vd[9];
            memcpy(Vd, V + 9 * p, sizeof(Vd));
            for (int k = 0; k < 3; k++) Vd[k * 4] += diag[nc + 3 * p + k] / radius;
            double* Vi = Vinv + 9 * p;
            if (!inv3(Vd, Vi)) { ok = 0; break; }
            /* W_p (nc x 3) = sum over obs of point p of J_c' J_p (scaled) */
            int o0 = P.pstart[p], o1 = P.pstart[p + 1];
            /* touched camera columns: calib + frames of these obs */
            memset(Wp, 0, sizeof(double) * nc * 3);
            for (int q = o0; q < o1; q++) {
                int o = P.plist[q];
                const double* Jo = P.J + (size_t)o * 2 * NJ;
                double js[2][NJ];
                for (int i = 0; i < NJ; i++) {
                    int c = col_of(&P, o, i);
                    double s = c >= 0 ? scale[c] : 0.0;
                    js[0][i] = Jo[i] * s;
                    js[1][i] = Jo[NJ + i] * s;
                }
                for (int i = 0; i < 10; i++) {
                    int c = col_of(&P, o, i);
                    if (c < 0) continue;
                    for (int k = 0; k < 3; k++)
                        Wp[c * 3 + k] += js[0][i] * js[0][10 + k] + js[1][i] * js[1][10 + k];
                    if (g_assembly == ORC_BA_SCHUR_CERES)     /* this row's F'F */
                        for (int j = 0; j < 10; j++) {
                            int cj = col_of(&P, o, j);
                            if (cj >= 0) S[c * nc + cj] += js[0][i] * js[0][j] + js[1][i] * js[1][j];
                        }
                }
            }
            double WV[3];
            const double* gp = g + nc + 3 * p;
            for (int i = 0; i < nc; i++) {
                const double* wi = Wp + i * 3;
                if (wi[0] == 0 && wi[1] == 0 && wi[2] == 0) continue;
                for (int k = 0; k < 3; k++) WV[k] = wi[0] * Vi[k] + wi[1] * Vi[3 + k] + wi[2] * Vi[6 + k];
                rc[i] -= WV[0] * gp[0] + WV[1] * gp[1] + WV[2] * gp[2];
                for (int j = 0; j < nc; j++) {
                    const double* wj = Wp + j * 3;
                    S[i * nc + j] -= WV[0] * wj[0] + WV[1] * wj[1] + WV[2] * wj[2];
                }
            }
        }
        reuse_diag = 0;
        if (ok) ok = solve_reduced(S, nc, rc);
        if (ok) {
            for (int i = 0; i < nc; i++) step[i] = rc[i];
            /* back substitution: y_p = Vinv (g_p - W_p' y_c) */
            for (int p = 0; p < np; p++) {
                int o0 = P.pstart[p], o1 = P.pstart[p + 1];
                double t[3] = {g[nc + 3 * p], g[nc + 3 * p + 1], g[nc + 3 * p + 2]};
                for (int q = o0; q < o1; q++) {
                    int o = P.plist[q];
                    const double* Jo = P.J + (size_t)o * 2 * NJ;
                    double jc_y[2] = {0, 0};
                    for (int i = 0; i < 10; i++) {
                        int c = col_of(&P, o, i);
                        if (c < 0) continue;
                        jc_y[0] += Jo[i] * scale[c] * step[c];
                        jc_y[1] += Jo[NJ + i] * scale[c] * step[c];
                    }
                    for (int k = 0; k < 3; k++) {
                        double s = scale[nc + 3 * p + k];
                        t[k] -= Jo[10 + k] * s * jc_y[0] + Jo[NJ + 10 + k] * s * jc_y[1];
                    }
                }
                const double* Vi = Vinv + 9 * p;
                for (int k = 0; k < 3; k++) step[nc + 3 * p + k] = Vi[3 * k] * t[0] + Vi[3 * k + 1] * t[1] + Vi[3 * k + 2] * t[2];
            }
            for (int i = 0; i < N; i++) {
                if (!isfinite(step[i])) { ok = 0; break; }
                step[i] = -step[i];
            }
        }
        int valid = 0;
        double mcc = 0;
        if (ok) {
            reuse_diag = 1;
            /* model cost change = -(J_s step) . (f + J_s step / 2) */
            for (int o = 0; o < no; o++) {
                const double* Jo = P.J + (size_t)o * 2 * NJ;
                double mr[2] = {0, 0};
                for (int i = 0; i < NJ; i++) {
                    int c = col_of(&P, o, i);
                    if (c < 0) continue;
                    double s = scale[c] * step[c];
                    mr[0] += Jo[i] * s;
                    mr[1] += Jo[NJ + i] * s;
                }
                mcc -= mr[0] * (P.r[2 * o] + mr[0] / 2.0) + mr[1] * (P.r[2 * o + 1] + mr[1] / 2.0);
            }
            valid = mcc > 0.0;
        }
        if (!valid) {
            if (++consecutive_invalid >= 5) { sum->termination = 3; sum->usable = 0; break; }
            radius /= decrease_factor;
            decrease_factor *= 2.0;
            reuse_diag = ok ? 1 : reuse_diag;
            if (radius <= 1e-32) { sum->termination = 2; break; }
            continue;
        }
        consecutive_invalid = 0;
        for (int i = 0; i < N; i++) xc[i] = x[i] + step[i] * scale[i];
        double snorm = 0;
        for (int i = 0; i < N; i++) snorm += (xc[i] - x[i]) * (xc[i] - x[i]);
        snorm = sqrt(snorm);
        unpack_x(&P, xc, K, E, X, E0);
        double cand = evaluate(&P, K, E, X, 0);
        if (!isfinite(cand)) cand = DBL_MAX;
        if (snorm <= 1e-8 * (xnorm + 1e-8)) { sum->termination = 1; break; }
        double cost_change = cost - cand;
        if (fabs(cost_change) <= 1e-6 * cost) { sum->termination = 1; break; }
        double rel = (cost - cand) / mcc;
        if (rel > 1e-3) {
            memcpy(x, xc, sizeof(double) * N);
            xnorm = 0;
            for (int i = 0; i < N; i++) if (used[i]) xnorm += x[i] * x[i];
            xnorm = sqrt(xnorm);
            cost = evaluate(&P, K, E, X, 1);
            have_jac = 1;
            double q = 2.0 * rel - 1.0;
            radius = radius / fmax(1.0 / 3.0, 1.0 - q * q * q);
            radius = fmin(1e16, radius);
            decrease_factor = 2.0;
            reuse_diag = 0;
            sum->successful_steps++;
        } else {
            radius /= decrease_factor;
            decrease_factor *= 2.0;
            reuse_diag = 1;
            if (radius <= 1e-32) { sum->termination = 2; break; }
        }
    }
    for (int k = iter > 0 ? iter - 1 : 0; k < g_trace_cap; k++) g_trace[k] = cost;
    sum->iterations = iter;
    sum->final_cost = cost;
    memcpy(K4, x, 4 * sizeof(double));
    memcpy(ext6 + 6, x + 4, (size_t)6 * (nf - 1) * sizeof(double));
    memcpy(pts3, x + nc, (size_t)3 * np * sizeof(double));
    free(used);
    free(x); free(xc); free(K); free(E); free(X); free(scale); free(g); free(diag); free(step);
    free(S); free(Vinv); free(V); free(Wp); free(rc);
    free(P.r); free(P.J); free(P.pstart); free(P.plist);
    return 0;
}
