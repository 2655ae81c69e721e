/*
 * CPU ORACLE (test infrastructure only; see oracle.h).  PARITY UNPINNED.
 *
 * k = 2 brute-force matching + Lowe ratio test.
 * Reference: matchFeatures featureMatchingCPU.cpp:17-43 (DescriptorMatcher
 * BRUTEFORCE = L2, BRUTEFORCE_HAMMING; knnMatch(query = previous frame,
 * train = candidate, k = 2) at :40) and its CUDA twin featureMatchingCUDA.cpp:
 * 19-46 (BF L1 for SIFT_BF, BF L2 for SIFT_FLANN, Hamming for ORB);
 * getGoodMatches featureMatchingCommon.cpp:37-50.
 * Restates OpenCV 4.8 core batchDistance(K = 2): distances in f32 (L2 = sqrt of
 * the squared sum, Hamming/L1 as sums), per query an insertion into a 2-slot
 * sorted list with strict comparisons while scanning train rows in index order,
 * i.e. the two smallest (distance, trainIdx) pairs in lexicographic order.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>

static float dist_row(const void* q, const void* t, int dim, int norm)
{
    if (norm == ORC_NORM_HAMMING) {
        const uint8_t* a = (const uint8_t*)q;
        const uint8_t* b = (const uint8_t*)t;
        int s = 0;
        for (int k = 0; k < dim; k++) s += __builtin_popcount((unsigned)(a[k] ^ b[k]));
        return (float)s;
    }
    const float* a = (const float*)q;
    const float* b = (const float*)t;
    float s = 0.f;
    if (norm == ORC_NORM_L1) {
        for (int k = 0; k < dim; k++) s += fabsf(a[k] - b[k]);
        return s;
    }
    for (int k = 0; k < dim; k++) {
        float d = a[k] - b[k];
        s += d * d;
    }
    return sqrtf(s);
}

void orc_knn2(const void* q, int nq, const void* t, int nt, int dim, int norm, int* idx, float* dist)
{
    size_t rb = norm == ORC_NORM_HAMMING ? (size_t)dim : (size_t)dim * sizeof(float);
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < nq; i++) {
        const uint8_t* qi = (const uint8_t*)q + rb * i;
        float d0 = FLT_MAX, d1 = FLT_MAX;
        int i0 = -1, i1 = -1;
        for (int j = 0; j < nt; j++) {
            float d = dist_row(qi, (const uint8_t*)t + rb * j, dim, norm);
            if (d < d1) {
                if (d0 > d) { d1 = d0; i1 = i0; d0 = d; i0 = j; }
                else { d1 = d; i1 = j; }
            }
        }
        idx[2 * i] = i0; idx[2 * i + 1] = i1;
        dist[2 * i] = d0; dist[2 * i + 1] = d1;
    }
}

/* L2 k = 2 over u8 descriptors: what orc_knn2 computes for f32 descriptors that
 * hold integers 0..255 (every SIFT descriptor, A.3's saturate_cast<uchar>).  The
 * f32 sum of squares is then a sum of integers whose partial sums stay below
 * 128 * 255^2 < 2^24, so every f32 addition is exact in any order and equals
 * this integer sum; the distance is the same sqrtf of the same value, and the
 * scan / tie rule is orc_knn2's.  A faster checker for large parity cases only
 * (tests/oracle_ffi.knn2 routes integer-valued f32 L2 inputs here; the CPU
 * suite checks both paths against each other). */
void orc_knn2_l2_u8(const uint8_t* q, int nq, const uint8_t* t, int nt, int* idx, float* dist)
{
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < nq; i++) {
        const uint8_t* qi = q + (size_t)128 * i;
        float d0 = FLT_MAX, d1 = FLT_MAX;
        int i0 = -1, i1 = -1;
        for (int j = 0; j < nt; j++) {
            const uint8_t* tj = t + (size_t)128 * j;
            int s = 0;
            for (int k = 0; k < 128; k++) {
                const int d = (int)qi[k] - (int)tj[k];
                s += d * d;
            }
            const float d = sqrtf((float)s);
            if (d < d1) {
                if (d0 > d) { d1 = d0; i1 = i0; d0 = d; i0 = j; }
                else { d1 = d; i1 = j; }
            }
        }
        idx[2 * i] = i0; idx[2 * i + 1] = i1;
        dist[2 * i] = d0; dist[2 * i + 1] = d1;
    }
}

/* getGoodMatches: keep m[0] iff m[0].distance < knnMatcherDistance * m[1].distance
 * (float promoted to double, strict).  Queries with no neighbour are skipped
 * (allMatches[i].empty()); with a single train row the reference reads m[1] out
 * of bounds -- restated here as "rejected". */
int orc_ratio(const int* idx, const float* dist, int nq, double ratio, orc_match* out)
{
    int m = 0;
    for (int i = 0; i < nq; i++) {
        if (idx[2 * i] < 0 || idx[2 * i + 1] < 0) continue;
        if ((double)dist[2 * i] < ratio * (double)dist[2 * i + 1]) {
            out[m].queryIdx = i;
            out[m].trainIdx = idx[2 * i];
            out[m].imgIdx = 0;
            out[m].distance = dist[2 * i];
            m++;
        }
    }
    return m;
}
