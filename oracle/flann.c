/*
 * CPU ORACLE (test infrastructure only; see oracle.h).
 *
 * Randomized KD-forest approximate 2-NN, restating the index the reference's
 * useFM-SIFT-FLANN CPU path builds per call: DescriptorMatcher::create(FLANNBASED)
 * (featureMatchingCPU.cpp:30-31) -> FlannBasedMatcher with the OpenCV defaults
 * KDTreeIndexParams(trees = 4) and SearchParams(checks = 32); the index is built
 * on the TRAIN descriptors (the candidate frame) on every knnMatch call (:40).
 * FLANN 1.x KDTreeIndex: split dimension drawn from the 5 highest-variance
 * dimensions of a 100-point sample, split value = sample mean, single-point
 * leaves; search descends every tree, queues the other branches by squared
 * plane distance and stops after `checks` leaf points.
 *
 * Approximate and randomized: NOT a parity target (the reference's own CUDA
 * build replaces it by exact BF-L2, featureMatchingCUDA.cpp:30-31).  It exists
 * only so bench.py's cpu_baseline times the reference's CPU matcher choice.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int c1, c2, feat; float val; } kd_node;
typedef struct { kd_node* nodes; int n; } kd_tree;

static uint64_t rng_next(uint64_t* s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int build(kd_tree* tr, const float* data, int dim, int* ind, int count, uint64_t* rng)
{
    int id = tr->n++;
    kd_node* nd = &tr->nodes[id];
    if (count == 1) { nd->c1 = nd->c2 = -1; nd->feat = ind[0]; nd->val = 0; return id; }
    double mean[256], var[256];
    int cnt = count < 100 ? count : 100;
    for (int k = 0; k < dim; k++) mean[k] = var[k] = 0;
    for (int i = 0; i < cnt; i++) {
        const float* p = data + (size_t)ind[i] * dim;
        for (int k = 0; k < dim; k++) mean[k] += p[k];
    }
    for (int k = 0; k < dim; k++) mean[k] /= cnt;
    for (int i = 0; i < cnt; i++) {
        const float* p = data + (size_t)ind[i] * dim;
        for (int k = 0; k < dim; k++) { double d = p[k] - mean[k]; var[k] += d * d; }
    }
    int top[5], ntop = 0;
    for (int k = 0; k < dim; k++) {
        if (ntop < 5 || var[k] > var[top[ntop - 1]]) {
            int j = ntop < 5 ? ntop++ : 4;
            while (j > 0 && var[k] > var[top[j - 1]]) { top[j] = top[j - 1]; j--; }
            top[j] = k;
        }
    }
    int feat = top[rng_next(rng) % (uint64_t)ntop];
    float val = (float)mean[feat];
    int lo = 0, hi = count - 1;
    while (lo <= hi) {
        if (data[(size_t)ind[lo] * dim + feat] < val) lo++;
        else { int t = ind[lo]; ind[lo] = ind[hi]; ind[hi] = t; hi--; }
    }
    if (lo == 0 || lo == count) lo = count / 2;
    nd->feat = feat; nd->val = val;
    int c1 = build(tr, data, dim, ind, lo, rng);
    int c2 = build(tr, data, dim, ind + lo, count - lo, rng);
    tr->nodes[id].c1 = c1; tr->nodes[id].c2 = c2;
    return id;
}

typedef struct { float d; int tree, node; } branch;
typedef struct { branch* a; int n, cap; } heap_t;

static void heap_push(heap_t* h, branch b)
{
    if (h->n == h->cap) { h->cap = h->cap ? 2 * h->cap : 256; h->a = (branch*)realloc(h->a, sizeof(branch) * h->cap); }
    int i = h->n++;
    while (i > 0) {
        int p = (i - 1) / 2;
        if (h->a[p].d <= b.d) break;
        h->a[i] = h->a[p]; i = p;
    }
    h->a[i] = b;
}

static int heap_pop(heap_t* h, branch* out)
{
    if (h->n == 0) return 0;
    *out = h->a[0];
    branch last = h->a[--h->n];
    int i = 0;
    for (;;) {
        int c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && h->a[c + 1].d < h->a[c].d) c++;
        if (h->a[c].d >= last.d) break;
        h->a[i] = h->a[c]; i = c;
    }
    if (h->n) h->a[i] = last;
    return 1;
}

typedef struct { float d0, d1; int i0, i1; int checks; } res2;

static void add_point(res2* r, float d, int idx)
{
    if (d < r->d1) {
        if (d < r->d0) { r->d1 = r->d0; r->i1 = r->i0; r->d0 = d; r->i0 = idx; }
        else { r->d1 = d; r->i1 = idx; }
    }
}

static void search_level(const kd_tree* trees, int ti, int node, float mindist, const float* q,
                         const float* data, int dim, int max_checks, res2* r, heap_t* h,
                         int* mark, int gen)
{
    const kd_node* nodes = trees[ti].nodes;
    for (;;) {
        const kd_node* nd = &nodes[node];
        if (nd->c1 < 0) {
            int idx = nd->feat;
            if (mark[idx] == gen) return;
            if (r->checks >= max_checks && r->i1 >= 0) return;
            mark[idx] = gen;
            r->checks++;
            const float* p = data + (size_t)idx * dim;
            float s = 0.f;
            for (int k = 0; k < dim; k++) { float d = q[k] - p[k]; s += d * d; }
            add_point(r, s, idx);
            return;
        }
        float diff = q[nd->feat] - nd->val;
        int best = diff < 0 ? nd->c1 : nd->c2;
        int other = diff < 0 ? nd->c2 : nd->c1;
        float nd2 = mindist + diff * diff;
        if (nd2 < r->d1 || r->i1 < 0) { branch b = {nd2, ti, other}; heap_push(h, b); }
        node = best;
    }
}

void orc_flann_knn2(const float* q, int nq, const float* t, int nt, int dim, int ntrees,
                    int checks, uint64_t seed, int* idx, float* dist)
{
    if (nt <= 0 || dim > 256) {
        for (int i = 0; i < 2 * nq; i++) { idx[i] = -1; dist[i] = FLT_MAX; }
        return;
    }
    kd_tree* trees = (kd_tree*)calloc((size_t)ntrees, sizeof(kd_tree));
    int* ind = (int*)malloc(sizeof(int) * (size_t)nt);
    uint64_t rng = seed;
    for (int ti = 0; ti < ntrees; ti++) {
        for (int i = 0; i < nt; i++) ind[i] = i;
        for (int i = nt - 1; i > 0; i--) {
            int j = (int)(rng_next(&rng) % (uint64_t)(i + 1));
            int tmp = ind[i]; ind[i] = ind[j]; ind[j] = tmp;
        }
        trees[ti].nodes = (kd_node*)malloc(sizeof(kd_node) * (size_t)(2 * nt));
        trees[ti].n = 0;
        build(&trees[ti], t, dim, ind, nt, &rng);
    }
    free(ind);
#pragma omp parallel
    {
        heap_t h = {0, 0, 0};
        int* mark = (int*)calloc((size_t)nt, sizeof(int));
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < nq; i++) {
            const float* qi = q + (size_t)i * dim;
            res2 r = {FLT_MAX, FLT_MAX, -1, -1, 0};
            h.n = 0;
            for (int ti = 0; ti < ntrees; ti++)
                search_level(trees, ti, 0, 0.f, qi, t, dim, checks, &r, &h, mark, i + 1);
            branch b;
            while ((r.checks < checks || r.i1 < 0) && heap_pop(&h, &b))
                search_level(trees, b.tree, b.node, b.d, qi, t, dim, checks, &r, &h, mark, i + 1);
            idx[2 * i] = r.i0; idx[2 * i + 1] = r.i1;
            dist[2 * i] = r.i0 >= 0 ? sqrtf(r.d0) : FLT_MAX;
            dist[2 * i + 1] = r.i1 >= 0 ? sqrtf(r.d1) : FLT_MAX;
        }
        free(mark);
        free(h.a);
    }
    for (int ti = 0; ti < ntrees; ti++) free(trees[ti].nodes);
    free(trees);
}
