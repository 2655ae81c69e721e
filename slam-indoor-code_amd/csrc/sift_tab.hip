// SIFT descriptors, gather formulation (keypoints sharing one angle and size).
//
// calcSIFTDescriptor (reference path: extractDescriptor -> cv::SIFT::compute,
// featureMatchingCPU.cpp:51-65) scatters every window sample into 8 histogram
// bins.  For FAST keypoints all angles are -1 deg and all sizes 7 px, so the
// sample geometry -- rotated bin coordinates, trilinear split, exp32f Gaussian
// weight -- is one fixed table per launch.  The table is reorganised per TARGET
// histogram cell: for each of the 20 cells that reach the descriptor (16 inner
// cells + the 4 column-5 cells whose o0 = -1 weight lands in column 4, see the
// 361-degree quirk in oracle/sift.c) it lists, in the reference's raster
// sample order, the samples that contribute and which corner of their 2 x 2
// cell footprint the target is.
//
// One lane owns one target cell (20 lanes per keypoint, 3 keypoints per
// one-wave workgroup) and accumulates into lane-private LDS slots, so every bin
// receives its contributions in exactly the reference's order and the
// descriptors are bit-identical to the oracle.  Slot layout per lane:
// position 0 = slot 9 of the cell to the left (the o0 = -1 quirk), positions
// 1..9 = slots 0..8, so a sample always adds v0 at o0 + 1 and v1 at o0 + 2
// (one ds_read2 / ds_write2 pair 64 dwords apart, no branch).  Positions are
// slot-major (p * 64 + lane): every lane stays in its own LDS bank whatever
// p is, so the read-modify-write is bank-conflict free (lane * 11 + p had
// conflicts on 63 % of the LDS-active cycles).  Padding entries carry weight 0:
// adding +0 to a non-negative partial sum is exact.
//
// Data movement: the geometry table lives in LDS for the whole launch (one
// persistent 8-wave workgroup per CU): 16-B per-sample records {rf, cf, w,
// (i, j)} shared by the 4 targets a sample reaches, and per-target u16 entries
// (record index << 2 | dc << 1 | dr) read four at a time.  Only the {mag, ori}
// sample itself comes from global memory (one 8-B gather per entry, issued a
// batch ahead); the previous per-lane 16-B table loads saturated the vector
// memory return path (measured: table + gather 3.7 of 6.1 ms).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

namespace {

constexpr int kTargets = 20;            // lanes per keypoint
constexpr int kKpPerWave = 3;
constexpr int kSlotStride = 64;         // slot-major: position p of lane L at p * 64 + L (bank L for every p)
constexpr int kWavesDefault = 12;       // waves per workgroup (independent keypoint triples)
constexpr int kMaxRec = 2816;           // sample records (size 7: 2761 + 2 zero records)
constexpr int kMaxRows2 = 256;          // item rows of 2, both parity tables (size 7: 2 x ~128)

struct TabParams {
    const float2* grad;
    int w, h, pitch;    // pitch: grad_pitch(w), the padded map's row stride
    const slam_keypoint* kps;
    const int* kp_frame;
    const int* total;
    int cap;
    const float4* rec;                  // [nrec] {rf, cf, w, (i & 255) | (j & 255) << 8}
    const uint2* ent;                   // [2 parities][rows2 + 2][kTargets], 2 u32 items each
    int nrec, rows2;                    // rows2 = item rows walked (the table holds 2 more)
    SiftTabMeta meta;
    uint8_t* desc_u8;
    float* desc_f32;
    int* norm_i8;
};

__device__ __forceinline__ void wave_sync()
{
    // lanes of one wave exchange data through LDS: LDS executes a wave's
    // accesses in order, so only compiler reordering has to be prevented
    __builtin_amdgcn_wave_barrier();
    __asm__ volatile("" ::: "memory");
}

template <bool kCheck>
__device__ __forceinline__ void tab_walk(const TabParams& p, const float4* rec, const uint2* E, const float2* P,
                                         int ptx, int pty, float* my)
{
    const float bins_per_rad = 8 / 360.f;
    const float ori_deg = p.meta.ori_deg;
    const int w = p.w, h = p.h;
    // one gather fetches the item's two horizontally adjacent samples (i, j), (i, j + 1)
    auto gather2 = [&](const float4& r) -> float4 {
        const int ij = __float_as_int(r.w);
        const int i = (int)(int8_t)(ij & 0xff), j = (int)(int8_t)((ij >> 8) & 0xff);
        const int off = i * p.pitch + j;
        if (kCheck) {
            const int rr = pty + i, cc = ptx + j;
            const bool rin = (unsigned)(rr - 1) < (unsigned)(h - 2);
            const bool in0 = rin && (unsigned)(cc - 1) < (unsigned)(w - 2);
            const bool in1 = rin && (unsigned)(cc) < (unsigned)(w - 2);
            float2 a = P[in0 ? off : 0], b = P[in1 ? off + 1 : 0];
            if (!in0) a.x = 0.f;           // sample outside the image: contributes +0
            if (!in1) b.x = 0.f;
            return make_float4(a.x, a.y, b.x, b.y);
        }
        return *reinterpret_cast<const float4*>(P + off);
    };
    uint2 e0 = E[0], e1 = E[kTargets], e2;
    float4 rc[4], rn[4];
    float4 gc[2], gn[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint32_t code = u ? e0.y : e0.x;
        rc[2 * u] = rec[code & 0x3fffu];
        rc[2 * u + 1] = rec[(code & 0x3fffu) + 1];
    }
#pragma unroll
    for (int u = 0; u < 2; u++) gc[u] = gather2(rc[2 * u]);
    const int rows = p.rows2;
    for (int m = 0; m < rows; m++) {
        e2 = E[(m + 2) * kTargets];                          // table holds 2 prefetch rows
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t code = u ? e1.y : e1.x;
            rn[2 * u] = rec[code & 0x3fffu];
            rn[2 * u + 1] = rec[(code & 0x3fffu) + 1];
        }
#pragma unroll
        for (int u = 0; u < 2; u++) gn[u] = gather2(rn[2 * u]);
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t code = u ? e0.y : e0.x;
#pragma unroll
            for (int sm = 0; sm < 2; sm++) {
                const float4 r = rc[2 * u + sm];
                const float mo_m = sm ? gc[u].z : gc[u].x;
                const float mo_o = sm ? gc[u].w : gc[u].y;
                const uint32_t fl = code >> (14 + 2 * sm);   // bit 0 dr, bit 1 dc
                float obin = __fmul_rn(__fsub_rn(mo_o, ori_deg), bins_per_rad);
                float mag = __fmul_rn(mo_m, r.z);
                if (sm == 1 && !(code & (1u << 18))) mag = 0.f;   // single-sample item: +0
                int o0 = (int)floorf(obin);
                obin = __fsub_rn(obin, (float)o0);
                o0 += o0 < 0 ? 8 : 0;
                o0 -= o0 >= 8 ? 8 : 0;
                const float v_r1 = __fmul_rn(mag, r.x);
                const float br = (fl & 1u) ? v_r1 : __fsub_rn(mag, v_r1);
                const float v_c1 = __fmul_rn(br, r.y);
                const float v = (fl & 2u) ? v_c1 : __fsub_rn(br, v_c1);
                const float v1 = __fmul_rn(v, obin);
                const float v0 = __fsub_rn(v, v1);
                float* sp = my + (o0 + 1) * kSlotStride;
                const float a0 = sp[0], a1 = sp[kSlotStride];
                sp[0] = __fadd_rn(a0, v0);
                sp[kSlotStride] = __fadd_rn(a1, v1);
            }
        }
        e0 = e1;
        e1 = e2;
#pragma unroll
        for (int u = 0; u < 4; u++) rc[u] = rn[u];
#pragma unroll
        for (int u = 0; u < 2; u++) gc[u] = gn[u];
    }
}

template <int kWaves>
__global__ __launch_bounds__(64 * kWaves) void sift_desc_tab(TabParams p)
{
    __shared__ float4 rec[kMaxRec];
    __shared__ uint2 ent[kMaxRows2 * kTargets];
    __shared__ float slots[kWaves][10 * kSlotStride];
    __shared__ float raw[kWaves][kKpPerWave][128];
    __shared__ float scal[kWaves][kKpPerWave];
    __shared__ float part[kWaves][kKpPerWave][8];
    __shared__ int nrm[kWaves][kKpPerWave][kTargets];

    for (int k = threadIdx.x; k < p.nrec; k += blockDim.x) rec[k] = p.rec[k];
    for (int k = threadIdx.x; k < 2 * (p.rows2 + 2) * kTargets; k += blockDim.x) ent[k] = p.ent[k];
    __syncthreads();   // the only workgroup barrier: waves below run independent triples

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ks = lane / kTargets, t = lane - ks * kTargets;   // keypoint slot (3 = idle lanes), target cell
    int total = *p.total;
    if (total > p.cap) total = p.cap;
    float* sl = slots[wave];
    float* my = &sl[lane];
    const int R = 1 + t / 5, C = 1 + t % 5;                     // target cell (R, C), C = 5: quirk only
    const int rad = p.meta.radius;

    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so the
    // keypoint triples are split into 8 contiguous ranges, one per XCD group
    // (blockIdx % 8); each XCD walks a compact raster band of keypoints whose
    // gradient windows overlap, and its L2 serves the re-reads.
    const int ntri = (total + kKpPerWave - 1) / kKpPerWave;
    const int xg = blockIdx.x & 7;
    const int nw = (gridDim.x >> 3) * kWaves, wi = (blockIdx.x >> 3) * kWaves + wave;
    const int per = (ntri + 7) >> 3;
    const int tri_end = min(ntri, (xg + 1) * per);
    for (int tri = xg * per + wi; tri < tri_end; tri += nw) {
        const int g = tri * kKpPerWave + ks;
        const bool act = ks < kKpPerWave && g < total;
#pragma unroll
        for (int s = 0; s < 10; s++) my[s * kSlotStride] = 0.f;
        int ptx = p.w / 2, pty = p.h / 2;
        size_t fo = 0;
        if (act) {
            const slam_keypoint kp = p.kps[g];
            ptx = __float2int_rn(kp.x);
            pty = __float2int_rn(kp.y);
            fo = (size_t)p.kp_frame[g] * grad_frame(p.w, p.h);
        }
        const float2* P = p.grad + fo + grad_origin(p.w) + (size_t)pty * p.pitch + ptx;
        // the parity table whose pairs start at even pixel columns: 16-byte aligned loads
        const uint2* E = ent + (size_t)(ptx & 1) * (p.rows2 + 2) * kTargets + t;
        const bool interior = ptx - rad >= 1 && ptx + rad <= p.w - 2 && pty - rad >= 1 && pty + rad <= p.h - 2;
        if (__all(interior))
            tab_walk<false>(p, rec, E, P, ptx, pty, my);
        else
            tab_walk<true>(p, rec, E, P, ptx, pty, my);
        wave_sync();
        float* rws = raw[wave][ks < kKpPerWave ? ks : 0];
        // fold (slot0 += slot8, slot1 += slot9 of the same memory cell) for the 16 inner cells
        if (act && C <= 4) {
            const float* nxt = &sl[lane + 1];                    // lane of cell (R, C + 1)
            float* rw = rws + ((R - 1) * 4 + (C - 1)) * 8;
            rw[0] = __fadd_rn(my[1 * kSlotStride], my[9 * kSlotStride]);
            rw[1] = __fadd_rn(my[2 * kSlotStride], nxt[0]);
#pragma unroll
            for (int q = 2; q < 8; q++) rw[q] = my[(q + 1) * kSlotStride];
        }
        wave_sync();
        // first norm: 8 fma chains over k = q + 8m (one lane each), then the
        // v_reduce_sum order; clamp + sequential second norm on one lane
        if (act && t < 8) {
            float a = 0.f;
#pragma unroll 4
            for (int m = 0; m < 16; m++) { const float v = rws[t + 8 * m]; a = __fmaf_rn(v, v, a); }
            part[wave][ks][t] = a;
        }
        wave_sync();
        if (act && t == 0) {
            const float* l = part[wave][ks];
            const float nrm2 = __fadd_rn(__fadd_rn(__fadd_rn(l[0], l[4]), __fadd_rn(l[1], l[5])),
                                         __fadd_rn(__fadd_rn(l[2], l[6]), __fadd_rn(l[3], l[7])));
            const float thr = __fmul_rn(cr_sqrtf(nrm2), 0.2f);
            float n2 = 0.f;
#pragma unroll 4
            for (int k = 0; k < 128; k++) {
                const float v = fminf(rws[k], thr);
                rws[k] = v;
                n2 = __fadd_rn(n2, __fmul_rn(v, v));
            }
            const float sq = cr_sqrtf(n2);
            scal[wave][ks] = cr_divf(512.f, sq > FLT_EPSILON ? sq : FLT_EPSILON);
        }
        wave_sync();
        if (act && C <= 4) {
            const int cell = (R - 1) * 4 + (C - 1);
            const float sc = scal[wave][ks];
            const float* rw = rws + cell * 8;
            uint8_t* du = p.desc_u8 + (size_t)g * 128 + cell * 8;
            int ns = 0;
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                float v = rintf(__fmul_rn(rw[q], sc));
                v = fminf(fmaxf(v, 0.f), 255.f);
                const int iv = (int)v;
                if (q < 4) lo |= (uint32_t)iv << (8 * q);
                else hi |= (uint32_t)iv << (8 * (q - 4));
                ns += (iv - 128) * (iv - 128);
                if (p.desc_f32) p.desc_f32[(size_t)g * 128 + cell * 8 + q] = v;
            }
            *reinterpret_cast<uint2*>(du) = make_uint2(lo, hi);
            nrm[wave][ks][t] = ns;
        }
        wave_sync();
        if (act && t == 0) {
            int s = 0;
            for (int q = 0; q < kTargets; q++)
                if (q % 5 != 4) s += nrm[wave][ks][q];
            p.norm_i8[g] = s;
        }
        wave_sync();
    }
}

}  // namespace

// host replica of hal::exp32f (identical operations to oracle/sift.c)
float host_exp32f(float x, const float* tab)
{
    const double exp_prescale = 1.4426950408889634073599246810019 * 64;
    const double exp_max_val = 3000. * 64;
    const float A4 = (float)(1.000000000000002438532970795181890933776 / .9670371139572337719125840413672004409288e-2);
    const float A3 = (float)(.6931471805521448196800669615864773144641 / .9670371139572337719125840413672004409288e-2);
    const float A2 = (float)(.2402265109513301490103372422686535526573 / .9670371139572337719125840413672004409288e-2);
    const float A1 = (float)(.5550339366753125211915322047004666939128e-1 / .9670371139572337719125840413672004409288e-2);
    const float minval = (float)(-exp_max_val / exp_prescale);
    const float maxval = (float)(exp_max_val / exp_prescale);
    float xf = x < minval ? minval : x;
    xf = xf > maxval ? maxval : xf;
    xf = xf * (float)exp_prescale;
    int xi = (int)std::lrintf(xf);
    xf = (xf - (float)xi) * (float)(1. / 64);
    float yf = tab[xi & 63];
    int t = (xi >> 6) + 127;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    union { int32_t i; float f; } u;
    u.i = t << 23;
    yf = yf * u.f;
    float z = xf + A1;
    z = std::fma(z, xf, A2);
    z = std::fma(z, xf, A3);
    z = std::fma(z, xf, A4);
    return z * yf;
}


// Build (or reuse) the per-target table for keypoints of one (angle, size);
// false when the gather path does not apply (radius clipped by a tiny image).
bool sift_tab_prepare(slam_ctx* c, hipStream_t s, float kp_angle, float kp_size, int w, int h)
{
    if (c->opt_sift_kernel == SLAM_SIFT_KERNEL_GENERAL) return false;
    float angle = 360.f - kp_angle;
    if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    const float ori = angle, scl = kp_size * 0.5f;
    float cos_t = cosf(ori * (float)(M_PI / 180));
    float sin_t = sinf(ori * (float)(M_PI / 180));
    const float exp_scale = -1.f / (4 * 4 * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = (int)std::lrintf(hist_width * 1.4142135623730951f * (4 + 1) * 0.5f);
    const int diag = (int)std::sqrt((double)w * w + (double)h * h);
    if (radius > diag || radius > 127) return false;
    if (c->sift_tab_valid && c->sift_tab_angle == kp_angle && c->sift_tab_size == kp_size) return true;
    cos_t /= hist_width;
    sin_t /= hist_width;
    // per-sample records (raster order) and per-target lists of (record, corner)
    struct LE { int i, j, rec, dr, dc; };
    std::vector<float4> recs;
    std::vector<std::vector<LE>> lists(kTargets);
    for (int i = -radius; i <= radius; i++)
        for (int j = -radius; j <= radius; j++) {
            const float c_rot = (float)j * cos_t - (float)i * sin_t;
            const float r_rot = (float)j * sin_t + (float)i * cos_t;
            const float rbin = r_rot + (float)(4 / 2) - 0.5f;
            const float cbin = c_rot + (float)(4 / 2) - 0.5f;
            if (!(rbin > -1 && rbin < 4 && cbin > -1 && cbin < 4)) continue;
            const float wexp = host_exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, c->sift.exptab);
            const int r0 = (int)std::floor(rbin), c0 = (int)std::floor(cbin);
            const int idx = (int)recs.size();
            union { int32_t i; float f; } ij;
            ij.i = (i & 255) | ((j & 255) << 8);
            recs.push_back(make_float4(rbin - (float)r0, cbin - (float)c0, wexp, ij.f));
            for (int dr = 0; dr < 2; dr++)
                for (int dc = 0; dc < 2; dc++) {
                    const int R = r0 + 1 + dr, C = c0 + 1 + dc;
                    if (R < 1 || R > 4 || C < 1 || C > 5) continue;
                    lists[(R - 1) * 5 + (C - 1)].push_back({i, j, idx, dr, dc});
                }
        }
    // two zero records (weight 0 at the keypoint) for padding items and their partner: +0
    const int zrec = (int)recs.size();
    recs.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
    recs.push_back(make_float4(0.f, 0.f, 0.f, 0.f));
    if ((int)recs.size() > kMaxRec || zrec >= (1 << 14)) return false;
    // items: a sample and, when the target's next sample is its right neighbour,
    // that one too: rec | dr0 << 14 | dc0 << 15 | dr1 << 16 | dc1 << 17 | pair << 18.
    // Two tables: pairs start at even j (par 0) or odd j (par 1); a keypoint with
    // x parity q uses table q, so every pair is one 16-byte aligned load
    // (grad rows and frames have an even pixel count).
    std::vector<std::vector<uint32_t>> items[2];
    size_t mx = 0;
    for (int par = 0; par < 2; par++) {
        items[par].resize(kTargets);
        for (int t = 0; t < kTargets; t++) {
            const auto& L = lists[t];
            for (size_t k = 0; k < L.size();) {
                const LE& a0 = L[k];
                uint32_t it = (uint32_t)a0.rec | (uint32_t)a0.dr << 14 | (uint32_t)a0.dc << 15;
                if (((a0.j & 1) == par) && k + 1 < L.size() && L[k + 1].i == a0.i && L[k + 1].j == a0.j + 1 &&
                    L[k + 1].rec == a0.rec + 1) {
                    it |= (uint32_t)L[k + 1].dr << 16 | (uint32_t)L[k + 1].dc << 17 | 1u << 18;
                    k += 2;
                } else {
                    k += 1;
                }
                items[par][t].push_back(it);
            }
            mx = std::max(mx, items[par][t].size());
        }
    }
    const int rows2 = (int)((mx + 1) / 2);
    if (2 * (rows2 + 2) > kMaxRows2) return false;
    // layout [par][row2][target][2]: lane t reads one u64 = 2 consecutive items of its list
    std::vector<uint32_t> ent32((size_t)2 * (rows2 + 2) * kTargets * 2, (uint32_t)zrec);
    for (int par = 0; par < 2; par++)
        for (int t = 0; t < kTargets; t++)
            for (size_t k = 0; k < items[par][t].size(); k++)
                ent32[(((size_t)par * (rows2 + 2) + k / 2) * kTargets + t) * 2 + (k % 2)] = items[par][t][k];
    SiftTabMeta m;
    std::memset(&m, 0, sizeof(m));
    m.len = rows2 * 2;
    m.radius = radius;
    m.ori_deg = ori;
    const size_t rec_bytes = recs.size() * sizeof(float4), ent_bytes = ent32.size() * sizeof(uint32_t);
    if (c->sift_tab.ensure(rec_bytes + ent_bytes) != hipSuccess) return false;
    std::vector<uint8_t> blob(rec_bytes + ent_bytes);
    std::memcpy(blob.data(), recs.data(), rec_bytes);
    std::memcpy(blob.data() + rec_bytes, ent32.data(), ent_bytes);
    if (hipMemcpyAsync(c->sift_tab.p, blob.data(), blob.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        return false;
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    c->sift_meta = m;
    c->sift_tab_nrec = (int)recs.size();
    c->sift_tab_valid = true;
    c->sift_tab_angle = kp_angle;
    c->sift_tab_size = kp_size;
    return true;
}

hipError_t launch_sift_desc_tab(slam_ctx* c, hipStream_t s, int w, int h, int cap, int write_f32)
{
    hipError_t e;
    if ((e = c->desc_u8.ensure((size_t)cap * 128)) != hipSuccess) return e;
    if ((e = c->desc_norm.ensure((size_t)cap * 4)) != hipSuccess) return e;
    if (write_f32 && (e = c->desc_f32.ensure((size_t)cap * 128 * 4)) != hipSuccess) return e;
    TabParams p;
    p.grad = c->grad.as<float2>(); p.w = w; p.h = h; p.pitch = grad_pitch(w);
    p.kps = c->kps.as<slam_keypoint>(); p.kp_frame = c->kp_frame.as<int>(); p.total = c->misc.as<int>();
    p.cap = cap;
    p.nrec = c->sift_tab_nrec;
    p.rows2 = c->sift_meta.len / 2;
    p.rec = c->sift_tab.as<float4>();
    p.ent = reinterpret_cast<const uint2*>(c->sift_tab.as<uint8_t>() + (size_t)p.nrec * sizeof(float4));
    p.meta = c->sift_meta;
    p.desc_u8 = c->desc_u8.as<uint8_t>(); p.desc_f32 = write_f32 ? c->desc_f32.as<float>() : nullptr;
    p.norm_i8 = c->desc_norm.as<int>();
    // persistent: one 8-wave workgroup per CU (the LDS table is loaded once per
    // workgroup); a multiple of 8 workgroups for the XCD split
    const int waves = kWavesDefault;
    int grid = c->cu_count;
    const int need = (cap + kKpPerWave * waves - 1) / (kKpPerWave * waves);
    if (grid > need) grid = need;
    grid = (grid + 7) & ~7;
    if (grid < 8) grid = 8;
    prof_begin(c, 1, s);
    if (waves == 8) hipLaunchKernelGGL(sift_desc_tab<8>, dim3(grid), dim3(64 * 8), 0, s, p);
    else if (waves == 12) hipLaunchKernelGGL(sift_desc_tab<12>, dim3(grid), dim3(64 * 12), 0, s, p);
    else hipLaunchKernelGGL(sift_desc_tab<16>, dim3(grid), dim3(64 * 16), 0, s, p);
    prof_end(c, 1, s);
    return hipGetLastError();
}

}  // namespace slamhip
