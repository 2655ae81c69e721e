// C ABI of libslamhip (include/slamhip.h): context management, the reference
// entry points on host buffers, and the device-resident candidate batch.
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "slamhip_internal.h"

namespace slamhip {

hipError_t DevBuf::ensure(size_t n)
{
    if (n <= bytes && p) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
    size_t want = n < 256 ? 256 : n;
    want = (want + 4095) & ~(size_t)4095;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) bytes = want;
    return e;
}

void DevBuf::release()
{
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

int set_err(slam_ctx* c, int code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

void prof_begin(slam_ctx* c, int fam, hipStream_t s)
{
    if (!c->prof_on) return;
    ProfFamily& f = c->prof[fam];
    if ((int)f.ev.size() < 2 * (f.used + 1)) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
        f.ev.push_back(a);
        f.ev.push_back(b);
    }
    (void)hipEventRecord(f.ev[2 * f.used], s);
}

void prof_end(slam_ctx* c, int fam, hipStream_t s)
{
    if (!c->prof_on) return;
    ProfFamily& f = c->prof[fam];
    if ((int)f.ev.size() < 2 * (f.used + 1)) return;
    (void)hipEventRecord(f.ev[2 * f.used + 1], s);
    f.used++;
}

// ---- host restatements (identical arithmetic to oracle/sift.c) ----
float sift_sigma_diff()
{
    float s = 1.6f * 1.6f - 0.5f * 0.5f;
    return std::sqrt(s > 0.01f ? s : 0.01f);
}

int gauss_kernel_f32(int n, double sigma, float* k)
{
    double sigmaX = sigma > 0 ? sigma : (double)n * 0.15 + 0.35;
    double scale2X = -0.125 / (sigmaX * sigmaX);
    int n2 = (n - 1) / 2;
    double values[64];
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = std::exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2.0;
    sum += 1.0;
    if ((n & 1) == 0) sum += 1.0;
    double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; i++) {
        double t = values[i] * mul1;
        k[i] = (float)t;
        k[n - 1 - i] = (float)t;
    }
    k[n2] = (float)mul1;
    if ((n & 1) == 0) k[n2 + 1] = k[n2];
    return n;
}

void init_consts(slam_ctx* c)
{
    std::memset(&c->sift, 0, sizeof(c->sift));
    float sig = sift_sigma_diff();
    c->sift.ksize = (int)std::lrint((double)sig * 4 * 2 + 1) | 1;
    gauss_kernel_f32(c->sift.ksize, (double)sig, c->sift.gauss);
    for (int i = 0; i < 64; i++)
        c->sift.exptab[i] = (float)(std::exp2((double)i / 64.0) * .9670371139572337719125840413672004409288e-2);
    std::memset(&c->orb, 0, sizeof(c->orb));
    gauss_kernel_f32(7, 2.0, c->orb.gauss);
}


// keypoint-dependent rotation terms computed on the host with the same libm
// calls as the reference (calcSIFTDescriptor cosf/sinf; computeOrbDescriptors cos/sin)
void sift_kp_cs(const slam_keypoint* k, int n, std::vector<float>& cs)
{
    cs.resize((size_t)2 * n);
    for (int i = 0; i < n; i++) {
        float angle = 360.f - k[i].angle;
        if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        cs[2 * i] = cosf(angle * (float)(M_PI / 180));
        cs[2 * i + 1] = sinf(angle * (float)(M_PI / 180));
    }
}

int stream_sync(slam_ctx* c, hipStream_t s, bool poll)
{
    // poll: the wait is short (a batch step, one LM iteration) and sits on the
    // critical path behind a pinned async copy, so the host polls an event
    // instead of sleeping in a blocking wait (BA W = 8: 9.0 -> 8.2 ms per
    // window).  The host-buffer entry points keep the blocking wait: their
    // pageable copies have already waited, and the extra event cost them more
    // than it saved.
    if (!poll) {
        SLAM_HIP(c, hipStreamSynchronize(s));
        return SLAM_OK;
    }
    if (!c->ev_sync) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
    SLAM_HIP(c, hipEventRecord(c->ev_sync, s));
    for (;;) {
        const hipError_t e = hipEventQuery(c->ev_sync);
        if (e == hipSuccess) return SLAM_OK;
        if (e != hipErrorNotReady) return set_err(c, SLAM_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
    }
}

void* readback(slam_ctx* c, size_t n)
{
    if (n <= c->h_rb_bytes && c->h_rb) return c->h_rb;
    if (c->h_rb) (void)hipHostFree(c->h_rb);
    c->h_rb = nullptr;
    c->h_rb_bytes = 0;
    const size_t want = (n + 65535) & ~(size_t)65535;
    if (hipHostMalloc(&c->h_rb, want, hipHostMallocDefault) != hipSuccess) {
        c->h_rb = nullptr;
        return nullptr;
    }
    c->h_rb_bytes = want;
    return c->h_rb;
}

}  // namespace slamhip

using namespace slamhip;

namespace {

int pick_tsplit_fill(const slam_ctx* c, int nq, int nframes, int max_nt);
int split_rows_for(int norm);

// A batch queued by slam_batch_extract_async owns the frame / keypoint /
// descriptor / match buffers until slam_batch_finish takes it.
int async_guard(slam_ctx* c)
{
    if (c->async.state != 0) return set_err(c, SLAM_E_INVALID_ARG, "an asynchronous batch is in flight (slam_batch_finish)");
    return SLAM_OK;
}


// kNN key modes (knn.hip): 0 L2, 1 Hamming, 2 sqrt keys, 3 packed L2, 4 packed Hamming, 5 packed L1
constexpr int kModeL2 = 0, kModeSqrt = 2, kModeL2P = 3, kModeHamP = 4, kModeL1P = 5;

// choose a train split so that one matching launch fills the chip; packed L2
// and Hamming keys carry 10 index bits, so a split holds at most 1024 train rows
int pick_tsplit(const slam_ctx* c, int nq, int nframes, int max_nt, int mode)
{
    int t = pick_tsplit_fill(c, nq, nframes, max_nt);
    if (mode == kModeL2P || mode == kModeHamP) t = std::max(t, (max_nt + 1023) / 1024);
    if (mode == kModeL1P) t = std::max(t, (max_nt + (1 << 17) - 1) >> 17);
    return t;
}

// train rows one split of a packed-key launch can index (knn.hip: L2 keys carry
// 10 index bits, L1 keys 17, Hamming float keys 10 fraction bits)
int split_rows_for(int norm)
{
    return norm == SLAM_NORM_L1 ? (1 << 17) : 1024;
}

int pick_tsplit_fill(const slam_ctx* c, int nq, int nframes, int max_nt)
{
    int qblocks = (nq + 255) / 256;
    int blocks = qblocks * nframes;
    int want = (2 * c->cu_count + blocks - 1) / (blocks > 0 ? blocks : 1);
    int maxs = (max_nt + 63) / 64;
    if (want > maxs) want = maxs;
    if (want < 1) want = 1;
    if (want > 64) want = 64;
    return want;
}

// pinned readback space of at least n bytes (hipHostMalloc, grown on demand)


bool sift_desc_to_u8(const float* d, int n, std::vector<uint8_t>& out, double* maxnorm)
{
    out.resize((size_t)n * 128);
    double mx = 0;
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int k = 0; k < 128; k++) {
            float v = d[(size_t)i * 128 + k];
            if (!(v >= 0.f && v <= 255.f) || v != std::floor(v)) return false;
            out[(size_t)i * 128 + k] = (uint8_t)v;
            s += (double)v * v;
        }
        mx = std::max(mx, std::sqrt(s));
    }
    *maxnorm = mx;
    return true;
}

int norm_for(int matcher, int norm)
{
    if (norm == SLAM_NORM_DEFAULT) return matcher == SLAM_ORB_BF ? SLAM_NORM_HAMMING : SLAM_NORM_L2;
    return norm;
}

// knn over host descriptor sets; fills top_idx/top_dist (host) and, when
// out != nullptr, the ratio-test survivors in query order
int knn_host(slam_ctx* c, const void* q, int nq, const void* t, int nt, int matcher, int norm, double ratio,
             int* idx_out, float* dist_out, slam_dmatch* out, int cap, int* n_out)
{
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    if (int rc = async_guard(c)) return rc;
    norm = norm_for(matcher, norm);
    const bool orb = matcher == SLAM_ORB_BF;
    if (orb && norm != SLAM_NORM_HAMMING) return set_err(c, SLAM_E_UNSUPPORTED, "ORB descriptors need NORM_HAMMING");
    if (!orb && norm != SLAM_NORM_L2 && norm != SLAM_NORM_L1)
        return set_err(c, SLAM_E_UNSUPPORTED, "SIFT descriptors need NORM_L2 or NORM_L1");
    if (n_out) *n_out = 0;
    if (nq <= 0) return SLAM_OK;
    hipStream_t s = c->stream;
    const int kb = orb ? kOrbExpBytes : 128;
    const bool l1 = !orb && norm == SLAM_NORM_L1;
    int mode = orb ? kModeHamP : kModeL2;
    // query / train uploads (internal format)
    if (orb) {
        SLAM_HIP(c, c->qbuf.ensure((size_t)(nq + (nt > 0 ? nt : 0)) * 32));
        SLAM_HIP(c, c->tbuf.ensure((size_t)(nq + (nt > 0 ? nt : 0)) * kOrbExpBytes));
        uint8_t* raw = c->qbuf.as<uint8_t>();
        int8_t* ex = c->tbuf.as<int8_t>();
        SLAM_HIP(c, hipMemcpyAsync(raw, q, (size_t)nq * 32, hipMemcpyHostToDevice, s));
        if (nt > 0) SLAM_HIP(c, hipMemcpyAsync(raw + (size_t)nq * 32, t, (size_t)nt * 32, hipMemcpyHostToDevice, s));
        SLAM_HIP(c, launch_orb_expand(s, raw, nq + (nt > 0 ? nt : 0), ex));
    } else {
        std::vector<uint8_t> qu, tu;
        double mq = 0, mt = 0;
        if (!sift_desc_to_u8((const float*)q, nq, qu, &mq) || !sift_desc_to_u8((const float*)t, nt, tu, &mt))
            return set_err(c, SLAM_E_UNSUPPORTED, "SIFT descriptors must be integer-valued in [0, 255]");
        if (l1) mode = kModeL1P;                   // CUDA-build SIFT_BF: exact integer L1 keys
        else if (mq + mt > 2048.0) mode = kModeSqrt;   // sqrt keys: f32 sqrt may tie distinct d^2 beyond 2048
        else if ((mq + mt) * (mq + mt) < (double)((1 << 21) - 1)) mode = kModeL2P;   // packed keys
        else mode = kModeL2;
        SLAM_HIP(c, c->tbuf.ensure((size_t)(nq + nt) * 128));
        SLAM_HIP(c, c->query_norm.ensure((size_t)(nq + nt) * 4 + 16));
        uint8_t* d = c->tbuf.as<uint8_t>();
        SLAM_HIP(c, hipMemcpyAsync(d, qu.data(), qu.size(), hipMemcpyHostToDevice, s));
        if (nt > 0) SLAM_HIP(c, hipMemcpyAsync(d + (size_t)nq * 128, tu.data(), tu.size(), hipMemcpyHostToDevice, s));
        SLAM_HIP(c, launch_norms_u8(s, d, nq + nt, c->query_norm.as<int32_t>()));
    }
    const uint8_t* dq = orb ? (const uint8_t*)c->tbuf.p : c->tbuf.as<uint8_t>();
    const uint8_t* dt = dq + (size_t)nq * kb;
    const int32_t* qn = orb ? nullptr : c->query_norm.as<int32_t>();
    const int32_t* tn = orb ? nullptr : c->query_norm.as<int32_t>() + nq;
    int4 info = make_int4(0, nt > 0 ? nt : 0, 0, 0);
    SLAM_HIP(c, c->misc.ensure(256));
    SLAM_HIP(c, hipMemcpyAsync(c->misc.as<char>() + 64, &info, sizeof(info), hipMemcpyHostToDevice, s));
    const int32_t* dinfo = (const int32_t*)(c->misc.as<char>() + 64);
    const int tsplit = pick_tsplit(c, nq, 1, nt > 0 ? nt : 1, mode);
    SLAM_HIP(c, c->knn_part.ensure((size_t)tsplit * nq * sizeof(int4)));
    SLAM_HIP(c, c->match_rec.ensure((size_t)nq * (sizeof(slam_dmatch) + sizeof(int2) + sizeof(float2))));
    SLAM_HIP(c, c->match_flag.ensure((size_t)nq));
    SLAM_HIP(c, c->match_cnt.ensure(64));
    SLAM_HIP(c, c->match_out.ensure((size_t)nq * sizeof(slam_dmatch)));
    SLAM_HIP(c, hipMemsetAsync(c->match_cnt.p, 0, 64, s));
    SLAM_HIP(c, launch_knn(c, s, kb, dq, qn, nq, dt, tn, dinfo, 1, nt, mode, tsplit, c->knn_part.as<int4>()));
    slam_dmatch* rec = c->match_rec.as<slam_dmatch>();
    int2* tidx = reinterpret_cast<int2*>(rec + nq);
    float2* tdist = reinterpret_cast<float2*>(tidx + nq);
    SLAM_HIP(c, launch_knn_finish(c, s, c->knn_part.as<int4>(), nq, 1, tsplit, qn, mode, ratio, dinfo, tidx, tdist,
                                  rec, c->match_flag.as<uint8_t>(), c->match_cnt.as<int32_t>()));
    if (idx_out) {
        SLAM_HIP(c, hipMemcpyAsync(idx_out, tidx, (size_t)nq * sizeof(int2), hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipMemcpyAsync(dist_out, tdist, (size_t)nq * sizeof(float2), hipMemcpyDeviceToHost, s));
    }
    if (out) {
        SLAM_HIP(c, launch_compact(c, s, rec, c->match_flag.as<uint8_t>(), nq, 1, c->match_out.as<slam_dmatch>(),
                                   c->match_cnt.as<int32_t>() + 4, nq));
        int cnt = 0;
        SLAM_HIP(c, hipMemcpyAsync(&cnt, c->match_cnt.as<int32_t>() + 4, 4, hipMemcpyDeviceToHost, s));
        int rc = stream_sync(c, s);
        if (rc) return rc;
        *n_out = cnt;
        if (cnt > cap) return set_err(c, SLAM_E_CAPACITY, "match buffer too small");
        SLAM_HIP(c, hipMemcpy(out, c->match_out.p, (size_t)cnt * sizeof(slam_dmatch), hipMemcpyDeviceToHost));
        return SLAM_OK;
    }
    return stream_sync(c, s);
}

void orb_kp_ab(const slam_keypoint* k, int n, std::vector<float>& ab)
{
    ab.resize((size_t)2 * n);
    for (int i = 0; i < n; i++) {
        float angle = k[i].angle * (float)(M_PI / 180.f);
        ab[2 * i] = cosf(angle);
        ab[2 * i + 1] = sinf(angle);
    }
}

int upload_image(slam_ctx* c, const uint8_t* img, int w, int h, size_t step, int channels, const uint8_t** dimg,
                 size_t* dstep)
{
    const size_t row = (size_t)w * channels;
    SLAM_HIP(c, c->frames_in.ensure(row * h));
    // images of 256 KB and more: rows into pinned staging on the host thread pool,
    // then one DMA (a pageable copy of a 1080p BGR frame went through the runtime's
    // small staging buffers at a fraction of the link rate)
    const size_t bytes = row * h;
    if (bytes >= (256u << 10)) {
        if (c->ev_up) SLAM_HIP(c, hipEventSynchronize(c->ev_up));   // the previous upload has left the buffer
        else SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_up, hipEventDisableTiming));
        if (c->h_up_bytes < bytes) {
            if (c->h_up) (void)hipHostFree(c->h_up);
            c->h_up = nullptr;
            c->h_up_bytes = 0;
            const size_t want = (bytes + 65535) & ~(size_t)65535;
            SLAM_HIP(c, hipHostMalloc(&c->h_up, want, hipHostMallocDefault));
            c->h_up_bytes = want;
        }
        uint8_t* st = static_cast<uint8_t*>(c->h_up);
        if (step == row) {
            host_copy(st, img, bytes);
        } else {
            const int nb = std::min(h, 16);
            host_parallel_run(nb, [&](int b) {
                for (int y = b; y < h; y += nb) std::memcpy(st + (size_t)y * row, img + (size_t)y * step, row);
            });
        }
        SLAM_HIP(c, hipMemcpyAsync(c->frames_in.p, st, bytes, hipMemcpyHostToDevice, c->stream));
        SLAM_HIP(c, hipEventRecord(c->ev_up, c->stream));
    } else if (step == row) {
        SLAM_HIP(c, hipMemcpyAsync(c->frames_in.p, img, row * h, hipMemcpyHostToDevice, c->stream));
    } else {
        SLAM_HIP(c, hipMemcpy2DAsync(c->frames_in.p, row, img, step, row, h, hipMemcpyHostToDevice, c->stream));
    }
    *dimg = c->frames_in.as<uint8_t>();
    *dstep = row;
    return SLAM_OK;
}

bool valid_image(int w, int h, size_t step, int channels)
{
    return w > 0 && h > 0 && (channels == 1 || channels == 3 || channels == 4) && step >= (size_t)w * channels;
}

}  // namespace

extern "C" {

int slam_abi_version(void) { return SLAMHIP_ABI_VERSION; }

int slam_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

slam_ctx* slam_create(int device) { return slam_create_prio(device, 0); }

slam_ctx* slam_create_prio(int device, int priority)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    slam_ctx* c = new slam_ctx();
    c->device = device;
    int least = 0, greatest = 0;
    hipError_t e;
    if (priority > 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
        e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest);
    else
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = prop.multiProcessorCount;
    init_consts(c);
    return c;
}

void slam_destroy(slam_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->gray, &c->scores, &c->masks, &c->band_cnt, &c->band_pref, &c->frame_info, &c->ftmp,
                      &c->grad, &c->orbblur, &c->kps, &c->kp_frame, &c->desc_u8, &c->desc_f32,
                      &c->desc_norm, &c->desc_exp, &c->query_norm, &c->knn_part, &c->match_rec, &c->match_flag,
                      &c->match_cnt, &c->match_out, &c->frames_in, &c->qbuf, &c->tbuf, &c->misc, &c->ba_obs,
                      &c->ba_par, &c->ba_jac, &c->ba_red, &c->ba_S, &c->ba_aux, &c->sd_pyr, &c->sd_cand,
                      &c->sd_kps, &c->sd_kpc, &c->sift_tab, &c->sift_band_buf, &c->sift_cols_buf, &c->sift_cols_park, &c->sift_colw_buf, &c->sift_split, &c->sift_split_cnt, &c->geom};
    for (DevBuf* b : bufs) b->release();
    if (c->h_up) (void)hipHostFree(c->h_up);
    if (c->ev_up) (void)hipEventDestroy(c->ev_up);
    if (c->h_rb) (void)hipHostFree(c->h_rb);
    if (c->h_win) (void)hipHostFree(c->h_win);
    if (c->ev_win) (void)hipEventDestroy(c->ev_win);
    if (c->ev_rdev) (void)hipEventDestroy(c->ev_rdev);
    if (c->ev_order) (void)hipEventDestroy(c->ev_order);
    for (hipEvent_t e : c->ev_stage)
        if (e) (void)hipEventDestroy(e);
    if (c->h_async) (void)hipHostFree(c->h_async);
    for (auto& f : c->prof)
        for (hipEvent_t e : f.ev) (void)hipEventDestroy(e);
    if (c->ev_sync) (void)hipEventDestroy(c->ev_sync);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* slam_last_error(const slam_ctx* c) { return c ? c->err.c_str() : "no context"; }

int slam_synchronize(slam_ctx* c)
{
    if (!c) return SLAM_E_INVALID_ARG;
    return stream_sync(c, c->stream);
}

int slam_matcher_type(int use_sift_bf, int use_sift_flann, int use_orb)
{
    if (use_sift_bf) return SLAM_SIFT_BF;
    if (use_sift_flann) return SLAM_SIFT_FLANN;
    if (use_orb) return SLAM_ORB_BF;
    return SLAM_E_BAD_MATCHER;
}

int slam_select_good(const int32_t* counts, int n, int required, int skip_head, int first_fit)
{
    int good = SLAM_FRAME_NOT_FOUND, best = 0;
    for (int i = n - 1; i >= skip_head; i--) {
        if (counts[i] >= required && counts[i] >= best) {
            good = i;
            best = counts[i];
            if (first_fit) break;
        }
    }
    return good;
}

namespace {
// A winner queued by slam_batch_result_begin is read from kps / match_* on the
// context stream; work on another stream that rewrites those buffers waits for it.
int win_guard(slam_ctx* c, hipStream_t s)
{
    if (c->win_pending && s != c->stream) SLAM_HIP(c, hipStreamWaitEvent(s, c->ev_win, 0));
    return SLAM_OK;
}

// SLAM_OPT_SIFT_KERNEL dispatch for keypoints sharing one angle and size
// (uniform) or not: AUTO takes colw (FAST keypoints) or band, then tab, then the
// general kernel; a forced
// kernel whose schedule does not apply is refused (SLAM_E_UNSUPPORTED), never
// replaced by another.  *kernel = the SLAM_SIFT_KERNEL_* that runs.
int pick_sift_kernel(slam_ctx* c, hipStream_t s, bool uniform, float angle, float size, int w, int h, int* kernel)
{
    const int opt = c->opt_sift_kernel;
    if (opt == SLAM_SIFT_KERNEL_COLW) {
        if (!uniform || !sift_band_prepare(c, s, angle, size, w, h) || !c->sift_colw_valid ||
            sift_band_obin_mode(c) != 1)
            return set_err(c, SLAM_E_UNSUPPORTED, "the forced SIFT descriptor kernel cannot run these keypoints");
        *kernel = SLAM_SIFT_KERNEL_BAND;
        c->last_sift_kernel = SLAM_SIFT_KERNEL_COLW;
        return SLAM_OK;
    }
    if (opt == SLAM_SIFT_KERNEL_COLS) {
        // the one-keypoint-per-lane A/B kernel runs behind the band kernel's launch
        // path (its tables are built with the band tables)
        if (!uniform || !sift_band_prepare(c, s, angle, size, w, h) || !c->sift_cols_valid ||
            sift_band_obin_mode(c) != 1)
            return set_err(c, SLAM_E_UNSUPPORTED, "the forced SIFT descriptor kernel cannot run these keypoints");
        *kernel = SLAM_SIFT_KERNEL_BAND;
        c->last_sift_kernel = SLAM_SIFT_KERNEL_COLS;
        return SLAM_OK;
    }
    if (uniform && (opt == SLAM_SIFT_KERNEL_AUTO || opt == SLAM_SIFT_KERNEL_BAND) &&
        sift_band_prepare(c, s, angle, size, w, h)) {
        *kernel = SLAM_SIFT_KERNEL_BAND;
        // AUTO: the column-per-wave kernel runs behind the band launch path when its
        // tables were built (FAST keypoints: floor(obin) in [-9, -1])
        if (opt == SLAM_SIFT_KERNEL_AUTO && c->sift_colw_valid && sift_colw_enabled() && !sift_band4_enabled() &&
            sift_band_obin_mode(c) == 1) {
            c->last_sift_kernel = SLAM_SIFT_KERNEL_COLW;
            return SLAM_OK;
        }
    }
    else if (uniform && (opt == SLAM_SIFT_KERNEL_AUTO || opt == SLAM_SIFT_KERNEL_TAB) &&
             sift_tab_prepare(c, s, angle, size, w, h))
        *kernel = SLAM_SIFT_KERNEL_TAB;
    else if (opt == SLAM_SIFT_KERNEL_AUTO || opt == SLAM_SIFT_KERNEL_GENERAL)
        *kernel = SLAM_SIFT_KERNEL_GENERAL;
    else
        return set_err(c, SLAM_E_UNSUPPORTED, "the forced SIFT descriptor kernel cannot run these keypoints");
    c->last_sift_kernel = *kernel;
    return SLAM_OK;
}

// fastExtractor on an image already in device memory (d_img) or uploaded from
// host memory (img) first
int fast_common(slam_ctx* c, hipStream_t s, const uint8_t* img, const uint8_t* d_img, int w, int h, size_t step,
                int channels, int threshold, int nonmax, int type, slam_keypoint* out, int cap, int* n_out)
{
    if (!c || !n_out || (cap > 0 && !out)) return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    *n_out = 0;
    if (type != SLAM_FAST_TYPE_9_16 && type != SLAM_FAST_TYPE_7_12 && type != SLAM_FAST_TYPE_5_8)
        return set_err(c, SLAM_E_INVALID_ARG, "FAST detector type");
    if (w <= 0 || h <= 0 || (!img && !d_img)) return SLAM_OK;   // empty image -> no keypoints
    if (!valid_image(w, h, step, channels)) return SLAM_E_INVALID_ARG;
    if (w > 4096) return set_err(c, SLAM_E_UNSUPPORTED, "width > 4096");
    SLAM_HIP(c, hipSetDevice(c->device));
    const uint8_t* dimg = d_img;
    size_t dstep = step;
    int rc = 0;
    if (!d_img) {
        rc = upload_image(c, img, w, h, step, channels, &dimg, &dstep);
        if (rc) return rc;
    }
    if ((rc = win_guard(c, s))) return rc;
    SLAM_HIP(c, launch_fast_detect(c, s, dimg, dstep * h, dstep, channels, 1, w, h, threshold, nonmax, 0, type));
    const int kcap = std::max(cap, 1);
    SLAM_HIP(c, launch_fast_emit(c, s, 1, w, h, kcap));
    int4 info;
    SLAM_HIP(c, hipMemcpyAsync(&info, c->frame_info.p, sizeof(info), hipMemcpyDeviceToHost, s));
    rc = stream_sync(c, s);
    if (rc) return rc;
    // info.z: the unclipped count (no border filter here, so it equals the
    // filtered count; info.y is clipped to the capacity by fast_finalize)
    *n_out = info.z;
    if (info.z > cap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    if (info.z > 0)
        SLAM_HIP(c, hipMemcpy(out, c->kps.p, (size_t)info.z * sizeof(slam_keypoint), hipMemcpyDeviceToHost));
    return SLAM_OK;
}
}  // namespace

int slam_fast(slam_ctx* c, const uint8_t* img, int w, int h, size_t step, int channels, int threshold, int nonmax,
              int type, slam_keypoint* out, int cap, int* n_out)
{
    return fast_common(c, c ? c->stream : nullptr, img, nullptr, w, h, step, channels, threshold, nonmax, type, out,
                       cap, n_out);
}

int slam_fast_dev(slam_ctx* c, void* stream, const uint8_t* d_img, int w, int h, size_t step, int channels,
                  int threshold, int nonmax, int type, slam_keypoint* out, int cap, int* n_out)
{
    if (!c) return SLAM_E_INVALID_ARG;
    return fast_common(c, stream ? (hipStream_t)stream : c->stream, nullptr, d_img, w, h, step, channels, threshold,
                       nonmax, type, out, cap, n_out);
}

int slam_describe(slam_ctx* c, const uint8_t* img, int w, int h, size_t step, int channels, int matcher,
                  slam_keypoint* kps, int* n_inout, void* desc)
{
    if (!c || !n_inout) return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    int n = *n_inout;
    if (n < 0 || (n > 0 && (!kps || !desc))) return SLAM_E_INVALID_ARG;
    if (!img || w <= 0 || h <= 0) { *n_inout = 0; return SLAM_OK; }
    if (!valid_image(w, h, step, channels)) return SLAM_E_INVALID_ARG;
    SLAM_HIP(c, hipSetDevice(c->device));
    const bool orb = matcher == SLAM_ORB_BF;
    if (orb) {
        // KeyPointsFilter::runByImageBorder(keypoints, image.size(), 31): in place, order kept
        int m = 0;
        if (!(h <= 2 * kOrbEdge || w <= 2 * kOrbEdge)) {
            for (int i = 0; i < n; i++) {
                long x = std::lrint(kps[i].x), y = std::lrint(kps[i].y);
                if (x >= kOrbEdge && x < w - kOrbEdge && y >= kOrbEdge && y < h - kOrbEdge) kps[m++] = kps[i];
            }
        }
        n = m;
        *n_inout = n;
        for (int i = 0; i < n; i++)
            if (kps[i].octave != 0) return set_err(c, SLAM_E_UNSUPPORTED, "ORB keypoints must be octave 0");
    } else {
        for (int i = 0; i < n; i++)
            if (kps[i].octave != 0) return set_err(c, SLAM_E_UNSUPPORTED, "SIFT keypoints must be octave 0");
    }
    if (n == 0) return SLAM_OK;
    hipStream_t s = c->stream;
    const uint8_t* dimg;
    size_t dstep;
    int rc = upload_image(c, img, w, h, step, channels, &dimg, &dstep);
    if (rc) return rc;
    SLAM_HIP(c, launch_gray(c, s, dimg, dstep, channels, w, h));
    SLAM_HIP(c, c->kps.ensure((size_t)n * sizeof(slam_keypoint)));
    SLAM_HIP(c, c->kp_frame.ensure((size_t)n * sizeof(int)));
    SLAM_HIP(c, c->misc.ensure(256));
    SLAM_HIP(c, c->qbuf.ensure((size_t)n * 2 * sizeof(float)));
    SLAM_HIP(c, hipMemcpyAsync(c->kps.p, kps, (size_t)n * sizeof(slam_keypoint), hipMemcpyHostToDevice, s));
    SLAM_HIP(c, hipMemsetAsync(c->kp_frame.p, 0, (size_t)n * sizeof(int), s));
    SLAM_HIP(c, hipMemcpyAsync(c->misc.p, &n, sizeof(int), hipMemcpyHostToDevice, s));
    std::vector<float> rot;
    if (orb) orb_kp_ab(kps, n, rot);
    else sift_kp_cs(kps, n, rot);
    SLAM_HIP(c, hipMemcpyAsync(c->qbuf.p, rot.data(), rot.size() * sizeof(float), hipMemcpyHostToDevice, s));
    if (orb) {
        SLAM_HIP(c, launch_orb_blur(c, s, 1, w, h));
        SLAM_HIP(c, launch_orb_desc(c, s, 1, w, h, c->qbuf.as<float>(), n));
        SLAM_HIP(c, hipMemcpyAsync(desc, c->desc_u8.p, (size_t)n * 32, hipMemcpyDeviceToHost, s));
    } else {
        // gather path when every keypoint has the same angle and size (FAST: -1, 7)
        // (and every keypoint inside the image: the table kernels read the window
        // around it from the padded gradient map without a per-keypoint test)
        bool uniform = true;
        for (int i = 0; i < n && uniform; i++)
            uniform = kps[i].angle == kps[0].angle && kps[i].size == kps[0].size && kps[i].x >= 0.f &&
                      kps[i].x <= (float)(w - 1) && kps[i].y >= 0.f && kps[i].y <= (float)(h - 1);
        // the kernel is picked before the gradient map is written: the band kernel
        // takes the map with obin stored per pixel (its table checks the map's size)
        SLAM_HIP(c, c->grad.ensure((size_t)grad_frame(w, h) * 8));
        int kernel = 0;
        if ((rc = pick_sift_kernel(c, s, uniform, kps[0].angle, kps[0].size, w, h, &kernel))) return rc;
        const int obin = kernel == SLAM_SIFT_KERNEL_BAND ? sift_band_obin_mode(c) : 0;
        SLAM_HIP(c, launch_sift_base(c, s, 1, w, h, obin, c->sift_band.ori_deg));
        if (kernel == SLAM_SIFT_KERNEL_BAND) {
            SLAM_HIP(c, launch_sift_desc_band(c, s, w, h, n, 1, obin));
        } else if (kernel == SLAM_SIFT_KERNEL_TAB) {
            SLAM_HIP(c, launch_sift_desc_tab(c, s, w, h, n, 1));
        } else {
            SLAM_HIP(c, launch_sift_desc(c, s, 1, w, h, c->qbuf.as<float>(), n, 1));
        }
        SLAM_HIP(c, hipMemcpyAsync(desc, c->desc_f32.p, (size_t)n * 128 * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    return stream_sync(c, s);
}

int slam_sift_detect(slam_ctx* c, const uint8_t* img, int w, int h, size_t step, int channels, slam_keypoint* kps,
                     int cap, int* n_out, float* desc)
{
    if (c && c->async.state) return async_guard(c);
    if (!c || !n_out || cap < 0 || (cap > 0 && !kps)) return SLAM_E_INVALID_ARG;
    *n_out = 0;
    if (!img || w <= 0 || h <= 0) return SLAM_OK;
    if (!valid_image(w, h, step, channels)) return SLAM_E_INVALID_ARG;
    SLAM_HIP(c, hipSetDevice(c->device));
    c->batch.unpublish();       // the detector stages through the batch buffers
    const uint8_t* dimg;
    size_t dstep;
    int rc = upload_image(c, img, w, h, step, channels, &dimg, &dstep);
    if (rc) return rc;
    if ((rc = sift_detect(c, dimg, dstep, channels, w, h, kps, cap, n_out, desc))) return rc;
    if (*n_out > cap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    return SLAM_OK;
}

int slam_sift_detect_batch(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h, int channels,
                           slam_keypoint* kps, int cap, int32_t* n_out, float* desc)
{
    if (c && c->async.state) return async_guard(c);
    if (!c || nframes < 0 || cap < 0) return SLAM_E_INVALID_ARG;
    if (nframes == 0) return SLAM_OK;
    if (!n_out || (cap > 0 && !kps)) return SLAM_E_INVALID_ARG;
    for (int f = 0; f < nframes; f++) n_out[f] = 0;
    if (w <= 0 || h <= 0) return SLAM_OK;
    if (!d_frames || (channels != 1 && channels != 3) || w < 3 || h < 3) return SLAM_E_INVALID_ARG;
    if (nframes > kSiftDetectMaxFrames) return set_err(c, SLAM_E_INVALID_ARG, "nframes above kSiftDetectMaxFrames");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // the detector stages its keypoints, frames and descriptors in the context's
    // batch buffers: a published batch is gone (slam_batch_* results refuse), and
    // a caller stream waits for the context stream's earlier readers of them
    c->batch.unpublish();
    if (s != c->stream) {
        if (!c->ev_order) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming));
        SLAM_HIP(c, hipEventRecord(c->ev_order, c->stream));
        SLAM_HIP(c, hipStreamWaitEvent(s, c->ev_order, 0));
    }
    int rc = sift_detect_batch(c, s, d_frames, nframes, w, h, channels, kps, cap, n_out, desc);
    if (rc) return rc;
    for (int f = 0; f < nframes; f++)
        if (n_out[f] > cap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    return SLAM_OK;
}

int slam_reconstruct(slam_ctx* c, const double* K, const double* R1, const double* t1, const double* R2,
                     const double* t2, const float* pts1, const float* pts2, int n, double* out)
{
    if (!c || !K || !R1 || !t1 || !R2 || !t2 || n < 0 || (n > 0 && (!pts1 || !pts2 || !out)))
        return SLAM_E_INVALID_ARG;
    if (n == 0) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    return triangulate(c, K, R1, t1, R2, t2, pts1, pts2, n, out);
}

int slam_estimate_transformation(slam_ctx* c, const float* pts1, const float* pts2, int n, const double* K,
                                 int use_ransac, double prob, double threshold, double distance_threshold, double* R,
                                 double* t, uint8_t* chirality, uint8_t* ransac_mask, int* passed)
{
    if (!c || !K || !R || !t || !passed || n < 0 || (n > 0 && (!pts1 || !pts2))) return SLAM_E_INVALID_ARG;
    *passed = 0;
    if (n == 0) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    return relative_pose(c, pts1, pts2, n, K, use_ransac, prob, threshold, distance_threshold, R, t, chirality,
                         ransac_mask, passed);
}

int slam_solve_pnp_ransac(slam_ctx* c, const float* obj, const float* img, int n, const double* K,
                          int iterations_count, float reprojection_error, double confidence, double* rvec,
                          double* tvec, uint8_t* inlier_mask, int* n_inliers, int* found)
{
    if (!c || !K || !rvec || !tvec || !n_inliers || !found || n < 0 || (n > 0 && (!obj || !img)))
        return SLAM_E_INVALID_ARG;
    *found = 0;
    *n_inliers = 0;
    SLAM_HIP(c, hipSetDevice(c->device));
    return pnp_ransac(c, obj, img, n, K, iterations_count, reprojection_error, confidence, rvec, tvec, inlier_mask,
                      n_inliers, found);
}

int slam_knn2(slam_ctx* c, const void* q, int nq, const void* t, int nt, int matcher, int norm, int* idx,
              float* dist)
{
    if (!c || nq < 0 || nt < 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t)) return SLAM_E_INVALID_ARG;
    if (nq == 0) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    return knn_host(c, q, nq, t, nt, matcher, norm, 0.0, idx, dist, nullptr, 0, nullptr);
}

int slam_match(slam_ctx* c, const void* q, int nq, const void* t, int nt, int matcher, int norm, double ratio,
               slam_dmatch* out, int cap, int* n_out)
{
    if (!c || !n_out || nq < 0 || nt < 0 || (nq > 0 && !q) || (nt > 0 && !t)) return SLAM_E_INVALID_ARG;
    *n_out = 0;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    // DescriptorMatcher::knnMatch with an empty train or query set -> no matches
    if (nq == 0 || nt == 0) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    return knn_host(c, q, nq, t, nt, matcher, norm, ratio, nullptr, nullptr, out, cap, n_out);
}

int slam_match_frame(slam_ctx* c, const void* prev_desc, int nprev, const uint8_t* img, int w, int h, size_t step,
                     int channels, int matcher, int norm, double ratio, slam_keypoint* kps, int* n_inout,
                     slam_dmatch* out, int cap, int* n_out)
{
    if (!c || !n_inout || !n_out) return SLAM_E_INVALID_ARG;
    *n_out = 0;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    const size_t dbytes = matcher == SLAM_ORB_BF ? 32 : 128 * sizeof(float);
    std::vector<uint8_t> desc((size_t)std::max(*n_inout, 1) * dbytes);
    int rc = slam_describe(c, img, w, h, step, channels, matcher, kps, n_inout, desc.data());
    if (rc) return rc;
    return slam_match(c, prev_desc, nprev, desc.data(), *n_inout, matcher, norm, ratio, out, cap, n_out);
}

// ---- device-resident batch ----

size_t slam_batch_desc_bytes(int matcher, int n)
{
    if (n < 0) return 0;
    if (matcher == SLAM_ORB_BF) return (size_t)n * kOrbExpBytes;
    return (size_t)n * 128 + (size_t)n * 4;
}

// ---- batch pieces: enqueue (no host sync) / commit (after the read-back) ----

// gray + FAST + emit + descriptors for every frame, queued on s; *cap_out = the
// keypoint capacity
static int batch_extract_enqueue(slam_ctx* c, hipStream_t s, const uint8_t* d_frames, int nframes, int w, int h,
                                 int threshold, int matcher, int* cap_out)
{
    const bool orb = matcher == SLAM_ORB_BF;
    // the previous batch's host state is dropped before anything is queued; the
    // new batch is published only by batch_extract_commit, together with its
    // per-frame vectors, so a failed enqueue or commit leaves no frame count
    // that indexes vectors of another size
    c->batch.unpublish();
    // keypoint capacity: 1/16 of the pixels per frame (FAST-9 with NMS keeps at
    // most one corner per 2 x 2 block), at least 4096
    const long per = std::max(4096L, (long)w * h / 16);
    const int cap = (int)std::min(per * nframes, 64L * 1024 * 1024);
    *cap_out = cap;
    int rc = win_guard(c, s);
    if (rc) return rc;
    for (hipEvent_t& e : c->ev_stage)
        if (!e) SLAM_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // FAST of these frames already on the device (slam_batch_fast, e.g.
    // fillVideoFrameBatch's count pass over the same batch): taken as it is
    const int border = orb ? kOrbEdge : 0;
    const slam_ctx::FastReuse& R = c->fast_reuse;
    static const bool reuse_on = [] { const char* e = getenv("SLAMHIP_FAST_REUSE"); return !(e && e[0] == '0'); }();
    const bool reuse = reuse_on && R.gen == c->fast_gen && R.frames == d_frames && R.nframes == nframes && R.w == w &&
                       R.h == h && R.thr == threshold && R.border == border && R.cap == cap;
    c->fast_reused = reuse;
    if (!reuse) {
        SLAM_HIP(c, launch_fast_detect(c, s, d_frames, (size_t)w * h * 3, (size_t)w * 3, 3, nframes, w, h, threshold, 1,
                                       border));
        SLAM_HIP(c, launch_fast_emit(c, s, nframes, w, h, cap));
    }
    if (orb) {
        SLAM_HIP(c, launch_orb_blur(c, s, nframes, w, h));
        SLAM_HIP(c, hipEventRecord(c->ev_stage[0], s));
        SLAM_HIP(c, launch_orb_desc(c, s, nframes, w, h, nullptr, cap));
        SLAM_HIP(c, hipEventRecord(c->ev_stage[1], s));
        c->stage_recorded = true;
    } else {
        // the kernel is picked first (its table checks the gradient map's size):
        // for the band kernel the map stores obin per pixel
        SLAM_HIP(c, c->grad.ensure((size_t)nframes * grad_frame(w, h) * 8));
        int kernel = 0;
        if ((rc = pick_sift_kernel(c, s, true, -1.f, 7.f, w, h, &kernel))) return rc;   // FAST: angle -1, size 7
        const int obin = kernel == SLAM_SIFT_KERNEL_BAND ? sift_band_obin_mode(c) : 0;
        SLAM_HIP(c, launch_sift_base(c, s, nframes, w, h, obin, c->sift_band.ori_deg));
        SLAM_HIP(c, hipEventRecord(c->ev_stage[0], s));
        if (kernel == SLAM_SIFT_KERNEL_BAND) {
            SLAM_HIP(c, launch_sift_desc_band(c, s, w, h, cap, 0, obin));
        } else if (kernel == SLAM_SIFT_KERNEL_TAB) {
            SLAM_HIP(c, launch_sift_desc_tab(c, s, w, h, cap, 0));
        } else {
            SLAM_HIP(c, launch_sift_desc(c, s, nframes, w, h, nullptr, cap, 0));
        }
        SLAM_HIP(c, hipEventRecord(c->ev_stage[1], s));
        c->stage_recorded = true;
    }
    return SLAM_OK;
}

// host batch state from the read-back frame table (info[0..nframes) + the total
// in info[nframes].x)
static int batch_extract_commit(slam_ctx* c, hipStream_t s, const int4* info, int nframes, int w, int h,
                                int matcher, int cap, int32_t* kp_counts)
{
    BatchState& B = c->batch;
    B.unpublish();
    const int total = info[nframes].x;
    if (total > cap) return set_err(c, SLAM_E_CAPACITY, "batch keypoint capacity exceeded");
    B.total_kps = total;
    B.kp_counts.resize(nframes);
    B.kp_counts_raw.resize(nframes);
    B.kp_offsets.resize(nframes);
    int mx = 0;
    for (int f = 0; f < nframes; f++) {
        B.kp_offsets[f] = info[f].x;
        B.kp_counts[f] = info[f].y;
        B.kp_counts_raw[f] = info[f].z;
        mx = std::max(mx, info[f].y);
        if (kp_counts) kp_counts[f] = info[f].z;
    }
    B.est_max_nt = mx;
    B.w = w; B.h = h; B.matcher = matcher;
    B.have_desc = true;
    B.nframes = nframes;   // published last: every per-frame vector now holds nframes entries
    return SLAM_OK;
}

// kNN + ratio of every extracted frame vs the query, queued on s.  max_nt: the
// largest per-frame train count the launch is sized for (packed L2 keys need
// ceil(max_nt / tsplit) <= 1024).  *launched = 0 when there is nothing to match.
static int batch_match_enqueue(slam_ctx* c, hipStream_t s, int nf, int matcher, const void* d_query, int nq,
                               int norm, double ratio, int max_nt, int* launched)
{
    BatchState& B = c->batch;
    const bool orb = matcher == SLAM_ORB_BF;
    norm = norm_for(matcher, norm);
    B.have_matches = false;
    *launched = 0;
    if ((orb && norm != SLAM_NORM_HAMMING) || (!orb && norm != SLAM_NORM_L2 && norm != SLAM_NORM_L1))
        return set_err(c, SLAM_E_UNSUPPORTED, "unsupported norm for the batch matcher");
    B.matched_nq = nq;
    B.have_matches = true;
    if (nq == 0) return SLAM_OK;
    const int rc = win_guard(c, s);
    if (rc) return rc;
    max_nt = std::max(max_nt, 1);
    // batch SIFT descriptors: |d| <= 512 + 6 by construction, so d^2 < 2^21 - 1 (packed keys)
    const int mode = orb ? kModeHamP : norm == SLAM_NORM_L1 ? kModeL1P : kModeL2P;
    const int tsplit = pick_tsplit(c, nq, nf, max_nt, mode);
    SLAM_HIP(c, c->knn_part.ensure((size_t)nf * tsplit * nq * sizeof(int4)));
    SLAM_HIP(c, c->match_rec.ensure((size_t)nf * nq * sizeof(slam_dmatch)));
    SLAM_HIP(c, c->match_flag.ensure((size_t)nf * nq));
    SLAM_HIP(c, c->match_cnt.ensure((size_t)nf * 8 + 64));
    SLAM_HIP(c, hipMemsetAsync(c->match_cnt.p, 0, (size_t)nf * 4, s));
    const uint8_t* dq = (const uint8_t*)d_query;
    const int32_t* qn = orb ? nullptr : (const int32_t*)(dq + (size_t)nq * 128);
    const void* t = orb ? c->desc_exp.p : c->desc_u8.p;
    const int32_t* tn = orb ? nullptr : c->desc_norm.as<int32_t>();
    SLAM_HIP(c, launch_knn(c, s, orb ? kOrbExpBytes : 128, dq, qn, nq, t, tn, c->frame_info.as<int32_t>(), nf, max_nt, mode,
                           tsplit, c->knn_part.as<int4>()));
    SLAM_HIP(c, launch_knn_finish(c, s, c->knn_part.as<int4>(), nq, nf, tsplit, qn, mode, ratio,
                                  c->frame_info.as<int32_t>(), nullptr, nullptr, c->match_rec.as<slam_dmatch>(),
                                  c->match_flag.as<uint8_t>(), c->match_cnt.as<int32_t>()));
    *launched = tsplit;
    return SLAM_OK;
}

int slam_batch_extract(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h, int threshold,
                       int matcher, int32_t* kp_counts)
{
    if (!c || !d_frames || nframes <= 0 || w <= 0 || h <= 0) return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    if (w > 4096) return set_err(c, SLAM_E_UNSUPPORTED, "width > 4096");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    int cap = 0;
    int rc = batch_extract_enqueue(c, s, d_frames, nframes, w, h, threshold, matcher, &cap);
    if (rc) return rc;
    // frame table and total into pinned memory: two DMA copies, one sync
    int4* info = (int4*)readback(c, sizeof(int4) * (nframes + 1));
    if (!info) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    SLAM_HIP(c, hipMemcpyAsync(info, c->frame_info.p, sizeof(int4) * nframes, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(info + nframes, c->misc.p, sizeof(int), hipMemcpyDeviceToHost, s));
    rc = stream_sync(c, s, true);
    if (rc) return rc;
    return batch_extract_commit(c, s, info, nframes, w, h, matcher, cap, kp_counts);
}

int slam_batch_fast(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h, int threshold,
                    int32_t* kp_counts)
{
    if (!c || !d_frames || nframes <= 0 || w <= 0 || h <= 0) return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    if (w > 4096) return set_err(c, SLAM_E_UNSUPPORTED, "width > 4096");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    BatchState& B = c->batch;
    B.unpublish();
    const long per = std::max(4096L, (long)w * h / 16);
    const int cap = (int)std::min(per * nframes, 64L * 1024 * 1024);
    int rc = win_guard(c, s);
    if (rc) return rc;
    // gray + FAST-9 + NMS + the raster-order emit of slam_batch_extract, no descriptors
    SLAM_HIP(c, launch_fast_detect(c, s, d_frames, (size_t)w * h * 3, (size_t)w * 3, 3, nframes, w, h, threshold, 1, 0));
    SLAM_HIP(c, launch_fast_emit(c, s, nframes, w, h, cap));
    {
        // recorded only when the caller has vouched (SLAM_OPT_FAST_REUSE) that the
        // frames' contents stay as they are until the extraction: the reuse test
        // compares pointers, and a freed and reallocated buffer can come back at
        // the same address holding other frames
        slam_ctx::FastReuse& R = c->fast_reuse;
        R.frames = d_frames; R.nframes = nframes; R.w = w; R.h = h; R.thr = threshold; R.border = 0; R.cap = cap;
        R.gen = c->opt_fast_reuse ? c->fast_gen : ~0ull;   // the batch extraction of these frames takes them
    }
    int4* info = (int4*)readback(c, sizeof(int4) * (nframes + 1));
    if (!info) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    SLAM_HIP(c, hipMemcpyAsync(info, c->frame_info.p, sizeof(int4) * nframes, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(info + nframes, c->misc.p, sizeof(int), hipMemcpyDeviceToHost, s));
    rc = stream_sync(c, s, true);
    if (rc) return rc;
    const int est = B.est_max_nt;             // the fused matcher's size estimate is not this batch's
    rc = batch_extract_commit(c, s, info, nframes, w, h, SLAM_SIFT_FLANN, cap, kp_counts);
    B.est_max_nt = est;
    B.have_desc = false;
    return rc;
}

int slam_batch_match(slam_ctx* c, void* stream, const void* d_query, int nq, int norm, double ratio,
                     int32_t* match_counts)
{
    BatchState& B = c ? c->batch : *(BatchState*)nullptr;
    if (!c || B.nframes <= 0 || nq < 0 || (nq > 0 && !d_query)) return SLAM_E_INVALID_ARG;
    if (!B.have_desc) return set_err(c, SLAM_E_INVALID_ARG, "the batch holds keypoints only (slam_batch_fast)");
    if (int rc = async_guard(c)) return rc;
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const int nf = B.nframes;
    int max_nt = 1;
    for (int f = 0; f < nf; f++) max_nt = std::max(max_nt, B.kp_counts[f]);
    int launched = 0;
    int rc = batch_match_enqueue(c, s, nf, B.matcher, d_query, nq, norm, ratio, max_nt, &launched);
    if (rc) return rc;
    if (!launched) {
        if (match_counts) for (int f = 0; f < nf; f++) match_counts[f] = 0;
        return SLAM_OK;
    }
    if (match_counts) {
        int32_t* rb = (int32_t*)readback(c, (size_t)nf * 4);
        if (!rb) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
        SLAM_HIP(c, hipMemcpyAsync(rb, c->match_cnt.p, (size_t)nf * 4, hipMemcpyDeviceToHost, s));
        rc = stream_sync(c, s, true);
        if (rc) return rc;
        std::memcpy(match_counts, rb, (size_t)nf * 4);
    }
    return SLAM_OK;
}

int slam_batch_extract_match(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                             int threshold, int matcher, const void* d_query, int nq, int norm, double ratio,
                             int32_t* kp_counts, int32_t* match_counts)
{
    return slam_batch_extract_match_ev(c, stream, d_frames, nframes, w, h, threshold, matcher, d_query, nq, norm,
                                       ratio, nullptr, kp_counts, match_counts);
}

int slam_batch_extract_match_ev(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                                int threshold, int matcher, const void* d_query, int nq, int norm, double ratio,
                                void* query_ready, int32_t* kp_counts, int32_t* match_counts)
{
    if (!c || !d_frames || nframes <= 0 || w <= 0 || h <= 0 || nq < 0 || (nq > 0 && !d_query))
        return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    if (w > 4096) return set_err(c, SLAM_E_UNSUPPORTED, "width > 4096");
    BatchState& B = c->batch;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // the first batch (no size estimate yet): the two calls, with their host sync
    // in between (ORB's matcher expansion is written by orb_desc itself, so ORB
    // queues its kNN behind the extraction like SIFT)
    if (B.est_max_nt <= 0 || B.w != w || B.h != h) {
        int rc = slam_batch_extract(c, stream, d_frames, nframes, w, h, threshold, matcher, kp_counts);
        if (rc) return rc;
        if (query_ready) SLAM_HIP(c, hipStreamWaitEvent(s, (hipEvent_t)query_ready, 0));
        return slam_batch_match(c, stream, d_query, nq, norm, ratio, match_counts);
    }
    SLAM_HIP(c, hipSetDevice(c->device));
    int cap = 0;
    int rc = batch_extract_enqueue(c, s, d_frames, nframes, w, h, threshold, matcher, &cap);
    if (rc) return rc;
    // only the kNN reads the query set: the extraction above is queued before
    // the wait, so it overlaps the query's producer (an RCCL broadcast)
    if (query_ready) SLAM_HIP(c, hipStreamWaitEvent(s, (hipEvent_t)query_ready, 0));
    // the kNN launch is sized on the previous batch's largest frame (+25 %): it
    // reads each frame's actual (capacity-clipped) count from the device frame
    // table, so only the packed-key split bound depends on the estimate
    const int est = B.est_max_nt + B.est_max_nt / 4 + 64;
    int launched = 0;
    rc = batch_match_enqueue(c, s, nframes, matcher, d_query, nq, norm, ratio, est, &launched);
    if (rc) return rc;
    // frame table, total and match counts: one read-back, one sync
    const size_t bi = sizeof(int4) * (nframes + 1);
    char* rb = (char*)readback(c, bi + (size_t)nframes * 4);
    if (!rb) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    int4* info = (int4*)rb;
    int32_t* mc = (int32_t*)(rb + bi);
    SLAM_HIP(c, hipMemcpyAsync(info, c->frame_info.p, sizeof(int4) * nframes, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(info + nframes, c->misc.p, sizeof(int), hipMemcpyDeviceToHost, s));
    if (launched) SLAM_HIP(c, hipMemcpyAsync(mc, c->match_cnt.p, (size_t)nframes * 4, hipMemcpyDeviceToHost, s));
    rc = stream_sync(c, s, true);
    if (rc) return rc;
    const bool matched = B.have_matches;
    rc = batch_extract_commit(c, s, info, nframes, w, h, matcher, cap, kp_counts);
    if (rc) return rc;
    B.have_matches = matched;
    // a frame larger than the split bound allows (packed keys hold split_rows_for's index bits
    // per split): the speculative match is discarded and redone at its size
    const int split_rows = split_rows_for(norm_for(matcher, norm));
    if (launched && (B.est_max_nt + launched - 1) / launched > split_rows)
        return slam_batch_match(c, stream, d_query, nq, norm, ratio, match_counts);
    if (match_counts) {
        if (launched) std::memcpy(match_counts, mc, (size_t)nframes * 4);
        else for (int f = 0; f < nframes; f++) match_counts[f] = 0;
    }
    return SLAM_OK;
}

// ---- asynchronous batch: the three halves of slam_batch_extract_match ----

int slam_batch_extract_async(slam_ctx* c, void* stream, const uint8_t* d_frames, int nframes, int w, int h,
                             int threshold, int matcher)
{
    if (!c || !d_frames || nframes <= 0 || w <= 0 || h <= 0) return SLAM_E_INVALID_ARG;
    if (int rc = async_guard(c)) return rc;
    if (matcher < 0 || matcher > 2) return set_err(c, SLAM_E_BAD_MATCHER, "invalid matcher type");
    if (w > 4096) return set_err(c, SLAM_E_UNSUPPORTED, "width > 4096");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const size_t need = sizeof(int4) * (nframes + 1) + (size_t)nframes * 4;
    if (c->h_async_bytes < need) {
        if (c->h_async) (void)hipHostFree(c->h_async);
        c->h_async = nullptr;
        c->h_async_bytes = 0;
        const size_t want = (need + 65535) & ~(size_t)65535;
        SLAM_HIP(c, hipHostMalloc(&c->h_async, want, hipHostMallocDefault));
        c->h_async_bytes = want;
    }
    int cap = 0;
    int rc = batch_extract_enqueue(c, s, d_frames, nframes, w, h, threshold, matcher, &cap);
    if (rc) return rc;
    int4* info = static_cast<int4*>(c->h_async);
    SLAM_HIP(c, hipMemcpyAsync(info, c->frame_info.p, sizeof(int4) * nframes, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipMemcpyAsync(info + nframes, c->misc.p, sizeof(int), hipMemcpyDeviceToHost, s));
    auto& A = c->async;
    A = slam_ctx::Async();
    A.state = 1;
    A.s = s;
    A.nframes = nframes; A.w = w; A.h = h; A.matcher = matcher; A.cap = cap;
    return SLAM_OK;
}

namespace {
// the queued extraction's host batch state (after a wait on its stream)
int async_commit(slam_ctx* c, int32_t* kp_counts)
{
    auto& A = c->async;
    if (A.committed) {
        if (kp_counts)
            for (int f = 0; f < A.nframes; f++) kp_counts[f] = c->batch.kp_counts_raw[f];
        return SLAM_OK;
    }
    const bool matched = c->batch.have_matches;
    int rc = batch_extract_commit(c, A.s, static_cast<const int4*>(c->h_async), A.nframes, A.w, A.h, A.matcher,
                                  A.cap, kp_counts);
    if (rc) return rc;
    c->batch.have_matches = matched;
    A.committed = true;
    return SLAM_OK;
}
}  // namespace

int slam_batch_match_async(slam_ctx* c, const void* d_query, int nq, int norm, double ratio, void* query_ready)
{
    if (!c || nq < 0 || (nq > 0 && !d_query)) return SLAM_E_INVALID_ARG;
    auto& A = c->async;
    if (A.state != 1) return set_err(c, SLAM_E_INVALID_ARG, "no queued extraction to match (slam_batch_extract_async)");
    SLAM_HIP(c, hipSetDevice(c->device));
    BatchState& B = c->batch;
    hipStream_t s = A.s;
    int rc = 0;
    int max_nt;
    if (B.est_max_nt <= 0 || B.w != A.w || B.h != A.h) {
        // a first batch has no size estimate: the extraction is taken first (one
        // wait), then matched at its size
        if ((rc = stream_sync(c, s, true))) return rc;
        if ((rc = async_commit(c, nullptr))) return rc;
        max_nt = 1;
        for (int f = 0; f < A.nframes; f++) max_nt = std::max(max_nt, B.kp_counts[f]);
    } else {
        max_nt = B.est_max_nt + B.est_max_nt / 4 + 64;   // as slam_batch_extract_match_ev
    }
    if (query_ready) SLAM_HIP(c, hipStreamWaitEvent(s, (hipEvent_t)query_ready, 0));
    int launched = 0;
    if ((rc = batch_match_enqueue(c, s, A.nframes, A.matcher, d_query, nq, norm, ratio, max_nt, &launched))) return rc;
    if (launched) {
        int32_t* mc = reinterpret_cast<int32_t*>(static_cast<char*>(c->h_async) + sizeof(int4) * (A.nframes + 1));
        SLAM_HIP(c, hipMemcpyAsync(mc, c->match_cnt.p, (size_t)A.nframes * 4, hipMemcpyDeviceToHost, s));
    }
    A.state = 2;
    A.launched = launched;
    A.norm = norm;
    A.nq = nq;
    A.ratio = ratio;
    A.query = d_query;
    return SLAM_OK;
}

int slam_batch_finish(slam_ctx* c, int32_t* kp_counts, int32_t* match_counts)
{
    if (!c) return SLAM_E_INVALID_ARG;
    auto& A = c->async;
    if (A.state == 0) return set_err(c, SLAM_E_INVALID_ARG, "no asynchronous batch in flight");
    int rc = stream_sync(c, A.s, true);
    if (rc) { A = slam_ctx::Async(); return rc; }
    const int state = A.state;
    BatchState& B = c->batch;
    rc = async_commit(c, kp_counts);       // keeps the queued match's state across the republish
    if (rc) { A = slam_ctx::Async(); return rc; }
    const slam_ctx::Async done = A;
    A = slam_ctx::Async();                 // the buffers are the caller's again
    if (state == 1) return SLAM_OK;        // extraction only
    // a frame larger than the split bound allows (packed keys hold split_rows_for's index bits
    // per split): the speculative match is discarded and redone at its size
    const int split_rows = split_rows_for(norm_for(done.matcher, done.norm));
    if (done.launched && (B.est_max_nt + done.launched - 1) / done.launched > split_rows)
        return slam_batch_match(c, done.s, done.query, done.nq, done.norm, done.ratio, match_counts);
    if (match_counts) {
        const int32_t* mc =
            reinterpret_cast<const int32_t*>(static_cast<const char*>(c->h_async) + sizeof(int4) * (done.nframes + 1));
        if (done.launched) std::memcpy(match_counts, mc, (size_t)done.nframes * 4);
        else for (int f = 0; f < done.nframes; f++) match_counts[f] = 0;
    }
    return SLAM_OK;
}

void* slam_context_stream(slam_ctx* c) { return c ? (void*)c->stream : nullptr; }

int slam_batch_fast_reused(const slam_ctx* c) { return c && c->fast_reused ? 1 : 0; }

int slam_batch_counts(slam_ctx* c, int32_t* raw_counts, int32_t* desc_counts, int cap)
{
    if (!c || cap < 0) return SLAM_E_INVALID_ARG;
    const BatchState& B = c->batch;
    if (cap < B.nframes) return set_err(c, SLAM_E_CAPACITY, "count arrays shorter than the batch");
    for (int f = 0; f < B.nframes; f++) {
        if (raw_counts) raw_counts[f] = B.kp_counts_raw[f];
        if (desc_counts) desc_counts[f] = B.kp_counts[f];
    }
    return B.nframes;
}

int slam_batch_export_desc(slam_ctx* c, void* stream, int frame, void* d_dst, int* n)
{
    if (!c || !d_dst || !n || frame < 0 || frame >= c->batch.nframes) return SLAM_E_INVALID_ARG;
    if (!c->batch.have_desc) return set_err(c, SLAM_E_INVALID_ARG, "the batch holds keypoints only (slam_batch_fast)");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const BatchState& B = c->batch;
    const int off = B.kp_offsets[frame], cnt = B.kp_counts[frame];
    *n = cnt;
    uint8_t* dst = (uint8_t*)d_dst;
    if (B.matcher == SLAM_ORB_BF) {
        SLAM_HIP(c, hipMemcpyAsync(dst, c->desc_exp.as<uint8_t>() + (size_t)off * kOrbExpBytes, (size_t)cnt * kOrbExpBytes,
                                   hipMemcpyDeviceToDevice, s));
    } else {
        SLAM_HIP(c, hipMemcpyAsync(dst, c->desc_u8.as<uint8_t>() + (size_t)off * 128, (size_t)cnt * 128,
                                   hipMemcpyDeviceToDevice, s));
        SLAM_HIP(c, hipMemcpyAsync(dst + (size_t)cnt * 128, c->desc_norm.as<int32_t>() + off, (size_t)cnt * 4,
                                   hipMemcpyDeviceToDevice, s));
    }
    return SLAM_OK;
}

int slam_batch_get_keypoints(slam_ctx* c, int frame, slam_keypoint* out, int cap, int* n)
{
    if (!c || !n || frame < 0 || frame >= c->batch.nframes) return SLAM_E_INVALID_ARG;
    const int cnt = c->batch.kp_counts[frame];
    *n = cnt;
    if (cnt > cap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    SLAM_HIP(c, hipSetDevice(c->device));
    SLAM_HIP(c, hipStreamSynchronize(c->stream));
    SLAM_HIP(c, hipMemcpy(out, c->kps.as<slam_keypoint>() + c->batch.kp_offsets[frame], (size_t)cnt * sizeof(slam_keypoint),
                          hipMemcpyDeviceToHost));
    return SLAM_OK;
}

int slam_batch_get_descriptors(slam_ctx* c, int frame, void* out, int cap, int* n)
{
    if (!c || !n || frame < 0 || frame >= c->batch.nframes) return SLAM_E_INVALID_ARG;
    const BatchState& B = c->batch;
    if (!B.have_desc) return set_err(c, SLAM_E_INVALID_ARG, "the batch holds keypoints only (slam_batch_fast)");
    const int cnt = B.kp_counts[frame], off = B.kp_offsets[frame];
    *n = cnt;
    if (cnt > cap) return set_err(c, SLAM_E_CAPACITY, "descriptor buffer too small");
    SLAM_HIP(c, hipSetDevice(c->device));
    SLAM_HIP(c, hipStreamSynchronize(c->stream));
    if (B.matcher == SLAM_ORB_BF) {
        SLAM_HIP(c, hipMemcpy(out, c->desc_u8.as<uint8_t>() + (size_t)off * 32, (size_t)cnt * 32, hipMemcpyDeviceToHost));
    } else {
        std::vector<uint8_t> u((size_t)cnt * 128);
        SLAM_HIP(c, hipMemcpy(u.data(), c->desc_u8.as<uint8_t>() + (size_t)off * 128, u.size(), hipMemcpyDeviceToHost));
        float* o = (float*)out;
        for (size_t i = 0; i < u.size(); i++) o[i] = (float)u[i];
    }
    return SLAM_OK;
}

int slam_batch_get_result(slam_ctx* c, int frame, slam_keypoint* kps, int kcap, int* nk, slam_dmatch* matches,
                          int mcap, int* nm)
{
    if (!c || !nk || !nm || frame < 0 || frame >= c->batch.nframes || !c->batch.have_matches)
        return SLAM_E_INVALID_ARG;
    const BatchState& B = c->batch;
    const int cntk = B.kp_counts[frame], nq = B.matched_nq;
    *nk = cntk;
    *nm = 0;
    if (cntk > kcap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    // the frame's compacted matches, its keypoints and the match count land in
    // the pinned readback buffer behind one sync (the per-item getters take three)
    const size_t kb = (size_t)cntk * sizeof(slam_keypoint), mb = (size_t)nq * sizeof(slam_dmatch);
    char* rb = static_cast<char*>(readback(c, 64 + kb + mb));
    if (!rb) return set_err(c, SLAM_E_HIP, "pinned readback allocation failed");
    int32_t* cnt_dev = c->match_cnt.as<int32_t>() + B.nframes;
    if (nq > 0) {
        SLAM_HIP(c, c->match_out.ensure(mb));
        const size_t o = (size_t)frame * nq;
        SLAM_HIP(c, launch_compact(c, s, c->match_rec.as<slam_dmatch>() + o, c->match_flag.as<uint8_t>() + o, nq, 1,
                                   c->match_out.as<slam_dmatch>(), cnt_dev, nq));
        SLAM_HIP(c, hipMemcpyAsync(rb, cnt_dev, 4, hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipMemcpyAsync(rb + 64 + kb, c->match_out.p, mb, hipMemcpyDeviceToHost, s));
    } else {
        *reinterpret_cast<int32_t*>(rb) = 0;
    }
    if (kb)
        SLAM_HIP(c, hipMemcpyAsync(rb + 64, c->kps.as<slam_keypoint>() + B.kp_offsets[frame], kb, hipMemcpyDeviceToHost, s));
    int rc = stream_sync(c, s, true);
    if (rc) return rc;
    const int cntm = *reinterpret_cast<const int32_t*>(rb);
    *nm = cntm;
    if (kb) std::memcpy(kps, rb + 64, kb);
    if (cntm > mcap) return set_err(c, SLAM_E_CAPACITY, "match buffer too small");
    if (cntm) std::memcpy(matches, rb + 64 + kb, (size_t)cntm * sizeof(slam_dmatch));
    return SLAM_OK;
}

int slam_batch_result_begin(slam_ctx* c, int frame)
{
    if (!c || frame < 0 || frame >= c->batch.nframes || !c->batch.have_matches) return SLAM_E_INVALID_ARG;
    const BatchState& B = c->batch;
    const int cntk = B.kp_counts[frame], nq = B.matched_nq;
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    // the same queue as slam_batch_get_result, into the context's own pinned
    // buffer (not the shared readback space: later calls reuse that before
    // this one is taken), and an event instead of a sync
    const size_t kb = (size_t)cntk * sizeof(slam_keypoint), mb = (size_t)nq * sizeof(slam_dmatch);
    if (c->win_pending) {
        // the previous result is still in flight: it must land before the buffer is reused
        SLAM_HIP(c, hipEventSynchronize(c->ev_win));
        c->win_pending = 0;
    }
    if (c->h_win_bytes < 64 + kb + mb) {
        if (c->h_win) (void)hipHostFree(c->h_win);
        c->h_win = nullptr;
        c->h_win_bytes = 0;
        const size_t want = (64 + kb + mb + 65535) & ~(size_t)65535;
        SLAM_HIP(c, hipHostMalloc(&c->h_win, want, hipHostMallocDefault));
        c->h_win_bytes = want;
    }
    if (!c->ev_win) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_win, hipEventDisableTiming));
    char* rb = static_cast<char*>(c->h_win);
    int32_t* cnt_dev = c->match_cnt.as<int32_t>() + B.nframes;
    if (nq > 0) {
        SLAM_HIP(c, c->match_out.ensure(mb));
        const size_t o = (size_t)frame * nq;
        SLAM_HIP(c, launch_compact(c, s, c->match_rec.as<slam_dmatch>() + o, c->match_flag.as<uint8_t>() + o, nq, 1,
                                   c->match_out.as<slam_dmatch>(), cnt_dev, nq));
        SLAM_HIP(c, hipMemcpyAsync(rb, cnt_dev, 4, hipMemcpyDeviceToHost, s));
        SLAM_HIP(c, hipMemcpyAsync(rb + 64 + kb, c->match_out.p, mb, hipMemcpyDeviceToHost, s));
    } else {
        *reinterpret_cast<int32_t*>(rb) = 0;
    }
    if (kb)
        SLAM_HIP(c, hipMemcpyAsync(rb + 64, c->kps.as<slam_keypoint>() + B.kp_offsets[frame], kb, hipMemcpyDeviceToHost, s));
    SLAM_HIP(c, hipEventRecord(c->ev_win, s));
    c->win_pending = 1;
    c->win_nk = cntk;
    c->win_kb = kb;
    return SLAM_OK;
}

int slam_batch_result_end(slam_ctx* c, slam_keypoint* kps, int kcap, int* nk, slam_dmatch* matches, int mcap, int* nm)
{
    if (!c || !nk || !nm || !c->win_pending) return SLAM_E_INVALID_ARG;
    *nk = c->win_nk;
    *nm = 0;
    for (;;) {
        const hipError_t e = hipEventQuery(c->ev_win);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return set_err(c, SLAM_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
    }
    const char* rb = static_cast<const char*>(c->h_win);
    const size_t kb = c->win_kb;
    const int cntm = *reinterpret_cast<const int32_t*>(rb);
    *nm = cntm;
    // a capacity error keeps the result pending: the caller retries with the reported sizes
    if (c->win_nk > kcap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    if (cntm > mcap) return set_err(c, SLAM_E_CAPACITY, "match buffer too small");
    c->win_pending = 0;
    if (kb) std::memcpy(kps, rb + 64, kb);
    if (cntm) std::memcpy(matches, rb + 64 + kb, (size_t)cntm * sizeof(slam_dmatch));
    return SLAM_OK;
}

int slam_batch_result_dev(slam_ctx* c, void* stream, int frame, void* d_matches, int nm, void* d_kps, int kcap)
{
    if (!c || frame < 0 || frame >= c->batch.nframes || !c->batch.have_matches || nm < 0 || kcap < 0)
        return SLAM_E_INVALID_ARG;
    const BatchState& B = c->batch;
    const int cntk = B.kp_counts[frame], nq = B.matched_nq;
    if (cntk > kcap) return set_err(c, SLAM_E_CAPACITY, "keypoint buffer too small");
    if (nm > nq) return set_err(c, SLAM_E_INVALID_ARG, "more matches than queries");
    if ((cntk > 0 && !d_kps) || (nm > 0 && !d_matches)) return SLAM_E_INVALID_ARG;
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    const int rc = win_guard(c, s);   // match_out may still feed a queued slam_batch_result_begin
    if (rc) return rc;
    if (nq > 0 && nm > 0) {
        // the ratio-test survivors in query order (the compaction of slam_batch_get_matches), then
        // the caller's nm of them: never more than the destination holds
        const size_t mb = (size_t)nq * sizeof(slam_dmatch);
        SLAM_HIP(c, c->match_out.ensure(mb));
        const size_t o = (size_t)frame * nq;
        SLAM_HIP(c, launch_compact(c, s, c->match_rec.as<slam_dmatch>() + o, c->match_flag.as<uint8_t>() + o, nq, 1,
                                   c->match_out.as<slam_dmatch>(), c->match_cnt.as<int32_t>() + B.nframes, nq));
        SLAM_HIP(c, hipMemcpyAsync(d_matches, c->match_out.p, (size_t)nm * sizeof(slam_dmatch),
                                   hipMemcpyDeviceToDevice, s));
    }
    if (cntk > 0)
        SLAM_HIP(c, hipMemcpyAsync(d_kps, c->kps.as<slam_keypoint>() + B.kp_offsets[frame],
                                   (size_t)cntk * sizeof(slam_keypoint), hipMemcpyDeviceToDevice, s));
    if (s != c->stream) {
        // the compaction and copies read kps / match_* and write match_out on the
        // caller's stream: later work on the context stream (a result_begin, a
        // get_matches, the next batch) rewrites those buffers, so it waits for them
        if (!c->ev_rdev) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_rdev, hipEventDisableTiming));
        SLAM_HIP(c, hipEventRecord(c->ev_rdev, s));
        SLAM_HIP(c, hipStreamWaitEvent(c->stream, c->ev_rdev, 0));
    }
    return SLAM_OK;
}

int slam_order_after(slam_ctx* c, void* waiter, void* stream)
{
    if (!c) return SLAM_E_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (s == (hipStream_t)waiter) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    if (!c->ev_order) SLAM_HIP(c, hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming));
    SLAM_HIP(c, hipEventRecord(c->ev_order, s));
    SLAM_HIP(c, hipStreamWaitEvent((hipStream_t)waiter, c->ev_order, 0));
    return SLAM_OK;
}

int slam_order_after_stage(slam_ctx* c, void* waiter, int stage)
{
    if (!c || stage < SLAM_STAGE_DESC_START || stage > SLAM_STAGE_DESC_END) return SLAM_E_INVALID_ARG;
    if (!c->stage_recorded) return set_err(c, SLAM_E_INVALID_ARG, "no extraction queued on this context yet");
    SLAM_HIP(c, hipSetDevice(c->device));
    SLAM_HIP(c, hipStreamWaitEvent((hipStream_t)waiter, c->ev_stage[stage], 0));
    return SLAM_OK;
}

int slam_last_sift_kernel(const slam_ctx* c) { return c ? c->last_sift_kernel : SLAM_E_INVALID_ARG; }

int slam_batch_get_matches(slam_ctx* c, int frame, slam_dmatch* out, int cap, int* n)
{
    if (!c || !n || frame < 0 || frame >= c->batch.nframes || !c->batch.have_matches) return SLAM_E_INVALID_ARG;
    const int nq = c->batch.matched_nq;
    *n = 0;
    if (nq == 0) return SLAM_OK;
    SLAM_HIP(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    SLAM_HIP(c, c->match_out.ensure((size_t)nq * sizeof(slam_dmatch)));
    const size_t o = (size_t)frame * nq;
    int32_t* cnt_dev = c->match_cnt.as<int32_t>() + c->batch.nframes;
    SLAM_HIP(c, launch_compact(c, s, c->match_rec.as<slam_dmatch>() + o, c->match_flag.as<uint8_t>() + o, nq, 1,
                               c->match_out.as<slam_dmatch>(), cnt_dev, nq));
    int cnt = 0;
    SLAM_HIP(c, hipMemcpyAsync(&cnt, cnt_dev, 4, hipMemcpyDeviceToHost, s));
    int rc = stream_sync(c, s);
    if (rc) return rc;
    *n = cnt;
    if (cnt > cap) return set_err(c, SLAM_E_CAPACITY, "match buffer too small");
    SLAM_HIP(c, hipMemcpy(out, c->match_out.p, (size_t)cnt * sizeof(slam_dmatch), hipMemcpyDeviceToHost));
    return SLAM_OK;
}

int slam_set_option(slam_ctx* c, int option, int value)
{
    if (!c) return SLAM_E_INVALID_ARG;
    switch (option) {
    case SLAM_OPT_SIFT_KERNEL:
        if (value < SLAM_SIFT_KERNEL_AUTO || value > SLAM_SIFT_KERNEL_COLW)
            return set_err(c, SLAM_E_INVALID_ARG, "unknown SIFT kernel");
        c->opt_sift_kernel = value;
        c->sift_band_valid = false;   // rebuilt (or refused) by the next prepare
        c->sift_cols_valid = false;
        c->sift_colw_valid = false;
        c->sift_tab_valid = false;
        return SLAM_OK;
    case SLAM_OPT_PNP_SUMS:
        if (value != SLAM_PNP_SUMS_ORDERED && value != SLAM_PNP_SUMS_PAIRWISE)
            return set_err(c, SLAM_E_INVALID_ARG, "unknown PnP sum mode");
        c->opt_pnp_sums = value;
        return SLAM_OK;
    case SLAM_OPT_SIFT_BAND_SPLIT:
        if (value < SLAM_BAND_SPLIT_OFF || value > SLAM_BAND_SPLIT_ALL4)
            return set_err(c, SLAM_E_INVALID_ARG, "unknown band split mode");
        c->opt_band_split = value;
        return SLAM_OK;
    case SLAM_OPT_FAST_REUSE:
        if (value != 0 && value != 1) return set_err(c, SLAM_E_INVALID_ARG, "SLAM_OPT_FAST_REUSE takes 0 or 1");
        c->opt_fast_reuse = value;
        return SLAM_OK;
    default:
        return set_err(c, SLAM_E_INVALID_ARG, "unknown option");
    }
}

int slam_profile_enable(slam_ctx* c, int on)
{
    if (!c) return SLAM_E_INVALID_ARG;
    c->prof_on = on != 0;
    for (auto& f : c->prof) f.used = 0;
    return SLAM_OK;
}

int slam_profile_read(slam_ctx* c, int family, double* avg_ms, int* launches)
{
    if (!c || family < 0 || family >= 8 || !avg_ms || !launches) return SLAM_E_INVALID_ARG;
    ProfFamily& f = c->prof[family];
    *avg_ms = 0;
    *launches = f.used;
    if (f.used == 0) return SLAM_OK;
    SLAM_HIP(c, hipEventSynchronize(f.ev[2 * f.used - 1]));
    double sum = 0;
    for (int i = 0; i < f.used; i++) {
        float ms = 0;
        SLAM_HIP(c, hipEventElapsedTime(&ms, f.ev[2 * i], f.ev[2 * i + 1]));
        sum += ms;
    }
    *avg_ms = sum / f.used;
    f.used = 0;
    return SLAM_OK;
}

int slam_ba(slam_ctx* c, double* K4, int nframes, double* ext6, int npoints, double* pts3, int nobs,
            const int32_t* of, const int32_t* op, const double* oxy, int loss, double a, int max_iters,
            slam_ba_summary* sum)
{
    if (!c || !K4 || !sum || nframes <= 0 || !ext6 || npoints < 0 || nobs < 0) return SLAM_E_INVALID_ARG;
    if (nobs > 0 && (!of || !op || !oxy || !pts3)) return SLAM_E_INVALID_ARG;
    for (int o = 0; o < nobs; o++)
        if (of[o] < 0 || of[o] >= nframes || op[o] < 0 || op[o] >= npoints) return SLAM_E_INVALID_ARG;
    SLAM_HIP(c, hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    int rc = ba_solve(c, K4, nframes, ext6, npoints, pts3, nobs, of, op, oxy, loss, a, max_iters, sum);
    sum->total_time_in_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

}  // extern "C"
