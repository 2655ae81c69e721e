// Deterministic synthetic "indoor" sequence: the input the benchmark and the
// parity tests feed the hot path.  A textured planar scene --
// random axis-aligned rectangles (wall posters, furniture edges) with per-rect
// BGR colours over a smooth gradient -- viewed by a camera that translates,
// yaws (in-plane rotation) and moves forward (zoom) a little every frame;
// nearest-texel sampling plus hash noise in [-3, 3] per channel.  Rectangle
// corners give dense, repeatable FAST-9 corners; consecutive frames overlap
// heavily, so kNN + ratio matching finds thousands of correspondences.
// Pure integer / float host code: identical bytes on every x86-64 machine.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <algorithm>

#include <hip/hip_runtime.h>

#include "slamhip_internal.h"

namespace {

__host__ __device__ inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rect { int x0, y0, x1, y1; uint8_t b, g, r; };

struct World {
    int W, H;
    std::vector<uint8_t> px;   // W x H x 3
};

void build_world(World& wd, int fw, int fh, uint64_t seed)
{
    wd.W = fw * 2;
    wd.H = fh * 2;
    wd.px.assign((size_t)wd.W * wd.H * 3, 0);
    for (int y = 0; y < wd.H; y++)
        for (int x = 0; x < wd.W; x++) {
            uint8_t* p = &wd.px[((size_t)y * wd.W + x) * 3];
            p[0] = (uint8_t)(90 + (x * 60) / wd.W);
            p[1] = (uint8_t)(100 + (y * 50) / wd.H);
            p[2] = (uint8_t)(110 + ((x + y) * 40) / (wd.W + wd.H));
        }
    // rectangle density scales with area: ~1 rectangle per 420 px^2 of world
    long nrect = (long)wd.W * wd.H / 420;
    uint64_t s = seed * 0x2545F4914F6CDD1Dull + 17;
    for (long i = 0; i < nrect; i++) {
        uint64_t a = mix64(s + 4 * i), b = mix64(s + 4 * i + 1), c = mix64(s + 4 * i + 2);
        int w = 4 + (int)(a % 40), h = 4 + (int)((a >> 20) % 40);
        int x0 = (int)((b & 0xffffffff) % (uint64_t)wd.W), y0 = (int)((b >> 32) % (uint64_t)wd.H);
        Rect r{x0, y0, x0 + w < wd.W ? x0 + w : wd.W, y0 + h < wd.H ? y0 + h : wd.H,
               (uint8_t)(c & 255), (uint8_t)((c >> 8) & 255), (uint8_t)((c >> 16) & 255)};
        for (int y = r.y0; y < r.y1; y++) {
            uint8_t* p = &wd.px[((size_t)y * wd.W + r.x0) * 3];
            for (int x = r.x0; x < r.x1; x++, p += 3) { p[0] = r.b; p[1] = r.g; p[2] = r.r; }
        }
    }
}

// one frame's camera: world texel of pixel (x, y) = o + [cs -sn; sn cs] (p - c)
struct Cam { double cs, sn, ox, oy, cx, cy; uint64_t fseed; };

Cam camera(int w, int h, int worldW, int worldH, int k, uint64_t seed, int path)
{
    double s, th, ox, oy;
    if (path == SLAM_SYNTH_DRIFT) {
        // camera: forward motion (zoom-in 0.15 %/frame), yaw 0.25 deg/frame,
        // lateral drift (3, 1.5) px/frame in world texels.  The view zooms in
        // without bound, so the texture (and the FAST count) thins out along
        // the sequence: ~10.2k keypoints at frame 0, ~6.3k at frame 210 (1080p)
        s = 1.0 / (1.0 + 0.0015 * k);
        th = 0.25 * k * M_PI / 180.0;
        ox = worldW * 0.5 - 3.0 * k * 0.5 - w * 0.25;
        oy = worldH * 0.5 - 1.5 * k * 0.5 - h * 0.1;
    } else {
        // a bounded walk that stays inside the textured volume: the camera
        // sweeps a Lissajous loop of +-25 % x +-14 % of the frame size
        // (<= ~4 texels per frame), yaws +-4 deg and moves back and forth
        // +-2 % along its axis, so the texel density in view -- and with it
        // the FAST count at one threshold -- stays within a few per cent of
        // frame 0's along any number of frames (configs[1]: 10k +- 10 %)
        const double tau = 2.0 * M_PI;
        s = 1.0 + 0.02 * std::sin(tau * k / 251.0);
        th = 4.0 * M_PI / 180.0 * std::sin(tau * k / 307.0);
        ox = worldW * 0.5 + 0.25 * w * std::sin(tau * k / 401.0);
        oy = worldH * 0.5 + 0.14 * h * std::sin(tau * k / 263.0 + 1.0);
    }
    Cam c;
    c.cs = std::cos(th) * s;
    c.sn = std::sin(th) * s;
    c.ox = ox;
    c.oy = oy;
    c.cx = w * 0.5;
    c.cy = h * 0.5;
    c.fseed = mix64(seed ^ (0x51ED270B27E3C3A5ull * (uint64_t)(k + 1)));
    return c;
}

// std::lround (half away from zero) without the library: exact, the same on host and device
__host__ __device__ inline long round_away(double x)
{
    double t = trunc(x);
    if (fabs(x - t) >= 0.5) t += x < 0 ? -1.0 : 1.0;
    return (long)t;
}

// nearest texel + hash noise in [-3, 3] per channel (every double operation
// separate: no contraction, so host and device give the same bytes)
__host__ __device__ inline void synth_pixel(const uint8_t* world, int worldW, int worldH, const Cam& c, int x, int y,
                                            uint8_t* d)
{
    const double dx = x - c.cx, dy = y - c.cy;
    const double a = c.cs * dx, b = c.sn * dy, e = c.sn * dx, f = c.cs * dy;
    long u = round_away((c.ox + a) - b);
    long v = round_away((c.oy + e) + f);
    if (u < 0) u = 0;
    if (u >= worldW) u = worldW - 1;
    if (v < 0) v = 0;
    if (v >= worldH) v = worldH - 1;
    const uint8_t* p = world + ((size_t)v * worldW + u) * 3;
    const uint64_t n = mix64(c.fseed + (uint64_t)y * 0x100000001B3ull + (uint64_t)x);
    for (int ch = 0; ch < 3; ch++) {
        int nz = (int)((n >> (8 * ch)) & 7) - 3;     // [-3, 4]
        if (nz > 3) nz = 0;
        const int val = p[ch] + nz;
        d[ch] = (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
    }
}

__global__ __launch_bounds__(256) void synth_render(const uint8_t* world, int worldW, int worldH, const Cam* cams, int w,
                                                    int h, uint8_t* out)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
    if (x >= w) return;
    synth_pixel(world, worldW, worldH, cams[f], x, y, out + (((size_t)f * h + y) * w + x) * 3);
}

}  // namespace

extern "C" int slam_synth_sequence(int w, int h, int first, int count, uint64_t seed, int path, uint8_t* out)
{
    if (w < 16 || h < 16 || count < 0 || first < 0 || !out) return SLAM_E_INVALID_ARG;
    if (path != SLAM_SYNTH_DRIFT && path != SLAM_SYNTH_STEADY) return SLAM_E_INVALID_ARG;
    World wd;
    build_world(wd, w, h, seed);
    for (int f = 0; f < count; f++) {
        const Cam c = camera(w, h, wd.W, wd.H, first + f, seed, path);
        uint8_t* dst = out + (size_t)f * w * h * 3;
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) synth_pixel(wd.px.data(), wd.W, wd.H, c, x, y, dst + ((size_t)y * w + x) * 3);
    }
    return SLAM_OK;
}

extern "C" int slam_synth_frames(int w, int h, int first, int count, uint64_t seed, uint8_t* out)
{
    return slam_synth_sequence(w, h, first, count, seed, SLAM_SYNTH_DRIFT, out);
}

extern "C" int slam_synth_sequence_dev(slam_ctx* c, void* stream, int w, int h, int first, int count, uint64_t seed,
                                       int path, uint8_t* d_out)
{
    if (!c || w < 16 || h < 16 || count < 0 || first < 0 || (count > 0 && !d_out)) return SLAM_E_INVALID_ARG;
    if (path != SLAM_SYNTH_DRIFT && path != SLAM_SYNTH_STEADY) return SLAM_E_INVALID_ARG;
    if (count == 0) return SLAM_OK;
    if (hipSetDevice(c->device) != hipSuccess) return SLAM_E_HIP;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // the world texture: built on the host once per (size, seed), kept on the device
    if (!c->synth_world.p || c->synth_w != w || c->synth_h != h || c->synth_seed != seed) {
        World wd;
        build_world(wd, w, h, seed);
        if (c->synth_world.ensure(wd.px.size()) != hipSuccess) return SLAM_E_HIP;
        if (hipMemcpy(c->synth_world.p, wd.px.data(), wd.px.size(), hipMemcpyHostToDevice) != hipSuccess) return SLAM_E_HIP;
        c->synth_w = w;
        c->synth_h = h;
        c->synth_seed = seed;
    }
    std::vector<Cam> cams(count);
    for (int f = 0; f < count; f++) cams[f] = camera(w, h, 2 * w, 2 * h, first + f, seed, path);
    if (c->synth_cams.ensure(cams.size() * sizeof(Cam)) != hipSuccess) return SLAM_E_HIP;
    if (hipMemcpyAsync(c->synth_cams.p, cams.data(), cams.size() * sizeof(Cam), hipMemcpyHostToDevice, s) != hipSuccess)
        return SLAM_E_HIP;
    for (int f0 = 0; f0 < count; f0 += 65535) {
        const int n = std::min(count - f0, 65535);
        hipLaunchKernelGGL(synth_render, dim3((w + 255) / 256, h, n), dim3(256), 0, s, c->synth_world.as<uint8_t>(),
                           2 * w, 2 * h, c->synth_cams.as<Cam>() + f0, w, h, d_out + (size_t)f0 * w * h * 3);
    }
    if (hipGetLastError() != hipSuccess) return SLAM_E_HIP;
    // the camera table is host memory of this call: done before returning
    return hipStreamSynchronize(s) == hipSuccess ? SLAM_OK : SLAM_E_HIP;
}
