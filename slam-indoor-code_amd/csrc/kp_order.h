// The detector's host-side keypoint order (removeDuplicatedSorted's
// KeypointGreater) and its radix form.  Host-only C++ (no HIP): included by
// siftdet.hip and by tests/cpp/kp_order_test.cpp, which checks kp_order
// against std::sort with kp_less on the CPU.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/slamhip.h"

namespace slamhip {

// removeDuplicatedSorted's KeypointGreater
inline bool kp_less(const slam_keypoint& a, const slam_keypoint& b)
{
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    if (a.octave != b.octave) return a.octave > b.octave;
    return a.class_id > b.class_id;
}

// the KeypointGreater order of src[0 .. n) as (x, index) pairs: an LSD radix
// sort of x's order-preserving bits (three 11-bit passes, stable), then each
// run of equal x ordered by the full comparator -- the sequence std::sort with
// kp_less gives (keypoints that compare equal are identical in every field),
// at a tenth of its time on 8k keypoints
inline void kp_order(const slam_keypoint* src, int n, std::vector<std::pair<float, int>>& ord)
{
    ord.resize((size_t)n);
    if (n <= 0) return;
    std::vector<uint64_t> a((size_t)n), b((size_t)n);     // key << 32 | index
    for (int i = 0; i < n; i++) {
        uint32_t u;
        std::memcpy(&u, &src[i].x, 4);
        if (u == 0x80000000u) u = 0;                         // -0 sorts with +0
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        a[(size_t)i] = (uint64_t)u << 32 | (uint32_t)i;
    }
    constexpr int kBits = 11, kBuckets = 1 << kBits;
    std::vector<int> cnt(kBuckets);
    for (int pass = 0; pass < 3; pass++) {
        const int sh = 32 + pass * kBits;
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int i = 0; i < n; i++) cnt[(a[(size_t)i] >> sh) & (kBuckets - 1)]++;
        int run = 0;
        for (int d = 0; d < kBuckets; d++) { const int c = cnt[(size_t)d]; cnt[(size_t)d] = run; run += c; }
        for (int i = 0; i < n; i++) b[(size_t)cnt[(a[(size_t)i] >> sh) & (kBuckets - 1)]++] = a[(size_t)i];
        a.swap(b);
    }
    for (int i = 0; i < n; i++) {
        const int k = (int)(uint32_t)a[(size_t)i];
        ord[(size_t)i] = {src[k].x, k};
    }
    for (int i = 0; i < n;) {
        int j = i + 1;
        while (j < n && (a[(size_t)j] >> 32) == (a[(size_t)i] >> 32)) j++;
        if (j - i > 1)
            std::sort(ord.begin() + i, ord.begin() + j, [&](const std::pair<float, int>& u, const std::pair<float, int>& v) {
                return kp_less(src[u.second], src[v.second]);
            });
        i = j;
    }
}

}  // namespace slamhip
