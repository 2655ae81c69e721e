"""Occupancy guard for the step's hot kernels (CPU: compiles, no GPU).

The kernels' speed depends on how many waves per SIMD their register and LDS
budgets allow, and an innocent-looking edit can cost a wave: round 3's
Hamming-key change kept the L2 kernel's per-row keys live across its MFMAs,
126 -> 168 VGPRs, 4 -> 3 waves per SIMD, knn_mfma 1.72 -> 2.09 ms per
210-frame step.  This compiles the sources device-only with the compiler's
resource-usage remarks and checks each hot kernel's occupancy against the
budget its design assumes.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "slam-indoor-code_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# (source, mangled-name fragment, minimum waves per SIMD)
BUDGETS = [
    ("knn.hip", "knn_mfma_pkILi128ELb0ELi2ELi4E", 4),    # SIFT L2, int8 MFMA (126 VGPRs)
    ("knn.hip", "knn_mfma_pkILi128ELb1ELi2ELi4E", 4),    # ORB Hamming, FP4 MFMA
    ("sift_colw.hip", "sift_desc_colw", 2),              # column per wave (forced kernel): one 8-wave block per CU (LDS)
    ("sift_band.hip", "sift_desc_bandILb1ELi2EE", 2),    # one 8-wave block per CU (LDS); frac + position plane
    ("sift_band.hip", "sift_desc_bandILb1ELi1EE", 2),    # obin stored per pixel
    ("sift_band.hip", "sift_desc_band4ILb1ELb1ELb1EE", 4),   # 16 keypoints per wave, LDS-DMA stage: two 8-wave blocks per CU
    ("sift_band.hip", "sift_desc_band4ILb1ELb1ELb0EE", 4),   # 16 keypoints per wave, register stage
    ("sift.hip", "sift_blur_gradILi2EE", 8),
    ("sift.hip", "sift_blur_gradILi1EE", 8),
    ("fast.hip", "fast_detectILi1ELi16EE", 8),
]


def _usage(src):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-munsafe-fp-atomics",
           "-I" + os.path.join(ROOT, "include"), "-x", "hip", "--cuda-device-only", "-c",
           os.path.join(CSRC, src), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = kernels.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.parametrize("src", sorted({b[0] for b in BUDGETS}))
def test_hot_kernel_occupancy(src):
    kernels = _usage(src)
    for s, frag, waves in BUDGETS:
        if s != src:
            continue
        hits = [v for k, v in kernels.items() if frag in k]
        assert hits, f"{frag} not found in {src}"
        for v in hits:
            assert v.get("Occupancy [waves/SIMD]", 0) >= waves, (frag, v)
            assert v.get("VGPRs Spill", 0) == 0, (frag, v)
