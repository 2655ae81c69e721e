"""What would a tolerance-mode SIFT descriptor change?  (diagnostics, CPU)

The reference's calcSIFTDescriptor sums every bin in raster sample order in f32;
sift_desc_band reproduces that order bit-exactly.  oracle/sift.c's diagnostic
variants relax it the ways a faster, non-bit-exact kernel would:
  1 the samples in reverse order (any other summation order, f32),
  2 fp16-rounded inputs (mag and the bin fractions to 11 significant bits: an
    f16-input MFMA formulation), f32 sums,
  3 f64 sums (order-free), rounded to f32.
On synthetic 1080p frames at the bench's FAST threshold: the element-exact
fraction and max |delta| against the reference, and whether the ratio-test
match counts (the batch search's selection input) stay identical.
usage: python scripts/diag/sift_tolerance.py [nframes]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "slam-indoor-code_amd"))
import oracle_ffi as O  # noqa: E402
import slamhip  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
O.oracle().orc_sift_set_variant.argtypes = [ctypes.c_int]
frames = slamhip.synth_frames(1920, 1080, 0, n + 1, seed=1234, path=slamhip.SYNTH_STEADY)
thr = 33
kps = [O.fast(f, thr, True) for f in frames]
res = {}
ref = []
for v in (0, 1, 2, 3):
    O.oracle().orc_sift_set_variant(v)
    ds = [O.sift(f, k) for f, k in zip(frames, kps)]
    O.oracle().orc_sift_set_variant(0)
    if v == 0:
        ref = ds
        counts0 = []
    d = np.concatenate([np.abs(a.astype(np.int32) - b.astype(np.int32)).ravel() for a, b in zip(ds, ref)])
    counts = []
    for i in range(1, n + 1):
        ri, rd = O.knn2(ds[0], ds[i], O.NORM_L2)
        counts.append(int(len(O.ratio(ri, rd, 0.7))))
    if v == 0:
        counts0 = counts
    res[v] = {"exact_frac": float((d == 0).mean()), "max_abs": int(d.max()), "frac_le1": float((d <= 1).mean()),
              "match_counts": counts, "match_counts_equal_ref": counts == counts0}
    print(v, json.dumps(res[v]), flush=True)
print(json.dumps({"keypoints_per_frame": [len(k) for k in kps], "variants": res}))
