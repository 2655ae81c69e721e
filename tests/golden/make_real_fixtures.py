"""Real-image parity fixtures from the photos the reference ships.

Provenance: /root/reference/docs/artifact/calibration/ (the reference repo's own
calibration photos: for_calib_1/*.JPG, 3264 x 2448 RGB; for_calib_2/*.jpg,
748 x 480 grayscale fisheye).  They are decoded here with PIL (12.2, build
container only) and stored as raw pixel arrays, so the tests need neither PIL
nor the reference tree; JPEG decoding happens once, in this script.

  real_vga.npz   bgr: 4 x 480 x 640 x 3 u8 centre-offset crops of for_calib_1
                 {1, 4, 7, 10}.JPG (RGB -> BGR channel order, as cv::imread
                 hands frames to the reference); gray: 2 x 480 x 748 u8
                 for_calib_2/Fisheye2_{1,2}.jpg (single-channel input path)
  real_1080p.npz bgr: 1 x 1080 x 1920 x 3 u8 crop of for_calib_1/2.JPG

Each file also holds the oracle's FAST-9 keypoint counts at thresholds 10 and
20 (`fast_counts`), regenerated here, which the CPU suite re-checks.
Run from the repo root:  python tests/golden/make_real_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
SRC = "/root/reference/docs/artifact/calibration"


def load_rgb(name):
    from PIL import Image
    return np.asarray(Image.open(os.path.join(SRC, name)).convert("RGB"))


def load_gray(name):
    from PIL import Image
    return np.asarray(Image.open(os.path.join(SRC, name)).convert("L"))


def crop(img, w, h, fx=0.5, fy=0.5):
    H, W = img.shape[:2]
    x0 = int((W - w) * fx)
    y0 = int((H - h) * fy)
    return np.ascontiguousarray(img[y0:y0 + h, x0:x0 + w])


def fast_counts(images):
    import oracle_ffi as O
    return np.array([[len(O.fast(im, t, True)) for t in (10, 20)] for im in images], np.int32)


def main():
    vga = [crop(load_rgb(f"for_calib_1/{i}.JPG"), 640, 480, 0.45 + 0.03 * k, 0.5)[..., ::-1]
           for k, i in enumerate((1, 4, 7, 10))]
    vga = np.ascontiguousarray(np.stack(vga))
    gray = np.stack([load_gray(f"for_calib_2/Fisheye2_{i}.jpg") for i in (1, 2)])
    np.savez_compressed(os.path.join(HERE, "real_vga.npz"), bgr=vga, gray=gray,
                        fast_counts=fast_counts(list(vga) + list(gray)))
    hd = np.ascontiguousarray(crop(load_rgb("for_calib_1/2.JPG"), 1920, 1080)[..., ::-1])[None]
    np.savez_compressed(os.path.join(HERE, "real_1080p.npz"), bgr=hd, fast_counts=fast_counts(list(hd)))
    for f in ("real_vga.npz", "real_1080p.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
