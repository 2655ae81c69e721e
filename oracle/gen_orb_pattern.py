"""Regenerate oracle/orb_pattern.h from scikit-image's ORB position table (data only).

The table equals OpenCV's bit_pattern_31_ used by cv::ORB (reference call site
src/mainModule/featureMatching/featureMatchingCPU.cpp:60).  Run in the build
container: python oracle/gen_orb_pattern.py
"""
import numpy as np

SRC = "/opt/conda/lib/python3.9/site-packages/skimage/feature/orb_descriptor_positions.txt"

def main():
    p = np.loadtxt(SRC).astype(int)
    assert p.shape == (256, 4)
    body = "\n".join("    %d,%d, %d,%d," % tuple(r) for r in p)
    with open(__file__.replace("gen_orb_pattern.py", "orb_pattern.h")) as f:
        cur = f.read()
    assert body in cur, "orb_pattern.h is stale"
    print("orb_pattern.h matches", SRC)

if __name__ == "__main__":
    main()
