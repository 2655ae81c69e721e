"""slamhip: MI355X (gfx950) implementation of the FIT-2023-SLAM-indoor
extract -> match -> windowed-BA hot path, behind the reference's interface.

    import slamhip
    kps = slamhip.fastExtractor(frame, threshold=31)
    kps, desc = slamhip.extractDescriptor(frame, kps, slamhip.SIFT_FLANN)

The compute runs in libslamhip.so (hand-written HIP kernels); this package is
the host-side mirror of the reference's mainModule headers plus the
device-resident candidate scan (slamhip.batch).
"""
from ._lib import (DMATCH_DTYPE, EMPTY_BATCH, FRAME_NOT_FOUND, KEYPOINT_DTYPE, LOSS_ARCTAN, LOSS_CAUCHY,
                   LOSS_HUBER, LOSS_NONE, LOSS_TRIVIAL, LOSS_TUKEY, NORM_DEFAULT, NORM_HAMMING, NORM_L1, NORM_L2,
                   ORB_BF, SIFT_BF, SIFT_FLANN, TYPE_5_8, TYPE_7_12, TYPE_9_16, SIGNATURES, SlamError, lib)
from .api import (Context, GlobalData, MatcherTypeError, TemporalImageData, ba_rmse, bundle_adjust_arrays,
                  bundleAdjustment, default_context, extractDescriptor, fastExtractor, getGoodMatches,
                  estimateTransformation, reconstruct, siftDetectAndCompute, siftDetectAndComputeBatch, SiftBatch, solvePnPRansac,
                  getMatcherTypeIndex, knnMatch2, loss_from_config, matchFeatures, matchFramesPairFeatures,
                  rodrigues_to_matrix, rodrigues_to_vector, selectGoodFrame, synth_frames,
                  SYNTH_DRIFT, SYNTH_STEADY, synth_frames_dev)
from .config import ConfigError, ConfigService, reference_example

__all__ = [n for n in dir() if not n.startswith("_")]
