"""ctypes binding of libslamhip (include/slamhip.h).

The shared library is built in-tree (``make -C slam-indoor-code_amd``) and loaded
from this directory.  There is no CPU fallback: if the library or a GPU is
missing, the calls that need them raise.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libslamhip.so")

# include/slamhip.h enums
SLAM_OK = 0
SLAM_E_INVALID_ARG = -1
SLAM_E_BAD_MATCHER = -2
SLAM_E_HIP = -3
SLAM_E_CAPACITY = -4
SLAM_E_NO_DEVICE = -5
SLAM_E_UNSUPPORTED = -6
SLAM_E_SOLVER = -7

SIFT_BF, SIFT_FLANN, ORB_BF = 0, 1, 2
NORM_DEFAULT, NORM_L1, NORM_L2, NORM_HAMMING = 0, 2, 4, 6
TYPE_5_8, TYPE_7_12, TYPE_9_16 = 0, 1, 2
LOSS_NONE, LOSS_TRIVIAL, LOSS_HUBER, LOSS_CAUCHY, LOSS_ARCTAN, LOSS_TUKEY = range(6)
EMPTY_BATCH, FRAME_NOT_FOUND = -2, -1
OPT_SIFT_KERNEL = 1
OPT_SIFT_BAND_SPLIT = 2
OPT_PNP_SUMS = 3
OPT_FAST_REUSE = 4
PNP_SUMS_ORDERED, PNP_SUMS_PAIRWISE = 0, 1
BAND_SPLIT_OFF, BAND_SPLIT_AUTO, BAND_SPLIT_ALL, BAND_SPLIT_ALL4 = 0, 1, 2, 3
STAGE_DESC_START, STAGE_DESC_END = 0, 1     # slam_order_after_stage
SIFT_KERNEL_AUTO, SIFT_KERNEL_BAND, SIFT_KERNEL_TAB, SIFT_KERNEL_GENERAL, SIFT_KERNEL_COLS, SIFT_KERNEL_COLW = 0, 1, 2, 3, 4, 5

# byte-identical to cv::KeyPoint / cv::DMatch
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"),
                         ("distance", "<f4")])
assert KEYPOINT_DTYPE.itemsize == 28 and DMATCH_DTYPE.itemsize == 16


class BASummary(ctypes.Structure):
    _fields_ = [("initial_cost", ctypes.c_double), ("final_cost", ctypes.c_double),
                ("num_residuals", ctypes.c_int32), ("iterations", ctypes.c_int32),
                ("successful_steps", ctypes.c_int32), ("termination", ctypes.c_int32),
                ("usable", ctypes.c_int32), ("total_time_in_seconds", ctypes.c_double)]


# exported symbols and their signatures: (restype, argtypes)
_P, _I, _SZ, _D, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_double, ctypes.c_uint64
SIGNATURES = {
    "slam_abi_version": (_I, []),
    "slam_device_count": (_I, []),
    "slam_create": (_P, [_I]),
    "slam_create_prio": (_P, [_I, _I]),
    "slam_destroy": (None, [_P]),
    "slam_last_error": (ctypes.c_char_p, [_P]),
    "slam_synchronize": (_I, [_P]),
    "slam_matcher_type": (_I, [_I, _I, _I]),
    "slam_fast": (_I, [_P, _P, _I, _I, _SZ, _I, _I, _I, _I, _P, _I, _P]),
    "slam_fast_dev": (_I, [_P, _P, _P, _I, _I, _SZ, _I, _I, _I, _I, _P, _I, _P]),
    "slam_describe": (_I, [_P, _P, _I, _I, _SZ, _I, _I, _P, _P, _P]),
    "slam_sift_detect": (_I, [_P, _P, _I, _I, _SZ, _I, _P, _I, _P, _P]),
    "slam_sift_detect_batch": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P]),
    "slam_reconstruct": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "slam_estimate_transformation": (_I, [_P, _P, _P, _I, _P, _I, _D, _D, _D, _P, _P, _P, _P, _P]),
    "slam_solve_pnp_ransac": (_I, [_P, _P, _P, _I, _P, _I, ctypes.c_float, _D, _P, _P, _P, _P, _P]),
    "slam_rodrigues": (_I, [_P, _I, _P]),
    "slam_knn2": (_I, [_P, _P, _I, _P, _I, _I, _I, _P, _P]),
    "slam_match": (_I, [_P, _P, _I, _P, _I, _I, _I, _D, _P, _I, _P]),
    "slam_match_frame": (_I, [_P, _P, _I, _P, _I, _I, _SZ, _I, _I, _I, _D, _P, _P, _P, _I, _P]),
    "slam_select_good": (_I, [_P, _I, _I, _I, _I]),
    "slam_ba": (_I, [_P, _P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _D, _I, ctypes.POINTER(BASummary)]),
    "slam_batch_extract": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "slam_batch_match": (_I, [_P, _P, _P, _I, _I, _D, _P]),
    "slam_batch_extract_match": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _D, _P, _P]),
    "slam_batch_extract_match_ev": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _D, _P, _P, _P]),
    "slam_batch_extract_async": (_I, [_P, _P, _P, _I, _I, _I, _I, _I]),
    "slam_batch_match_async": (_I, [_P, _P, _I, _I, _D, _P]),
    "slam_batch_finish": (_I, [_P, _P, _P]),
    "slam_context_stream": (_P, [_P]),
    "slam_batch_desc_bytes": (_SZ, [_I, _I]),
    "slam_batch_counts": (_I, [_P, _P, _P, _I]),
    "slam_batch_export_desc": (_I, [_P, _P, _I, _P, _P]),
    "slam_batch_get_keypoints": (_I, [_P, _I, _P, _I, _P]),
    "slam_batch_get_descriptors": (_I, [_P, _I, _P, _I, _P]),
    "slam_batch_get_matches": (_I, [_P, _I, _P, _I, _P]),
    "slam_batch_get_result": (_I, [_P, _I, _P, _I, _P, _P, _I, _P]),
    "slam_batch_result_begin": (_I, [_P, _I]),
    "slam_batch_result_end": (_I, [_P, _P, _I, _P, _P, _I, _P]),
    "slam_batch_result_dev": (_I, [_P, _P, _I, _P, _I, _P, _I]),
    "slam_order_after": (_I, [_P, _P, _P]),
    "slam_order_after_stage": (_I, [_P, _P, _I]),
    "slam_set_option": (_I, [_P, _I, _I]),
    "slam_batch_fast_reused": (_I, [_P]),
    "slam_last_sift_kernel": (_I, [_P]),
    "slam_profile_enable": (_I, [_P, _I]),
    "slam_profile_read": (_I, [_P, _I, _P, _P]),
    "slam_synth_frames": (_I, [_I, _I, _I, _I, _U64, _P]),
    "slam_synth_sequence": (_I, [_I, _I, _I, _I, _U64, _I, _P]),
    "slam_batch_fast": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "slam_synth_sequence_dev": (_I, [_P, _P, _I, _I, _I, _I, _U64, _I, _P]),
}

_lib = None


def lib():
    """Load libslamhip.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is None:
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME
        # libamdhip64.so.7).  Loading it first makes libslamhip bind to that same
        # runtime by SONAME; loading libslamhip first would put two HIP runtimes
        # in one process and torch would then see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise OSError(f"libslamhip.so not built: {LIB_PATH} (run make -C slam-indoor-code_amd)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ptr(a):
    """data pointer of a numpy array (None for None)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


class SlamError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"slamhip error {code}: {msg}")
        self.code = code


def check(code, ctx=None):
    if code == SLAM_OK:
        return
    msg = ""
    if ctx is not None:
        m = lib().slam_last_error(ctx)
        msg = m.decode() if m else ""
    raise SlamError(code, msg)
