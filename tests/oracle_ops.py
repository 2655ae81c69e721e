"""CPU-oracle implementation of the operations slamhip.cycle drives (test
infrastructure only: the checker for the pipeline parity tests and the CPU
plumbing run of BASELINE configs[0]).  Same method names and return values as
slamhip.cycle.GpuOps; every numeric step is the oracle's C restatement
(oracle/*.c), the control flow is the product's own slamhip.cycle."""
import numpy as np

import oracle_ffi as O

SIFT_BF, SIFT_FLANN, ORB_BF = 0, 1, 2


class OracleOps:
    def __init__(self, flann=False):
        # flann=True: useFM-SIFT-FLANN as the reference's CPU build runs it (KD-forest,
        # approximate); False: exact BF-L2 (the reference's CUDA build, and the GPU path)
        self.flann = flann

    def fast(self, frame, threshold):
        return O.fast(frame, threshold, True)

    def describe(self, frame, kps, matcher):
        if matcher == ORB_BF:
            return O.orb(frame, kps)
        k = np.ascontiguousarray(kps, O.KP).copy()
        return k, O.sift(frame, k)

    def match_frame(self, prev_desc, frame, kps, matcher, ratio):
        k, d = self.describe(frame, kps, matcher)
        if len(prev_desc) == 0 or len(k) == 0:
            return k, np.zeros(0, O.DM)
        if matcher == ORB_BF:
            idx, dist = O.knn2(prev_desc, d, O.NORM_HAMMING)
        elif matcher == SIFT_FLANN and self.flann:
            idx, dist = O.flann_knn2(prev_desc, d)
        else:
            idx, dist = O.knn2(prev_desc, d, O.NORM_L2)
        return k, O.ratio(idx, dist, ratio)

    def estimate_transformation(self, p1, p2, K, use_ransac, prob, threshold, distance):
        ok, R, t, cm, _, _ = O.estimate_transformation(p1, p2, K, use_ransac, prob, threshold, distance)
        return ok, R, t, cm

    def reconstruct(self, K, R1, t1, R2, t2, p1, p2):
        return O.reconstruct(K, R1, t1, R2, t2, p1, p2)

    def solve_pnp(self, obj, img, K):
        st, r, t, _, _ = O.solve_pnp_ransac(obj, img, K)
        return bool(st), r, t

    def rodrigues(self, rvec):
        return O.rodrigues(np.asarray(rvec, np.float64).reshape(3))[0]

    def ba(self, K4, ext, pts, obs_frame, obs_point, obs_xy, loss, loss_param):
        k, e, p, s = O.ba(K4, ext, pts, obs_frame, obs_point, obs_xy, loss, loss_param)
        K4[...] = k
        ext[...] = e
        pts[...] = p
        return s


class OracleBatchEngine:
    """The per-candidate work of slamhip.batch.ShardedScan (DeviceBatch's
    extract_match / batch_counts / export_desc) on the oracle and host memory,
    so the sharded search's control flow and collectives can run under gloo on
    the CPU.  Query sets use the library's internal SIFT layout: n x 128 u8
    descriptors, then n int32 |d - 128|^2 (slam_batch_desc_bytes)."""

    def __init__(self):
        self.kps, self.desc, self.mts = [], [], []

    @staticmethod
    def pack(desc):
        d = np.asarray(desc).astype(np.uint8)
        nrm = ((d.astype(np.int64) - 128) ** 2).sum(1).astype(np.int32)
        return np.concatenate([d.reshape(-1), nrm.view(np.uint8)])

    def extract_match(self, frames, threshold, matcher, query, nq, ratio, query_ready=None):
        assert matcher in (SIFT_BF, SIFT_FLANN)
        fr = frames.numpy() if hasattr(frames, "numpy") else np.asarray(frames)
        q = (query.numpy() if hasattr(query, "numpy") else np.asarray(query))[:nq * 128]
        qd = q.reshape(nq, 128).astype(np.float32)
        self.kps, self.desc, self.mts = [], [], []
        kc, mc = [], []
        for f in fr:
            k = O.fast(f, threshold, True)
            d = O.sift(f, k)
            self.kps.append(k)
            self.desc.append(d)
            kc.append(len(k))
            if nq == 0 or len(d) == 0:
                mc.append(0)
                self.mts.append(None)
                continue
            idx, dist = O.knn2(qd, d, O.NORM_L2)
            m = O.ratio(idx, dist, ratio)
            self.mts.append(m)
            mc.append(len(m))
        return np.array(kc, np.int32), np.array(mc, np.int32)

    def keypoints(self, frame):
        return self.kps[frame]

    def matches(self, frame, nq):
        return self.mts[frame]

    def batch_counts(self):
        return np.array([len(d) for d in self.desc], np.int64)

    def export_desc(self, frame, out):
        b = self.pack(self.desc[frame])
        out[:len(b)] = __import__("torch").from_numpy(b)
        return out, len(self.desc[frame])
