"""Device-resident candidate scan: the data-parallel caller of the hot path.

Mirrors findGoodFrameFromBatch (reference src/mainModule/cycleProcessing/
batch.cpp:59-99) with its single-thread selection semantics (:101-160; the
multi-thread variant :162-226/:270-316 computes the same candidates
speculatively and selects with the same rule, minus its data races):

  1. batch fill (fillVideoFrameBatch :228-267): FAST on every incoming frame,
     frames with fewer than requiredExtractedPointsCount keypoints are skipped;
  2. previous good frame's descriptors computed once (the reference recomputes
     them on every search, :113 / :178 -- same values);
  3. every candidate: descriptors + kNN(k = 2) + ratio test vs the previous
     frame, all candidates at once on the GPU (speculative, like the threads);
  4. selection: scan from the tail down to skipFramesFromBatchHead, good iff
     |matches| >= requiredMatchedPointsCount and >= best so far; first-fit stops
     at the first good one; on success the batch becomes the elements AFTER the
     good index (:92-97).

Multi-GPU (ShardedScan): candidate k runs on rank k % world (the reference's
thread stride, :183-187); the previous good frame's descriptors are broadcast
over RCCL from the rank that owns them, per-candidate match counts are
all-gathered, every rank applies the same selection, and the winner's rank
becomes the next broadcast root.
"""
import ctypes

import numpy as np

from . import _lib as L
from ._lib import DMATCH_DTYPE, KEYPOINT_DTYPE, check, lib, ptr
from .api import default_context


def _torch():
    import torch  # device memory + streams + torch.distributed (RCCL); plumbing only
    return torch


class DeviceBatch:
    """slam_batch_* over frames that already live in HBM (a uint8 torch tensor
    of shape (n, h, w, 3) on the context's device)."""

    def __init__(self, ctx=None):
        self.ctx = ctx or default_context()
        self.c = self.ctx.handle
        self.matcher = None
        self.nframes = 0

    def _stream(self):
        torch = _torch()
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def extract(self, frames, threshold, matcher):
        """gray + FAST + descriptors for every frame; returns raw FAST counts."""
        n, h, w, ch = frames.shape
        assert ch == 3 and frames.is_contiguous() and frames.is_cuda
        counts = np.zeros(n, np.int32)
        check(lib().slam_batch_extract(self.c, self._stream(), ctypes.c_void_p(frames.data_ptr()), n, w, h,
                                       int(threshold), int(matcher), ptr(counts)), self.c)
        self.matcher, self.nframes = matcher, n
        return counts

    def fast(self, frames, threshold, reuse=False):
        """fillVideoFrameBatch's FAST (slam_batch_fast): gray + FAST-9 + NMS of
        every frame in one device pass, no descriptors; returns the per-frame
        keypoint counts (the keypoints stay in the batch: keypoints(f)).
        reuse=True (SLAM_OPT_FAST_REUSE) lets the next extraction of the same
        tensor take these results: only for frames whose contents do not change
        before that extraction (e.g. views of an immutable sequence)."""
        n, h, w, ch = frames.shape
        assert ch == 3 and frames.is_contiguous() and frames.is_cuda
        counts = np.zeros(n, np.int32)
        check(lib().slam_set_option(self.c, L.OPT_FAST_REUSE, 1 if reuse else 0), self.c)
        check(lib().slam_batch_fast(self.c, self._stream(), ctypes.c_void_p(frames.data_ptr()), n, w, h,
                                    int(threshold), ptr(counts)), self.c)
        self.matcher, self.nframes = None, n
        return counts

    def batch_counts(self):
        """descriptor-bearing keypoints per frame of the last extract (host copy)."""
        out = np.zeros(max(self.nframes, 1), np.int32)
        n = lib().slam_batch_counts(self.c, None, ptr(out), len(out))
        if n < 0:
            check(n, self.c)
        return out[:n].astype(np.int64)

    def desc_bytes(self, n):
        return lib().slam_batch_desc_bytes(int(self.matcher), int(n))

    def export_desc(self, frame, out=None):
        """frame's descriptors in the matcher's device format (torch uint8).
        Later work on torch's current stream (e.g. an RCCL broadcast of `out`)
        is ordered after the copy: with torch's default stream the library runs
        on its own non-blocking stream, so the copy is ordered explicitly."""
        torch = _torch()
        n = ctypes.c_int(0)
        cnt = self.keypoint_count(frame)
        if out is None:
            out = torch.empty(max(self.desc_bytes(cnt), 1), dtype=torch.uint8, device="cuda")
        s = self._stream()
        check(lib().slam_batch_export_desc(self.c, s, int(frame), ctypes.c_void_p(out.data_ptr()),
                                           ctypes.byref(n)), self.c)
        check(lib().slam_order_after(self.c, s, s), self.c)
        return out, n.value

    def keypoint_count(self, frame):
        n = ctypes.c_int(0)
        rc = lib().slam_batch_get_keypoints(self.c, int(frame), None, 0, ctypes.byref(n))
        if rc not in (L.SLAM_OK, L.SLAM_E_CAPACITY):
            check(rc, self.c)
        return n.value

    def match(self, query, nq, ratio, norm=L.NORM_DEFAULT):
        """kNN + ratio of every frame vs the query set (device, matcher format)."""
        counts = np.zeros(self.nframes, np.int32)
        check(lib().slam_batch_match(self.c, self._stream(), ctypes.c_void_p(query.data_ptr()), int(nq), int(norm),
                                     float(ratio), ptr(counts)), self.c)
        return counts

    def extract_match(self, frames, threshold, matcher, query, nq, ratio, norm=L.NORM_DEFAULT, query_ready=None):
        """extract + match with one host sync (slam_batch_extract_match); returns
        (raw FAST counts, match counts), as extract() then match() would.
        query_ready: a torch.cuda.Event recorded after the query's producer (the
        RCCL broadcast); only the kNN waits on it, the extraction runs ahead."""
        n, h, w, ch = frames.shape
        assert ch == 3 and frames.is_contiguous() and frames.is_cuda
        kc = np.zeros(n, np.int32)
        mc = np.zeros(n, np.int32)
        ev = ctypes.c_void_p(query_ready.cuda_event) if query_ready is not None else None
        check(lib().slam_batch_extract_match_ev(self.c, self._stream(), ctypes.c_void_p(frames.data_ptr()), n, w, h,
                                                int(threshold), int(matcher), ctypes.c_void_p(query.data_ptr()),
                                                int(nq), int(norm), float(ratio), ev, ptr(kc), ptr(mc)), self.c)
        self.matcher, self.nframes = matcher, n
        return kc, mc

    def extract_async(self, frames, threshold, matcher):
        """slam_batch_extract_async: queue gray + FAST + descriptors of every
        frame on the context's stream and return at once; finish() takes them."""
        n, h, w, ch = frames.shape
        assert ch == 3 and frames.is_contiguous() and frames.is_cuda
        # the extraction runs on the context's own (non-blocking) stream: order it
        # after whatever torch queued that produces `frames` (a stack, an
        # index_select, a copy) -- a device-side wait, no host block
        torch = _torch()
        torch.cuda.ExternalStream(lib().slam_context_stream(self.c), device=frames.device).wait_stream(
            torch.cuda.current_stream(frames.device))
        check(lib().slam_batch_extract_async(self.c, None, ctypes.c_void_p(frames.data_ptr()), n, w, h,
                                             int(threshold), int(matcher)), self.c)
        self._async = (n, matcher)

    def match_async(self, query, nq, ratio, norm=L.NORM_DEFAULT, query_ready=None):
        """slam_batch_match_async: queue the kNN + ratio test of the queued
        extraction against the query set, behind query_ready (a torch event)."""
        ev = ctypes.c_void_p(query_ready.cuda_event) if query_ready is not None else None
        check(lib().slam_batch_match_async(self.c, ctypes.c_void_p(query.data_ptr()), int(nq), int(norm),
                                           float(ratio), ev), self.c)

    def finish(self):
        """slam_batch_finish: wait for the queued batch; (raw FAST counts, match counts)."""
        n, matcher = self._async
        kc = np.zeros(n, np.int32)
        mc = np.zeros(n, np.int32)
        self._async = None
        check(lib().slam_batch_finish(self.c, ptr(kc), ptr(mc)), self.c)
        self.matcher, self.nframes = matcher, n
        return kc, mc

    def keypoints(self, frame):
        cnt = self.keypoint_count(frame)
        out = np.zeros(max(cnt, 1), KEYPOINT_DTYPE)
        n = ctypes.c_int(0)
        check(lib().slam_batch_get_keypoints(self.c, int(frame), ptr(out), len(out), ctypes.byref(n)), self.c)
        return out[:n.value]

    def descriptors(self, frame):
        cnt = self.keypoint_count(frame)
        if self.matcher == L.ORB_BF:
            out = np.zeros((max(cnt, 1), 32), np.uint8)
        else:
            out = np.zeros((max(cnt, 1), 128), np.float32)
        n = ctypes.c_int(0)
        check(lib().slam_batch_get_descriptors(self.c, int(frame), ptr(out), len(out), ctypes.byref(n)), self.c)
        return out[:n.value]

    def result(self, frame, nq):
        """frame's (keypoints, matches) with one host sync (slam_batch_get_result)"""
        kc = self.keypoint_count(frame)
        kps = np.empty(max(kc, 1), KEYPOINT_DTYPE)
        mts = np.empty(max(nq, 1), DMATCH_DTYPE)
        nk, nm = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().slam_batch_get_result(self.c, int(frame), ptr(kps), len(kps), ctypes.byref(nk), ptr(mts), len(mts),
                                          ctypes.byref(nm)), self.c)
        return kps[:nk.value], mts[:nm.value]

    def result_begin(self, frame, nq):
        """queue frame's (keypoints, matches) to the host without waiting
        (slam_batch_result_begin); result_end() takes them, typically after the
        next batch's own sync"""
        check(lib().slam_batch_result_begin(self.c, int(frame)), self.c)
        self._pending = (self.keypoint_count(frame), int(nq))

    def result_end(self):
        kc, nq = self._pending
        kps = np.empty(max(kc, 1), KEYPOINT_DTYPE)
        mts = np.empty(max(nq, 1), DMATCH_DTYPE)
        nk, nm = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().slam_batch_result_end(self.c, ptr(kps), len(kps), ctypes.byref(nk), ptr(mts), len(mts),
                                          ctypes.byref(nm)), self.c)
        self._pending = None
        return kps[:nk.value], mts[:nm.value]

    def result_dev(self, frame, nm, d_matches, d_kps, kcap):
        """frame's ratio-test matches (the first nm, query order) and keypoints
        into device memory (data pointers), queued without a host sync
        (slam_batch_result_dev); later work on torch's current stream is ordered
        after the copies."""
        s = self._stream()
        check(lib().slam_batch_result_dev(self.c, s, int(frame), ctypes.c_void_p(d_matches), int(nm),
                                          ctypes.c_void_p(d_kps), int(kcap)), self.c)
        check(lib().slam_order_after(self.c, s, s), self.c)

    def matches(self, frame, nq):
        out = np.zeros(max(nq, 1), DMATCH_DTYPE)
        n = ctypes.c_int(0)
        check(lib().slam_batch_get_matches(self.c, int(frame), ptr(out), len(out), ctypes.byref(n)), self.c)
        return out[:n.value]


def select_good(match_counts, required, skip_head, first_fit):
    a = np.ascontiguousarray(match_counts, np.int32)
    return lib().slam_select_good(ptr(a), len(a), int(required), int(skip_head), int(bool(first_fit)))


class Conditions:
    """DataProcessingConditions (mainCycleStructures.h:21-33), hot-path fields."""

    def __init__(self, featureExtractingThreshold=10, requiredExtractedPointsCount=0, frameBatchSize=30,
                 skipFramesFromBatchHead=0, useFirstFitInBatch=True, requiredMatchedPointsCount=0,
                 matcherType=L.SIFT_FLANN, knnMatcherDistance=0.7):
        self.featureExtractingThreshold = featureExtractingThreshold
        self.requiredExtractedPointsCount = requiredExtractedPointsCount
        self.frameBatchSize = frameBatchSize
        self.skipFramesFromBatchHead = skipFramesFromBatchHead
        self.useFirstFitInBatch = useFirstFitInBatch
        self.requiredMatchedPointsCount = requiredMatchedPointsCount
        self.matcherType = matcherType
        self.knnMatcherDistance = knnMatcherDistance

    @classmethod
    def from_config(cls, cfg):
        from .api import getMatcherTypeIndex
        g = cfg.getValue
        return cls(int(g("featureExtractingThreshold")), int(g("requiredExtractedPointsCount")),
                   int(g("framesBatchSize")), int(g("skipFramesFromBatchHead")), bool(g("useFirstFitInBatch")),
                   int(g("requiredMatchedPointsCount")), getMatcherTypeIndex(cfg), float(g("knnMatcherDistance")))


def find_good_frame(db, frames_gpu, prev_desc, nprev, cond):
    """One search over frames_gpu (the batch, already filled) against the previous
    good frame's device descriptors.  Returns (goodIndex, kp_counts, match_counts,
    in_batch) where in_batch are the frame indices that passed the FAST filter."""
    # extract + match with one host sync; candidates the batch filter drops
    # (batch.cpp:247) are matched too, but their counts never reach the selection
    kp, counts = db.extract_match(frames_gpu, cond.featureExtractingThreshold, cond.matcherType, prev_desc, nprev,
                                  cond.knnMatcherDistance)
    in_batch = np.nonzero(kp >= cond.requiredExtractedPointsCount)[0]
    if len(in_batch) == 0:
        return L.EMPTY_BATCH, kp, None, in_batch
    good = select_good(counts[in_batch], cond.requiredMatchedPointsCount, cond.skipFramesFromBatchHead,
                       cond.useFirstFitInBatch)
    return good, kp, counts, in_batch


def owner_of(k, world):
    """(rank, local index) of global candidate k under the thread stride
    (batch.cpp:183-187: thread i takes candidates i, i + threads, ...)."""
    return int(k) % world, int(k) // world


def interleave_shards(per_rank):
    """per_rank[r]: (n_r, c) rows of rank r's candidates in local order ->
    (sum n_r, c) rows in global candidate order (k -> rank k % world)."""
    world = len(per_rank)
    total = sum(len(x) for x in per_rank)
    cols = per_rank[0].shape[1] if per_rank and per_rank[0].ndim == 2 else 1
    out = np.zeros((total, cols), np.int32)
    for r, x in enumerate(per_rank):
        idx = np.arange(r, total, world)
        if len(idx) != len(x):
            raise ValueError(f"rank {r} holds {len(x)} candidates, stride layout expects {len(idx)}")
        out[idx] = x
    return out


def exchange_counts(kp, counts, world, device, extra=None, pad_to=None, collective=None):
    """All-gather each rank's per-candidate (keypoint count, match count[, extra])
    rows (ragged shards padded with -1 rows) and return the global arrays,
    identical on every rank.  `device`: "cuda" (RCCL) or "cpu" (gloo, tests).
    `extra`: a third per-candidate column (e.g. descriptor counts, so that every
    rank knows the winner's query size without another collective).  `pad_to`:
    an upper bound of every rank's shard size known to all ranks (skips the
    all-reduce of the shard sizes).  `collective`: run the all-gather even at
    world 1 (default: only when world > 1)."""
    cols = [np.asarray(kp, np.int32), np.asarray(counts, np.int32)]
    if extra is not None:
        cols.append(np.asarray(extra, np.int32))
    if not (world > 1 if collective is None else collective):
        out = tuple(c.copy() for c in cols)
        return out
    torch = _torch()
    import torch.distributed as dist
    local = torch.tensor(np.stack(cols, 1).reshape(-1, len(cols)), dtype=torch.int32, device=device)
    n_local = local.shape[0]
    if pad_to is None:
        nmax = torch.tensor([n_local], dtype=torch.int32, device=device)
        dist.all_reduce(nmax, op=dist.ReduceOp.MAX)
        pad_to = int(nmax.item())
    pad = torch.full((max(int(pad_to), 1), len(cols)), -1, dtype=torch.int32, device=device)
    pad[:n_local] = local
    gathered = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad)
    g = [x.cpu().numpy() for x in gathered]
    per_rank = [gi[gi[:, 0] >= 0] for gi in g]            # keypoint counts are >= 0; -1 = padding
    allc = interleave_shards(per_rank)
    return tuple(allc[:, k].copy() for k in range(len(cols)))


def select_global(kp_all, mc_all, cond):
    """The selection every rank applies to the gathered counts: batch filter
    (requiredExtractedPointsCount, batch.cpp:245-253) then the tail-first rule
    (batch.cpp:136-146).  Returns (good index into in_batch or EMPTY_BATCH /
    -1, in_batch)."""
    in_batch = np.nonzero(np.asarray(kp_all) >= cond.requiredExtractedPointsCount)[0]
    if len(in_batch) == 0:
        return L.EMPTY_BATCH, in_batch
    good = select_good(np.asarray(mc_all)[in_batch], cond.requiredMatchedPointsCount,
                       cond.skipFramesFromBatchHead, cond.useFirstFitInBatch)
    return good, in_batch


def broadcast_prev(prev_buf, nbytes, owner, world):
    """The previous good frame's descriptors, owner rank -> every rank."""
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(prev_buf[:max(int(nbytes), 1)], src=owner)


class ShardedScan:
    """Candidate sharding over the ranks of a torch.distributed group (RCCL).

    `engine` does the per-candidate work: by default a DeviceBatch (the HIP
    library); it needs extract_match(frames, threshold, matcher, query, nq,
    ratio, query_ready=None) -> (raw FAST counts, match counts) and
    batch_counts() -> descriptor counts of the last call.  `device` is where the
    exchange tensors live: "cuda" (RCCL) or "cpu" (gloo)."""

    def __init__(self, rank, world, ctx=None, engine=None, device="cuda"):
        self.rank, self.world = rank, world
        self.db = engine if engine is not None else DeviceBatch(ctx)
        self.device = device

    def shard(self, nframes):
        """global candidate indices owned by this rank (thread stride, batch.cpp:183-187)."""
        return np.arange(self.rank, nframes, self.world)

    def search(self, frames_local, prev_buf, nprev, owner, cond, pad_to=None):
        """frames_local: this rank's candidates; prev_buf: uint8 device buffer large
        enough for the previous descriptors, valid on rank `owner`.  Returns
        (good, kp_all, mc_all, in_batch, desc_all) -- the global selection, the
        all-gathered per-candidate counts (identical on every rank) and every
        candidate's descriptor count (the next query size, known to all ranks).
        pad_to: an upper bound of every rank's shard size known to all ranks
        (skips one all-reduce)."""
        # (1) exchange: previous good frame's descriptors, owner -> all (RCCL
        # broadcast).  Only the kNN waits for it: the wait is put on a side
        # stream whose event the library orders the match behind, so the
        # extraction of this rank's candidates overlaps the transfer
        ready = None
        coll = self._collective()
        if coll:
            import torch.distributed as dist
            nb = lib().slam_batch_desc_bytes(int(cond.matcherType), int(nprev))
            work = dist.broadcast(prev_buf[:max(int(nb), 1)], src=owner, async_op=True)
            ready = self._after(work)
        n_local = len(frames_local)
        if n_local > 0:
            kp, counts = self.db.extract_match(frames_local, cond.featureExtractingThreshold, cond.matcherType,
                                               prev_buf, nprev, cond.knnMatcherDistance, query_ready=ready)
            dc = self.db.batch_counts()
        else:
            # fewer candidates than ranks (a short batch tail): nothing to extract,
            # but this rank still joins the collectives with an empty shard
            if ready is not None and self.device == "cuda":
                ready.synchronize()
            kp = counts = dc = np.zeros(0, np.int32)
        # (2) exchange: per-candidate (kp, match, descriptor) counts -> all ranks
        kp_all, mc_all, dc_all = exchange_counts(kp, counts, self.world, self.device, extra=dc, pad_to=pad_to,
                                                 collective=coll)
        good, in_batch = select_global(kp_all, mc_all, cond)
        return good, kp_all, mc_all, in_batch, dc_all

    def advance(self, good, in_batch, dc_all, prev_buf, owner, nprev):
        """hand-over after a search: the winner's descriptors become the next
        query set.  The rank that owns the winner exports them into prev_buf (it
        is the next broadcast root); every rank learns the next query size from
        the gathered descriptor counts.  Returns (owner, nprev)."""
        if good < 0:
            return owner, nprev
        gi = int(in_batch[good])
        owner, li = owner_of(gi, self.world)
        if owner == self.rank:
            self.db.export_desc(li, prev_buf)
        return owner, int(dc_all[gi])

    def winner(self, good, in_batch, dc_all, mc_all, nq):
        """the winner's keypoints and ratio-test matches on every rank (the third
        exchange of SURVEY.md 8(e): the owner broadcasts them, so the rank that
        drives the per-frame pipeline holds what findGoodFrameFromBatch returns,
        batch.cpp:92-97).  Sizes come from the gathered counts, so no size
        exchange is needed.  Returns (keypoints, matches) or (None, None)."""
        if good < 0:
            return None, None
        if self._device_exchange():
            return self.winner_end(self._winner_dev_begin(good, in_batch, dc_all, mc_all))
        gi = int(in_batch[good])
        owner, li = owner_of(gi, self.world)
        nk, nm = int(dc_all[gi]), int(mc_all[gi])
        if owner == self.rank:
            if hasattr(self.db, "result"):
                kps, mts = self.db.result(li, nq)
            else:
                kps = self.db.keypoints(li)
                mts = self.db.matches(li, nq) if nm > 0 else np.zeros(0, DMATCH_DTYPE)
            kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
            mts = np.ascontiguousarray(mts, DMATCH_DTYPE) if mts is not None else np.zeros(0, DMATCH_DTYPE)
            if len(kps) != nk or len(mts) != nm:
                raise RuntimeError("winner's keypoint / match counts differ from the gathered counts")
        if not self._collective() or self.world == 1:
            return kps, mts
        torch = _torch()
        import torch.distributed as dist
        nbytes = nk * KEYPOINT_DTYPE.itemsize + nm * DMATCH_DTYPE.itemsize
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        if owner == self.rank:
            host = np.concatenate([kps.view(np.uint8).reshape(-1), mts.view(np.uint8).reshape(-1)])
            if nbytes:
                buf[:nbytes].copy_(torch.from_numpy(host))
        dist.broadcast(buf, src=owner)
        if owner == self.rank:
            return kps, mts
        b = buf[:nbytes].cpu().numpy()
        kb = nk * KEYPOINT_DTYPE.itemsize
        return b[:kb].view(KEYPOINT_DTYPE).copy(), b[kb:].view(DMATCH_DTYPE).copy()

    def winner_begin(self, good, in_batch, dc_all, mc_all, nq):
        """winner() in two halves; winner_end() takes the result, typically
        after the next search's own sync, so the copies overlap that search
        instead of costing a sync of their own.
          - one rank: the transfer is queued (slam_batch_result_begin);
          - more ranks on the GPU: the owner writes the winner's matches and
            keypoints into a device buffer (slam_batch_result_dev, no host round
            trip), RCCL broadcasts it, and every rank queues one copy to pinned
            host memory behind the broadcast;
          - otherwise (gloo on the CPU) the token carries winner()'s result."""
        if good >= 0 and self.world == 1 and hasattr(self.db, "result_begin"):
            gi = int(in_batch[good])
            _, li = owner_of(gi, 1)
            self.db.result_begin(li, nq)
            return ("queued", int(dc_all[gi]), int(mc_all[gi]))
        if good >= 0 and self._device_exchange():
            return self._winner_dev_begin(good, in_batch, dc_all, mc_all)
        return ("done", self.winner(good, in_batch, dc_all, mc_all, nq))

    def winner_end(self, token):
        if token[0] == "done":
            return token[1]
        if token[0] == "device":
            _, ev, host, nk, nm = token
            ev.synchronize()
            b = host.numpy()
            mb = nm * DMATCH_DTYPE.itemsize
            mts = b[:mb].view(DMATCH_DTYPE).copy()
            kps = b[mb:mb + nk * KEYPOINT_DTYPE.itemsize].view(KEYPOINT_DTYPE).copy()
            return kps, mts
        kps, mts = self.db.result_end()
        if len(kps) != token[1] or len(mts) != token[2]:
            raise RuntimeError("winner's keypoint / match counts differ from the gathered counts")
        return kps, mts

    def _device_exchange(self):
        """the winner travels device to device (RCCL) when more ranks share the
        scan on GPUs and the engine can write its result into device memory"""
        return self.world > 1 and self.device == "cuda" and hasattr(self.db, "result_dev")

    def _winner_dev_begin(self, good, in_batch, dc_all, mc_all):
        """SURVEY.md 8(e) exchange 3 without a host round trip: layout [matches
        nm x 16 B][keypoints nk x 28 B]; sizes from the gathered counts"""
        torch = _torch()
        import torch.distributed as dist
        gi = int(in_batch[good])
        owner, li = owner_of(gi, self.world)
        nk, nm = int(dc_all[gi]), int(mc_all[gi])
        mb, kb = nm * DMATCH_DTYPE.itemsize, nk * KEYPOINT_DTYPE.itemsize
        n = max(mb + kb, 1)
        buf = torch.empty(n, dtype=torch.uint8, device="cuda")
        if owner == self.rank:
            base = buf.data_ptr()
            self.db.result_dev(li, nm, base, base + mb, nk)
        dist.broadcast(buf, src=owner)          # torch's stream waits for it on the device
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.copy_(buf, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ("device", ev, host, nk, nm)

    def _query_ready(self, prev_buf, nprev, owner, cond):
        """(1) the previous good frame's descriptors, owner -> all ranks (async
        RCCL broadcast), and an event the kNN waits on: recorded on torch's
        stream behind the broadcast -- or, on one rank, behind the owner's
        export (export_desc orders torch's stream after it)."""
        if self._collective():
            import torch.distributed as dist
            nb = lib().slam_batch_desc_bytes(int(cond.matcherType), int(nprev))
            work = dist.broadcast(prev_buf[:max(int(nb), 1)], src=owner, async_op=True)
            return self._after(work)
        if self.device != "cuda":
            return None
        torch = _torch()
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def _collective(self):
        """collectives run whenever a process group is up (world 1 included: the
        same broadcast / all-gather path, one rank)."""
        if self.world > 1:
            return True
        try:
            import torch.distributed as dist
            return dist.is_available() and dist.is_initialized()
        except ImportError:
            return False

    def _after(self, work):
        """an event the kNN can wait on for `work` (None off the GPU, where the
        collective has completed when wait() returns)."""
        if self.device != "cuda":
            work.wait()
            return None
        torch = _torch()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            work.wait()               # side stream waits on the RCCL stream (no host block)
            ev = torch.cuda.Event()
            ev.record(side)
        return ev


class PipelinedScan:
    """ShardedScan over two contexts whose searches overlap on the device.

    A search's extraction (gray, FAST, descriptors of its candidates) needs no
    result of the previous search; only its kNN waits for the previous winner's
    descriptors (batch.cpp:113-127: the previous good frame is the query).  So
    while the host takes search k -- its counts, the count all-gather, the
    selection, the winner's hand-over and result -- the device already runs
    search k + 1's extraction, queued on the other context
    (slam_batch_extract_async).  Each search's results, selections and
    hand-overs are exactly ShardedScan's; only the host waits move.

    Use: queue(frames, cond) before the first search, then per search
    search(frames_local, prev_buf, nprev, owner, cond, pad_to, next_frames)
    (next_frames: the candidates of the search after this one, whose extraction
    is queued before this one is taken; None after the last), then
    winner_begin / advance / winner_end as ShardedScan's.

    overlap: where search k + 1's extraction may start on the device -- "knn"
    after search k's kNN (no two large kernels share the chip), "desc_end"
    when search k's descriptor kernel has finished (beside its kNN), or
    "desc_start" when it has been reached (its workgroups hold the CUs; the
    next gray / FAST / blur take CUs as its tail frees them).  Results are the
    same in every mode: each context's own work stays in its stream order."""

    OVERLAPS = {"desc_start": L.STAGE_DESC_START, "desc_end": L.STAGE_DESC_END}

    def __init__(self, rank, world, device_index=0, device="cuda", contexts=None, overlap="knn"):
        from .api import Context
        if overlap != "knn" and overlap not in self.OVERLAPS:
            raise ValueError(f"overlap: 'knn', 'desc_end' or 'desc_start', not {overlap!r}")
        self.overlap = overlap
        self.rank, self.world, self.device = rank, world, device
        self.ctxs = contexts or [Context(device_index), Context(device_index)]
        self.scans = [ShardedScan(rank, world, engine=DeviceBatch(c), device=device) for c in self.ctxs]
        self.k = 0               # the next search runs on scans[k % 2]
        self.queued = None       # the scan whose extraction is queued

    @property
    def last(self):
        """the scan of the last search taken (its batch holds that search's results)"""
        return self.scans[(self.k - 1) % 2]

    @property
    def db(self):
        return self.last.db

    def queue(self, frames_local, cond):
        sc = self.scans[self.k % 2]
        if self.queued is sc:
            raise RuntimeError("the next search's extraction is already queued")
        if len(frames_local) > 0:
            sc.db.extract_async(frames_local, cond.featureExtractingThreshold, cond.matcherType)
        self.queued = sc

    def search(self, frames_local, prev_buf, nprev, owner, cond, pad_to=None, next_frames=None):
        sc = self.scans[self.k % 2]
        if self.queued is not sc:
            self.queue(frames_local, cond)
        ready = sc._query_ready(prev_buf, nprev, owner, cond)
        n_local = len(frames_local)
        if n_local > 0:
            sc.db.match_async(prev_buf, nprev, cond.knnMatcherDistance, query_ready=ready)
        self.k += 1
        self.queued = None
        if next_frames is not None:
            # search k + 1's extraction, on the other context, starts when this
            # search's kNN is done: the device never idles while the host takes
            # this search, and no two big kernels share the chip (their launch
            # times stay those of the sequential schedule)
            other = self.scans[self.k % 2]
            waiter = lib().slam_context_stream(other.db.c)
            if self.overlap == "knn" or n_local == 0:
                check(lib().slam_order_after(sc.db.c, waiter, None), sc.db.c)
            else:
                check(lib().slam_order_after_stage(sc.db.c, waiter, self.OVERLAPS[self.overlap]), sc.db.c)
            self.queue(next_frames, cond)
        if n_local > 0:
            kp, counts = sc.db.finish()
            dc = sc.db.batch_counts()
        else:
            if ready is not None and self.device == "cuda":
                ready.synchronize()
            kp = counts = dc = np.zeros(0, np.int32)
        kp_all, mc_all, dc_all = exchange_counts(kp, counts, self.world, self.device, extra=dc, pad_to=pad_to,
                                                 collective=sc._collective())
        good, in_batch = select_global(kp_all, mc_all, cond)
        return good, kp_all, mc_all, in_batch, dc_all

    def advance(self, good, in_batch, dc_all, prev_buf, owner, nprev):
        return self.last.advance(good, in_batch, dc_all, prev_buf, owner, nprev)

    def winner(self, good, in_batch, dc_all, mc_all, nq):
        return self.last.winner(good, in_batch, dc_all, mc_all, nq)

    def winner_begin(self, good, in_batch, dc_all, mc_all, nq):
        sc = self.last
        return (sc, sc.winner_begin(good, in_batch, dc_all, mc_all, nq))

    def winner_end(self, token):
        sc, tok = token
        return sc.winner_end(tok)

    def drain(self):
        """take a queued extraction that no search will use (the buffers return to the caller)"""
        if self.queued is not None and self.queued.db.__dict__.get("_async"):
            self.queued.db.finish()
        self.queued = None

    def close(self):
        self.drain()
        for c in self.ctxs:
            c.close()
