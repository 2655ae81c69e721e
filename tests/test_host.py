"""CPU tests of the host side: the C ABI library loads and exports every symbol
include/slamhip.h declares (no compute calls), the host-only ABI entry points,
the reference-interface mirror (config, matcher type, ratio test, selection),
and the multi-rank exchange/selection logic with gloo at world size 2."""
import ctypes
import json
import os
import re
import socket
import tempfile

import numpy as np
import pytest

import oracle_ffi as O
import slamhip
from slamhip import _lib as L
from slamhip import batch as B
from slamhip import config as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "slamhip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(slam_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding covers exactly the declared ABI
    assert set(L.SIGNATURES) == set(names)


def test_library_resolves_every_symbol_at_load():
    """lazy binding would defer an undefined internal symbol (a definition left
    out of a build) to its first call on the GPU box: bind everything now"""
    import subprocess
    import sys
    code = ("import ctypes, os, sys; l = ctypes.CDLL(sys.argv[1], mode=os.RTLD_NOW | os.RTLD_LOCAL); "
            "print(l.slam_abi_version())")
    r = subprocess.run([sys.executable, "-c", code, L.LIB_PATH], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "3", r.stdout + r.stderr


def test_library_has_gfx950_code_object_and_no_oracle_link():
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"liboracle" not in blob and b"orc_" not in blob


def test_abi_version_and_host_only_entry_points():
    lib = L.lib()
    assert lib.slam_abi_version() == 3
    # getMatcherTypeIndex priority: SIFT_BF > SIFT_FLANN > ORB (featureMatchingCommon.cpp:13-21)
    assert lib.slam_matcher_type(1, 1, 1) == L.SIFT_BF
    assert lib.slam_matcher_type(0, 1, 1) == L.SIFT_FLANN
    assert lib.slam_matcher_type(0, 0, 1) == L.ORB_BF
    assert lib.slam_matcher_type(0, 0, 0) == L.SLAM_E_BAD_MATCHER
    # internal device format: SIFT u8[128] + i32 norm side array; ORB +-1 FP4[256] (128 B)
    assert lib.slam_batch_desc_bytes(L.SIFT_BF, 10) == 10 * (128 + 4)
    assert lib.slam_batch_desc_bytes(L.ORB_BF, 10) == 10 * 128
    # null-context calls fail with a status, never crash
    assert lib.slam_synchronize(None) == L.SLAM_E_INVALID_ARG
    assert lib.slam_profile_enable(None, 1) == L.SLAM_E_INVALID_ARG


def test_get_matcher_type_index_raises_like_reference():
    cfg = C.ConfigService({"useFM-SIFT-BF": False, "useFM-SIFT-FLANN": False, "useFM-ORB": False})
    with pytest.raises(slamhip.MatcherTypeError):
        slamhip.getMatcherTypeIndex(cfg)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_select_good_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    for n in (0, 1, 2, 7, 30):
        counts = rng.integers(0, 1000, n).astype(np.int32)
        if n > 3:
            counts[rng.integers(0, n, 2)] = counts.max()      # ties
        for req in (0, 300, 700, 2000):
            for skip in (0, 1, 3):
                for ff in (0, 1):
                    got = B.select_good(counts, req, skip, ff)
                    assert got == O.select_good(counts, req, skip, ff), (n, req, skip, ff)


def test_get_good_matches_strict_ratio():
    idx = np.array([[3, 4], [5, 6], [7, 8]], np.int32)
    dist = np.array([[7.0, 10.0], [6.9, 10.0], [0.0, 0.0]], np.float32)
    good = slamhip.getGoodMatches(idx, dist, 0.7)
    # d0 < 0.7 * d1 in double: 7.0 < 7.000000000000001 holds; 0 < 0 does not
    exp = [q for q in range(3) if float(dist[q, 0]) < 0.7 * float(dist[q, 1])]
    assert [int(m["queryIdx"]) for m in good] == exp


def test_config_check_json_and_comments():
    text = """{
      // comment
      "featureExtractingThreshold": 31, /* block */
      "useFM-SIFT-FLANN": true
    }"""
    stripped = C.strip_comments(text)
    d = json.loads(stripped)
    assert d["featureExtractingThreshold"] == 31 and d["useFM-SIFT-FLANN"] is True


def test_interleave_and_owner():
    per = [np.array([[0, 10], [2, 12], [4, 14], [6, 16]], np.int32),
           np.array([[1, 11], [3, 13], [5, 15]], np.int32)]
    allc = B.interleave_shards(per)
    assert allc[:, 0].tolist() == list(range(7))
    assert allc[:, 1].tolist() == list(range(10, 17))
    assert [B.owner_of(k, 2) for k in (0, 1, 5, 6)] == [(0, 0), (1, 0), (1, 2), (0, 3)]
    with pytest.raises(ValueError):
        B.interleave_shards([per[1], per[0]])            # shard sizes violate the stride layout


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, outdir, kp_all, mc_all, prev_bytes):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = np.arange(rank, len(kp_all), world)
        kp_all_r, mc_all_r = B.exchange_counts(kp_all[mine], mc_all[mine], world, "cpu")
        cond = B.Conditions(requiredExtractedPointsCount=100, requiredMatchedPointsCount=500,
                            skipFramesFromBatchHead=0, useFirstFitInBatch=True)
        good, in_batch = B.select_global(kp_all_r, mc_all_r, cond)
        owner, li = B.owner_of(in_batch[good], world) if good >= 0 else (-1, -1)
        # the previous good frame's descriptors travel from their owner (rank 1)
        buf = torch.zeros(len(prev_bytes) + 16, dtype=torch.uint8)
        if rank == 1:
            buf[:len(prev_bytes)] = torch.from_numpy(prev_bytes)
        B.broadcast_prev(buf, len(prev_bytes), 1, world)
        # bench.py's form: third column (descriptor counts), known pad length and
        # the broadcast issued asynchronously
        dc = kp_all[mine] * 3 + rank
        kp2, mc2, dc2 = B.exchange_counts(kp_all[mine], mc_all[mine], world, "cpu", extra=dc, pad_to=5)
        buf2 = torch.zeros(len(prev_bytes), dtype=torch.uint8)
        if rank == 1:
            buf2[:] = torch.from_numpy(prev_bytes[::-1].copy())
        dist.broadcast(buf2, src=1, async_op=True).wait()
        res = {"kp2": kp2.tolist(), "mc2": mc2.tolist(), "dc2": dc2.tolist(),
               "prev2_ok": bool(np.array_equal(buf2.numpy(), prev_bytes[::-1])),
               "kp": kp_all_r.tolist(), "mc": mc_all_r.tolist(), "good": int(good),
               "in_batch": in_batch.tolist(), "owner": owner, "local": li,
               "prev_ok": bool(np.array_equal(buf[:len(prev_bytes)].numpy(), prev_bytes)),
               "tail_untouched": bool((buf[len(prev_bytes):] == 0).all())}
        json.dump(res, open(os.path.join(outdir, f"r{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


def test_sharded_exchange_and_selection_gloo_world2():
    import torch.multiprocessing as mp
    rng = np.random.default_rng(7)
    n = 9                                                  # ragged: rank 0 owns 5, rank 1 owns 4
    kp_all = rng.integers(50, 400, n).astype(np.int32)
    kp_all[[2, 5]] = [20, 30]                              # filtered out of the batch
    mc_all = rng.integers(0, 1200, n).astype(np.int32)
    prev = rng.integers(0, 256, 1000).astype(np.uint8)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_main, args=(2, _free_port(), d, kp_all, mc_all, prev), nprocs=2, join=True)
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(2)]
    in_batch = np.nonzero(kp_all >= 100)[0]
    good = O.select_good(mc_all[in_batch], 500, 0, 1)
    for r in res:
        assert r["kp"] == kp_all.tolist() and r["mc"] == mc_all.tolist()
        assert r["in_batch"] == in_batch.tolist()
        assert r["good"] == good
        if good >= 0:
            assert (r["owner"], r["local"]) == (int(in_batch[good]) % 2, int(in_batch[good]) // 2)
        assert r["prev_ok"] and r["tail_untouched"]
        assert r["kp2"] == kp_all.tolist() and r["mc2"] == mc_all.tolist() and r["prev2_ok"]
        assert r["dc2"] == (kp_all * 3 + np.arange(n) % 2).tolist()


def test_orb_pattern_product_copy_matches_oracle():
    """the product's rBRIEF table (csrc/orb_pattern.h) equals the oracle's copy"""
    import re
    def table(path):
        txt = open(path).read()
        return [int(v) for v in re.findall(r"-?\d+", txt[txt.index("{"):txt.index("}")])]
    a = table(os.path.join(ROOT, "slam-indoor-code_amd", "csrc", "orb_pattern.h"))
    b = table(os.path.join(ROOT, "oracle", "orb_pattern.h"))
    assert len(a) == 1024 and a == b


def _search_rank_main(rank, world, port, outdir, frames, first, batches, use_pad=False):
    """ShardedScan.search + advance over several searches, gloo on the CPU, the
    per-candidate work on the oracle (tests/oracle_ops.OracleBatchEngine)"""
    import torch
    import torch.distributed as dist
    from oracle_ops import OracleBatchEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = OracleBatchEngine()
        scan = B.ShardedScan(rank, world, engine=eng, device="cpu")
        cond = B.Conditions(featureExtractingThreshold=12, requiredExtractedPointsCount=50,
                            requiredMatchedPointsCount=40, matcherType=1, knnMatcherDistance=0.7)
        prev = torch.zeros(200000, dtype=torch.uint8)
        owner, nprev = 0, 0
        if rank == 0:                                   # the first good frame's descriptors live on rank 0
            d0 = O.sift(first, O.fast(first, 12, True))
            b = eng.pack(d0)
            prev[:len(b)] = torch.from_numpy(b)
            nprev = len(d0)
        t = torch.tensor([nprev], dtype=torch.int32)
        dist.broadcast(t, src=0)
        nprev = int(t.item())
        out = []
        for lo, hi in batches:
            local = frames[lo:hi][scan.shard(hi - lo)]
            pad = (hi - lo + world - 1) // world if use_pad else None      # bench.py's fixed all-gather rows
            good, kp_all, mc_all, in_batch, dc_all = scan.search(local, prev, nprev, owner, cond, pad_to=pad)
            wk, wm = scan.winner(good, in_batch, dc_all, mc_all, nprev)
            owner, nprev = scan.advance(good, in_batch, dc_all, prev, owner, nprev)
            out.append({"good": int(good), "kp": kp_all.tolist(), "mc": mc_all.tolist(), "dc": dc_all.tolist(),
                        "owner": owner, "nprev": nprev,
                        "wk": None if wk is None else wk.tobytes().hex(), "wm": None if wm is None else wm.tobytes().hex()})
        json.dump(out, open(os.path.join(outdir, f"s{rank}.json"), "w"))
    finally:
        dist.destroy_process_group()


def test_sharded_search_gloo_world2():
    """ShardedScan.search / advance at world 2 against a single-process oracle
    run of the same searches: per-candidate counts, selection, winner hand-over
    (the next query is the winner's descriptors, broadcast from its owner), and
    a one-candidate batch that leaves rank 1 with an empty shard"""
    import torch.multiprocessing as mp
    import slamhip
    frames = slamhip.synth_frames(160, 120, 0, 9, seed=1234)
    first = frames[0]
    batches = [(1, 6), (6, 7), (7, 9)]               # 5 candidates, then 1 (rank 1 empty), then 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_search_rank_main, args=(2, _free_port(), d, frames, first, batches), nprocs=2, join=True)
        res = [json.load(open(os.path.join(d, f"s{r}.json"))) for r in range(2)]
    assert res[0] == res[1]
    # single-process reference of the same searches
    prev = O.sift(first, O.fast(first, 12, True))
    for (lo, hi), r in zip(batches, res[0]):
        kc, mc, dc, ds = [], [], [], []
        for f in frames[lo:hi]:
            k = O.fast(f, 12, True)
            dd = O.sift(f, k)
            idx, dist = O.knn2(prev, dd, O.NORM_L2)
            kc.append(len(k)); dc.append(len(dd)); ds.append(dd)
            mc.append(len(O.ratio(idx, dist, 0.7)))
        assert r["kp"] == kc and r["mc"] == mc and r["dc"] == dc
        in_batch = np.nonzero(np.array(kc) >= 50)[0]
        good = O.select_good(np.array(mc)[in_batch], 40, 0, 1) if len(in_batch) else -2
        assert r["good"] == good
        if good >= 0:
            gi = int(in_batch[good])
            assert r["owner"] == gi % 2 and r["nprev"] == dc[gi]
            # the winner's keypoints and matches, broadcast from its owner to every rank
            k = O.fast(frames[lo + gi], 12, True)
            idx, dist = O.knn2(prev, ds[gi], O.NORM_L2)
            assert r["wk"] == k.tobytes().hex() and r["wm"] == O.ratio(idx, dist, 0.7).tobytes().hex()
            prev = ds[gi]
    assert any(r["good"] >= 0 for r in res[0])


@pytest.mark.parametrize("world,n", [(2, 21), (3, 22)])
def test_sharded_search_ragged_gloo(world, n):
    """configs[3]'s ragged layout (framesBatchSize 210 over 8 ranks is 27 / 26
    per rank): n candidates over `world` ranks by the thread stride
    (batch.cpp:181-187), the all-gather padded to ceil(n / world) rows as
    bench.py runs it, checked against one single-rank search of the same
    candidates (counts in global order, selection, winner, hand-over)"""
    import torch.multiprocessing as mp
    import slamhip
    frames = slamhip.synth_frames(160, 120, 0, n + 1, seed=1234)
    batches = [(1, n + 1)]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_search_rank_main, args=(world, _free_port(), d, frames, frames[0], batches, True), nprocs=world,
                 join=True)
        res = [json.load(open(os.path.join(d, f"s{r}.json"))) for r in range(world)]
    assert all(r == res[0] for r in res)
    prev = O.sift(frames[0], O.fast(frames[0], 12, True))
    kc, mc, dc = [], [], []
    for f in frames[1:]:
        k = O.fast(f, 12, True)
        dd = O.sift(f, k)
        idx, dist = O.knn2(prev, dd, O.NORM_L2)
        kc.append(len(k)); dc.append(len(dd)); mc.append(len(O.ratio(idx, dist, 0.7)))
    r = res[0][0]
    assert r["kp"] == kc and r["mc"] == mc and r["dc"] == dc
    in_batch = np.nonzero(np.array(kc) >= 50)[0]
    good = O.select_good(np.array(mc)[in_batch], 40, 0, 1)
    assert r["good"] == good and good >= 0
    gi = int(in_batch[good])
    assert r["owner"] == gi % world and r["nprev"] == dc[gi]


def test_device_only_frames_refuse_host_paths():
    """DeviceMedia(None, dev) frames hold no host pixels (a zero
    placeholder); every host-pixel operation raises instead of processing black
    images (GpuOps.describe / match_frame, the host scan of
    find_good_frame_from_batch)."""
    import torch
    from slamhip import cycle
    dev = torch.zeros((3, 8, 8, 3), dtype=torch.uint8)
    media = cycle.DeviceMedia(None, dev)
    f = media.next_frame()
    assert f.host_valid is False
    with pytest.raises(ValueError):
        cycle._host_pixels(f)
    host = cycle.DeviceMedia(np.ones((3, 8, 8, 3), np.uint8), dev).next_frame()
    assert cycle._host_pixels(host).sum() == 8 * 8 * 3
