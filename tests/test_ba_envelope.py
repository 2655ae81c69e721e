"""The BA window checker's tiers (tests/ba_envelope.py) on the oracle alone:
identical results pass the cost tier, a converged oracle never falls back to a
looser tier, and at the iteration cap a window outside the raw envelope fails
(north_star's 1e-4 px RMSE bar is reported beside it, not as a pass)."""
import math
import types

import numpy as np

import ba_envelope
import oracle_ffi as O
from slamhip import synthba


def _window():
    w = synthba.make_window(nframes=3, npoints=120, seed=5)
    w.update(loss=O.LOSS_NONE, loss_param=0.0)
    return w, O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"])


def _summary(rs, cost):
    return types.SimpleNamespace(final_cost=cost, initial_cost=rs.initial_cost, iterations=rs.iterations)


def test_identical_window_passes_cost_tier():
    w, (K4, ext, pts, rs) = _window()
    r = ba_envelope.window_vs_oracle({"in": w, "out": (K4, ext, pts)}, _summary(rs, rs.final_cost), threads=1)
    assert r["ok"] and r["tier"] == "cost" and r["final_cost_rel_diff"] == 0.0


def test_converged_oracle_rejects_cost_gap(monkeypatch):
    """the oracle reported converged (synthba's windows run to the cap: their
    born-once tracks keep moving), a 1e-5 cost gap: no envelope, no RMSE tier"""
    w, (K4, ext, pts, rs) = _window()
    real = O.ba

    def converged(*a, **k):
        out = real(*a, **k)
        out[3].iterations, out[3].termination = 12, 1
        return out
    monkeypatch.setattr(ba_envelope.O, "ba", converged)
    r = ba_envelope.window_vs_oracle({"in": w, "out": (K4, ext, pts)}, _summary(rs, rs.final_cost * (1 + 1e-5)),
                                     threads=1)
    assert r["rmse_abs_diff_px"] <= 1e-4
    assert not r["ok"] and r["tier"] is None and "envelope" not in r


def test_capped_oracle_outside_envelope_fails(monkeypatch):
    """the oracle forced to 'at the cap', each order's cost spread by 1e-7 relative"""
    w, (K4, ext, pts, rs) = _window()
    real = O.ba

    def capped(*a, **k):
        out = real(*a, **k)
        s = out[3]
        s.iterations, s.termination = 50, 0
        s.final_cost *= 1 + 1e-7 * (np.random.default_rng(int(a[3].sum() * 1e3) % 2**32).random() - 0.5)
        return out
    monkeypatch.setattr(ba_envelope.O, "ba", capped)
    base = ba_envelope.O.ba(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"])[3].final_cost
    io = {"in": w, "out": (K4, ext, pts)}
    # the spread is ~1e-7, so a 2e-6 gap is outside the envelope: a failure,
    # with north_star's RMSE bar met and reported
    nres = 2 * len(w["obs_frame"])
    r = ba_envelope.window_vs_oracle(io, _summary(rs, base * (1 + 2e-6)), orders=4, orders_max=8, threads=1)
    assert r["envelope"]["orders"] == 8 and r["envelope"]["gpu_outside_rel"] > 0
    assert not r["ok"] and r["tier"] is None and r["north_star_ok"]
    # inside the envelope: passes
    r = ba_envelope.window_vs_oracle(io, _summary(rs, base), orders=4, orders_max=8, threads=1)
    assert r["ok"] and r["tier"] in ("cost", "envelope")
    # an RMSE gap beyond 1e-4 px: north_star's bar missed too
    far = (math.sqrt(base / nres) + 2e-4) ** 2 * nres
    r = ba_envelope.window_vs_oracle(io, _summary(rs, far), orders=4, orders_max=8, threads=1)
    assert not r["ok"] and not r["north_star_ok"]


def test_capped_window_converged_evidence(monkeypatch):
    """outside the capped envelope with a resolver: both re-solved without the
    cap; the GPU optimum inside the oracle's envelope of optima is reported as
    evidence, "ok" stays False"""
    w, (K4, ext, pts, rs) = _window()
    real = O.ba

    def capped(*a, max_iters=50, **k):
        out = real(*a, max_iters=max_iters, **k)
        s = out[3]
        if max_iters <= 50:
            s.iterations, s.termination = 50, 0
        s.final_cost *= 1 + 1e-7 * (np.random.default_rng(int(a[3].sum() * 1e3) % 2**32).random() - 0.5)
        return out
    monkeypatch.setattr(ba_envelope.O, "ba", capped)
    base = real(w["K4"], w["ext"], w["pts"], w["obs_frame"], w["obs_point"], w["obs_xy"], max_iters=500)[3].final_cost
    io = {"in": w, "out": (K4, ext, pts)}
    calls = []

    def resolve(win, iters):
        calls.append(iters)
        return types.SimpleNamespace(final_cost=base, termination=1, iterations=80)
    r = ba_envelope.window_vs_oracle(io, _summary(rs, rs.final_cost * (1 + 2e-6)), orders=4, orders_max=8, threads=1,
                                     resolve=resolve)
    assert calls == [500] and not r["ok"]
    c = r["converged"]
    assert c["all_converged"] and c["oracle_min"] <= c["oracle_max"] and len(c["oracle_iterations"]) == 4
    assert c["gpu_inside"] == (c["oracle_min"] <= base <= c["oracle_max"])


def test_lm_path_check_on_the_oracle_itself():
    """lm_path_check (the per-iteration bar of test_ba_b210_lm_path_per_iteration):
    the oracle's own order-0 LL' trace and its SimplicialLDLT trace lie inside
    the envelope at every k; a cost moved by one envelope width above it at
    k = 1 is reported outside (and the verdict fails)"""
    w = synthba.make_window(nframes=4, npoints=200, seed=11)
    w.update(loss=O.LOSS_HUBER, loss_param=4.0)
    ks = [1, 2, 3, 5]
    lo, hi, tr = ba_envelope.lm_path_envelope(w, max(ks), orders=4, threads=2)
    assert tr.shape == (2, 4, 5) and (lo <= hi).all()
    for sv in (0, 1):
        g = [tr[sv, 0, k - 1] for k in ks]
        r = ba_envelope.lm_path_check(w, g, ks, orders=4, orders_max=4, threads=2)
        assert r["ok"] and [x["k"] for x in r["rows"]] == ks
    g = [tr[0, 0, k - 1] for k in ks]
    g[0] = hi[0] + max(hi[0] - lo[0], abs(hi[0]) * 1e-9)
    r = ba_envelope.lm_path_check(w, g, ks, orders=4, orders_max=4, threads=2)
    assert not r["ok"] and not r["rows"][0]["inside"] and all(x["inside"] for x in r["rows"][1:])
