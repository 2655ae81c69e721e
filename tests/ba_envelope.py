"""BA window parity against the oracle on identical inputs -- TEST INFRASTRUCTURE
(the checker of tests/test_cycle_1080p.py and of bench.py's pipeline leg).

bundleAdjustment (bundleAdjustment.cpp:73-129) solves one window with Ceres's
LM on BAThreadsCnt threads (:111), whose residual / gradient / Schur sums are
partitioned by thread: the reference itself has no single summation order.
The GPU sums in its own order, so a window is compared with oracle/ba.c run on
the SAME inputs (the GPU run's recorded window, not the oracle pipeline's,
whose earlier windows may already have moved the poses):

  * final cost within 1e-6 relative and RMSE within 1e-4 px of the oracle
    (north_star's bar) -- whether or not the oracle converged;
  * otherwise, when the oracle runs into the 50-iteration cap (no convergence:
    every step is still moving, so 1e-15 summation differences grow along the
    LM path): the oracle's own reordering envelope -- the same window with its
    observations in n different orders (order 0 = the reference's
    AddResidualBlock order; odd orders shuffle the observations inside each
    frame; even orders shuffle all of them and relabel the points, which
    reorders the oracle's per-point Schur accumulation as Ceres's multithreaded
    eliminator does), the spread valid summation orders produce.  The GPU's final cost must lie in the raw [lo, hi] ("ok").
    With n orders a further valid order falls outside it with probability
    2 / (n + 1): 16 orders first, and 64 when the GPU falls outside the 16
    (both counts reported);
  * a converged oracle outside the 1e-6 / 1e-4 px bar fails.

A window outside the capped envelope can also be re-solved without the cap
(`resolve`, <= 500 iterations, on the GPU) beside the oracle's own orders at
<= 500 iterations: "converged" then says whether both converge and the GPU's
optimum lies inside the oracle's envelope of optima.  It is evidence about the
solver, reported, not a pass ("ok" stays False).

Beside "ok", every window reports north_star's own bar -- "BA reprojection
error within 1e-4 px of the Ceres reference" -- as "north_star_ok" (RMSE
alone; the 1e-6 relative cost bar is this suite's, ~200x stricter at 1 px
RMSE), and the tier "ok" passed ("cost", "envelope" or None).

Also reported per window: observations, points observed, points with a single
observation (a born-once track: the snapshot quirk of SURVEY 8(a) -- its V
block has rank 2, so only the LM damping holds it along its viewing ray), the
largest |point change| between the GPU and order-0 oracle solutions, and
whether that point is a runaway (|X| > 1e4 m) in both runs.
"""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle_ffi as O

COST_REL = 1e-6
RMSE_PX = 1e-4


def _order(of, s):
    """observation order s: 0 = as given; odd s = a random order inside each
    frame; even s > 0 = a random order of all observations"""
    if s == 0:
        return np.arange(len(of))
    if s % 2 == 0:
        return np.random.default_rng(s).permutation(len(of))
    return np.lexsort((np.random.default_rng(s).random(len(of)), of))


def oracle_order(w, s, max_iters=50, trace=None, solver=0):
    """oracle/ba.c on window w with its observations in order s (see _order);
    solver: O.BA_SOLVER_LLT / _LDLT, the reduced system's factorisation"""
    of, op, oxy = w["obs_frame"], w["obs_point"], w["obs_xy"]
    idx = _order(of, s)
    if s > 0 and s % 2 == 0:
        # point i of the relabelled window is point perm[i]: the same problem,
        # its points' Schur contributions summed in another order
        perm = np.random.default_rng(1_000_003 + s).permutation(len(w["pts"]))
        inv = np.empty_like(perm)
        inv[perm] = np.arange(len(perm))
        return O.ba(w["K4"], w["ext"], w["pts"][perm], of[idx], inv[op[idx]], oxy[idx], w["loss"], w["loss_param"],
                    max_iters=max_iters, trace=trace, solver=solver)
    return O.ba(w["K4"], w["ext"], w["pts"], of[idx], op[idx], oxy[idx], w["loss"], w["loss_param"],
                max_iters=max_iters, trace=trace, solver=solver)


def lm_path_envelope(w, kmax, orders=16, threads=8, solvers=(0, 1)):
    """The oracle's cost after each LM iteration k = 1..kmax (trace[k - 1] = a
    run capped at k) over `orders` observation orders under each factorisation
    in `solvers` -- the dense LL' restatement and Eigen SimplicialLDLT's
    arithmetic, the solver the reference's configuration runs (Ceres 2.2,
    SPARSE_SCHUR on EIGEN_SPARSE, bundleAdjustment.cpp:108-114).  Its AMD
    ordering cannot be restated, so neither factorisation's rounding is the
    reference's; both bound its variety together with the order of the sums
    (the reference's BAThreadsCnt threads partition them).  Returns (lo, hi,
    traces[solver][order][k])."""
    def one(job):
        sv, s = job
        tr = np.zeros(kmax, np.float64)
        oracle_order(w, s, max_iters=kmax, trace=tr, solver=sv)
        return tr
    jobs = [(sv, s) for sv in solvers for s in range(orders)]
    with ThreadPoolExecutor(threads) as ex:
        tr = np.stack(list(ex.map(one, jobs))).reshape(len(solvers), orders, kmax)
    return tr.min((0, 1)), tr.max((0, 1)), tr


def lm_path_check(w, gpu_costs, ks, orders=16, orders_max=64, threads=8):
    """gpu_costs[i] = the GPU's cost capped at ks[i] iterations.  Inside the
    envelope of lm_path_envelope at every k (16 orders per factorisation; a k
    outside it is tried again with orders_max, as the endpoint check does).
    Returns a per-k table and the verdict."""
    kmax = max(ks)
    rows, ok = [], True
    lo, hi, _ = lm_path_envelope(w, kmax, orders, threads)
    wide = None
    for k, g in zip(ks, gpu_costs):
        i = k - 1
        n = orders
        l, h = lo[i], hi[i]
        if not (l <= g <= h) and orders_max > orders:
            if wide is None:
                wide = lm_path_envelope(w, kmax, orders_max, threads)
            l, h, n = wide[0][i], wide[1][i], orders_max
        inside = bool(l <= g <= h)
        ok = ok and inside
        width = max(h - l, 1e-300)
        rows.append({"k": int(k), "gpu": float(g), "lo": float(l), "hi": float(h), "orders": int(n),
                     "width_rel": float((h - l) / max(abs(l), 1e-300)), "pos": float((g - l) / width),
                     "inside": inside})
    return {"ok": ok, "rows": rows}


def window_vs_oracle(io, summary, orders=16, threads=8, orders_max=64, resolve=None, resolve_iters=500):
    """io: {"in": inputs dict (K4, ext, pts, obs_frame, obs_point, obs_xy, loss,
    loss_param), "out": (K4, ext, pts) of the GPU solve}; summary: the GPU's
    slam_ba_summary.  Returns a dict with the verdict under "ok"."""
    w = io["in"]
    of, op, oxy = w["obs_frame"], w["obs_point"], w["obs_xy"]
    loss, a = w["loss"], w["loss_param"]
    nres = 2 * len(of)

    def run(s, max_iters=50):
        return oracle_order(w, s, max_iters)

    base = run(0)
    rs = base[3]
    converged = rs.termination == 1 and rs.iterations < 50
    rmse = lambda c: math.sqrt(c / max(1, nres))
    g_cost, o_cost = summary.final_cost, rs.final_cost
    res = {"observations": int(len(of)), "gpu_final_cost": g_cost, "oracle_final_cost": o_cost,
           "gpu_rmse": rmse(g_cost), "oracle_rmse": rmse(o_cost), "gpu_iterations": int(summary.iterations),
           "oracle_iterations": int(rs.iterations), "oracle_converged": bool(converged),
           "initial_cost_rel_diff": abs(summary.initial_cost - rs.initial_cost) / max(rs.initial_cost, 1e-300),
           "rmse_abs_diff_px": abs(rmse(g_cost) - rmse(o_cost)),
           "final_cost_rel_diff": abs(g_cost - o_cost) / max(o_cost, 1e-300)}
    cnt = np.bincount(op, minlength=len(w["pts"]))
    seen = cnt > 0
    res["points_observed"] = int(seen.sum())
    res["points_single_observation"] = int((cnt == 1).sum())
    gp, rp = io["out"][2], base[2]
    d = np.abs(gp - rp).max(1)
    d[~seen] = 0.0
    k = int(np.argmax(d))
    res["points_max_abs_diff"] = float(d[k])
    res["points_max_diff_point"] = {"observations": int(cnt[k]), "gpu_norm": float(np.linalg.norm(gp[k])),
                                    "oracle_norm": float(np.linalg.norm(rp[k])),
                                    "runaway_in_both": bool(np.linalg.norm(gp[k]) > 1e4 and
                                                            np.linalg.norm(rp[k]) > 1e4)}
    res["points_runaway"] = {"gpu": int((np.linalg.norm(gp[seen], axis=1) > 1e4).sum()),
                             "oracle": int((np.linalg.norm(rp[seen], axis=1) > 1e4).sum())}
    res["points_max_abs_diff_multi_obs"] = float(d[cnt >= 2].max()) if (cnt >= 2).any() else 0.0
    res["north_star_ok"] = bool(res["rmse_abs_diff_px"] <= RMSE_PX)
    if res["final_cost_rel_diff"] <= COST_REL and res["rmse_abs_diff_px"] <= RMSE_PX:
        res["bar"] = f"final cost {COST_REL:g} rel and RMSE {RMSE_PX:g} px of the oracle"
        res["tier"] = "cost"
        res["ok"] = True
        return res
    if converged:
        res["bar"] = f"oracle converged: final cost {COST_REL:g} rel, RMSE {RMSE_PX:g} px"
        res["tier"] = None
        res["ok"] = False
        return res
    env = [o_cost]
    with ThreadPoolExecutor(threads) as ex:
        for n in (orders, orders_max):
            env += [r[3].final_cost for r in ex.map(run, range(len(env), n))]
            lo, hi = min(env), max(env)
            if lo <= g_cost <= hi:
                break
    wd = hi - lo
    res["envelope"] = {"orders": len(env), "final_cost_min": lo, "final_cost_max": hi, "width": wd,
                       "width_rel": wd / o_cost, "rmse_min": rmse(lo), "rmse_max": rmse(hi),
                       "rmse_width_px": rmse(hi) - rmse(lo)}
    # north_star's 1e-4 px against the oracle's own spread: when valid summation
    # orders of the oracle itself spread their RMSE wider than the bar, no
    # implementation can be held to it on this window (reported, not barred)
    res["oracle_rmse_spread_px"] = rmse(hi) - rmse(lo)
    res["north_star_attainable"] = bool(res["oracle_rmse_spread_px"] <= RMSE_PX)
    inside = bool(lo <= g_cost <= hi)
    res["envelope"]["gpu_outside_rel"] = 0.0 if inside else min(abs(g_cost - lo), abs(g_cost - hi)) / o_cost
    res["bar"] = (f"oracle at the 50-iteration cap and the GPU beyond {COST_REL:g} rel / {RMSE_PX:g} px: GPU final "
                  f"cost inside the raw reordering envelope [min, max] of {orders} orders, else of {orders_max} "
                  "(a window outside it fails)")
    res["tier"] = "envelope" if inside else None
    res["ok"] = inside
    if not inside and resolve is not None:
        g = resolve(w, resolve_iters)        # the GPU's summary without the cap
        with ThreadPoolExecutor(threads) as ex:
            rs2 = [r[3] for r in ex.map(lambda s: run(s, resolve_iters), range(orders))]
        oc = [r.final_cost for r in rs2]
        all_conv = g.termination == 1 and all(r.termination == 1 for r in rs2)
        res["converged"] = {"max_iters": resolve_iters, "orders": orders, "gpu_final_cost": g.final_cost,
                            "gpu_iterations": int(g.iterations), "oracle_min": min(oc), "oracle_max": max(oc),
                            "oracle_iterations": [int(r.iterations) for r in rs2], "all_converged": bool(all_conv),
                            "gpu_inside": bool(all_conv and min(oc) <= g.final_cost <= max(oc))}
    return res
