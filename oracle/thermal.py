"""Exact optimum of the reference's thermal integer programme -- TEST INFRASTRUCTURE ONLY.

The reference MILP (`dragg/mpc_calc.py:291-446`) separates (checked by
`tests/test_oracle_golden.py::test_model_is_separable`) into
  * the thermal integer part: indoor air T driven by the hvac duty of the season's mode
    (`mpc_calc.py:303-324`) and the tank Tw driven by the water-heater duty and by T
    (`mpc_calc.py:329-340`), duties integer in 0..S (`mpc_calc.py:171-173, 344-349`);
  * the battery LP and the PV LP.
Each thermal part is one integer chain

    x_{k+1} = A_k x_k + C_k + g u_k,   u_k in {0..S},   x_1 in [lo0, hi0],  x_{k+1} in [lo, hi],
    minimise sum_k q_k u_k,            q_k = gamma^k price_k * (duty power) * S

solved here by an assumption-free BACKWARD dynamic programme over exact step functions:
V_k(x) = min_u q_k u + V_{k+1}(A_k x + C_k + g u) is piecewise constant in x; it is carried
as its sorted breakpoints and values (no grid, no dominance rule, any sign of q), then the
optimal schedule is recovered forward by evaluating V_{k+1} at the exact successor states.
This is the independent checker of the GPU's forward Pareto-front DP (`dp_front`), which
relies on a monotonicity property this module does not assume.

The tank chain depends on T through its C_k (`mpc_calc.py:330-332`, coefficient e ~ 4e-5):
`thermal_optimum` solves T first and Tw given that T, as the GPU does; whether that can miss
the joint optimum is checked against HiGHS on the full model by the proven-optimum fixtures
(tests/golden/proven/).  Boxes are widened by the same 1e-9 relative tolerance as the kernel.
"""
import numpy as np

TOL = 1e-9
TAP = 15.0        # mpc_calc.py:181


def _tol(v):
    return TOL * (1 + abs(v))


def chain_T(hc, si):
    """Indoor-air chain of one solve (`mpc_calc.py:303-324, 344-349, 441-446`).

    The season picks the active duty: heating (h, g > 0) when max(oat + noise) <= 30, cooling
    (c, g < 0) otherwise (`mpc_calc.py:303-309`)."""
    H, S, dt = hc.H, hc.S, hc.dt
    inv_c = 1.0 / (hc.C * dt)
    iR = 1.0 / hc.R
    aT = 1.0 + (-iR * 3600) * inv_c
    if si.winter:
        g, P = hc.Ph * 3600 * inv_c, hc.Ph
    else:
        g, P = -(hc.Pc * 3600 * inv_c), hc.Pc
    w = np.power(hc.discount * np.ones(H), np.arange(H)) * np.asarray(si.price, float)[:H]
    oat = np.asarray(si.oat, float)
    return dict(A=np.full(H, aT), C=oat[1:H + 1] * iR * 3600 * inv_c, q=w * (S * P), g=g, x0=float(si.T0),
                lo0=hc.Tmin, hi0=hc.Tmax, lo=hc.Tmin, hi=hc.Tmax, S=S)


def chain_W(hc, si, T_path):
    """Tank chain given the indoor-air trajectory T_1..T_H (`mpc_calc.py:329-340`).  The
    un-mixed one-step value temp_wh (`mpc_calc.py:336-340`) differs from Tw_1 by a constant,
    so its bounds tighten the box of Tw_1 (lo0, hi0)."""
    H, S, dt = hc.H, hc.S, hc.dt
    inv_w = 1.0 / (hc.Cw * dt)
    iRw = 1.0 / hc.Rw
    draw = np.asarray(si.draw, float)
    df = draw[1:H + 1] / hc.V
    rem = 1 - df
    d15 = df * TAP
    e = iRw * 3600 * inv_w
    f = hc.Pw * 3600 * inv_w
    A = rem + (-rem * iRw) * 3600 * inv_w
    C = e * np.asarray(T_path, float) + (d15 + ((-d15) * iRw) * 3600 * inv_w)
    Tw0 = float(si.Tw0)
    c0 = rem[0] + (-rem[0] * iRw) * 3600 * inv_w
    dd0 = d15[0] + ((-d15[0]) * iRw) * 3600 * inv_w
    Kc = (Tw0 + ((-Tw0) * iRw) * 3600 * inv_w) - c0 * Tw0 - dd0
    w = np.power(hc.discount * np.ones(H), np.arange(H)) * np.asarray(si.price, float)[:H]
    return dict(A=A, C=C, q=w * (S * hc.Pw), g=f, x0=Tw0, lo0=max(hc.Twmin, hc.Twmin - Kc),
                hi0=min(hc.Twmax, hc.Twmax - Kc), lo=hc.Twmin, hi=hc.Twmax, S=S)


def _box(ch, k):
    """Tolerance-widened box of x_{k+1}."""
    lo, hi = (ch["lo0"], ch["hi0"]) if k == 0 else (ch["lo"], ch["hi"])
    return lo - _tol(lo), hi + _tol(hi)


def value_functions(ch):
    """Backward step-function DP.  Returns [V_1 .. V_H] as (breakpoints, values): V_k(x) =
    values[i] for breakpoints[i] <= x < breakpoints[i+1] (inf outside)."""
    A, C, q, g, S = ch["A"], ch["C"], ch["q"], ch["g"], ch["S"]
    H = len(A)
    lo, hi = _box(ch, H - 1)
    V = [None] * (H + 1)
    V[H] = (np.array([lo, hi]), np.array([0.0]))
    for k in range(H - 1, 0, -1):                      # V_k over the box of x_k
        B, val = V[k + 1]
        cands = [((B - C[k] - g * u) / A[k], val + q[k] * u) for u in range(S + 1)]
        blo, bhi = _box(ch, k - 1)
        pts = np.unique(np.clip(np.concatenate([c[0] for c in cands]), blo, bhi))
        if len(pts) < 2:
            return None
        mid = 0.5 * (pts[:-1] + pts[1:])
        best = np.full(len(mid), np.inf)
        for Bu, Vu in cands:
            i = np.searchsorted(Bu, mid, side="right") - 1
            ok = (i >= 0) & (i < len(Vu))
            best = np.minimum(best, np.where(ok, Vu[np.clip(i, 0, len(Vu) - 1)], np.inf))
        keep = np.ones(len(best), bool)
        keep[1:] = best[1:] != best[:-1]
        V[k] = (np.r_[pts[:-1][keep], pts[-1]], best[keep])
    return V


def _eval(Vk, x):
    B, val = Vk
    if x < B[0] or x > B[-1]:
        return np.inf
    i = min(int(np.searchsorted(B, x, side="right")) - 1, len(val) - 1)
    return float(val[i])


def solve_chain(ch):
    """Exact optimum of one chain: (cost, duties[H], states x_1..x_H) or None if no schedule."""
    A, C, q, g, S = ch["A"], ch["C"], ch["q"], ch["g"], ch["S"]
    H = len(A)
    V = value_functions(ch)
    if V is None:
        return None
    x, cost, us, xs = ch["x0"], 0.0, [], []
    for k in range(H):
        lo, hi = _box(ch, k)
        best, bu, bx = np.inf, -1, None
        for u in range(S + 1):
            xn = A[k] * x + (g * u + C[k])
            if not (lo <= xn <= hi):
                continue
            v = q[k] * u + (_eval(V[k + 1], xn) if k + 1 < H else 0.0)
            if v < best:
                best, bu, bx = v, u, xn
        if bu < 0:
            return None
        us.append(bu)
        xs.append(bx)
        cost += q[k] * bu
        x = bx
    return cost, np.array(us), np.array(xs)


def thermal_optimum(hc, si):
    """Sequential exact optimum: indoor air, then the tank given that indoor trajectory.
    Returns dict(cost, cost_T, cost_W, u_T, x_T, u_W, x_W) or None if either chain has no
    integer schedule."""
    T = solve_chain(chain_T(hc, si))
    if T is None:
        return None
    W = solve_chain(chain_W(hc, si, T[2]))
    if W is None:
        return None
    return dict(cost=T[0] + W[0], cost_T=T[0], cost_W=W[0], u_T=T[1], x_T=T[2], u_W=W[1], x_W=W[2])


def brute_force(ch):
    """Enumeration of every duty schedule (tiny chains only): the checker's own checker."""
    import itertools
    A, C, q, g, S = ch["A"], ch["C"], ch["q"], ch["g"], ch["S"]
    H = len(A)
    best = None
    for us in itertools.product(range(S + 1), repeat=H):
        x, ok = ch["x0"], True
        for k, u in enumerate(us):
            x = A[k] * x + (g * u + C[k])
            lo, hi = _box(ch, k)
            if not (lo <= x <= hi):
                ok = False
                break
        if ok:
            c = float(np.dot(q, us))
            if best is None or c < best:
                best = c
    return best


def exact_milp(hc, si, th="solve"):
    """The optimum of the reference's whole MILP (`mpc_calc.py:291-451`) for one solve, or None
    if it is infeasible: the integer columns fixed to the exact thermal schedule `th`
    (`thermal_optimum`, computed here unless given), the remaining columns (battery, PV, grid,
    cost) solved as an LP by HiGHS.  The model is separable (no row
    couples the duty columns with the battery / PV columns, only the linear objective), so the
    LP optimum is the MILP optimum; tests/test_oracle_thermal.py pins this against every
    fixture record HiGHS proved optimal or infeasible."""
    from scipy.optimize import linprog
    from oracle import mpc as M
    if isinstance(th, str):
        th = thermal_optimum(hc, si)
    if th is None:
        return None
    P = M.build_problem(hc, si)
    Lay = P["layout"]
    n = P["c"].shape[0]
    lb, ub = np.full(n, -np.inf), np.full(n, np.inf)
    on, off = ("hvac_heat_on", "hvac_cool_on") if si.winter else ("hvac_cool_on", "hvac_heat_on")
    for key, vals in ((on, th["u_T"]), (off, np.zeros(hc.H)), ("wh_heat_on", th["u_W"])):
        o = Lay.off[key]
        lb[o:o + hc.H] = ub[o:o + hc.H] = np.asarray(vals, float)
    res = linprog(P["c"], A_ub=P["A_ub"], b_ub=P["b_ub"], A_eq=P["A_eq"], b_eq=P["b_eq"],
                  bounds=list(zip(lb, ub)), method="highs")
    return float(res.fun) if res.status == 0 else None
