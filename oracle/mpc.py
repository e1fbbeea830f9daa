"""Numpy restatement of the reference's per-home MPC step (`dragg/mpc_calc.py`).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Every function cites the
reference lines it restates.  The MILP is assembled in the reference's own
variable and row order (the order cvxpy sees it: variables in creation order,
constraints in list order) and solved with scipy's HiGHS, the stand-in for the
absent GLPK_MI backend (`mpc_calc.py:141-145, 447-451`).

Redis is restated as a per-home dict of ``str`` values (redis-py with
`decode_responses=True`, `redis_client.py:16`): floats are stored as
``repr(float(x))`` so the fallback's first-character parse
(`mpc_calc.py:537-539`) sees exactly what the reference sees.
"""
from dataclasses import dataclass, field

import numpy as np

TAP_TEMP = 15.0  # mpc_calc.py:181

BASE_KEYS = ("p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "temp_in_ev_opt", "temp_wh_ev_opt",
             "hvac_cool_on_opt", "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws")  # :482
PV_KEYS = ("p_pv_opt", "u_pv_curt_opt")                       # :507
BATT_KEYS = ("p_batt_ch", "p_batt_disch", "e_batt_opt")       # :512


def enc(v):
    """Value as redis-py stores it (str); floats via repr (`redis_client.py:16` decode_responses)."""
    if isinstance(v, str):
        return v
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        return str(int(v))
    return repr(float(v))


# --------------------------------------------------------------------------------------------
# Per-home constants (setup_base_problem :134-191, setup_battery_problem :233-249,
# setup_pv_problem :251-262)
# --------------------------------------------------------------------------------------------
@dataclass
class HomeConst:
    name: str
    type: str
    S: int
    dt: int
    H: int
    discount: float
    R: float
    C: float           # c * 1000
    Pc: float          # p_c / S  (per duty unit)
    Ph: float
    Rw: float          # r * 1000
    Pw: float          # p / S
    Cw: float          # tank_size * 4.2
    V: float           # tank_size
    Tmin: float
    Tmax: float
    Twmin: float
    Twmax: float
    T_init: float
    Tw_init: float
    draw_sizes: list
    batt: dict = field(default_factory=dict)
    pv: dict = field(default_factory=dict)

    @property
    def has_batt(self):
        return "battery" in self.type       # :93 ('batt' in type at :602 is equivalent)

    @property
    def has_pv(self):
        return "pv" in self.type            # :96, :504, :600


def home_const(home):
    """`MPCCalc.setup_base_problem` + battery/pv setup (`mpc_calc.py:134-191, 233-262`)."""
    hems = home["hems"]
    S = max(1, int(hems["sub_subhourly_steps"]))
    dt = max(1, int(hems["hourly_agg_steps"]))
    H = max(1, int(hems["horizon"] * dt))
    batt, pv = {}, {}
    if "battery" in home["type"]:
        b = home["battery"]
        cap = float(b["capacity"])
        batt = dict(rate=float(b["max_rate"]), cap=cap,
                    Emin=float(b["capacity_lower"]) * cap, Emax=float(b["capacity_upper"]) * cap,
                    eta_c=float(b["ch_eff"]), eta_d=float(b["disch_eff"]),
                    E_init=float(b["e_batt_init"]) * cap)
    if "pv" in home["type"]:
        pv = dict(area=float(home["pv"]["area"]), eff=float(home["pv"]["eff"]))
    return HomeConst(
        name=home["name"], type=home["type"], S=S, dt=dt, H=H, discount=float(hems["discount_factor"]),
        R=float(home["hvac"]["r"]), C=float(home["hvac"]["c"]) * 1000,
        Pc=float(home["hvac"]["p_c"]) / S, Ph=float(home["hvac"]["p_h"]) / S,
        Rw=float(home["wh"]["r"]) * 1000, Pw=float(home["wh"]["p"]) / S,
        Cw=float(home["wh"]["tank_size"]) * 4.2, V=float(home["wh"]["tank_size"]),
        Tmin=float(home["hvac"]["temp_in_min"]), Tmax=float(home["hvac"]["temp_in_max"]),
        Twmin=float(home["wh"]["temp_wh_min"]), Twmax=float(home["wh"]["temp_wh_max"]),
        T_init=float(home["hvac"]["temp_in_init"]), Tw_init=float(home["wh"]["temp_wh_init"]),
        draw_sizes=list(home["wh"]["draw_sizes"]), batt=batt, pv=pv)


def max_load(hc):
    """`mpc_calc.py:191`."""
    return (max(hc.Pc, hc.Ph) + hc.Pw) * hc.S


# --------------------------------------------------------------------------------------------
# Per-step inputs
# --------------------------------------------------------------------------------------------
def water_draws(hc, t):
    """`MPCCalc.water_draws` (`mpc_calc.py:193-204`): hourly draws lagged by H/dt+1 hours,
    repeated dt times and divided by dt; entries past the first dt are 3-point moving averages."""
    H, dt = hc.H, hc.dt
    lag = H // dt + 1
    padded = lag * [0] + list(hc.draw_sizes)
    raw = padded[t // dt: t // dt + lag]
    raw = np.repeat(raw, dt) / dt
    out = list(raw[:dt])
    for i in range(dt, H + 1):
        out.append(np.average(raw[i - 1:i + 2]))
    draw = np.array(out, dtype=float)
    return draw, draw / hc.V, 1 - draw / hc.V


def env_slice(all_oat, all_ghi, all_tou, start_hour_index, t, H):
    """`set_environmental_variables` slicing (`mpc_calc.py:211-226`)."""
    s = start_hour_index + t
    e = s + H + 1
    return (np.asarray(all_oat[s:e], float), np.asarray(all_ghi[s:e], float),
            np.asarray(all_tou[s:e], float))


def season_is_winter(oat, noise):
    """`mpc_calc.py:220-223, 303-309`: max(oat[0], oat[1:] + 1.1^k * noise_k) <= 30."""
    H = len(noise)
    ev = np.array(oat, dtype=float).copy()
    ev[1:] = ev[1:] + np.power(1.1 * np.ones(H), np.arange(H)) * np.asarray(noise, float)
    return bool(max(ev) <= 30)


def total_price(tou, reward_price, H):
    """`mpc_calc.py:353`: rp[:H] + tou[:H]; rp must have length 1 or >= H (else numpy raises)."""
    rp = np.array(reward_price[:H], dtype=float)
    return rp + np.asarray(tou, float)[:H]


# --------------------------------------------------------------------------------------------
# Problem assembly (`add_base_constraints :291-353`, `add_pv_constraints :375-385`,
# `add_battery_constraints :355-373`, `set_*_p_grid :387-432`, `solve_mpc :434-446`)
# --------------------------------------------------------------------------------------------
class Layout:
    """Variable offsets in cvxpy creation order (`mpc_calc.py:165-173, 247-249, 261-262, 441`)."""

    def __init__(self, hc):
        H = hc.H
        sizes = [("p_load", H), ("temp_in_ev", H + 1), ("temp_in", 1), ("temp_wh_ev", H + 1),
                 ("temp_wh", 1), ("p_grid", H), ("hvac_cool_on", H), ("hvac_heat_on", H),
                 ("wh_heat_on", H)]
        if hc.has_batt:
            sizes += [("p_batt_ch", H), ("p_batt_disch", H), ("e_batt", H + 1)]
        if hc.has_pv:
            sizes += [("p_pv", H), ("u_pv_curt", H)]
        sizes += [("cost", H)]
        self.off, self.size, n = {}, {}, 0
        for k, s in sizes:
            self.off[k], self.size[k] = n, s
            n += s
        self.n = n
        self.integer = np.zeros(n, dtype=int)
        for k in ("hvac_cool_on", "hvac_heat_on", "wh_heat_on"):
            self.integer[self.off[k]:self.off[k] + H] = 1

    def idx(self, k, i=0):
        return self.off[k] + i

    def get(self, x, k):
        return x[self.off[k]:self.off[k] + self.size[k]]


@dataclass
class StepInput:
    t: int
    T0: float
    Tw0: float
    E0: float
    oat: np.ndarray      # H+1
    ghi: np.ndarray      # H+1
    price: np.ndarray    # H (total price)
    draw: np.ndarray     # H+1 draw sizes
    winter: bool


class Rows:
    def __init__(self, n):
        self.n = n
        self.eq, self.beq, self.ub, self.bub = [], [], [], []

    def add(self, kind, coefs, b):
        row = np.zeros(self.n)
        for j, v in coefs:
            row[j] += v
        (self.eq if kind == "eq" else self.ub).append(row)
        (self.beq if kind == "eq" else self.bub).append(b)


def build_problem(hc, si):
    """Assemble c, A_eq, b_eq, A_ub, b_ub, integrality exactly as the reference's cvxpy model."""
    H, S, dt = hc.H, hc.S, hc.dt
    L = Layout(hc)
    rw = Rows(L.n)
    T, Tw, Ts, Tws = "temp_in_ev", "temp_wh_ev", "temp_in", "temp_wh"
    c_, h_, w_ = "hvac_cool_on", "hvac_heat_on", "wh_heat_on"
    inv_c = 1.0 / (hc.C * dt)
    inv_w = 1.0 / (hc.Cw * dt)
    iR, iRw = 1.0 / hc.R, 1.0 / hc.Rw
    if si.winter:       # :303-309
        hmax, cmax = S, 0
    else:
        hmax, cmax = 0, S
    draw_frac = si.draw / hc.V
    rem = 1 - draw_frac
    # --- indoor air (:313-326)
    rw.add("eq", [(L.idx(T, 0), 1.0)], si.T0)
    for k in range(H):
        a_T = 1.0 + (-iR * 3600) * inv_c
        rw.add("eq", [(L.idx(T, k + 1), 1.0), (L.idx(T, k), -a_T),
                      (L.idx(c_, k), hc.Pc * 3600 * inv_c), (L.idx(h_, k), -(hc.Ph * 3600 * inv_c))],
               si.oat[k + 1] * iR * 3600 * inv_c)
    for k in range(H):
        rw.add("ub", [(L.idx(T, k + 1), -1.0)], -hc.Tmin)
    for k in range(H):
        rw.add("ub", [(L.idx(T, k + 1), 1.0)], hc.Tmax)
    rw.add("eq", [(L.idx(Ts), 1.0), (L.idx(c_, 0), hc.Pc * 3600 * inv_c), (L.idx(h_, 0), -hc.Ph * 3600 * inv_c)],
           si.T0 + ((si.oat[1] - si.T0) * iR) * 3600 * inv_c)
    rw.add("ub", [(L.idx(Ts), 1.0)], hc.Tmax)
    rw.add("ub", [(L.idx(Ts), -1.0)], -hc.Tmin)
    # --- water heater (:329-340)
    rw.add("eq", [(L.idx(Tw, 0), 1.0)], si.Tw0)
    for k in range(H):
        r = rem[k + 1]
        d15 = draw_frac[k + 1] * TAP_TEMP
        zT = iRw * 3600 * inv_w
        zTw = (-r * iRw) * 3600 * inv_w
        zw = hc.Pw * 3600 * inv_w
        zc = ((-d15) * iRw) * 3600 * inv_w
        rw.add("eq", [(L.idx(Tw, k + 1), 1.0), (L.idx(Tw, k), -(r + zTw)), (L.idx(T, k + 1), -zT),
                      (L.idx(w_, k), -zw)], d15 + zc)
    for k in range(H + 1):
        rw.add("ub", [(L.idx(Tw, k), -1.0)], -hc.Twmin)
    for k in range(H + 1):
        rw.add("ub", [(L.idx(Tw, k), 1.0)], hc.Twmax)
    rw.add("eq", [(L.idx(Tws), 1.0), (L.idx(T, 1), -iRw * 3600 * inv_w), (L.idx(w_, 0), -hc.Pw * 3600 * inv_w)],
           si.Tw0 + (-si.Tw0 * iRw) * 3600 * inv_w)
    rw.add("ub", [(L.idx(Tws), -1.0)], -hc.Twmin)
    rw.add("ub", [(L.idx(Tws), 1.0)], hc.Twmax)
    # --- load and duty bounds (:342-349)
    for k in range(H):
        rw.add("eq", [(L.idx("p_load", k), 1.0), (L.idx(c_, k), -S * hc.Pc), (L.idx(h_, k), -S * hc.Ph),
                      (L.idx(w_, k), -S * hc.Pw)], 0.0)
    for var, ub in ((c_, cmax), (h_, hmax), (w_, S)):
        for k in range(H):
            rw.add("ub", [(L.idx(var, k), 1.0)], float(ub))
        for k in range(H):
            rw.add("ub", [(L.idx(var, k), -1.0)], 0.0)
    # --- pv (:380-385)
    if hc.has_pv:
        g = hc.pv["area"] * hc.pv["eff"]
        for k in range(H):
            rw.add("eq", [(L.idx("p_pv", k), 1.0), (L.idx("u_pv_curt", k), g * si.ghi[k] / 1000)],
                   g * si.ghi[k] / 1000)
        for k in range(H):
            rw.add("ub", [(L.idx("u_pv_curt", k), -1.0)], 0.0)
        for k in range(H):
            rw.add("ub", [(L.idx("u_pv_curt", k), 1.0)], 1.0)
    # --- battery (:361-373)
    if hc.has_batt:
        b = hc.batt
        for k in range(H):
            rw.add("eq", [(L.idx("e_batt", k + 1), 1.0), (L.idx("e_batt", k), -1.0),
                          (L.idx("p_batt_ch", k), -b["eta_c"] / dt),
                          (L.idx("p_batt_disch", k), -(1.0 / b["eta_d"]) / dt)], 0.0)
        rw.add("eq", [(L.idx("e_batt", 0), 1.0)], si.E0)
        for k in range(H):
            rw.add("ub", [(L.idx("p_batt_ch", k), 1.0)], b["rate"])
        for k in range(H):
            rw.add("ub", [(L.idx("p_batt_ch", k), -1.0)], 0.0)
        for k in range(H):
            rw.add("ub", [(L.idx("p_batt_disch", k), -1.0)], b["rate"])
        for k in range(H):
            rw.add("ub", [(L.idx("p_batt_disch", k), 1.0)], 0.0)
        for k in range(H):
            rw.add("ub", [(L.idx("e_batt", k + 1), 1.0)], b["Emax"])
        for k in range(H):
            rw.add("ub", [(L.idx("e_batt", k + 1), -1.0)], -b["Emin"])
    # --- grid balance (:393-432)
    for k in range(H):
        co = [(L.idx("p_grid", k), 1.0), (L.idx("p_load", k), -1.0)]
        if hc.has_batt:
            co += [(L.idx("p_batt_ch", k), -float(S)), (L.idx("p_batt_disch", k), -float(S))]
        if hc.has_pv:
            co += [(L.idx("p_pv", k), float(S))]
        rw.add("eq", co, 0.0)
    # --- cost and objective (:441-446)
    for k in range(H):
        rw.add("eq", [(L.idx("cost", k), 1.0), (L.idx("p_grid", k), -si.price[k])], 0.0)
    cobj = np.zeros(L.n)
    weights = np.power(hc.discount * np.ones(H), np.arange(H))
    cobj[L.off["cost"]:L.off["cost"] + H] = weights
    return dict(c=cobj, A_eq=np.array(rw.eq), b_eq=np.array(rw.beq), A_ub=np.array(rw.ub),
                b_ub=np.array(rw.bub), integrality=L.integer.copy(), layout=L)


def solve_problem(P, integer=True, time_limit=60.0, mip_rel_gap=1e-6):
    """HiGHS (scipy.optimize.milp) in place of cvxpy+GLPK_MI (`mpc_calc.py:447-454`).

    Returns (status_str, x, objective).  Integer columns are reported as exact integers
    (GLPK_MI's glp_intopt rounds them); a time limit with an incumbent counts as optimal."""
    from scipy.optimize import milp, LinearConstraint, Bounds
    cons = [LinearConstraint(P["A_eq"], P["b_eq"], P["b_eq"]),
            LinearConstraint(P["A_ub"], -np.inf, P["b_ub"])]
    integ = P["integrality"] if integer else np.zeros_like(P["integrality"])
    res = milp(P["c"], constraints=cons, integrality=integ, bounds=Bounds(-np.inf, np.inf),
               options={"time_limit": time_limit, "mip_rel_gap": mip_rel_gap, "presolve": True})
    if res.x is None:
        return ({2: "infeasible", 3: "unbounded"}.get(res.status, "solver_error"), None, None)
    x = res.x.copy()
    if integer:
        x[integ == 1] = np.floor(x[integ == 1] + 0.5)
    return "optimal", x, float(P["c"] @ x)


# --------------------------------------------------------------------------------------------
# Result extraction + infeasibility fallback (`cleanup_and_finish :476-596`)
# --------------------------------------------------------------------------------------------
def first_char_float(s):
    """`float(str_value[0])` (`mpc_calc.py:537-539`); raises ValueError on '-', 'n', 'i'."""
    return float(str(s)[0])


def cleanup(hc, si, status, x, prev_hash, counter_in):
    """Return (optimal_vals dict, counter_out).  `prev_hash` is the home's redis hash (str values)."""
    H, S = hc.H, hc.S
    ov = {}
    keys = list(BASE_KEYS)
    if status == "optimal":                                      # :486-526
        L = Layout(hc)
        g = lambda k: L.get(x, k)  # noqa: E731
        st = {}
        st["p_grid_opt"] = (g("p_grid") / S).tolist()
        st["forecast_p_grid_opt"] = (g("p_grid")[1:] / S).tolist() + [0]
        st["p_load_opt"] = (g("p_load") / S).tolist()
        st["temp_in_ev_opt"] = g("temp_in_ev")[1:].tolist()
        st["temp_in_opt"] = g("temp_in").tolist()
        st["temp_wh_ev_opt"] = g("temp_wh_ev")[1:].tolist()
        st["temp_wh_opt"] = g("temp_wh").tolist()
        st["hvac_cool_on_opt"] = (g("hvac_cool_on") / S).tolist()
        st["hvac_heat_on_opt"] = (g("hvac_heat_on") / S).tolist()
        st["wh_heat_on_opt"] = (g("wh_heat_on") / S).tolist()
        st["cost_opt"] = g("cost").tolist()
        st["waterdraws"] = list(si.draw)
        if hc.has_pv:
            st["p_pv_opt"] = g("p_pv").tolist()
            st["u_pv_curt_opt"] = g("u_pv_curt").tolist()
            keys += list(PV_KEYS)
        if hc.has_batt:
            st["e_batt_opt"] = g("e_batt").tolist()[1:]
            st["p_batt_ch"] = g("p_batt_ch").tolist()
            st["p_batt_disch"] = g("p_batt_disch").tolist()
            keys += list(BATT_KEYS)
        for k in keys:
            ov[k] = st[k][0]
            for j in range(H):
                ov[f"{k}_{j}"] = st[k][j]
        ov["temp_wh_opt"] = st["temp_wh_opt"][0]
        ov["temp_in_opt"] = st["temp_in_opt"][0]
        ov["correct_solve"] = 1
        ov["solve_counter"] = 0
        return ov, 0
    # ---- failure (:527-595)
    counter = counter_in + 1
    ov["correct_solve"] = 0
    hmax, cmax = (S, 0) if si.winter else (0, S)
    hmin = cmin = 0
    whmax, whmin = S, 0
    alpha = 3600 / (hc.C * hc.dt)
    alpha_w = 3600 / (hc.Cw * hc.dt)

    def sim(T0, Tw0, cool, heat, wh):
        nT = float(T0 + 3600 * ((((si.oat[1] - T0) / hc.R)) - cool * hc.Pc + heat * hc.Ph) / (hc.C * hc.dt))
        nTw = float(Tw0 + 3600 * ((((nT - Tw0) / hc.Rw)) + wh * hc.Pw) / (hc.Cw * hc.dt))
        return nT, nTw

    if counter < H and si.t > 0:                                  # :533-557
        for k in BASE_KEYS:
            ov[k] = prev_hash[f"{k}_{counter}"]
        wh = first_char_float(ov["wh_heat_on_opt"])
        cool = first_char_float(ov["hvac_cool_on_opt"])
        heat = first_char_float(ov["hvac_heat_on_opt"])
        nT, nTw = sim(si.T0, si.Tw0, cool, heat, wh)
        if nT > hc.Tmax:
            heat, cool = hmin, cmax
        elif nT < hc.Tmin:
            heat, cool = hmax, cmin
        if nTw < hc.Twmin:
            wh = whmax
    else:                                                         # :559-574
        counter = int(np.clip(counter, H, None))
        if si.T0 > hc.Tmax:
            heat, cool = hmin, cmax
        elif si.T0 < hc.Tmin:
            heat, cool = hmax, cmin
        else:
            heat, cool = hmin, cmin
        wh = whmax if si.Tw0 < hc.Twmin else whmin
    nT, nTw = sim(si.T0, si.Tw0, cool, heat, wh)                 # :576-582
    ov["wh_heat_on_opt"] = wh / S
    ov["hvac_heat_on_opt"] = heat / S
    ov["hvac_cool_on_opt"] = cool / S
    ov["temp_in_opt"] = nT
    ov["temp_wh_opt"] = nTw
    ov["solve_counter"] = counter
    ov["p_load_opt"] = wh * hc.Pw + cool * hc.Pc + heat * hc.Ph
    ov["forecast_p_grid_opt"] = ov["p_load_opt"]
    ov["waterdraws"] = si.draw[0]
    ov["p_grid_opt"] = ov["p_load_opt"]
    ov["cost_opt"] = ov["p_grid_opt"] * si.price[0]
    return ov, counter


# --------------------------------------------------------------------------------------------
# One home-step through the redis-hash restatement (`run_home :649-672`)
# --------------------------------------------------------------------------------------------
def initial_conditions(hc, t, hash_, draw):
    """`get_initial_conditions` (`mpc_calc.py:264-289`) -> (T0, Tw0, E0, counter)."""
    mix = lambda T: (T * (hc.V - draw[0]) + TAP_TEMP * draw[0]) / hc.V  # noqa: E731
    if t == 0:
        return hc.T_init, mix(hc.Tw_init), (hc.batt["E_init"] if hc.has_batt else None), 0
    T0 = float(hash_["temp_in_opt"])
    Tw0 = mix(float(hash_["temp_wh_opt"]))
    E0 = None
    if hc.has_batt:
        E0 = float(hash_["e_batt_opt"])          # KeyError if the home never solved (reference too)
        float(hash_["p_batt_ch"]) - float(hash_["p_batt_disch"])
    return T0, Tw0, E0, int(hash_["solve_counter"])


def run_home_step(hc, t, hash_, env, noise, solver=None):
    """One `run_home` (`mpc_calc.py:649-672`) on a dict hash; returns (status, optimal_vals).

    env: dict(oat, ghi, tou, start_hour_index, reward_price).  `solver(P) -> (status, x, obj)`
    defaults to the HiGHS MILP."""
    draw, _, _ = water_draws(hc, t)
    T0, Tw0, E0, counter = initial_conditions(hc, t, hash_, draw)
    oat, ghi, tou = env_slice(env["oat"], env["ghi"], env["tou"], env["start_hour_index"], t, hc.H)
    price = total_price(tou, env["reward_price"], hc.H)
    si = StepInput(t=t, T0=T0, Tw0=Tw0, E0=E0, oat=oat, ghi=ghi, price=price, draw=draw,
                   winter=season_is_winter(oat, noise))
    P = build_problem(hc, si)
    try:
        status, x, _ = (solver or solve_problem)(P)
    except Exception:                           # :450-454 (exceptions swallowed)
        status, x = None, None
    ov, _ = cleanup(hc, si, status, x, hash_, counter)
    for k, v in ov.items():                     # redis_write_optimal_vals :100-107
        hash_[k] = enc(v)
    return status, ov, si
