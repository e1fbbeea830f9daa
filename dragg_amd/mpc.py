"""Host side of the batched MPC: home packing, device-resident hash arrays, launches.

This is the MI355X-native replacement of `dragg/mpc_calc.py`'s per-home solve: all homes
of a timestep are solved by ONE kernel launch of libdragg_mi355x.so (one 64-lane
workgroup per home).  Per-home parameters, the redis "hash" of each home and the
environment lists live on the GPU as fp64 struct-of-arrays tensors (home index
innermost).  See `dragg_amd.calc.MPCCalc` for the per-home facade with the
reference's interface.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L

TAP_TEMP = 15.0  # mpc_calc.py:181


def _f(x):
    return float(x)


def hems_dims(home):
    """(S, dt, H, discount) exactly as `setup_base_problem` derives them (mpc_calc.py:148-152)."""
    hems = home["hems"]
    S = max(1, int(hems["sub_subhourly_steps"]))
    dt = max(1, int(hems["hourly_agg_steps"]))
    H = max(1, int(hems["horizon"] * dt))
    return S, dt, H, float(hems["discount_factor"])


def pack_homes(homes, template=None):
    """home dicts (aggregator.py:423-449 schema) -> (params [NPARAM][N], types [N], draws [hours][N], dims).

    Derived constants are computed with the reference's own float expressions
    (mpc_calc.py:157-189, 239-244, 257-258, 274).  `template`: a home of the community whose
    hems settings give the dims of an empty shard (N = 0, more ranks than homes)."""
    N = len(homes)
    if N == 0 and template is None:
        raise ValueError("no homes")
    S, dt, H, disc = hems_dims(homes[0] if N else template)
    for h in homes:
        if hems_dims(h) != (S, dt, H, disc):
            raise ValueError("all homes of a batch must share the hems settings (responsive_hems)")
    P = np.zeros((L.NPARAM, N))
    types = np.zeros(N, dtype=np.int32)
    nd = max((len(h["wh"]["draw_sizes"]) for h in homes), default=1)
    draws = np.zeros((nd, N))
    for i, h in enumerate(homes):
        if h["type"] not in L.TYPE_CODE:
            raise ValueError(f"unknown home type {h['type']!r}")
        types[i] = L.TYPE_CODE[h["type"]]
        hv, wh = h["hvac"], h["wh"]
        P[L.P["R"], i] = _f(hv["r"])
        P[L.P["C"], i] = _f(hv["c"]) * 1000
        P[L.P["PC"], i] = _f(hv["p_c"]) / S
        P[L.P["PH"], i] = (_f(hv["p_h"])) / S
        P[L.P["RW"], i] = _f(wh["r"]) * 1000
        P[L.P["PW"], i] = _f(wh["p"]) / S
        P[L.P["CW"], i] = _f(wh["tank_size"]) * 4.2
        P[L.P["V"], i] = _f(wh["tank_size"])
        P[L.P["TMIN"], i] = _f(hv["temp_in_min"])
        P[L.P["TMAX"], i] = _f(hv["temp_in_max"])
        P[L.P["TWMIN"], i] = _f(wh["temp_wh_min"])
        P[L.P["TWMAX"], i] = _f(wh["temp_wh_max"])
        P[L.P["TINIT"], i] = _f(hv["temp_in_init"])
        P[L.P["TWINIT"], i] = _f(wh["temp_wh_init"])
        if "battery" in h["type"]:
            b = h["battery"]
            cap = _f(b["capacity"])
            P[L.P["BRATE"], i] = _f(b["max_rate"])
            P[L.P["EMIN"], i] = _f(b["capacity_lower"]) * cap
            P[L.P["EMAX"], i] = _f(b["capacity_upper"]) * cap
            P[L.P["ETAC"], i] = _f(b["ch_eff"])
            P[L.P["ETAD"], i] = _f(b["disch_eff"])
            P[L.P["EINIT"], i] = _f(b["e_batt_init"]) * cap
        if "pv" in h["type"]:
            P[L.P["PVAREA"], i] = _f(h["pv"]["area"])
            P[L.P["PVEFF"], i] = _f(h["pv"]["eff"])
        ds = np.asarray(h["wh"]["draw_sizes"], dtype=float)
        draws[:len(ds), i] = ds
    return P, types, draws, dict(S=S, dt=dt, H=H, discount=disc, n_draw_hours=nd)


class MPCBatch:
    """A device-resident batch of homes that share one environment.

    Parameters
    ----------
    homes : list of home dicts (the `all_homes` records of the aggregator).
    oat, ghi, tou : full-length redis lists (aggregator.py:653-662), any sequence of floats.
    start_index : `start_hour_index` (aggregator.py:630-638).
    reward_price : the redis 'reward_price' list (length 1 or >= H, mpc_calc.py:353).
    int_mode : 'round' (default: the reference MILP -- thermal integer duty cycles by DP, the
        battery LP by an exact piecewise-linear DP), 'relax' (the LP relaxation by ADMM + exact
        vertex polish) or 'round_lp' (the relaxation for status / battery, then the integer DP).
    seed : key of the on-device season-noise stream used when no noise is supplied.
    home_offset, home_stride : global community index of home i is home_offset + i*home_stride
        (the season-noise key), so a shard draws the same numbers as the whole community.
    template_home : a home of the community, for the dims of an empty shard (homes == []):
        its steps are no-ops and its sums zero.
    exact : int_mode round: every chain the Pareto-front DP cannot take (a feasible set narrower
        than one duty step -- ~0.3 homes per 10k-home step --, mixed-sign prices without a usable
        bound, RL fronts past 2,048 labels) by the exact step-function DP (slow) instead of the
        bucketed DP's schedule (DRAGG_FLAG_EXACT).  Statuses are exact either way.
    """

    def __init__(self, homes, oat=None, ghi=None, tou=None, start_index=0, reward_price=(0.0,),
                 int_mode="round", seed=0, max_iter=4000, check_every=10, device="cuda", home_offset=0,
                 home_stride=1, template_home=None, exact=False):
        if int_mode not in L.INT_MODES:
            raise ValueError(f"int_mode must be one of {sorted(L.INT_MODES)}, not {int_mode!r}")
        self.lib = L.load()
        if not torch.cuda.is_available():
            raise L.DraggError("no GPU visible: the batched MPC has no CPU fallback")
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.homes = homes
        self.names = [h["name"] for h in homes]
        P, types, draws, dm = pack_homes(homes, template_home)
        self.N, self.H, self.S, self.dt = len(homes), dm["H"], dm["S"], dm["dt"]
        dev = self.device
        self.params = torch.tensor(P, dtype=torch.float64, device=dev).contiguous()
        self.types = torch.tensor(types, dtype=torch.int32, device=dev)
        self.types_host = types
        self.draws = torch.tensor(draws, dtype=torch.float64, device=dev).contiguous()
        self.dims = L.Dims(n_homes=self.N, horizon=self.H, sub_steps=self.S, dt=self.dt,
                           n_draw_hours=dm["n_draw_hours"], n_env=0, n_rp=1,
                           int_mode=L.INT_MODES[int_mode],
                           max_iter=max_iter, check_every=check_every, discount=dm["discount"],
                           flags=L.FLAG_EXACT if exact else 0)
        self.seed = int(seed)
        self.home_offset = int(home_offset)
        self.home_stride = int(home_stride)
        self.set_environment(oat if oat is not None else [0.0], ghi if ghi is not None else [0.0],
                             tou if tou is not None else [0.0], start_index)
        self.workspace = None
        self.lag = None
        self.set_reward_price(reward_price)
        self.vals = torch.full((L.NVAL, self.N), float("nan"), dtype=torch.float64, device=dev)
        # the forecast fields <key>_<j>: stored home-contiguous ([N][NFC][H], dragg_mi355x.h: one home's
        # fields are one 5.7 KB run the solver writes with coalesced stores), seen here as the
        # [NFC][H][N] view the rest of the host code indexes
        self.fc_store = torch.full((self.N, L.NFC, self.H), float("nan"), dtype=torch.float64, device=dev)
        self.fc = self.fc_store.permute(1, 2, 0)
        self.status = torch.zeros(self.N, dtype=torch.int32, device=dev)
        self.iters = torch.zeros(self.N, dtype=torch.int32, device=dev)
        self.obj = torch.zeros(self.N, dtype=torch.float64, device=dev)
        self.relax_obj = torch.zeros(self.N, dtype=torch.float64, device=dev)
        self.int_path = torch.zeros(self.N, dtype=torch.int32, device=dev)
        self.agg = torch.zeros(3, dtype=torch.float64, device=dev)
        self.cycles = None
        rc = self.lib.dragg_mpc_lds_bytes(ctypes.byref(self.dims))
        if rc < 0:
            L.check(rc)
        self.lds_bytes = rc
        self._ensure_workspace()

    # ------------------------------------------------------------------ environment
    def set_environment(self, oat, ghi, tou, start_index):
        # (lag mode: a side pass still in flight holds raw pointers to the current lists, and their blocks
        # belong to the main stream's allocator pool: join it before they can be freed and reused)
        if getattr(self, "lag", None) is not None:
            self.drain()
        dev = self.device
        self.oat = torch.tensor(np.asarray(oat, dtype=float), dtype=torch.float64, device=dev)
        self.ghi = torch.tensor(np.asarray(ghi, dtype=float), dtype=torch.float64, device=dev)
        self.tou = torch.tensor(np.asarray(tou, dtype=float), dtype=torch.float64, device=dev)
        self.start_index = int(start_index)
        self.dims.n_env = int(min(len(oat), len(ghi), len(tou)))

    def set_reward_price(self, rp):
        """The redis 'reward_price' list (mpc_calc.py:630-637): host values, or a device tensor
        (e.g. an RL action broadcast over RCCL), taken without a host round trip."""
        if torch.is_tensor(rp):
            rp = rp.detach().to(device=self.device, dtype=torch.float64).reshape(-1).contiguous()
            n = rp.numel()
        else:
            rp = np.asarray([float(v) for v in rp], dtype=float)
            n = len(rp)
        if n != 1 and n < self.H:
            # np.array(rp[:H]) + tou[:H] raises in the reference (mpc_calc.py:353)
            raise ValueError(f"operands could not be broadcast together: reward_price has {n} "
                             f"entries, horizon is {self.H}")
        if getattr(self, "lag", None) is not None:
            self.drain()                     # (as in set_environment: the side pass reads self.rp)
        self.rp = rp if torch.is_tensor(rp) else torch.tensor(rp, dtype=torch.float64, device=self.device)
        self.dims.n_rp = n
        if self.workspace is not None or hasattr(self, "vals"):
            self._ensure_workspace()

    def _ensure_workspace(self):
        """Device scratch of dragg_mpc_workspace_bytes(dims) bytes (it grows when a reward-price list makes
        RL prices possible: the cell bound's rows); the lag mode's side workspace likewise."""
        ws = self.lib.dragg_mpc_workspace_bytes(ctypes.byref(self.dims))
        if ws < 0:
            L.check(int(ws))
        need = max(1, (ws + 7) // 8) if ws > 0 else 0
        have = self.workspace.numel() if self.workspace is not None else 0
        if need > have:
            self.drain()
            self.workspace = torch.empty(need, dtype=torch.int64, device=self.device)
            if self.lag is not None:
                self.lag["side_ws"] = self._side_workspace()

    def _side_workspace(self):
        """The lag mode's side workspace: only the lists and per-block scratch of the side pass
        (dragg_mpc_side_workspace_bytes; the per-home regions stay in self.workspace)."""
        sb = self.lib.dragg_mpc_side_workspace_bytes(ctypes.byref(self.dims))
        if sb < 0:
            L.check(int(sb))
        return torch.empty(max(1, (sb + 7) // 8), dtype=torch.int64, device=self.device)

    # ------------------------------------------------------------------ structs
    def _problem(self):
        return L.Problem(params=L.ptr(self.params), home_type=L.ptr(self.types), draw_hourly=L.ptr(self.draws),
                         oat=L.ptr(self.oat), ghi=L.ptr(self.ghi), tou=L.ptr(self.tou),
                         reward_price=L.ptr(self.rp), start_index=self.start_index,
                         home_offset=self.home_offset, seed=self.seed, workspace=L.ptr(self.workspace),
                         home_stride=self.home_stride)

    def _hash(self):
        return L.Hash(vals=L.ptr(self.vals), fc=L.ptr(self.fc_store))

    def _out(self, hist=None):
        return L.Out(status=L.ptr(self.status), iters=L.ptr(self.iters), obj=L.ptr(self.obj),
                     relax_obj=L.ptr(self.relax_obj), hist=L.ptr(hist), cycles=L.ptr(self.cycles),
                     int_path=L.ptr(self.int_path))

    def enable_phase_timing(self, on=True):
        """Stamp per-phase shader cycles of every home into self.cycles [NPHASE][N] (diagnostic)."""
        self.cycles = (torch.zeros((L.NPHASE, self.N), dtype=torch.int64, device=self.device) if on else None)

    # ------------------------------------------------------------------ launches
    def step(self, t, noise=None, hist=None, stream=None):
        """One closed-loop timestep for every home (run_iteration, aggregator.py:711-726)."""
        with torch.cuda.device(self.device):
            self.drain(stream)
            if self.lag is not None:
                self.lag["next"] = None          # the clocks no longer describe the state
            return self._step(t, noise, hist, stream)

    # ------------------------------------------------------------------ lag mode
    def enable_lag(self, ring=128):
        """Lag mode (dragg_mpc_step_main / _side, include/dragg_mi355x.h): a home whose chain needs the
        step-function DP finishes that step on a side stream while the other homes go on with their
        next steps; it catches up there.  Allocates the side pass's workspace, the per-home clocks, a
        ring of `ring` per-step list pairs (the main pass of step t + ring waits for the side pass of
        step t), the side stream and the events that order the two passes."""
        if self.dims.int_mode not in (L.INT_ROUND, L.INT_FAIL):
            raise ValueError("lag mode needs int_mode 'round' (or 'fail')")
        dev = self.device
        with torch.cuda.device(dev):
            self.lag = {
                "ring": int(ring),
                "lists": torch.zeros((ring, 2, L.lag_list_ints(self.N)), dtype=torch.int32, device=dev),
                "clock": torch.zeros(max(1, self.N), dtype=torch.int32, device=dev),
                "side_ws": self._side_workspace() if self.workspace is not None else None,
                # (a high-priority side stream, measured in round 6: no change -- the 8-way shard holding
                # home 7519 0.8476-0.8482 against 0.8457-0.8489 ms/step, profiles/r06/ab/prio*)
                "stream": torch.cuda.Stream(device=dev),
                "main_done": torch.cuda.Event(),
                "side_done": [torch.cuda.Event() for _ in range(ring)],
                "recorded": [False] * ring,
                "next": None,                   # the step the clocks are ready for
                "pending": False,               # side work not yet joined into the main stream
            }

    def step_lagged(self, t, hist, status_row, stream=None, path_row=None, sums_row=None):
        """One timestep in lag mode: the main pass on `stream` (default: the current one), the side pass
        on the side stream after it.  `hist` ([NVAL][N]), `status_row` ([N] int32) and `path_row` ([N]
        int32, the int_path bits; default self.int_path) receive the step's per-home results -- a
        lagging home's later -- so they must be this step's own rows; nothing of the step may be read
        before drain().  `sums_row` ([3] f64, optional): collect_data's sums of the step, from `hist`,
        computed on the side stream after the step's side pass (dragg_mpc_aggregate_rows)."""
        with torch.cuda.device(self.device):
            return self._step_lagged(t, hist, status_row, stream, path_row, sums_row)

    def _step_lagged(self, t, hist, status_row, stream, path_row=None, sums_row=None):
        lg = self.lag
        if lg is None:
            raise RuntimeError("enable_lag() first")
        assert hist is not None and status_row is not None and status_row.dtype == torch.int32
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        side = lg["stream"]
        slot = t % lg["ring"]
        lag = L.Lag(clock=L.ptr(lg["clock"]), skipped=L.ptr(lg["lists"][slot, 0]), narrow=L.ptr(lg["lists"][slot, 1]),
                    side_workspace=L.ptr(lg["side_ws"]))
        if lg["next"] != t:
            # (the first lag-mode step, or one after a serial step: every step before t is complete)
            self.drain(main)
            L.check(self.lib.dragg_mpc_lag_reset(ctypes.byref(self.dims), ctypes.byref(lag), int(t),
                                                  L.stream_ptr(main, self.device)))
        if lg["recorded"][slot]:
            main.wait_event(lg["side_done"][slot])      # the side pass of step t - ring is done with the lists
        prob, hsh = self._problem(), self._hash()
        out = L.Out(status=L.ptr(status_row), iters=L.ptr(self.iters), obj=L.ptr(self.obj),
                    relax_obj=L.ptr(self.relax_obj), hist=L.ptr(hist), cycles=None,
                    int_path=L.ptr(path_row if path_row is not None else self.int_path))
        L.check(self.lib.dragg_mpc_step_main(ctypes.byref(self.dims), ctypes.byref(prob), ctypes.byref(hsh),
                                             ctypes.byref(out), int(t), ctypes.byref(lag), L.stream_ptr(main, self.device)))
        lg["main_done"].record(main)
        side.wait_event(lg["main_done"])
        L.check(self.lib.dragg_mpc_step_side(ctypes.byref(self.dims), ctypes.byref(prob), ctypes.byref(hsh),
                                             ctypes.byref(out), int(t), ctypes.byref(lag), L.stream_ptr(side, self.device)))
        if sums_row is not None:
            L.check(self.lib.dragg_mpc_aggregate_rows(ctypes.byref(self.dims), L.ptr(hist), 1, L.ptr(sums_row),
                                                      L.stream_ptr(side, self.device)))
        lg["side_done"][slot].record(side)
        lg["recorded"][slot] = True
        lg["last"] = slot
        lg["next"] = t + 1
        lg["pending"] = True
        self._keep = (hist, status_row, path_row, sums_row)

    def drain(self, stream=None):
        """Join the side stream into `stream` (default: the current one): after this, everything the
        lag-mode steps wrote is visible in stream order."""
        lg = self.lag
        if lg is None or not lg["pending"]:
            return
        main = stream if stream is not None else torch.cuda.current_stream(self.device)
        main.wait_event(lg["side_done"][lg["last"]])
        lg["pending"] = False

    def aggregate_rows(self, rows, stream=None):
        """collect_data sums of every history row of `rows` ([T][NVAL][N]) -> [T][3] (bit-identical to
        aggregate() on each row)."""
        with torch.cuda.device(self.device):
            out = torch.empty((rows.shape[0], 3), dtype=torch.float64, device=self.device)
            L.check(self.lib.dragg_mpc_aggregate_rows(ctypes.byref(self.dims), L.ptr(rows.contiguous()),
                                                      int(rows.shape[0]), L.ptr(out),
                                                      L.stream_ptr(stream, self.device)))
            return out

    def _step(self, t, noise, hist, stream):
        if noise is not None:
            noise = noise.to(device=self.device, dtype=torch.float64).contiguous()
            assert tuple(noise.shape) == (self.H, self.N)
        prob, hsh, out = self._problem(), self._hash(), self._out(hist)
        L.check(self.lib.dragg_mpc_step(ctypes.byref(self.dims), ctypes.byref(prob), ctypes.byref(hsh),
                                        ctypes.byref(out), int(t), L.ptr(noise), L.stream_ptr(stream, self.device)))
        self._keep = (noise, hist)
        return self.status

    def solve_explicit(self, t, T0, Tw0, E0, counter, winter, draw, oat, ghi, price, stream=None):
        """Independent per-home solves with explicit inputs ([N] and [H+1 or H][N] arrays)."""
        with torch.cuda.device(self.device):
            return self._solve_explicit(t, T0, Tw0, E0, counter, winter, draw, oat, ghi, price, stream)

    def _solve_explicit(self, t, T0, Tw0, E0, counter, winter, draw, oat, ghi, price, stream):
        self.drain(stream)
        dev, N, H = self.device, self.N, self.H

        def d(x, shape, dtype=torch.float64):
            tt = torch.as_tensor(np.asarray(x), dtype=dtype).to(dev).reshape(shape).contiguous()
            return tt
        ex_t = {
            "t": d(t, (N,), torch.int32), "T0": d(T0, (N,)), "Tw0": d(Tw0, (N,)),
            "E0": d(np.nan_to_num(np.asarray(E0, dtype=float)), (N,)),
            "counter": d(counter, (N,), torch.int32), "winter": d(winter, (N,), torch.int32),
            "draw": d(draw, (H + 1, N)), "oat": d(oat, (H + 1, N)), "ghi": d(ghi, (H + 1, N)),
            "price": d(price, (H, N)),
        }
        ex = L.Explicit(**{k: L.ptr(v) for k, v in ex_t.items()})
        prob, hsh, out = self._problem(), self._hash(), self._out()
        L.check(self.lib.dragg_mpc_solve_explicit(ctypes.byref(self.dims), ctypes.byref(prob), ctypes.byref(ex),
                                                  ctypes.byref(hsh), ctypes.byref(out),
                                                  L.stream_ptr(stream, self.device)))
        self._keep = ex_t
        return self.status

    def aggregate(self, stream=None):
        """collect_data sums (aggregator.py:751-753) -> device tensor [agg_load, forecast_load, agg_cost].
        A home whose fields are absent (a crashed home: the reference raises KeyError in
        collect_data, aggregator.py:750-752) makes the sums NaN."""
        with torch.cuda.device(self.device):
            return self._aggregate(stream)

    def _aggregate(self, stream):
        self.drain(stream)
        hsh = self._hash()
        L.check(self.lib.dragg_mpc_aggregate(ctypes.byref(self.dims), ctypes.byref(hsh), L.ptr(self.agg),
                                             L.stream_ptr(stream, self.device)))
        return self.agg

    def season_noise(self, t, stream=None):
        with torch.cuda.device(self.device):
            return self._season_noise(t, stream)

    def _season_noise(self, t, stream):
        out = torch.empty((self.H, self.N), dtype=torch.float64, device=self.device)
        L.check(self.lib.dragg_mpc_season_noise(ctypes.byref(self.dims), self.seed, self.home_offset,
                                                self.home_stride, int(t), L.ptr(out),
                                                L.stream_ptr(stream, self.device)))
        return out

    # ------------------------------------------------------------------ hash views
    def hash_dict(self, i, as_str=True):
        """The home's redis hash as `hgetall` would return it (str values, absent fields omitted)."""
        self.drain()
        vals = self.vals[:, i].cpu().numpy()
        fc = self.fc[:, :, i].cpu().numpy()
        out = {}
        for k, name in enumerate(L.FC_KEYS):
            for j in range(self.H):
                if not np.isnan(fc[k, j]):
                    out[f"{name}_{j}"] = fc[k, j]
        for k, name in enumerate(L.VAL_KEYS):
            if not np.isnan(vals[k]):
                out[name] = vals[k]
        if "solve_counter" in out:
            out["solve_counter"] = int(out["solve_counter"])
        if "correct_solve" in out:
            out["correct_solve"] = int(out["correct_solve"])
        if as_str:
            out = {k: (str(v) if isinstance(v, int) else repr(float(v))) for k, v in out.items()}
        return out
