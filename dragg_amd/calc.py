"""Per-home facade with the reference's `MPCCalc` interface (mpc_calc.py:16-98, 649-672).

For code written against `MPCCalc(home).run_home()` + `manage_home` under a pool map
(aggregator.py:723-724).  `MPCCalc` objects registered on one `Community` share a single
device batch: the first `run_home()` of a timestep launches the solver for EVERY home of the
community (one `dragg_mpc_step`), the other homes find their results already in the device
hash.  Calling `run_home()` for every home of a step, in any order, is therefore the
reference's `pool.map(manage_home, homes)`; a home whose solve hits one of the reference's
crashing paths raises the reference's exception from its own `run_home()`.

The home's redis hash is the device hash: `Community.hgetall(name)` returns it with the
reference's field names and str values, as redis does; `MPCCalc.optimal_vals` holds the
home's hash after its latest step, as numbers.
"""
from . import _lib as L
from .inputs import max_load
from .mpc import MPCBatch

# The reference's plug point: home['hems']['solver'] names a cvxpy backend, and an unknown name
# falls back to GLPK_MI (mpc_calc.py:141-145).  The duty variables are integer
# (mpc_calc.py:171-173), so what a backend does depends on whether it takes a MILP:
# * GLPK_MI (and GUROBI, when gurobipy is installed: it is not in the reference's
#   requirements.txt, and without it cvxpy raises like ECOS below) solve the MILP to
#   optimality -> this build's exact MILP path, int_mode "round";
# * ECOS is not MIP-capable: cvxpy raises SolverError on an integer problem, the bare except of
#   mpc_calc.py:450-454 sets solved = False and EVERY solve takes the fallback thermostat ->
#   int_mode "fail" (status solver_error).  cvxpy is not pinned (requirements.txt) nor importable
#   here, so this is parity unpinned; it follows cvxpy's documented MIP-capability check.
# The build's own modes may be named directly ("relax": the LP relaxation, "round_lp", "fail").
SOLVER_MODES = {"GLPK_MI": "round", "GUROBI": "round", "ECOS": "fail"}


def int_mode_for(home):
    """The int_mode a home's hems.solver selects (mpc_calc.py:141-145)."""
    name = str(home.get("hems", {}).get("solver", "GLPK_MI"))
    if name in L.INT_MODES:
        return name
    return SOLVER_MODES.get(name, "round")


class Community:
    """The redis side of a run for a set of homes: environment lists, `current_values`
    timestep, `reward_price`, and the per-home hashes (device resident).

    The reference's MPCCalc(home) reads its environment from the redis server the aggregator
    filled (mpc_calc.py:117-132); here `make_default()` plays that role: MPCCalc(home) without a
    community attaches to the default one."""

    _default = None

    def __init__(self, homes, oat, ghi, tou, start_hour_index, reward_price=(0.0,), int_mode=None, seed=0,
                 device="cuda"):
        int_mode = int_mode or (int_mode_for(homes[0]) if homes else "round")
        self.batch = MPCBatch(homes, oat, ghi, tou, start_hour_index, reward_price, int_mode=int_mode, seed=seed,
                              device=device)
        self.index = {h["name"]: i for i, h in enumerate(homes)}
        self.timestep = 0
        self._solved = -1
        self._status = None

    # aggregator.py:664-675 (redis_set_current_values)
    def set_timestep(self, t):
        self.timestep = int(t)

    def set_reward_price(self, rp):
        self.batch.set_reward_price(rp)

    def solve(self):
        """Solve every home for the current timestep (once per timestep)."""
        if self._solved != self.timestep:
            self.batch.step(self.timestep)
            self._status = self.batch.status.cpu().numpy()
            self._solved = self.timestep
        return self._status

    def hgetall(self, name):
        return self.batch.hash_dict(self.index[name], as_str=True)

    def make_default(self):
        """Register as the community that MPCCalc(home) attaches to."""
        Community._default = self
        return self

    @classmethod
    def default(cls):
        if cls._default is None:
            raise RuntimeError("no community: build one with Community(...).make_default() first (the reference "
                               "needs its redis server filled by the aggregator, mpc_calc.py:117-132)")
        return cls._default


def manage_home(home):
    """mpc_calc.py:16-22."""
    home.run_home()


class MPCCalc:
    """mpc_calc.py:24-98: `MPCCalc(home)` (the default community) or `MPCCalc(home, community)`."""

    def __init__(self, home, community=None):
        community = community if community is not None else Community.default()
        if home["name"] not in community.index:
            raise KeyError(f"home {home['name']!r} is not part of the community")
        want = int_mode_for(home)
        have = [k for k, v in L.INT_MODES.items() if v == community.batch.dims.int_mode][0]
        if want != have:
            raise ValueError(f"home {home['name']!r} asks for solver {home['hems'].get('solver')!r} "
                             f"(int_mode {want!r}) but its community solves with {have!r}")
        self.home = home
        self.name = home["name"]
        self.type = home["type"]
        self.community = community
        self.i = community.index[self.name]
        self.max_load = max_load(home)
        self.timestep = 0
        self.optimal_vals = {}

    def run_home(self):
        """One timestep of this home (mpc_calc.py:649-672)."""
        st = int(self.community.solve()[self.i])
        if st == L.ST_ERR_MISSING:
            raise KeyError("e_batt_opt" if "battery" in self.type else "temp_in_opt")
        if st == L.ST_ERR_PARSE:
            raise ValueError("could not convert string to float: '-'")
        self.timestep = self.community.timestep
        self.optimal_vals = self.community.batch.hash_dict(self.i, as_str=False)
        self.counter = int(self.optimal_vals.get("solve_counter", 0))
        return None
