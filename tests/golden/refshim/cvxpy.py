"""Minimal cvxpy stand-in used ONLY by tests/golden/make_golden.py (this container).

TEST INFRASTRUCTURE, never imported by the product (`dragg_amd`) or on the GPU box.

The reference (`dragg/mpc_calc.py`) builds its per-home MILP with a small subset
of cvxpy (Variable / Constant / slicing / + - * / / multiply / sum / == <= >= /
Minimize / Problem.solve).  cvxpy and its GLPK_MI backend are not installed in
this image, so this module collects the same affine expressions into sparse
rows and solves the resulting MILP with scipy's HiGHS (`scipy.optimize.milp`),
the documented stand-in for GLPK_MI (see DESIGN.md "Oracle").

Besides the reference-visible behaviour, `Problem.solve` records the assembled
problem (c, A_eq, b_eq, A_ub, b_ub, integrality) plus the LP-relaxation optimum
in `Problem.last_record`, so the harness can emit golden vectors.
"""
import numpy as np
from scipy.optimize import milp, LinearConstraint, Bounds

# the home whose problem is being solved (set by the harness's noise hook, per worker process), and
# GOLDEN_OWN: the home indices this run proves (a run split over processes by home: a home's closed
# loop depends on its own solves only, so each process proves its homes and solves the others fast)
CURRENT_HOME = [None]
_OWN = __import__("os").environ.get("GOLDEN_OWN")
OWN = None if not _OWN else {int(v) for v in _OWN.split(",")}

GLPK_MI = "GLPK_MI"
GLPK = "GLPK"
ECOS = "ECOS"
GUROBI = "GUROBI"

_VAR_COUNTER = [0]


class SolverError(Exception):
    pass


def _as_expr(x):
    if isinstance(x, Expression):
        return x
    return Constant(x)


class Expression:
    """Affine expression: sum_v coef[v] @ var_v + const, vector of length m (or scalar, shape ())."""

    def __init__(self, terms, const, shape):
        self.terms = terms          # dict var_id -> (Variable, 2-D coef array m x n_var)
        self.const = np.asarray(const, dtype=float).reshape(-1)
        self.shape = shape          # () or (m,)

    # ---- helpers -----------------------------------------------------------
    @property
    def size(self):
        return int(np.prod(self.shape)) if self.shape else 1

    def is_constant(self):
        return not self.terms

    def _broadcast(self, m):
        if self.size == m:
            return self
        if self.size != 1:
            raise ValueError(f"cannot broadcast expression of size {self.size} to {m}")
        terms = {k: (v, np.repeat(c, m, axis=0)) for k, (v, c) in self.terms.items()}
        return Expression(terms, np.repeat(self.const, m), (m,))

    @staticmethod
    def _combine(a, b, sb):
        a = _as_expr(a)
        b = _as_expr(b)
        m = max(a.size, b.size)
        shape = a.shape if a.size >= b.size else b.shape
        if a.size != b.size:
            a, b = a._broadcast(m), b._broadcast(m)
            shape = (m,)
        terms = {k: (v, c.copy()) for k, (v, c) in a.terms.items()}
        for k, (v, c) in b.terms.items():
            if k in terms:
                terms[k] = (v, terms[k][1] + sb * c)
            else:
                terms[k] = (v, sb * c)
        return Expression(terms, a.const + sb * b.const, shape)

    def _scale(self, s):
        s = np.asarray(s, dtype=float)
        if s.size == 1:
            s = float(s.reshape(-1)[0])
            return Expression({k: (v, c * s) for k, (v, c) in self.terms.items()}, self.const * s, self.shape)
        s = s.reshape(-1)
        base = self._broadcast(s.size)
        return Expression({k: (v, c * s[:, None]) for k, (v, c) in base.terms.items()},
                          base.const * s, (s.size,))

    # ---- arithmetic --------------------------------------------------------
    def __add__(self, o):
        return Expression._combine(self, o, 1.0)

    def __radd__(self, o):
        return Expression._combine(o, self, 1.0)

    def __sub__(self, o):
        return Expression._combine(self, o, -1.0)

    def __rsub__(self, o):
        return Expression._combine(o, self, -1.0)

    def __neg__(self):
        return self._scale(-1.0)

    def __mul__(self, o):
        o = _as_expr(o)
        if o.is_constant() and o.size == 1:
            return self._scale(o.const)
        if self.is_constant() and self.size == 1:
            return o._scale(self.const)
        raise ValueError("shim supports only scalar * expression (the reference uses no other '*')")

    __rmul__ = __mul__

    def __truediv__(self, o):
        o = _as_expr(o)
        if not (o.is_constant() and o.size == 1):
            raise ValueError("division only by scalar constants")
        return self._scale(1.0 / o.const[0])

    def __getitem__(self, idx):
        if not self.shape:
            raise IndexError("scalar expression")
        rows = np.arange(self.size)[idx]
        scalar = np.ndim(rows) == 0
        rows = np.atleast_1d(rows)
        terms = {k: (v, c[rows]) for k, (v, c) in self.terms.items()}
        return Expression(terms, self.const[rows], () if scalar else (rows.size,))

    # ---- constraints -------------------------------------------------------
    def __eq__(self, o):
        return Constraint(self - o, "eq")

    def __le__(self, o):
        return Constraint(self - o, "le")

    def __ge__(self, o):
        return Constraint(_as_expr(o) - self, "le")

    __hash__ = object.__hash__

    # ---- values ------------------------------------------------------------
    @property
    def value(self):
        out = self.const.copy()
        for k, (v, c) in self.terms.items():
            if v._value is None:
                return None
            out = out + c @ np.atleast_1d(v._value)
        if not self.shape:
            return np.float64(out[0])
        return out


class Constant(Expression):
    def __init__(self, value):
        arr = np.asarray(value, dtype=float)
        super().__init__({}, arr.reshape(-1), arr.shape if arr.ndim else ())
        self._cval = arr

    @property
    def value(self):
        if self._cval.ndim == 0:
            return np.float64(self._cval)
        return self._cval.copy()


class Variable(Expression):
    def __init__(self, shape=(), integer=False, name=None):
        if isinstance(shape, int):
            shape = (shape,)
        n = int(np.prod(shape)) if shape else 1
        _VAR_COUNTER[0] += 1
        self.id = _VAR_COUNTER[0]
        self.n = n
        self.integer = integer
        self._value = None
        super().__init__({self.id: (self, np.eye(n))}, np.zeros(n), tuple(shape))

    @property
    def value(self):
        if self._value is None:
            return None
        if not self.shape:
            return np.float64(self._value[0])
        return self._value.copy()

    @value.setter
    def value(self, v):
        self._value = None if v is None else np.atleast_1d(np.asarray(v, dtype=float))


class Constraint:
    def __init__(self, expr, kind):
        self.expr = expr  # expr (==|<=) 0
        self.kind = kind


def multiply(a, b):
    a, b = _as_expr(a), _as_expr(b)
    if a.is_constant():
        return b._scale(a.const if a.size > 1 else a.const[0])
    if b.is_constant():
        return a._scale(b.const if b.size > 1 else b.const[0])
    raise ValueError("multiply needs one constant operand")


def sum(expr):  # noqa: A001 (mirrors cvxpy.sum)
    expr = _as_expr(expr)
    terms = {k: (v, c.sum(axis=0, keepdims=True)) for k, (v, c) in expr.terms.items()}
    return Expression(terms, [expr.const.sum()], ())


class Minimize:
    def __init__(self, expr):
        self.expr = _as_expr(expr)


class Problem:
    last_record = None
    time_limit = float(__import__("os").environ.get("GOLDEN_MILP_TIME_LIMIT", "60"))
    # 0 = prove optimality outright (the proven-optimum fixtures); 1e-6 was round 1's setting
    mip_rel_gap = float(__import__("os").environ.get("GOLDEN_MIP_REL_GAP", "1e-6"))

    def __init__(self, objective, constraints):
        self.objective = objective
        self.constraints = list(constraints)
        self.status = None
        self.value = None

    def is_dcp(self):
        return True

    def _assemble(self):
        vars_ = {}
        for e in [self.objective.expr] + [c.expr for c in self.constraints]:
            for k, (v, _) in e.terms.items():
                vars_[k] = v
        order = sorted(vars_)
        off, col = {}, 0
        for k in order:
            off[k] = col
            col += vars_[k].n
        nvar = col

        def dense(e):
            M = np.zeros((e.size, nvar))
            for k, (v, c) in e.terms.items():
                M[:, off[k]:off[k] + v.n] += c
            return M

        cobj = dense(self.objective.expr)[0]
        eq_A, eq_b, ub_A, ub_b = [], [], [], []
        for c in self.constraints:
            M = dense(c.expr)
            if c.kind == "eq":
                eq_A.append(M)
                eq_b.append(-c.expr.const)
            else:
                ub_A.append(M)
                ub_b.append(-c.expr.const)
        integ = np.zeros(nvar, dtype=int)
        for k in order:
            if vars_[k].integer:
                integ[off[k]:off[k] + vars_[k].n] = 1
        A_eq = np.vstack(eq_A) if eq_A else np.zeros((0, nvar))
        b_eq = np.concatenate(eq_b) if eq_b else np.zeros(0)
        A_ub = np.vstack(ub_A) if ub_A else np.zeros((0, nvar))
        b_ub = np.concatenate(ub_b) if ub_b else np.zeros(0)
        return vars_, order, off, cobj, A_eq, b_eq, A_ub, b_ub, integ, float(self.objective.expr.const[0])

    @staticmethod
    def _run(cobj, A_eq, b_eq, A_ub, b_ub, integ):
        lim, gap = Problem.time_limit, Problem.mip_rel_gap
        if OWN is not None and CURRENT_HOME[0] not in OWN:     # another process proves this home
            lim, gap = float(__import__("os").environ.get("GOLDEN_OTHER_LIMIT", "2")), 1e-2
        cons = []
        if A_eq.shape[0]:
            cons.append(LinearConstraint(A_eq, b_eq, b_eq))
        if A_ub.shape[0]:
            cons.append(LinearConstraint(A_ub, -np.inf, b_ub))
        return milp(cobj, constraints=cons, integrality=integ,
                    bounds=Bounds(-np.inf, np.inf),
                    options={"time_limit": lim, "mip_rel_gap": gap, "presolve": True})

    def solve(self, solver=None, verbose=False, **kw):
        vars_, order, off, cobj, A_eq, b_eq, A_ub, b_ub, integ, c0 = self._assemble()
        t_start = __import__("time").time()
        res = self._run(cobj, A_eq, b_eq, A_ub, b_ub, integ)
        t_milp = __import__("time").time() - t_start
        relax = self._run(cobj, A_eq, b_eq, A_ub, b_ub, np.zeros_like(integ))
        # HiGHS milp status: 0 optimal, 1 iteration/time limit, 2 infeasible, 3 unbounded, 4 other
        status = {0: "optimal", 2: "infeasible", 3: "unbounded"}.get(res.status, "solver_error")
        if res.status == 1 and res.x is not None:
            # time limit with an incumbent: GLPK_MI would have run to its optimum; keep the
            # incumbent (its gap is recorded) rather than inventing a solver failure.
            status = "optimal"
        Problem.last_record = dict(cobj=cobj, A_eq=A_eq, b_eq=b_eq, A_ub=A_ub, b_ub=b_ub, integ=integ,
                                   order=[(vars_[k], off[k]) for k in order],
                                   status=status, milp_status=int(res.status),
                                   mip_gap=getattr(res, "mip_gap", None), milp_seconds=t_milp, x=None if res.x is None else res.x.copy(),
                                   obj=None if res.x is None else float(res.fun + c0),
                                   relax_status=relax.status,
                                   relax_x=None if relax.x is None else relax.x.copy(),
                                   relax_obj=None if relax.x is None else float(relax.fun + c0))
        if status == "solver_error":
            raise SolverError(res.message)
        if res.x is not None:
            # GLPK_MI reports integer columns as exact integers (glp_intopt rounds them,
            # floor(x + 0.5) -> never -0.0); HiGHS returns them within tolerance.
            x = res.x.copy()
            x[integ == 1] = np.floor(x[integ == 1] + 0.5)
            res.x = x
            Problem.last_record["x"] = x.copy()
        self.status = status
        if status == "optimal":
            for k in order:
                vars_[k].value = res.x[off[k]:off[k] + vars_[k].n]
            self.value = float(res.fun + c0)
        else:
            for k in order:
                vars_[k].value = None
        return self.value
