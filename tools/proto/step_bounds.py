"""Prototype: how many breakpoints of the step-function DP's V_k survive the prune
L_k(x) + V_k(x) <= U with L_k the LP cost-to-reach (the kernel's) vs a forward cell bound."""
import json, sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle import mpc as M, thermal as TH

def tw(v): return 1e-9 * (1 + abs(v))

def lp_reach(ch):
    """L_k (k = 1..H): convex PL lower bound of the cost to reach x_k from x0 (duties continuous)."""
    A, C, q, g, S = ch["A"], ch["C"], ch["q"], ch["g"], ch["S"]
    H = len(A); assert g > 0
    px, pv = np.array([ch["x0"]]), np.array([0.0]); L = [None] * (H + 1)
    for k in range(H):
        px = A[k] * px + C[k]; d = g * S; sg = q[k] / g
        sl = np.diff(pv) / np.diff(px) if len(px) > 1 else np.array([])
        j = int(np.sum(sl < sg))
        px = np.r_[px[:j + 1], px[j:] + d]; pv = np.r_[pv[:j + 1], pv[j:] + sg * d]
        lo, hi = TH._box(ch, k)
        if px[0] > hi or px[-1] < lo: return None
        a, b = max(lo, px[0]), min(hi, px[-1])
        va, vb = np.interp(a, px, pv), np.interp(b, px, pv)
        inn = (px > a) & (px < b)
        px, pv = np.r_[a, px[inn], b], np.r_[va, pv[inn], vb]
        L[k + 1] = (px, pv)
    return L

def lp_min(f, a, b):
    px, pv = f
    a, b = max(a, px[0]), min(b, px[-1])
    if a > b: return np.inf
    inn = (px > a) & (px < b)
    return min(np.interp(a, px, pv), np.interp(b, px, pv), pv[inn].min() if inn.any() else np.inf)

def cell_reach(ch, ncell):
    A, C, q, g, S = ch["A"], ch["C"], ch["q"], ch["g"], ch["S"]
    H = len(A)
    lo, hi = ch["lo"] - tw(ch["lo"]), ch["hi"] + tw(ch["hi"])
    e = np.linspace(lo, hi, ncell + 1); w = e[1] - e[0]
    R = [None] * (H + 1)
    x1 = A[0] * ch["x0"] + C[0] + g * np.arange(S + 1)
    r = np.full(ncell, np.inf)
    for u in range(S + 1):
        c = int(np.floor((x1[u] - lo) / w))
        if 0 <= c < ncell: r[c] = min(r[c], q[0] * u)
    R[1] = r
    for k in range(1, H):
        nr = np.full(ncell, np.inf); fin = np.nonzero(np.isfinite(r))[0]
        for u in range(S + 1):
            l = A[k] * e[fin] + C[k] + g * u; h = A[k] * e[fin + 1] + C[k] + g * u
            c0 = np.clip(np.floor((l - lo) / w).astype(int), 0, ncell - 1)
            c1 = np.clip(np.floor((h - lo) / w).astype(int), 0, ncell - 1)
            ok = (h >= lo) & (l <= hi)
            v = r[fin] + q[k] * u
            for off in range(0, 4):
                cc = c0 + off; m = ok & (cc <= c1)
                np.minimum.at(nr, cc[m], v[m])
        R[k + 1] = nr; r = nr
    return e, R

def kept(V, Lf, U, cells=None):
    """per stage k = 1..H-1: (breakpoint intervals of V_k, those with min bound + v <= U)"""
    out = []
    for k in range(1, len(V) - 1):
        B, val = V[k]
        n = len(val); m = 0
        for i in range(n):
            if not np.isfinite(val[i]): continue
            a, b = B[i], B[i + 1]
            if cells is None:
                lb = lp_min(Lf[k], a, b)
            else:
                e, R = cells
                w = e[1] - e[0]
                c0 = max(0, int(np.floor((a - e[0]) / w))); c1 = min(len(e) - 2, int(np.floor((b - e[0]) / w)))
                lb = R[k][c0:c1 + 1].min() if c1 >= c0 else np.inf
            if lb + val[i] <= U + 1e-9: m += 1
        out.append((n, m))
    return out

cases = json.load(open('/root/repo/tools/proto/narrow_cases.json'))
for cs in cases[:int(sys.argv[1]) if len(sys.argv) > 1 else 6]:
    hc = M.home_const(cs['home'])
    si = M.StepInput(t=cs['t'], T0=cs['T0'], Tw0=cs['Tw0'], E0=cs['E0'] or 0.0, oat=np.array(cs['oat']),
                     ghi=np.array(cs['ghi']), price=np.array(cs['price']), draw=np.array(cs['draw']), winter=cs['winter'])
    T = TH.solve_chain(TH.chain_T(hc, si))
    if T is None: print(cs['i'], cs['t'], 'T infeasible'); continue
    ch = TH.chain_W(hc, si, T[2])
    sol = TH.solve_chain(ch)
    if sol is None: print(cs['i'], cs['t'], 'W infeasible'); continue
    V = TH.value_functions(ch)
    L = lp_reach(ch)
    lb = L[len(ch['A'])][1].min()
    opt = sol[0]; ub = opt + 0.15 * abs(opt)
    U1 = lb + 0.65 * (ub - lb)
    row = [cs['i'], cs['t'], round(opt, 4), round(lb, 4)]
    tot = sum(n for n, _ in kept(V, L, np.inf))
    row.append(tot)
    for U in (opt, U1):
        row.append(sum(m for _, m in kept(V, L, U)))
    for nc in (1024, 4096):
        cr = cell_reach(ch, nc)
        lbc = cr[1][len(ch['A'])].min()
        row.append(round(lbc, 4))
        for U in (opt, U1):
            row.append(sum(m for _, m in kept(V, L, U, cells=cr)))
    print(row, flush=True)
