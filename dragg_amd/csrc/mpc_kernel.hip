// mpc_kernel.hip -- batched per-home HEMS MPC for MI355X (gfx950, CDNA4).
//
// One 64-lane workgroup (one wavefront) owns one home for one timestep.  The home's MILP
// (dragg/mpc_calc.py:291-446) is separable: the default path (int_mode round,
// mpc_direct_kernel) solves it exactly -- the two thermal integer chains by a forward
// Pareto-front DP (dp_front: labels (state, cost) with dominance filters on two bucket grids,
// optionally pruned by an LP cost-to-go bound), the battery LP by an exact convex
// piecewise-linear DP (battery_lp), PV curtailment in closed form -- in a first launch
// (DM_FRONT); homes whose chains leave the front DP's scope (front overflow, mixed-sign prices
// without a usable bound) are finished by a second launch (DM_BUCKET) with the bucketed DP.
// int_mode relax / round_lp (mpc_home_kernel) solve the LP relaxation by an OSQP-style ADMM
// whose block-tridiagonal KKT factor lives in LDS, with an exact basis polish every
// `check_every` iterations, then (round_lp) the same integer DP.  The reference's result
// extraction / fallback thermostat (mpc_calc.py:476-596) writes the per-home hash arrays in
// place.  See DESIGN.md for the formulation and roofline.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <limits.h>
#include <stdlib.h>
#include <stdio.h>

#include "../../include/dragg_mi355x.h"

#define DEV static __device__ __forceinline__

// sha-256 of this file and the header, stamped by dragg_amd/build.py (-DDRAGG_SOURCE_HASH): the host
// refuses a library whose stamp differs from the sources beside it (dragg_amd/_lib.py); the prefix lets
// the build find the stamp in the .so without loading it
#ifndef DRAGG_SOURCE_HASH
#define DRAGG_SOURCE_HASH "unstamped"
#endif
#define kSourcePrefix "dragg-source-sha256:"
static const char kSourceStamp[] = kSourcePrefix DRAGG_SOURCE_HASH;

namespace {

constexpr int NS = 8;        // variable slots per stage
constexpr int NR = 3;        // dynamics rows per stage
constexpr int RS = 4;        // row stride per stage in LDS
constexpr int WAVE = 64;
constexpr int NB_CAP = 336;          // DP buckets per chain (config ranges need <= ~327 at any dt)
constexpr int NBND = 8;              // box-boundary buckets per stage (dp_zspace; 4-5 in practice)
constexpr int NF = NB_CAP;              // front capacity (labels) of dp_front
constexpr int NF_BOUND = 240;           // ... when the LP bound is on: its W table follows the front
static_assert((NB_CAP + 8 - NF_BOUND) * 16 >= 3 * 64 * 8, "the W table lives in rmin past the front");
constexpr int NF_BIG = 2048;            // front capacity of the second launch's exact pass
constexpr int SECOND_SLOTS = 512;       // blocks of the persistent second launch (2 per CU)
constexpr int PRUNE_AT = 64;            // front size that switches on the LP-bound pruning
constexpr int NF_HOT = 168;             // front capacity of the hot launch (front_layout): less LDS
                                        //   per home, more homes per CU; a larger front defers
constexpr int NTB_HOT = 64;           // key / cost buckets per stage of the hot launch's front DP
                                      //   (small fronts: a one-bucket-per-lane scan; measured 128: +6 % time)
constexpr int NTB = 192;              // ... of the second launch's regular front DP and round_lp
constexpr int NTB_BIG = 256;          // ... of the big exact pass (fronts up to NF_BIG)
constexpr int NT_STEPS = 512;            // threads of a DM_NARROW block (8 waves)
constexpr double STEP_U_FRAC = 0.65;     // the step-function DP's first bound: lb + this (ub - lb)
constexpr int NARROW_SLOTS = 16;         // blocks of the persistent DM_NARROW launch
// the exact step-function DP (dp_steps, DM_NARROW)
constexpr int NP_CAP = 32768;             // breakpoints of one V_k
constexpr int POOL_CAP = 1 << 20;         // breakpoints of all V_k of one chain (the pool)
// merge points over the stages of one step-function DP pass: a bound on one chain's work (~40 ms at the
// measured ~25 M merge points/s of one block); the bench's narrow chains take 74-160 k
constexpr long long STEP_WORK_CAP = 2000000;
constexpr int STEP_MAXU = 16;             // duty values 0..S (S <= 15)
constexpr int MC_CAP = 8 * NP_CAP;        // merged candidate points of one stage ((S + 1) np, S <= 7)
constexpr int STEP_CH = 8;                // merged outputs per merge work item, at most (fewer on small stages)
constexpr int LW_ROWS = 256;              // rows of the LP bounds L_k / W_k per slot (H < LW_ROWS)
constexpr int NF_MID = 384;              // front capacity of the mid launch (DM_MID)
constexpr int RS_HOLD = 4;               // ILP = 2 front DP: child pairs held in registers from pass 1 to pass 3
// RL-priced chains (a price change at most stages): the exact front DPs prune by a cell bound -- a lower
// bound of the INTEGER cost-to-go per cell of a uniform grid over the chain's box (cell_rows), 1-3 %
// below the optimum where the LP cost-to-go is ~13 % below -- and a beam pass (fronts truncated to the
// BEAM_K labels of least cost + bound) gives the upper bound (measured on the bench's RL price, oracle
// prototype: the beam's schedule is the optimum on 18 of 20 chains, within 0.03 % on the others; the
// exact pass's fronts then hold 22-280 labels, where the LP bound and the bucketed schedule's cost left
// 30 % of the chains past 2,048)
constexpr int NCELL = 1024;              // cells of the grid
// a row of the cell bound in the workspace: NCELL 16-bit codes; code q is the lower bound offset + q scale with
// one (offset, scale) per home (from the chain's duty costs: every cost-to-go lies in [sum of the negative,
// sum of the positive stage costs]), rounded DOWN at encoding so that it stays below the f32 value it stands
// for; 0xFFFF is +inf.  Half the bytes of f32 rows (2 GB per launch at 10k homes, H = 48, round 5)
constexpr int CELL_STRIDE = NCELL;
constexpr unsigned CELL_INF = 0xFFFFu;
constexpr int BEAM_K = 32;               // labels a beam stage keeps (7 BEAM_K children fit NF_MID; measured
                                         //   RL action at 48: 20.1 ms, 32: 19.6 ms)
constexpr int CELL_TRIES = 8;            // bisection steps on the bound after a pass past the capacity
constexpr int NTB_MID = 128;             // ... and its key / cost buckets per stage
constexpr int MID_SLOTS_MAX = 2048;      // blocks of the persistent mid launch (~7 per CU at H = 48)
// exchange area of a multi-wave front DP: per-pass survivor masks, per-wave counts / ranges / minima
// (one mask per 64-child pass of a full front of `cap` labels with S = 6: 7 children per label)
__host__ __device__ constexpr int xch_passes(int cap) { return (cap * 7 + 63) / 64; }
__host__ __device__ constexpr int xch_bytes(int cap) { return xch_passes(cap) * 8 + 8 * 8 + 8 * 5 * 4; }
constexpr int NW_MID = 1;                // waves per home of the mid launch
constexpr int NW_BIG = 4;                // waves per home of the big launch (2 blocks per CU: 8 waves)
enum Slot { S_U = 0, S_W = 1, S_T = 2, S_TW = 3, S_CH = 4, S_DIS = 5, S_E = 6, S_PAD = 7 };

constexpr double SIGMA = 1e-6;
constexpr double ALPHA = 1.6;
constexpr double RHO0 = 0.1;
constexpr double RHO_EQ = 1e3;      // equality rows get RHO_EQ * rho (OSQP convention)
constexpr double TAP = 15.0;        // mpc_calc.py:181
constexpr double EPS_PINF = 1e-5;
constexpr double TOL_P = 1e-9;
constexpr double TOL_D = 1e-9;

// --------------------------------------------------------------------------------------
// LDS carve
// --------------------------------------------------------------------------------------
struct Lds {
    double *Lf, *Df;                   // [H][64] sub-diagonal factor blocks, inverse pivots
    double *al, *be, *beq;             // [H][3][8], [H][3][8], [H][4]
    double *x, *zb, *yb, *lo, *hi, *q; // [8H]
    double *r, *t1, *t2;               // [8H] rhs / solve temporaries
    double *ybp;                       // [8H] previous box duals (certificate)
    double *yeq, *zeq, *yeqp, *lam;    // [4H], [4H], [4H], [4(H+1)]
    double *draw, *oat, *ghi, *price;  // [H+1], [H+1], [H+1], [H+1]
    double *sc;                        // [32] scalars
    int *at, *basic, *seg;             // [8H], [4H], [12H]
};

__host__ __device__ inline int lds_doubles(int H) {
    return 64 * H * 2 + 24 * H * 2 + 4 * H + 8 * H * 10 + 4 * H * 3 + 4 * (H + 1) + 4 * (H + 1) + 32 +
           (8 * H + 4 * H + 12 * H + 1) / 2 + 2;
}

DEV Lds carve(double* s, int H) {
    Lds L;
    L.Lf = s; s += 64 * H;
    L.Df = s; s += 64 * H;
    L.al = s; s += 24 * H;
    L.be = s; s += 24 * H;
    L.beq = s; s += 4 * H;
    L.x = s; s += 8 * H;
    L.lo = s; s += 8 * H;
    L.hi = s; s += 8 * H;
    L.q = s; s += 8 * H;
    L.zb = s; s += 8 * H;      // zb, yb, r, t1, t2, ybp: contiguous 48H doubles, reused as
    L.yb = s; s += 8 * H;      // the integer DP's bin arrays once the ADMM has finished
    L.r = s; s += 8 * H;
    L.t1 = s; s += 8 * H;
    L.t2 = s; s += 8 * H;
    L.ybp = s; s += 8 * H;
    L.yeq = s; s += 4 * H;
    L.zeq = s; s += 4 * H;
    L.yeqp = s; s += 4 * H;
    L.lam = s; s += 4 * (H + 1);
    L.draw = s; s += H + 1;
    L.oat = s; s += H + 1;
    L.ghi = s; s += H + 1;
    L.price = s; s += H + 1;
    L.sc = s; s += 32;
    L.at = reinterpret_cast<int*>(s);
    L.basic = L.at + 8 * H;
    L.seg = L.basic + 4 * H;
    return L;
}

// --------------------------------------------------------------------------------------
// wave helpers
// --------------------------------------------------------------------------------------
DEV double sum8(double v) {           // sum over the 8 lanes of a group (lane bits 0..2)
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    return v;
}
DEV double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
DEV double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
DEV bool wave_any(bool p) { return __any(p); }

// Wave-wide reductions and scans on DPP lane moves (VALU, no LDS round trip as __shfl_*'s
// ds_bpermute takes): butterfly inside each 16-lane row (quad_perm xor 1, xor 2, half-row
// and row mirrors), then the four row results read into scalars and combined in row order.
// Every lane returns the same value; the combination order is fixed, so results are
// deterministic.
template <int CTRL, typename T>
DEV T dpp_mov(T v) { return __builtin_amdgcn_update_dpp((T)0, v, CTRL, 0xf, 0xf, true); }
// v_readlane on the 32-bit halves (the builtin takes an int: a double would be converted)
DEV int read_lane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
DEV unsigned read_lane(unsigned v, int l) { return (unsigned)__builtin_amdgcn_readlane((int)v, l); }
DEV double read_lane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <typename T, typename Op>
DEV T dpp_reduce(T v, Op op) {
    v = op(v, dpp_mov<0xB1>(v));          // quad_perm [1,0,3,2]
    v = op(v, dpp_mov<0x4E>(v));          // quad_perm [2,3,0,1]
    v = op(v, dpp_mov<0x141>(v));         // row_half_mirror
    v = op(v, dpp_mov<0x140>(v));         // row_mirror
    const T r0 = read_lane(v, 0), r1 = read_lane(v, 16);
    const T r2 = read_lane(v, 32), r3 = read_lane(v, 48);
    return op(op(r0, r1), op(r2, r3));
}
DEV double dpp_sum(double v) { return dpp_reduce(v, [](double a, double b) { return a + b; }); }
DEV int dpp_isum(int v) { return dpp_reduce(v, [](int a, int b) { return a + b; }); }
DEV int dpp_imin(int v) { return dpp_reduce(v, [](int a, int b) { return min(a, b); }); }
DEV int dpp_imax(int v) { return dpp_reduce(v, [](int a, int b) { return max(a, b); }); }
// inclusive prefix sum over the 64 lanes: Hillis-Steele inside each row (row_shr 1, 2, 4, 8;
// lanes shifted in from outside the row read 0), then the totals of the rows below added
DEV double dpp_scan(double v, int lane) {
    v += dpp_mov<0x111>(v);
    v += dpp_mov<0x112>(v);
    v += dpp_mov<0x114>(v);
    v += dpp_mov<0x118>(v);
    const double t0 = read_lane(v, 15), t1 = read_lane(v, 31);
    const double t2 = read_lane(v, 47);
    const int row = lane >> 4;
    const double t01 = t0 + t1;
    const double off = row == 0 ? 0.0 : row == 1 ? t0 : row == 2 ? t01 : t01 + t2;
    return row == 0 ? v : v + off;
}

// order LDS accesses between the lanes of ONE wave (code running on a single wave of a
// multi-wave workgroup must not use __syncthreads)
DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// workgroup reductions for nt = 64 * waves threads (red: >= nt / 64 doubles of LDS scratch);
// the per-wave partials are combined in wave order, so the result is deterministic
DEV double block_sum(double v, double* red, int lane, int nt) {
    v = wave_sum(v);
    if (nt <= WAVE) return v;
    __syncthreads();
    if ((lane & (WAVE - 1)) == 0) red[lane / WAVE] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < nt / WAVE; ++i) s += red[i];
    __syncthreads();
    return s;
}
DEV double block_max(double v, double* red, int lane, int nt) {
    v = wave_max(v);
    if (nt <= WAVE) return v;
    __syncthreads();
    if ((lane & (WAVE - 1)) == 0) red[lane / WAVE] = v;
    __syncthreads();
    double s = red[0];
    for (int i = 1; i < nt / WAVE; ++i) s = fmax(s, red[i]);
    __syncthreads();
    return s;
}

// per-phase shader-cycle stamps (dragg_mpc_out.cycles; diagnostic, off when NULL)
struct Prof {
    unsigned long long acc[DRAGG_NPHASE];
    unsigned long long t;
    bool on;
    __device__ __forceinline__ void start(bool enable) {
        on = enable;
        for (int i = 0; i < DRAGG_NPHASE; ++i) acc[i] = 0;
        t = on ? __builtin_amdgcn_s_memtime() : 0;
    }
    __device__ __forceinline__ void mark(int phase) {
        if (!on) return;
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        acc[phase] += n - t;
        t = n;
    }
};

// --------------------------------------------------------------------------------------
// keyed season noise: Philox4x32-10 + Box-Muller (replaces the worker-global
// np.random.randn of mpc_calc.py:222, which is not reproducible across runs)
// --------------------------------------------------------------------------------------
DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
DEV void normal_pair(uint64_t seed, int home, int t, int pair, double* z0, double* z1) {
    uint32_t c[4] = {(uint32_t)home, (uint32_t)t, (uint32_t)pair, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t a = ((uint64_t)(c[0] >> 5) << 26) | (c[1] >> 6);
    const uint64_t b = ((uint64_t)(c[2] >> 5) << 26) | (c[3] >> 6);
    const double u1 = ((double)a + 1.0) * 0x1.0p-53;   // (0, 1]
    const double u2 = (double)b * 0x1.0p-53;           // [0, 1)
    const double rad = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586 * u2;
    *z0 = rad * cos(th);
    *z1 = rad * sin(th);
}

// Python's float(repr(v)[0]) for the fallback's duty parse (mpc_calc.py:537-539).
// repr uses scientific notation below 1e-4.  Returns -1 where the reference raises.
DEV double leading_char_value(double v) {
    if (!(v == v) || isinf(v) || v < 0.0 || signbit(v)) return -1.0;   // 'n', 'i', '-'
    if (v == 0.0) return 0.0;
    if (v >= 1e-4) return v < 1.0 ? 0.0 : floor(v / pow(10.0, floor(log10(v))));
    double e = floor(log10(v));
    double d = floor(v / pow(10.0, e));
    if (d >= 10.0) d = 9.0;
    if (d < 1.0) d = 1.0;
    return d;
}

// --------------------------------------------------------------------------------------
// per-home scalars (registers, identical in every lane)
// --------------------------------------------------------------------------------------
struct Home {
    int H, S, dt, type, nrows;
    bool batt, pv, winter;
    double R, C, Pc, Ph, Rw, Pw, Cw, V, Tmin, Tmax, Twmin, Twmax, Tinit, Twinit;
    double brate, Emin, Emax, etac, etad, Einit, pvA, pvEta;
    double gamma;
    // derived
    double inv_c, inv_w, iR, iRw, aT, g, e, f, Pact;
    // step inputs
    int t, counter;
    double T0, Tw0, E0;
};

DEV void load_params(Home& h, const double* P, int N, int i) {
    h.R = P[DRAGG_P_R * N + i];       h.C = P[DRAGG_P_C * N + i];
    h.Pc = P[DRAGG_P_PC * N + i];     h.Ph = P[DRAGG_P_PH * N + i];
    h.Rw = P[DRAGG_P_RW * N + i];     h.Pw = P[DRAGG_P_PW * N + i];
    h.Cw = P[DRAGG_P_CW * N + i];     h.V = P[DRAGG_P_V * N + i];
    h.Tmin = P[DRAGG_P_TMIN * N + i]; h.Tmax = P[DRAGG_P_TMAX * N + i];
    h.Twmin = P[DRAGG_P_TWMIN * N + i]; h.Twmax = P[DRAGG_P_TWMAX * N + i];
    h.Tinit = P[DRAGG_P_TINIT * N + i]; h.Twinit = P[DRAGG_P_TWINIT * N + i];
    h.brate = P[DRAGG_P_BRATE * N + i]; h.Emin = P[DRAGG_P_EMIN * N + i];
    h.Emax = P[DRAGG_P_EMAX * N + i];   h.etac = P[DRAGG_P_ETAC * N + i];
    h.etad = P[DRAGG_P_ETAD * N + i];   h.Einit = P[DRAGG_P_EINIT * N + i];
    h.pvA = P[DRAGG_P_PVAREA * N + i];  h.pvEta = P[DRAGG_P_PVEFF * N + i];
}

DEV void derive(Home& h) {
    h.inv_c = 1.0 / (h.C * h.dt);                 // 1 / (home_c * dt)   mpc_calc.py:317
    h.inv_w = 1.0 / (h.Cw * h.dt);                // 1 / (wh_c * dt)     mpc_calc.py:332
    h.iR = 1.0 / h.R;
    h.iRw = 1.0 / h.Rw;
    h.aT = 1.0 + (-h.iR * 3600) * h.inv_c;        // coefficient of T_k in T_{k+1}
    if (h.winter) { h.g = h.Ph * 3600 * h.inv_c;    h.Pact = h.S * h.Ph; }
    else          { h.g = -(h.Pc * 3600 * h.inv_c); h.Pact = h.S * h.Pc; }
    h.e = h.iRw * 3600 * h.inv_w;                 // coefficient of T_{k+1} in Tw_{k+1}
    h.f = h.Pw * 3600 * h.inv_w;                  // coefficient of w_k
}

DEV bool slot_active(const Home& h, int j) { return j < 4 || (h.batt && j < 7); }

// --------------------------------------------------------------------------------------
// build the chain LP (add_base/pv/battery_constraints, set_*_p_grid, solve_mpc)
// --------------------------------------------------------------------------------------
DEV void build(const Home& h, const Lds& L, int lane) {
    const int H = h.H;
    for (int k = lane; k < H; k += WAVE) {
        double* A = L.al + k * 24;
        double* B = L.be + k * 24;
#pragma unroll
        for (int m = 0; m < 24; ++m) { A[m] = 0.0; B[m] = 0.0; }
        const double df = L.draw[k + 1] / h.V;
        const double rem = 1 - df;
        // indoor air (mpc_calc.py:314-317)
        A[0 * 8 + S_T] = 1.0; A[0 * 8 + S_U] = -h.g; B[0 * 8 + S_T] = -h.aT;
        L.beq[k * RS + 0] = L.oat[k + 1] * h.iR * 3600 * h.inv_c;
        // water heater with draw mixing (mpc_calc.py:330-332)
        const double ck = rem + (-rem * h.iRw) * 3600 * h.inv_w;
        const double d15 = df * TAP;
        A[1 * 8 + S_TW] = 1.0; A[1 * 8 + S_T] = -h.e; A[1 * 8 + S_W] = -h.f; B[1 * 8 + S_TW] = -ck;
        L.beq[k * RS + 1] = d15 + ((-d15) * h.iRw) * 3600 * h.inv_w;
        L.beq[k * RS + 2] = 0.0;
        L.beq[k * RS + 3] = 0.0;
        // battery state of charge (mpc_calc.py:363-365)
        if (h.batt) {
            A[2 * 8 + S_E] = 1.0; B[2 * 8 + S_E] = -1.0;
            A[2 * 8 + S_CH] = -h.etac / h.dt;
            A[2 * 8 + S_DIS] = -(1.0 / h.etad) / h.dt;
        }
        // bounds and costs (mpc_calc.py:318-349, 367-372, 441-446)
        const double w = pow(h.gamma, (double)k) * L.price[k];
        const int o = k * NS;
        L.lo[o + S_U] = 0.0;      L.hi[o + S_U] = h.S;      L.q[o + S_U] = w * h.Pact;
        L.lo[o + S_W] = 0.0;      L.hi[o + S_W] = h.S;      L.q[o + S_W] = w * (h.S * h.Pw);
        L.lo[o + S_T] = h.Tmin;   L.hi[o + S_T] = h.Tmax;   L.q[o + S_T] = 0.0;
        L.lo[o + S_TW] = h.Twmin; L.hi[o + S_TW] = h.Twmax; L.q[o + S_TW] = 0.0;
        if (h.batt) {
            L.lo[o + S_CH] = 0.0;       L.hi[o + S_CH] = h.brate;  L.q[o + S_CH] = w * h.S;
            L.lo[o + S_DIS] = -h.brate; L.hi[o + S_DIS] = 0.0;     L.q[o + S_DIS] = w * h.S;
            L.lo[o + S_E] = h.Emin;     L.hi[o + S_E] = h.Emax;    L.q[o + S_E] = 0.0;
        } else {
            L.lo[o + S_CH] = L.hi[o + S_CH] = L.q[o + S_CH] = 0.0;
            L.lo[o + S_DIS] = L.hi[o + S_DIS] = L.q[o + S_DIS] = 0.0;
            L.lo[o + S_E] = L.hi[o + S_E] = L.q[o + S_E] = 0.0;
        }
        L.lo[o + S_PAD] = L.hi[o + S_PAD] = L.q[o + S_PAD] = 0.0;
    }
    __syncthreads();
    if (lane == 0) {
        // fold the fixed initial states into stage 0 (mpc_calc.py:313, 329, 366)
        const double rem1 = 1 - L.draw[1] / h.V;
        const double c0 = rem1 + (-rem1 * h.iRw) * 3600 * h.inv_w;
        const double d0 = L.beq[1];
        L.beq[0] += h.aT * h.T0;
        L.beq[1] += c0 * h.Tw0;
        if (h.batt) L.beq[2] += h.E0;
        // temp_wh (the un-mixed one-step value, mpc_calc.py:336-340) differs from Tw_1 by a
        // constant, so its bounds become a tightened box on Tw_1.
        const double Kc = (h.Tw0 + ((-h.Tw0) * h.iRw) * 3600 * h.inv_w) - c0 * h.Tw0 - d0;
        L.lo[S_TW] = fmax(h.Twmin, h.Twmin - Kc);
        L.hi[S_TW] = fmin(h.Twmax, h.Twmax - Kc);
        L.sc[8] = Kc;
    }
    __syncthreads();
}

// Exact forward-interval feasibility of the T and E chains (+ outer test for Tw).
DEV bool presolve_infeasible(const Home& h, const Lds& L) {
    if (!(h.Twmin <= h.Tw0 && h.Tw0 <= h.Twmax)) return true;          // temp_wh_ev[0] bounds
    double Tlo = h.T0, Thi = h.T0, Wlo = h.Tw0, Whi = h.Tw0, Elo = h.E0, Ehi = h.E0;
    const double gS = h.g * h.S;
    for (int k = 0; k < h.H; ++k) {
        const int o = k * NS;
        const double bk = L.oat[k + 1] * h.iR * 3600 * h.inv_c;
        double lo = h.aT * Tlo + bk + fmin(0.0, gS), hi = h.aT * Thi + bk + fmax(0.0, gS);
        Tlo = fmax(lo, L.lo[o + S_T]); Thi = fmin(hi, L.hi[o + S_T]);
        if (Tlo > Thi + TOL_P * (1 + fabs(Thi))) return true;
        const double ck = (k == 0) ? 0.0 : -L.be[k * 24 + 1 * 8 + S_TW];
        const double bw = L.beq[k * RS + 1];           // stage 0 already holds c0*Tw0
        lo = ck * Wlo + bw + h.e * Tlo; hi = ck * Whi + bw + h.e * Thi + h.f * h.S;
        Wlo = fmax(lo, L.lo[o + S_TW]); Whi = fmin(hi, L.hi[o + S_TW]);
        if (Wlo > Whi + TOL_P * (1 + fabs(Whi))) return true;
        if (h.batt) {
            lo = Elo - h.brate * (1.0 / h.etad) / h.dt; hi = Ehi + h.brate * h.etac / h.dt;
            Elo = fmax(lo, h.Emin); Ehi = fmin(hi, h.Emax);
            if (Elo > Ehi + TOL_P * (1 + fabs(Ehi))) return true;
        }
    }
    return false;
}

// --------------------------------------------------------------------------------------
// KKT = sigma I + rho_eq A_eq'A_eq + rho I (box rows): block-tridiagonal, 8x8 blocks,
// block LDL' with explicit inverse pivots.  lane = 8*i + j owns entry (i, j).
// --------------------------------------------------------------------------------------
DEV void factor(const Home& h, const Lds& L, int lane, double rho) {
    const int i = lane >> 3, j = lane & 7;
    const double rq = RHO_EQ * rho;
    const bool acti = slot_active(h, i);
    for (int k = 0; k < h.H; ++k) {
        const double* A = L.al + k * 24;
        double kd = 0.0;
#pragma unroll
        for (int r = 0; r < NR; ++r) kd += A[r * 8 + i] * A[r * 8 + j];
        if (k + 1 < h.H) {
            const double* B1 = L.be + (k + 1) * 24;
#pragma unroll
            for (int r = 0; r < NR; ++r) kd += B1[r * 8 + i] * B1[r * 8 + j];
        }
        kd *= rq;
        if (i == j) kd += SIGMA + (acti ? rho : 1.0);
        if (k > 0) {
            const double* B = L.be + k * 24;
            double ko = 0.0;
#pragma unroll
            for (int r = 0; r < NR; ++r) ko += A[r * 8 + i] * B[r * 8 + j];
            ko *= rq;                                     // K_{k,k-1}(i, j)
            const double* Dp = L.Df + (k - 1) * 64;
            double lk = 0.0;
#pragma unroll
            for (int l = 0; l < 8; ++l) lk += __shfl(ko, i * 8 + l) * Dp[l * 8 + j];
            L.Lf[k * 64 + lane] = lk;                     // L_k = K_{k,k-1} D_{k-1}^{-1}
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < 8; ++l) s += __shfl(lk, i * 8 + l) * __shfl(ko, j * 8 + l);
            kd -= s;                                      // D_k = K_kk - L_k K_{k,k-1}'
        }
        // in-place Gauss-Jordan sweep inverse of the SPD pivot block
        double m = kd;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const double piv = __shfl(m, p * 9);
            const double mip = __shfl(m, i * 8 + p);
            const double mpj = __shfl(m, p * 8 + j);
            const double ip = 1.0 / piv;
            if (i == p && j == p) m = ip;
            else if (i == p) m = mpj * ip;
            else if (j == p) m = -mip * ip;
            else m = m - mip * mpj * ip;
        }
        L.Df[k * 64 + lane] = m;
    }
    __syncthreads();
}

// solve KKT x = r in place (r -> x)
DEV void kkt_solve(const Home& h, const Lds& L, int lane) {
    const int i = lane >> 3, j = lane & 7;
    const int H = h.H;
    for (int k = 0; k < H; ++k) {                          // forward: z_k = r_k - L_k z_{k-1}
        double s = 0.0;
        if (k > 0) s = sum8(L.Lf[k * 64 + lane] * L.t1[(k - 1) * 8 + j]);
        if (j == 0) L.t1[k * 8 + i] = L.r[k * 8 + i] - s;
        __syncthreads();
    }
    for (int k = 0; k < H; ++k) {                          // v_k = D_k^{-1} z_k
        const double s = sum8(L.Df[k * 64 + lane] * L.t1[k * 8 + j]);
        if (j == 0) L.t2[k * 8 + i] = s;
    }
    __syncthreads();
    for (int k = H - 1; k >= 0; --k) {                     // backward: x_k = v_k - L_{k+1}' x_{k+1}
        double s = 0.0;
        if (k + 1 < H) s = sum8(L.Lf[(k + 1) * 64 + j * 8 + i] * L.r[(k + 1) * 8 + j]);
        if (j == 0) L.r[k * 8 + i] = L.t2[k * 8 + i] - s;
        __syncthreads();
    }
}

// A_eq' v at element e=(k, jj) for a row vector v[4H]
DEV double at_times(const Home& h, const Lds& L, const double* v, int k, int jj) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < NR; ++r) s += L.al[k * 24 + r * 8 + jj] * v[k * RS + r];
    if (k + 1 < h.H) {
#pragma unroll
        for (int r = 0; r < NR; ++r) s += L.be[(k + 1) * 24 + r * 8 + jj] * v[(k + 1) * RS + r];
    }
    return s;
}
// A_eq x at row (k, r) for an element vector x[8H]
DEV double a_times(const Lds& L, const double* xv, int k, int r) {
    double s = 0.0;
#pragma unroll
    for (int jj = 0; jj < NS; ++jj) s += L.al[k * 24 + r * 8 + jj] * xv[k * 8 + jj];
    if (k > 0) {
#pragma unroll
        for (int jj = 0; jj < NS; ++jj) s += L.be[k * 24 + r * 8 + jj] * xv[(k - 1) * 8 + jj];
    }
    return s;
}

// --------------------------------------------------------------------------------------
// exact basis polish.  The LP is three scalar "chains" (indoor T driven by the hvac duty,
// tank Tw driven by the wh duty and T, battery E driven by charge/discharge):
//     x_{k+1} = A_k x_k + sum_i B_{k,i} v_{k,i} + C_k ,   boxes on x_{k+1} and v_{k,i}.
// Given the ADMM active-set guess, a vertex of such a chain is fixed segment by segment:
// between two states pinned at a bound exactly one input is basic (free), which is solved
// by a forward sweep from the segment start and a backward sweep from its pinned end.
// Row duals follow by the mirrored recursion; degenerate segments (no free input) pick,
// among the locally dual-feasible bases, the one whose first dual is most favourable to
// the previous pinned state.  Success = every bound and every reduced-cost sign holds,
// i.e. an exact, certified LP optimum (the vertex a simplex solver would return).
// Runs on lane 0 (the work is a few sequential passes over the horizon).
// --------------------------------------------------------------------------------------
struct Chain {
    int H, sx, ni, sv0, sv1, row;
    double x0;
    const double *A, *B, *C, *kap;   // [H], [H][2], [H], [H]   (scratch in L.r)
    int* seg;                        // [H][4]: start, end, m (-1 tail, -2 degenerate), mi
    int nseg;
};

DEV int chain_sv(const Chain& c, int i) { return i == 0 ? c.sv0 : c.sv1; }

DEV double chain_bv(const Chain& c, const Lds& L, int kk) {
    double bv = 0.0;
    for (int i = 0; i < c.ni; ++i) bv += c.B[kk * 2 + i] * L.t1[kk * 8 + chain_sv(c, i)];
    return bv;
}

// Forward/backward vertex solve of one chain.  The ADMM classification (L.at) is repaired
// in place where it is inconsistent with a vertex:
//  * a pinned segment whose forward sweep lands strictly inside the state box -> unpin it;
//  * a pinned segment that misses its bound -> free the latest input that can close the gap;
//  * two free inputs in one segment -> pin the state between them closest to its bound.
DEV bool chain_primal(Chain& c, const Lds& L) {
    const int H = c.H;
    double* t1 = L.t1;
    c.nseg = 0;
    int start = 0, rescans = 0;
    double xprev = c.x0;
    while (start < H) {
        int j = -1;
        for (int kk = start; kk < H; ++kk)
            if (L.at[kk * 8 + c.sx] != 0) { j = kk + 1; break; }
        const int end = j > 0 ? j : H;
        int nfree = 0, m = -1, mi = 0, mfirst = -1;
        for (int kk = start; kk < end; ++kk)
            for (int i = 0; i < c.ni; ++i)
                if (L.at[kk * 8 + chain_sv(c, i)] == 0) {
                    if (mfirst < 0) mfirst = kk;
                    ++nfree; m = kk; mi = i;
                }
        if (j < 0) {                                            // tail: no pinned end
            if (nfree) return false;
            double xc = xprev;
            for (int kk = start; kk < end; ++kk) {
                xc = c.A[kk] * xc + chain_bv(c, L, kk) + c.C[kk];
                t1[kk * 8 + c.sx] = xc;
            }
            int* sg = c.seg + 4 * c.nseg++;
            sg[0] = start; sg[1] = end; sg[2] = -1; sg[3] = 0;
            break;
        }
        const int ej = (j - 1) * 8 + c.sx;
        const double xlo = L.lo[ej], xhi = L.hi[ej];
        const double xj = (L.at[ej] == -1) ? xlo : xhi;
        if (nfree > 1) {
            int bk = -1;
            double best = 0.0;
            for (int kk = mfirst; kk < m; ++kk) {
                const int e = kk * 8 + c.sx;
                const double span = fmax(L.hi[e] - L.lo[e], 1e-12);
                const double dist = fmin(fabs(L.x[e] - L.lo[e]), fabs(L.hi[e] - L.x[e])) / span;
                if (bk < 0 || dist < best) { best = dist; bk = kk; }
            }
            if (bk < 0 || rescans > H) return false;
            const int e = bk * 8 + c.sx;
            L.at[e] = (fabs(L.x[e] - L.lo[e]) <= fabs(L.hi[e] - L.x[e])) ? -1 : 1;
            t1[e] = L.at[e] == -1 ? L.lo[e] : L.hi[e];
            ++rescans;
            continue;
        }
        if (nfree == 0) {                                       // degenerate / misclassified
            double xc = xprev;
            for (int kk = start; kk < end; ++kk) {
                xc = c.A[kk] * xc + chain_bv(c, L, kk) + c.C[kk];
                t1[kk * 8 + c.sx] = xc;
            }
            const bool at_b = fabs(xc - xj) <= TOL_P * (1 + fabs(xj));
            if (!at_b && xc >= xlo - TOL_P * (1 + fabs(xlo)) && xc <= xhi + TOL_P * (1 + fabs(xhi)) &&
                rescans <= H) {
                L.at[ej] = 0;                                   // lands inside the box: not pinned
                ++rescans;
                continue;
            }
            if (at_b) {
                t1[ej] = xj;
                int* sg = c.seg + 4 * c.nseg++;
                sg[0] = start; sg[1] = end; sg[2] = -2; sg[3] = 0;
                xprev = xj;
                start = end;
                continue;
            }
            // misses its bound: free the latest input whose move closes the gap within its box
            m = -1;
            double gain = 1.0;
            for (int kk = end - 1; kk >= start && m < 0; --kk) {
                for (int i = 0; i < c.ni; ++i) {
                    const double b = c.B[kk * 2 + i];
                    if (b == 0.0) continue;
                    const int ev = kk * 8 + chain_sv(c, i);
                    const double nv = t1[ev] + (xj - xc) / (b * gain);
                    if (nv >= L.lo[ev] - TOL_P * (1 + fabs(L.lo[ev])) && nv <= L.hi[ev] + TOL_P * (1 + fabs(L.hi[ev]))) {
                        m = kk; mi = i;
                        break;
                    }
                }
                gain *= c.A[kk];
            }
            if (m < 0) return false;
        }
        // exactly one basic input v_{m,mi}: forward to x_m, backward from the pinned x_j
        double xc = xprev;
        for (int kk = start; kk < m; ++kk) {
            xc = c.A[kk] * xc + chain_bv(c, L, kk) + c.C[kk];
            t1[kk * 8 + c.sx] = xc;
        }
        const double xm = xc;
        double xn = xj;
        t1[ej] = xj;
        for (int kk = end - 1; kk > m; --kk) {
            xn = (xn - chain_bv(c, L, kk) - c.C[kk]) / c.A[kk];
            t1[(kk - 1) * 8 + c.sx] = xn;
        }
        double rest = 0.0;
        for (int i = 0; i < c.ni; ++i)
            if (i != mi) rest += c.B[m * 2 + i] * t1[m * 8 + chain_sv(c, i)];
        t1[m * 8 + chain_sv(c, mi)] = (xn - c.A[m] * xm - rest - c.C[m]) / c.B[m * 2 + mi];
        int* sg = c.seg + 4 * c.nseg++;
        sg[0] = start; sg[1] = end; sg[2] = m; sg[3] = mi;
        xprev = xj;
        start = end;
    }
    return true;
}

DEV bool sign_ok(int a, double d, double tol) { return !((a == -1 && d < -tol) || (a == 1 && d > tol)); }

// duals of one segment given its basic choice (cand: -1 = pinned/tail state basic, else
// k*2+i of the basic input); writes lam[i0..end-1] (lam[end] is known)
DEV void seg_duals(const Chain& c, const Lds& L, double* lam, int i0, int end, int cand) {
    auto An = [&](int k) { return k + 1 < c.H ? c.A[k + 1] : 0.0; };
    if (cand < 0) {
        for (int k = end - 1; k >= i0; --k) lam[k] = An(k) * lam[k + 1] - L.q[k * 8 + c.sx] - c.kap[k];
        return;
    }
    const int m = cand >> 1, mi = cand & 1;
    lam[m] = L.q[m * 8 + chain_sv(c, mi)] / c.B[m * 2 + mi];
    for (int k = m - 1; k >= i0; --k) lam[k] = An(k) * lam[k + 1] - L.q[k * 8 + c.sx] - c.kap[k];
    for (int k = m; k < end - 1; ++k) lam[k + 1] = (lam[k] + L.q[k * 8 + c.sx] + c.kap[k]) / An(k);
}

DEV bool chain_dual(const Chain& c, const Lds& L, double* lam /*[H+1]*/, double* trial, double tol) {
    const int H = c.H;
    auto An = [&](int k) { return k + 1 < H ? c.A[k + 1] : 0.0; };
    lam[H] = 0.0;
    for (int s = c.nseg - 1; s >= 0; --s) {
        const int* sg = c.seg + 4 * s;
        const int i0 = sg[0], end = sg[1], m = sg[2], mi = sg[3];
        if (m >= 0) {
            seg_duals(c, L, lam, i0, end, m * 2 + mi);
        } else if (m == -1) {
            seg_duals(c, L, lam, i0, end, -1);
        } else {
            const int side = i0 > 0 ? L.at[(i0 - 1) * 8 + c.sx] : 0;
            bool found = false;
            double best = 0.0;
            for (int cand = -1; cand < 2 * (end - i0); ++cand) {
                const int cc = cand < 0 ? -1 : ((i0 + (cand >> 1)) * 2 + (cand & 1));
                if (cand >= 0 && (cand & 1) >= c.ni) continue;
                for (int k = i0; k <= end; ++k) trial[k] = lam[k];
                seg_duals(c, L, trial, i0, end, cc);
                bool fine = true;
                for (int k = i0; k < end && fine; ++k)
                    for (int i = 0; i < c.ni; ++i) {
                        if (cc == k * 2 + i) continue;
                        const int e = k * 8 + chain_sv(c, i);
                        if (!sign_ok(L.at[e], L.q[e] - c.B[k * 2 + i] * trial[k], tol)) fine = false;
                    }
                if (fine && cc >= 0) {
                    const int k = end - 1;
                    const double dx = L.q[k * 8 + c.sx] + c.kap[k] + trial[k] - An(k) * trial[k + 1];
                    if (!sign_ok(L.at[k * 8 + c.sx], dx, tol)) fine = false;
                }
                if (!fine) continue;
                const double score = trial[i0] * (side == -1 ? 1.0 : (side == 1 ? -1.0 : 0.0));
                if (!found || score < best) {
                    found = true;
                    best = score;
                    for (int k = i0; k < end; ++k) lam[k] = trial[k];
                }
            }
            if (!found) return false;
        }
    }
    // reduced costs of every nonbasic variable of the chain
    for (int s = 0; s < c.nseg; ++s) {
        const int* sg = c.seg + 4 * s;
        const int i0 = sg[0], end = sg[1], m = sg[2], mi = sg[3];
        for (int k = i0; k < end; ++k)
            for (int i = 0; i < c.ni; ++i) {
                if (m >= 0 && k == m && i == mi) continue;
                const int e = k * 8 + chain_sv(c, i);
                if (L.at[e] == 0) return false;
                if (!sign_ok(L.at[e], L.q[e] - c.B[k * 2 + i] * lam[k], tol)) return false;
            }
        if (m >= 0) {
            const int k = end - 1;
            const double dx = L.q[k * 8 + c.sx] + c.kap[k] + lam[k] - An(k) * lam[k + 1];
            if (!sign_ok(L.at[k * 8 + c.sx], dx, tol)) return false;
        }
    }
    return true;
}

// fill the chain coefficient scratch (L.r: A[H], B[2H], C[H], kap[H]) for chain `which`
// (0 = indoor T, 1 = tank Tw, 2 = battery E), consistent with build()
DEV void chain_coefs(const Home& h, const Lds& L, int which, Chain& c, int* seg) {
    const int H = h.H;
    double* A = L.r; double* B = L.r + H; double* C = L.r + 3 * H; double* kap = L.r + 4 * H;
    for (int k = 0; k < H; ++k) {
        kap[k] = 0.0;
        if (which == 0) {
            A[k] = h.aT; B[k * 2] = h.g; B[k * 2 + 1] = 0.0;
            C[k] = L.oat[k + 1] * h.iR * 3600 * h.inv_c;
        } else if (which == 1) {
            const double df = L.draw[k + 1] / h.V, rem = 1 - df, d15 = df * TAP;
            A[k] = rem + (-rem * h.iRw) * 3600 * h.inv_w; B[k * 2] = h.f; B[k * 2 + 1] = 0.0;
            C[k] = h.e * L.t1[k * 8 + S_T] + (d15 + ((-d15) * h.iRw) * 3600 * h.inv_w);
        } else {
            A[k] = 1.0; B[k * 2] = h.etac / h.dt; B[k * 2 + 1] = (1.0 / h.etad) / h.dt; C[k] = 0.0;
        }
    }
    c.H = H; c.A = A; c.B = B; c.C = C; c.kap = kap; c.seg = seg; c.nseg = 0;
    if (which == 0) { c.sx = S_T; c.ni = 1; c.sv0 = S_U; c.sv1 = S_U; c.row = 0; c.x0 = h.T0; }
    else if (which == 1) { c.sx = S_TW; c.ni = 1; c.sv0 = S_W; c.sv1 = S_W; c.row = 1; c.x0 = h.Tw0; }
    else { c.sx = S_E; c.ni = 2; c.sv0 = S_CH; c.sv1 = S_DIS; c.row = 2; c.x0 = h.E0; }
}

DEV bool polish(const Home& h, const Lds& L, int lane) {
    const int H = h.H, n = NS * H;
    for (int e = lane; e < n; e += WAVE) {
        const int jj = e & 7;
        int a = 2;                                          // 2 = inactive slot
        double v = 0.0;
        if (slot_active(h, jj)) {
            const double zb = L.zb[e], yb = L.yb[e];
            a = (zb - L.lo[e] < -yb) ? -1 : ((L.hi[e] - zb < yb) ? 1 : 0);
            v = (a == -1) ? L.lo[e] : (a == 1 ? L.hi[e] : L.x[e]);
        }
        L.at[e] = a;
        L.t1[e] = v;
    }
    double qmax = 0.0;
    for (int e = lane; e < n; e += WAVE) qmax = fmax(qmax, fabs(L.q[e]));
    qmax = wave_max(qmax);
    __syncthreads();
    if (lane == 0) {
        bool ok = true;
        double* mu = L.zeq;                 // [H+1] tank duals (zeq is scratch here)
        double* trial = L.t2;               // [H+1]
        Chain cT, cW, cE;
        // primal: T, then Tw (its C depends on T)
        chain_coefs(h, L, 0, cT, L.seg);
        ok = chain_primal(cT, L);
        if (ok) { chain_coefs(h, L, 1, cW, L.seg + 4 * H); ok = chain_primal(cW, L); }
        // duals: Tw first (mu), then T with the coupling kap_k = -e mu_k (T_{k+1} sits in row W_k)
        const double tol = TOL_D * (qmax + 1e-30);
        if (ok) ok = chain_dual(cW, L, mu, trial, tol);
        if (ok) {
            const int nsegT = cT.nseg;            // chain_coefs refills the scratch and resets nseg
            chain_coefs(h, L, 0, cT, L.seg);
            cT.nseg = nsegT;
            double* kap = L.r + 4 * H;
            for (int k = 0; k < H; ++k) kap[k] = -h.e * mu[k];
            double* lam = L.t2 + (H + 1);   // t2 holds 8H >= 2(H+1)
            ok = chain_dual(cT, L, lam, trial, tol);
        }
        if (ok && h.batt) {
            chain_coefs(h, L, 2, cE, L.seg + 8 * H);
            ok = chain_primal(cE, L);
            if (ok) ok = chain_dual(cE, L, L.t2 + 2 * (H + 1), trial, tol);
        }
        L.sc[0] = ok ? 0.0 : 1.0;
    }
    __syncthreads();
    if (L.sc[0] != 0.0) return false;
    bool bad = false;
    for (int e = lane; e < n; e += WAVE) {
        if (L.at[e] == 2) continue;
        const double v = L.t1[e];
        if (!(v >= L.lo[e] - TOL_P * (1 + fabs(L.lo[e])) && v <= L.hi[e] + TOL_P * (1 + fabs(L.hi[e])))) bad = true;
    }
    return !wave_any(bad);
}

// --------------------------------------------------------------------------------------
// OSQP-style ADMM on  min q'x  s.t.  A_eq x = b,  lo <= x <= hi
// returns dragg_status; on DRAGG_ST_OPTIMAL, L.x holds the exact vertex
// --------------------------------------------------------------------------------------
DEV int admm(const Home& h, const Lds& L, int lane, int max_iter, int check, int* iters, Prof& pf) {
    const int H = h.H, n = NS * H, m = RS * H;
    double rho = RHO0;
    for (int e = lane; e < n; e += WAVE) {
        L.x[e] = 0.0; L.yb[e] = 0.0; L.ybp[e] = 0.0;
        L.zb[e] = fmin(fmax(0.0, L.lo[e]), L.hi[e]);
    }
    for (int e = lane; e < m; e += WAVE) { L.yeq[e] = 0.0; L.yeqp[e] = 0.0; }
    __syncthreads();
    pf.mark(DRAGG_PH_ITER);
    factor(h, L, lane, rho);
    pf.mark(DRAGG_PH_FACTOR);
    for (int it = 1; it <= max_iter; ++it) {
        const double rq = RHO_EQ * rho;
        // rhs = sigma x - q + A_eq'(rq b - y_eq) + (rho z_b - y_b)
        for (int e = lane; e < m; e += WAVE) {
            const int r = e & 3;
            L.zeq[e] = (r < h.nrows) ? rq * L.beq[e] - L.yeq[e] : 0.0;
        }
        __syncthreads();
        for (int e = lane; e < n; e += WAVE) {
            const int k = e >> 3, jj = e & 7;
            L.r[e] = slot_active(h, jj)
                         ? SIGMA * L.x[e] - L.q[e] + at_times(h, L, L.zeq, k, jj) + rho * L.zb[e] - L.yb[e]
                         : 0.0;
        }
        __syncthreads();
        kkt_solve(h, L, lane);                             // L.r = x~
        for (int e = lane; e < m; e += WAVE) {
            const int k = e >> 2, r = e & 3;
            if (r < h.nrows) {
                const double zh = a_times(L, L.r, k, r);
                const double zt = ALPHA * zh + (1 - ALPHA) * L.beq[e];
                L.yeq[e] += rq * (zt - L.beq[e]);
            }
        }
        for (int e = lane; e < n; e += WAVE) {
            if (!slot_active(h, e & 7)) continue;
            const double xt = L.r[e];
            const double zt = ALPHA * xt + (1 - ALPHA) * L.zb[e];
            const double zn = fmin(fmax(zt + L.yb[e] / rho, L.lo[e]), L.hi[e]);
            L.yb[e] += rho * (zt - zn);
            L.x[e] = ALPHA * xt + (1 - ALPHA) * L.x[e];
            L.zb[e] = zn;
        }
        __syncthreads();
        if (it % check != 0) continue;
        pf.mark(DRAGG_PH_ITER);
        const bool pol = polish(h, L, lane);
        pf.mark(DRAGG_PH_POLISH);
        if (pol) {
            for (int e = lane; e < n; e += WAVE) L.x[e] = L.t1[e];
            __syncthreads();
            *iters = it;
            return DRAGG_ST_OPTIMAL;
        }
        // residuals, infeasibility certificate and rho adaptation
        double rp = 0, rd = 0, nax = 0, nz = 0, naty = 0, nq = 0, ndy = 0, natdy = 0, supp = 0;
        for (int e = lane; e < m; e += WAVE) {
            const int k = e >> 2, r = e & 3;
            if (r >= h.nrows) { L.zeq[e] = 0.0; continue; }
            const double ax = a_times(L, L.x, k, r);
            rp = fmax(rp, fabs(ax - L.beq[e]));
            nax = fmax(nax, fabs(ax));
            nz = fmax(nz, fabs(L.beq[e]));
            const double dy = L.yeq[e] - L.yeqp[e];
            ndy = fmax(ndy, fabs(dy));
            supp += L.beq[e] * dy;
            L.zeq[e] = dy;                                  // reuse as dy_eq
        }
        __syncthreads();
        for (int e = lane; e < n; e += WAVE) {
            const int k = e >> 3, jj = e & 7;
            if (!slot_active(h, jj)) continue;
            rp = fmax(rp, fabs(L.x[e] - L.zb[e]));
            nax = fmax(nax, fabs(L.x[e]));
            nz = fmax(nz, fabs(L.zb[e]));
            const double aty = at_times(h, L, L.yeq, k, jj) + L.yb[e];
            rd = fmax(rd, fabs(L.q[e] + aty));
            naty = fmax(naty, fabs(aty));
            nq = fmax(nq, fabs(L.q[e]));
            const double dyb = L.yb[e] - L.ybp[e];
            ndy = fmax(ndy, fabs(dyb));
            supp += dyb > 0 ? L.hi[e] * dyb : L.lo[e] * dyb;
            natdy = fmax(natdy, fabs(at_times(h, L, L.zeq, k, jj) + dyb));
            L.ybp[e] = L.yb[e];
        }
        for (int e = lane; e < m; e += WAVE) L.yeqp[e] = L.yeq[e];
        rp = wave_max(rp); rd = wave_max(rd); nax = wave_max(nax); nz = wave_max(nz);
        naty = wave_max(naty); nq = wave_max(nq); ndy = wave_max(ndy); natdy = wave_max(natdy);
        supp = wave_sum(supp);
        __syncthreads();
        if (ndy > 1e-12 && natdy < EPS_PINF * ndy && supp < -EPS_PINF * ndy) {
            *iters = it;
            return DRAGG_ST_INFEASIBLE_CERT;
        }
        const double sp = rp / fmax(fmax(nax, nz), 1e-12);
        const double sd = rd / fmax(fmax(naty, nq), 1e-12);
        double nr = rho * sqrt(sp / fmax(sd, 1e-12));
        nr = fmin(fmax(nr, 1e-6), 1e6);
        pf.mark(DRAGG_PH_CHECK);
        if (nr > 5.0 * rho || nr < 0.2 * rho) {
            rho = nr;
            factor(h, L, lane, rho);
            pf.mark(DRAGG_PH_FACTOR);
        }
    }
    *iters = max_iter;
    return DRAGG_ST_MAX_ITER;
}

// --------------------------------------------------------------------------------------
// integer duty cycles (mpc_calc.py:171-173, 344-349).  The thermal MILP is two integer
// chains -- indoor T driven by the hvac duty, then tank Tw driven by the wh duty (and by
// T through a 4e-5 coupling).  Each is solved by a forward dynamic programme over the
// state discretised into bins of 1/NBU of one duty unit's effect: per bin the cheapest
// label is kept with its EXACT state value, so every kept path is exactly feasible and
// costed; a bin collision is the only approximation.  Pull formulation: each lane owns
// target bins and scans the (1-2) source bins that can reach it per duty value, so a
// stage is conflict-free and fully lane-parallel.  Back-pointers (source bin, duty)
// live in the freed KKT-factor LDS.  On the golden fixtures this reproduces the
// reference's MILP optimum (see tests/test_gpu_parity.py).
// --------------------------------------------------------------------------------------
constexpr int NBU = 8;

struct DpChain {
    int H, S, sx, sv;
    double g;
    const double* A;    // [H]
    const double* C;    // [H]
    double x0;
};

// returns false if no integer schedule keeps the chain inside its box
DEV bool dp_chain(const Home& h, const Lds& L, const DpChain& c, int lane) {
    const int H = c.H, S = c.S;
    double glo = INFINITY, ghi = -INFINITY;
    for (int k = 0; k < H; ++k) {
        glo = fmin(glo, L.lo[k * 8 + c.sx]);
        ghi = fmax(ghi, L.hi[k * 8 + c.sx]);
    }
    const int cap = min(512, 12 * H);
    double w = fabs(c.g) / NBU;
    int nb = (int)floor((ghi - glo) / w) + 1;
    if (nb > cap) { w = (ghi - glo) / (cap - 1); nb = cap; }
    double* cc = L.zb;                      // cost of the label in each bin
    double* cx = L.zb + nb;                 // its exact state
    double* nc = L.zb + 2 * nb;
    double* nx = L.zb + 3 * nb;             // zb..ybp are contiguous: 48H doubles >= 4 nb
    uint16_t* par = reinterpret_cast<uint16_t*>(L.Lf);   // [H][nb] (source bin << 4 | duty)
    const double BIG = INFINITY;
    for (int k = 0; k < H; ++k) {
        const double Ak = c.A[k], Ck = c.C[k], ck = L.q[k * 8 + c.sv];
        const double lo = L.lo[k * 8 + c.sx], hi = L.hi[k * 8 + c.sx];
        const double tlo = lo - TOL_P * (1 + fabs(lo)), thi = hi + TOL_P * (1 + fabs(hi));
        for (int B = lane; B < nb; B += WAVE) {
            double best = BIG, bx = 0.0;
            int bp = 0xFFFF;
            for (int u = 0; u <= S; ++u) {
                if (k == 0) {
                    const double xn = Ak * c.x0 + c.g * u + Ck;
                    if (xn < tlo || xn > thi) continue;
                    if ((int)floor((xn - glo) / w) != B) continue;
                    const double cn = ck * u;
                    if (cn < best) { best = cn; bx = xn; bp = u; }
                    continue;
                }
                // source states x with A x + g u + C inside bin B
                const double xa = (glo + B * w - c.g * u - Ck) / Ak;
                const double xb = (glo + (B + 1) * w - c.g * u - Ck) / Ak;
                int s0 = (int)floor((fmin(xa, xb) - glo) / w) - 1, s1 = (int)floor((fmax(xa, xb) - glo) / w) + 1;
                s0 = s0 < 0 ? 0 : s0;
                s1 = s1 >= nb ? nb - 1 : s1;
                for (int sb = s0; sb <= s1; ++sb) {
                    const double cs = cc[sb];
                    if (!(cs < BIG)) continue;
                    const double xn = Ak * cx[sb] + c.g * u + Ck;
                    if (xn < tlo || xn > thi) continue;
                    if ((int)floor((xn - glo) / w) != B) continue;
                    const double cn = cs + ck * u;
                    if (cn < best) { best = cn; bx = xn; bp = (sb << 4) | u; }
                }
            }
            nc[B] = best;
            nx[B] = bx;
            par[k * nb + B] = (uint16_t)bp;
        }
        __syncthreads();
        for (int B = lane; B < nb; B += WAVE) { cc[B] = nc[B]; cx[B] = nx[B]; }
        __syncthreads();
    }
    // cheapest final label (lowest bin on ties, deterministic)
    double best = BIG;
    int bb = -1;
    for (int B = lane; B < nb; B += WAVE)
        if (cc[B] < best) { best = cc[B]; bb = B; }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bb, o);
        if (ob < best || (ob == best && oi >= 0 && (bb < 0 || oi < bb))) { best = ob; bb = oi; }
    }
    if (bb < 0) return false;
    if (lane == 0) {
        int b = bb;
        for (int k = H - 1; k >= 0; --k) {
            const int p = par[k * nb + b];
            L.x[k * 8 + c.sv] = (double)(p & 15);
            b = p >> 4;
        }
        double x = c.x0;                    // exact forward trajectory of the chosen duties
        for (int k = 0; k < H; ++k) {
            x = c.A[k] * x + c.g * L.x[k * 8 + c.sv] + c.C[k];
            L.x[k * 8 + c.sx] = x;
        }
    }
    __syncthreads();
    return true;
}

template <int SS, int CAP = NF, int CAPB = NF_BOUND, int PS = NB_CAP, int NBK = NTB, int NW = 1, bool CELL = false,
          int ILP = 1>
DEV int dp_front(const struct FrontBufs& B, int H, int tid, double g, double x0, double lo0, double hi0, double lo,
                 double hi, int sx, int sv, bool use_bound = false, double ub_ext = INFINITY,
                 double* best_out = nullptr, int beam_k = 0);

// int_mode round_lp: the integer duties after the relaxation, by the exact front DP (the
// default path's, dp_front) with its buffers in the KKT-factor LDS the ADMM no longer needs
// and its back-pointers in the workspace; the binned dp_chain only where the front DP does not
// apply (mixed-sign prices, a too-narrow feasible set, S != 6)
DEV bool round_duties(const Home& h, const Lds& L, int lane, uint16_t* par);

// closed-form PV curtailment (mpc_calc.py:382-384): u multiplies a cost coefficient
// gamma^k price_k S A eta ghi_k / 1000, so u = 1 only where that coefficient is negative
// (u = 0 at a zero coefficient, the lower-bound vertex).
DEV double pv_curt(const Lds& L, int k) { return (L.price[k] < 0.0 && L.ghi[k] > 0.0) ? 1.0 : 0.0; }

// objective sum_k gamma^k price_k p_grid_k (mpc_calc.py:441-446) for the solution in L.x;
// also leaves p_grid_k in L.t2[k]
DEV double objective(const Home& h, const Lds& L, int lane, int nt = WAVE, double* red = nullptr) {
    double s = 0.0;
    for (int k = lane; k < h.H; k += nt) {
        const int o = k * 8;
        const double u = L.x[o + S_U], w = L.x[o + S_W];
        const double cc = h.winter ? 0.0 : u, hh = h.winter ? u : 0.0;
        double pl = (h.S * h.Pc) * cc + (h.S * h.Ph) * hh + (h.S * h.Pw) * w;
        double pg = pl;
        if (h.batt) pg += h.S * (L.x[o + S_CH] + L.x[o + S_DIS]);
        if (h.pv) pg -= h.S * (h.pvA * h.pvEta * L.ghi[k] * (1 - pv_curt(L, k)) / 1000);
        L.t2[k] = pg;
        s += pow(h.gamma, (double)k) * (L.price[k] * pg);
    }
    s = block_sum(s, red, lane, nt);
    __syncthreads();
    return s;
}

struct Io {
    double* vals;          // [NVAL][N]
    double* fc;            // [N][NFC][H] (home-contiguous)
    int N, home;
    __device__ double& v(int key) const { return vals[(size_t)key * N + home]; }
    __device__ double& f(int key, int j, int H) const { return fc[((size_t)home * DRAGG_NFC + key) * H + j]; }
};

// success branch of cleanup_and_finish (mpc_calc.py:486-526)
DEV void write_success(const Home& h, const Lds& L, const Io& io, int lane, int nt = WAVE) {
    const int H = h.H;
    const double S = h.S;
    for (int j = lane; j < H; j += nt) {
        const int o = j * 8;
        const double u = L.x[o + S_U], w = L.x[o + S_W];
        const double cc = h.winter ? 0.0 : u, hh = h.winter ? u : 0.0;
        const double pl = (h.S * h.Pc) * cc + (h.S * h.Ph) * hh + (h.S * h.Pw) * w;
        const double pg = L.t2[j];
        io.f(DRAGG_K_P_GRID, j, H) = pg / S;
        io.f(DRAGG_K_FORECAST_P_GRID, j, H) = (j + 1 < H) ? L.t2[j + 1] / S : 0.0;
        io.f(DRAGG_K_P_LOAD, j, H) = pl / S;
        io.f(DRAGG_K_TEMP_IN_EV, j, H) = L.x[o + S_T];
        io.f(DRAGG_K_TEMP_WH_EV, j, H) = L.x[o + S_TW];
        io.f(DRAGG_K_HVAC_COOL, j, H) = cc / S;
        io.f(DRAGG_K_HVAC_HEAT, j, H) = hh / S;
        io.f(DRAGG_K_WH_HEAT, j, H) = w / S;
        io.f(DRAGG_K_COST, j, H) = L.price[j] * pg;
        io.f(DRAGG_K_WATERDRAWS, j, H) = L.draw[j];
        if (h.pv) {
            const double up = pv_curt(L, j);
            io.f(DRAGG_K_P_PV, j, H) = h.pvA * h.pvEta * L.ghi[j] * (1 - up) / 1000;
            io.f(DRAGG_K_U_PV_CURT, j, H) = up;
        }
        if (h.batt) {
            io.f(DRAGG_K_P_BATT_CH, j, H) = L.x[o + S_CH];
            io.f(DRAGG_K_P_BATT_DISCH, j, H) = L.x[o + S_DIS];
            io.f(DRAGG_K_E_BATT, j, H) = L.x[o + S_E];
        }
        if (j == 0) {          // the un-suffixed fields are the j = 0 values (mpc_calc.py:516)
            for (int key = 0; key < DRAGG_NFC; ++key) {
                const bool is_pv = key == DRAGG_K_P_PV || key == DRAGG_K_U_PV_CURT;
                const bool is_b = key == DRAGG_K_P_BATT_CH || key == DRAGG_K_P_BATT_DISCH || key == DRAGG_K_E_BATT;
                if ((!is_pv || h.pv) && (!is_b || h.batt)) io.v(key) = io.f(key, 0, H);
            }
        }
    }
    if (lane == 0) {
        const double u0 = L.x[S_U], w0 = L.x[S_W];
        const double c0 = h.winter ? 0.0 : u0, h0 = h.winter ? u0 : 0.0;
        const double Ts = (h.T0 + ((L.oat[1] - h.T0) * h.iR) * 3600 * h.inv_c) -
                          (h.Pc * 3600 * h.inv_c) * c0 + (h.Ph * 3600 * h.inv_c) * h0;
        const double Tws = (h.Tw0 + ((-h.Tw0) * h.iRw) * 3600 * h.inv_w) + h.e * L.x[S_T] + h.f * w0;
        io.v(DRAGG_V_TEMP_IN_OPT) = Ts;
        io.v(DRAGG_V_TEMP_WH_OPT) = Tws;
        io.v(DRAGG_V_CORRECT_SOLVE) = 1.0;
        io.v(DRAGG_V_SOLVE_COUNTER) = 0.0;
    }
}

// failure branch (mpc_calc.py:527-595); returns dragg_status (ERR_PARSE where the
// reference would raise)
DEV int write_fallback(const Home& h, const Lds& L, const Io& io, int status) {
#pragma clang fp contract(off)   // bit-identical to the reference's float expressions
    const int H = h.H;
    const double S = h.S;
    int counter = h.counter + 1;
    const double hmax = h.winter ? S : 0.0, cmax = h.winter ? 0.0 : S;
    const double hmin = 0.0, cmin = 0.0, whmax = S, whmin = 0.0;
    const double oat1 = L.oat[1];
    double heat, cool, wh;
    double cp_fc[DRAGG_NFC];
    bool copied = false;
    if (counter < H && h.t > 0) {                               // :533-557
        for (int k = 0; k <= DRAGG_K_WATERDRAWS; ++k) cp_fc[k] = io.f(k, counter, H);
        copied = true;
        wh = leading_char_value(cp_fc[DRAGG_K_WH_HEAT]);
        cool = leading_char_value(cp_fc[DRAGG_K_HVAC_COOL]);
        heat = leading_char_value(cp_fc[DRAGG_K_HVAC_HEAT]);
        if (wh < 0 || cool < 0 || heat < 0) return DRAGG_ST_ERR_PARSE;
        const double nT = (double)(h.T0 + 3600 * ((((oat1 - h.T0) / h.R)) - cool * h.Pc + heat * h.Ph) /
                                              (h.C * h.dt));
        const double nW = (double)(h.Tw0 + 3600 * ((((nT - h.Tw0) / h.Rw)) + wh * h.Pw) / (h.Cw * h.dt));
        if (nT > h.Tmax) { heat = hmin; cool = cmax; }
        else if (nT < h.Tmin) { heat = hmax; cool = cmin; }
        if (nW < h.Twmin) wh = whmax;
    } else {                                                    // :559-574
        counter = counter < H ? H : counter;
        if (h.T0 > h.Tmax) { heat = hmin; cool = cmax; }
        else if (h.T0 < h.Tmin) { heat = hmax; cool = cmin; }
        else { heat = hmin; cool = cmin; }
        wh = (h.Tw0 < h.Twmin) ? whmax : whmin;
    }
    const double nT = h.T0 + 3600 * ((((oat1 - h.T0) / h.R)) - cool * h.Pc + heat * h.Ph) / (h.C * h.dt);
    const double nW = h.Tw0 + 3600 * (((nT - h.Tw0) / h.Rw) + (wh * h.Pw)) / (h.Cw * h.dt);
    if (copied) {
        io.v(DRAGG_K_TEMP_IN_EV) = cp_fc[DRAGG_K_TEMP_IN_EV];
        io.v(DRAGG_K_TEMP_WH_EV) = cp_fc[DRAGG_K_TEMP_WH_EV];
    }
    io.v(DRAGG_V_CORRECT_SOLVE) = 0.0;
    io.v(DRAGG_K_WH_HEAT) = wh / S;
    io.v(DRAGG_K_HVAC_HEAT) = heat / S;
    io.v(DRAGG_K_HVAC_COOL) = cool / S;
    io.v(DRAGG_V_TEMP_IN_OPT) = nT;
    io.v(DRAGG_V_TEMP_WH_OPT) = nW;
    io.v(DRAGG_V_SOLVE_COUNTER) = (double)counter;
    const double pl = wh * h.Pw + cool * h.Pc + heat * h.Ph;
    io.v(DRAGG_K_P_LOAD) = pl;
    io.v(DRAGG_K_FORECAST_P_GRID) = pl;
    io.v(DRAGG_K_WATERDRAWS) = L.draw[0];
    io.v(DRAGG_K_P_GRID) = pl;
    io.v(DRAGG_K_COST) = pl * L.price[0];
    return status;
}

struct KArgs {
    dragg_mpc_dims d;
    dragg_mpc_problem p;
    dragg_mpc_explicit ex;
    double* vals;
    double* fc;
    dragg_mpc_out out;
    const double* noise;
    int t;
    int force_steps;       // diagnostic (DRAGG_FORCE_STEP_DP=1): every home to the exact step DP
    // lag mode (dragg_mpc_step_main / _side): homes whose previous step is still being solved on the
    // side stream are skipped by the main pass and solved by the side pass after it
    char* lws;             // the lists and per-block scratch regions (NULL: problem.workspace's)
    int* clk;              // [N] timesteps completed per home (LAG_SIDE set: completed by the side pass)
    int* skip;             // step_main: homes whose clock is behind, for the side pass (list)
    int* hot_list;         // step_side: the hot launch takes its homes off this list
    int* nar;              // the step-function DP's list (NULL: the workspace's)
    int side;              // 1 in the side pass: its completions publish with a release
    int step_pool_cap;     // the step-function DP's pool per chain (POOL_CAP; a diagnostic knob shrinks it)
    long long step_work_cap;   // ... its work bound per pass (0: STEP_WORK_CAP)
    int narrow_lds;        // the step-function launch's LDS bytes per block (0: all a CU has, narrow_layout)
};

// a clock value the side pass wrote: the reader must acquire before it reads the home's rows
constexpr int LAG_SIDE = 1 << 30;

// lag mode: the home's step is complete (every thread of the block calls it, after every write of the
// home): its clock moves to t + 1.  The main pass's next step reads it in stream order; a side-pass
// completion is read by a CONCURRENT main-pass kernel, so its writes are released first (agent scope:
// the other XCDs' L2s) and the clock carries LAG_SIDE so that the reader acquires
DEV void lag_finish(const KArgs& a, int home) {
    if (!a.clk) return;
    if (a.side) __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(a.clk + home, (a.t + 1) | (a.side ? LAG_SIDE : 0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// --------------------------------------------------------------------------------------
// kernel prologue shared by both solve paths: per-home constants, the step's inputs
// (get_initial_conditions, water_draws, set_environmental_variables, the season draw).
// Returns DRAGG_ST_ERR_MISSING where the reference raises KeyError, else -1.
// --------------------------------------------------------------------------------------
template <bool EXPLICIT>
DEV int prologue(const KArgs& a, Home& h, const Lds& L, const Io& io, int lane, int nt, double* red) {
    const int home = io.home;
    const int N = a.d.n_homes;
    h.H = a.d.horizon; h.S = a.d.sub_steps; h.dt = a.d.dt; h.gamma = a.d.discount;
    h.type = a.p.home_type[home];
    h.pv = (h.type & 1) != 0;
    h.batt = (h.type & 2) != 0;
    h.nrows = h.batt ? 3 : 2;
    load_params(h, a.p.params, N, home);
    const int H = h.H;
    int status_pre = -1;
    if (EXPLICIT) {
        h.t = a.ex.t[home];
        h.T0 = a.ex.T0[home]; h.Tw0 = a.ex.Tw0[home]; h.E0 = h.batt ? a.ex.E0[home] : 0.0;
        h.counter = a.ex.counter[home];
        h.winter = a.ex.winter[home] != 0;
        for (int i = lane; i <= H; i += nt) {
            L.draw[i] = a.ex.draw[(size_t)i * N + home];
            L.oat[i] = a.ex.oat[(size_t)i * N + home];
            L.ghi[i] = a.ex.ghi[(size_t)i * N + home];
            L.price[i] = (i < H) ? a.ex.price[(size_t)i * N + home] : 0.0;
        }
        __syncthreads();
    } else {
#pragma clang fp contract(off)   // draw sizes, Tw0 mixing and the season test as in numpy
        const int t = a.t;
        h.t = t;
        const int dt = h.dt;
        const int lag = H / dt + 1;                           // mpc_calc.py:194
        const int nraw = lag * dt;
        const int base_hour = t / dt;
        const int s0 = a.p.start_index + t;
        auto rawv = [&](int idx) -> double {                  // np.repeat(list, dt) / dt
            const int hh = base_hour + idx / dt - lag;
            const double v = (hh >= 0 && hh < a.d.n_draw_hours) ? a.p.draw_hourly[(size_t)hh * N + home] : 0.0;
            return v / dt;
        };
        for (int i = lane; i <= H; i += nt) {
            double d;
            if (i < dt) d = rawv(i);
            else if (i + 1 < nraw) d = ((rawv(i - 1) + rawv(i)) + rawv(i + 1)) / 3.0;
            else d = (rawv(i - 1) + rawv(i)) / 2.0;
            L.draw[i] = d;
            L.oat[i] = a.p.oat[s0 + i];
            L.ghi[i] = a.p.ghi[s0 + i];
            const double rp = a.p.reward_price[a.d.n_rp == 1 ? 0 : (i < a.d.n_rp ? i : a.d.n_rp - 1)];
            L.price[i] = (i < H) ? rp + a.p.tou[s0 + i] : 0.0;
        }
        // season draw (mpc_calc.py:220-223, 303-309)
        double mx = -INFINITY;
        for (int k = lane; k < H; k += nt) {
            double z;
            if (a.noise) z = a.noise[(size_t)k * N + home];
            else {
                double z0, z1;
                normal_pair(a.p.seed, a.p.home_offset + home * max(a.p.home_stride, 1), t, k >> 1, &z0, &z1);
                z = (k & 1) ? z1 : z0;
            }
            mx = fmax(mx, a.p.oat[s0 + k + 1] + pow(1.1, (double)k) * z);
        }
        mx = block_max(mx, red, lane, nt);
        mx = fmax(mx, a.p.oat[s0]);
        h.winter = mx <= 30.0;
        __syncthreads();
        const double d0 = L.draw[0];
        if (t == 0) {
            h.T0 = h.Tinit;
            h.Tw0 = (h.Twinit * (h.V - d0) + TAP * d0) / h.V;
            h.E0 = h.batt ? h.Einit : 0.0;
            h.counter = 0;
        } else {
            const double Tp = io.v(DRAGG_V_TEMP_IN_OPT), Wp = io.v(DRAGG_V_TEMP_WH_OPT);
            const double cnt = io.v(DRAGG_V_SOLVE_COUNTER);
            h.T0 = Tp;
            h.Tw0 = (Wp * (h.V - d0) + TAP * d0) / h.V;
            h.counter = (int)cnt;
            h.E0 = h.batt ? io.v(DRAGG_K_E_BATT) : 0.0;
            bool missing = !(Tp == Tp) || !(Wp == Wp) || !(cnt == cnt);
            if (h.batt)
                missing = missing || !(h.E0 == h.E0) || !(io.v(DRAGG_K_P_BATT_CH) == io.v(DRAGG_K_P_BATT_CH)) ||
                          !(io.v(DRAGG_K_P_BATT_DISCH) == io.v(DRAGG_K_P_BATT_DISCH));
            if (missing) status_pre = DRAGG_ST_ERR_MISSING;
        }
    }
    return status_pre;
}


// reload the per-home scalars after a DP so that they need not stay live in registers through it
DEV void reload_home(Home& h, const KArgs& a, int home, const double* sv) {
    const int N = a.d.n_homes;
    h.H = a.d.horizon; h.S = a.d.sub_steps; h.dt = a.d.dt; h.gamma = a.d.discount;
    h.type = a.p.home_type[home];
    h.pv = (h.type & 1) != 0;
    h.batt = (h.type & 2) != 0;
    h.nrows = h.batt ? 3 : 2;
    load_params(h, a.p.params, N, home);
    h.t = (int)sv[0]; h.counter = (int)sv[1]; h.winter = sv[2] != 0.0;
    h.T0 = sv[3]; h.Tw0 = sv[4]; h.E0 = sv[5];
    derive(h);
}

DEV void write_missing(const KArgs& a, int home) {
    a.out.status[home] = DRAGG_ST_ERR_MISSING;
    a.out.iters[home] = 0;
    a.out.obj[home] = NAN;
    a.out.relax_obj[home] = NAN;
    if (a.out.int_path) a.out.int_path[home] = 0;
}

// --------------------------------------------------------------------------------------
// LP kernel (int_mode relax / round_lp): one workgroup (one wave) per home, ADMM + polish
// --------------------------------------------------------------------------------------
template <bool EXPLICIT>
__global__ __launch_bounds__(64) void mpc_home_kernel(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int home = blockIdx.x;
    const int lane = threadIdx.x;
    const int N = a.d.n_homes;
    if (home >= N) return;
    Home h;
    const int H = a.d.horizon;
    Lds L = carve(smem, H);
    Io io{a.vals, a.fc, N, home};
    Prof pf;
    pf.start(a.out.cycles != nullptr);
    if (prologue<EXPLICIT>(a, h, L, io, lane, WAVE, nullptr) == DRAGG_ST_ERR_MISSING) {
        if (lane == 0) write_missing(a, home);
        return;
    }
    derive(h);
    build(h, L, lane);

    // ---------------- solve (solve_mpc)
    int iters = 0;
    int status;
    if (presolve_infeasible(h, L)) status = DRAGG_ST_INFEASIBLE;
    else {
        const int mi = a.d.max_iter > 0 ? a.d.max_iter : 4000;
        const int ce = a.d.check_every > 0 ? a.d.check_every : 10;
        pf.mark(DRAGG_PH_SETUP);
        status = admm(h, L, lane, mi, ce, &iters, pf);
    }
    pf.mark(DRAGG_PH_SETUP);
    double relax = NAN, obj = NAN;
    if (status == DRAGG_ST_OPTIMAL) {
        relax = objective(h, L, lane);
        pf.mark(DRAGG_PH_WRITE);
        if (a.d.int_mode == DRAGG_INT_ROUND_LP &&
            !round_duties(h, L, lane, a.p.workspace ? reinterpret_cast<uint16_t*>(a.p.workspace) +
                                                          (size_t)home * H * NB_CAP : nullptr))
            status = DRAGG_ST_ROUND_FAIL;
        pf.mark(DRAGG_PH_INTEGER);
        if (status == DRAGG_ST_OPTIMAL) obj = objective(h, L, lane);
    }

    // ---------------- cleanup_and_finish + redis_write_optimal_vals
    if (status == DRAGG_ST_OPTIMAL) {
        write_success(h, L, io, lane);
    } else if (lane == 0) {
        status = write_fallback(h, L, io, status);
    }
    status = __shfl(status, 0);
    if (lane == 0) {
        a.out.status[home] = status;
        a.out.iters[home] = iters;
        a.out.obj[home] = obj;
        a.out.relax_obj[home] = relax;
    }
    if (a.out.hist && lane == 0)      // lane 0 wrote every vals field of this home
        for (int k = 0; k < DRAGG_NVAL; ++k) a.out.hist[(size_t)k * N + home] = io.v(k);
    pf.mark(DRAGG_PH_WRITE);
    if (pf.on && lane == 0)
        for (int k = 0; k < DRAGG_NPHASE; ++k) a.out.cycles[(size_t)k * N + home] = (int64_t)pf.acc[k];
}

// ======================================================================================
// Direct integer path (int_mode = DRAGG_INT_ROUND, the default).
//
// The reference MILP (mpc_calc.py:291-446) is separable: its objective is
// sum_k gamma^k price_k p_grid_k with p_grid = p_load [+ S(ch + dis)] [- S p_pv], and no
// constraint couples the thermal variables (T, Tw, hvac/wh duties), the battery
// (E, ch, dis) and the PV curtailment.  So the MILP optimum is
//   thermal integer programme (two integer chains)      -> binned forward DP  (dp_thermal)
// + battery LP (one continuous storage chain)            -> exact convex piecewise-linear
//                                                           value-function DP (battery_lp)
// + PV LP (separable per stage)                          -> closed form        (pv_curt)
// No relaxation / ADMM is needed on this path; the LP kernel above remains the solver of
// the relaxation (int_mode relax) and of the relaxation-then-round variant (round_lp).
// ======================================================================================

struct LdsD {
    double *draw, *oat, *ghi, *price;   // [H+1]
    double *x;                          // [8H] solution in the stage-slot layout of the LP path
    double *t2;                         // [H] p_grid (objective)
    double *cA, *cC, *cq;               // [H] coefficients of the chain being solved
    double *sc;                         // [32] scalars / reduction scratch
    double *bx0, *bp1, *bp2;            // [H] battery: merged-domain origin, psi segment offsets
    double2 *lab;                       // [NB_CAP] DP labels (dp_front: front A (key, cost);
                                        //   dp_zspace / dp_fixed: (cost, exact state))
    double2 *rmin;                      // [NB_CAP+8] dp_front: front B; dp_zspace: cheapest
                                        //   source label per key; dp_fixed: second label buffer
    // --- tail, a union: dp_front's arrays or dp_zspace's (never live together)
    unsigned long long *kb, *cb;        // [NTB]  dp_front: per key / cost bucket packed extremes
    unsigned *mh, *kl;                  // [NTB]  dp_front: scans of kb / cb
    unsigned *flo, *fhi;                // [H+1]  dp_front: feasible-set hull of x_k (fixed point)
    double2 *cand;                      // [NBND][S+1] boundary-bucket candidates per duty
    double *rt;                         // [H+2] zero-duty reference trajectory of the chain
    int *candp;                         // [NBND][S+1] candidate records
    int16_t *tarr, *rsrc;               // [NB_CAP], [NB_CAP+8] source keys, source of rmin
    double *sgS, *sgL;                  // battery segments [2][seg_cap], in lab / rmin (the
                                        //   battery LP runs after the thermal DPs)
    double* wl;                         // [3][WAVE] dp_front's W table (points, values, slopes)
    char* xch;                          // [xch_bytes(cap)] a multi-wave DP's exchange area
    uint16_t* par;                      // [H][NB_CAP] DP back-pointers (global workspace)
};

__host__ __device__ inline int seg_cap(int H) { return ((2 * H + 2 + 63) / 64) * 64; }

// The battery LP runs after the thermal DPs: its segment lists live in lab (sgS) and rmin
// (sgL); for H up to ~60 its recovery arrays (bx0, bp1, bp2) also fit in lab and the
// objective's p_grid (t2) in rmin ("compact" layout), else they get arrays of their own.
__host__ __device__ inline bool direct_compact(int H) {
    return 2 * seg_cap(H) + 3 * H <= 2 * NB_CAP && 2 * seg_cap(H) + H <= 2 * (NB_CAP + 8);
}
__host__ __device__ inline bool direct_fits(int H) { return seg_cap(H) <= NB_CAP; }

// Byte offsets of the direct kernel's LDS carve (one function for the device carve and the
// host's launch size, so the two cannot disagree).
// direct kernel workspace: [N][H][NB_CAP] u16 DP back-pointers, then [N][8H] f64 solutions
__host__ __device__ inline size_t par_region_bytes(int N, int H) {
    return ((size_t)N * H * NB_CAP * sizeof(uint16_t) + 255) / 256 * 256;
}
// then [N][8H] f64 solutions, the list of homes the hot launch defers to the second one
// ([N] i32 + its length) and (256-aligned) the second launch's back-pointer rows
// [SECOND_SLOTS][H][NF_BIG] u16, one block of that persistent launch per slot.  From the deferred
// list to the end of the mid launch's rows (below) the workspace holds only lists and per-block
// scratch: that span is all the lag mode's side workspace needs (side_workspace_bytes); the per-home
// regions (back-pointers, solutions, LP rows, cell rows) come before or after it.
__host__ __device__ inline size_t defer_offset(int N, int H) { return par_region_bytes(N, H) + (size_t)N * 8 * H * 8; }
__host__ __device__ inline size_t big_region_offset(int N, int H) {
    return (defer_offset(N, H) + (size_t)(N + 2) * sizeof(int) + 255) / 256 * 256;
}
__host__ __device__ inline size_t big_region_bytes(int H) { return (size_t)SECOND_SLOTS * H * NF_BIG * sizeof(uint16_t); }
// then the list of homes the second launch hands to DM_NARROW ([N] i32 + its length) and
// (256-aligned) DM_NARROW's step-function storage, one region per block of that launch
__host__ __device__ inline size_t step_slot_bytes() {
    // the V_k pool (breakpoints, values) [POOL_CAP] f64 each and a stage's point ids [MC_CAP] i32 x 2
    // (merge ping-pong; the free one then holds the values' codes) past the LDS capacity (dp_steps)
    return (size_t)2 * POOL_CAP * sizeof(double) + (size_t)2 * MC_CAP * sizeof(int) +
           (size_t)2 * LW_ROWS * 64 * 2 * sizeof(double);
}
__host__ __device__ inline int narrow_slots(int N) { return N < NARROW_SLOTS ? N : NARROW_SLOTS; }
__host__ __device__ inline size_t narrow_list_offset(int N, int H) {
    return (big_region_offset(N, H) + big_region_bytes(H) + 255) / 256 * 256;
}
__host__ __device__ inline size_t narrow_region_offset(int N, int H) {
    return (narrow_list_offset(N, H) + (size_t)(N + 2) * sizeof(int) + 255) / 256 * 256;
}
// then the list of homes the mid launch hands to the big one ([N] i32 + length) and (256-aligned)
// the mid launch's back-pointer rows [MID_SLOTS_MAX][H][NF_MID] u16
__host__ __device__ inline size_t mid_list_offset(int N, int H) {
    return (narrow_region_offset(N, H) + (size_t)narrow_slots(N) * step_slot_bytes() + 255) / 256 * 256;
}
__host__ __device__ inline size_t mid_region_offset(int N, int H) {
    return (mid_list_offset(N, H) + (size_t)(N + 2) * sizeof(int) + 255) / 256 * 256;
}
// then (256-aligned) the front DP's LP cost-to-go rows [N][H + 1][64] (x, v), per home
__host__ __device__ inline size_t w_region_offset(int N, int H) {
    return (mid_region_offset(N, H) + (size_t)MID_SLOTS_MAX * H * NF_MID * sizeof(uint16_t) + 255) / 256 * 256;
}
__host__ __device__ inline size_t w_region_bytes(int N, int H) { return (size_t)N * (H + 1) * 64 * 16; }
// the lag mode's side workspace: the lists and per-block scratch [defer_offset, w_region_offset)
__host__ __device__ inline size_t side_workspace_bytes(int N, int H) { return w_region_offset(N, H) - defer_offset(N, H); }
// then (256-aligned), with a reward-price list (dims.n_rp > 1: RL prices possible), the cell bound's
// rows of every home's indoor-air chain [N][H + 1][CELL_STRIDE] u16 codes (cell_kernel; row 0: the header --
// valid flag, offset, scale as three f32)
__host__ __device__ inline size_t cell_region_offset(int N, int H) {
    return (w_region_offset(N, H) + w_region_bytes(N, H) + 255) / 256 * 256;
}
__host__ __device__ inline size_t cell_region_bytes(int N, int H, bool cells) {
    return cells ? (size_t)N * (H + 1) * CELL_STRIDE * sizeof(uint16_t) : 0;
}
__host__ __device__ inline size_t direct_workspace_bytes(int N, int H, bool cells) {
    return cell_region_offset(N, H) + cell_region_bytes(N, H, cells);
}

struct DirectLayout {
    int draw, oat, ghi, price, cA, cC, cq, sc, t2, bx0, bp1, bp2, lab, rmin, tail;
    int kb, cb, mh, kl, flo, fhi;             // dp_front tail
    int cand, rt, candp, tarr, rsrc;          // dp_zspace tail
    int wl, sgS, sgL, xch;                    // front_layout only: W table, battery segment lists, exchange
    int bytes;
};

// The hot launch (DM_FRONT) runs only the front DP: fronts of NF_HOT labels, the W table, the
// bucket arrays and hulls; the battery LP (after both chains) reuses that region.  Occupancy is
// what this buys (8 -> 11 homes per CU at H = 48: 2.44 -> 2.13 ms per bench step; measured the
// other way: 7 homes per CU cost +11 % time, 6 +43 %).
__host__ __device__ inline DirectLayout front_layout(int H) {
    DirectLayout o{};
    int p = 0;
    auto take = [&](int bytes, int align) { p = (p + align - 1) / align * align; const int r = p; p += bytes; return r; };
    o.draw = take(8 * (H + 1), 16);
    o.oat = take(8 * (H + 1), 8);
    o.ghi = take(8 * (H + 1), 8);
    o.price = take(8 * (H + 1), 8);
    o.cA = take(8 * H, 8);
    o.cC = take(8 * H, 8);
    o.cq = take(8 * H, 8);
    o.sc = take(8 * 32, 8);
    o.tail = p;
    o.lab = take(16 * NF_HOT, 16);
    o.rmin = take(16 * NF_HOT, 16);
    o.wl = take(8 * 3 * WAVE, 16);
    o.kb = take(16 * NTB_HOT, 16);                  // per bucket {key ref u64, mh u32, pad}: one 16-B load
    o.cb = take(16 * NTB_HOT, 16);                  // per bucket {cost ref u64, kl u32, pad}
    o.mh = o.kb + 8;
    o.kl = o.cb + 8;
    o.flo = take(4 * (H + 1), 4);
    o.fhi = take(4 * (H + 1), 4);
    o.xch = take(xch_bytes(NF_HOT), 16);
    const int dp_end = p;
    p = o.tail;                                  // the battery LP's arrays over the dead DP region
    o.sgS = take(16 * seg_cap(H), 16);
    o.sgL = take(16 * seg_cap(H), 16);
    o.bx0 = take(8 * H, 8);
    o.bp1 = take(8 * H, 8);
    o.bp2 = take(8 * H, 8);
    o.t2 = take(8 * H, 8);
    o.cand = o.rt = o.candp = o.tarr = o.rsrc = -1;
    o.bytes = (max(dp_end, p) + 15) / 16 * 16;
    return o;
}

__host__ __device__ inline DirectLayout direct_layout(int H, int S) {
    DirectLayout o{};
    int p = 0;
    auto take = [&](int bytes, int align) { p = (p + align - 1) / align * align; const int r = p; p += bytes; return r; };
    o.draw = take(8 * (H + 1), 16);
    o.oat = take(8 * (H + 1), 8);
    o.ghi = take(8 * (H + 1), 8);
    o.price = take(8 * (H + 1), 8);
    o.cA = take(8 * H, 8);
    o.cC = take(8 * H, 8);
    o.cq = take(8 * H, 8);
    o.sc = take(8 * 32, 8);
    o.t2 = o.bx0 = o.bp1 = o.bp2 = -1;
    if (!direct_compact(H)) {
        o.t2 = take(8 * H, 8);
        o.bx0 = take(8 * H, 8);
        o.bp1 = take(8 * H, 8);
        o.bp2 = take(8 * H, 8);
    }
    o.lab = take(16 * NB_CAP, 16);
    o.rmin = take(16 * (NB_CAP + 8), 16);
    o.tail = p;
    // dp_front tail
    o.kb = take(16 * NTB, 16);                  // per bucket {key ref u64, mh u32, pad}: one 16-B load
    o.cb = take(16 * NTB, 16);                  // per bucket {cost ref u64, kl u32, pad}
    o.mh = o.kb + 8;
    o.kl = o.cb + 8;
    o.flo = take(4 * (H + 1), 4);
    o.fhi = take(4 * (H + 1), 4);
    const int end_front = p;
    // dp_zspace tail (same origin)
    p = o.tail;
    o.cand = take(16 * NBND * (S + 1), 16);
    o.rt = take(8 * (H + 2), 8);
    o.candp = take(4 * NBND * (S + 1), 4);
    o.tarr = take(2 * NB_CAP, 2);
    o.rsrc = take(2 * (NB_CAP + 8), 2);
    o.bytes = (max(end_front, p) + 15) / 16 * 16;
    return o;
}

__host__ __device__ inline int direct_lds_bytes(int H, int S) { return direct_layout(H, S).bytes; }

// DM_NARROW: the direct layout, then the step DP's LDS (StepBufs): offsets / counts / W-row points
// [H + 1] i32, scan scratch, list ranges, the reachable hull and the cut domains [H + 1] f64, the
// recovery's duty values, L_k's table, then a pool with the rest of the CU's LDS: per stage V_{k+1}
// (B, V) and the merge buffers (keys f64 x 2, ids i32 x 2) where they fit
struct NarrowLayout { int off, cnt, wc, lc, red, xr, rng, rl, rh, dlo, dhi, xv, lt, sp, spb, bytes; };
__host__ __device__ inline NarrowLayout narrow_layout(int H, int S, int lds_cap = 0) {
    NarrowLayout o{};
    int p = direct_layout(H, S).bytes;
    auto take = [&](int bytes, int align) { p = (p + align - 1) / align * align; const int r = p; p += bytes; return r; };
    o.off = take(4 * (H + 1), 4);
    o.cnt = take(4 * (H + 1), 4);
    o.wc = take(4 * (H + 1), 4);
    o.lc = take(4 * (H + 1), 4);
    o.red = take(4 * 32, 4);
    o.xr = take(4 * (NT_STEPS / 64) * STEP_MAXU, 4);
    o.rng = take(4 * (4 * STEP_MAXU + 8), 4);
    o.rl = take(8 * (H + 1), 8);
    o.rh = take(8 * (H + 1), 8);
    o.dlo = take(8 * (H + 1), 8);
    o.dhi = take(8 * (H + 1), 8);
    o.xv = take(8 * STEP_MAXU, 8);
    o.lt = take(8 * (3 * WAVE + 2), 16);
    // the pool takes what is left of the CU's LDS (>= the waves' PL tables of lp_cut)
    o.sp = take(0, 16);
    // (lds_cap > 0, DRAGG_NARROW_LDS_KB: a smaller block that shares a CU with hot-launch blocks -- it need
    // not wait for a CU to drain completely -- at the price of stages that spill to the workspace sooner)
    const int cap_ = lds_cap > 0 ? min(lds_cap, 160 * 1024 - 256) : 160 * 1024 - 256;
    o.spb = max(NT_STEPS / 64 * 6 * WAVE * 8, (cap_ - o.sp - 64) / 64 * 64);
    p = o.sp + o.spb;
    o.bytes = (p + 15) / 16 * 16;
    return o;
}

// The second launch: the direct layout, and over its DP arrays (from lab on; the bucketed DP
// is done with them, its schedule is in the global solution array) the big exact pass's
// fronts [NF_BIG], W table, bucket arrays and hull.
struct BigLayout {
    int fa, fb, wl, kb, cb, mh, kl, flo, fhi, xch, bytes;
};
__host__ __device__ inline BigLayout big_layout(int H, int S) {
    const DirectLayout d = direct_layout(H, S);
    BigLayout o{};
    int p = d.lab;
    auto take = [&](int bytes, int align) { p = (p + align - 1) / align * align; const int r = p; p += bytes; return r; };
    o.fa = take(16 * NF_BIG, 16);
    o.fb = take(16 * NF_BIG, 16);
    o.wl = take(8 * 3 * WAVE, 16);
    o.kb = take(16 * NTB_BIG, 16);                  // per bucket {key ref u64, mh u32, pad}: one 16-B load
    o.cb = take(16 * NTB_BIG, 16);                  // per bucket {cost ref u64, kl u32, pad}
    o.mh = o.kb + 8;
    o.kl = o.cb + 8;
    o.flo = take(4 * (H + 1), 4);
    o.fhi = take(4 * (H + 1), 4);
    p = max(p, d.bytes);                         // past the direct layout too: the regular front DP of
    o.xch = take(max(xch_bytes(NF_BIG), xch_bytes(NF)), 16);   // the (multi-wave) launch uses it as well
    o.bytes = (p + 15) / 16 * 16;
    return o;
}

// The mid launch: the direct layout, and over its DP arrays the exact pass's fronts [NF_MID],
// W table, bucket arrays and hull: ~20 KB at H = 48, ~7 blocks per CU (the big layout: 2)
__host__ __device__ inline BigLayout mid_layout(int H, int S) {
    const DirectLayout d = direct_layout(H, S);
    BigLayout o{};
    int p = d.lab;
    auto take = [&](int bytes, int align) { p = (p + align - 1) / align * align; const int r = p; p += bytes; return r; };
    o.fa = take(16 * NF_MID, 16);
    o.fb = take(16 * NF_MID, 16);
    o.wl = take(8 * 3 * WAVE, 16);
    o.kb = take(16 * NTB_MID, 16);                  // per bucket {key ref u64, mh u32, pad}: one 16-B load
    o.cb = take(16 * NTB_MID, 16);                  // per bucket {cost ref u64, kl u32, pad}
    o.mh = o.kb + 8;
    o.kl = o.cb + 8;
    o.flo = take(4 * (H + 1), 4);
    o.fhi = take(4 * (H + 1), 4);
    p = max(p, d.bytes);
    o.xch = take(max(xch_bytes(NF_MID), xch_bytes(NF)), 16);
    // (the RL path's cell rows are read from the workspace, not staged in LDS: 4 KB per block more cost a
    // block per CU -- measured RL action 18.0 ms against 20.1 ms with the row in LDS)
    o.bytes = (p + 15) / 16 * 16;
    return o;
}

DEV LdsD carve_front(double* smem, int H) {
    const DirectLayout o = front_layout(H);
    char* b = reinterpret_cast<char*>(smem);
    auto D = [&](int off) { return reinterpret_cast<double*>(b + off); };
    LdsD L{};
    L.draw = D(o.draw); L.oat = D(o.oat); L.ghi = D(o.ghi); L.price = D(o.price);
    L.x = nullptr;                                               // global workspace (kernel)
    L.cA = D(o.cA); L.cC = D(o.cC); L.cq = D(o.cq);
    L.sc = D(o.sc);
    L.lab = reinterpret_cast<double2*>(b + o.lab);
    L.rmin = reinterpret_cast<double2*>(b + o.rmin);
    L.wl = D(o.wl);
    L.kb = reinterpret_cast<unsigned long long*>(b + o.kb);
    L.cb = reinterpret_cast<unsigned long long*>(b + o.cb);
    L.mh = reinterpret_cast<unsigned*>(b + o.mh);
    L.kl = reinterpret_cast<unsigned*>(b + o.kl);
    L.flo = reinterpret_cast<unsigned*>(b + o.flo);
    L.fhi = reinterpret_cast<unsigned*>(b + o.fhi);
    L.sgS = D(o.sgS); L.sgL = D(o.sgL);
    L.bx0 = D(o.bx0); L.bp1 = D(o.bp1); L.bp2 = D(o.bp2); L.t2 = D(o.t2);
    L.xch = b + o.xch;
    L.par = nullptr;                                             // set by the kernel
    return L;
}

DEV LdsD carve_direct(double* smem, int H, int S) {
    const DirectLayout o = direct_layout(H, S);
    char* b = reinterpret_cast<char*>(smem);
    auto D = [&](int off) { return reinterpret_cast<double*>(b + off); };
    LdsD L;
    L.draw = D(o.draw); L.oat = D(o.oat); L.ghi = D(o.ghi); L.price = D(o.price);
    L.x = nullptr;                                               // global workspace (kernel)
    L.cA = D(o.cA); L.cC = D(o.cC); L.cq = D(o.cq);
    L.sc = D(o.sc);
    L.lab = reinterpret_cast<double2*>(b + o.lab);
    L.rmin = reinterpret_cast<double2*>(b + o.rmin);
    L.kb = reinterpret_cast<unsigned long long*>(b + o.kb);
    L.cb = reinterpret_cast<unsigned long long*>(b + o.cb);
    L.mh = reinterpret_cast<unsigned*>(b + o.mh);
    L.kl = reinterpret_cast<unsigned*>(b + o.kl);
    L.flo = reinterpret_cast<unsigned*>(b + o.flo);
    L.fhi = reinterpret_cast<unsigned*>(b + o.fhi);
    L.cand = reinterpret_cast<double2*>(b + o.cand);
    L.rt = D(o.rt);
    L.candp = reinterpret_cast<int*>(b + o.candp);
    L.tarr = reinterpret_cast<int16_t*>(b + o.tarr);
    L.rsrc = reinterpret_cast<int16_t*>(b + o.rsrc);
    L.wl = reinterpret_cast<double*>(L.rmin + NF_BOUND);        // past the bounded front
    const int sc = seg_cap(H);
    L.sgS = reinterpret_cast<double*>(L.lab);
    L.sgL = reinterpret_cast<double*>(L.rmin);
    if (direct_compact(H)) {
        L.bx0 = L.sgS + 2 * sc;
        L.bp1 = L.bx0 + H;
        L.bp2 = L.bp1 + H;
        L.t2 = L.sgL + 2 * sc;
    } else {
        L.t2 = D(o.t2); L.bx0 = D(o.bx0); L.bp1 = D(o.bp1); L.bp2 = D(o.bp2);
    }
    L.par = nullptr;                                             // set by the kernel
    return L;
}

// the LP path's view (x, t2, environment) for objective / write_success / write_fallback
DEV Lds lp_view(const LdsD& D) {
    Lds L{};
    L.x = D.x; L.t2 = D.t2;
    L.draw = D.draw; L.oat = D.oat; L.ghi = D.ghi; L.price = D.price;
    L.sc = D.sc;
    return L;
}

// Exact interval feasibility of the T and E chains and the outer test of the Tw chain:
// presolve_infeasible of the LP path, on the direct path's inputs.
DEV bool presolve_direct(const Home& h, const LdsD& L, double twlo0, double twhi0, int lane) {
    if (!(h.Twmin <= h.Tw0 && h.Tw0 <= h.Twmax)) return true;          // temp_wh_ev[0] bounds
    double Tlo = h.T0, Thi = h.T0, Wlo = h.Tw0, Whi = h.Tw0, Elo = h.E0, Ehi = h.E0;
    const double gS = h.g * h.S;
    // stage k's coefficients, one stage per lane (a division each, off the serial chain); the
    // interval recursion then reads them with v_readlane (same expressions as the serial form)
    const bool lanes = h.H <= WAVE;
    double bq = 0.0, cq = 0.0, dq = 0.0;
    const int wl = lane & (WAVE - 1);                 // every wave of the workgroup keeps a copy
    if (lanes && wl < h.H) {
        bq = L.oat[wl + 1] * h.iR * 3600 * h.inv_c;
        const double df = L.draw[wl + 1] / h.V, rem = 1 - df, d15 = df * TAP;
        cq = rem + (-rem * h.iRw) * 3600 * h.inv_w;
        dq = d15 + ((-d15) * h.iRw) * 3600 * h.inv_w;
    }
    const double edis = h.brate * (1.0 / h.etad) / h.dt, echg = h.brate * h.etac / h.dt;
    bool bad = false;
    for (int k = 0; k < h.H; ++k) {
        double bk, ck, dk;
        if (lanes) {
            bk = read_lane(bq, k); ck = read_lane(cq, k); dk = read_lane(dq, k);
        } else {
            bk = L.oat[k + 1] * h.iR * 3600 * h.inv_c;
            const double df = L.draw[k + 1] / h.V, rem = 1 - df, d15 = df * TAP;
            ck = rem + (-rem * h.iRw) * 3600 * h.inv_w;
            dk = d15 + ((-d15) * h.iRw) * 3600 * h.inv_w;
        }
        // no early exit: the flags are or-ed (the result is the same, and the recursion has no
        // branch waiting on each comparison)
        double lo = h.aT * Tlo + bk + fmin(0.0, gS), hi = h.aT * Thi + bk + fmax(0.0, gS);
        Tlo = fmax(lo, h.Tmin); Thi = fmin(hi, h.Tmax);
        bad |= Tlo > Thi + TOL_P * (1 + fabs(Thi));
        const double wlo = k == 0 ? twlo0 : h.Twmin, whi = k == 0 ? twhi0 : h.Twmax;
        const double w0 = k == 0 ? h.Tw0 : 0.0;
        lo = (k == 0 ? ck * w0 : ck * Wlo) + dk + h.e * Tlo;
        hi = (k == 0 ? ck * w0 : ck * Whi) + dk + h.e * Thi + h.f * h.S;
        Wlo = fmax(lo, wlo); Whi = fmin(hi, whi);
        bad |= Wlo > Whi + TOL_P * (1 + fabs(Whi));
        if (h.batt) {
            lo = Elo - edis; hi = Ehi + echg;
            Elo = fmax(lo, h.Emin); Ehi = fmin(hi, h.Emax);
            bad |= Elo > Ehi + TOL_P * (1 + fabs(Ehi));
        }
    }
    return bad;
}

// --------------------------------------------------------------------------------------
// Thermal integer chain  x_{k+1} = A_k x_k + g u_k + C_k,  u_k in {0..S},  x_{k+1} in box_k,
// minimise sum_k cq_k u_k.  Forward DP over the state discretised into nb bins of width w
// (1/NBU of one duty unit's effect, or wider if the box needs more than NB_CAP bins); each
// bin keeps its cheapest label with its EXACT state, so every kept path is exactly
// feasible and costed (a bin collision is the only approximation).  Pull form: the thread
// owning target bin B scans, per duty u, the source bins whose states can land in B (the
// map is monotone, A_k > 0: ceil(1/A_k) + 2 candidates, 3 while A_k > 1/2), so a stage is
// conflict-free; labels are double-buffered, one barrier per stage.  Back-pointer byte =
// u | (source - first candidate) << 4, decoded by recomputing the first candidate.
// --------------------------------------------------------------------------------------
struct DpGeom {
    double glo, w, iw;
    int nb;
};

DEV DpGeom dp_geom(double glo, double ghi, double g) {
    DpGeom G;
    G.glo = glo;
    G.w = fabs(g) / NBU;
    G.nb = (int)floor((ghi - glo) / G.w) + 1;
    if (G.nb > NB_CAP) { G.w = (ghi - glo) / (NB_CAP - 1); G.nb = NB_CAP; }
    G.iw = 1.0 / G.w;
    return G;
}

// first candidate source bin for target bin B at a stage with A (iA = 1/A) and
// base = g u + C: states below (bin_lo(B) - base) / A cannot reach B
DEV int dp_first_source(const DpGeom& G, int B, double iA, double base) {
    const double xa = (G.glo + B * G.w - base) * iA;
    return (int)floor((xa - G.glo) * G.iw - 1e-7);
}

template <int SS>
DEV bool dp_fixed(const Home& h, LdsD& L, int lane, int nt, double g, double x0, double lo0, double hi0,
                    double lo, double hi, int sx, int sv) {
    constexpr int NU = SS > 0 ? SS + 1 : 16;
    const int H = h.H;
    const int S = SS > 0 ? SS : h.S;
    const DpGeom G = dp_geom(fmin(lo0, lo), fmax(hi0, hi), g);
    const int nb = G.nb;
    double2* cur = L.lab;
    double2* nxt = L.rmin;
    const double BIG = INFINITY;
    for (int k = 0; k < H; ++k) {
        const double Ak = L.cA[k], Ck = L.cC[k], ck = L.cq[k];
        const double blo = k == 0 ? lo0 : lo, bhi = k == 0 ? hi0 : hi;
        const double tlo = blo - TOL_P * (1 + fabs(blo)), thi = bhi + TOL_P * (1 + fabs(bhi));
        const double iA = 1.0 / Ak;
        // the offset is stored in 4 bits: A_k < 1/14 (a tank nearly emptied in one step)
        // caps the window at 16 candidates
        const int ncand = (int)fmin(16.0, ceil(iA) + 2.0);
        for (int B = lane; B < nb; B += nt) {
            const double fB = (double)B, fB1 = (double)(B + 1);
            double best = BIG, bx = 0.0;
            int bp = 0xFF;
            // label x lands in bin B  <=>  floor((x - glo) / w) == B  <=>  B <= t < B + 1
            auto consider = [&](double xn, double cn, int code) {
                const double t = (xn - G.glo) * G.iw;
                const bool ok = (xn >= tlo) & (xn <= thi) & (t >= fB) & (t < fB1) & (cn < best);
                best = ok ? cn : best;
                bx = ok ? xn : bx;
                bp = ok ? code : bp;
            };
            if (k == 0) {
                for (int u = 0; u <= S; ++u)
                    consider(fma(Ak, x0, fma(g, (double)u, Ck)), ck * u, u);
            } else {
                for (int u = 0; u <= S; ++u) {
                    const double bs = fma(g, (double)u, Ck);
                    const int s0 = dp_first_source(G, B, iA, bs);
                    for (int d = 0; d < ncand; ++d) {
                        const int sb = s0 + d;
                        const double2 lv = cur[min(max(sb, 0), nb - 1)];
                        const double cs = (sb >= 0 && sb < nb) ? lv.x : BIG;
                        consider(fma(Ak, lv.y, bs), fma(ck, (double)u, cs), u | (d << 4));
                    }
                }
            }
            nxt[B] = make_double2(best, bx);
            L.par[k * NB_CAP + B] = (uint16_t)bp;
        }
        __syncthreads();
        double2* t = cur; cur = nxt; nxt = t;
    }
    // cheapest final label (lowest bin on ties, deterministic)
    double best = BIG;
    int bb = -1;
    for (int B = lane; B < nb; B += nt)
        if (cur[B].x < best) { best = cur[B].x; bb = B; }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bb, o);
        if (ob < best || (ob == best && oi >= 0 && (bb < 0 || oi < bb))) { best = ob; bb = oi; }
    }
    if (nt > WAVE) {
        int* ri = reinterpret_cast<int*>(L.sc + 16);
        if ((lane & (WAVE - 1)) == 0) { L.sc[lane / WAVE] = best; ri[lane / WAVE] = bb; }
        __syncthreads();
        best = L.sc[0]; bb = ri[0];
        for (int i = 1; i < nt / WAVE; ++i) {
            const double ob = L.sc[i];
            const int oi = ri[i];
            if (ob < best || (ob == best && oi >= 0 && (bb < 0 || oi < bb))) { best = ob; bb = oi; }
        }
        __syncthreads();
    }
    if (bb < 0) return false;
    if (lane == 0) {
        int b = bb;
        for (int k = H - 1; k >= 0; --k) {
            const int p = L.par[k * NB_CAP + b];
            const int u = p & 15;
            L.x[k * 8 + sv] = (double)u;
            if (k > 0) b = dp_first_source(G, b, 1.0 / L.cA[k], fma(g, (double)u, L.cC[k])) + (p >> 4);
        }
        double x = x0;                      // exact forward trajectory of the chosen duties
        for (int k = 0; k < H; ++k) {
            x = fma(L.cA[k], x, fma(g, L.x[k * 8 + sv], L.cC[k]));
            L.x[k * 8 + sx] = x;
        }
    }
    __syncthreads();
    return true;
}

// --------------------------------------------------------------------------------------
// The same DP on buckets that move with the chain's zero-duty reference trajectory
// r_{k+1} = A_k r_k + C_k.  With z = (x - r_k)/w + c_k (c_0 = 1/2, c_{k+1} = A_k c_k) the
// dynamics become z' = A_k z + sh*u with sh = +-NBU an integer (w = |g|/NBU), so a label's
// target bucket is floor(A_k z) + sh*u: ONE key T_s = floor(A_k z_s) per source bucket, and
// the sources of (target b, duty u) are exactly the run {s : T_s = b - sh*u} (1-2 buckets,
// found through an inverse table).  Labels keep their EXACT state x, as in dp_fixed, and
// every kept path is exactly feasible; buckets are the only approximation.  Each stage:
// keys -> inverse table -> pull over target buckets; three barriers.
// Returns 1 solved, 0 no integer schedule, -1 geometry unsupported (more than NB_CAP
// buckets: the caller uses dp_fixed with wider bins).
// --------------------------------------------------------------------------------------
template <int SS>
DEV int dp_zspace(const Home& h, LdsD& L, int lane, int nt, double g, double x0, double lo0, double hi0,
                  double lo, double hi, int sx, int sv) {
    constexpr int NU = SS > 0 ? SS + 1 : 16;
    const int H = h.H;
    const int S = SS > 0 ? SS : h.S;
    // buckets per duty unit: NBU at 15-min steps, proportionally more at coarser steps so that
    // the bucket width (in degrees) does not grow with the step length
    const int nbu = max(NBU, (4 * NBU) / max(1, h.dt));
    const double w = fabs(g) / nbu, iw = 1.0 / w;
    const int sh = g > 0.0 ? nbu : -nbu;
    const double BIG = INFINITY;
    {
        const double tl = lo - TOL_P * (1 + fabs(lo)), th = hi + TOL_P * (1 + fabs(hi));
        if ((th - tl) * iw + 4.0 > (double)NB_CAP) return -1;
    }
    const double zspan = 30000.0;                                 // int16 keys and sources
    if (lane == 0) {
        double r = x0;
        L.rt[0] = r;
        for (int k = 0; k < H; ++k) {
            r = fma(L.cA[k], r, L.cC[k]);
            L.rt[k + 1] = r;
        }
    }
    __syncthreads();
    // bucket window of the labels x_{k+1} (tolerance-widened box, one bucket of margin)
    auto window = [&](int k, double c1, int* blo) -> int {
        const double bl = k == 0 ? lo0 : lo, bh = k == 0 ? hi0 : hi;
        const double tl = bl - TOL_P * (1 + fabs(bl)), th = bh + TOL_P * (1 + fabs(bh));
        const double r = L.rt[k + 1];
        *blo = (int)floor((tl - r) * iw + c1) - 1;
        return (int)floor((th - r) * iw + c1) + 1 - *blo + 1;
    };
    double2* lab = L.lab;
    for (int k = 0; k <= H; ++k) {                                // keys must fit in int16
        const double zr = fmax(fabs((lo - L.rt[k]) * iw), fabs((hi - L.rt[k]) * iw));
        if (!(zr < zspan)) return -1;
    }
    // stage 0: from the single initial label (z = 1/2) to buckets sh*u + floor(A_0 / 2) = sh*u
    double c = 0.5;
    double cn1 = L.cA[0] * c;
    int blo;
    int nbz = window(0, cn1, &blo);
    {
        const double A0 = L.cA[0], C0 = L.cC[0], q0 = L.cq[0];
        const double tl = lo0 - TOL_P * (1 + fabs(lo0)), th = hi0 + TOL_P * (1 + fabs(hi0));
        for (int j = lane; j < nbz; j += nt) { lab[j] = make_double2(BIG, 0.0); L.par[j] = 0xFFFF; }
        __syncthreads();
        for (int u = lane; u <= S; u += nt) {
            const int j = sh * u + (int)floor(cn1) - blo;
            const double xn = fma(A0, x0, fma(g, (double)u, C0));
            if (j >= 0 && j < nbz && xn >= tl && xn <= th) {
                lab[j] = make_double2(q0 * u, xn);
                L.par[j] = (uint16_t)(u << 12);
            }
        }
        __syncthreads();
    }
    c = cn1;
    // source key of a label for the next stage: T = floor(A z), z clamped into its bucket
    // (keeps T monotone in the bucket index); an empty bucket uses its centre
    auto key = [&](double2 lv, int b, double A, double r, double cz) -> int16_t {
        const double fb = (double)b;
        double zz = lv.x < BIG ? (lv.y - r) * iw + cz : fb + 0.5;
        zz = fmin(fmax(zz, fb), fb + 0.999999);
        return (int16_t)floor(A * zz);
    };
    // key hull of the finite labels [kfl, kfh]: the next stage's targets b = key + sh*u
    // (u in 0..S) outside its reach have no candidate, so the window is clipped to it (one
    // wave; the tank chain's labels sit in a narrow band of its box).  Bit-identical: only
    // empty buckets are dropped and the order of the kept ones is unchanged.
    int kfl = INT_MIN / 2, kfh = INT_MAX / 2;
    const bool clip = nt == WAVE;
    if (H > 1) {
        int hl = INT_MAX, hh = INT_MIN;
        for (int s = lane; s < nbz; s += nt) {
            const int T = key(lab[s], blo + s, L.cA[1], L.rt[1], c);
            L.tarr[s] = T;
            if (lab[s].x < BIG) { hl = min(hl, T); hh = max(hh, T); }
        }
        if (clip) { kfl = dpp_imin(hl); kfh = dpp_imax(hh); }
        __syncthreads();
    }
    for (int k = 1; k < H; ++k) {
        const double Ak = L.cA[k], Ck = L.cC[k], ck = L.cq[k];
        const double tl = lo - TOL_P * (1 + fabs(lo)), th = hi + TOL_P * (1 + fabs(hi));
        // target window of stage k+1 and its box-boundary buckets: a bucket strictly inside the
        // box (margin far above rounding) accepts every label landing in it, so only a run's
        // cheapest label can win there; the 4-5 boundary buckets need every run member with
        // the exact box test.
        const double c1 = Ak * c;
        int blo1;
        int nbz1 = window(k, c1, &blo1);
        if (clip) {
            const int lo1 = max(blo1, kfl + min(0, sh * S)), hi1 = min(blo1 + nbz1 - 1, kfh + max(0, sh * S));
            if (lo1 > hi1) return 0;                      // no finite label can go on
            blo1 = lo1;
            nbz1 = hi1 - lo1 + 1;
        }
        const double r1 = L.rt[k + 1];
        int jin0 = (int)ceil((tl - r1) * iw + c1 + 1e-6) - blo1;
        int jin1 = (int)floor((th - r1) * iw + c1 - 1e-6) - 1 - blo1;
        jin0 = min(max(jin0, 0), nbz1);
        jin1 = min(max(jin1, jin0 - 1), nbz1 - 1);
        const int nleft = jin0, nbnd = jin0 + (nbz1 - 1 - jin1);
        if (nbnd > NBND) return -1;                       // degenerate box: caller uses dp_fixed
        struct Best { double c, x; int p; };
        auto consider = [&](Best& B, double2 lv, double base, int u, int src) {
            const double xn = fma(Ak, lv.y, base);
            const double cn = fma(ck, (double)u, lv.x);
            const bool ok = (xn >= tl) & (xn <= th) & (cn < B.c);
            B.c = ok ? cn : B.c;
            B.x = ok ? xn : B.x;
            B.p = ok ? (src | (u << 12)) : B.p;
        };
        // (b) per key m: the cheapest label of the run {s : T_s = m} (ascending s, first minimum)
        //     and its bucket, at index m - mlo + 1 (keys skipped by the contraction: rsrc = -1;
        //     indices 0 and M + 2 are empty sentinels, so a clamped index needs no range test).
        //     Runs are 1-2 buckets while A_k > 2/3: both members are loaded up front.
        const int mlo = L.tarr[0], mhi = L.tarr[nbz - 1], M = mhi - mlo;
        if (lane == 0) {
            L.rmin[0] = make_double2(BIG, 0.0); L.rsrc[0] = -1;
            L.rmin[M + 2] = make_double2(BIG, 0.0); L.rsrc[M + 2] = -1;
        }
        const double iA = 1.0 / Ak;
        for (int s = lane; s < nbz; s += nt) {
            // every key and label this bucket may need, read together (the edge reads are
            // clamped and their values replaced)
            const int T = L.tarr[s];
            int Tp = L.tarr[max(s - 1, 0)], Tn = L.tarr[min(s + 1, nbz - 1)], Tn2 = L.tarr[min(s + 2, nbz - 1)];
            const double2 l0 = lab[s];
            const double2 l1 = lab[min(s + 1, nbz - 1)];
            Tp = s > 0 ? Tp : mlo - 1;
            Tn = s + 1 < nbz ? Tn : mhi + 1;
            Tn2 = s + 2 < nbz ? Tn2 : mhi + 1;
            if (T > Tp + 1)                                   // keys skipped by the map (rare)
                for (int m = Tp + 1; m < T; ++m) { L.rmin[m - mlo + 1] = make_double2(BIG, 0.0); L.rsrc[m - mlo + 1] = -1; }
            if (T > Tp) {                                     // s heads the run of key T
                const bool take1 = Tn == T && l1.x < l0.x;
                double2 bl = take1 ? l1 : l0;
                int bs = take1 ? s + 1 : s;
                if (Tn2 == T)                                 // runs of 3+ (A_k < 2/3)
                    for (int s2 = s + 2; s2 < nbz && L.tarr[s2] == T; ++s2) {
                        const double2 lv = lab[s2];
                        if (lv.x < bl.x) { bl = lv; bs = s2; }
                    }
                L.rmin[T - mlo + 1] = bl;
                L.rsrc[T - mlo + 1] = (int16_t)bs;
            }
        }
        // boundary (bucket q, duty u) pairs, one per lane: the run of key m = b - sh*u is
        // located from the near-linear key map (T_s ~ A s) and walked to, then every member is
        // tested against the exact box
        for (int idx = lane; idx < nbnd * (S + 1); idx += nt) {
            constexpr int NUC = SS > 0 ? SS + 1 : 1;           // compile-time divisor when known
            const int q = SS > 0 ? idx / NUC : idx / (S + 1);
            const int u = idx - q * (S + 1);
            const int j = q < nleft ? q : jin1 + 1 + (q - nleft);
            const int m = blo1 + j - sh * u;
            Best B{BIG, 0.0, 0xFFFF};
            if (m >= mlo && m <= mhi) {
                // T_s = floor(A z), z in [b, b+1): a member's bucket b lies in
                // (m/A - 1, (m+1)/A); one bucket of margin each side covers rounding
                const int sa = max((int)floor(m * iA) - 2 - blo, 0);
                const int sb = min((int)floor((m + 1) * iA) + 1 - blo, nbz - 1);
                const double base = fma(g, (double)u, Ck);
                constexpr int W = 6;
                if (sb - sa < W) {
                    int tk[W];
                    double2 lv[W];
#pragma unroll
                    for (int i = 0; i < W; ++i) {
                        const int s3 = min(sa + i, sb);
                        tk[i] = L.tarr[s3];
                        lv[i] = lab[s3];
                    }
#pragma unroll
                    for (int i = 0; i < W; ++i)
                        if (sa + i <= sb && tk[i] == m) consider(B, lv[i], base, u, sa + i);
                } else {
                    for (int s3 = sa; s3 <= sb; ++s3)
                        if (L.tarr[s3] == m) consider(B, lab[s3], base, u, s3);
                }
            }
            L.cand[idx] = make_double2(B.c, B.x);
            L.candp[idx] = B.p;
        }
        __syncthreads();
        // (c) targets, written over the label array in place (nothing here reads it or the
        //     keys), each with its key for the next stage.  Interior buckets: the first (in duty
        //     order) cheapest run minimum, with its state and source carried along; the box test
        //     is implied.
        const bool more = k + 1 < H;
        const double An = more ? L.cA[k + 1] : 1.0;
        // the first (in duty order) cheapest run minimum of target j (SS > 0: keys of all
        // duties inside [0, M+2] for most interior buckets, no clamping)
        auto pick = [&](int j, double& bc, int& bu) {
            const int m0 = blo1 + j - mlo + 1;
            bc = BIG;
            bu = -1;
            if constexpr (SS > 0) {
                double lv[NU];
                const bool inside = min(m0, m0 - sh * SS) >= 0 && max(m0, m0 - sh * SS) <= M + 2;
                if (inside) {
#pragma unroll
                    for (int u = 0; u < NU; ++u) lv[u] = L.rmin[m0 - sh * u].x;
                } else {
#pragma unroll
                    for (int u = 0; u < NU; ++u) lv[u] = L.rmin[min(max(m0 - sh * u, 0), M + 2)].x;
                }
                // first cheapest duty by a pairwise tournament (the right operand wins only when
                // strictly cheaper, so ties keep the lower duty): log2 depth instead of a chain
                double cv[NU];
                int cu[NU];
#pragma unroll
                for (int u = 0; u < NU; ++u) { cv[u] = fma(ck, (double)u, lv[u]); cu[u] = u; }
#pragma unroll
                for (int st = 1; st < NU; st <<= 1)
#pragma unroll
                    for (int u = 0; u + st < NU; u += 2 * st) {
                        const bool ok = cv[u + st] < cv[u];
                        cv[u] = ok ? cv[u + st] : cv[u];
                        cu[u] = ok ? cu[u + st] : cu[u];
                    }
                const bool any = cv[0] < bc;
                bc = any ? cv[0] : bc;
                bu = any ? cu[0] : bu;
            } else {
                for (int u = 0; u <= S; ++u) {
                    const double cn = fma(ck, (double)u, L.rmin[min(max(m0 - sh * u, 0), M + 2)].x);
                    if (cn < bc) { bc = cn; bu = u; }
                }
            }
        };
        // run-minimum index of the winning duty (a valid index when there is none)
        auto win = [&](int j, int bu) { return min(max(blo1 + j - mlo + 1 - sh * max(bu, 0), 0), M + 2); };
        int hl = INT_MAX, hh = INT_MIN;                   // key hull of this stage's finite labels
        auto emit = [&](int j, double bc, int bu, double2 src, int rs) {
            double2 out = make_double2(BIG, 0.0);
            int p = 0xFFFF;
            if (bu >= 0) {
                out = make_double2(bc, fma(Ak, src.y, fma(g, (double)bu, Ck)));
                p = rs | (bu << 12);
            }
            lab[j] = out;
            L.par[k * NB_CAP + j] = (uint16_t)p;
            if (more) {
                const int T = key(out, blo1 + j, An, r1, c1);
                L.tarr[j] = T;
                hl = bu >= 0 ? min(hl, T) : hl;
                hh = bu >= 0 ? max(hh, T) : hh;
            }
        };
        // one target per lane and pass: with the tournament pick a target's chain is short, and
        // pairing targets (more registers, a clamped repeat past the end) measured slower
        for (int j = jin0 + lane; j <= jin1; j += nt) {
            double bc;
            int bu;
            pick(j, bc, bu);
            const int wi = win(j, bu);
            emit(j, bc, bu, L.rmin[wi], L.rsrc[wi]);
        }
        // boundary buckets: the first cheapest of their per-duty candidates
        for (int q = lane; q < nbnd; q += nt) {
            const int j = q < nleft ? q : jin1 + 1 + (q - nleft);
            Best B{BIG, 0.0, 0xFFFF};
            if constexpr (SS > 0) {
                double2 cv[NU];
                int cp[NU];
#pragma unroll
                for (int u = 0; u < NU; ++u) { cv[u] = L.cand[q * NU + u]; cp[u] = L.candp[q * NU + u]; }
#pragma unroll
                for (int u = 0; u < NU; ++u) {
                    const bool ok = cv[u].x < B.c;
                    B.c = ok ? cv[u].x : B.c;
                    B.x = ok ? cv[u].y : B.x;
                    B.p = ok ? cp[u] : B.p;
                }
            } else {
                for (int u = 0; u <= S; ++u) {
                    const double2 cv = L.cand[q * (S + 1) + u];
                    if (cv.x < B.c) { B.c = cv.x; B.x = cv.y; B.p = L.candp[q * (S + 1) + u]; }
                }
            }
            const double2 out = make_double2(B.c, B.x);
            lab[j] = out;
            L.par[k * NB_CAP + j] = (uint16_t)B.p;
            if (more) {
                const int T = key(out, blo1 + j, An, r1, c1);
                L.tarr[j] = T;
                hl = B.p != 0xFFFF ? min(hl, T) : hl;
                hh = B.p != 0xFFFF ? max(hh, T) : hh;
            }
        }
        if (clip && more) { kfl = dpp_imin(hl); kfh = dpp_imax(hh); }
        __syncthreads();
        blo = blo1; nbz = nbz1; c = c1;
    }
    // cheapest final label (lowest bucket on ties, deterministic)
    double best = BIG;
    int bb = -1;
    for (int j = lane; j < nbz; j += nt)
        if (lab[j].x < best) { best = lab[j].x; bb = j; }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bb, o);
        if (ob < best || (ob == best && oi >= 0 && (bb < 0 || oi < bb))) { best = ob; bb = oi; }
    }
    if (nt > WAVE) {
        int* ri = reinterpret_cast<int*>(L.sc + 16);
        if ((lane & (WAVE - 1)) == 0) { L.sc[lane / WAVE] = best; ri[lane / WAVE] = bb; }
        __syncthreads();
        best = L.sc[0]; bb = ri[0];
        for (int i = 1; i < nt / WAVE; ++i) {
            const double ob = L.sc[i];
            const int oi = ri[i];
            if (ob < best || (ob == best && oi >= 0 && (bb < 0 || oi < bb))) { best = ob; bb = oi; }
        }
        __syncthreads();
    }
    if (bb < 0) return 0;
    if (lane == 0) {
        int j = bb;
        for (int k = H - 1; k >= 0; --k) {
            const int p = L.par[k * NB_CAP + j];
            L.x[k * 8 + sv] = (double)(p >> 12);
            j = p & 0xFFF;
        }
        double x = x0;                      // exact forward trajectory (the labels' arithmetic)
        for (int k = 0; k < H; ++k) {
            x = fma(L.cA[k], x, fma(g, L.x[k * 8 + sv], L.cC[k]));
            L.x[k * 8 + sx] = x;
        }
    }
    __syncthreads();
    return 1;
}

template <int SS>
DEV bool dp_thermal(const Home& h, LdsD& L, int lane, int nt, double g, double x0, double lo0, double hi0,
                    double lo, double hi, int sx, int sv) {
    const int r = dp_zspace<SS>(h, L, lane, nt, g, x0, lo0, hi0, lo, hi, sx, sv);
    if (r >= 0) return r == 1;
    return dp_fixed<SS>(h, L, lane, nt, g, x0, lo0, hi0, lo, hi, sx, sv);
}

// --------------------------------------------------------------------------------------
// EXACT thermal chain DP: forward Pareto fronts (dp_front).
//
// Chain  x_{k+1} = A_k x_k + C_k + g u_k,  u_k in {0..S},  x_1 in [lo0, hi0],
// x_{k+1} in [lo, hi] (k >= 1),  minimise sum_k q_k u_k  (q_k = gamma^k price_k P S:
// mpc_calc.py:314-317, 330-332, 318-349, 441-446).
//
// Key s = dx * x oriented so that a larger key is "more duty done" when every q_k >= 0
// (dx = sign g) and "less duty done" when every q_k <= 0 (dx = -sign g).  The cost-to-go
// V_k(s) is then non-increasing in s on the set F_k of states that still have a feasible
// continuation, so a label (s_a, c_a) with s_a >= s_b, c_a <= c_b makes (s_b, c_b) useless.
// No bucketing approximation: every kept label carries its exact state and cost, and a
// label is dropped only when another label provably dominates it.  Checked against an
// assumption-free backward step-function DP (oracle/thermal.py) and HiGHS proven optima.
//
// F_k (states of stage k with a feasible continuation) is the hull of the box and the
// preimage of F_{k+1} under the stage map; with F_{k+1} at least one duty step wide the
// preimages of consecutive duties overlap, so the hull is exact (narrower: the caller falls
// back).  Children outside F_{k+1} are dropped (they could dominate and then die).
//
// One stage on one wave; the front is an UNSORTED list (nothing needs its order):
//  1. every child (parent i, duty u) inside F_{k+1} falls in one of NTB equal KEY buckets
//     of the children's key range and one of NTB equal COST buckets of their cost range;
//     64-bit LDS atomics keep per key bucket the cheapest child (largest key among equally
//     cheap ones) and per cost bucket the largest-key child (cheapest among equal keys),
//     as 32-bit ordered bounds rounded outward (cost up, key down);
//  2. two wave scans: mh_b = min cost over the key buckets above b, kl_b = max key over
//     the cost buckets below b;
//  3. a child is dropped if one of these four references provably dominates it (its own
//     key rounded up, cost rounded down): a key bucket above, its key bucket's cheapest
//     child, a cost bucket below, its cost bucket's largest-key child.  Key buckets alone
//     cannot separate labels of equal duty totals (a tank without draws: A = 1 - 4e-5, keys
//     equal to 1e-5 while costs differ), cost buckets can;
//  4. the others are appended (wave ballot, parent order) as the new front.
// A dominated child that no reference catches is kept: that only costs work (measured:
// fronts within 0.1-0.4 % of the exact Pareto fronts at NTB = 256).  Back-pointer (parent | duty << 12) per new label goes to the
// global workspace.  Returns 1 solved (optimal for the chain), 0 no integer schedule, -1 not
// applicable (mixed-sign prices, a feasible set narrower than one duty step, front
// overflow): the caller falls back.
// --------------------------------------------------------------------------------------
struct FrontBufs {
    double2 *fa, *fb;                    // [NF] fronts (key, cost), ping-pong
    unsigned long long* kb;              // [NTB] key buckets: packed (cost up | ~key down) minima
    unsigned long long* cb;              // [NTB] cost buckets: packed (key down | ~cost up) maxima
    unsigned* mh;                        // [NTB] ordered min cost over the key buckets above
    unsigned* kl;                        // [NTB] ordered max key over the cost buckets below
    unsigned *flo, *fhi;                 // [H + 1] feasible-set hull of x_k: 32-bit fixed point
                                         //   over the chain's widened box, rounded outward
    const double *cA, *cC, *cq;          // [H] chain coefficients and duty costs
    double* x;                           // [8H] stage-slot solution (writes slots sx, sv)
    uint16_t* par;                       // global back-pointer rows, packed densely (row k at flo[k])
    double2* wg;                         // [H + 1][WAVE] global: LP cost-to-go W_j as points (x, v),
                                         //   +inf padded; nullptr = no bound pruning
    double *wlx, *wlv, *wls;             // [WAVE] LDS: the current stage's W (points, slopes)
    char* xch;                           // [xch_bytes(CAP)] LDS: the waves' exchange area (NW > 1)
    // dp_front<..., CELL = true>: the cell bound in place of W
    const uint16_t* cg;                  // [H + 1][CELL_STRIDE] global: cell_rows' lower bounds of x_k's cost-to-go
    double c_lo, c_inv;                  // the grid: cell of x = floor((x - c_lo) c_inv)
    float c_off, c_sc;                   // the codes' offset and scale (cell_rows)
};

// 1 / w to about 1 ulp: v_rcp_f64 and one Newton step (no IEEE division sequence)
DEV double rcp_nr(double w) {
    double r = __builtin_amdgcn_rcp(w);
    return fma(fma(-w, r, 1.0), r, r);
}

// W, a convex piecewise-linear function, as m <= 64 points (x_i, v_i), one per lane (+inf past
// m), ascending in x.  Value at a uniform point p inside [x_0, x_{m-1}] (v_readlane of the
// segment found by a ballot).
DEV double pl_eval(double wx, double wv, int m, double p) {
    const int cnt = __popcll(__ballot(wx <= p));
    const int i = min(max(cnt - 1, 0), m - 2);
    const double x0 = read_lane(wx, i), x1 = read_lane(wx, i + 1);
    const double v0 = read_lane(wv, i), v1 = read_lane(wv, i + 1);
    const double w = x1 - x0;
    return w > 0.0 ? fma((p - x0) * rcp_nr(w), v1 - v0, v0) : fmin(v0, v1);
}
// the lanes' points of one W into the LDS table (points, slopes to the next point)
DEV void w_to_lds(const FrontBufs& B, int lane, double wx, double wv) {
    const double nx = __shfl_down(wx, 1), nv = __shfl_down(wv, 1);
    const double s = (lane < WAVE - 1 && nx < INFINITY && nx > wx) ? (nv - wv) * rcp_nr(nx - wx) : 0.0;
    B.wlx[lane] = wx;
    B.wlv[lane] = wv;
    B.wls[lane] = s;
}
// W(x) at a per-lane point from the LDS table: binary search, then the segment's line (its linear
// extension outside [x_0, x_{m-1}], where the integer programme has no schedule anyway).  st0 = the
// largest power of two <= m - 1 for a row of m points (w_st0): log2(m) dependent LDS reads, not 6
// (rows of a tariff day hold a handful of points; the table past m is +inf)
DEV int w_st0(int m) { return m <= 1 ? 0 : 1 << (31 - __builtin_clz((unsigned)(m - 1))); }
DEV double w_eval(const FrontBufs& B, double x, int st0) {
    int i = 0;
    for (int st = st0; st > 0; st >>= 1)
        if (B.wlx[i + st] <= x) i += st;
    return fma(x - B.wlx[i], B.wls[i], B.wlv[i]);
}
// two points' W in lockstep (the same search depth): the same values as two w_eval calls
DEV void w_eval2(const FrontBufs& B, double x, double y, int st0, double& wx, double& wy) {
    int i = 0, j = 0;
    for (int st = st0; st > 0; st >>= 1) {
        const double a = B.wlx[i + st], b = B.wlx[j + st];
        if (a <= x) i += st;
        if (b <= y) j += st;
    }
    wx = fma(x - B.wlx[i], B.wls[i], B.wlv[i]);
    wy = fma(y - B.wlx[j], B.wls[j], B.wlv[j]);
}
// inclusive scan over the 64 lanes with identity id (lanes shifted in from outside a row
// keep id: bound_ctrl off), rows combined through v_readlane
template <int CTRL, typename T>
DEV T dpp_mov_or(T v, T id) { return __builtin_amdgcn_update_dpp(id, v, CTRL, 0xf, 0xf, false); }
template <typename T, typename Op>
DEV T dpp_iscan(T v, int lane, T id, Op op) {
    v = op(v, dpp_mov_or<0x111>(v, id));
    v = op(v, dpp_mov_or<0x112>(v, id));
    v = op(v, dpp_mov_or<0x114>(v, id));
    v = op(v, dpp_mov_or<0x118>(v, id));
    const T t0 = read_lane(v, 15), t1 = read_lane(v, 31), t2 = read_lane(v, 47);
    const int row = lane >> 4;
    const T o1 = t0, o2 = op(t0, t1), o3 = op(o2, t2);
    const T off = row == 1 ? o1 : row == 2 ? o2 : o3;
    return row == 0 ? v : op(v, off);
}

// The cell bound of one chain: row k of cg (k = 1 .. H) holds, per cell [a, b] of a uniform grid of
// NCELL cells over the chain's box, a LOWER bound of the integer cost-to-go of every state x_k in the
// cell (widened by rounding margins): row H = 0 on the cells meeting x_H's box, and row k = min over
// the duties u of q_k u + min of row k + 1 over the cells the image A [a, b] + C + g u meets inside
// x_{k+1}'s box (+inf where none) -- a minimum over a superset of the states a schedule can reach,
// rounded down to f32.  r0 / r1: two LDS rows of scratch (NCELL + 1 floats each at least).  Every thread of the block calls it; false
// (no bound) on a degenerate stage (A <= 0).
// a cell's lower bound from its 16-bit code (offset + q scale, +inf for CELL_INF)
// floor and convert in one instruction (v_cvt_flr_i32_f32; the compiler emits v_floor + v_cvt for (int)floorf):
// the cell kernel's image indices, RL action -1.0 % (round 6)
DEV int cvt_flr(float x) { int r; asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x)); return r; }
DEV float cell_dec(unsigned q, float off, float sc) { return q == CELL_INF ? INFINITY : fmaf((float)q, sc, off); }
// row 0 of a home's cell rows holds no bound: its first three f32 are the rows' valid flag (1), offset, scale
DEV bool cell_rows_valid(const uint16_t* cg) { return reinterpret_cast<const float*>(cg)[0] == 1.0f; }
DEV float cell_off(const uint16_t* cg) { return reinterpret_cast<const float*>(cg)[1]; }
DEV float cell_sc(const uint16_t* cg) { return reinterpret_cast<const float*>(cg)[2]; }
// a f32 lower bound to its 16-bit code, rounded down: decoded, it is at most x (the scale is at least 4 ulps of
// every value of the chain's range, so one step down after the floor suffices; x >= the offset)
DEV unsigned cell_enc(float x, float off, float sc, float inv) {
    if (!(x < INFINITY)) return CELL_INF;
    float qf = fminf(65534.0f, fmaxf(0.0f, floorf((x - off) * inv)));
    if (fmaf(qf, sc, off) > x) qf -= 1.0f;
    return (unsigned)fmaxf(qf, 0.0f);
}

// the cell grid over a chain's box [bl, bh] (widened past every tolerance of the labels' box tests)
DEV void cell_grid(double bl, double bh, double& c_lo, double& c_inv) {
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    c_lo = bl - 8.0 * tw(bl);
    c_inv = (double)NCELL / ((bh + 8.0 * tw(bh)) - c_lo);
}

template <int NT, int SS>
DEV bool cell_rows(uint16_t* cg, float* r0, float* r1, const double* cA, const double* cC, const double* cq, int H, int S,
                   double g, double lo0, double hi0, double lo, double hi, double c_lo, double c_inv, int tid) {
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    const double dlt = 1.0 / c_inv;
    const double eps = 16.0 * TOL_P * (1.0 + fabs(c_lo) + NCELL * dlt);     // past the cell lookup's rounding
    auto bxl = [&](int k) { const double b = k <= 1 ? lo0 : lo; return b - tw(b); };   // box of x_k
    auto bxh = [&](int k) { const double b = k <= 1 ? hi0 : hi; return b + tw(b); };
    for (int k = 0; k < H; ++k)
        if (!(cA[k] > 0.0)) return false;                  // (uniform)
    // the codes' scale: every cost-to-go of x_k (k >= 1) lies in [sum of min(0, q_j S), sum of max(0, q_j S)]
    // over j >= 1 (the rows' values are rounded down below their true ones: the offset sits a margin lower)
    double slo = 0.0, shi = 0.0;
    for (int k = 1; k < H; ++k) { slo += fmin(0.0, cq[k] * S); shi += fmax(0.0, cq[k] * S); }
    const float off = __double2float_rd(slo - 1e-6 * (1.0 + fabs(slo) + fabs(shi)));
    const float sc = __double2float_ru(fmax((shi - (double)off) / 65534.0, (fabs((double)off) + fabs(shi) + 1e-30) * 0x1p-21));
    const float inv = 1.0f / sc;
    if (tid == 0) {
        float* const hd = reinterpret_cast<float*>(cg);      // row 0: the header (valid flag written by the caller)
        hd[1] = off;
        hd[2] = sc;
    }
    // cells meeting a box [l, h]: [cell(l - eps), cell(h + eps)] (clamped to the grid)
    auto cell_span = [&](double l, double h, int& c0, int& c1) {
        c0 = max(0, (int)floor((l - eps - c_lo) * c_inv));
        c1 = min(NCELL - 1, (int)floor((h + eps - c_lo) * c_inv));
    };
    {
        int c0, c1;
        cell_span(bxl(H), bxh(H), c0, c1);
        for (int j = tid; j < NCELL; j += NT) {
            const float v = (j >= c0 && j <= c1) ? 0.0f : INFINITY;
            r0[j] = v;
            cg[(size_t)H * CELL_STRIDE + j] = (uint16_t)cell_enc(v, off, sc, inv);
        }
    }
    __syncthreads();
    float* nxt = r0;
    float* cur = r1;
    for (int k = H - 1; k >= 1; --k) {
        const double A = cA[k], C = cC[k], q = cq[k];
        int b0, b1;
        cell_span(bxl(k), bxh(k), b0, b1);
        // the image of cell j = [a_j - eps, b_j + eps] under duty u, in cell units of x_{k+1}: its ends are
        // affine in j (slope A), lo_u + j A and lo_u + (j + 1) A + w; widened by a margin far above the
        // rounding of this form and of the labels' own arithmetic (tw) -- a superset of the
        // cells the states of cell j reach (outside the grid: clamped, where no state stays feasible)
        // (f32 from here: the cell units of the ends are below ~2^13, their f32 rounding ~1e-3 of a cell at
        // most -- the 0.01-cell margin covers it; values rounded down at every step: still lower bounds)
        const double mg = 0.01 + (2.0 * tw(fabs(C) + fabs(A) * (fabs(c_lo) + NCELL * dlt) + fabs(g) * S) + eps) * c_inv;
        const float basef = (float)((fma(A, c_lo - eps, C) - c_lo) * c_inv - mg);    // lo_0 at j = 0 (u = 0)
        const float wdf = (float)(2.0 * (A * eps * c_inv + mg));                        // the image's extra width
        const float Af = (float)A, guf = (float)(g * c_inv);
        const float qlo = __double2float_rd(q);
        if (Af + wdf < 1.0f) {
            // an image narrower than a cell meets cells i0 and i0 + 1 at most: the pair minima of V_{k+1}
            // once (pm[i + 1] = min(V[i], V[i + 1]), V = +inf past the grid), then one load per duty
            // (with +inf pads: pp[i0 + 2] for a clamped i0 in [-2, NCELL + 1] is +inf at i0 = -2, NCELL, NCELL + 1
            // and min(V[i0], V[i0 + 1]) between -- no range test per duty lookup: RL action -1.9 %, round 6)
            float* const pp = cur;                 // (the stage's output row is written after: pp first)
            for (int i = tid; i <= NCELL; i += NT) {
                const float va = i >= 1 ? nxt[i - 1] : INFINITY, vb = i < NCELL ? nxt[i] : INFINITY;
                pp[i + 1] = fminf(va, vb);
            }
            if (tid < 3) pp[tid == 0 ? 0 : NCELL + 1 + tid] = INFINITY;
            __syncthreads();
            float outv[(NCELL + NT - 1) / NT];
#pragma unroll
            for (int r = 0; r < (NCELL + NT - 1) / NT; ++r) {
                const int j = r * NT + tid;
                float best = INFINITY;
                if (j < NCELL && j >= b0 && j <= b1) {
                    const float lj = fmaf((float)j, Af, basef);
                    float mv[SS + 1];
#pragma unroll
                    for (int u = 0; u <= SS; ++u) {
                        const float l = fmaf((float)u, guf, lj);
                        const int i0 = cvt_flr(fminf(fmaxf(l, -2.0f), (float)NCELL + 1.0f));
                        mv[u] = pp[i0 + 2];
                    }
                    // f32: q rounded down (u >= 0), each sum lowered by 2 ulps past its rounding
#pragma unroll
                    for (int u = 0; u <= SS; ++u) best = fminf(best, fmaf(qlo, (float)u, mv[u]));
                    best = best < INFINITY ? best - fabsf(best) * 2.4e-7f - 1e-30f : INFINITY;
                }
                outv[r] = best;
            }
            __syncthreads();                       // (every thread read pp: the row may be written)
#pragma unroll
            for (int r = 0; r < (NCELL + NT - 1) / NT; ++r) {
                const int j = r * NT + tid;
                if (j < NCELL) { cur[j] = outv[r]; cg[(size_t)k * CELL_STRIDE + j] = (uint16_t)cell_enc(outv[r], off, sc, inv); }
            }
            __syncthreads();
            float* t_ = nxt; nxt = cur; cur = t_;
            continue;
        }
        for (int j = tid; j < NCELL; j += NT) {
            double best = INFINITY;
            if (j >= b0 && j <= b1) {
                const float lj = fmaf((float)j, Af, basef);
                // every duty's (one or two) loads issued together: clamped indices, the test after
                float m0[SS + 1], m1[SS + 1];
                int span[SS + 1];
#pragma unroll
                for (int u = 0; u <= SS; ++u) {
                    const float l = fmaf((float)u, guf, lj), h = l + Af + wdf;
                    const bool in = h >= 0.0f && l <= (float)NCELL;
                    const int i0 = in ? min(NCELL - 1, max(0, (int)floorf(l))) : 0;
                    const int i1 = in ? min(NCELL - 1, max(i0, (int)floorf(h))) : 0;
                    m0[u] = nxt[i0];
                    m1[u] = nxt[min(i0 + 1, i1)];
                    span[u] = in ? i1 - i0 : -1;
                }
#pragma unroll
                for (int u = 0; u <= SS; ++u) {
                    if (span[u] < 0) continue;
                    float m = fminf(m0[u], m1[u]);
                    if (span[u] > 1) {                     // (a stage with A > 1: a wider image)
                        const int i0 = min(NCELL - 1, max(0, (int)floorf(fmaf((float)u, guf, lj))));
                        for (int i = i0 + 2; i <= i0 + span[u]; ++i) m = fminf(m, nxt[i]);
                    }
                    if (m < INFINITY) best = fmin(best, fma(q, (double)u, (double)m));
                }
            }
            const float v = best < INFINITY ? __double2float_rd(best) : INFINITY;
            cur[j] = v;
            cg[(size_t)k * CELL_STRIDE + j] = (uint16_t)cell_enc(v, off, sc, inv);
        }
        __syncthreads();
        float* t_ = nxt; nxt = cur; cur = t_;
    }
    return true;
}

template <int SS, int CAP, int CAPB, int PS, int NBK, int NW, bool CELL, int ILP>
DEV int dp_front(const FrontBufs& B, int H, int tid, double g, double x0, double lo0, double hi0, double lo,
                 double hi, int sx, int sv, bool use_bound, double ub_ext, double* best_out, int beam_k) {
    // ILP = 2 (one wave, few homes per GPU: the launch is as long as its slowest home): passes 1 and 3 take
    // two 64-child chunks per iteration, so that their LDS round trips overlap; same children, same order
    // ILP = 3: two chunks, none held (the side pass's hot kernel: its persistent loop leaves no registers)
    static_assert(ILP == 1 || ((ILP == 2 || ILP == 3) && NW == 1), "two chunks per pass on one wave only");
    constexpr int HOLD = ILP == 2 ? RS_HOLD : 0;        // child pairs held in registers from pass 1 to pass 3
    // NW waves share one home's DP (latency: few homes per GPU): every wave runs the same
    // uniform control flow (W table, hulls and scans are computed redundantly or by wave 0), the
    // children of a stage are split into contiguous pass ranges per wave, and survivors keep the
    // single-wave (parent, duty) order: the fronts, and so the result, are bit-identical for any NW
    constexpr int NT = NW * WAVE;
    const int lane = tid & (WAVE - 1);
    const int wid = NW > 1 ? tid / WAVE : 0;
    constexpr int XP = xch_passes(CAP);
    static_assert(NW == 1 || (SS == 6 && NW <= 8), "the exchange area is sized for S = 6 and up to 8 waves");
    unsigned long long* const xmask = reinterpret_cast<unsigned long long*>(B.xch);
    double* const xbest = reinterpret_cast<double*>(B.xch + XP * 8);
    unsigned* const xint = reinterpret_cast<unsigned*>(B.xch + XP * 8 + 8 * 8);   // [5][8]
    static_assert(SS > 0 && SS < 16, "duty count must be a compile-time constant below 16");
    static_assert(CAP <= PS && CAPB <= PS && PS <= 4096, "back-pointer rows hold a 12-bit parent index");
    constexpr int NU = SS + 1;
    constexpr int BPL = NBK / WAVE;      // buckets per lane in the scan
    static_assert(NBK % WAVE == 0, "");
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    auto umin = [](unsigned a, unsigned b) { return a < b ? a : b; };
    auto umax = [](unsigned a, unsigned b) { return a > b ? a : b; };
    // (a) sign of the duty costs: the orientation of the key
    bool pos = false, neg = false;
    for (int k = lane; k < H; k += WAVE) {
        const double q = B.cq[k];
        pos = pos || q > 0.0;
        neg = neg || q < 0.0;
    }
    pos = __any(pos);
    neg = __any(neg);
    // the key orientation needs duty prices of one sign; otherwise (or on a feasible set narrower
    // than a duty step, whose hull may hold unreachable states) the DP runs without dominance,
    // on the bound alone (below), or falls back
    bool nodom = pos && neg;
    const double dx = ((g > 0.0) != neg) ? 1.0 : -1.0;
    // (b) feasible-set hulls F_H .. F_1 (every lane computes, lane 0 stores).  Stored as 32-bit
    //     fixed point over [hb, hb + 2^32 hs], a range past every stage box and its tolerance
    //     (values outside it would be cut by the stage box anyway): lower ends rounded down,
    //     upper ends up, so the stored hull contains the computed one (one unit ~ box / 2^32)
    const double hb0 = fmin(lo0, lo), he0 = fmax(hi0, hi);
    const double hb = hb0 - 4.0 * tw(hb0), hw = (he0 + 4.0 * tw(he0)) - hb;
    const double hs = hw * 0x1p-32, his = 0x1p32 * rcp_nr(hw);
    auto enc_lo = [&](double v) { return (unsigned)fmin(fmax((v - hb) * his, 0.0), 4294967295.0); };
    auto enc_hi = [&](double v) { return (unsigned)fmin(fmax((v - hb) * his + 1.0, 0.0), 4294967295.0); };
    {
        bool empty = false, narrow = false;
        double l = H == 1 ? lo0 : lo, u = H == 1 ? hi0 : hi;
        l -= tw(l);
        u += tw(u);
        if (tid == 0) { B.flo[H] = enc_lo(l); B.fhi[H] = enc_hi(u); }
        const double gmin = fmin(0.0, g * SS), gmax = fmax(0.0, g * SS);
        for (int k = H - 1; k >= 1 && !empty; --k) {
            narrow = narrow || (u - l < fabs(g));
            const double A = B.cA[k], C = B.cC[k];
            const double iA = rcp_nr(A);                 // ~1 ulp; tw() below widens past it
            const double pl = (l - C - gmax) * iA, ph = (u - C - gmin) * iA;
            const double bl = k == 1 ? lo0 : lo, bh = k == 1 ? hi0 : hi;
            l = fmax(pl, bl - tw(bl));
            u = fmin(ph, bh + tw(bh));
            l -= tw(l);
            u += tw(u);
            empty = l > u;
            if (tid == 0) { B.flo[k] = enc_lo(l); B.fhi[k] = enc_hi(u); }
        }
        if (empty) return 0;
        nodom = nodom || narrow;
    }
    // (c) the LP cost-to-go W_j(x_j) (duties continuous in [0, S]) for j = H .. 1: convex,
    //     piecewise linear, a lower bound of the integer cost-to-go.  From W_{j+1}: the duty's
    //     cheapest use is full duty left of the minimiser of v + (q/g) x and none right of it,
    //     so W_j is W_{j+1}'s point list with the minimiser doubled, the left part shifted by
    //     -max(0, gS) at cost q S [g > 0], the right part by -min(0, gS) at q S [g < 0], mapped
    //     through x = (y - C) / A and cut to x_j's box.  One point per lane, rows in B.wg.
    //     More than 64 points, or a degenerate stage: no bound (exact all the same).
    //     On by request (prices that change at most stages: fronts grow large without it) and
    //     wherever dominance is off; the plain front DP is cheaper on piecewise-constant tariffs.
    double UBT = INFINITY;
    // W rows are stored and loaded only up to their point counts (lane j of wc0 / wc1 holds row j's
    // / row 64 + j's count): no +inf padding goes through memory
    int wc0 = 0, wc1 = 0;
    auto set_count = [&](int j, int m) {
        if ((j & (WAVE - 1)) == lane) { if (j < WAVE) wc0 = m; else wc1 = m; }
    };
    auto row_m = [&](int j) -> int { return j < WAVE ? read_lane(wc0, j) : read_lane(wc1, j - WAVE); };
    auto load_row = [&](int j) -> double2 {
        const int m = row_m(j);
        return lane < m ? B.wg[j * WAVE + lane] : make_double2(INFINITY, INFINITY);
    };
    // kf: the stage the DP continues from (rows W_{kf+1} .. W_H are built); the greedy upper bound
    // starts there from a label (gx0, c0) of the front (a feasible completion of it bounds the optimum)
    auto make_bound = [&](int kf, double gx0, double c0) -> bool {
        if (H >= 2 * WAVE) return false;                 // row counts held for 128 rows (a 32 h horizon)
#ifdef DRAGG_STAGE_PROF
        const unsigned long long mb_t0 = __builtin_amdgcn_s_memtime();
#endif
        bool prune = true;
        {
            double bl = H == 1 ? lo0 : lo, bh = H == 1 ? hi0 : hi;
            bl -= tw(bl);
            bh += tw(bh);
            double wx = lane == 0 ? bl : lane == 1 ? bh : INFINITY, wv = lane < 2 ? 0.0 : INFINITY;
            int m = 2;
            if (wid == 0 && lane < m) B.wg[H * WAVE + lane] = make_double2(wx, wv);
            set_count(H, m);
            for (int j = H - 1; j >= max(1, kf + 1); --j) {
                const double A = B.cA[j], C = B.cC[j], q = B.cq[j];
                if (!(A > 0.0) || m + 1 > WAVE) { prune = false; break; }
                const double zs = g * SS, cS = q * SS;
                const double zlo = fmin(0.0, zs), zhi = fmax(0.0, zs);
                const double cL = zs > 0.0 ? cS : 0.0, cR = zs > 0.0 ? 0.0 : cS;
                const double F = lane < m ? fma(q * rcp_nr(g), wx, wv) : INFINITY;
                const double Fm = dpp_reduce(F, [](double a, double b) { return fmin(a, b); });
                const int js = __ffsll((long long)__ballot(F == Fm)) - 1;
                const double px = __shfl_up(wx, 1), pv = __shfl_up(wv, 1);
                const int m1 = m + 1;
                const double iA = rcp_nr(A);
                double nx = lane <= js ? wx - zhi : px - zlo;
                double nv = lane <= js ? wv + cL : pv + cR;
                nx = (nx - C) * iA;
                if (lane >= m1) { nx = INFINITY; nv = INFINITY; }
                double cl = j == 1 ? lo0 : lo, ch = j == 1 ? hi0 : hi;
                cl -= tw(cl);
                ch += tw(ch);
                const double dl = fmax(cl, read_lane(nx, 0)), dh = fmin(ch, read_lane(nx, m1 - 1));
                if (!(dl <= dh)) { prune = false; break; }
                const double vdl = pl_eval(nx, nv, m1, dl), vdh = pl_eval(nx, nv, m1, dh);
                const bool in = lane < m1 && nx > dl && nx < dh;
                const unsigned long long bal = __ballot(in);
                const int m2 = __popcll(bal) + 2;
                if (m2 > WAVE) { prune = false; break; }
                // compact: the points inside (dl, dh) are a contiguous run of lanes (nx ascending),
                // so the new row is that run shifted to lanes 1 .. m2 - 2 (one lane shuffle, no barrier)
                const int first = bal ? __ffsll((long long)bal) - 1 : 0;
                const int src = min(max(lane - 1 + first, 0), WAVE - 1);
                const double sx_ = __shfl(nx, src), sv_ = __shfl(nv, src);
                wx = lane == 0 ? dl : lane == m2 - 1 ? dh : lane < m2 ? sx_ : INFINITY;
                wv = lane == 0 ? vdl : lane == m2 - 1 ? vdh : lane < m2 ? sv_ : INFINITY;
                m = m2;
                if (wid == 0 && lane < m) B.wg[j * WAVE + lane] = make_double2(wx, wv);
                set_count(j, m);
            }
        }
#ifdef DRAGG_STAGE_PROF
        const unsigned long long mb_t1 = __builtin_amdgcn_s_memtime();
        if (tid == 0) B.x[7 * 8 + S_PAD] += (double)(mb_t1 - mb_t0);
#endif
        // (d) an upper bound: the cost of one feasible schedule, greedy in q u + W_{k+1}(x') (the
        //     labels' own arithmetic).  Children with cost + W > bound (+ a margin past rounding)
        //     cannot lead to the optimum and are dropped.
        if (prune) {
            double qabs = 0.0;
            for (int k = lane; k < H; k += WAVE) qabs += fabs(B.cq[k]) * SS;
            qabs = dpp_sum(qabs);
            double gx = gx0, ub = c0;
            // a caller's bound (the cost of a schedule it has: the bucketed DP's in the mid / big
            // launches) makes the greedy pass unnecessary (RL action 33.7 -> 30.5 ms).  (Last step's
            // plan shifted by a stage as the hot launch's bound, measured: looser than the greedy
            // one, driver window 1.45 -> 1.55 ms)
            bool gok = !(ub_ext < INFINITY);
            // (the W table is wave 0's to load and write; every wave reads it.)  Rows in flight three
            // stages ahead: a stage of this pass is far shorter than a global load's latency
            const double2 NONE = make_double2(INFINITY, INFINITY);
            double2 cur = (wid == 0 && gok) ? load_row(kf + 1) : NONE;
            double2 n1 = (wid == 0 && gok && kf + 2 <= H) ? load_row(kf + 2) : NONE;
            double2 n2 = (wid == 0 && gok && kf + 3 <= H) ? load_row(kf + 3) : NONE;
            for (int k = kf; k < H && gok; ++k) {
                const double2 n3 = (wid == 0 && k + 4 <= H) ? load_row(k + 4) : NONE;
                if (wid == 0) w_to_lds(B, lane, cur.x, cur.y);
                __syncthreads();
                const double A = B.cA[k], C = B.cC[k], q = B.cq[k];
                double bl = k == 0 ? lo0 : lo, bh = k == 0 ? hi0 : hi;
                bl -= tw(bl);
                bh += tw(bh);
                if (k + 1 < H) {
                    bl = fmax(bl, fma((double)B.flo[k + 1], hs, hb));
                    bh = fmin(bh, fma((double)B.fhi[k + 1], hs, hb));
                }
                const double xc = fma(A, gx, fma(g, (double)lane, C));
                double val = INFINITY;
                if (lane <= SS && xc >= bl && xc <= bh) val = (double)lane * q + w_eval(B, xc, w_st0(row_m(k + 1)));
                const double vm = dpp_reduce(val, [](double a, double b) { return fmin(a, b); });
                if (!(vm < INFINITY)) { gok = false; break; }
                const int bu = __ffsll((long long)__ballot(val == vm)) - 1;
                gx = read_lane(xc, bu);
                ub = fma(q, (double)bu, ub);
                cur = n1; n1 = n2; n2 = n3;
                __syncthreads();
            }
            if (gok) UBT = ub + TOL_P * (1.0 + fabs(ub) + qabs);
            // a caller's upper bound (the cost of a schedule it already has), with the same margin
            if (ub_ext < INFINITY) { UBT = fmin(UBT, ub_ext + TOL_P * (1.0 + fabs(ub_ext) + qabs)); gok = true; }
            if (!gok) prune = false;
        }
#ifdef DRAGG_STAGE_PROF
        if (tid == 0) B.x[8 * 8 + S_PAD] += (double)(__builtin_amdgcn_s_memtime() - mb_t1);
#endif
        return prune;
    };
    bool prune;
    if constexpr (CELL) {
        // the cell bound (B.cg) prunes from stage 0 on against the caller's upper bound; a beam pass
        // (beam_k > 0) runs without one: its truncation keeps the fronts small, with or without dominance
        double qabs = 0.0;
        for (int k = lane; k < H; k += WAVE) qabs += fabs(B.cq[k]) * SS;
        qabs = dpp_sum(qabs);
        prune = ub_ext < INFINITY;
        if (prune) UBT = ub_ext + TOL_P * (1.0 + fabs(ub_ext) + qabs);
        if (nodom && !prune && beam_k == 0) return (pos && neg) ? -1 : -2;
    } else {
        prune = B.wg != nullptr && (use_bound || nodom) && make_bound(0, x0, 0.0);
        if (nodom && !prune) return nodom && (pos && neg) ? -1 : -2;
    }
    int capn = prune ? CAPB : CAP;                   // front capacity (overflow: -3)
    bool tried = CELL || prune || B.wg == nullptr;   // the bound is built at most once
    // the cell bound's row of the stage's children, read from the workspace (cell_kernel's rows: staging
    // them in LDS cost a block per CU of the mid launch, measured slower)
    const uint16_t* crow = B.cg + CELL_STRIDE;
    auto cell_at = [&](double x) -> double {
        const int c = min(NCELL - 1, max(0, (int)floor((x - B.c_lo) * B.c_inv)));
        return (double)cell_dec(crow[c], B.c_off, B.c_sc);
    };
    auto bound_at = [&](double x, int wst_) -> double {
        if constexpr (CELL) return cell_at(x); else return w_eval(B, x, wst_);
    };
    auto bound_at2 = [&](double x, double y, int wst_, double& bx_, double& by_) {
        if constexpr (CELL) { bx_ = cell_at(x); by_ = cell_at(y); } else w_eval2(B, x, y, wst_, bx_, by_);
    };
    // the front stores each label's exact STATE x (not its key dx * x) and cost
    double2* fa = B.fa;
    double2* fb = B.fb;
    if (tid == 0) fa[0] = make_double2(x0, 0.0);
    int n = 1;
    double xmin = x0, xmax = x0, cmin = 0.0, cmax = 0.0;    // state / cost range of the front
    const unsigned long long below = (1ull << lane) - 1ull;  // lanes < this one
    for (int b = tid; b < NBK; b += NT) { B.kb[2 * b] = ~0ull; B.cb[2 * b] = 0ull; }
    // W_{k+1} of the stage in the LDS table, W_{k+2} in flight
    double2 wnext = make_double2(INFINITY, INFINITY);
    if constexpr (CELL) {
    } else if (prune && wid == 0) {
        const double2 w1 = load_row(1);
        w_to_lds(B, lane, w1.x, w1.y);
        if (H >= 2) wnext = load_row(2);
    }
    __syncthreads();
#ifdef DRAGG_STAGE_PROF
    // diagnostic: shader-clock cycles per stage section (0 ranges, 1 pass 1, 2 scans, 3 pass 3,
    // 4 reductions / clears / W table, 5 stages), added into the S_PAD slots of stages 0..5
    unsigned long long sp_acc[7] = {0, 0, 0, 0, 0, 0, 0}, sp_t = __builtin_amdgcn_s_memtime();
#define SP_MARK(i) do { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); sp_acc[i] += n_ - sp_t; sp_t = n_; } while (0)
#endif
    // back-pointer rows are packed densely: row k (the survivors of stage k) starts at pbase, kept in
    // B.flo[k] (dead from stage k on: stage k - 1 was its last reader), so that a home's rows are
    // one contiguous run of ~sum n_k entries (the traceback stages them in LDS, below)
    int pbase = 0;
    for (int k = 0; k < H; ++k) {
#ifdef DRAGG_STAGE_PROF
        sp_acc[5] += 1;
        sp_t = __builtin_amdgcn_s_memtime();
#endif
        if (tid == 0) B.flo[k] = (unsigned)pbase;
        uint16_t* const prow = B.par + pbase;
        // a front past PRUNE_AT labels (a tariff boundary inside the horizon): build the LP
        // bound now and prune the remaining stages by it.  Only while the front fits the bounded
        // capacity (the W table's LDS follows it) -- and, when fa is that buffer, stays clear of it.
#ifdef DRAGG_STAGE_PROF
        const bool sp_trig = !tried && n > PRUNE_AT && n <= CAPB;
        if (sp_trig) SP_MARK(0);
#endif
        if (!tried && n > PRUNE_AT && n <= CAPB) {
            tried = true;
            // the rows from this stage on, the greedy bound from the front's cheapest label
            double bc = INFINITY, bx = 0.0;
            int bi = -1;
            for (int i = tid; i < n; i += NT) {
                const double2 Li = fa[i];
                if (Li.y < bc) { bc = Li.y; bx = Li.x; bi = i; }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const double oc = __shfl_xor(bc, o), ox = __shfl_xor(bx, o);
                const int oi = __shfl_xor(bi, o);
                if (oc < bc || (oc == bc && oi >= 0 && (bi < 0 || oi < bi))) { bc = oc; bx = ox; bi = oi; }
            }
            if constexpr (NW > 1) {
                __syncthreads();
                if (lane == 0) { xbest[wid] = bc; xint[wid] = (unsigned)bi; }
                __syncthreads();
                bc = xbest[0]; bi = (int)xint[0];
                for (int w = 1; w < NW; ++w) {
                    const double oc = xbest[w];
                    const int oi = (int)xint[w];
                    if (oc < bc || (oc == bc && oi >= 0 && (bi < 0 || oi < bi))) { bc = oc; bi = oi; }
                }
                bx = fa[bi].x;
                __syncthreads();
            }
            if (make_bound(k, bx, bc)) {
                prune = true;
                capn = CAPB;
                if (wid == 0) {
                    const double2 wk = load_row(k + 1);
                    w_to_lds(B, lane, wk.x, wk.y);
                    wnext = k + 2 <= H ? load_row(k + 2) : make_double2(INFINITY, INFINITY);
                }
            }
            __syncthreads();
        }
#ifdef DRAGG_STAGE_PROF
        if (sp_trig) SP_MARK(6);
#endif
        const double A = B.cA[k], C = B.cC[k], q = B.cq[k];
        double bl = k == 0 ? lo0 : lo, bh = k == 0 ? hi0 : hi;
        bl -= tw(bl);
        bh += tw(bh);
        if (k + 1 < H) {
            bl = fmax(bl, fma((double)B.flo[k + 1], hs, hb));
            bh = fmin(bh, fma((double)B.fhi[k + 1], hs, hb));
        }
        const int wst = (prune && !CELL) ? w_st0(row_m(k + 1)) : 0;   // W_{k+1}'s search depth
        // the children's state and cost ranges (widened past rounding) define the two bucket
        // grids of this stage.  A child's position in a range as a 32-bit fixed-point number
        // v = (key - lo) * NBK * 2^23 / (hi - lo) (one fma from the state) gives its bucket
        // (v >> 23) and, v being computed to far better than one unit, conservative bounds
        // v - 1 <= V <= v + 2 of the exact monotone position V: references use the bound that
        // understates them, the tested child the one that overstates it.
        double xl = fmax(bl, fma(A, xmin, C) + fmin(0.0, g * SS));
        double xh = fmin(bh, fma(A, xmax, C) + fmax(0.0, g * SS));
        if (!(xl <= xh)) return 0;                       // no child can stay feasible
        xl -= tw(xl); xh += tw(xh);
        double clo = cmin + fmin(0.0, q * SS), chi = cmax + fmax(0.0, q * SS);
        clo -= tw(clo); chi += tw(chi);
        // scales ~ NBK 2^23 / width by a refined reciprocal (any scale near it will do: the
        // positions are monotone and their bounds hold for the scale actually used)
        const double FX = (double)NBK * 8388608.0;        // NBK * 2^23 <= 2^31
        const double ksc = FX * rcp_nr(xh - xl), csc = FX * rcp_nr(chi - clo);
        // key position: (dx x - key_lo) * ksc with key_lo = dx > 0 ? xl : -xh
        const double kmul = dx * ksc, kadd = -(dx > 0.0 ? xl : -xh) * ksc;
        const double cadd = -clo * csc;
        auto fixp = [](double y) { return (unsigned)fmax(y, 0.0); };   // y < 2^31 + 1
        auto dn = [](unsigned v) { return max(v, 1u) - 1u; };
        // children are numbered c = NU * parent + duty and spread over the lanes (a stage
        // with n labels takes ceil(NU n / 64) passes, not NU ceil(n / 64))
        const int nc = n * NU;
#ifdef DRAGG_STAGE_PROF
        SP_MARK(0);
#endif
        // 1. per key bucket the cheapest child (largest key among equally cheap ones), per
        //    cost bucket the largest-key child (cheapest among equal keys), both as
        //    understated bounds (cost up, key down), by 64-bit LDS atomics
        auto bucket_refs_v = [&](unsigned vk, unsigned vc) {
            const unsigned cu = vc + 2u, kd = dn(vk);
            atomicMin(&B.kb[2 * min(NBK - 1, (int)(vk >> 23))], ((unsigned long long)cu << 32) | (unsigned long long)(~kd));
            atomicMax(&B.cb[2 * min(NBK - 1, (int)(vc >> 23))], ((unsigned long long)kd << 32) | (unsigned long long)(~cu));
        };
        auto bucket_refs = [&](double xc, double cc) { bucket_refs_v(fixp(fma(xc, kmul, kadd)), fixp(fma(cc, csc, cadd))); };
        // ILP = 2: children c and c + NT of a pair; the first RS pairs' states, costs and box / bound verdicts
        // stay in registers for pass 3 (no second load of their parents, no second bound search)
        double r_x1[HOLD > 0 ? HOLD : 1], r_x2[HOLD > 0 ? HOLD : 1], r_c1[HOLD > 0 ? HOLD : 1], r_c2[HOLD > 0 ? HOLD : 1];
        unsigned r_v[HOLD > 0 ? HOLD : 1][4];                    // and their fixed-point positions (vk, vc of each child)
        unsigned r_keep = 0u;                        // bit 2r: pair r's first child passed, 2r + 1: its second
        auto pair1 = [&](int c, double& xc, double& cc, double& x2, double& c2c, bool& k1, bool& k2) {
            const int c2 = c + NT;
            const bool h1 = c < nc, h2 = c2 < nc;
            const int i = h1 ? c / NU : 0, u = c - i * NU;
            const int i2 = h2 ? c2 / NU : i, u2 = h2 ? c2 - i2 * NU : u;
            const double2 Li = fa[i], L2 = fa[i2];
            xc = fma(A, Li.x, fma(g, (double)u, C)); x2 = fma(A, L2.x, fma(g, (double)u2, C));
            cc = fma(q, (double)u, Li.y); c2c = fma(q, (double)u2, L2.y);
            k1 = h1 && xc >= bl && xc <= bh; k2 = h2 && x2 >= bl && x2 <= bh;
            if (prune) {
                double b1, b2;
                bound_at2(xc, x2, wst, b1, b2);
                k1 = k1 && cc + b1 <= UBT;
                k2 = k2 && c2c + b2 <= UBT;
            }
        };
        if constexpr (ILP >= 2) {
#pragma unroll
            for (int r = 0; r < HOLD; ++r) {
                if (r * 2 * NT < nc && !nodom) {
                    double xc, cc, x2, c2c;
                    bool k1, k2;
                    pair1(tid + r * 2 * NT, xc, cc, x2, c2c, k1, k2);
                    r_x1[r] = xc; r_c1[r] = cc; r_x2[r] = x2; r_c2[r] = c2c;
                    r_keep |= (k1 ? 1u : 0u) << (2 * r) | (k2 ? 2u : 0u) << (2 * r);
                    r_v[r][0] = fixp(fma(xc, kmul, kadd)); r_v[r][1] = fixp(fma(cc, csc, cadd));
                    r_v[r][2] = fixp(fma(x2, kmul, kadd)); r_v[r][3] = fixp(fma(c2c, csc, cadd));
                    if (k1) bucket_refs_v(r_v[r][0], r_v[r][1]);
                    if (k2) bucket_refs_v(r_v[r][2], r_v[r][3]);
                }
            }
            for (int c = tid + HOLD * 2 * NT; c < nc && !nodom; c += 2 * NT) {
                double xc, cc, x2, c2c;
                bool k1, k2;
                pair1(c, xc, cc, x2, c2c, k1, k2);
                if (k1) bucket_refs(xc, cc);
                if (k2) bucket_refs(x2, c2c);
            }
        } else {
            for (int c = tid; c < nc && !nodom; c += NT) {
                const int i = c / NU, u = c - i * NU;
                const double2 Li = fa[i];
                const double xc = fma(A, Li.x, fma(g, (double)u, C));
                const double cc = fma(q, (double)u, Li.y);
                if (xc >= bl && xc <= bh && (!prune || cc + bound_at(xc, wst) <= UBT)) bucket_refs(xc, cc);
            }
        }
        __syncthreads();
#ifdef DRAGG_STAGE_PROF
        SP_MARK(1);
#endif
        // 2. mh[b] = min cost over the key buckets above b (lane l holds key chunk 63 - l:
        //    "above" = lower lanes, an exclusive prefix-min); kl[b] = max key over the cost
        //    buckets below b (lane l holds cost chunk l: an exclusive prefix-max)
        if (!nodom && wid == 0) {
            const int c0 = (WAVE - 1 - lane) * BPL, d0 = lane * BPL;
            unsigned bm[BPL], bk[BPL];
            unsigned lm = ~0u, lk = 0u;
#pragma unroll
            for (int j = 0; j < BPL; ++j) {
                bm[j] = (unsigned)(B.kb[2 * (c0 + j)] >> 32);
                lm = umin(lm, bm[j]);
                bk[j] = (unsigned)(B.cb[2 * (d0 + j)] >> 32);
                lk = umax(lk, bk[j]);
            }
            const unsigned im = dpp_iscan(lm, lane, ~0u, umin);
            const unsigned ik = dpp_iscan(lk, lane, 0u, umax);
            unsigned rm = __shfl_up(im, 1), rk = __shfl_up(ik, 1);
            if (lane == 0) { rm = ~0u; rk = 0u; }
#pragma unroll
            for (int j = BPL - 1; j >= 0; --j) {
                B.mh[4 * (c0 + j)] = rm;
                rm = umin(rm, bm[j]);
            }
#pragma unroll
            for (int j = 0; j < BPL; ++j) {
                B.kl[4 * (d0 + j)] = rk;
                rk = umax(rk, bk[j]);
            }
        }
        __syncthreads();
#ifdef DRAGG_STAGE_PROF
        SP_MARK(2);
#endif
        // 3. survivors appended to the other buffer in (parent, duty) order.  A child X is
        //    dropped when one of four references provably dominates it (X's bounds
        //    overstated: key up, cost down):
        //    - a key bucket above holds a child no dearer:          cost_dn(X) >= mh
        //    - its key bucket's cheapest child Y:    key_up(X) <= key(Y), cost_dn(X) >= cost(Y)
        //    - a cost bucket below holds a child with no smaller key:  key_up(X) <= kl
        //    - its cost bucket's largest-key child Y' likewise
        //    (the per-bucket tests need one strict inequality: X may be the reference)
        int nn = 0;
        unsigned kmn = ~0u, kmx = 0u, cmn = ~0u, cmx = 0u;  // survivors' fixed-point ranges
        // child c of this stage: state, cost, fixed-point positions and the keep decision
        auto child = [&](int c, int& i, int& u, double& xc, double& cc, unsigned& vk, unsigned& vc) -> bool {
            const bool have = c < nc;
            i = have ? c / NU : 0;
            u = c - i * NU;
            const double2 Li = fa[i];
            xc = fma(A, Li.x, fma(g, (double)u, C));
            cc = fma(q, (double)u, Li.y);
            vk = fixp(fma(xc, kmul, kadd));
            vc = fixp(fma(cc, csc, cadd));
            return have && xc >= bl && xc <= bh;
        };
        auto undominated = [&](unsigned vk, unsigned vc) -> bool {
            const int kbk = min(NBK - 1, (int)(vk >> 23)), cbk = min(NBK - 1, (int)(vc >> 23));
            const unsigned ku = vk + 2u, cd = dn(vc);
            // a bucket's reference and its scan value in one 16-B load each
            const uint4 rk_ = reinterpret_cast<const uint4*>(B.kb)[kbk], rc_ = reinterpret_cast<const uint4*>(B.cb)[cbk];
            const unsigned ycu = rk_.y, ykd = ~rk_.x;
            const unsigned zkd = rc_.y, zcu = ~rc_.x;
            const bool d1 = cd >= rk_.z;
            const bool d2 = ku <= ykd && cd >= ycu && (ku < ykd || cd > ycu);
            const bool d3 = ku <= rc_.z;
            const bool d4 = ku <= zkd && cd >= zcu && (ku < zkd || cd > zcu);
            return !(d1 || d2 || d3 || d4);
        };
        auto eval = [&](int c, int& i, int& u, double& xc, double& cc, unsigned& vk, unsigned& vc) -> bool {
            bool keep = child(c, i, u, xc, cc, vk, vc);
            if (keep && prune) keep = cc + bound_at(xc, wst) <= UBT;
            if (keep && !nodom) keep = undominated(vk, vc);
            return keep;
        };
        unsigned Kmn, Kmx, Cmn, Cmx;
        auto append = [&](bool keep, int i, int u, double xc, double cc, unsigned vk, unsigned vc) {
            const unsigned long long bal = __ballot(keep);
            const int slot = nn + __popcll(bal & below);
            nn += __popcll(bal);
            if (keep && slot < capn) {
                fb[slot] = make_double2(xc, cc);
                prow[slot] = (uint16_t)(i | (u << 12));
                kmn = umin(kmn, vk); kmx = umax(kmx, vk);
                cmn = umin(cmn, vc); cmx = umax(cmx, vc);
            }
        };
        if constexpr (ILP >= 2) {
            auto pair3 = [&](int i, int u, int i2, int u2, double xc, double cc, double x2, double c2c, unsigned vk,
                             unsigned vc, unsigned vk2, unsigned vc2, bool k1, bool k2) {
                if (!nodom) {
                    const bool n1 = undominated(vk, vc), n2 = undominated(vk2, vc2);
                    k1 = k1 && n1;
                    k2 = k2 && n2;
                }
                append(k1, i, u, xc, cc, vk, vc);
                append(k2, i2, u2, x2, c2c, vk2, vc2);
            };
            auto fresh = [&](int c0) {
                int i, u, i2, u2;
                double xc, cc, x2, c2c;
                unsigned vk, vc, vk2, vc2;
                bool k1 = child(c0 + lane, i, u, xc, cc, vk, vc);
                bool k2 = child(c0 + WAVE + lane, i2, u2, x2, c2c, vk2, vc2);
                if (prune) {
                    double b1, b2;
                    bound_at2(xc, x2, wst, b1, b2);
                    k1 = k1 && cc + b1 <= UBT;
                    k2 = k2 && c2c + b2 <= UBT;
                }
                pair3(i, u, i2, u2, xc, cc, x2, c2c, vk, vc, vk2, vc2, k1, k2);
            };
#pragma unroll
            for (int r = 0; r < HOLD; ++r) {
                const int c0 = r * 2 * WAVE;
                if (c0 < nc) {
                    if (!nodom) {                       // pass 1's children (the same arithmetic, kept)
                        const int c = c0 + lane, c2 = c + WAVE;
                        const int i = c < nc ? c / NU : 0, i2 = c2 < nc ? c2 / NU : i;
                        pair3(i, c - i * NU, i2, c2 < nc ? c2 - i2 * NU : c - i * NU, r_x1[r], r_c1[r], r_x2[r], r_c2[r],
                              r_v[r][0], r_v[r][1], r_v[r][2], r_v[r][3], (r_keep >> (2 * r)) & 1u,
                              (r_keep >> (2 * r + 1)) & 1u);
                    } else {
                        fresh(c0);
                    }
                }
            }
            for (int c0 = HOLD * 2 * WAVE; c0 < nc; c0 += 2 * WAVE) fresh(c0);
            Kmn = dpp_reduce(kmn, umin); Kmx = dpp_reduce(kmx, umax);
            Cmn = dpp_reduce(cmn, umin); Cmx = dpp_reduce(cmx, umax);
        } else if constexpr (NW == 1) {
            for (int c0 = 0; c0 < nc; c0 += WAVE) {
                int i, u;
                double xc, cc;
                unsigned vk, vc;
                const bool keep = eval(c0 + lane, i, u, xc, cc, vk, vc);
                append(keep, i, u, xc, cc, vk, vc);
            }
            Kmn = dpp_reduce(kmn, umin); Kmx = dpp_reduce(kmx, umax);
            Cmn = dpp_reduce(cmn, umin); Cmx = dpp_reduce(cmx, umax);
        } else {
            // (a) each wave decides its contiguous passes, keeping the survivor masks; (b) after the
            // exchange, each wave appends its survivors at its offset (the waves below it first)
            const int P = (nc + WAVE - 1) / WAVE;
            const int p0 = wid * P / NW, p1 = (wid + 1) * P / NW;
            int cnt = 0;
            for (int p = p0; p < p1; ++p) {
                int i, u;
                double xc, cc;
                unsigned vk, vc;
                const bool keep = eval(p * WAVE + lane, i, u, xc, cc, vk, vc);
                const unsigned long long bal = __ballot(keep);
                if (lane == 0) xmask[p] = bal;
                cnt += __popcll(bal);
                if (keep) { kmn = umin(kmn, vk); kmx = umax(kmx, vk); cmn = umin(cmn, vc); cmx = umax(cmx, vc); }
            }
            kmn = dpp_reduce(kmn, umin); kmx = dpp_reduce(kmx, umax);
            cmn = dpp_reduce(cmn, umin); cmx = dpp_reduce(cmx, umax);
            if (lane == 0) {
                xint[0 * 8 + wid] = (unsigned)cnt; xint[1 * 8 + wid] = kmn; xint[2 * 8 + wid] = kmx;
                xint[3 * 8 + wid] = cmn; xint[4 * 8 + wid] = cmx;
            }
            __syncthreads();
            int off = 0;
            Kmn = ~0u; Kmx = 0u; Cmn = ~0u; Cmx = 0u;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const int cw = (int)xint[w];
                off += w < wid ? cw : 0;
                nn += cw;
                Kmn = umin(Kmn, xint[8 + w]); Kmx = umax(Kmx, xint[16 + w]);
                Cmn = umin(Cmn, xint[24 + w]); Cmx = umax(Cmx, xint[32 + w]);
            }
            for (int p = p0; p < p1; ++p) {
                const unsigned long long bal = xmask[p];
                if ((bal >> lane) & 1ull) {
                    const int c = p * WAVE + lane;
                    const int i = c / NU, u = c - i * NU;
                    const double2 Li = fa[i];
                    const int slot = off + __popcll(bal & below);
                    if (slot < capn) {
                        fb[slot] = make_double2(fma(A, Li.x, fma(g, (double)u, C)), fma(q, (double)u, Li.y));
                        prow[slot] = (uint16_t)(i | (u << 12));
                    }
                }
                off += __popcll(bal);
            }
        }
#ifdef DRAGG_FRONT_STATS
        if (tid == 0) B.x[k * 8 + S_PAD] += (double)nn * (sx == S_T ? 1.0 : 1e4) +
                                            (k == 0 ? (prune ? 1e8 : 0.0) * (sx == S_T ? 1.0 : 2.0) : 0.0);
#endif
        if (nn == 0) return 0;                       // no child left inside the feasible set
        if constexpr (CELL && NW == 1) {
            // beam: keep the beam_k labels of least cost + bound (index order inside the threshold's
            // bucket), the threshold by two histogram levels; in-order compaction chunk by chunk (a label
            // only moves down), its back-pointer with it
            if (beam_k > 0 && nn > beam_k && nn <= capn) {
                // each label's cost + bound once (its cell row is in the workspace) into the key buckets'
                // LDS, free until the stage's end (beam fronts: nn <= 7 beam_k = 224 <= 2 NBK doubles in the mid
                // launch; with NBK doubles only, as before round 6, the cache never held: RL action -1.4 %)
                double* const fv = reinterpret_cast<double*>(B.kb);
                const bool fcache = nn <= 2 * NBK;         // (the key buckets' 16-B records: 2 NBK doubles)
                double fl = INFINITY, fh = -INFINITY;
                for (int i = lane; i < nn; i += WAVE) {
                    const double2 Li = fb[i];
                    const double f = Li.y + cell_at(Li.x);
                    if (fcache) fv[i] = f;
                    fl = fmin(fl, f); fh = fmax(fh, f);
                }
                auto f_of = [&](int i) { return fcache ? fv[i] : fb[i].y + cell_at(fb[i].x); };
                fl = dpp_reduce(fl, [](double a_, double b_) { return fmin(a_, b_); });
                fh = dpp_reduce(fh, [](double a_, double b_) { return fmax(a_, b_); });
                // the threshold by two histograms of 64 buckets (LDS atomics): over [fl, fh], then over the
                // bucket in which the count of labels below reaches beam_k
                int* const hl = reinterpret_cast<int*>(B.xch);      // (one wave: the exchange area is free)
                double bl_ = fl, bsc = fh > fl ? 64.0 / (fh - fl) : 0.0;
                auto bucket_of = [&](double f, double b0_, double sc_) {
                    return f < INFINITY ? min(63, max(0, (int)((f - b0_) * sc_))) : 64;
                };
                int need = beam_k;                         // labels still to keep at the current level
                double thr_lo = -INFINITY;                  // labels with f < thr_lo are kept
                double thr_in = INFINITY, fcut = INFINITY;  // finally: keep f < thr_in, and of [thr_in, fcut)
                int need_in = 0;                            //   the first need_in in index order
                for (int lvl = 0; lvl < 2; ++lvl) {
                    hl[lane] = 0;
                    wave_sync();
                    for (int i = lane; i < nn; i += WAVE) {
                        const double f = f_of(i);
                        if (f >= thr_lo && (lvl == 0 || f < bl_ + 64.0 / bsc)) {
                            const int bk = bucket_of(f, bl_, bsc);
                            if (bk < 64) atomicAdd(hl + bk, 1);
                        }
                    }
                    wave_sync();
                    const int cnt_ = hl[lane];
                    const int incl = dpp_iscan(cnt_, lane, 0, [](int a_, int b_) { return a_ + b_; });
                    const int bs = __ffsll((long long)__ballot(incl >= need)) - 1;
                    wave_sync();
                    if (bs < 0 || bsc == 0.0) {                // (fewer finite labels than needed, or one f)
                        thr_in = INFINITY; fcut = INFINITY; need_in = 0;
                        if (bsc == 0.0 && bs >= 0) { thr_in = fl; fcut = INFINITY; need_in = need; }
                        break;
                    }
                    const int below_bs = read_lane(incl, bs) - read_lane(cnt_, bs);
                    thr_in = bl_ + bs / bsc;
                    fcut = bl_ + (bs + 1) / bsc;
                    need_in = need - below_bs;
                    if (lvl == 1) break;
                    // keep the buckets below bs; refine inside bs
                    need = need_in;
                    thr_lo = thr_in;
                    bl_ = thr_in;
                    bsc *= 64.0;
                }
                int kept = 0, nin = 0;
                for (int i0 = 0; i0 < nn; i0 += WAVE) {
                    const int i = i0 + lane;
                    double2 Li = make_double2(0.0, 0.0);
                    uint16_t pr = 0;
                    bool must = false, cand = false;
                    if (i < nn) {
                        Li = fb[i];
                        pr = prow[i];
                        const double f = f_of(i);
                        must = f < thr_in;
                        cand = !must && f < fcut;
                    }
                    const unsigned long long bc = __ballot(cand);
                    const bool keep_ = must || (cand && nin + __popcll(bc & below) < need_in);
                    nin += __popcll(bc);
                    const unsigned long long bal = __ballot(keep_);
                    const int pos_ = kept + __popcll(bal & below);
                    kept += __popcll(bal);
                    if (keep_ && pos_ < beam_k) {
                        fb[pos_] = Li;
                        prow[pos_] = pr;
                    }
                }
                nn = min(kept, beam_k);
            }
        }
        if (nn > capn) return -3;                    // front overflow
#ifdef DRAGG_STAGE_PROF
        SP_MARK(3);
#endif
        // the next stage's state and cost ranges from the survivors' positions: the exact
        // position V of a value lies in [v - 1, v + 2], widened past the back-conversion's
        // rounding
        {
            const double klo = dx > 0.0 ? xl : -xh;
            const double ik = (xh - xl) * (1.0 / FX);     // ~1 / ksc; tw() covers the difference
            const double k1 = fma((double)Kmn - 1.0, ik, klo), k2 = fma((double)Kmx + 2.0, ik, klo);
            const double x1 = dx > 0.0 ? k1 : -k2, x2 = dx > 0.0 ? k2 : -k1;
            xmin = x1 - tw(x1);
            xmax = x2 + tw(x2);
            const double ic = (chi - clo) * (1.0 / FX);
            const double c1 = fma((double)Cmn - 1.0, ic, clo), c2 = fma((double)Cmx + 2.0, ic, clo);
            cmin = c1 - tw(c1);
            cmax = c2 + tw(c2);
        }
        for (int b = tid; b < NBK && !nodom; b += NT) { B.kb[2 * b] = ~0ull; B.cb[2 * b] = 0ull; }
        if constexpr (CELL) {
            crow = B.cg + (size_t)(k + 2) * CELL_STRIDE;
        } else if (prune && k + 1 < H && wid == 0) {
            w_to_lds(B, lane, wnext.x, wnext.y);
            if (k + 3 <= H) wnext = load_row(k + 3);
        }
        __syncthreads();
#ifdef DRAGG_STAGE_PROF
        SP_MARK(4);
#endif
        double2* tmp = fa; fa = fb; fb = tmp;
        n = nn;
        pbase += nn;
    }
#ifdef DRAGG_STAGE_PROF
    if (tid == 0) for (int i = 0; i < 7; ++i) B.x[i * 8 + S_PAD] += (double)sp_acc[i];
#endif
    // the cheapest final label (lowest index on ties)
    double best = INFINITY;
    int bi = -1;
    for (int i = tid; i < n; i += NT)
        if (fa[i].y < best) { best = fa[i].y; bi = i; }
    for (int o = 32; o > 0; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob < best || (ob == best && oi >= 0 && (bi < 0 || oi < bi))) { best = ob; bi = oi; }
    }
    if constexpr (NW > 1) {
        if (lane == 0) { xbest[wid] = best; xint[wid] = (unsigned)bi; }
        __syncthreads();
        best = xbest[0]; bi = (int)xint[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            const double ob = xbest[w];
            const int oi = (int)xint[w];
            if (ob < best || (ob == best && oi >= 0 && (bi < 0 || oi < bi))) { best = ob; bi = oi; }
        }
    }
    if (best_out) *best_out = best;
    // the traceback: H dependent reads of the back-pointer rows.  When the dense rows (pbase entries)
    // and the duties fit the fronts' LDS (dead now), one coalesced copy puts them there, so that those
    // reads and the forward pass's are LDS round trips, not L2 ones (A/B: driver window -0.7 %, RL
    // action -3 %)
    double2* const f0 = fa < fb ? fa : fb;
    const int cap_b = ((fa < fb ? fb : fa) == f0 + CAP ? 2 : 1) * CAP * (int)sizeof(double2);
    const int tb = (2 * pbase + 15) / 16 * 16;
    const bool staged = tb + H <= cap_b && (reinterpret_cast<uintptr_t>(B.par) & 15) == 0;
    uint16_t* const lpar = reinterpret_cast<uint16_t*>(f0);
    uint8_t* const ldu = reinterpret_cast<uint8_t*>(f0) + tb;
    __syncthreads();
    if (staged) {
        const uint4* src = reinterpret_cast<const uint4*>(B.par);
        uint4* dst = reinterpret_cast<uint4*>(f0);
        for (int i = tid; i < tb / 16; i += NT) dst[i] = src[i];
        __syncthreads();
    }
    if (tid == 0) {
        const uint16_t* const pr = staged ? lpar : B.par;
        int j = bi;
        for (int k = H - 1; k >= 0; --k) {
            const int p = pr[B.flo[k] + j];
            B.x[k * 8 + sv] = (double)(p >> 12);
            if (staged) ldu[k] = (uint8_t)(p >> 12);
            j = p & 0xFFF;
        }
        double x = x0;                      // exact forward trajectory (the labels' arithmetic)
        for (int k = 0; k < H; ++k) {
            x = fma(B.cA[k], x, fma(g, staged ? (double)ldu[k] : B.x[k * 8 + sv], B.cC[k]));
            B.x[k * 8 + sx] = x;
        }
    }
    __syncthreads();
    return 1;
}

DEV bool round_duties(const Home& h, const Lds& L, int lane, uint16_t* par) {
    const int H = h.H;
    // coefficient arrays live in L.yeq / L.zeq / L.yeqp (4H each, free after the ADMM); the
    // front DP's arrays in the KKT factor blocks Lf / Df (128 H doubles)
    double* cA = L.yeq;
    double* cC = L.zeq;
    double* cq = L.yeqp;
    double* f = L.Lf;
    FrontBufs B;
    B.fa = reinterpret_cast<double2*>(f); f += 2 * NF;
    B.fb = reinterpret_cast<double2*>(f); f += 2 * NF;
    B.kb = reinterpret_cast<unsigned long long*>(f); f += 2 * NTB;     // (bucket records of 16 B, dp_front)
    B.cb = reinterpret_cast<unsigned long long*>(f); f += 2 * NTB;
    B.mh = reinterpret_cast<unsigned*>(B.kb) + 2;
    B.kl = reinterpret_cast<unsigned*>(B.cb) + 2;
    B.flo = reinterpret_cast<unsigned*>(f); f += (H + 2) / 2;
    B.fhi = reinterpret_cast<unsigned*>(f); f += (H + 2) / 2;
    B.cA = cA; B.cC = cC; B.cq = cq; B.x = L.x; B.par = par;
    B.wg = nullptr; B.wlx = B.wlv = B.wls = nullptr;     // no bound pruning on this path
    B.xch = nullptr;                                     // one wave
    B.cg = nullptr; B.c_lo = 0.0; B.c_inv = 0.0; B.c_off = 0.0f; B.c_sc = 0.0f;
    const bool front = h.S == 6 && par != nullptr && (f - L.Lf) <= 128 * H;
    for (int k = lane; k < H; k += WAVE) {
        cA[k] = h.aT;
        cC[k] = L.oat[k + 1] * h.iR * 3600 * h.inv_c;
        cq[k] = L.q[k * 8 + S_U];
    }
    __syncthreads();
    int r = front ? dp_front<6>(B, H, lane, h.g, h.T0, h.Tmin, h.Tmax, h.Tmin, h.Tmax, S_T, S_U) : -1;
    if (r < 0) {
        DpChain cT{H, h.S, S_T, S_U, h.g, cA, cC, h.T0};
        if (!dp_chain(h, L, cT, lane)) return false;
    } else if (r == 0) {
        return false;
    }
    for (int k = lane; k < H; k += WAVE) {
        const double df = L.draw[k + 1] / h.V, rem = 1 - df, d15 = df * TAP;
        cA[k] = rem + (-rem * h.iRw) * 3600 * h.inv_w;
        cC[k] = h.e * L.x[k * 8 + S_T] + (d15 + ((-d15) * h.iRw) * 3600 * h.inv_w);
        cq[k] = L.q[k * 8 + S_W];
    }
    __syncthreads();
    // the tank's stage-0 box is tightened by temp_wh's bounds (build(): lo/hi of slot S_TW)
    r = front ? dp_front<6>(B, H, lane, h.f, h.Tw0, L.lo[S_TW], L.hi[S_TW], h.Twmin, h.Twmax, S_TW, S_W) : -1;
    if (r >= 0) return r == 1;
    DpChain cW{H, h.S, S_TW, S_W, h.f, cA, cC, h.Tw0};
    return dp_chain(h, L, cW, lane);
}

// --------------------------------------------------------------------------------------
// Battery LP (mpc_calc.py:355-373 with its p_grid / cost terms): min sum_k q_k (ch_k + dis_k),
// E_{k+1} = E_k + a ch_k + b dis_k (a = eta_c/dt, b = 1/(eta_d dt)), 0 <= ch <= r,
// -r <= dis <= 0, Emin <= E_{1..H} <= Emax, q_k = S gamma^k price_k.
// The cost-to-go V_k(E) is convex piecewise linear.  With psi_k(z) the cheapest cost of
// moving E_k -> E_k - z in one stage (two linear pieces: charge / discharge, or for q < 0
// the charge-while-discharging edge), V_k = clip(V_{k+1} [inf-convolution] psi_k): the
// sorted (slope, length) segment list of V_{k+1} merged with psi_k's two segments, then
// cut to [Emin, Emax].  Each stage is a rank count + a scatter + a prefix scan on one wave.
// Recovery needs, per stage, only the merged domain origin and the offsets of psi_k's two
// segments in the merged order: the optimal split of a position p along the merged list
// takes psi's share of the first p units of length.  Exact, no iteration.
// Runs on one wave; at most 2H + 1 segments.
// --------------------------------------------------------------------------------------
DEV void battery_psi(const Home& h, double q, double* s1, double* l1, double* s2, double* l2) {
    const double a = h.etac / h.dt, b = (1.0 / h.etad) / h.dt, r = h.brate;
    if (q >= 0.0) { *s1 = -q / a; *l1 = a * r; *s2 = -q / b; *l2 = b * r; }   // charge | discharge
    else          { *s1 = -q / b; *l1 = b * r; *s2 = -q / a; *l2 = a * r; }   // full-charge edge first
}

DEV bool battery_lp(const Home& h, LdsD& L, int lane) {
    const int H = h.H;
    const int cap = seg_cap(H);
    const double a = h.etac / h.dt, b = (1.0 / h.etad) / h.dt, r = h.brate;
    const double x0psi = -a * r;
    double* S0 = L.sgS;  double* L0 = L.sgL;          // current list
    double* S1 = L.sgS + cap; double* L1 = L.sgL + cap;
    int n = 1;
    double x0 = h.Emin;                               // V_H: free terminal state, slope 0
    if (lane == 0) { S0[0] = 0.0; L0[0] = h.Emax - h.Emin; }
    wave_sync();
    bool feasible = true;
    for (int k = H - 1; k >= 0; --k) {
        double s1, l1, s2, l2;
        battery_psi(h, L.cq[k], &s1, &l1, &s2, &l2);
        // ranks: psi's segments go after existing segments of equal slope
        int c1 = 0, c2 = 0;
        double p1 = 0.0, p2 = 0.0;
        for (int i = lane; i < n; i += WAVE) {
            const double si = S0[i], li = L0[i];
            if (si <= s1) { ++c1; p1 += li; }
            if (si <= s2) { ++c2; p2 += li; }
        }
        c1 = dpp_isum(c1); c2 = dpp_isum(c2);
        p1 = dpp_sum(p1); p2 = dpp_sum(p2);
        const int r1 = c1, r2 = c2 + 1;               // merged positions of psi's segments
        p2 += l1;                                     // psi 1 precedes psi 2 (s1 <= s2)
        for (int i = lane; i < n; i += WAVE) {
            const double si = S0[i];
            const int j = i + (s1 < si ? 1 : 0) + (s2 < si ? 1 : 0);
            S1[j] = si; L1[j] = L0[i];
        }
        if (lane == 0) { S1[r1] = s1; L1[r1] = l1; S1[r2] = s2; L1[r2] = l2; }
        const double X0M = x0 + x0psi;
        if (lane == 0) { L.bx0[k] = X0M; L.bp1[k] = p1; L.bp2[k] = p2; }
        n += 2;
        wave_sync();
        double tot = 0.0;
        for (int i = lane; i < n; i += WAVE) tot += L1[i];
        tot = dpp_sum(tot);
        if (k == 0) {                                 // E_0 is fixed: it must lie in the domain
            const double p = h.E0 - X0M;
            feasible = p >= -TOL_P * (1 + fabs(h.E0)) && p <= tot + TOL_P * (1 + fabs(h.E0));
            break;
        }
        // cut the merged list to E_k in [Emin, Emax] (k >= 1)
        const double cl = fmax(0.0, h.Emin - X0M), chi = fmin(tot, h.Emax - X0M);
        if (!(cl <= chi + TOL_P * (1 + fabs(h.Emax)))) { feasible = false; break; }
        // exclusive prefix of lengths in list order (lane-contiguous chunks)
        const int per = (n + WAVE - 1) / WAVE;
        const int i0 = lane * per, i1 = min(n, i0 + per);
        double loc = 0.0;
        for (int i = i0; i < i1; ++i) loc += L1[i];
        const double inc = dpp_scan(loc, lane);
        double pre = inc - loc;
        int first = n, last = -1;
        for (int i = i0; i < i1; ++i) {
            const double st = pre, en = pre + L1[i];
            const double ns = fmax(st, cl), ne = fmin(en, chi);
            if (ne > ns) { first = min(first, i); last = max(last, i); }
            L1[i] = fmax(0.0, ne - ns);
            pre = en;
        }
        first = dpp_imin(first);
        last = dpp_imax(last);
        wave_sync();
        const int nn = last >= first ? last - first + 1 : 0;
        for (int i = lane; i < nn; i += WAVE) { S0[i] = S1[first + i]; L0[i] = L1[first + i]; }
        if (nn == 0 && lane == 0) { S0[0] = 0.0; L0[0] = 0.0; }   // a single feasible point
        n = nn == 0 ? 1 : nn;
        x0 = X0M + cl;
        wave_sync();
    }
    if (!feasible) return false;
    if (lane == 0) {                                  // forward recovery of E, ch, dis
        double E = h.E0;
        for (int k = 0; k < H; ++k) {
            double s1, l1, s2, l2;
            battery_psi(h, L.cq[k], &s1, &l1, &s2, &l2);
            const double p = E - L.bx0[k];
            const double z = x0psi + fmin(fmax(p - L.bp1[k], 0.0), l1) + fmin(fmax(p - L.bp2[k], 0.0), l2);
            const double dlt = -z;                   // E_{k+1} - E_k
            double chv, dis;
            if (L.cq[k] >= 0.0) {
                if (dlt >= 0.0) { chv = fmin(dlt / a, r); dis = 0.0; }
                else            { chv = 0.0; dis = fmax(dlt / b, -r); }
            } else {
                chv = fmin(r, (dlt + b * r) / a);
                dis = fmax(-r, fmin(0.0, (dlt - a * chv) / b));
            }
            E = E + (h.etac * chv + dis / h.etad) / h.dt;   // mpc_calc.py:363-365
            L.x[k * 8 + S_CH] = chv;
            L.x[k * 8 + S_DIS] = dis;
            L.x[k * 8 + S_E] = E;
        }
    }
    wave_sync();
    return true;
}

// --------------------------------------------------------------------------------------
// EXACT thermal chain DP without any dominance assumption: backward step functions (dp_steps).
//
// The front DP's dominance needs every feasible set F_k at least one duty step wide (and prices
// of one sign).  A tank whose feasible window narrows below one duty step (a large draw ahead: the
// tank must be nearly full when it starts) breaks it: the states from which that window can be hit
// form a comb of period ~ one duty step, and the cost-to-go is not monotone on it (measured: the
// Pareto fronts then miss the optimum by up to 30 %, the bucketed approximation by up to 8.5 %).
// This DP assumes nothing: V_k(x) = min_u q_k u + V_{k+1}(A_k x + C_k + g u) is piecewise CONSTANT
// in x, carried backward as sorted breakpoints and values (+inf where no schedule exists), the
// MILP optimum recovered forward by evaluating V_{k+1} at the exact successor states (lowest duty
// on ties) -- the algorithm of the CPU oracle (oracle/thermal.py).
//
// Only the states that can lie on an optimal path are needed: with U >= the optimum (the cost of
// a schedule the caller holds, or of the feasibility pass's schedule), the domain of V_k is cut to
// D_k = {x : L_k(x) + W_k(x) <= U}, L_k the LP cost-to-reach of x_k from x_0 and W_k the LP
// cost-to-go (duties continuous: both convex piecewise linear lower bounds, lp_rows / lp_cut), an
// interval that holds every optimal state.  The cut DP's value is >= the true V_k everywhere and
// equal along every optimal path, so the recovered schedule is the uncut DP's (the same lowest-duty
// rule picks among the same optimal continuations); measured on the bench's narrow tanks: 3-15x
// fewer breakpoints (oracle prototype, same optimum and schedule on every case).
//
// One block of NT threads (DM_NARROW).  Per stage: V_{k+1} staged in LDS; the (S+1) preimage
// lists P_u(i) = (B_i - g u - C) / A of its breakpoints merged in the total order (P, u, i) by
// per-chunk binary searches and monotone walks (no rank tables), each merged point writing the
// value of the elementary interval it starts (min over the duties of q u + V_{k+1} on the interval
// of list u holding it); then zero-width intervals dropped and equal neighbours merged (two block
// scans) into the next V_k of a pool in the workspace.  Returns 1 solved (X written), 0 no integer
// schedule, -3 past the pool / stage capacity, -6 the cut domains lost the schedule (U below the
// optimum: rounding; the caller retries uncut).
// --------------------------------------------------------------------------------------

// block scans for NT = 64 * waves threads (red: >= NT / 64 + 1 ints of LDS); a barrier on both
// sides, so consecutive calls may share `red`
template <int NT>
DEV int block_excl_scan(int v, int* red, int tid, int* tot) {
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
    const int inc = dpp_iscan(v, lane, 0, [](int a, int b) { return a + b; });
    __syncthreads();
    if (lane == WAVE - 1) red[w] = inc;
    __syncthreads();
    int off = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) {
        const int r = red[i];
        off += i < w ? r : 0;
        all += r;
    }
    *tot = all;
    __syncthreads();
    return off + inc - v;
}
// ... with one barrier: the caller keeps `red` (>= NT / 64 ints) for this call alone until a later barrier
template <int NT>
DEV int block_excl_scan1(int v, int* red, int tid, int* tot) {
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
    const int inc = dpp_iscan(v, lane, 0, [](int a, int b) { return a + b; });
    if (lane == WAVE - 1) red[w] = inc;
    __syncthreads();
    int off = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) {
        const int r = red[i];
        off += i < w ? r : 0;
        all += r;
    }
    *tot = all;
    return off + inc - v;
}
template <int NT>
DEV int block_excl_max1(int v, int* red, int tid) {     // max over the threads before this one (-1: none)
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
    const int inc = dpp_iscan(v, lane, -1, [](int a, int b) { return max(a, b); });
    int ex = __shfl_up(inc, 1);
    if (lane == 0) ex = -1;
    if (lane == WAVE - 1) red[w] = inc;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) ex = max(ex, i < w ? red[i] : -1);
    return ex;
}
template <int NT>
DEV int block_excl_max(int v, int* red, int tid) {      // max over the threads before this one (-1: none)
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
    const int inc = dpp_iscan(v, lane, -1, [](int a, int b) { return max(a, b); });
    int ex = __shfl_up(inc, 1);
    if (lane == 0) ex = -1;
    __syncthreads();
    if (lane == WAVE - 1) red[w] = inc;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT / WAVE; ++i) ex = max(ex, i < w ? red[i] : -1);
    __syncthreads();
    return ex;
}

template <int V> struct IntC { static constexpr int value = V; };

struct StepBufs {
    double *PB, *PV;              // global [POOL_CAP]: breakpoints / values of V_k, stage after stage
    int *GIA, *GIB;               // global [MC_CAP]: a stage's point ids (u << 24 | i), ping-pong, past the LDS pool
    double2 *Lrow, *Wrow;         // global [LW_ROWS][WAVE] (x, v): the LP rows L_k / W_k (lp_rows / lp_cut)
    int *off, *cnt, *wc, *lc;     // LDS [H + 1]: pool offset of V_k, its values m (m + 1 breakpoints),
                                  //   points of the W row / L row of x_k (lp_rows / lp_cut)
    int *red;                     // LDS [32] scan scratch (two scans of a stage: [0, 16), [16, 32))
    int *xr;                      // LDS [NT / 64][STEP_MAXU] vector-scan scratch
    int *rng;                     // LDS [4 STEP_MAXU + 8]: per-list index ranges of a stage, run offsets
    double *rl, *rh;              // LDS [H + 1] reachable hull of x_k (widened)
    double *dlo, *dhi;            // LDS [H + 1] the LP sublevel domain of x_k (-inf / +inf: uncut)
    double *xv;                   // LDS [STEP_MAXU] recovery: value of each duty
    double *lt;                   // LDS [3][WAVE] + 2: L_k as a table (points, values, slopes), its
                                  //   minimiser and minimum (the cost pruning)
    char* sp;                     // LDS pool [spb] bytes: per stage V_{k+1} (B, V) and the merge buffers
    int spb;                      //   (lp_cut: the waves' PL tables)
    int pool_cap;                 // breakpoints of all V_k of the chain (<= POOL_CAP; a knob shrinks it)
    long long work_cap;           // merge points over all stages of one pass: the work bound of a chain
};

// exclusive prefix sums over the NT threads of the block of v[0..n) (n <= STEP_MAXU), in place
// (xr: >= NT / 64 * STEP_MAXU ints of LDS, the caller's alone until a later barrier); one barrier
template <int NT, int MU = STEP_MAXU>
DEV void block_excl_scan_vec(int* v, int n, int* xr, int tid) {
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
    int inc[MU];
#pragma unroll
    for (int j = 0; j < MU; ++j) inc[j] = j < n ? dpp_iscan(v[j], lane, 0, [](int a, int b) { return a + b; }) : 0;
    if (lane == WAVE - 1)
#pragma unroll
        for (int j = 0; j < MU; ++j) if (j < n) xr[w * STEP_MAXU + j] = inc[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MU; ++j) {
        if (j >= n) continue;
        int off = 0;
        for (int i = 0; i < w; ++i) off += xr[i * STEP_MAXU + j];
        v[j] = off + inc[j] - v[j];
    }
}

// a PL function of m <= 64 points (one per lane, ascending) into an LDS table: points, values,
// slopes to the next point (0 past the last)
DEV void pl_to_lds(double* T, int lane, double x, double v, int m) {
    const double nx = __shfl_down(x, 1), nv = __shfl_down(v, 1);
    const double s = (lane < m - 1 && nx > x) ? (nv - v) * rcp_nr(nx - x) : 0.0;
    T[lane] = lane < m ? x : INFINITY;
    T[WAVE + lane] = lane < m ? v : INFINITY;
    T[2 * WAVE + lane] = s;
}
// value at x of the table's function, +inf outside [x_0, x_{m-1}]
DEV double pl_tab(const double* T, int m, double x) {
    if (m < 1 || !(x >= T[0] && x <= T[m - 1])) return INFINITY;
    int i = 0;
    for (int st = w_st0(m); st > 0; st >>= 1)
        if (i + st < m && T[i + st] <= x) i += st;
    return fma(x - T[i], T[2 * WAVE + i], T[WAVE + i]);
}

// The LP bounds of one chain (duties continuous in [0, S]) and the cut domains D_k:
//   W_j (cost-to-go of x_j, backward from W_H = 0 on the box; make_bound's construction) on wave 1,
//   L_k (cost-to-reach of x_k from x_0, forward: the inf-convolution of L_k mapped through the
//   stage with the duty's linear cost, i.e. its slope list with the segment of slope q/g and
//   length |g S| merged in, cut to the box) on wave 0, both as rows of <= 64 points;
//   then every wave w takes the stages k = 1 + w, 1 + w + NW, ...: D_k = the sublevel set
//   {L_k + W_k <= U} (convex: an interval, its ends interpolated on the segments where the sum
//   crosses U, widened past rounding).  A row that would pass 64 points, or an empty cut, leaves
//   the stages it covers uncut (-inf, +inf).  Every thread of the block calls it.
template <int NT>
DEV void lp_rows(const StepBufs& Sb, const double* cA, const double* cC, const double* cq, int H, int S, double g,
                 double x0, double lo0, double hi0, double lo, double hi, int tid) {
    static_assert(NT >= 2 * WAVE, "two waves build the rows");
    const int lane = tid & (WAVE - 1), wid = tid / WAVE;
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    auto boxl = [&](int k) { const double b = k == 0 ? lo0 : lo; return b - tw(b); };   // box of x_{k+1}
    auto boxh = [&](int k) { const double b = k == 0 ? hi0 : hi; return b + tw(b); };
    double2* const Lrow = Sb.Lrow;
    double2* const Wrow = Sb.Wrow;
    int* const lcnt = Sb.lc;
    const double zs = g * S, zlo = fmin(0.0, zs), zhi = fmax(0.0, zs);
    for (int k = tid; k <= H; k += NT) { Sb.dlo[k] = -INFINITY; Sb.dhi[k] = INFINITY; Sb.wc[k] = 0; lcnt[k] = 0; }
    __syncthreads();
    // cut a PL function in lanes (nx ascending, m1 points) to [bl, bh]; false if empty
    auto cut = [&](double& nx, double& nv, int m1, double bl, double bh, int& m) -> bool {
        const double dl = fmax(bl, read_lane(nx, 0)), dh = fmin(bh, read_lane(nx, m1 - 1));
        if (!(dl <= dh)) return false;
        const double vdl = m1 >= 2 ? pl_eval(nx, nv, m1, dl) : read_lane(nv, 0);
        const double vdh = m1 >= 2 ? pl_eval(nx, nv, m1, dh) : read_lane(nv, 0);
        const bool in = lane < m1 && nx > dl && nx < dh;
        const unsigned long long bal = __ballot(in);
        const int m2 = __popcll(bal) + 2;
        if (m2 > WAVE) return false;
        const int first = bal ? __ffsll((long long)bal) - 1 : 0;
        const int src = min(max(lane - 1 + first, 0), WAVE - 1);
        const double sx_ = __shfl(nx, src), sv_ = __shfl(nv, src);
        nx = lane == 0 ? dl : lane == m2 - 1 ? dh : lane < m2 ? sx_ : INFINITY;
        nv = lane == 0 ? vdl : lane == m2 - 1 ? vdh : lane < m2 ? sv_ : INFINITY;
        m = m2;
        return true;
    };
    if (wid == 1) {
        // W rows, j = H .. 1
        double wx = lane == 0 ? boxl(H - 1) : lane == 1 ? boxh(H - 1) : INFINITY, wv = lane < 2 ? 0.0 : INFINITY;
        int m = 2;
        if (lane < m) Wrow[H * WAVE + lane] = make_double2(wx, wv);
        if (lane == 0) Sb.wc[H] = m;
        for (int j = H - 1; j >= 1; --j) {
            const double A = cA[j], C = cC[j], q = cq[j];
            if (!(A > 0.0) || m + 1 > WAVE) break;
            const double cS = q * S;
            const double cL = zs > 0.0 ? cS : 0.0, cR = zs > 0.0 ? 0.0 : cS;
            const double F = lane < m ? fma(q * rcp_nr(g), wx, wv) : INFINITY;
            const double Fm = dpp_reduce(F, [](double a, double b) { return fmin(a, b); });
            const int js = __ffsll((long long)__ballot(F == Fm)) - 1;
            const double px = __shfl_up(wx, 1), pv = __shfl_up(wv, 1);
            const int m1 = m + 1;
            double nx = lane <= js ? wx - zhi : px - zlo;
            double nv = lane <= js ? wv + cL : pv + cR;
            nx = (nx - C) * rcp_nr(A);
            if (lane >= m1) { nx = INFINITY; nv = INFINITY; }
            if (!cut(nx, nv, m1, boxl(j - 1), boxh(j - 1), m)) break;
            wx = nx; wv = nv;
            if (lane < m) Wrow[j * WAVE + lane] = make_double2(wx, wv);
            if (lane == 0) Sb.wc[j] = m;
        }
    } else if (wid == 0) {
        // L rows, k = 1 .. H (L_0: the point x_0 at cost 0)
        double lx = lane == 0 ? x0 : INFINITY, lv = lane == 0 ? 0.0 : INFINITY;
        int m = 1;
        for (int k = 0; k < H; ++k) {
            const double A = cA[k], C = cC[k], sg = cq[k] * rcp_nr(g);
            if (!(A > 0.0) || m + 1 > WAVE) break;
            if (lane < m) lx = fma(A, lx, C);
            const double nx_ = __shfl_down(lx, 1), nv_ = __shfl_down(lv, 1);
            const double w = nx_ - lx;
            const bool seg = lane < m - 1;
            const double sl = seg ? (w > 0.0 ? (nv_ - lv) * rcp_nr(w) : (nv_ > lv ? INFINITY : -INFINITY)) : INFINITY;
            const int p = __popcll(__ballot(seg && sl < sg));          // segments flatter than the duty's
            const double ux = __shfl_up(lx, 1), uv = __shfl_up(lv, 1);
            const int m1 = m + 1;
            double nx = lane <= p ? lx + zlo : ux + zhi;
            double nv = lane <= p ? fma(sg, zlo, lv) : fma(sg, zhi, uv);
            if (lane >= m1) { nx = INFINITY; nv = INFINITY; }
            if (!cut(nx, nv, m1, boxl(k), boxh(k), m)) break;
            lx = nx; lv = nv;
            if (lane < m) Lrow[(k + 1) * WAVE + lane] = make_double2(lx, lv);
            if (lane == 0) lcnt[k + 1] = m;
        }
    }
    __syncthreads();
}
// the minimum of L_H: the chain's LP relaxation optimum (every thread; +inf without the row)
DEV double lp_bound(const StepBufs& Sb, int H, int tid) {
    const int lane = tid & (WAVE - 1), ml = Sb.lc[H];
    const double v = lane < ml ? Sb.Lrow[H * WAVE + lane].y : INFINITY;
    return dpp_reduce(v, [](double a, double b) { return fmin(a, b); });
}
// the cut domains D_k = {L_k + W_k <= U} from the rows of lp_rows (any U, again and again)
template <int NT>
DEV void lp_cut(const StepBufs& Sb, int H, double U, int tid) {
    const int lane = tid & (WAVE - 1), wid = tid / WAVE;
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    const double2* const Lrow = Sb.Lrow;
    const double2* const Wrow = Sb.Wrow;
    const int* const lcnt = Sb.lc;
    for (int k = tid; k <= H; k += NT) { Sb.dlo[k] = -INFINITY; Sb.dhi[k] = INFINITY; }
    __syncthreads();
    // the sublevel set of every stage, one wave per stage (its own two PL tables in bs)
    double* const TL = reinterpret_cast<double*>(Sb.sp) + wid * 6 * WAVE;
    double* const TW = TL + 3 * WAVE;
    for (int k = 1 + wid; k <= H; k += NT / WAVE) {
        const int ml = lcnt[k], mw = Sb.wc[k];
        if (ml < 1 || mw < 2) continue;
        const double2 l = lane < ml ? Lrow[k * WAVE + lane] : make_double2(INFINITY, INFINITY);
        const double2 w = lane < mw ? Wrow[k * WAVE + lane] : make_double2(INFINITY, INFINITY);
        pl_to_lds(TL, lane, l.x, l.y, ml);
        pl_to_lds(TW, lane, w.x, w.y, mw);
        wave_sync();
        // the sum at both point sets (+inf outside either domain)
        const double fl = lane < ml ? l.y + pl_tab(TW, mw, l.x) : INFINITY;
        const double fw = lane < mw ? w.y + pl_tab(TL, ml, w.x) : INFINITY;
        auto rmin = [](double a, double b) { return fmin(a, b); };
        auto rmax = [](double a, double b) { return fmax(a, b); };
        const double xa = dpp_reduce(fmin(fl <= U ? l.x : INFINITY, fw <= U ? w.x : INFINITY), rmin);
        if (!(xa < INFINITY)) { wave_sync(); continue; }          // (rounding: leave the stage uncut)
        const double xb = dpp_reduce(fmax(fl <= U && lane < ml ? l.x : -INFINITY, fw <= U && lane < mw ? w.x : -INFINITY), rmax);
        const double xp = dpp_reduce(fmax(lane < ml && l.x < xa ? l.x : -INFINITY, lane < mw && w.x < xa ? w.x : -INFINITY), rmax);
        const double xs = dpp_reduce(fmin(lane < ml && l.x > xb ? l.x : INFINITY, lane < mw && w.x > xb ? w.x : INFINITY), rmin);
        auto f_at = [&](double x) {                                // the sum at one of the points
            return dpp_reduce(fmin(lane < ml && l.x == x ? fl : INFINITY, lane < mw && w.x == x ? fw : INFINITY), rmin);
        };
        const double fa = f_at(xa), fb = f_at(xb), fp = f_at(xp), fs = f_at(xs);
        double a = xa, b = xb;
        if (fp < INFINITY && fp > fa) a = xp + (xa - xp) * ((fp - U) / (fp - fa));
        if (fs < INFINITY && fs > fb) b = xb + (xs - xb) * ((U - fb) / (fs - fb));
        a = fmin(a, xa); b = fmax(b, xb);
        if (lane == 0) { Sb.dlo[k] = a - 4.0 * tw(a); Sb.dhi[k] = b + 4.0 * tw(b); }
        wave_sync();
    }
    __syncthreads();
}

template <int NT>
DEV int dp_steps(const StepBufs& Sb, const double* cA, const double* cC, const double* cq, int H, int S, double g,
                 double x0, double lo0, double hi0, double lo, double hi, double* X, int sx, int sv, int tid,
                 bool feas_only, bool cut_domains, double U = INFINITY) {
    // feas_only: every duty cost taken as 0, so V_k is 0 on the states with a feasible continuation and
    // +inf elsewhere; equal neighbours merge, so V_k is the feasible set as a union of a few intervals.
    // Its breakpoints are the finite region's ends of the full DP's (the same preimage arithmetic),
    // so the feasibility verdict is the full DP's -- at a fraction of its cost (no cost steps).
    // cut_domains: V_k only on Sb.dlo/dhi (lp_rows / lp_cut); else those are ignored.  U < inf (with
    // cut_domains): V_k is also set to +inf on every interval where L_k (lp_rows' cost-to-reach rows)
    // plus V_k exceeds U -- no state there lies on a schedule of cost <= U.
    auto tw = [](double v) { return TOL_P * (1 + fabs(v)); };
    auto boxlo = [&](int k) { const double b = k == 0 ? lo0 : lo; return b - tw(b); };   // box of x_{k+1}
    auto boxhi = [&](int k) { const double b = k == 0 ? hi0 : hi; return b + tw(b); };
    const int NU = S + 1;
    const int lane = tid & (WAVE - 1), wid = tid / WAVE;
    const int fail = cut_domains ? -6 : 0;
    // forward reachable hull R_{k+1} of x_{k+1} (interval arithmetic, widened past rounding)
    if (tid == 0) {
        double l = x0, u = x0;
        const double gmin = fmin(0.0, g * S), gmax = fmax(0.0, g * S);
        Sb.rl[0] = x0; Sb.rh[0] = x0;
        for (int k = 0; k < H; ++k) {
            double a = cA[k] * l + cC[k] + gmin, b = cA[k] * u + cC[k] + gmax;
            a -= tw(a); b += tw(b);
            l = fmax(a, boxlo(k)); u = fmin(b, boxhi(k));
            Sb.rl[k + 1] = l; Sb.rh[k + 1] = u;
        }
    }
    __syncthreads();
    for (int k = 1; k <= H; ++k)
        if (!(Sb.rl[k] <= Sb.rh[k])) return 0;            // no state of stage k stays in its box
    auto dom_lo = [&](int k) { return cut_domains ? fmax(Sb.rl[k], Sb.dlo[k]) : Sb.rl[k]; };
    auto dom_hi = [&](int k) { return cut_domains ? fmin(Sb.rh[k], Sb.dhi[k]) : Sb.rh[k]; };
    // V_H = 0 on its domain
    {
        const double l = dom_lo(H), u = dom_hi(H);
        if (!(l <= u)) return fail;
        if (tid == 0) { Sb.PB[0] = l; Sb.PB[1] = u; Sb.PV[0] = 0.0; Sb.off[H] = 0; Sb.cnt[H] = 1; }
    }
    int top = 2;                                          // next free pool entry (every thread)
    long long work = 0;                                   // merge points so far (the work bound)
    __syncthreads();
#ifdef DRAGG_STEP_PROF
    unsigned long long sp_t = __builtin_amdgcn_s_memtime();
    auto sp_mark = [&](int slot_) {
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();
        if (tid == 0 && !feas_only && slot_ < H) X[slot_ * 8 + S_PAD] += (double)(n_ - sp_t);
        sp_t = n_;
    };
#define SPM(i) sp_mark(i)
#else
#define SPM(i) do {} while (0)
#endif
    for (int k = H - 1; k >= 1; --k) {
        const double A = cA[k], C = cC[k], q = feas_only ? 0.0 : cq[k];
        const double iA = 1.0 / A;
        const int m = Sb.cnt[k + 1], np = m + 1;
        const double* const Bg = Sb.PB + Sb.off[k + 1];
        const double* const Vg = Sb.PV + Sb.off[k + 1];
        // the LDS pool: V_{k+1} (B, V) when it fits, then the merge buffers when they fit too
        double* const bs = reinterpret_cast<double*>(Sb.sp);
        const bool staged = 8 * np <= Sb.spb;
        // V_{k+1}'s values too when they fit (both loads in flight together; first read after the merge)
        const bool lds_v = staged && 16 * np + 32 <= Sb.spb;
        if (staged)
            for (int i = tid; i < np; i += NT) {
                bs[i] = Bg[i];
                if (lds_v && i < m) bs[np + i] = Vg[i];
            }
        // the cost pruning's L_k as an LDS table (wave 0), its minimiser and minimum
        const bool prune = U < INFINITY && Sb.lc[k] >= 1;
        if (prune && wid == 0) {
            const int ml = Sb.lc[k];
            const double2 l = lane < ml ? Sb.Lrow[k * WAVE + lane] : make_double2(INFINITY, INFINITY);
            pl_to_lds(Sb.lt, lane, l.x, l.y, ml);
            const double lm = dpp_reduce(l.y, [](double a_, double b_) { return fmin(a_, b_); });
            const int jm = __ffsll((long long)__ballot(lane < ml && l.y == lm)) - 1;
            if (lane == 0) { Sb.lt[3 * WAVE] = read_lane(l.x, jm); Sb.lt[3 * WAVE + 1] = lm; }
        }
        // the domain of x_k: its box, the reachable hull, the cut
        const double dl = fmax(boxlo(k - 1), dom_lo(k)), dh = fmin(boxhi(k - 1), dom_hi(k));
        if (!(dl <= dh)) return fail;
        __syncthreads();
        const int top2 = 1 << (31 - __builtin_clz((unsigned)np));   // largest power of two <= np
        // list u holds P_u(i) = (B_i - g u - C) / A; the merged order is (P, u): a point of a lower
        // duty first on equal P.  Per list, the points inside (dl, dh) and the last one <= dl (its
        // interval holds dl): indices [lo_u, hi_u).  (The stage is instantiated per memory space of its
        // arrays -- LDS or the workspace -- so that LDS accesses compile to ds_ loads.)
        auto ranges = [&](const auto* Bk) {
            auto P = [&](int u, int i) { return (Bk[i] - g * (double)u - C) * iA; };
            if (wid == 0) {                               // (NU <= STEP_MAXU < 64: one wave)
                const int u = lane;
                int ilo = 0, ihi = 0, first = 0;
                if (u < NU) {
                    int le = 0, lt = 0;                   // points <= dl, points < dh
                    for (int st = top2; st > 0; st >>= 1) {
                        if (le + st <= np && P(u, le + st - 1) <= dl) le += st;
                        if (lt + st <= np && P(u, lt + st - 1) < dh) lt += st;
                    }
                    ilo = max(0, le - 1);
                    ihi = max(lt, ilo);
                    first = (le >= 1 && ilo < ihi) ? 1 : 0;   // its first point is <= dl
                }
                // run offsets ro(u) = points of the lists before u, and the totals, by wave scans
                const int len = ihi - ilo;
                const int inc = dpp_iscan(len, lane, 0, [](int a_, int b_) { return a_ + b_; });
                const int jls = dpp_iscan(first, lane, 0, [](int a_, int b_) { return a_ + b_; });
                const int all = __shfl(inc, NU - 1), jall = __shfl(jls, NU - 1);
                if (u < NU) {
                    Sb.rng[u] = ilo;
                    Sb.rng[STEP_MAXU + u] = ihi;
                    Sb.rng[2 * STEP_MAXU + u] = first;
                    Sb.rng[3 * STEP_MAXU + u] = inc - len;
                } else if (u <= STEP_MAXU) {
                    Sb.rng[3 * STEP_MAXU + u] = all;
                }
                if (lane == 0) Sb.rng[4 * STEP_MAXU + 1] = jall;
            }
        };
        if (staged) ranges(bs); else ranges(Bg);
        __syncthreads();
        const int Mc = Sb.rng[3 * STEP_MAXU + STEP_MAXU], jl = Sb.rng[4 * STEP_MAXU + 1];
        if (Mc > MC_CAP) return -3;
        work += Mc;
        if (work > Sb.work_cap) return -3;                 // (uniform: every thread read the same Mc)
        // run offsets: list u's points at [ro(u), ro(u + 1)) of the merge buffers
        auto ro = [&](int u) { return Sb.rng[3 * STEP_MAXU + min(u, STEP_MAXU)]; };
        SPM(21);
        // The merge: the lists written as runs of (key P, id = u << 24 | i) into buffer 0, then pairs of
        // adjacent runs merged level by level (merge path: every thread takes an equal segment of a
        // pair's output, its start found by a co-rank binary search), then each merged point's value --
        // the value of the elementary interval it starts: min over the lists of q u + V_{k+1} on the
        // interval of the list's last point at or before it (running per-list counts, their chunk
        // offsets by one block scan), pruned by L_k -- and the compaction of the intervals of [dl, dh].
        int res = 1, tot = 0;
        auto stage = [&](const auto* Bk, const auto* Vk, auto* I0, auto* I1, auto mu) {
            constexpr int MU = decltype(mu)::value;       // lists in registers in the values pass (>= NU)
            auto P = [&](int u, int i) { return (Bk[i] - g * (double)u - C) * iA; };
            auto uof = [](int id) { return id >> 24; };
            auto key = [&](int id) { return P(uof(id), id & 0xFFFFFF); };
            // a before b in the merged order (P, u); the caller passes keys it already holds
            auto less = [&](double ka, int ia, double kb, int ib) { return ka < kb || (ka == kb && uof(ia) < uof(ib)); };
            for (int e = tid; e < Mc; e += NT) {
                int u = 0;
                while (u < NU - 1 && e >= ro(u + 1)) ++u;
                I0[e] = (u << 24) | (Sb.rng[u] + (e - ro(u)));
            }
            __syncthreads();
            auto* Is = I0; auto* Id = I1;
            // outputs per work item: about one item per thread (a shorter walk after each co-rank search)
            const int CHm = min(STEP_CH, max(2, (Mc + NT - 1) / NT));
            for (int w = 1; w < NU; w *= 2) {             // runs of w lists -> runs of 2w lists
                const int npair = (NU + 2 * w - 1) / (2 * w);
                int nseg = 0;
                for (int pp = 0; pp < npair; ++pp) {
                    const int o0 = ro(pp * 2 * w), o2 = ro(min(NU, (pp + 1) * 2 * w));
                    nseg += (o2 - o0 + CHm - 1) / CHm;
                }
                for (int it = tid; it < nseg; it += NT) {
                    int pp = 0, r = it, o0 = 0, o1 = 0, o2 = 0;
                    for (; pp < npair; ++pp) {
                        o0 = ro(pp * 2 * w); o1 = ro(min(NU, pp * 2 * w + w)); o2 = ro(min(NU, (pp + 1) * 2 * w));
                        const int ns = (o2 - o0 + CHm - 1) / CHm;
                        if (r < ns) break;
                        r -= ns;
                    }
                    const int la = o1 - o0, lb = o2 - o1;
                    const int d0 = r * CHm, d1 = min(d0 + CHm, la + lb);
                    // co-rank: the A points among the first d0 outputs
                    int lo_ = max(0, d0 - lb), hi_ = min(d0, la);
                    while (lo_ < hi_) {
                        const int mid = (lo_ + hi_) >> 1;
                        const int ib = Is[o1 + d0 - mid - 1], ia = Is[o0 + mid];
                        if (less(key(ib), ib, key(ia), ia)) hi_ = mid;
                        else lo_ = mid + 1;
                    }
                    int ia_ = lo_, ib_ = d0 - lo_;
                    int xa = ia_ < la ? Is[o0 + ia_] : 0, xb = ib_ < lb ? Is[o1 + ib_] : 0;
                    double ka = ia_ < la ? key(xa) : INFINITY, kb = ib_ < lb ? key(xb) : INFINITY;
                    for (int d = d0; d < d1; ++d) {
                        const bool ta = ib_ >= lb || (ia_ < la && less(ka, xa, kb, xb));
                        Id[o0 + d] = ta ? xa : xb;
                        if (ta) {
                            ++ia_;
                            if (ia_ < la) { xa = Is[o0 + ia_]; ka = key(xa); }
                        } else {
                            ++ib_;
                            if (ib_ < lb) { xb = Is[o1 + ib_]; kb = key(xb); }
                        }
                    }
                }
                __syncthreads();
                auto* ti = Is; Is = Id; Id = ti;
            }
            SPM(25);
            // values: Is holds the merged points; the free buffer receives each one's interval value as a
            // code j << 24 | idx (the value is q j + V_{k+1}[idx], recomputed bit-identically; -1: +inf)
            auto* const VAL = Id;
            auto dec = [&](int c) -> double { return c < 0 ? INFINITY : fma(q, (double)(c >> 24), Vk[c & 0xFFFFFF]); };
            const int per = (Mc + NT - 1) / NT;
            const int p0 = min(Mc, tid * per), p1 = min(Mc, p0 + per);
            int cnt[MU];
#pragma unroll
            for (int j = 0; j < MU; ++j) cnt[j] = 0;
            for (int p = p0; p < p1; ++p) {
                const int u = uof(Is[p]);
#pragma unroll
                for (int j = 0; j < MU; ++j) cnt[j] += (j == u) ? 1 : 0;
            }
            block_excl_scan_vec<NT, MU>(cnt, NU, Sb.xr, tid);     // points of each list before the chunk
            double cur[MU];
            int cc[MU];
#pragma unroll
            for (int j = 0; j < MU; ++j) {
                const int idx = Sb.rng[j] + cnt[j] - 1;   // (j < NU: rng is defined)
                const bool ok = j < NU && cnt[j] >= 1 && idx < m;
                cur[j] = ok ? fma(q, (double)j, Vk[idx]) : INFINITY;
                cc[j] = ok ? (j << 24) | idx : -1;
            }
            for (int p = p0; p < p1; ++p) {
                const int id = Is[p], u = uof(id), i = id & 0xFFFFFF;
                const double v = i < m ? fma(q, (double)u, Vk[i]) : INFINITY;
                double best = INFINITY;
                int bc = -1;
#pragma unroll
                for (int j = 0; j < MU; ++j) {
                    if (j == u) { cur[j] = v; cc[j] = i < m ? id : -1; }
                    if (cur[j] < best) { best = cur[j]; bc = cc[j]; }
                }
                VAL[p] = bc;
            }
            __syncthreads();
            SPM(26);
            // intervals of [dl, dh]: t = 0 starts at dl (the value of the last merged point <= dl),
            // t >= 1 at merged point jl + t - 1; zero-width ones dropped, the L_k + V_k > U pruning
            // applied, equal neighbours merged
            const int T = Mc - jl + 1;
            const int pt = (T + NT - 1) / NT;
            const int t0 = min(T, tid * pt), t1 = min(T, t0 + pt);
            auto start = [&](int t) { return t == 0 ? dl : t >= T ? dh : key(Is[jl + t - 1]); };
            auto raw = [&](int t) { return t == 0 ? (jl > 0 ? dec(VAL[jl - 1]) : INFINITY) : dec(VAL[jl + t - 1]); };
            // the pruning: min of the convex L_k over [a, b] is L at the clamp of its minimiser (+inf outside
            // its domain), by a table pointer that only moves right along the chunk
            const double xm = prune ? Sb.lt[3 * WAVE] : 0.0, lmin = prune ? Sb.lt[3 * WAVE + 1] : 0.0;
            const int ml = prune ? Sb.lc[k] : 0;
            int jt = 0;
            auto Lat = [&](double x) -> double {
                if (!(x >= Sb.lt[0] && x <= Sb.lt[ml - 1])) return INFINITY;
                while (jt + 1 < ml && Sb.lt[jt + 1] <= x) ++jt;
                return fma(x - Sb.lt[jt], Sb.lt[2 * WAVE + jt], Sb.lt[WAVE + jt]);
            };
            auto Lseek = [&](double x) {
                jt = 0;
                for (int st = w_st0(ml); st > 0; st >>= 1)
                    if (jt + st < ml && Sb.lt[jt + st] <= x) jt += st;
            };
            auto value = [&](int t, double a_, double b_) {
                double v = raw(t);
                if (prune && v < INFINITY) {
                    const double lb_ = xm < a_ ? Lat(a_) : xm > b_ ? Lat(b_) : lmin;
                    if (v + lb_ > U) v = INFINITY;
                }
                return v;
            };
            int lastnz = -1;
            {
                double s0 = start(t0);
                for (int t = t0; t < t1; ++t) {
                    const double s1 = start(t + 1);
                    if (s1 > s0) lastnz = t;
                    s0 = s1;
                }
            }
            const int prevnz = block_excl_max1<NT>(lastnz, Sb.red, tid);
            double pv0 = 0.0;                              // the previous nonzero interval's (pruned) value
            if (prevnz >= 0) {
                const double a_ = start(prevnz), b_ = start(prevnz + 1);
                if (prune) Lseek(a_);
                pv0 = value(prevnz, a_, b_);
            }
            auto walk = [&](auto&& emit) {                 // the chunk's kept intervals, in order
                bool have = prevnz >= 0;
                double pv = pv0;
                double s0 = start(t0);
                if (prune) Lseek(s0);
                for (int t = t0; t < t1; ++t) {
                    const double s1 = start(t + 1);
                    if (s1 > s0) {
                        const double v = value(t, s0, s1);
                        if (!have || v != pv) emit(s0, v);
                        have = true;
                        pv = v;
                    }
                    s0 = s1;
                }
            };
            int c = 0;
            walk([&](double, double) { ++c; });
            int o = block_excl_scan1<NT>(c, Sb.red + 16, tid, &tot);
            if (tot == 0) { res = fail; return; }          // (a zero-width domain)
            if (tot + 1 > NP_CAP || top + tot + 1 > Sb.pool_cap) { res = -3; return; }
            double* const OB = Sb.PB + top;
            double* const OV = Sb.PV + top;
            walk([&](double s_, double v_) { OB[o] = s_; OV[o] = v_; ++o; });
        };
        // the pool: V_{k+1}'s breakpoints (and values when they fit too), then the merge buffers when
        // they fit as well (ids i32 x 2; the free one then holds the values' codes)
        const bool lds_m = staged && 8 * (lds_v ? 2 : 1) * np + 8 * Mc + 32 <= Sb.spb;
        SPM(24);
        // (S <= 7, every tariff of the reference: 8 lists in registers; more: the workspace path)
        if (NU > 8) {
            stage(Bg, Vg, Sb.GIA, Sb.GIB, IntC<STEP_MAXU>{});
        } else if (lds_m) {
            int* const i0 = reinterpret_cast<int*>(Sb.sp + ((8 * (lds_v ? 2 : 1) * np + 15) & ~15));
            if (lds_v) stage(bs, bs + np, i0, i0 + Mc, IntC<8>{});
            else stage(bs, Vg, i0, i0 + Mc, IntC<8>{});
        } else if (staged) {
            stage(bs, Vg, Sb.GIA, Sb.GIB, IntC<8>{});
        } else {
            stage(Bg, Vg, Sb.GIA, Sb.GIB, IntC<8>{});
        }
        if (res != 1) return res;
        double* const OB = Sb.PB + top;
        if (tid == 0) { OB[tot] = dh; Sb.cnt[k] = tot; Sb.off[k] = top; }
        SPM(23);
#ifdef DRAGG_STEP_PROF
        if (tid == 0 && !feas_only) {
            X[14 * 8 + S_PAD] += (double)np; X[15 * 8 + S_PAD] = fmax(X[15 * 8 + S_PAD], (double)np);
            X[16 * 8 + S_PAD] += (8 * np > Sb.spb ? 1.0 : 0.0) + (16 * np + 8 * Mc + 32 > Sb.spb ? 1000.0 : 0.0);
            X[18 * 8 + S_PAD] += (double)Mc;
        }
#endif
        top += tot + 1;
        __syncthreads();
    }
#undef SPM
#ifdef DRAGG_STEP_PROF
    const unsigned long long rec_t0 = __builtin_amdgcn_s_memtime();
#endif
    // forward recovery: wave u evaluates duty u's successor (q u + V_{k+1}(x') by a 64-ary search of
    // V_{k+1}'s breakpoints), the cheapest wins, lowest duty on ties (the oracle's rule)
    double x = x0;
    for (int k = 0; k < H; ++k) {
        for (int u = wid; u < NU; u += NT / WAVE) {
            const double xn = fma(cA[k], x, fma(g, (double)u, cC[k]));
            const double qu = feas_only ? 0.0 : cq[k] * (double)u;
            double val = INFINITY;
            if (xn >= boxlo(k) && xn <= boxhi(k)) {
                if (k + 1 < H) {
                    const int m = Sb.cnt[k + 1];
                    const double* const B = Sb.PB + Sb.off[k + 1];
                    const double* const V = Sb.PV + Sb.off[k + 1];
                    if (xn >= B[0] && xn <= B[m]) {
                        // the count of breakpoints <= xn: B[lo_] <= xn, the count in (lo_, lo_ + n_]
                        int lo_ = 0, n_ = m + 1;
                        while (n_ > WAVE) {
                            const int st = (n_ + WAVE - 1) / WAVE;
                            const int j = lo_ + lane * st;
                            const int cnt_ = __popcll(__ballot(lane * st < n_ && B[j] <= xn));
                            const int nl = lo_ + (cnt_ - 1) * st;
                            n_ = min(st, lo_ + n_ - nl);
                            lo_ = nl;
                        }
                        const int a = lo_ + __popcll(__ballot(lane < n_ && B[lo_ + min(lane, n_ - 1)] <= xn));
                        val = fma(feas_only ? 0.0 : cq[k], (double)u, V[min(a - 1, m - 1)]);
                    }
                } else {
                    val = qu;
                }
            }
            if (lane == 0) Sb.xv[u] = val;
        }
        __syncthreads();
        double vm = INFINITY;
        int bu = -1;
        for (int u = 0; u < NU; ++u)
            if (Sb.xv[u] < vm) { vm = Sb.xv[u]; bu = u; }
        if (bu < 0) return fail;                           // (uniform: no duty keeps a schedule)
        x = fma(cA[k], x, fma(g, (double)bu, cC[k]));
        if (tid == 0) { X[k * 8 + sv] = (double)bu; X[k * 8 + sx] = x; }
        __syncthreads();
    }
#ifdef DRAGG_STEP_PROF
    if (tid == 0) X[13 * 8 + S_PAD] += (double)(__builtin_amdgcn_s_memtime() - rec_t0);
#endif
    return 1;
}

// The direct path is two launches.  DM_FRONT (the hot one, one block per home) runs the exact
// front DP with fronts of up to NF labels (NF_BOUND with the LP bound).  A home where it does not
// apply (front overflow -- stage-varying RL prices --, mixed-sign prices, a too-narrow feasible set,
// S != 6) is appended to a list in the workspace and left untouched (nothing of its hash written).
// DM_BUCKET, a persistent launch of SECOND_SLOTS blocks, then solves the listed homes: each chain
// by the same front DP where it applies; otherwise by the bucketed DP (dp_thermal, an
// approximation) whose schedule's cost then bounds an exact front DP with fronts of up to NF_BIG
// labels (its own back-pointer rows per block), which replaces that schedule by the optimum.  Only
// a chain that outgrows even NF_BIG keeps the bucketed schedule (int_path records it).  Keeping the
// bucketed DP and the big pass out of DM_FRONT keeps their registers and LDS out of the hot kernel.
enum DirectMode { DM_FRONT = 0, DM_BUCKET = 1, DM_NARROW = 2, DM_MID = 3 };

// list entries: home | BK_DONE / BK_OK | deferred chain << 30 (homes < 2^28)
constexpr int HOME_MASK = 0x0FFFFFFF;
constexpr int BK_OK = 1 << 28;           // the bucketed DP found a schedule (in the solution rows)
constexpr int BK_DONE = 1 << 29;         // the bucketed DP already ran for the deferred chain (mid -> big)
constexpr int BK_BEAM = (int)(1u << 31); // ... and that schedule is the beam pass's (diagnostic: int_path bit 17)
// step-function list entries (bit 31, the big list's BK_BEAM): a chain the hot launch handed straight over
// (a feasible set narrower than one duty step, dp_front -2), whose bucketed DP -- the upper bound of the
// step-function DP and its capacity escape's schedule -- the step-function launch runs itself
constexpr int BK_NEED = (int)(1u << 31);

template <bool EXPLICIT, int MODE, int NW = 1, int ILP = 1>
DEV void solve_direct(const KArgs& a, int home, double* smem, int slot, int first_chain, int eflags = 0) {
    constexpr bool SECOND = MODE == DM_BUCKET || MODE == DM_MID;   // the bucketed DP + an exact big-front pass
    constexpr int NT = NW * WAVE;
    const int lane = threadIdx.x;
    const int N = a.d.n_homes;
    const int H = a.d.horizon;
    char* const ws = reinterpret_cast<char*>(a.p.workspace);            // per-home rows
    char* const lw = a.lws ? a.lws : ws;                                 // lists, per-block scratch
    int* const list = reinterpret_cast<int*>(lw + defer_offset(N, H));     // [N] + length at [N]
    int* const nlist = a.nar ? a.nar : reinterpret_cast<int*>(lw + narrow_list_offset(N, H));   // -> DM_NARROW
    int* const blist = reinterpret_cast<int*>(lw + mid_list_offset(N, H));      // DM_MID -> DM_BUCKET
    Home h;
    LdsD D = MODE == DM_FRONT ? carve_front(smem, H) : carve_direct(smem, H, a.d.sub_steps);
    D.par = reinterpret_cast<uint16_t*>(ws) + (size_t)home * H * NB_CAP;
    // the stage-slot solution lives in the workspace too (after every home's back-pointers):
    // it is written once per chain and read by the cleanup, so LDS goes to the DP
    D.x = reinterpret_cast<double*>(ws + par_region_bytes(N, H)) + (size_t)home * 8 * H;
    Lds L = lp_view(D);
    Io io{a.vals, a.fc, N, home};
    Prof pf;
    pf.start(a.out.cycles != nullptr);
    if (prologue<EXPLICIT>(a, h, L, io, lane, NT, D.sc) == DRAGG_ST_ERR_MISSING) {
        if (lane == 0) {
            write_missing(a, home);
        }
        lag_finish(a, home);
        return;
    }
    derive(h);
    // temp_wh (the un-mixed one-step value, mpc_calc.py:336-340) differs from Tw_1 by a
    // constant Kc, so its bounds become a tightened box on Tw_1 (as in build()).
    double twlo0, twhi0;
    {
        const double rem1 = 1 - D.draw[1] / h.V;
        const double c0 = rem1 + (-rem1 * h.iRw) * 3600 * h.inv_w;
        const double d15 = D.draw[1] / h.V * TAP;
        const double d0 = d15 + ((-d15) * h.iRw) * 3600 * h.inv_w;
        const double Kc = (h.Tw0 + ((-h.Tw0) * h.iRw) * 3600 * h.inv_w) - c0 * h.Tw0 - d0;
        twlo0 = fmax(h.Twmin, h.Twmin - Kc);
        twhi0 = fmin(h.Twmax, h.Twmax - Kc);
    }
    int status = presolve_direct(h, D, twlo0, twhi0, lane) ? DRAGG_ST_INFEASIBLE : DRAGG_ST_OPTIMAL;
    // a named solver that raises on the MILP (int_mode fail): the reference's except branch sets
    // solved = False before any status exists, and cleanup_and_finish runs the fallback
    if (a.d.int_mode == DRAGG_INT_FAIL) status = DRAGG_ST_SOLVER_ERROR;
    double* const saved = D.sc + 20;                    // step inputs, for reload_home
    if (lane == 0) {
        saved[0] = h.t; saved[1] = h.counter; saved[2] = h.winter ? 1.0 : 0.0;
        saved[3] = h.T0; saved[4] = h.Tw0; saved[5] = h.E0; saved[6] = twlo0; saved[7] = twhi0;
    }
    __syncthreads();
    pf.mark(DRAGG_PH_SETUP);
    double obj = NAN;
    int int_path = 0;
    if (status == DRAGG_ST_OPTIMAL) {
        // chain 0: indoor air (mpc_calc.py:314-317), u = duty of the season's mode (:303-309);
        // chain 1: water heater given T (mpc_calc.py:330-332).  One DP instantiation for both.
        bool ok = true;
        // prices that change at more than a quarter of the stages (RL reward prices; a tariff
        // changes a few times a day) grow fronts past NF_BOUND at most homes (measured: 9,990 of
        // 10,000): the hot launch hands these homes to the second one right away, which prunes
        // with the LP bound.  (Pruning by bound at every tariff boundary too: -14 % latency of
        // the slowest homes over the first 48 steps of the bench, but +13 % time over all 96.)
        int changes = 0;                              // (every wave counts all stages)
        for (int k = lane & (WAVE - 1); k < H; k += WAVE) changes += (k > 0 && D.price[k] != D.price[k - 1]) ? 1 : 0;
        changes = dpp_isum(changes);
        const bool rl_prices = changes * 4 > H;
        const bool use_bound = rl_prices;
        if (MODE == DM_FRONT && a.force_steps) {
            if (lane == 0) nlist[atomicAdd(nlist + N, 1)] = home;
            return;
        }
        if (MODE == DM_FRONT && rl_prices) {
            if (lane == 0) list[atomicAdd(list + N, 1)] = home;
            return;
        }
        // (the second launch resumes a home at the chain the hot launch deferred: the indoor-air
        // chain's schedule is already in the global solution array when the tank chain deferred)
        for (int chain = first_chain; chain < 2 && ok; ++chain) {
            reload_home(h, a, home, saved);
            twlo0 = saved[6]; twhi0 = saved[7];
            for (int k = lane; k < H; k += NT) {
                const double wk = pow(h.gamma, (double)k) * D.price[k];
                if (chain == 0) {
                    D.cA[k] = h.aT;
                    D.cC[k] = D.oat[k + 1] * h.iR * 3600 * h.inv_c;
                    D.cq[k] = wk * h.Pact;
#if defined(DRAGG_FRONT_STATS) || defined(DRAGG_FRONT_STATS2) || defined(DRAGG_STAGE_PROF) || defined(DRAGG_STEP_PROF)
                    D.x[k * 8 + S_PAD] = 0.0;             // (the diagnostics' accumulators)
#endif
                    // the battery slots are read only for a battery home (objective, write_success), whose
                    // battery LP writes them all: the other homes skip the stores (1.5 KB per home-step)
                    if (h.batt) { D.x[k * 8 + S_CH] = 0.0; D.x[k * 8 + S_DIS] = 0.0; D.x[k * 8 + S_E] = 0.0; }
                } else {
                    const double df = D.draw[k + 1] / h.V, rem = 1 - df, d15 = df * TAP;
                    D.cA[k] = rem + (-rem * h.iRw) * 3600 * h.inv_w;
                    D.cC[k] = h.e * D.x[k * 8 + S_T] + (d15 + ((-d15) * h.iRw) * 3600 * h.inv_w);
                    D.cq[k] = wk * (h.S * h.Pw);
                }
            }
            __syncthreads();
            const bool c0 = chain == 0;
            const double g = c0 ? h.g : h.f, x0 = c0 ? h.T0 : h.Tw0;
            const double lo0 = c0 ? h.Tmin : twlo0, hi0 = c0 ? h.Tmax : twhi0;
            const double lo = c0 ? h.Tmin : h.Twmin, hi = c0 ? h.Tmax : h.Twmax;
            const int sx = c0 ? S_T : S_TW, sv = c0 ? S_U : S_W;
            // the exact front DP; the bucketed DP only where it does not apply (mixed-sign
            // prices, a feasible set narrower than one duty step, front overflow, S != 6)
            int r = -5;                                    // reason 5: the exact DP not run (S != 6)
            double2* const wg = reinterpret_cast<double2*>(ws + w_region_offset(N, H)) + (size_t)home * (H + 1) * WAVE;
            if constexpr (MODE == DM_NARROW) {
                // the exact step-function DP (any prices, any feasible sets)
                const NarrowLayout nl = narrow_layout(H, a.d.sub_steps, a.narrow_lds);
                char* const sb = reinterpret_cast<char*>(smem);
                double* const sw = reinterpret_cast<double*>(lw + narrow_region_offset(N, H) +
                                                             (size_t)slot * step_slot_bytes());
                int* const swi = reinterpret_cast<int*>(sw + 2 * (size_t)POOL_CAP);
                double2* const swr = reinterpret_cast<double2*>(swi + 2 * (size_t)MC_CAP);
                const StepBufs SB{sw, sw + POOL_CAP, swi, swi + MC_CAP, swr, swr + (size_t)LW_ROWS * WAVE,
                                  reinterpret_cast<int*>(sb + nl.off), reinterpret_cast<int*>(sb + nl.cnt),
                                  reinterpret_cast<int*>(sb + nl.wc), reinterpret_cast<int*>(sb + nl.lc),
                                  reinterpret_cast<int*>(sb + nl.red), reinterpret_cast<int*>(sb + nl.xr),
                                  reinterpret_cast<int*>(sb + nl.rng),
                                  reinterpret_cast<double*>(sb + nl.rl), reinterpret_cast<double*>(sb + nl.rh),
                                  reinterpret_cast<double*>(sb + nl.dlo), reinterpret_cast<double*>(sb + nl.dhi),
                                  reinterpret_cast<double*>(sb + nl.xv), reinterpret_cast<double*>(sb + nl.lt),
                                  sb + nl.sp, nl.spb, min(POOL_CAP, max(64, a.step_pool_cap)),
                                  a.step_work_cap > 0 ? a.step_work_cap : STEP_WORK_CAP};
                auto steps = [&](bool feas, bool cut, double U_ = INFINITY) {
                    return dp_steps<NT>(SB, D.cA, D.cC, D.cq, H, h.S, g, x0, lo0, hi0, lo, hi, D.x, sx, sv, lane, feas, cut, U_);
                };
                auto sched_cost = [&]() {                  // (every wave sums all stages)
                    double c = 0.0;
                    for (int k = lane & (WAVE - 1); k < H; k += WAVE) c += D.cq[k] * D.x[k * 8 + sv];
                    return dpp_sum(c);
                };
                // an upper bound on the chain's optimum: the bucketed schedule the mid / big launch left in the
                // solution rows; without one the feasibility pass (all duty costs 0: the feasible set as a few
                // intervals, microseconds) decides whether any schedule exists and gives one
                if (chain == first_chain && (eflags & BK_NEED)) {
                    // the bucketed schedule of a chain the hot launch handed over (what the mid launch computes
                    // for the chains it hands over), here on all NT threads (dp_thermal is bit-identical for any
                    // thread count)
                    const bool okb = dp_thermal<6>(h, D, lane, NT, g, x0, lo0, hi0, lo, hi, sx, sv);
                    eflags = BK_DONE | (okb ? BK_OK : 0);
                }
                double ub = (chain == first_chain && (eflags & BK_OK)) ? sched_cost() : INFINITY;
                // the bucketed schedule (x, u per stage) kept aside in the chain's battery slots (zero until
                // the battery LP, which runs after both chains): what stands in if the DP runs out of room
                const bool have_bk = ub < INFINITY;
                if (have_bk) {
                    for (int k = lane; k < H; k += NT) { D.x[k * 8 + S_CH] = D.x[k * 8 + sx]; D.x[k * 8 + S_DIS] = D.x[k * 8 + sv]; }
                    __syncthreads();
                }
#ifdef DRAGG_STEP_PROF
                unsigned long long pt = __builtin_amdgcn_s_memtime();
                auto pmark = [&](int slot_) {
                    const unsigned long long n_ = __builtin_amdgcn_s_memtime();
                    if (lane == 0 && slot_ < H) D.x[slot_ * 8 + S_PAD] += (double)(n_ - pt);
                    pt = n_;
                };
                if (lane == 0) D.x[19 * 8 + S_PAD] = ub;
#define PMARK(i) pmark(i)
#else
#define PMARK(i) do {} while (0)
#endif
                r = ub < INFINITY ? 1 : steps(true, false);
                PMARK(10);
                if (r == 1) {
                    if (!(ub < INFINITY)) ub = sched_cost();
                    double qabs = 0.0;
                    for (int k = lane & (WAVE - 1); k < H; k += WAVE) qabs += fabs(D.cq[k]) * h.S;
                    qabs = dpp_sum(qabs);
                    __syncthreads();
                    auto Umargin = [&](double u_) { return u_ + TOL_P * (1.0 + fabs(u_) + qabs); };
                    const double U = Umargin(ub);
                    lp_rows<NT>(SB, D.cA, D.cC, D.cq, H, h.S, g, x0, lo0, hi0, lo, hi, lane);
                    // A first try at a smaller bound: U1 = lb + STEP_U_FRAC (ub - lb), lb the LP relaxation.  The
                    // cut DP is exact whenever its bound is >= the optimum, and a schedule it returns costs >= the
                    // optimum, so one costing <= U1 IS the optimum; otherwise (U1 below the optimum: no schedule, or
                    // a dearer one) the DP runs again at U.  The work grows fast with the bound (the bench's narrow
                    // tanks: 2.4x the merge points at the bucketed schedule's cost, ~15 % above the optimum, than
                    // at the optimum), and the optimum lies 0.55-0.7 of the way from lb to that cost there.
                    const double lb = lp_bound(SB, H, lane);
                    bool first = false;
                    if (lb < ub) {
                        const double U1 = Umargin(lb + STEP_U_FRAC * (ub - lb));
                        if (U1 < U) {
                            lp_cut<NT>(SB, H, U1, lane);
                            PMARK(11);
                            first = steps(false, true, U1) == 1 && sched_cost() <= U1;
                            PMARK(12);
                            __syncthreads();
                        }
                    }
#ifdef DRAGG_STEP_PROF
                    if (lane == 0) { D.x[20 * 8 + S_PAD] = ub; if (first) D.x[17 * 8 + S_PAD] += 1e6; }
#endif
                    if (first) {
                        r = 1;
                    } else {
                        lp_cut<NT>(SB, H, U, lane);
#ifdef DRAGG_STEP_PROF
                        if (lane == 0) {
                            int ncut = 0;
                            for (int k = 1; k <= H; ++k) ncut += (SB.dlo[k] > -INFINITY) ? 1 : 0;
                            D.x[17 * 8 + S_PAD] += 100.0 * ncut;
                        }
#endif
                        PMARK(11);
                        r = steps(false, true, U);              // V_k on the cut domains, pruned by L_k + V_k <= U
                        PMARK(12);
                    }
                    if (r == -6) {                          // (rounding put the optimum outside a cut: uncut)
#ifdef DRAGG_STEP_PROF
                        if (lane == 0) D.x[17 * 8 + S_PAD] += 1.0;
#endif
                        r = steps(false, false);
                    }
                    if (r < 0) {
#ifdef DRAGG_STEP_PROF
                        if (lane == 0) D.x[17 * 8 + S_PAD] += 10.0;
#endif
                        // past the pool's capacity or the work bound: the bucketed schedule stands in (the mid /
                        // big launch's, a feasible schedule whose cost bounded the DP), else the feasibility
                        // pass's; flagged approximate (reason 6)
                        if (have_bk) {
                            for (int k = lane; k < H; k += NT) { D.x[k * 8 + sx] = D.x[k * 8 + S_CH]; D.x[k * 8 + sv] = D.x[k * 8 + S_DIS]; }
                            __syncthreads();
                            r = 1;
                        } else {
                            r = steps(true, false);
                        }
                        int_path |= (1 << chain) | (6 << (4 + 4 * chain));
                    }
                }
                if (have_bk) {
                    for (int k = lane; k < H; k += NT) { D.x[k * 8 + S_CH] = 0.0; D.x[k * 8 + S_DIS] = 0.0; }
                    __syncthreads();
                }
#undef PMARK
                ok = r == 1;
                if (!ok) int_path |= 1 << (13 + chain);
                continue;
            }
            // (RL prices: the indoor-air chain skips the regular front DP -- its fronts outgrow it -- for the
            // cell-bound path below; the tank chain's fronts stay small: it tries it first)
            if (h.S == 6 && !(SECOND && rl_prices && chain == 0)) {
                double* const wl = D.wl;
                // (a multi-wave second launch: the exchange area of its mid / big layout, past the
                // direct layout's arrays)
                char* const xch = MODE == DM_FRONT ? D.xch
                                : reinterpret_cast<char*>(smem) + (MODE == DM_MID ? mid_layout(H, a.d.sub_steps).xch
                                                                                  : big_layout(H, a.d.sub_steps).xch);
                const FrontBufs FB{D.lab, D.rmin, D.kb, D.cb, D.mh, D.kl, D.flo, D.fhi, D.cA, D.cC, D.cq, D.x, D.par,
                                   wg, wl, wl + WAVE, wl + 2 * WAVE, xch};
                if constexpr (MODE == DM_FRONT)
                    r = dp_front<6, NF_HOT, NF_HOT, NB_CAP, NTB_HOT, NW, false, ILP>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv,
                                                                                   use_bound);
                else
                    // (64 key / cost buckets, as in the hot launch: the RL tank chain's DP here, rotated A/B
                    // round 6: RL action -2.0 % against 192 buckets, 128: -0.6 %; the full day unchanged)
                    r = dp_front<6, NF, NF_BOUND, NB_CAP, NTB_HOT, NW>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, use_bound);
#ifdef DRAGG_FRONT_STATS2
                // diagnostic: the T chain's fronts when the bound is the optimum itself
                if (c0 && r == 1 && use_bound) {
                    double best = INFINITY;
                    dp_front<6, NF, NF_BOUND, NB_CAP, NTB, NW>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, use_bound, INFINITY, &best);
                    for (int k = lane; k < H; k += NT) D.x[k * 8 + S_PAD] = 0.0;
                    __syncthreads();
                    r = dp_front<6, NF, NF_BOUND, NB_CAP, NTB, NW>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, use_bound, best);
                }
#endif
            }
            if (r >= 0) {
                ok = r == 1;
            } else if (MODE == DM_FRONT) {                 // leave the home to a later launch
                // a feasible set narrower than one duty step (-2): no front DP takes the chain (the mid launch's
                // would return -2 again) and the exact step-function DP solves it; the mid launch would only run
                // the bucketed DP for that DP's bound, so the chain goes straight to the step-function launch,
                // which runs the bucketed DP itself (BK_NEED): one launch fewer on the chain's path (lag mode:
                // a lagging home's side pass is hot + step-function, not hot + mid + step-function)
                if (lane == 0) {
                    if (r == -2 && h.S == 6) nlist[atomicAdd(nlist + N, 1)] = home | (chain << 30) | BK_NEED;
                    else list[atomicAdd(list + N, 1)] = home | (chain << 30);
                }
                return;
            } else {
                pf.mark(DRAGG_PH_INTEGER);
                const BigLayout bl = MODE == DM_MID ? mid_layout(H, a.d.sub_steps) : big_layout(H, a.d.sub_steps);
                char* const sb = reinterpret_cast<char*>(smem);
                double* const wl = reinterpret_cast<double*>(sb + bl.wl);
                uint16_t* const bpar = MODE == DM_MID
                    ? reinterpret_cast<uint16_t*>(lw + mid_region_offset(N, H)) + (size_t)slot * H * NF_MID
                    : reinterpret_cast<uint16_t*>(lw + big_region_offset(N, H)) + (size_t)slot * H * NF_BIG;
                // RL prices: the cell bound of the indoor-air chain (cell_kernel's rows of this home, before the
                // mid launch); the tank chain keeps the LP bound (its fronts stay small under RL prices)
                uint16_t* const cg = reinterpret_cast<uint16_t*>(ws + cell_region_offset(N, H)) + (size_t)home * (H + 1) * CELL_STRIDE;
                double c_lo = 0.0, c_inv = 0.0;
                const bool have_cells = SECOND && rl_prices && h.S == 6 && chain == 0 && a.d.n_rp > 1 && cell_rows_valid(cg);
                if (have_cells) cell_grid(fmin(lo0, lo), fmax(hi0, hi), c_lo, c_inv);
                const float c_off = have_cells ? cell_off(cg) : 0.0f, c_sc = have_cells ? cell_sc(cg) : 0.0f;
                const FrontBufs FB{reinterpret_cast<double2*>(sb + bl.fa), reinterpret_cast<double2*>(sb + bl.fb),
                                   reinterpret_cast<unsigned long long*>(sb + bl.kb),
                                   reinterpret_cast<unsigned long long*>(sb + bl.cb),
                                   reinterpret_cast<unsigned*>(sb + bl.mh), reinterpret_cast<unsigned*>(sb + bl.kl),
                                   reinterpret_cast<unsigned*>(sb + bl.flo), reinterpret_cast<unsigned*>(sb + bl.fhi),
                                   D.cA, D.cC, D.cq, D.x, bpar, wg, wl, wl + WAVE, wl + 2 * WAVE,
                                   sb + bl.xch, cg, c_lo, c_inv, c_off, c_sc};
                // a chain the mid launch handed over: its upper-bound schedule (the beam's or the bucketed
                // DP's) is in the solution rows already (the mid pass overflowed without writing them),
                // only the big pass is left
                bool beam_ub = false;
                if (have_cells) int_path |= 1 << 16;       // (diagnostic bits 16-18: cell bound, beam bound, big launch)
                if (MODE == DM_BUCKET) int_path |= 1 << 18;
                if (SECOND && chain == first_chain && (eflags & BK_DONE)) {
                    ok = (eflags & BK_OK) != 0;
                    beam_ub = (eflags & BK_BEAM) != 0;
                } else {
                    // the upper bound's schedule: under RL prices the beam pass (fronts cut to the BEAM_K
                    // labels of least cost + cell bound), else / failing that the bucketed DP
                    int rb = -1;
                    if constexpr (MODE == DM_MID) {
                        if (have_cells) {
                            __syncthreads();
                            rb = dp_front<6, NF_MID, NF_MID, NF_MID, NTB_MID, NW, true>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx,
                                                                                    sv, false, INFINITY, nullptr, BEAM_K);
                        }
                    }
                    ok = rb == 1;
                    beam_ub = ok;
                    if (!ok)
                        ok = h.S == 6 ? dp_thermal<6>(h, D, lane, NT, g, x0, lo0, hi0, lo, hi, sx, sv)
                                      : dp_thermal<0>(h, D, lane, NT, g, x0, lo0, hi0, lo, hi, sx, sv);
                }
                if (beam_ub) int_path |= 1 << 17;
                pf.mark(DRAGG_PH_ITER);                   // (round: the bucketed DP / the beam)
                int r2 = r;
                // the big pass, except for a feasible set narrower than one duty step (no
                // dominance there: its fronts outgrow any capacity, measured)
                if (h.S == 6 && r != -2) {
                    // the exact pass with big fronts, bounded by the schedule's cost
                    double ub = INFINITY;
                    if (ok) {                              // (every wave sums all stages)
                        double c = 0.0;
                        for (int k = lane & (WAVE - 1); k < H; k += WAVE) c += D.cq[k] * D.x[k * 8 + sv];
                        ub = dpp_sum(c);
                    }
                    __syncthreads();
                    // keeps the schedule in D.x unless it finds (and writes) the optimum
                    auto cell_pass = [&](double U) {
                        if constexpr (MODE == DM_MID)
                            return dp_front<6, NF_MID, NF_MID, NF_MID, NTB_MID, NW, true>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, true, U);
                        else
                            return dp_front<6, NF_BIG, NF_BIG, NF_BIG, NTB_BIG, NW, true>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, true, U);
                    };
                    if (have_cells) {
                        r2 = cell_pass(ub);
                        // past the capacity at the schedule's cost (its slack over the optimum lets too many
                        // labels through): bisection on the bound between the cell bound at x0 and that cost.
                        // A pass at U >= the optimum returns the optimum (every label of an optimal schedule
                        // passes cost + bound <= U); one below it finds no schedule (0)
                        if (r2 == -3 && ok) {
                            double lo_u = INFINITY;
                            {
                                const int u = lane & (WAVE - 1);
                                double v = INFINITY;
                                if (u <= 6) {
                                    const double x1 = fma(D.cA[0], x0, fma(g, (double)u, D.cC[0]));
                                    const double tl = lo0 - TOL_P * (1 + fabs(lo0)), th = hi0 + TOL_P * (1 + fabs(hi0));
                                    if (x1 >= tl && x1 <= th)
                                        v = fma(D.cq[0], (double)u,
                                                (double)cell_dec(cg[CELL_STRIDE + min(NCELL - 1, max(0, (int)floor((x1 - c_lo) * c_inv)))],
                                                                 c_off, c_sc));
                                }
                                lo_u = dpp_reduce(v, [](double a_, double b_) { return fmin(a_, b_); });
                            }
                            double hi_u = ub;
                            for (int tr = 0; tr < CELL_TRIES && r2 == -3 && lo_u < hi_u; ++tr) {
                                const double U = 0.5 * (lo_u + hi_u);
                                if (!(U > lo_u && U < hi_u)) break;
                                __syncthreads();
                                r2 = cell_pass(U);
                                if (r2 == 0) { lo_u = U; r2 = -3; }       // the optimum is above U
                                else if (r2 == -3) hi_u = U;              // still too many labels
                            }
                        }
                    } else if constexpr (MODE == DM_MID) {
                        r2 = dp_front<6, NF_MID, NF_MID, NF_MID, NTB_MID, NW>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, true, ub);
                    } else {
                        r2 = dp_front<6, NF_BIG, NF_BIG, NF_BIG, NTB_BIG, NW>(FB, H, lane, g, x0, lo0, hi0, lo, hi, sx, sv, true, ub);
                    }
                    pf.mark(DRAGG_PH_POLISH);             // (round: the mid / big exact pass)
                    if (MODE == DM_MID && r2 == -3) {         // past NF_MID: the big launch's 2,048-label fronts
                        // (an RL-priced chain went straight to the bucketed DP: the big launch reuses
                        // its schedule; other chains ran the regular front DP first and start over)
                        if (lane == 0)
                            blist[atomicAdd(blist + N, 1)] = home | (chain << 30) |
                                                             (rl_prices ? BK_DONE | (ok ? BK_OK : 0) | (beam_ub ? BK_BEAM : 0) : 0);
                        return;
                    }
                    if (r2 == 1) ok = true;
                    else if (r2 == 0 && !ok) ok = false;      // exact: no integer schedule
                    else if (r2 == 0) r2 = -4;                // bound inconsistent with the schedule: keep it
                }
                // no exact pass took the chain (a feasible set narrower than one duty step, mixed-sign
                // prices without a usable bound, a front past the big launch's capacity, S != 6): the
                // exact step-function DP of DM_NARROW solves it, with the bucketed schedule's cost as
                // its bound (BK_OK) -- or, where the bucketed DP found none, decides that no schedule exists
                // Exception (measured): an RL-priced chain past the big launch's 2,048 labels keeps its bucketed
                // schedule unless DRAGG_FLAG_EXACT is set -- under a price that changes at every stage the
                // step-function DP's value functions explode (the bench's smooth-price action: 776 ms with
                // it against 30 ms without); int_path records the chain (reason 3)
                if (MODE == DM_BUCKET && r2 == -3 && rl_prices && ok && !(a.d.flags & DRAGG_FLAG_EXACT)) {
                    int_path |= (1 << chain) | (3 << (4 + 4 * chain));
                } else if (r2 < 0) {
                    if (lane == 0) nlist[atomicAdd(nlist + N, 1)] = home | (chain << 30) | BK_DONE | (ok ? BK_OK : 0);
                    return;
                }
            }
            if (!ok) int_path |= 1 << (13 + chain);        // ROUND_FAIL decided by this chain
        }
        pf.mark(DRAGG_PH_INTEGER);
        reload_home(h, a, home, saved);
        if (!ok) status = DRAGG_ST_ROUND_FAIL;
        if (ok && h.batt) {
            for (int k = lane; k < H; k += NT) D.cq[k] = pow(h.gamma, (double)k) * D.price[k] * h.S;
            __syncthreads();
            bool bok = true;
            if (lane < WAVE) bok = battery_lp(h, D, lane);
            if (lane == 0) D.sc[31] = bok ? 1.0 : 0.0;
            __syncthreads();
            if (D.sc[31] == 0.0) status = DRAGG_ST_INFEASIBLE;
            __syncthreads();
        }
        pf.mark(DRAGG_PH_BATTERY);
        if (status == DRAGG_ST_OPTIMAL) obj = objective(h, L, lane, NT, D.sc);
    }
    if (status == DRAGG_ST_OPTIMAL) {
        write_success(h, L, io, lane, NT);
    } else if (lane == 0) {
        status = write_fallback(h, L, io, status);
    }
    if (lane == 0) {
        a.out.status[home] = status;
        a.out.iters[home] = 0;
        a.out.obj[home] = obj;
        a.out.relax_obj[home] = NAN;
        if (a.out.int_path)
            a.out.int_path[home] = int_path | (MODE != DM_FRONT ? (1 << 12) : 0) | (MODE == DM_NARROW ? (1 << 15) : 0);
    }
    if (a.out.hist && lane == 0)      // lane 0 wrote every vals field of this home
        for (int k = 0; k < DRAGG_NVAL; ++k) a.out.hist[(size_t)k * N + home] = io.v(k);
    pf.mark(DRAGG_PH_WRITE);
    if (pf.on && lane == 0)        // (the factor / check slots: the cell kernel's, int_mode round)
        for (int k = 0; k < DRAGG_NPHASE; ++k)
            if (k != DRAGG_PH_FACTOR && k != DRAGG_PH_CHECK) a.out.cycles[(size_t)k * N + home] = (int64_t)pf.acc[k];
    lag_finish(a, home);
}

template <bool EXPLICIT, int MODE, int NW = 1, int ILP = 1>
__global__ __launch_bounds__(WAVE * NW, MODE == DM_FRONT ? (ILP > 1 ? 2 : 3) : MODE == DM_NARROW ? 1 : 2) void mpc_direct_kernel(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    char* const ws = a.lws ? a.lws : reinterpret_cast<char*>(a.p.workspace);
    const int N = a.d.n_homes, H = a.d.horizon;
    __shared__ int take;
    if constexpr (MODE == DM_FRONT) {           // (the side pass's hot launch: side_front_kernel)
        const int home = blockIdx.x;
        if (home >= N) return;
        if (a.clk) {
            // lag mode, main pass: a home whose previous step is not complete yet goes to the side pass
            if (threadIdx.x == 0) take = __hip_atomic_load(a.clk + home, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            const int c = take;
            if ((c & ~LAG_SIDE) != a.t) {
                if (threadIdx.x == 0) a.skip[atomicAdd(a.skip + N, 1)] = home;
                return;
            }
            if (c & LAG_SIDE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the side pass's rows
        }
        solve_direct<EXPLICIT, MODE, NW, ILP>(a, home, smem, 0, 0);
        return;
    }
    // persistent: block b solves listed home b first, then takes the next ones off a shared counter
    // (dynamic: a block that drew short homes takes more; measured on the RL workload: 38.2 -> 34.0
    // ms per action against a static stride), each with its own scratch rows in the workspace (slot
    // b); blocks past the list's length leave at once, every block reaches its end and exits
    const size_t lo = MODE == DM_MID ? defer_offset(N, H) : MODE == DM_BUCKET ? mid_list_offset(N, H)
                    : narrow_list_offset(N, H);
    // (both passes' DM_NARROW in lag mode: the step's own list)
    int* const list = (MODE == DM_NARROW && a.nar) ? a.nar : reinterpret_cast<int*>(ws + lo);
    const int cnt = min(list[N], N);
    for (int j = blockIdx.x; j < cnt;) {
        const int e = list[j];                      // home | flags | deferred chain << 30
        const int home = e & HOME_MASK, chain = (e >> 30) & 1;
        if (home < N) solve_direct<EXPLICIT, MODE, NW>(a, home, smem, blockIdx.x, chain, e & (BK_DONE | BK_OK | BK_BEAM));
        __syncthreads();
        if (threadIdx.x == 0) take = (int)gridDim.x + atomicAdd(list + N + 1, 1);
        __syncthreads();
        j = take;
    }
}

// The cell bound rows of the indoor-air chain of every RL-priced home the hot launch deferred (its list,
// before the mid launch reads it): the step's inputs as the solve derives them (prologue), the chain's
// coefficients, cell_rows.  Blocks take the list entries by a static stride (the list's take counter is
// the mid launch's).
constexpr int NT_CELL = 256;
constexpr int CELL_BLOCKS = 1024;           // blocks of the cell kernel (4 per CU)
constexpr int CELL_ROW = NCELL + 16;        // an LDS row of cell_rows (the pair minima take NCELL + 1)
__host__ __device__ inline int cell_lds_bytes(int H) { return (front_layout(H).bytes + 15) / 16 * 16 + 2 * CELL_ROW * 4; }
__global__ __launch_bounds__(NT_CELL, 4) void cell_kernel(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = a.d.n_homes, H = a.d.horizon;
    const int tid = threadIdx.x;
    char* const ws = reinterpret_cast<char*>(a.p.workspace);
    char* const lw = a.lws ? a.lws : ws;
    const int* const list = reinterpret_cast<const int*>(lw + defer_offset(N, H));
    const int cnt = min(list[N], N);
    float* const r0 = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + (front_layout(H).bytes + 15) / 16 * 16);
    float* const r1 = r0 + CELL_ROW;
    for (int j = blockIdx.x; j < cnt; j += gridDim.x) {
        const int e = list[j];
        const int home = e & HOME_MASK;
        if (home >= N || ((e >> 30) & 1) != 0) continue;        // (uniform; chain 0 entries only)
        Home h;
        LdsD D = carve_front(smem, H);
        Lds L = lp_view(D);
        Io io{a.vals, a.fc, N, home};
        Prof pf;
        pf.start(a.out.cycles != nullptr);
        __syncthreads();
        if (prologue<false>(a, h, L, io, tid, NT_CELL, D.sc) == DRAGG_ST_ERR_MISSING) continue;
        derive(h);
        int changes = 0;
        for (int k = tid & (WAVE - 1); k < H; k += WAVE) changes += (k > 0 && D.price[k] != D.price[k - 1]) ? 1 : 0;
        changes = dpp_isum(changes);
        if (!(changes * 4 > H) || h.S != 6) continue;             // not RL-priced: the mid launch's regular path
        for (int k = tid; k < H; k += NT_CELL) {                  // the indoor-air chain (solve_direct, chain 0)
            const double wk = pow(h.gamma, (double)k) * D.price[k];
            D.cA[k] = h.aT;
            D.cC[k] = D.oat[k + 1] * h.iR * 3600 * h.inv_c;
            D.cq[k] = wk * h.Pact;
        }
        __syncthreads();
        double c_lo, c_inv;
        cell_grid(h.Tmin, h.Tmax, c_lo, c_inv);
        uint16_t* const cg = reinterpret_cast<uint16_t*>(ws + cell_region_offset(N, H)) + (size_t)home * (H + 1) * CELL_STRIDE;
        pf.mark(DRAGG_PH_CHECK);                   // (diagnostic: the prologue, in the check slot)
        const bool ok = cell_rows<NT_CELL, 6>(cg, r0, r1, D.cA, D.cC, D.cq, H, 6, h.g, h.Tmin, h.Tmax, h.Tmin, h.Tmax,
                                              c_lo, c_inv, tid);
        pf.mark(DRAGG_PH_FACTOR);                  // (diagnostic: the cell rows, in the factor slot)
        if (tid == 0) {
            reinterpret_cast<float*>(cg)[0] = ok ? 1.0f : 0.0f;
            if (pf.on) {
                a.out.cycles[(size_t)DRAGG_PH_CHECK * N + home] = (int64_t)pf.acc[DRAGG_PH_CHECK];
                a.out.cycles[(size_t)DRAGG_PH_FACTOR * N + home] = (int64_t)pf.acc[DRAGG_PH_FACTOR];
            }
        }
    }
}

// lag mode, the side pass's hot launch: a persistent consumer of the homes the main pass skipped (its own
// kernel, so that the main pass's hot kernel keeps its registers: one inlined solve, no list loop; two chunks
// per front-DP pass and two waves per SIMD: it holds a lagging home or two, whose latency is its time)
__global__ __launch_bounds__(WAVE, 2) void side_front_kernel(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = a.d.n_homes;
    int* const list = a.hot_list;
    const int cnt = min(list[N], N);
    __shared__ int take;
    for (int j = blockIdx.x; j < cnt;) {
        const int home = list[j] & HOME_MASK;
        if (home < N) solve_direct<false, DM_FRONT, 1, 3>(a, home, smem, blockIdx.x, 0, 0);
        __syncthreads();
        if (threadIdx.x == 0) take = (int)gridDim.x + atomicAdd(list + N + 1, 1);
        __syncthreads();
        j = take;
    }
}

// the device lists' (length, take counter) pairs to zero before a step's launches (NULL: none)
__global__ void reset_lists_kernel(int* a, int* b, int* c, int* d, int* e) {
    const int i = threadIdx.x;
    int* const p = i < 2 ? a : i < 4 ? b : i < 6 ? c : i < 8 ? d : i < 10 ? e : nullptr;
    if (p) p[i & 1] = 0;
}

// lag mode: every home's clock = t (the state the host holds: every step before t complete)
__global__ void lag_reset_kernel(int* clk, int N, int t) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) clk[i] = t;
}

// collect_data's three sums (aggregator.py:728-755) in one 1024-thread block: 16 waves of
// independent loads (a step's sums are a latency-bound 240 KB read at 10k homes), then a wave
// reduction and a pass over the 16 wave partials
constexpr int AGG_NT = 1024;
DEV void agg_sums(const double* vals, int N, double* out3) {
    __shared__ double red[3][AGG_NT / WAVE];
    const double* p0 = vals + (size_t)DRAGG_K_P_GRID * N;
    const double* p1 = vals + (size_t)DRAGG_K_FORECAST_P_GRID * N;
    const double* p2 = vals + (size_t)DRAGG_K_COST * N;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int i = threadIdx.x; i < N; i += AGG_NT) {   // NaN (absent field) propagates
        s0 += p0[i];
        s1 += p1[i];
        s2 += p2[i];
    }
    s0 = dpp_sum(s0); s1 = dpp_sum(s1); s2 = dpp_sum(s2);
    const int w = threadIdx.x / WAVE;
    if ((threadIdx.x & (WAVE - 1)) == 0) { red[0][w] = s0; red[1][w] = s1; red[2][w] = s2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double t = 0.0;
        for (int i = 0; i < AGG_NT / WAVE; ++i) t += red[threadIdx.x][i];
        out3[threadIdx.x] = t;
    }
}
__global__ __launch_bounds__(AGG_NT) void aggregate_kernel(const double* vals, int N, double* out3) {
    agg_sums(vals, N, out3);
}
// the sums of many steps at once, from the history rows the steps wrote ([rows][NVAL][N]): block r
// sums row r exactly as aggregate_kernel sums vals (the same code: bit-identical)
__global__ __launch_bounds__(AGG_NT) void aggregate_rows_kernel(const double* rows, int N, double* out) {
    agg_sums(rows + (size_t)blockIdx.x * DRAGG_NVAL * N, N, out + (size_t)blockIdx.x * 3);
}

__global__ void noise_kernel(int N, int H, uint64_t seed, int off, int stride, int t, double* out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int pairs = (H + 1) / 2;
    if (idx >= N * pairs) return;
    const int home = idx % N, pr = idx / N;
    double z0, z1;
    normal_pair(seed, off + home * stride, t, pr, &z0, &z1);
    out[(size_t)(2 * pr) * N + home] = z0;
    if (2 * pr + 1 < H) out[(size_t)(2 * pr + 1) * N + home] = z1;
}

bool direct_mode(const dragg_mpc_dims* d) { return d->int_mode == DRAGG_INT_ROUND || d->int_mode == DRAGG_INT_FAIL; }

size_t workspace_bytes(const dragg_mpc_dims* d) {
    // direct: [N][H][NB_CAP] u16 back-pointers, [N][8H] f64 solutions, the [N + 1] i32 list of
    // deferred homes, [N][H+1][64] LP cost-to-go rows, the second launch's [SECOND_SLOTS][H][NF_BIG]
    // u16 back-pointers; round_lp: the back-pointers of its front DP
    if (d->int_mode == DRAGG_INT_ROUND_LP) return par_region_bytes(d->n_homes, d->horizon);
    return direct_mode(d) ? direct_workspace_bytes(d->n_homes, d->horizon, d->n_rp > 1) : 0;
}

// per home, the hot launch's (int_mode round: DM_FRONT)
size_t kernel_lds_bytes(const dragg_mpc_dims* d) {
    return direct_mode(d) ? (size_t)front_layout(d->horizon).bytes : (size_t)lds_doubles(d->horizon) * 8;
}

int check_dims(const dragg_mpc_dims* d) {
    if (!d || d->n_homes < 0 || d->horizon < 1 || d->sub_steps < 1 || d->dt < 1) return DRAGG_E_ARG;
    if (d->n_homes > HOME_MASK) return DRAGG_E_ARG;                   // the deferred lists' home field
    if (d->int_mode < DRAGG_INT_ROUND || d->int_mode > DRAGG_INT_FAIL) return DRAGG_E_ARG;
    if (d->flags & ~DRAGG_FLAG_EXACT) return DRAGG_E_ARG;
    if (direct_mode(d) && d->sub_steps > 15) return DRAGG_E_ARG;     // 4-bit duty in the DP record
    if (direct_mode(d) && !direct_fits(d->horizon)) return DRAGG_E_HORIZON;
    if (kernel_lds_bytes(d) > 160 * 1024 - 256) return DRAGG_E_HORIZON;
    if (direct_mode(d) && big_layout(d->horizon, d->sub_steps).bytes > 160 * 1024 - 256) return DRAGG_E_HORIZON;
    if (direct_mode(d) && narrow_layout(d->horizon, d->sub_steps).bytes > 160 * 1024 - 256) return DRAGG_E_HORIZON;
    return DRAGG_OK;
}

// the dynamic LDS limit the launches raise: the 160 KB of a CU less room for the kernels' static
// LDS (the persistent launches' take slot)
constexpr int LDS_DYN_MAX = 160 * 1024 - 256;

template <typename K>
int launch_kernel(K kern, int& attr_state, const KArgs& a, int blocks, int nt, size_t lds, hipStream_t s) {
    if (!attr_state) {
        if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DYN_MAX) !=
            hipSuccess)
            return DRAGG_E_LDS;
        attr_state = 1;
    }
    if (a.d.n_homes == 0) return DRAGG_OK;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(nt), lds, s, a);
    return hipGetLastError() == hipSuccess ? DRAGG_OK : DRAGG_E_HIP;
}

// hipFuncSetAttribute is per device: the attribute state is kept per device (a process driving
// several GPUs sets it once on each)
constexpr int MAX_DEV = 64;

// Diagnostic knobs, read once per process (not on every step): DRAGG_WAVES_PER_HOME=1|2|4 forces
// the hot launch's waves per home (A/B runs); DRAGG_FORCE_STEP_DP=1 sends every home's chains to
// the step-function DP (DM_NARROW); DRAGG_STEP_POOL_CAP / DRAGG_STEP_WORK_CAP shrink that DP's pool
// and work bound (tests of its capacity path).  Unset: one wave per home, the regular launch order.  (Round 4
// measured and removed a prediction of the narrow homes before the hot launch with their step-function DP
// on a high-priority side stream beside it: 2.81 against 2.29 ms over the full day -- the side solves
// outlast the hot launch and take CUs from it -- and ~0.1 ms of prediction per step at 1,250 homes.)
struct Knobs {
    int waves = 1;
    int force_steps = 0;
    int step_pool_cap = POOL_CAP;     // DRAGG_STEP_POOL_CAP: a smaller step-function DP pool (tests of its
    long long step_work_cap = 0;      //   capacity path); DRAGG_STEP_WORK_CAP: its work bound (0: default)
    int side_grid[4] = {0, 0, 0, 0};  // DRAGG_SIDE_GRID=hot,mid,big,narrow: the side pass's blocks (A/B)
    int ilp = 0;                      // DRAGG_HOT_ILP=1|2: the hot launch's chunks per pass (0: by N, hot_ilp)
    int narrow_lds = 0;               // DRAGG_NARROW_LDS_KB=n: the step-function launch's LDS per block (A/B)
};
Knobs read_knobs() {
    Knobs r;
    const char* w = getenv("DRAGG_WAVES_PER_HOME");
    if (w && (w[0] == '1' || w[0] == '2' || w[0] == '4') && w[1] == 0) r.waves = w[0] - '0';
    const char* f = getenv("DRAGG_FORCE_STEP_DP");
    r.force_steps = (f && f[0] == '1') ? 1 : 0;
    const char* pc = getenv("DRAGG_STEP_POOL_CAP");
    if (pc && atoi(pc) > 0) r.step_pool_cap = atoi(pc);
    const char* wc = getenv("DRAGG_STEP_WORK_CAP");
    if (wc && atoll(wc) > 0) r.step_work_cap = atoll(wc);
    const char* sg = getenv("DRAGG_SIDE_GRID");
    if (sg) sscanf(sg, "%d,%d,%d,%d", &r.side_grid[0], &r.side_grid[1], &r.side_grid[2], &r.side_grid[3]);
    const char* nk = getenv("DRAGG_NARROW_LDS_KB");
    if (nk && atoi(nk) > 0) r.narrow_lds = min(atoi(nk), 159) * 1024;
    const char* il = getenv("DRAGG_HOT_ILP");
    if (il && (il[0] == '1' || il[0] == '2') && il[1] == 0) r.ilp = il[0] - '0';
    return r;
}
Knobs g_knobs = read_knobs();          // at library load; again only on dragg_mpc_reload_knobs()
const Knobs& knobs() { return g_knobs; }

// Waves per home of the hot launch: one (measured at 1,250 homes, the 8-GPU shard of the bench:
// 0.495 / 0.53 / 0.80 ms per step at 1 / 2 / 4 waves per home -- a stage's fixed latency (ranges,
// scans, barriers) dominates its passes at these front sizes, so extra waves only add barriers);
// DRAGG_WAVES_PER_HOME forces 2 or 4 (bit-identical results).
int hot_waves() { return knobs().waves; }

// Chunks per front-DP pass of the one-wave hot launch: two when the homes fit in two waves per SIMD
// (N <= 8 per CU: the launch then lasts as long as its slowest home, whose LDS round trips the second
// chunk overlaps), else one (three waves per SIMD hide them; the second chunk's registers would cost one)
int hot_ilp(int dev, int N) {
    if (knobs().ilp) return knobs().ilp;
    static int cus[MAX_DEV] = {};
    if (!cus[dev]) {
        hipDeviceProp_t prop{};
        cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }
    return N <= 8 * cus[dev] ? 2 : 1;
}

// blocks of the persistent mid launch: as many as the GPU holds at once at its LDS (<= MID_SLOTS_MAX),
// cached per (device, LDS bytes): a batch with another horizon gets its own occupancy
template <bool EXPLICIT>
int mid_slots(int dev, int H, int S) {
    constexpr int NC = 8;
    static int cache_lds[MAX_DEV][NC] = {};
    static int cache_slots[MAX_DEV][NC] = {};
    const int lds = mid_layout(H, S).bytes;
    for (int i = 0; i < NC; ++i)
        if (cache_lds[dev][i] == lds) return cache_slots[dev][i];
    hipDeviceProp_t prop{};
    int per_cu = 0;
    const void* k = (const void*)mpc_direct_kernel<EXPLICIT, DM_MID, NW_MID>;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
        hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DYN_MAX) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, NW_MID * WAVE, (size_t)lds) != hipSuccess)
        return SECOND_SLOTS;
    const int slots = max(1, min(MID_SLOTS_MAX, per_cu * prop.multiProcessorCount));
    for (int i = 0; i < NC; ++i)
        if (cache_lds[dev][i] == 0) { cache_lds[dev][i] = lds; cache_slots[dev][i] = slots; break; }
    return slots;
}

template <bool EXPLICIT>
int launch(const KArgs& a, hipStream_t s) {
    static int attr_dev[MAX_DEV][10] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return DRAGG_E_HIP;
    int* const attr = attr_dev[dev];
    const int N = a.d.n_homes;
    if (!direct_mode(&a.d)) return launch_kernel(mpc_home_kernel<EXPLICIT>, attr[0], a, N, 64, kernel_lds_bytes(&a.d), s);
    if (N == 0) return DRAGG_OK;
    // the deferred list starts empty (its length word), then the hot launch, then the second
    char* const wsb = reinterpret_cast<char*>(a.p.workspace);
    int* const len = reinterpret_cast<int*>(wsb + defer_offset(N, a.d.horizon)) + N;
    int* const nlen = reinterpret_cast<int*>(wsb + narrow_list_offset(N, a.d.horizon)) + N;
    int* const blen = reinterpret_cast<int*>(wsb + mid_list_offset(N, a.d.horizon)) + N;
    KArgs b = a;
    b.force_steps = knobs().force_steps;
    b.step_pool_cap = knobs().step_pool_cap;
    b.step_work_cap = knobs().step_work_cap;
    b.narrow_lds = knobs().narrow_lds;
    // each list's length and the persistent launch's take counter after it, in one tiny launch
    // (three 8-byte memsets cost three fills: ~13 us of a 0.49 ms step at 1,250 homes)
    hipLaunchKernelGGL(reset_lists_kernel, dim3(1), dim3(WAVE), 0, s, len, nlen, blen, nullptr, nullptr);
    if (hipGetLastError() != hipSuccess) return DRAGG_E_HIP;
    const size_t lds = kernel_lds_bytes(&a.d);
    const int nw = hot_waves();

    const int rc = nw == 4 ? launch_kernel(mpc_direct_kernel<EXPLICIT, DM_FRONT, 4>, attr[4], b, N, 4 * WAVE, lds, s)
                 : nw == 2 ? launch_kernel(mpc_direct_kernel<EXPLICIT, DM_FRONT, 2>, attr[3], b, N, 2 * WAVE, lds, s)
                 : hot_ilp(dev, N) == 2 ? launch_kernel(mpc_direct_kernel<EXPLICIT, DM_FRONT, 1, 2>, attr[8], b, N, WAVE, lds, s)
                                        : launch_kernel(mpc_direct_kernel<EXPLICIT, DM_FRONT, 1>, attr[1], b, N, WAVE, lds, s);
    if (rc) return rc;
    // RL prices possible (a reward-price list): the cell bound of the deferred homes' indoor-air chains
    if (a.d.n_rp > 1) {
        const int rcc = launch_kernel(cell_kernel, attr[7], b, min(N, CELL_BLOCKS), NT_CELL,
                                      (size_t)cell_lds_bytes(a.d.horizon), s);
        if (rcc) return rcc;
    }
    // the deferred homes: the mid launch (fronts of 384 labels, many blocks), its overflows to the
    // big launch (2,048 labels, 2 blocks per CU), what no front DP can take to the step-function DP
    const int rcm = launch_kernel(mpc_direct_kernel<EXPLICIT, DM_MID, NW_MID>, attr[6], b,
                                  min(N, mid_slots<EXPLICIT>(dev, a.d.horizon, a.d.sub_steps)), NW_MID * WAVE,
                                  (size_t)mid_layout(a.d.horizon, a.d.sub_steps).bytes, s);
    if (rcm) return rcm;
    const int rc2 = launch_kernel(mpc_direct_kernel<EXPLICIT, DM_BUCKET, NW_BIG>, attr[2], b, min(N, SECOND_SLOTS),
                                  NW_BIG * WAVE, (size_t)big_layout(a.d.horizon, a.d.sub_steps).bytes, s);
    if (rc2) return rc2;
    const int rcn = launch_kernel(mpc_direct_kernel<EXPLICIT, DM_NARROW, NT_STEPS / WAVE>, attr[5], b, min(N, NARROW_SLOTS),
                                  NT_STEPS, (size_t)narrow_layout(a.d.horizon, a.d.sub_steps, b.narrow_lds).bytes, s);
    return rcn;
}

// Lag mode: one timestep in two passes on two streams (the caller orders them: the side pass of step t
// after the main pass of step t, the main pass of step t + R after the side pass of step t when the
// caller's list ring holds R steps).
//  main: the hot launch over every home whose clock is at t (the others -- their previous step still on
//        the side stream -- listed in lag->skipped), the mid and big launches; the chains left for the
//        step-function DP go to lag->narrow and are NOT solved here;
//  side: the skipped homes' whole step (hot launch over lag->skipped, mid, big -- its own lists and
//        per-block scratch in lag->side_workspace) and the step-function DP over lag->narrow.
// A home's clock moves to t + 1 when its step is complete; so the next main pass solves every home
// whose step-function DP finished in time and leaves the others to the side stream, which runs behind.
// The side pass's persistent launches are small: it usually holds one or two lagging homes, and its
// empty blocks run beside the main pass's next hot launch.  Measured (driver window, 20 steps): a full-
// size side pass (256 / ~1,800 / 512 / 8 blocks) 1.482 ms/step, 16 / 16 / 16 / 2 blocks 1.434, 4 / 4 /
// 4 / 1 1.435, serial steps 1.427; full day 1.807 / 1.759 / 1.775 ms/step
constexpr int SIDE_HOT_BLOCKS = 16;         // persistent blocks of the side pass's hot launch
constexpr int SIDE_MID_BLOCKS = 16;         // ... mid launch
constexpr int SIDE_BIG_BLOCKS = 16;         // ... big launch
constexpr int SIDE_NARROW_BLOCKS = 2;       // ... step-function launch (each needs a whole CU's LDS)
// blocks of one side-pass launch: the DRAGG_SIDE_GRID entry (knob > 0) or the default, at most one per home
// and at most `slots` (the launch's per-block scratch regions), at least one
int side_grid_blocks(int knob, int dflt, int N, int slots) { return max(1, min(min(N, slots), knob > 0 ? knob : dflt)); }
void side_grids(int N, int out[4]) {
    const int* sg = knobs().side_grid;
    const int cap[4] = {N, MID_SLOTS_MAX, SECOND_SLOTS, narrow_slots(N)};
    const int dflt[4] = {SIDE_HOT_BLOCKS, SIDE_MID_BLOCKS, SIDE_BIG_BLOCKS, SIDE_NARROW_BLOCKS};
    for (int i = 0; i < 4; ++i) out[i] = side_grid_blocks(sg[i], dflt[i], N, cap[i]);
}
int launch_lag(const KArgs& a, bool side, hipStream_t s) {
    static int attr_dev[MAX_DEV][10] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return DRAGG_E_HIP;
    int* const attr = attr_dev[dev];
    const int N = a.d.n_homes, H = a.d.horizon;
    if (N == 0) return DRAGG_OK;
    char* const lw = a.lws;
    int* const len = reinterpret_cast<int*>(lw + defer_offset(N, H)) + N;
    int* const blen = reinterpret_cast<int*>(lw + mid_list_offset(N, H)) + N;
    KArgs b = a;
    // DRAGG_FORCE_STEP_DP holds here too: the hot launches list every home's chains in the step's narrow
    // list (lag->narrow), which the side pass's step-function launch then solves.  (DRAGG_WAVES_PER_HOME
    // does not: both passes run the one-wave hot kernel; the header says so.)
    b.force_steps = knobs().force_steps;
    b.step_pool_cap = knobs().step_pool_cap;
    b.step_work_cap = knobs().step_work_cap;
    b.narrow_lds = knobs().narrow_lds;
    const size_t lds = kernel_lds_bytes(&a.d);
    if (!side) {
        hipLaunchKernelGGL(reset_lists_kernel, dim3(1), dim3(WAVE), 0, s, len, blen, a.skip + N, a.nar + N, nullptr);
        if (hipGetLastError() != hipSuccess) return DRAGG_E_HIP;
        b.hot_list = nullptr;
        b.side = 0;
        int rc = hot_ilp(dev, N) == 2 ? launch_kernel(mpc_direct_kernel<false, DM_FRONT, 1, 2>, attr[8], b, N, WAVE, lds, s)
                                      : launch_kernel(mpc_direct_kernel<false, DM_FRONT, 1>, attr[1], b, N, WAVE, lds, s);
        if (!rc && a.d.n_rp > 1)
            rc = launch_kernel(cell_kernel, attr[7], b, min(N, CELL_BLOCKS), NT_CELL, (size_t)cell_lds_bytes(H), s);
        if (!rc) rc = launch_kernel(mpc_direct_kernel<false, DM_MID, NW_MID>, attr[6], b,
                                    min(N, mid_slots<false>(dev, H, a.d.sub_steps)), NW_MID * WAVE,
                                    (size_t)mid_layout(H, a.d.sub_steps).bytes, s);
        if (!rc) rc = launch_kernel(mpc_direct_kernel<false, DM_BUCKET, NW_BIG>, attr[2], b, min(N, SECOND_SLOTS),
                                    NW_BIG * WAVE, (size_t)big_layout(H, a.d.sub_steps).bytes, s);
        return rc;
    }
    // (lag->skipped and lag->narrow were zeroed by the main pass, which filled them)
    hipLaunchKernelGGL(reset_lists_kernel, dim3(1), dim3(WAVE), 0, s, len, blen, nullptr, nullptr, nullptr);
    if (hipGetLastError() != hipSuccess) return DRAGG_E_HIP;
    b.hot_list = a.skip;
    b.skip = nullptr;
    b.side = 1;
    // the persistent launches index per-block scratch by blockIdx.x: a DRAGG_SIDE_GRID entry is clamped to
    // its region's slots (the mid launch's MID_SLOTS_MAX rows, the big launch's SECOND_SLOTS, the
    // step-function launch's narrow_slots(N) pools; the hot and cell launches keep no per-block scratch)
    int grid[4];
    side_grids(N, grid);
    int rc = launch_kernel(side_front_kernel, attr[0], b, grid[0], WAVE, lds, s);
    b.hot_list = nullptr;
    if (!rc && a.d.n_rp > 1)
        rc = launch_kernel(cell_kernel, attr[7], b, grid[1], NT_CELL, (size_t)cell_lds_bytes(H), s);
    if (!rc) rc = launch_kernel(mpc_direct_kernel<false, DM_MID, NW_MID>, attr[6], b, grid[1], NW_MID * WAVE,
                                (size_t)mid_layout(H, a.d.sub_steps).bytes, s);
    if (!rc) rc = launch_kernel(mpc_direct_kernel<false, DM_BUCKET, NW_BIG>, attr[2], b, grid[2],
                                NW_BIG * WAVE, (size_t)big_layout(H, a.d.sub_steps).bytes, s);
    if (!rc) rc = launch_kernel(mpc_direct_kernel<false, DM_NARROW, NT_STEPS / WAVE>, attr[5], b,
                                grid[3], NT_STEPS, (size_t)narrow_layout(H, a.d.sub_steps, b.narrow_lds).bytes, s);
    return rc;
}

}  // namespace

extern "C" {

int dragg_mpc_abi_version(void) { return DRAGG_MPC_ABI_VERSION; }

const char* dragg_mpc_strerror(int code) {
    switch (code) {
        case DRAGG_OK: return "ok";
        case DRAGG_E_ARG: return "invalid argument";
        case DRAGG_E_HIP: return "HIP launch error";
        case DRAGG_E_LDS: return "cannot raise the dynamic LDS limit";
        case DRAGG_E_HORIZON: return "horizon too long for one workgroup's LDS";
        default: return "unknown error";
    }
}

int64_t dragg_mpc_workspace_bytes(const dragg_mpc_dims* dims) {
    const int rc = check_dims(dims);
    if (rc) return rc;
    return (int64_t)workspace_bytes(dims);
}

int64_t dragg_mpc_side_workspace_bytes(const dragg_mpc_dims* dims) {
    const int rc = check_dims(dims);
    if (rc) return rc;
    return direct_mode(dims) ? (int64_t)side_workspace_bytes(dims->n_homes, dims->horizon) : 0;
}

int dragg_mpc_side_grid(const dragg_mpc_dims* dims, int32_t* grid4) {
    const int rc = check_dims(dims);
    if (rc) return rc;
    if (!grid4) return DRAGG_E_ARG;
    int g[4];
    side_grids(dims->n_homes, g);
    for (int i = 0; i < 4; ++i) grid4[i] = dims->n_homes > 0 ? g[i] : 0;
    return DRAGG_OK;
}

const char* dragg_mpc_source_hash(void) { return kSourceStamp + sizeof(kSourcePrefix) - 1; }

int dragg_mpc_lds_bytes(const dragg_mpc_dims* dims) {
    const int rc = check_dims(dims);
    if (rc) return rc;
    return (int)kernel_lds_bytes(dims);
}

int dragg_mpc_step(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                   dragg_mpc_out* out, int32_t timestep, const double* noise, void* stream) {
    int rc = check_dims(dims);
    if (rc) return rc;
    // an empty shard (more ranks than homes) is a no-op; its per-home arrays may be NULL
    if (dims->n_homes == 0) return (prob && hash && out && timestep >= 0) ? DRAGG_OK : DRAGG_E_ARG;
    if (!prob || !hash || !out || timestep < 0 || !prob->params || !prob->home_type || !prob->oat ||
        !prob->ghi || !prob->tou || !prob->reward_price || !prob->draw_hourly || !hash->vals || !hash->fc ||
        !out->status || !out->iters || !out->obj || !out->relax_obj)
        return DRAGG_E_ARG;
    if (dims->n_rp != 1 && dims->n_rp < dims->horizon) return DRAGG_E_ARG;   // numpy broadcast error
    if (prob->start_index + timestep + dims->horizon >= dims->n_env) return DRAGG_E_ARG;
    if (direct_mode(dims) && !prob->workspace) return DRAGG_E_ARG;
    KArgs a{};
    a.d = *dims; a.p = *prob; a.vals = hash->vals; a.fc = hash->fc; a.out = *out; a.noise = noise;
    a.t = timestep;
    return launch<false>(a, (hipStream_t)stream);
}

static int lag_args(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                    dragg_mpc_out* out, int32_t timestep, const dragg_mpc_lag* lag, bool side, KArgs* a) {
    int rc = check_dims(dims);
    if (rc) return rc;
    if (!direct_mode(dims) || !lag || !prob || !hash || !out || timestep < 0) return DRAGG_E_ARG;
    if (dims->n_homes == 0) return DRAGG_OK;
    if (!lag->clock || !lag->skipped || !lag->narrow || (side && !lag->side_workspace) || !prob->params ||
        !prob->home_type || !prob->oat || !prob->ghi || !prob->tou || !prob->reward_price || !prob->draw_hourly ||
        !prob->workspace || !hash->vals || !hash->fc || !out->status || !out->iters || !out->obj || !out->relax_obj)
        return DRAGG_E_ARG;
    if (dims->n_rp != 1 && dims->n_rp < dims->horizon) return DRAGG_E_ARG;
    if (prob->start_index + timestep + dims->horizon >= dims->n_env) return DRAGG_E_ARG;
    if (timestep >= LAG_SIDE - 1) return DRAGG_E_ARG;
    *a = KArgs{};
    a->d = *dims; a->p = *prob; a->vals = hash->vals; a->fc = hash->fc; a->out = *out; a->noise = nullptr;
    a->t = timestep;
    // the side workspace holds only the span [defer_offset, w_region_offset) of the layout: its base stands
    // at defer_offset (the kernels address lists and per-block scratch as lws + their layout offset, all
    // inside that span; nothing below defer_offset is addressed through lws)
    a->lws = side ? reinterpret_cast<char*>(lag->side_workspace) - defer_offset(dims->n_homes, dims->horizon)
                  : reinterpret_cast<char*>(prob->workspace);
    a->clk = lag->clock; a->skip = lag->skipped; a->nar = lag->narrow;
    return DRAGG_OK;
}

int dragg_mpc_step_main(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                        dragg_mpc_out* out, int32_t timestep, const dragg_mpc_lag* lag, void* stream) {
    KArgs a;
    const int rc = lag_args(dims, prob, hash, out, timestep, lag, false, &a);
    if (rc || dims->n_homes == 0) return rc;
    return launch_lag(a, false, (hipStream_t)stream);
}

int dragg_mpc_step_side(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                        dragg_mpc_out* out, int32_t timestep, const dragg_mpc_lag* lag, void* stream) {
    KArgs a;
    const int rc = lag_args(dims, prob, hash, out, timestep, lag, true, &a);
    if (rc || dims->n_homes == 0) return rc;
    return launch_lag(a, true, (hipStream_t)stream);
}

int dragg_mpc_lag_reset(const dragg_mpc_dims* dims, const dragg_mpc_lag* lag, int32_t timestep, void* stream) {
    if (!dims || dims->n_homes < 0 || !lag || timestep < 0 || timestep >= LAG_SIDE - 1) return DRAGG_E_ARG;
    if (dims->n_homes == 0) return DRAGG_OK;
    if (!lag->clock) return DRAGG_E_ARG;
    hipLaunchKernelGGL(lag_reset_kernel, dim3((dims->n_homes + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       lag->clock, dims->n_homes, timestep);
    return hipGetLastError() == hipSuccess ? DRAGG_OK : DRAGG_E_HIP;
}

int dragg_mpc_aggregate_rows(const dragg_mpc_dims* dims, const double* rows, int32_t n_rows, double* out,
                             void* stream) {
    if (!dims || dims->n_homes < 0 || n_rows < 0 || (n_rows > 0 && (!out || (!rows && dims->n_homes > 0))))
        return DRAGG_E_ARG;
    if (n_rows == 0) return DRAGG_OK;
    hipLaunchKernelGGL(aggregate_rows_kernel, dim3(n_rows), dim3(AGG_NT), 0, (hipStream_t)stream, rows,
                       dims->n_homes, out);
    return hipGetLastError() == hipSuccess ? DRAGG_OK : DRAGG_E_HIP;
}

int dragg_mpc_solve_explicit(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob,
                             const dragg_mpc_explicit* in, dragg_mpc_hash* hash, dragg_mpc_out* out,
                             void* stream) {
    int rc = check_dims(dims);
    if (rc) return rc;
    if (dims->n_homes == 0) return (prob && in && hash && out) ? DRAGG_OK : DRAGG_E_ARG;
    if (!prob || !in || !hash || !out || !prob->params || !prob->home_type || !in->t || !in->T0 ||
        !in->Tw0 || !in->E0 || !in->counter || !in->winter || !in->draw || !in->oat || !in->ghi ||
        !in->price || !hash->vals || !hash->fc || !out->status || !out->iters || !out->obj ||
        !out->relax_obj)
        return DRAGG_E_ARG;
    if (direct_mode(dims) && !prob->workspace) return DRAGG_E_ARG;
    KArgs a{};
    a.d = *dims; a.p = *prob; a.ex = *in; a.vals = hash->vals; a.fc = hash->fc; a.out = *out;
    return launch<true>(a, (hipStream_t)stream);
}

void dragg_mpc_reload_knobs(void) { g_knobs = read_knobs(); }

int dragg_mpc_kernel_info_get(const dragg_mpc_dims* dims, dragg_mpc_kernel_info* info) {
    const int rc = check_dims(dims);
    if (rc) return rc;
    if (!info) return DRAGG_E_ARG;
    *info = dragg_mpc_kernel_info{};
    auto one = [&](const void* kern, int i, size_t lds, int nt) -> int {
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, kern) != hipSuccess) return DRAGG_E_HIP;
        // the launches raise the dynamic LDS limit first (launch_kernel); so does the query
        if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DYN_MAX) != hipSuccess)
            return DRAGG_E_LDS;
        int blocks = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kern, nt, lds) != hipSuccess) return DRAGG_E_HIP;
        info->vgprs[i] = fa.numRegs;
        info->scratch_bytes[i] = (int32_t)fa.localSizeBytes;
        info->lds_bytes[i] = (int32_t)lds;
        info->threads[i] = nt;
        info->blocks_per_cu[i] = blocks;
        return DRAGG_OK;
    };
    if (!direct_mode(dims)) return one((const void*)mpc_home_kernel<false>, 0, kernel_lds_bytes(dims), WAVE);
    const int H = dims->horizon, S = dims->sub_steps;
    int r = one((const void*)mpc_direct_kernel<false, DM_FRONT>, 0, kernel_lds_bytes(dims), WAVE);
    if (!r) r = one((const void*)mpc_direct_kernel<false, DM_BUCKET, NW_BIG>, 1, (size_t)big_layout(H, S).bytes,
                    NW_BIG * WAVE);
    if (!r) r = one((const void*)mpc_direct_kernel<false, DM_MID, NW_MID>, 2, (size_t)mid_layout(H, S).bytes,
                    NW_MID * WAVE);
    if (!r) r = one((const void*)mpc_direct_kernel<false, DM_NARROW, NT_STEPS / WAVE>, 3,
                    (size_t)narrow_layout(H, S, knobs().narrow_lds).bytes, NT_STEPS);
    return r;
}

int dragg_mpc_aggregate(const dragg_mpc_dims* dims, const dragg_mpc_hash* hash, double* out3, void* stream) {
    // n_homes == 0: the sums are zero (vals may be NULL)
    if (!dims || !hash || (!hash->vals && dims->n_homes > 0) || !out3 || dims->n_homes < 0) return DRAGG_E_ARG;
    hipLaunchKernelGGL(aggregate_kernel, dim3(1), dim3(AGG_NT), 0, (hipStream_t)stream, hash->vals,
                       dims->n_homes, out3);
    return hipGetLastError() == hipSuccess ? DRAGG_OK : DRAGG_E_HIP;
}

int dragg_mpc_season_noise(const dragg_mpc_dims* dims, uint64_t seed, int32_t home_offset, int32_t home_stride,
                           int32_t timestep, double* noise_out, void* stream) {
    if (!dims || dims->n_homes < 0 || dims->horizon < 1) return DRAGG_E_ARG;
    const int total = dims->n_homes * ((dims->horizon + 1) / 2);
    if (total == 0) return DRAGG_OK;
    if (!noise_out) return DRAGG_E_ARG;
    hipLaunchKernelGGL(noise_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       dims->n_homes, dims->horizon, seed, home_offset, max(home_stride, 1), timestep, noise_out);
    return hipGetLastError() == hipSuccess ? DRAGG_OK : DRAGG_E_HIP;
}

}  // extern "C"
