/*
 * dragg_mi355x.h -- C ABI of the batched MI355X (gfx950) home-MPC solver.
 *
 * Drop-in replacement for the per-home HEMS solve of corymosiman12/dragg:
 *
 *   reference                                   this ABI
 *   -----------------------------------------   ------------------------------------------
 *   MPCCalc.run_home()        mpc_calc.py:649   dragg_mpc_step()      (device-resident state)
 *     get_initial_conditions  mpc_calc.py:264     (initial state read from the hash arrays)
 *     water_draws             mpc_calc.py:193     (computed on device from draw_hourly)
 *     set_environmental_vars  mpc_calc.py:206     (slices of oat/ghi/tou + reward price)
 *     add_*_constraints       mpc_calc.py:291-432 (built on device, never materialised)
 *     solve_mpc (GLPK_MI)     mpc_calc.py:434     (int_mode round, default: the MILP solved
 *                                                  exactly -- thermal chains by an exact
 *                                                  Pareto-front DP, battery by an exact
 *                                                  piecewise-linear DP; relax / round_lp:
 *                                                  banded-KKT ADMM + exact vertex polish)
 *     cleanup_and_finish      mpc_calc.py:476     (success extraction / fallback thermostat)
 *     redis_write_optimal_vals mpc_calc.py:100    (hash arrays updated in place)
 *   manage_home + ProcessPool aggregator.py:723   one launch over all homes of a timestep
 *   collect_data sums         aggregator.py:751   dragg_mpc_aggregate() / dragg_mpc_aggregate_rows()
 *   run_baseline's loop       aggregator.py:757   dragg_mpc_step_main() + dragg_mpc_step_side()
 *                                                  (lag mode: a home still in its step-function DP
 *                                                  does not hold up the other homes' next steps)
 *   MPCCalc per-solve (explicit inputs)         dragg_mpc_solve_explicit()
 *
 * Conventions
 *  - Every pointer in the structs below is a DEVICE pointer (hipMalloc / torch
 *    CUDA tensors), fp64 unless stated; arrays are struct-of-arrays with the home
 *    index innermost: element (f, h) of a [F][N] array lives at f*N + h.
 *  - All entry points return 0 on success or a negative dragg_mpc_error code;
 *    nothing throws across the ABI.  Launches are asynchronous on `stream`
 *    (a hipStream_t, NULL = default stream); no host synchronisation inside.
 *  - The per-home redis hash (`redis_client.py`, all values str) is replaced by
 *    two fp64 arrays: `vals` [DRAGG_NVAL][N] (the scalar fields a step writes)
 *    and `fc` [N][DRAGG_NFC][H] (the `<key>_<j>` forecast fields, rewritten only
 *    by a successful solve).  NaN means "field absent from the hash".
 */
#ifndef DRAGG_MI355X_H
#define DRAGG_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRAGG_MPC_ABI_VERSION 9

/* home types (aggregator.py:425, 468, 520, 555); bit 0 = pv, bit 1 = battery */
enum dragg_home_type {
    DRAGG_BASE = 0, DRAGG_PV_ONLY = 1, DRAGG_BATTERY_ONLY = 2, DRAGG_PV_BATTERY = 3
};

/* per-home parameters, rows of params[DRAGG_NPARAM][N] (mpc_calc.py:157-189, 239-258) */
enum dragg_param {
    DRAGG_P_R = 0,        /* hvac.r                               */
    DRAGG_P_C,            /* hvac.c * 1000                        */
    DRAGG_P_PC,           /* hvac.p_c / S                         */
    DRAGG_P_PH,           /* hvac.p_h / S                         */
    DRAGG_P_RW,           /* wh.r * 1000                          */
    DRAGG_P_PW,           /* wh.p / S                             */
    DRAGG_P_CW,           /* wh.tank_size * 4.2                   */
    DRAGG_P_V,            /* wh.tank_size                         */
    DRAGG_P_TMIN, DRAGG_P_TMAX, DRAGG_P_TWMIN, DRAGG_P_TWMAX,
    DRAGG_P_TINIT,        /* hvac.temp_in_init                    */
    DRAGG_P_TWINIT,       /* wh.temp_wh_init                      */
    DRAGG_P_BRATE,        /* battery.max_rate                     */
    DRAGG_P_EMIN,         /* battery.capacity_lower * capacity    */
    DRAGG_P_EMAX,         /* battery.capacity_upper * capacity    */
    DRAGG_P_ETAC, DRAGG_P_ETAD,
    DRAGG_P_EINIT,        /* battery.e_batt_init * capacity       */
    DRAGG_P_PVAREA, DRAGG_P_PVEFF,
    DRAGG_NPARAM
};

/* forecast keys: rows of fc[N][DRAGG_NFC][H] (`<key>_<j>` hash fields, mpc_calc.py:514-520) */
enum dragg_fc_key {
    DRAGG_K_P_GRID = 0, DRAGG_K_FORECAST_P_GRID, DRAGG_K_P_LOAD, DRAGG_K_TEMP_IN_EV,
    DRAGG_K_TEMP_WH_EV, DRAGG_K_HVAC_COOL, DRAGG_K_HVAC_HEAT, DRAGG_K_WH_HEAT, DRAGG_K_COST,
    DRAGG_K_WATERDRAWS, DRAGG_K_P_PV, DRAGG_K_U_PV_CURT, DRAGG_K_P_BATT_CH,
    DRAGG_K_P_BATT_DISCH, DRAGG_K_E_BATT,
    DRAGG_NFC
};

/* scalar hash fields: rows of vals[DRAGG_NVAL][N]; rows 0..14 are the keys above, i.e. the
   un-suffixed `<key>` field (mpc_calc.py:516, 584-594) */
enum dragg_val {
    DRAGG_V_TEMP_IN_OPT = DRAGG_NFC, DRAGG_V_TEMP_WH_OPT, DRAGG_V_CORRECT_SOLVE,
    DRAGG_V_SOLVE_COUNTER,
    DRAGG_NVAL
};

/* per-home status written by a step (status[N]) */
enum dragg_status {
    DRAGG_ST_OPTIMAL = 0,          /* solved: the MILP optimum (round) / LP vertex (relax)      */
    DRAGG_ST_INFEASIBLE = 1,       /* proven infeasible by interval presolve                   */
    DRAGG_ST_INFEASIBLE_CERT = 2,  /* ADMM primal-infeasibility certificate                     */
    DRAGG_ST_MAX_ITER = 3,         /* no verified vertex within max_iter                         */
    DRAGG_ST_ROUND_FAIL = 4,       /* boxes pass presolve, but no integer duty schedule exists  */
    DRAGG_ST_ERR_PARSE = 5,        /* fallback's float(str[0]) would raise (mpc_calc.py:537)     */
    DRAGG_ST_ERR_MISSING = 6,      /* hash field missing at t>0 (KeyError, mpc_calc.py:280-289)  */
    DRAGG_ST_SOLVER_ERROR = 7      /* the named solver raised: prob.solve's exception is          */
                                   /* swallowed and the fallback runs (mpc_calc.py:450-454)       */
};

enum dragg_mpc_error {
    DRAGG_OK = 0, DRAGG_E_ARG = -1, DRAGG_E_HIP = -2, DRAGG_E_LDS = -3, DRAGG_E_HORIZON = -4
};

/* integer handling of the duty-cycle variables (mpc_calc.py:171-173) */
enum dragg_int_mode {
    DRAGG_INT_ROUND = 0,    /* MILP, exact: thermal front DP + battery LP DP (default) */
    DRAGG_INT_RELAX = 1,    /* LP relaxation (ADMM + exact vertex polish)             */
    DRAGG_INT_ROUND_LP = 2, /* LP relaxation for status/battery, then the integer DP  */
    DRAGG_INT_FAIL = 3      /* a solver that cannot take the MILP (hems.solver "ECOS": cvxpy's
                               ECOS is not MIP-capable, so prob.solve raises inside the try of
                               mpc_calc.py:450-454): every solve takes the fallback,
                               status DRAGG_ST_SOLVER_ERROR                           */
};

typedef struct dragg_mpc_dims {
    int32_t n_homes;       /* N (0 = an empty shard: every entry point is a no-op,
                              per-home pointers may be NULL; aggregate writes zeros)    */
    int32_t horizon;       /* H = prediction_horizon * dt            (mpc_calc.py:150) */
    int32_t sub_steps;     /* S = sub_subhourly_steps                (mpc_calc.py:148) */
    int32_t dt;            /* hourly_agg_steps                       (mpc_calc.py:149) */
    int32_t n_draw_hours;  /* columns of draw_hourly                                   */
    int32_t n_env;         /* length of oat/ghi/tou                                    */
    int32_t n_rp;          /* length of reward_price (1 or >= H, mpc_calc.py:353)      */
    int32_t int_mode;      /* dragg_int_mode                                           */
    int32_t max_iter;      /* ADMM iteration cap (<=0: default 4000)                   */
    int32_t check_every;   /* polish / residual check interval (<=0: default 10)       */
    double discount;       /* discount_factor                        (mpc_calc.py:152) */
    int32_t flags;         /* dragg_flag bits (0 = default)                             */
    int32_t reserved;
} dragg_mpc_dims;

/* dims.flags */
enum dragg_flag {
    /* int_mode round is exact on every TOU chain by default: a chain the Pareto-front DPs cannot
       take (a feasible set narrower than one duty step, mixed-sign prices without a usable bound, a
       front past 2,048 labels, S != 6) is solved by the exact step-function DP (out.int_path bit
       15).  The one exception: a chain under RL prices (a price change at more than H/4 stages)
       whose front passes 2,048 labels keeps its bucketed schedule (int_path reason 3) unless this
       flag is set -- there the step-function DP costs ~25x the whole RL action. */
    DRAGG_FLAG_EXACT = 1
};

typedef struct dragg_mpc_problem {
    const double* params;       /* [DRAGG_NPARAM][N]                                    */
    const int32_t* home_type;   /* [N] dragg_home_type                                  */
    const double* draw_hourly;  /* [n_draw_hours][N] wh.draw_sizes (aggregator.py:377)  */
    const double* oat;          /* [n_env] redis 'OAT' list                             */
    const double* ghi;          /* [n_env] redis 'GHI' list                             */
    const double* tou;          /* [n_env] redis 'tou' list                             */
    const double* reward_price; /* [n_rp]  redis 'reward_price' list                    */
    int32_t start_index;        /* start_hour_index (aggregator.py:630-638)             */
    int32_t home_offset;        /* global index of home 0 of this shard (noise key)     */
    uint64_t seed;              /* keyed season-noise stream when noise == NULL         */
    void* workspace;            /* device scratch, dragg_mpc_workspace_bytes(dims) bytes */
                                /* (int_mode round: DP back-pointers); may be NULL when  */
                                /* that size is 0                                        */
    int32_t home_stride;        /* global index of home i = home_offset + i*home_stride */
                                /* (strided shards; 0 or 1 = a contiguous shard)         */
    int32_t reserved;
} dragg_mpc_problem;

typedef struct dragg_mpc_hash {
    double* vals;               /* [DRAGG_NVAL][N]  in/out, NaN = absent               */
    double* fc;                 /* [N][DRAGG_NFC][H] in/out (home-contiguous since v7) */
} dragg_mpc_hash;

typedef struct dragg_mpc_out {
    int32_t* status;            /* [N] dragg_status                                     */
    int32_t* iters;             /* [N] ADMM iterations used (0 if presolve decided)    */
    double* obj;                /* [N] objective sum_k gamma^k price_k p_grid_k         */
    double* relax_obj;          /* [N] LP-relaxation objective (NaN if infeasible)     */
    double* hist;               /* optional [DRAGG_NVAL][N] copy of vals after the step */
    int64_t* cycles;            /* optional [DRAGG_NPHASE][N] shader cycles per phase   */
    int32_t* int_path;          /* optional [N] integer-DP path (int_mode round): 0 = the
                                   exact front DP solved both thermal chains; bit 0 / bit 1
                                   = the indoor-air / tank chain kept an approximate (feasible)
                                   schedule; bits 4-7 / 8-11 its reason: 3 = an RL-priced chain
                                   (a price change at more than H/4 stages) whose front passed
                                   the big launch's 2,048 labels keeps its bucketed schedule
                                   (default build; DRAGG_FLAG_EXACT sends it to the step-function
                                   DP), 6 = the exact step-function DP past its capacity (its pool
                                   of 2^20 breakpoints per chain, or its work bound of 2 M merge
                                   points per pass): the bucketed schedule it was handed stands in
                                   (else the feasibility pass's); bit 12 = solved by a later launch (its front
                                   outgrew the hot launch's capacity; still exact when
                                   bits 0-11 are 0); bits 13 / 14 = status ROUND_FAIL
                                   decided by the indoor-air / tank chain (no integer duty
                                   schedule for it); bit 15 = solved by the exact
                                   step-function DP (a feasible set narrower than one duty
                                   step, mixed-sign prices, S != 6, a front past 2,048)  */
} dragg_mpc_out;

/* solver phases timed into dragg_mpc_out.cycles (diagnostic; NULL = not stamped) */
enum dragg_phase {
    DRAGG_PH_SETUP = 0,   /* inputs, problem build, presolve              */
    DRAGG_PH_ITER,        /* ADMM iterations (rhs, KKT solve, updates);   */
                          /* int_mode round: the bucketed DP              */
    DRAGG_PH_FACTOR,      /* block-LDL' factorisations                    */
    DRAGG_PH_POLISH,      /* exact basis polish; int_mode round: the mid  */
                          /* / big launch's exact front pass              */
    DRAGG_PH_CHECK,       /* residuals, certificate, rho adaptation       */
    DRAGG_PH_INTEGER,     /* integer duty-cycle DP                        */
    DRAGG_PH_WRITE,       /* objective, cleanup_and_finish, hash writes   */
    DRAGG_PH_BATTERY,     /* exact battery LP (int_mode round)            */
    DRAGG_NPHASE
};

/* explicit per-solve inputs (parity tests and the per-home MPCCalc facade) */
typedef struct dragg_mpc_explicit {
    const int32_t* t;           /* [N] timestep (fallback rule needs t > 0)             */
    const double* T0;           /* [N] temp_in_init value                               */
    const double* Tw0;          /* [N] temp_wh_init value (after draw mixing)           */
    const double* E0;           /* [N] e_batt_init value (ignored for non-battery)      */
    const int32_t* counter;     /* [N] solve_counter read from the hash                 */
    const int32_t* winter;      /* [N] 1 = max(oat_ev) <= 30 (mpc_calc.py:303)          */
    const double* draw;         /* [H+1][N] draw_size                                   */
    const double* oat;          /* [H+1][N] oat_current                                 */
    const double* ghi;          /* [H+1][N] ghi_current                                 */
    const double* price;        /* [H][N]   total_price                                 */
} dragg_mpc_explicit;

/* Resources of the solver's launches as the code object and the runtime report them
   (hipFuncGetAttributes, hipOccupancyMaxActiveBlocksPerMultiprocessor on the current device):
   index 0 = the hot launch (int_mode round: DM_FRONT; relax / round_lp: the LP kernel),
   index 1 = the big launch (DM_BUCKET), index 2 = the mid launch (DM_MID), index 3 = the
   step-function launch (DM_NARROW); indices 1-3 are zeros outside int_mode round. */
#define DRAGG_NLAUNCH 4
typedef struct dragg_mpc_kernel_info {
    int32_t vgprs[DRAGG_NLAUNCH];          /* registers per lane (hipFuncAttributes.numRegs)   */
    int32_t scratch_bytes[DRAGG_NLAUNCH];  /* private memory per lane (spills; localSizeBytes) */
    int32_t lds_bytes[DRAGG_NLAUNCH];      /* dynamic LDS per workgroup at these dims          */
    int32_t threads[DRAGG_NLAUNCH];        /* threads per workgroup (one home per workgroup)   */
    int32_t blocks_per_cu[DRAGG_NLAUNCH];  /* resident workgroups per CU at that LDS           */
} dragg_mpc_kernel_info;

int dragg_mpc_abi_version(void);
const char* dragg_mpc_strerror(int code);

/* Dynamic LDS bytes one home (workgroup) needs for this horizon; < 0 if H unsupported. */
int dragg_mpc_lds_bytes(const dragg_mpc_dims* dims);

/* Device workspace bytes a launch with these dims needs (problem.workspace); < 0 on error. */
int64_t dragg_mpc_workspace_bytes(const dragg_mpc_dims* dims);

/* Device bytes of the lag mode's side workspace (dragg_mpc_lag.side_workspace; since v9): the side
   pass keeps only its device lists and per-block scratch there (the per-home regions are read from
   problem.workspace), ~0.5 GB at 10k homes, H = 48, against the workspace's 1.34 GB. */
int64_t dragg_mpc_side_workspace_bytes(const dragg_mpc_dims* dims);

/* The sha-256 of the sources this library was built from (the kernel file and this header; since
   v9): the host refuses a library whose stamp is not its sources' (a stale build). */
const char* dragg_mpc_source_hash(void);

/* One closed-loop timestep for all N homes: reads the hash arrays (t > 0) or the
   parameters (t == 0), solves, and writes the hash arrays back in place.
   noise: [H][N] standard normals for the season draw (mpc_calc.py:222) or NULL for the
   keyed on-device stream philox(seed, home, t). */
int dragg_mpc_step(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob,
                   dragg_mpc_hash* hash, dragg_mpc_out* out, int32_t timestep,
                   const double* noise, void* stream);

/* Independent solves with explicit inputs; hash supplies the fallback's forecast fields
   and receives the written fields exactly as in dragg_mpc_step. prob->oat/ghi/tou/
   reward_price/draw_hourly are ignored. */
int dragg_mpc_solve_explicit(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob,
                             const dragg_mpc_explicit* in, dragg_mpc_hash* hash,
                             dragg_mpc_out* out, void* stream);

/* Diagnostic knobs, read from the environment when the library loads and again only here (never
   per step): DRAGG_WAVES_PER_HOME=1|2|4 (the hot launch's waves per home; results bit-identical) and
   DRAGG_FORCE_STEP_DP=1 (every chain through the step-function DP; tests), DRAGG_STEP_POOL_CAP=n and
   DRAGG_STEP_WORK_CAP=n (a smaller pool / work bound of that DP; tests of its capacity path),
   DRAGG_HOT_ILP=1|2 (64-child chunks per front-DP pass of the one-wave hot launch; default: 2 at <= 8 homes
   per CU, else 1; results bit-identical), DRAGG_SIDE_GRID=hot,mid,big,narrow (the lag mode's side-pass
   grids, each clamped to 1 .. its launch's per-block scratch slots: dragg_mpc_side_grid reports the
   grids in effect), DRAGG_NARROW_LDS_KB=n (the step-function launch's LDS per block; default all of a
   CU's: a smaller block can share a CU with hot-launch blocks; results bit-identical).  Unset: the defaults.  Lag mode (dragg_mpc_step_main / _side) honours every knob
   but DRAGG_WAVES_PER_HOME: both its passes run the one-wave hot kernel. */
void dragg_mpc_reload_knobs(void);

/* The lag mode's side-pass grids for these dims under the current knobs: grid4 = blocks of its hot,
   mid (and cell), big and step-function launches (zeros for an empty shard).  Host-only query. */
int dragg_mpc_side_grid(const dragg_mpc_dims* dims, int32_t* grid4);

/* Fill `info` for these dims (needs a GPU: queries the current device). */
int dragg_mpc_kernel_info_get(const dragg_mpc_dims* dims, dragg_mpc_kernel_info* info);

/* collect_data sums (aggregator.py:751-753): out3 = {sum p_grid_opt, sum
   forecast_p_grid_opt, sum cost_opt} over the shard's homes; an absent field (NaN: a home
   the reference would have crashed on, KeyError at aggregator.py:750-752) makes its sum NaN. */
int dragg_mpc_aggregate(const dragg_mpc_dims* dims, const dragg_mpc_hash* hash, double* out3,
                        void* stream);

/* Lag mode (since v8): run_rbo_mpc's timestep loop (aggregator.py:757-778) has no feedback between
   homes, so a home whose chain needs the slow exact step-function DP need not hold up the others.
   A step is split into two passes the caller puts on two streams:
     dragg_mpc_step_main(t)  on the main stream: every home whose clock is at t (its previous step
                             complete) is solved by the hot / mid / big launches; a home whose clock
                             is behind is listed in `skipped`; chains left for the step-function DP
                             are listed in `narrow` (not solved here);
     dragg_mpc_step_side(t)  on the side stream, AFTER main(t) (an event): the skipped homes' whole
                             step (their own lists and per-block scratch in side_workspace) and the
                             step-function DP of every chain in `narrow`.
   A home's clock becomes t + 1 when its step is complete (a side-pass completion is published to
   the concurrently running main pass with an agent-scope release).  Each step needs its own
   skipped / narrow lists until its side pass has run: with a ring of R list pairs the main pass of
   step t + R must wait for the side pass of step t.  Results are bit-identical to dragg_mpc_step's
   (every home's solve is the same code on the same inputs), but per-step outputs of lagging homes
   land later: the caller reads them (status -- out.status should then be a per-step row --, hist
   rows, vals/fc) only after the side stream has drained, and takes collect_data's sums from the
   history rows (dragg_mpc_aggregate_rows).  Keyed season noise only (the NULL-noise stream);
   int_mode round / fail only. */
typedef struct dragg_mpc_lag {
    int32_t* clock;             /* [N] timesteps completed per home (dragg_mpc_lag_reset) */
    int32_t* skipped;           /* [DRAGG_LAG_LIST_INTS(N)] the step's homes left to the side pass */
    int32_t* narrow;            /* [DRAGG_LAG_LIST_INTS(N)] the step's step-function DP chains   */
    void* side_workspace;       /* dragg_mpc_side_workspace_bytes(dims) bytes, the side pass's own */
} dragg_mpc_lag;
#define DRAGG_LAG_LIST_INTS(n) ((n) + 4)

/* clock[] = timestep for every home (before the first lag-mode step after any other kind of step) */
int dragg_mpc_lag_reset(const dragg_mpc_dims* dims, const dragg_mpc_lag* lag, int32_t timestep, void* stream);
int dragg_mpc_step_main(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                        dragg_mpc_out* out, int32_t timestep, const dragg_mpc_lag* lag, void* stream);
int dragg_mpc_step_side(const dragg_mpc_dims* dims, const dragg_mpc_problem* prob, dragg_mpc_hash* hash,
                        dragg_mpc_out* out, int32_t timestep, const dragg_mpc_lag* lag, void* stream);

/* collect_data's sums of n_rows steps from their history rows ([n_rows][DRAGG_NVAL][N], the
   dragg_mpc_out.hist copies): out[r][3] exactly as dragg_mpc_aggregate on row r (bit-identical). */
int dragg_mpc_aggregate_rows(const dragg_mpc_dims* dims, const double* rows, int32_t n_rows, double* out,
                             void* stream);

/* The keyed season-noise stream used when noise == NULL: writes [H][N] normals for
   timestep t (exposed so the host and tests can reproduce the draw); home i of the shard
   draws the stream of global home home_offset + i*home_stride (home_stride 0 = 1). */
int dragg_mpc_season_noise(const dragg_mpc_dims* dims, uint64_t seed, int32_t home_offset,
                           int32_t home_stride, int32_t timestep, double* noise_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DRAGG_MI355X_H */
