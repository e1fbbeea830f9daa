"""ctypes binding of the C ABI in include/dragg_mi355x.h (libdragg_mi355x.so).

The library is built in-tree (dragg_amd/libdragg_mi355x.so, see dragg_amd/build.py).
There is deliberately no CPU fallback: if the library or a GPU is missing, every
entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DRAGG_LIB: an alternative build of the same library (kernel experiments); default in-tree
LIB_PATH = os.environ.get("DRAGG_LIB") or os.path.join(HERE, "libdragg_mi355x.so")

ABI_VERSION = 9

# enums (mirror include/dragg_mi355x.h)
BASE, PV_ONLY, BATTERY_ONLY, PV_BATTERY = 0, 1, 2, 3
TYPE_CODE = {"base": BASE, "pv_only": PV_ONLY, "battery_only": BATTERY_ONLY, "pv_battery": PV_BATTERY}

PARAMS = ["R", "C", "PC", "PH", "RW", "PW", "CW", "V", "TMIN", "TMAX", "TWMIN", "TWMAX", "TINIT",
          "TWINIT", "BRATE", "EMIN", "EMAX", "ETAC", "ETAD", "EINIT", "PVAREA", "PVEFF"]
NPARAM = len(PARAMS)
P = {k: i for i, k in enumerate(PARAMS)}

FC_KEYS = ["p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "temp_in_ev_opt", "temp_wh_ev_opt",
           "hvac_cool_on_opt", "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws",
           "p_pv_opt", "u_pv_curt_opt", "p_batt_ch", "p_batt_disch", "e_batt_opt"]
NFC = len(FC_KEYS)
VAL_KEYS = FC_KEYS + ["temp_in_opt", "temp_wh_opt", "correct_solve", "solve_counter"]
NVAL = len(VAL_KEYS)
K = {k: i for i, k in enumerate(VAL_KEYS)}

(ST_OPTIMAL, ST_INFEASIBLE, ST_INFEASIBLE_CERT, ST_MAX_ITER, ST_ROUND_FAIL, ST_ERR_PARSE, ST_ERR_MISSING,
 ST_SOLVER_ERROR) = range(8)
# int_path bits (dragg_mi355x.h): 0-11 = a chain left the exact front DP (chain bits + reasons);
# PATH_SECOND = the home was solved by the second launch (exact unless bits 0-11 are set)
PATH_APPROX_MASK = 0xFFF
PATH_SECOND = 1 << 12
PATH_FAIL_T, PATH_FAIL_TW = 1 << 13, 1 << 14     # ROUND_FAIL decided by the indoor-air / tank chain
PATH_STEPS = 1 << 15           # solved by the exact step-function DP (DM_NARROW launch)
STATUS_NAMES = ["optimal", "infeasible", "infeasible_cert", "max_iter", "round_fail", "err_parse",
                "err_missing", "solver_error"]

INT_ROUND, INT_RELAX, INT_ROUND_LP, INT_FAIL = 0, 1, 2, 3
FLAG_EXACT = 1                 # dims.flags: the step-function DP for every chain the front DP cannot take
INT_MODES = {"round": INT_ROUND, "relax": INT_RELAX, "round_lp": INT_ROUND_LP, "fail": INT_FAIL}

PHASES = ["setup", "iter", "factor", "polish", "check", "integer", "write", "battery"]
NPHASE = len(PHASES)

c_dp = ctypes.c_void_p  # device pointers are passed as raw integers


class Dims(ctypes.Structure):
    _fields_ = [("n_homes", ctypes.c_int32), ("horizon", ctypes.c_int32), ("sub_steps", ctypes.c_int32),
                ("dt", ctypes.c_int32), ("n_draw_hours", ctypes.c_int32), ("n_env", ctypes.c_int32),
                ("n_rp", ctypes.c_int32), ("int_mode", ctypes.c_int32), ("max_iter", ctypes.c_int32),
                ("check_every", ctypes.c_int32), ("discount", ctypes.c_double), ("flags", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class Problem(ctypes.Structure):
    _fields_ = [("params", c_dp), ("home_type", c_dp), ("draw_hourly", c_dp), ("oat", c_dp), ("ghi", c_dp),
                ("tou", c_dp), ("reward_price", c_dp), ("start_index", ctypes.c_int32),
                ("home_offset", ctypes.c_int32), ("seed", ctypes.c_uint64), ("workspace", c_dp),
                ("home_stride", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Hash(ctypes.Structure):
    _fields_ = [("vals", c_dp), ("fc", c_dp)]


class Out(ctypes.Structure):
    _fields_ = [("status", c_dp), ("iters", c_dp), ("obj", c_dp), ("relax_obj", c_dp), ("hist", c_dp),
                ("cycles", c_dp), ("int_path", c_dp)]


class Explicit(ctypes.Structure):
    _fields_ = [("t", c_dp), ("T0", c_dp), ("Tw0", c_dp), ("E0", c_dp), ("counter", c_dp), ("winter", c_dp),
                ("draw", c_dp), ("oat", c_dp), ("ghi", c_dp), ("price", c_dp)]


class Lag(ctypes.Structure):
    _fields_ = [("clock", c_dp), ("skipped", c_dp), ("narrow", c_dp), ("side_workspace", c_dp)]


def lag_list_ints(n):
    """DRAGG_LAG_LIST_INTS(n): a lag-mode list (entries, length, take counter)."""
    return n + 4


NLAUNCH = 4                    # DRAGG_NLAUNCH: hot, big, mid, narrow (dragg_mpc_kernel_info)
LAUNCH_NAMES = ["hot", "big", "mid", "narrow"]


class KernelInfo(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int32 * NLAUNCH) for f in ("vgprs", "scratch_bytes", "lds_bytes", "threads",
                                                         "blocks_per_cu")]


EXPORTS = ["dragg_mpc_abi_version", "dragg_mpc_strerror", "dragg_mpc_lds_bytes", "dragg_mpc_workspace_bytes",
           "dragg_mpc_kernel_info_get", "dragg_mpc_step",
           "dragg_mpc_solve_explicit", "dragg_mpc_aggregate", "dragg_mpc_season_noise", "dragg_mpc_reload_knobs",
           "dragg_mpc_lag_reset", "dragg_mpc_step_main", "dragg_mpc_step_side", "dragg_mpc_aggregate_rows",
           "dragg_mpc_side_workspace_bytes", "dragg_mpc_side_grid", "dragg_mpc_source_hash"]

_LIB = None


class DraggError(RuntimeError):
    pass


def check_stamp(path):
    """The in-tree library must be built from the sources beside it: its source stamp (sha-256 of
    csrc/ and the header, dragg_amd/build.py) must equal theirs.  A stale library -- sources edited,
    checked out or copied after the build -- is refused rather than run.  DRAGG_LIB (an experiment's
    alternative build from other sources) and a tree without the sources are not checked."""
    from . import build as B
    if os.environ.get("DRAGG_LIB") or os.path.abspath(path) != os.path.abspath(B.OUT) or not B.sources_present():
        return
    got, want = B.stamp_of(path), B.source_hash()
    if got != want:
        raise DraggError(f"{path} is stale: built from sources {got}, the sources are now {want}; rebuild it "
                         "with `python -m dragg_amd.build`")


def load(path=LIB_PATH):
    """Load the HIP library (raises if it was not built, or was built from other sources)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise DraggError(f"{path} not found: build it with `python -m dragg_amd.build` "
                         "(there is no CPU fallback)")
    check_stamp(path)
    lib = ctypes.CDLL(path)
    lib.dragg_mpc_abi_version.restype = ctypes.c_int
    lib.dragg_mpc_strerror.restype = ctypes.c_char_p
    lib.dragg_mpc_strerror.argtypes = [ctypes.c_int]
    lib.dragg_mpc_lds_bytes.argtypes = [ctypes.POINTER(Dims)]
    lib.dragg_mpc_workspace_bytes.argtypes = [ctypes.POINTER(Dims)]
    lib.dragg_mpc_workspace_bytes.restype = ctypes.c_int64
    lib.dragg_mpc_side_workspace_bytes.argtypes = [ctypes.POINTER(Dims)]
    lib.dragg_mpc_side_workspace_bytes.restype = ctypes.c_int64
    lib.dragg_mpc_side_grid.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(ctypes.c_int32)]
    lib.dragg_mpc_source_hash.restype = ctypes.c_char_p
    lib.dragg_mpc_step.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Problem), ctypes.POINTER(Hash),
                                   ctypes.POINTER(Out), ctypes.c_int32, c_dp, c_dp]
    lib.dragg_mpc_solve_explicit.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Problem),
                                             ctypes.POINTER(Explicit), ctypes.POINTER(Hash),
                                             ctypes.POINTER(Out), c_dp]
    lib.dragg_mpc_kernel_info_get.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(KernelInfo)]
    lib.dragg_mpc_reload_knobs.argtypes = []
    lib.dragg_mpc_reload_knobs.restype = None
    lib.dragg_mpc_aggregate.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Hash), c_dp, c_dp]
    lib.dragg_mpc_season_noise.argtypes = [ctypes.POINTER(Dims), ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, c_dp, c_dp]
    lib.dragg_mpc_lag_reset.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Lag), ctypes.c_int32, c_dp]
    for f in (lib.dragg_mpc_step_main, lib.dragg_mpc_step_side):
        f.argtypes = [ctypes.POINTER(Dims), ctypes.POINTER(Problem), ctypes.POINTER(Hash), ctypes.POINTER(Out),
                      ctypes.c_int32, ctypes.POINTER(Lag), c_dp]
    lib.dragg_mpc_aggregate_rows.argtypes = [ctypes.POINTER(Dims), c_dp, ctypes.c_int32, c_dp, c_dp]
    if lib.dragg_mpc_abi_version() != ABI_VERSION:
        raise DraggError("ABI version mismatch between dragg_amd and libdragg_mi355x.so")
    if not os.environ.get("DRAGG_LIB"):
        from . import build as B
        if B.sources_present() and lib.dragg_mpc_source_hash().decode() != B.source_hash():
            raise DraggError(f"{path}: the loaded library's source stamp is not the sources'")
    _LIB = lib
    return lib


def side_grid(dims):
    """The lag mode's side-pass grids (hot, mid, big, step-function) for these dims under the current
    knobs (DRAGG_SIDE_GRID clamped to each launch's per-block scratch; host-only query)."""
    g = (ctypes.c_int32 * 4)()
    check(load().dragg_mpc_side_grid(ctypes.byref(dims), g))
    return list(g)


def reload_knobs():
    """Re-read the diagnostic environment knobs (DRAGG_WAVES_PER_HOME, DRAGG_FORCE_STEP_DP): the library
    reads them once when it loads, never per step."""
    load().dragg_mpc_reload_knobs()


def kernel_info(dims):
    """The launches' registers, spills, LDS and resident workgroups per CU on the current device
    (dragg_mpc_kernel_info_get): {launch name: dict} for the hot, big, mid and narrow launches."""
    info = KernelInfo()
    check(load().dragg_mpc_kernel_info_get(ctypes.byref(dims), ctypes.byref(info)))
    return {LAUNCH_NAMES[i]: {"vgprs": info.vgprs[i], "scratch_bytes_per_lane": info.scratch_bytes[i],
                              "lds_bytes": info.lds_bytes[i], "threads": info.threads[i],
                              "blocks_per_cu": info.blocks_per_cu[i]} for i in range(NLAUNCH)}


def check(rc):
    if rc != 0:
        raise DraggError(f"dragg_mpc error {rc}: {load().dragg_mpc_strerror(rc).decode()}")
    return rc


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None, device=None):
    """The launch stream: `stream`, else the current stream of `device` (of the current device
    when None)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)
