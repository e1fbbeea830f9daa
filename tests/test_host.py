"""CPU tests of the host side: C ABI library/exports/struct layout, packing, keyed RNG,
synthetic inputs.  No GPU compute here."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dragg_mi355x.h")


@pytest.fixture(scope="module")
def lib_path():
    from dragg_amd import build
    return build.build()


def test_library_exports_every_header_symbol(lib_path):
    names = re.findall(r"^\w[\w\s\*]*?\b(dragg_mpc_\w+)\s*\(", open(HEADER).read(), re.M)
    assert len(names) >= 7
    lib = ctypes.CDLL(lib_path)
    for n in names:
        assert hasattr(lib, n), n
    from dragg_amd import _lib
    assert set(names) == set(_lib.EXPORTS)
    assert lib.dragg_mpc_abi_version() == _lib.ABI_VERSION


def test_results_library_exports_its_header():
    """libdragg_results.so (the host-side results.json formatter) exports include/dragg_results.h."""
    from dragg_amd import build as B
    path = B.build_results()
    names = re.findall(r"^\w[\w\s\*]*?\b(dragg_\w+)\s*\(", open(os.path.join(ROOT, "include", "dragg_results.h")).read(), re.M)
    assert set(names) == {"dragg_results_abi_version", "dragg_fmt_double", "dragg_fmt_series"}
    lib = ctypes.CDLL(path)
    for n in names:
        assert hasattr(lib, n), n
    assert not B.results_needs_build()


def test_ctypes_structs_match_c_layout(tmp_path):
    """sizeof/offsetof of every ABI struct, from gcc, against the ctypes mirrors."""
    from dragg_amd import _lib as L
    structs = {"dragg_mpc_dims": L.Dims, "dragg_mpc_problem": L.Problem, "dragg_mpc_hash": L.Hash,
               "dragg_mpc_out": L.Out, "dragg_mpc_explicit": L.Explicit}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', 'int main(void){']
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append('return 0;}')
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(line.split() for line in out if line)
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_enums_match_header():
    from dragg_amd import _lib as L
    h = open(HEADER).read()
    assert "DRAGG_NFC" in h and len(L.FC_KEYS) == 15 and len(L.VAL_KEYS) == 19
    # order of the fc keys in the header enum
    body = h[h.index("enum dragg_fc_key"):h.index("DRAGG_NFC\n")]
    keys = re.findall(r"DRAGG_K_(\w+)", body)
    want = ["P_GRID", "FORECAST_P_GRID", "P_LOAD", "TEMP_IN_EV", "TEMP_WH_EV", "HVAC_COOL", "HVAC_HEAT",
            "WH_HEAT", "COST", "WATERDRAWS", "P_PV", "U_PV_CURT", "P_BATT_CH", "P_BATT_DISCH", "E_BATT"]
    assert keys == want
    pbody = h[h.index("enum dragg_param"):h.index("DRAGG_NPARAM\n")]
    assert re.findall(r"DRAGG_P_(\w+)", pbody) == L.PARAMS


def test_pack_homes_matches_reference_constants():
    """pack_homes reproduces setup_base/battery/pv_problem's derived constants exactly."""
    from dragg_amd import _lib as L
    from dragg_amd.mpc import pack_homes
    from oracle import mpc as M
    from tests import fixtures as F
    d = F.load("c1_h24")
    P, types, draws, dm = pack_homes(d["homes"])
    assert (dm["S"], dm["dt"], dm["H"]) == (6, 4, 24)
    for i, h in enumerate(d["homes"]):
        hc = M.home_const(h)
        assert P[L.P["R"], i] == hc.R and P[L.P["C"], i] == hc.C and P[L.P["PC"], i] == hc.Pc
        assert P[L.P["PH"], i] == hc.Ph and P[L.P["RW"], i] == hc.Rw and P[L.P["PW"], i] == hc.Pw
        assert P[L.P["CW"], i] == hc.Cw and P[L.P["V"], i] == hc.V
        assert P[L.P["TMIN"], i] == hc.Tmin and P[L.P["TWMAX"], i] == hc.Twmax
        if hc.has_batt:
            assert P[L.P["EMIN"], i] == hc.batt["Emin"] and P[L.P["EINIT"], i] == hc.batt["E_init"]
        assert types[i] == L.TYPE_CODE[h["type"]]
        assert np.array_equal(draws[:len(hc.draw_sizes), i], hc.draw_sizes)


def philox_np(ctr, key):
    """Philox4x32-10 in numpy (uint64 arithmetic), the generator of the device season noise."""
    c = [np.uint64(x) for x in ctr]
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    M32 = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & M32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return [int(x) for x in c]


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors (kat_vectors)."""
    assert philox_np([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert philox_np([0xffffffff] * 4, [0xffffffff] * 2) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert philox_np([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_synthetic_weather_shapes():
    from dragg_amd.community import synthetic_weather, upsample, tou_hourly
    assert upsample([1, 2, 3, 4], 4).tolist() == [1, 1, 2, 2, 3, 3, 4, 4]      # aggregator.py:140-145
    assert upsample([1, 2], 1).tolist() == [1]
    assert upsample([1, 2], 3).tolist() == [1, 1, 2]
    t = tou_hourly(24)
    assert t[8] == 0.07 and t[9] == 0.09 and t[20] == 0.09 and t[21] == 0.07   # peak overwritten
    oat, ghi, tou = synthetic_weather(3, 4, 30, seed=1)
    assert len(oat) == len(ghi) == len(tou) == 3 * 24 * 4
    assert np.all(oat == np.trunc(oat)) and ghi.min() >= 0
    assert tou[-1] == tou[29 * 4]                                              # forward fill


def test_synthetic_homes_schema():
    from dragg_amd.community import synthetic_homes
    from dragg_amd.mpc import pack_homes
    homes = synthetic_homes(50, seed=3, days=2)
    types = [h["type"] for h in homes]
    assert types.count("base") == 20 and types.count("pv_battery") == 10
    P, ty, dr, dm = pack_homes(homes)
    assert dr.shape == (48, 50) and dm["H"] == 24
    for h in homes:
        assert h["hvac"]["temp_in_min"] < h["hvac"]["temp_in_init"] < h["hvac"]["temp_in_max"]
        assert max(h["wh"]["draw_sizes"]) <= h["wh"]["tank_size"]


def test_reward_price_length_rule():
    """mpc_calc.py:353 raises unless len(rp) is 1 or >= H; the host mirrors that."""
    from dragg_amd.mpc import MPCBatch
    with pytest.raises(ValueError):
        MPCBatch.set_reward_price(type("B", (), {"H": 24, "device": "cpu", "dims": type("D", (), {})()})(),
                                  [0.0] * 4)


def test_size_queries_without_gpu(lib_path):
    """dragg_mpc_lds_bytes / dragg_mpc_workspace_bytes are host-only queries (no GPU needed)."""
    from dragg_amd import _lib as L
    lib = L.load()
    d = L.Dims(n_homes=100, horizon=24, sub_steps=6, dt=4, n_draw_hours=48, n_env=0, n_rp=1,
               int_mode=L.INT_ROUND, max_iter=0, check_every=0, discount=0.92)
    ws = lib.dragg_mpc_workspace_bytes(ctypes.byref(d))
    # u16 back-pointer per front label and stage (NB_CAP = 336), rounded to 256 B, then the
    # [N][8H] f64 stage-slot solutions and the [N] i32 list (+ its length) of the homes deferred to
    # the second launch, then (256-aligned) the second launch's back-pointer rows [512 blocks][H][NF_BIG =
    # 2048] u16, then (256-aligned) the [N] i32 list (+ length) of homes for the step-function DP launch and
    # (256-aligned) its storage: min(N, 16) block slots of ([2][2^20] f64 breakpoints / values,
    # [2][8 x 32768] i32 merge ids, [2][256][64] (x, v) LP rows)
    par = (100 * 24 * 336 * 2 + 255) // 256 * 256
    defer = par + 100 * 8 * 24 * 8
    big_off = (defer + 102 * 4 + 255) // 256 * 256
    nl_off = (big_off + 512 * 24 * 2048 * 2 + 255) // 256 * 256
    nr_off = (nl_off + 102 * 4 + 255) // 256 * 256
    # then (256-aligned) the [N] i32 list (+ length) the mid launch hands to the big one and
    # (256-aligned) the mid launch's back-pointer rows [2048 blocks][H][NF_MID = 384] u16
    slot = 2 * 2 ** 20 * 8 + 2 * 8 * 32768 * 4 + 2 * 256 * 64 * 16
    ml_off = (nr_off + 16 * slot + 255) // 256 * 256
    mr_off = (ml_off + 102 * 4 + 255) // 256 * 256
    # then (256-aligned) the front DP's LP cost-to-go rows [N][H + 1][64] (x, v)
    w_off = (mr_off + 2048 * 24 * 384 * 2 + 255) // 256 * 256
    assert ws == (w_off + 100 * 25 * 64 * 16 + 255) // 256 * 256
    # the lag mode's side workspace: the lists and per-block scratch only, [defer, w_off)
    lib.dragg_mpc_side_workspace_bytes.restype = ctypes.c_int64
    assert lib.dragg_mpc_side_workspace_bytes(ctypes.byref(d)) == w_off - defer
    lds_direct = lib.dragg_mpc_lds_bytes(ctypes.byref(d))
    assert 0 < lds_direct <= 13 * 1024                 # the hot launch: >= 12 homes per CU at H = 24
    d.horizon = 48
    assert 0 < lib.dragg_mpc_lds_bytes(ctypes.byref(d)) <= 13 * 1024   # and at H = 48
    d.horizon = 24
    d.int_mode = L.INT_RELAX
    assert lib.dragg_mpc_workspace_bytes(ctypes.byref(d)) == 0
    assert lib.dragg_mpc_lds_bytes(ctypes.byref(d)) > lds_direct
    d.int_mode = 9
    assert lib.dragg_mpc_workspace_bytes(ctypes.byref(d)) < 0
    d.int_mode = L.INT_ROUND
    d.horizon = 400                                    # LP kernel's LDS is the binding limit
    d.int_mode = L.INT_RELAX
    assert lib.dragg_mpc_lds_bytes(ctypes.byref(d)) == -4


def test_side_grid_clamped_to_scratch_slots(lib_path, monkeypatch):
    """DRAGG_SIDE_GRID entries are clamped to each side launch's per-block scratch: the
    step-function launch's narrow_slots(N) = min(N, 16) pools, the big launch's 512 and the mid launch's
    2,048 rows, and to one block per home."""
    from dragg_amd import _lib as L
    d = L.Dims(n_homes=1000, horizon=48, sub_steps=6, dt=4, n_draw_hours=48, n_env=0, n_rp=1,
               int_mode=L.INT_ROUND, max_iter=0, check_every=0, discount=0.92)
    try:
        monkeypatch.delenv("DRAGG_SIDE_GRID", raising=False)
        L.reload_knobs()
        assert L.side_grid(d) == [16, 16, 16, 2]
        monkeypatch.setenv("DRAGG_SIDE_GRID", "5000,4096,9999,32")
        L.reload_knobs()
        assert L.side_grid(d) == [1000, 1000, 512, 16]
        d.n_homes = 3000
        assert L.side_grid(d) == [3000, 2048, 512, 16]
        d.n_homes = 5
        assert L.side_grid(d) == [5, 5, 5, 5]
        monkeypatch.setenv("DRAGG_SIDE_GRID", "0,-3,1,1")
        L.reload_knobs()
        assert L.side_grid(d) == [5, 5, 1, 1]
    finally:
        monkeypatch.delenv("DRAGG_SIDE_GRID", raising=False)
        L.reload_knobs()


def test_stale_library_refused(tmp_path, monkeypatch, lib_path):
    """The library carries its sources' sha-256 (dragg_amd/build.py); the loader refuses one whose stamp
    is not the sources' beside it."""
    from dragg_amd import _lib as L, build as B
    assert B.stamp_of(lib_path) == B.source_hash()
    assert not B.needs_build()
    L.check_stamp(lib_path)                           # the fresh build passes
    assert ctypes.CDLL(lib_path).dragg_mpc_source_hash  # exported
    stale = tmp_path / "stale.so"
    data = open(lib_path, "rb").read().replace(B.STAMP_PREFIX + B.source_hash().encode(),
                                               B.STAMP_PREFIX + b"0" * 64)
    stale.write_bytes(data)
    monkeypatch.setattr(B, "OUT", str(stale))
    monkeypatch.delenv("DRAGG_LIB", raising=False)
    assert B.needs_build()
    with pytest.raises(L.DraggError, match="stale"):
        L.check_stamp(str(stale))


def test_solver_name_plug_point():
    """home['hems']['solver'] (mpc_calc.py:141-145): the MILP backends -- and an unknown name,
    which the reference replaces by GLPK_MI -- select the exact MILP path; ECOS, which cvxpy
    refuses on an integer problem (every solve falls back, mpc_calc.py:450-454), selects the
    always-fallback mode; the build's own int_mode names select themselves."""
    from dragg_amd.calc import int_mode_for
    for name, mode in (("GLPK_MI", "round"), ("GUROBI", "round"), ("ECOS", "fail"), ("nonsense", "round"),
                       ("relax", "relax"), ("round_lp", "round_lp"), ("fail", "fail")):
        assert int_mode_for({"hems": {"solver": name}}) == mode
    assert int_mode_for({"hems": {}}) == "round"


def test_mpccalc_needs_a_community():
    """MPCCalc(home) without a community attaches to the default one; with none it raises."""
    from dragg_amd.calc import Community, MPCCalc
    Community._default = None
    with pytest.raises(RuntimeError):
        MPCCalc({"name": "h", "type": "base", "hems": {"solver": "GLPK_MI"}})
