"""Outputs of a dragg run: collected data, Summary, results.json, the community file.

SURVEY.md §8 row F1.  During a run the per-step hash fields stay on the GPU
(`DeviceAggregator.hist`, [T][19][N]); these functions turn them into the reference's files:

* `new_collected`       aggregator.py:589-615  `reset_collected_data` (key order kept)
* `append_history`      aggregator.py:737-750  `collect_data` (a field absent from the hash is
                        skipped; a field a fallback step did not rewrite is appended again,
                        as the reference re-reads the stale redis value)
* `aggregate_loads`     aggregator.py:748-751  np.sum over the homes' p_grid_opt, in home order
* `summary`             aggregator.py:783-816  `summarize_baseline` (incl. the trailing comma
                        that makes TOU / SPP a one-element tuple, written as [[...]])
* `run_dir`             aggregator.py:818-829  `set_run_dir`
* `write_results`       aggregator.py:831-844  `write_outputs`
* `write_home_configs`  aggregator.py:846-854
* `checkpoint_interval` aggregator.py:949-955
"""
import ctypes
import json
import os
from json.encoder import encode_basestring_ascii

import numpy as np

from . import _lib as L

BASE_KEYS = ["p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "temp_in_opt", "temp_wh_opt",
             "hvac_cool_on_opt", "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws",
             "correct_solve"]


def collect_keys(home_type):
    """The hash fields collect_data appends for a home type (aggregator.py:741-745)."""
    keys = list(BASE_KEYS)
    if "pv" in home_type:
        keys += ["p_pv_opt", "u_pv_curt_opt"]
    if "battery" in home_type:
        keys += ["p_batt_ch", "p_batt_disch", "e_batt_opt"]
    return keys


def new_collected(homes):
    """Per-home series, initial entries included (aggregator.py:589-615)."""
    out = {}
    for h in homes:
        d = {"type": h["type"], "temp_in_sp": h["hvac"]["temp_in_sp"], "temp_wh_sp": h["wh"]["temp_wh_sp"],
             "temp_in_opt": [h["hvac"]["temp_in_init"]], "temp_wh_opt": [h["wh"]["temp_wh_init"]]}
        for k in ("p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "hvac_cool_on_opt", "hvac_heat_on_opt",
                  "wh_heat_on_opt", "cost_opt", "waterdraws", "correct_solve"):
            d[k] = []
        if "pv" in h["type"]:
            d["p_pv_opt"] = []
            d["u_pv_curt_opt"] = []
        if "battery" in h["type"]:
            d["e_batt_opt"] = [h["battery"]["e_batt_init"]]
            d["p_batt_ch"] = []
            d["p_batt_disch"] = []
        out[h["name"]] = d
    return out


def append_history(collected, homes, hist):
    """Append steps of the hash history `hist` [T][NVAL][len(homes)] (NaN = field absent)
    to the homes' series, as collect_data does after each step."""
    hist = np.asarray(hist)
    for i, h in enumerate(homes):
        d = collected[h["name"]]
        for k in collect_keys(h["type"]):
            col = hist[:, L.K[k], i]
            d[k].extend(col[~np.isnan(col)].tolist())       # (Python floats of the same values)
    return collected


def aggregate_loads(hist):
    """Per-step community load: np.sum of the homes' p_grid_opt in home order
    (aggregator.py:748-751), from the hash history [T][NVAL][N]."""
    p = np.asarray(hist)[:, L.K["p_grid_opt"], :]
    return [np.sum([float(v) for v in row]) for row in p]


def summary(case, start, end, solve_time, horizon, num_homes, agg_loads, oat, ghi, rps, sps,
            tou=None, spp=None):
    """The results' "Summary" entry (aggregator.py:795-816)."""
    s = {"case": case, "start_datetime": start.strftime("%Y-%m-%d %H"),
         "end_datetime": end.strftime("%Y-%m-%d %H"), "solve_time": solve_time, "horizon": horizon,
         "num_homes": num_homes, "p_max_aggregate": max(agg_loads), "p_grid_aggregate": list(agg_loads),
         "OAT": list(oat), "GHI": list(ghi), "RP": list(rps), "p_grid_setpoint": list(sps)}
    if spp is not None:
        s["SPP"] = (list(spp),)
    else:
        s["TOU"] = (list(tou),)
    return s


def run_dir(outputs_dir, start, end, check_type, n_homes, horizon, dt_interval, sub_steps, solver, version):
    """outputs/<start>_<end>/<check>-homes_<N>-horizon_<h>-interval_<m>-<m//S>-solver_<s>/version-<v>
    (aggregator.py:818-829)."""
    date = f"{start.strftime('%Y-%m-%dT%H')}_{end.strftime('%Y-%m-%dT%H')}"
    mpc = (f"{check_type}-homes_{n_homes}-horizon_{horizon}-interval_{dt_interval}-"
           f"{dt_interval // sub_steps}-solver_{solver}")
    return os.path.join(outputs_dir, date, mpc, f"version-{version}")


def write_results(rdir, case, collected):
    """<run_dir>/<case>/results.json, indent 4 (aggregator.py:839-844): the bytes json.dump writes
    (dump_json)."""
    case_dir = os.path.join(rdir, case)
    os.makedirs(case_dir, exist_ok=True)
    path = os.path.join(case_dir, "results.json")
    dump_json(collected, path)
    return path


def _summary_part(summary_, lead):
    pieces, lists = [], []
    _layout(summary_, 1, pieces, lists)
    num = format_float_lists(lists)
    out = [(lead + '"Summary": ').encode("ascii")]
    for p in pieces:
        out.append(p.encode("ascii") if type(p) is str else num[p])
    out.append(b"\n}")
    return b"".join(out)


def write_results_history(rdir, case, all_homes, checked, hist, summary_, cache=None):
    """write_results(rdir, case, collected) for collected = new_collected(all_homes) + append_history(
    checked, hist) + {"Summary": summary_}, the same bytes, without building the Python lists: every
    home's series comes out of the history array [T][NVAL][len(checked)] (NaN = absent, skipped) and
    goes to the formatter in one call.  Falls back to the generic writer when a home's initial entry
    is not a float (json.dump would render an int as an int).

    `cache` (a dict the caller keeps): a rewrite of the same file for the same history (the reference
    writes results.json at the last checkpoint and again at the end, aggregator.py:768-778, 941-970,
    with only the Summary's solve_time new) keeps the file's homes part and rewrites the Summary."""
    hist = np.asarray(hist, dtype=np.float64)
    T = hist.shape[0]
    path = os.path.join(rdir, case, "results.json")
    sig = (id(all_homes), len(all_homes), id(checked), len(checked), hist.shape,
           hash(hist[-1].tobytes()) if T else 0)
    if cache is not None and path in cache and os.path.isfile(path):
        c_sig, prefix, size, mtime = cache[path]
        st = os.stat(path)
        if c_sig == sig and st.st_size == size and st.st_mtime_ns == mtime:
            tail = _summary_part(summary_, ",\n    " if all_homes else "{\n    ")
            with open(path, "r+b") as f:
                f.seek(prefix)
                f.write(tail)
                f.truncate()
            st = os.stat(path)
            cache[path] = (sig, prefix, st.st_size, st.st_mtime_ns)
            return path
    init_keys = ("temp_in_opt", "temp_wh_opt", "e_batt_opt")

    def init_of(h, k):
        return h["hvac"]["temp_in_init"] if k == "temp_in_opt" else (
            h["wh"]["temp_wh_init"] if k == "temp_wh_opt" else h["battery"]["e_batt_init"])
    pos = {h["name"]: i for i, h in enumerate(checked)}
    for h in all_homes:
        for k in init_keys:
            if (k != "e_batt_opt" or "battery" in h["type"]) and not isinstance(init_of(h, k), float):
                collected = new_collected(all_homes)
                append_history(collected, checked, hist)
                collected["Summary"] = summary_
                return write_results(rdir, case, collected)
    # per key: the [N][T] rows of the checked homes (NaN dropped), an initial entry first where the
    # series has one; one flat array of every series in document order
    keys_all = ["temp_in_opt", "temp_wh_opt", "p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "hvac_cool_on_opt",
                "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws", "correct_solve", "p_pv_opt",
                "u_pv_curt_opt", "e_batt_opt", "p_batt_ch", "p_batt_disch"]
    rows = {}
    for k in keys_all:
        M = np.ascontiguousarray(hist[:, L.K[k], :].T) if T else np.zeros((len(checked), 0))
        ok = ~np.isnan(M)
        rows[k] = (M[ok], np.cumsum(ok.sum(axis=1)))       # values, end offset of each home's run
    seq = []                # (key, home) in document order -> (values array, begin, end) + init
    parts, begins, ends = [], [], []
    base = 0
    key_base = {}
    for k in keys_all:
        v, _ = rows[k]
        key_base[k] = base
        parts.append(v)
        base += v.size
    inits = []
    for h in all_homes:
        t = h["type"]
        ks = ["temp_in_opt", "temp_wh_opt", "p_grid_opt", "forecast_p_grid_opt", "p_load_opt", "hvac_cool_on_opt",
              "hvac_heat_on_opt", "wh_heat_on_opt", "cost_opt", "waterdraws", "correct_solve"]
        if "pv" in t:
            ks += ["p_pv_opt", "u_pv_curt_opt"]
        if "battery" in t:
            ks += ["e_batt_opt", "p_batt_ch", "p_batt_disch"]
        i = pos.get(h["name"])
        for k in ks:
            if i is None:
                b_ = e_ = 0
            else:
                ends_k = rows[k][1]
                b_ = key_base[k] + (int(ends_k[i - 1]) if i > 0 else 0)
                e_ = key_base[k] + int(ends_k[i])
            if k in init_keys:
                inits.append(float(init_of(h, k)))
                seq.append((h, k, len(inits) - 1, b_, e_))
            else:
                seq.append((h, k, -1, b_, e_))
    # one array: the history values, then the initial entries; a series with an initial entry is rendered
    # as that entry, the separator and its history run
    hvals = np.concatenate(parts) if parts else np.zeros(0)
    x = np.concatenate([hvals, np.asarray(inits, dtype=np.float64)])
    ni = hvals.size
    sep = ",\n" + " " * 12
    begins = np.fromiter((b_ for _, _, _, b_, _ in seq), dtype=np.int64, count=len(seq))
    ends = np.fromiter((e_ for _, _, _, _, e_ in seq), dtype=np.int64, count=len(seq))
    body = format_series(x, begins, ends, sep)
    ib = np.fromiter((ni + j for _, _, j, _, _ in seq if j >= 0), dtype=np.int64)
    head = format_series(x, ib, ib + 1, sep)
    sp8 = "\n" + " " * 8
    case_dir = os.path.join(rdir, case)
    os.makedirs(case_dir, exist_ok=True)
    out, size = [], 0
    with open(path, "wb") as f:
        lead = "{\n    "
        si = 0
        hi = 0
        for h in all_homes:
            d = (lead + encode_basestring_ascii(h["name"]) + ": {" + sp8 + '"type": ' + encode_basestring_ascii(h["type"])
                 + "," + sp8 + '"temp_in_sp": ' + _scalar(h["hvac"]["temp_in_sp"]) + "," + sp8 + '"temp_wh_sp": '
                 + _scalar(h["wh"]["temp_wh_sp"]))
            lead = ",\n    "
            out.append(d.encode("ascii"))
            while si < len(seq) and seq[si][0] is h:
                _, k, j, b_, e_ = seq[si]
                out.append(("," + sp8 + '"' + k + '": ').encode("ascii"))
                if j >= 0:
                    out.append(b"[" + sep[1:].encode("ascii"))
                    out.append(head[hi])
                    hi += 1
                    if e_ > b_:
                        out.append(sep.encode("ascii"))
                        out.append(body[si])
                    out.append(b"\n        ]")
                elif e_ > b_:
                    out.append(b"[" + sep[1:].encode("ascii"))
                    out.append(body[si])
                    out.append(b"\n        ]")
                else:
                    out.append(b"[]")
                size += e_ - b_
                si += 1
            out.append(b"\n    }")
            if size > (1 << 20):
                f.write(b"".join(out))
                out, size = [], 0
        f.write(b"".join(out))
        prefix = f.tell()
        f.write(_summary_part(summary_, lead))
    if cache is not None:
        st = os.stat(path)
        cache[path] = (sig, prefix, st.st_size, st.st_mtime_ns)
    return path


def write_home_configs(outputs_dir, homes, n_homes):
    """outputs/all_homes-<N>-config.json (aggregator.py:846-854), as json.dump(indent=4) writes it."""
    path = os.path.join(outputs_dir, f"all_homes-{n_homes}-config.json")
    dump_json(homes, path)
    return path


# ---------------------------------------------------------------------------- the json writer
# json.dump(obj, f, indent=4) renders every number through Python's pure-Python indenting encoder
# and writes each token on its own: ~67 s for a 10k-home x 96-step results.json (the reference's
# cost too).  dump_json writes the SAME bytes: the structure laid out here exactly as
# json.encoder._make_iterencode lays it out (indent 4, item separator ",", key separator ": ",
# ensure_ascii, NaN / Infinity spellings), every non-empty list of floats rendered by
# libdragg_results.so (include/dragg_results.h: repr(float)'s digits and layout, OpenMP over the
# lists).  Byte-identity with json.dump: tests/test_results.py.
_RES = None


def _results_lib():
    global _RES
    if _RES is None:
        from . import build as B
        B.build_results()                      # (a no-op when the in-tree build is fresh)
        lib = ctypes.CDLL(B.RES_OUT)
        lib.dragg_fmt_series.restype = ctypes.c_int64
        lib.dragg_fmt_series.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]
        lib.dragg_fmt_double.restype = ctypes.c_int64
        lib.dragg_fmt_double.argtypes = [ctypes.c_double, ctypes.c_char_p]
        lib.dragg_results_abi_version.restype = ctypes.c_int
        if lib.dragg_results_abi_version() != 1:
            raise RuntimeError("libdragg_results.so: ABI version mismatch")
        _RES = lib
    return _RES


FMT_MAX = 32            # DRAGG_FMT_MAX


_FLOAT_TYPES = {float, np.float64}


def _float_list(o):
    """o is a non-empty list / tuple of floats only (float subclasses such as numpy.float64 included:
    json.dump renders them with float.__repr__ too)."""
    if not o:
        return False
    ts = set(map(type, o))
    return ts <= _FLOAT_TYPES or all(issubclass(t, float) for t in ts)


def format_series(x, begin, end, sep):
    """Lists x[begin[s]:end[s]] of a float64 array, each rendered as json.dump renders a list's numbers
    (repr(float), joined by `sep`) -> one bytes-like object per list (libdragg_results.so)."""
    lib = _results_lib()
    x = np.ascontiguousarray(x, dtype=np.float64)
    begin = np.ascontiguousarray(begin, dtype=np.int64)
    end = np.ascontiguousarray(end, dtype=np.int64)
    n = begin.size
    if n == 0:
        return []
    sepb = sep.encode("ascii")
    cap = (end - begin) * (FMT_MAX + len(sepb))
    ostarts = np.zeros(n, dtype=np.int64)
    if n > 1:
        np.cumsum(cap[:-1], out=ostarts[1:])
    buf = np.empty(int(cap.sum()) + 1, dtype=np.uint8)
    olen = np.zeros(n, dtype=np.int64)
    rc = lib.dragg_fmt_series(x.ctypes.data, begin.ctypes.data, end.ctypes.data, n, sepb, len(sepb), buf.ctypes.data,
                              ostarts.ctypes.data, olen.ctypes.data)
    if rc != 0:
        raise RuntimeError("dragg_fmt_series failed")
    mv = memoryview(buf)
    return [mv[a_:a_ + n_] for a_, n_ in zip(ostarts.tolist(), olen.tolist())]


def format_float_lists(lists):
    """[(values, separator)] -> one bytes-like object per list (the numbers joined by the separator)."""
    import itertools
    if not lists:
        return []
    out = [None] * len(lists)
    groups = {}
    for j, (_, sep) in enumerate(lists):
        groups.setdefault(sep, []).append(j)
    for sep, idx in groups.items():
        lens = np.fromiter((len(lists[j][0]) for j in idx), dtype=np.int64, count=len(idx))
        starts = np.zeros(len(idx) + 1, dtype=np.int64)
        np.cumsum(lens, out=starts[1:])
        x = np.fromiter(itertools.chain.from_iterable(lists[j][0] for j in idx), dtype=np.float64,
                        count=int(starts[-1]))
        for j, m in zip(idx, format_series(x, starts[:-1], starts[1:], sep)):
            out[j] = m
    return out


def _floatstr(o):
    if o != o:
        return "NaN"
    if o == float("inf"):
        return "Infinity"
    if o == -float("inf"):
        return "-Infinity"
    return float.__repr__(o)


def _key(k):
    if isinstance(k, str):
        return k
    if isinstance(k, float):
        return _floatstr(k)
    if k is True:
        return "true"
    if k is False:
        return "false"
    if k is None:
        return "null"
    if isinstance(k, int):
        return int.__repr__(k)
    raise TypeError(f"keys must be str, int, float, bool or None, not {k.__class__.__name__}")


def _scalar(o):
    """json.dump's rendering of a non-container value (None: a container)."""
    if isinstance(o, str):
        return encode_basestring_ascii(o)
    if o is None:
        return "null"
    if o is True:
        return "true"
    if o is False:
        return "false"
    if isinstance(o, int):
        return int.__repr__(o)
    if isinstance(o, float):
        return _floatstr(o)
    if isinstance(o, (list, tuple, dict)):
        return None
    raise TypeError(f"Object of type {o.__class__.__name__} is not JSON serializable")


def _layout(o, level, pieces, lists):
    """json.encoder._make_iterencode's layout at indent 4: text pieces, and (list index) placeholders
    for the lists of floats, whose (values, separator) go to `lists`."""
    s = _scalar(o)
    if s is not None:
        pieces.append(s)
        return
    close = "\n" + " " * (4 * level)
    nl = "\n" + " " * (4 * (level + 1))
    if isinstance(o, dict):
        if not o:
            pieces.append("{}")
            return
        inner_close = nl
        inner_nl = nl + "    "
        lead = "{" + nl
        for k, v in o.items():
            pieces.append(lead + encode_basestring_ascii(k if type(k) is str else _key(k)) + ": ")
            lead = "," + nl
            t = type(v)
            if t is float:
                pieces.append(_floatstr(v))
            elif t is str:
                pieces.append(encode_basestring_ascii(v))
            elif t is list and _float_list(v):           # (the bulk of a results.json: inline)
                pieces.append("[" + inner_nl)
                pieces.append(len(lists))
                lists.append((v, "," + inner_nl))
                pieces.append(inner_close + "]")
            else:
                _layout(v, level + 1, pieces, lists)
        pieces.append(close + "}")
        return
    if not o:
        pieces.append("[]")
        return
    if _float_list(o):
        pieces.append("[" + nl)
        pieces.append(len(lists))
        lists.append((o, "," + nl))
        pieces.append(close + "]")
        return
    lead = "[" + nl
    for v in o:
        pieces.append(lead)
        lead = "," + nl
        _layout(v, level + 1, pieces, lists)
    pieces.append(close + "]")


def dumps_json(obj):
    """json.dumps(obj, indent=4), the same str (dump_json's layout and number rendering)."""
    pieces, lists = [], []
    _layout(obj, 0, pieces, lists)
    num = format_float_lists(lists)
    return "".join(p if isinstance(p, str) else bytes(num[p]).decode("ascii") for p in pieces)


def dump_json(obj, path):
    """json.dump(obj, open(path, "w+"), indent=4), the same bytes (written in large pieces)."""
    pieces, lists = [], []
    _layout(obj, 0, pieces, lists)
    num = format_float_lists(lists)
    with open(path, "wb") as f:
        chunk, size = [], 0
        text = []
        for p in pieces:
            if type(p) is str:
                text.append(p)
                continue
            chunk.append("".join(text).encode("ascii"))
            text = []
            chunk.append(num[p])
            size += len(num[p])
            if size > (8 << 20):
                f.write(b"".join(chunk))
                chunk, size = [], 0
        chunk.append("".join(text).encode("ascii"))
        f.write(b"".join(chunk))


def checkpoint_interval(setting, dt):
    """Steps between checkpoint writes (aggregator.py:949-955)."""
    return {"hourly": dt, "daily": dt * 24, "weekly": dt * 24 * 7}.get(setting, 500)
