"""Helpers for the golden fixtures (tests/golden/*.json.gz, made by make_golden.py)."""
import functools
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(maxsize=None)
def load(name):
    with gzip.open(os.path.join(GOLDEN, f"{name}.json.gz"), "rt") as f:
        return json.load(f)


def config_text(params):
    """The scenario's config.toml (tests/golden/config_template.toml, as make_golden.py wrote it)."""
    with open(os.path.join(GOLDEN, "config_template.toml")) as f:
        return f.read().format(**params)


def scenarios():
    return sorted(f[:-8] for f in os.listdir(GOLDEN) if f.endswith(".json.gz"))


def explicit_inputs(d, records):
    """Stack per-record solve inputs into the [N] / [H+1][N] arrays of solve_explicit."""
    homes = {h["name"]: h for h in d["homes"]}
    hl = [homes[r["name"]] for r in records]
    col = lambda k: np.array([r[k] for r in records], dtype=float).T  # noqa: E731
    return hl, dict(
        t=np.array([r["t"] for r in records], dtype=np.int32),
        T0=np.array([r["T0"] for r in records]),
        Tw0=np.array([r["Tw0"] for r in records]),
        E0=np.array([np.nan if r["E0"] is None else r["E0"] for r in records]),
        counter=np.array([r["counter_in"] for r in records], dtype=np.int32),
        winter=np.array([1 if r["season"] == "winter" else 0 for r in records], dtype=np.int32),
        draw=col("draw_size"), oat=col("oat"), ghi=col("ghi"), price=col("total_price"),
    )


def prev_hash_arrays(records, H, fc_keys, val_keys):
    """fc [NFC][H][N] and vals [NVAL][N] from the records' previous redis hashes (NaN = absent)."""
    N = len(records)
    fc = np.full((len(fc_keys), H, N), np.nan)
    vals = np.full((len(val_keys), N), np.nan)
    for i, r in enumerate(records):
        for k, v in r["prev_hash"].items():
            name, _, j = k.rpartition("_")
            if name in fc_keys and j.isdigit():
                fc[fc_keys.index(name), int(j), i] = float(v)
            elif k in val_keys:
                vals[val_keys.index(k), i] = float(v)
    return fc, vals
