"""The committed measurement is reproducible from the committed profiles:
profiles/r0{3,5}/traffic_*.json recompute from the raw rocprofv3 passes under profiles/r0{3,5}/*_prof
(tools/make_traffic.py), and the committed bench lines' kernel time and derived rooflines agree with
the profile of the same command and window (within 5 %)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = {
    "driver": ["--steps", "20", "--warmup", "5"],
    "rl": ["--steps", "6", "--warmup", "1", "--workload", "rl", "--rl-price", "smooth", "--forecast-horizon", "1"],
}
# (round, the bench line of each workload measured on that round's build)
ROUNDS = {"r03": "bench_{}_line.json", "r05": os.path.join("lines", "{}.json")}


@pytest.mark.parametrize("rnd", sorted(ROUNDS))
@pytest.mark.parametrize("name", sorted(ARGS))
def test_traffic_recomputes_from_raw_passes(rnd, name, tmp_path):
    P = os.path.join(ROOT, "profiles", rnd)
    args = ARGS[name]
    prof = os.path.join(P, f"{name}_prof")
    if not os.path.isdir(prof):
        pytest.skip("no raw profile passes")
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_traffic.py"), "--prof", prof, "--out", str(out)]
                   + args, check=True, capture_output=True)
    got = json.load(open(out))
    ref = json.load(open(os.path.join(P, f"traffic_{name}.json")))
    assert got["workload"] == ref["workload"]
    assert got["kernel_ms_per_step"] == pytest.approx(ref["kernel_ms_per_step"], rel=1e-12)
    assert got["bytes_per_step"] == pytest.approx(ref["bytes_per_step"], rel=1e-12)
    for k, v in ref["sq_per_step"].items():
        assert got["sq_per_step"][k] == pytest.approx(v, rel=1e-12), k


@pytest.mark.parametrize("rnd", sorted(ROUNDS))
@pytest.mark.parametrize("name", sorted(ARGS))
def test_bench_line_agrees_with_its_profile(rnd, name):
    sys.path.insert(0, ROOT)
    import bench
    P = os.path.join(ROOT, "profiles", rnd)
    line = json.load(open(os.path.join(P, ROUNDS[rnd].format(name))))
    tj = json.load(open(os.path.join(P, f"traffic_{name}.json")))
    r = line["roofline"]
    assert r["profile_key"] == tj["workload"]                     # the same command and window
    assert r["kernel_ms"] == pytest.approx(tj["kernel_ms_per_step"], rel=0.05)
    # the derived rooflines recompute from the profile's own counters and kernel time
    ks = tj["kernel_ms_per_step"] * 1e-3
    cyc = bench.valu_cycles(tj["sq_per_step"])
    assert line["roofline_valu"]["frac"] == pytest.approx(cyc / ks / (bench.N_SIMD * bench.CLOCK), rel=1e-9)
    assert r["traffic"] == pytest.approx(tj["bytes_per_step"] / (r["kernel_ms"] * 1e-3) / 1e9, rel=1e-9)
    if "dp_work" in line:
        assert line["dp_work"]["achieved"] == pytest.approx(tj["front_stats"]["children_per_step"] / ks / 1e9, rel=1e-9)


def _lines(rnd):
    d = os.path.join(ROOT, "profiles", rnd, "lines")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".json")) if os.path.isdir(d) else []


@pytest.mark.parametrize("rnd", ["r06"])
def test_every_line_cites_only_its_own_workloads_counters(rnd):
    """a committed line takes its counters (roofline.traffic, the VALU / LDS
    rooflines) only from a rocprofv3 pass of its own command -- the same workload, window, shard and steps
    mode (bench.traffic_key since round 6) -- and has traffic null otherwise."""
    lines = _lines(rnd)
    if not lines:
        pytest.skip("no committed lines of this round")
    for path in lines:
        line = json.load(open(path))
        r = line.get("roofline") or {}
        key = r.get("profile_key")
        if line.get("metric", "").startswith("end-to-end"):
            continue
        assert key, path
        shard = line.get("shard_emulation")
        assert (", shard " in key) == bool(shard), (path, key)
        if shard:
            rank = "max" if shard.get("max_over_shards") else shard["shard_rank"]
            assert f", shard {rank} of {shard['shard_of']}" in key, (path, key)
        assert key.endswith(f", {line['steps_mode']} steps"), (path, key)
        src = r.get("traffic_source")
        if src is None:
            assert r.get("traffic") is None and "roofline_valu" not in line, path
            continue
        tj = json.load(open(os.path.join(ROOT, src)))
        assert tj["workload"] == key, (path, src)
        assert os.path.dirname(src).endswith(rnd), (path, src)            # this round's build
