#!/bin/bash
# diagnostic: the cost of the hash's forecast-field writes (home innermost, one block per home: every
# lane's store lands in its own cache line) against a home-contiguous layout (varlib/fcT.so; the host
# misreads its fc, timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fct
mkdir -p $OUT
for lib in cur fcT; do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/d_$lib.json 2> $OUT/e.err || { echo "failed"; tail -3 $OUT/e.err; exit 1; }
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 96 --warmup 4 --cpu-seconds 0 > $OUT/f_$lib.json 2> $OUT/e.err || { echo "failed"; exit 1; }
  DRAGG_LIB=$L timeout -k 10 300 python3 bench.py --steps 24 --warmup 2 --cpu-seconds 0 --homes 100000 --horizon-hours 6 > $OUT/c_$lib.json 2> $OUT/e.err || { echo "failed"; exit 1; }
done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/fct/*.json")):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 4), "ms/step")
PY
