#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/nan
mkdir -p $OUT
for lib in cur m1b1 m1b4; do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 200 python3 tools/nan_hunt.py --steps 100 > $OUT/$lib.txt 2>&1 || { echo "$lib failed"; tail -5 $OUT/$lib.txt; exit 1; }
  echo "== $lib"; tail -6 $OUT/$lib.txt
done
