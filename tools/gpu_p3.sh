#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
for lib in cur greg; do
  L=""; [ $lib != cur ] && L=$PWD/varlib/$lib.so
  DRAGG_LIB=$L timeout -k 10 200 python3 -u tools/ab_equal.py --dump gpurun_out/ab/$lib.npz --month 7 > gpurun_out/ab/$lib.log 2>&1 || { tail -5 gpurun_out/ab/$lib.log; exit 1; }
done
python3 tools/ab_equal.py --compare gpurun_out/ab/cur.npz gpurun_out/ab/greg.npz | tail -3
rm -f gpurun_out/ab/*.npz
SKIP_TESTS=1 TAG=r03x bash tools/gpu_r03m.sh
