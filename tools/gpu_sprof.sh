#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sprof}
mkdir -p $OUT
DRAGG_LIB=$PWD/varlib/sprof.so timeout -k 10 200 python3 tools/stage_prof.py --world 8 --steps 96 --out $OUT/stage_1250.json > /dev/null 2> $OUT/s1.err || { echo "stage prof failed"; tail -3 $OUT/s1.err; exit 1; }
DRAGG_LIB=$PWD/varlib/sprof.so timeout -k 10 200 python3 tools/stage_prof.py --world 1 --steps 96 --out $OUT/stage_10k.json > /dev/null 2> $OUT/s2.err || { echo "stage prof 10k failed"; exit 1; }
cat $OUT/stage_1250.json $OUT/stage_10k.json
