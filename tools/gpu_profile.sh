#!/bin/bash
# rocprofv3 passes over a short bench run (one counter group per pass, each under its own
# time limit).  Output: gpurun_out/prof/<pass>/...  Usage: bash tools/gpu_profile.sh [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${@:-"--homes 10000 --horizon-hours 12 --month 7 --steps 6 --warmup 1 --cpu-seconds 0"}
timeout -k 10 120 rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
pass() {
    name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
echo done
