#!/bin/bash
# rocprofv3 passes over a short bench run (one counter group per pass, each under its own
# time limit).  Output: gpurun_out/prof/<pass>/...  Usage: bash tools/gpu_profile.sh [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${@:-"--cpu-seconds 0"}          # the bench's default workload (96 steps), CPU leg skipped
timeout -k 10 120 rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
pass() {
    name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH || exit 1
pass sq3 SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT || exit 1
pass sq4 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
if [ -f abl/stats.so ] && [ -z "$NO_STATS" ]; then
  DRAGG_LIB=$PWD/abl/stats.so timeout -k 10 200 python tools/front_stats.py --json $OUT/front_stats.json -- $ARGS > $OUT/front_stats.log 2>&1 || exit 1
fi
echo done
