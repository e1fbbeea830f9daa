#!/bin/bash
# One GPU session: host probe, the GPU test suite, the driver's bench command, and the rocprofv3
# passes of that same command (kernel trace, SQ / FETCH / WRITE PMC passes, DP work from the stats
# variant).  Every GPU step has its own time limit; the first failure ends the script.
# Usage: bash tools/gpu_measure.sh TAG [bench args]   (default: the driver's command)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
ARGS=${@:-"--gpus 1 --steps 20 --warmup 5"}
OUT=gpurun_out/$TAG
mkdir -p $OUT/prof
{
  echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "MAX_JOBS=$MAX_JOBS OMP_NUM_THREADS=$OMP_NUM_THREADS"
  free -g | head -2
} > $OUT/host.txt 2>&1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu.txt; exit 1; }
  tail -3 $OUT/pytest_gpu.txt
fi
timeout -k 10 600 python3 bench.py $ARGS > $OUT/bench_line.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_line.json
PARGS="$ARGS --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o trace -- python3 bench.py $PARGS > $OUT/prof/trace.log 2>&1 || { echo "trace failed"; exit 1; }
pass() {
    name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/prof/$name -o $name -- python3 bench.py $PARGS > $OUT/prof/$name.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || { echo "sq1 failed"; exit 1; }
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH || { echo "sq2 failed"; exit 1; }
pass sq3 SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT || { echo "sq3 failed"; exit 1; }
pass sq4 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU || { echo "sq4 failed"; exit 1; }
pass fetch FETCH_SIZE || { echo "fetch failed"; exit 1; }
pass write WRITE_SIZE || { echo "write failed"; exit 1; }
if [ -f varlib/stats.so ] && [[ "$ARGS" != *"--workload rl"* ]]; then
  DRAGG_LIB=varlib/stats.so timeout -k 10 300 python3 tools/front_stats.py --json $OUT/prof/front_stats.json -- $PARGS > $OUT/prof/front_stats.log 2>&1 || { echo "front_stats failed"; exit 1; }
fi
echo measure-done
