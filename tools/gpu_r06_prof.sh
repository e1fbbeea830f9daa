#!/bin/bash
# Round-6 profiling: the rocprofv3 passes (tools/gpu_profile.sh: kernel trace, SQ x4, FETCH, WRITE, front
# statistics) of the bench commands in PROFS, each moved to gpurun_out/r06prof/<name>.  The first failure
# ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06prof
args_of() {
  case $1 in
    driver) echo --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 ;;
    shard8r7d) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-rank 7 ;;
    shard8r0d) echo --steps 20 --warmup 5 --cpu-seconds 0 --shard-of 8 --shard-rank 0 ;;
    rl) echo --workload rl --steps 6 --warmup 1 --cpu-seconds 0 ;;
  esac
}
for P in $PROFS; do
  rm -rf gpurun_out/prof
  ( [ "$P" != driver ] && export NO_STATS=1; bash tools/gpu_profile.sh $(args_of $P) ) || { echo "profile $P failed"; exit 1; }
  rm -rf gpurun_out/r06prof/$P
  mv gpurun_out/prof gpurun_out/r06prof/$P
  echo "profiled $P"
done
echo prof-done
