#!/bin/bash
# Round-5 profiling call: kernel traces of the 8-way straggler shard (lag mode and serial steps), then
# the rocprofv3 passes (tools/gpu_profile.sh) of the driver window and of the RL workload, each moved to
# its own directory under gpurun_out/.  Every GPU step runs under its own limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=tr1 TESTS=none LINES=none TRACE="shard8m7 shard8m7s" LINE_LIMIT=240 bash tools/gpu_r05.sh || exit 1
rm -rf gpurun_out/prof gpurun_out/prof_driver gpurun_out/prof_rl
bash tools/gpu_profile.sh --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 || exit 1
mv gpurun_out/prof gpurun_out/prof_driver
bash tools/gpu_profile.sh --workload rl --steps 6 --warmup 1 --cpu-seconds 0 || exit 1
mv gpurun_out/prof gpurun_out/prof_rl
echo prof-done
