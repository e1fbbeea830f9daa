#!/bin/bash
# Round-5 closing profile on the final build: the rocprofv3 passes (tools/gpu_profile.sh) of the driver
# window and of the RL workload, then (after tools/make_traffic.py has been run on them here, on the box) the
# two bench lines again so that their rooflines come from these passes; a kernel trace of the full day.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/prof gpurun_out/prof2_driver gpurun_out/prof2_rl
bash tools/gpu_profile.sh --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 || exit 1
mv gpurun_out/prof gpurun_out/prof2_driver
bash tools/gpu_profile.sh --workload rl --steps 6 --warmup 1 --cpu-seconds 0 || exit 1
mv gpurun_out/prof gpurun_out/prof2_rl
python3 tools/make_traffic.py --prof gpurun_out/prof2_driver --out profiles/r05/traffic_driver.json --steps 20 --warmup 5 --command "python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0" > /dev/null || exit 1
python3 tools/make_traffic.py --prof gpurun_out/prof2_rl --out profiles/r05/traffic_rl.json --workload rl --steps 6 --warmup 1 --command "python bench.py --workload rl --steps 6 --warmup 1 --cpu-seconds 0" > /dev/null || exit 1
cp profiles/r05/traffic_driver.json profiles/r05/traffic_rl.json gpurun_out/prof2_driver/
TAG=prof2 TESTS=none LINES="driver rl" TRACE="full96" bash tools/gpu_r05.sh || exit 1
echo prof2-done
