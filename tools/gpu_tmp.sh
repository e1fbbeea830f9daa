set -o pipefail
bash tools/gpu_final.sh || exit 1
bash tools/gpu_profile.sh || exit 1
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace1250 -o trace -- python3 bench.py --cpu-seconds 0 --homes 1250 > gpurun_out/prof/trace1250.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/tracerl -o trace -- python3 bench.py --cpu-seconds 0 --workload rl --steps 8 > gpurun_out/prof/tracerl.log 2>&1 || exit 1
timeout -k 10 200 python tools/count_paths.py 10000 12 16 7 rl 2>&1 | grep -v amdgpu.ids || exit 1
