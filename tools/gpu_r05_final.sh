#!/bin/bash
# Round-5 final check on the committed build: the GPU test suite, smoke(), the round's bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=final TESTS=tests TEST_LIMIT=900 LINES="driver full96 shard8maxd rl cfg1 shard8max" LINE_LIMIT=400 bash tools/gpu_r05.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
