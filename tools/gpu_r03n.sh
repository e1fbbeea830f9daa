#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r03n bash tools/gpu_r03m.sh || exit 1
mkdir -p varlib && mv sprof_hold.so varlib/sprof.so
TAG=r03n_s bash tools/gpu_sprof.sh | grep -E "trigger|\"50\"|\"100\""
