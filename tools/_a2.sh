set -o pipefail
T=${T:-a2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
DRAGG_LIB=varlib/stprof.so timeout -k 10 300 python3 tools/step_prof.py --steps 52 > gpurun_out/$T/step_prof.txt 2>&1 || { echo stprof failed; tail -5 gpurun_out/$T/step_prof.txt; exit 1; }
tail -3 gpurun_out/$T/step_prof.txt
timeout -k 10 300 python3 tools/ab_equal.py --dump /tmp/new.npz --steps 52 --first 34 > gpurun_out/$T/ab_new.log 2>&1 || { echo dump failed; tail -5 gpurun_out/$T/ab_new.log; exit 1; }
DRAGG_LIB=varlib/r04.so timeout -k 10 300 python3 tools/ab_equal.py --dump /tmp/old.npz --steps 52 --first 34 > gpurun_out/$T/ab_old.log 2>&1 || { echo dump failed; tail -5 gpurun_out/$T/ab_old.log; exit 1; }
python3 tools/ab_equal.py --compare /tmp/old.npz /tmp/new.npz | tail -5
TAG=$T TESTS=none LINES="full96" bash tools/gpu_r05.sh
