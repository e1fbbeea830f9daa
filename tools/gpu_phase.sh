set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/phase_breakdown.py --homes 10000 --steps 8 --horizon-hours 12 --month 7 > gpurun_out/phase_r02d.json 2>gpurun_out/phase_r02d.err || { tail -20 gpurun_out/phase_r02d.err; exit 1; }
cat gpurun_out/phase_r02d.json
