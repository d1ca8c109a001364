set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p2
timeout -k 10 120 python -u tools/fit_stamps.py cfg2 > gpurun_out/p2/fit_stamps_cfg2.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p2/cfg5 -o run -- python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/p2/cfg5.json 2> gpurun_out/p2/cfg5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p2/cfg2 -o run -- python -u bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/p2/cfg2.json 2> gpurun_out/p2/cfg2.err
echo done
