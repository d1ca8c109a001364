#!/bin/bash
# k_fit iteration loop on the GPU box: fit parity tests, per-phase stamps
# (diagnostic build) and rocprofv3 kernel stats of the product library on a
# config-2 bench run.  Outputs under gpurun_out/fit/.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/fit
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_ops.py -k "parzen or fit or split or categorical" > $O/tests.log 2>&1
timeout -k 10 120 python -u tools/fit_stamps.py cfg2 > $O/stamps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- \
    python -u bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/trace.log 2>&1
echo done
