#!/bin/bash
# SQ counters of k_fit on a config-2 bench run (separate --pmc passes, CSV
# output).  Diagnostic only.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/fitpmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    --output-format csv -d $O/p1 -o run -- python -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT \
    --output-format csv -d $O/p2 -o run -- python -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/p2.log 2>&1
echo done
