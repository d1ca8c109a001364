#!/bin/bash
# One GPU-box pass for a bench config: bench line, rocprofv3 kernel-trace stats
# and separate FETCH_SIZE / WRITE_SIZE PMC passes, each step under its own
# time limit, chained so the first failure ends the script.
#   usage: tools/gpu_profile.sh <cfg> <bench args...>
# outputs: gpurun_out/<cfg>/{bench.json,trace,fetch,write}; fold them into
# profiles/ afterwards with tools/rocpd_stats.py + tools/prof_summary.py.
set -euo pipefail
cfg=$1; shift
export TMPDIR=/tmp
O=gpurun_out/$cfg
mkdir -p "$O"
timeout -k 10 400 python -u bench.py --config "$cfg" "$@" > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- \
    python -u bench.py --config "$cfg" "$@" --no-cpu-baseline --no-e2e > "$O/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run -- \
    python -u bench.py --config "$cfg" "$@" --no-cpu-baseline --no-e2e > "$O/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o run -- \
    python -u bench.py --config "$cfg" "$@" --no-cpu-baseline --no-e2e > "$O/write.log" 2>&1
echo "done $cfg"
