set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_34; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/r634 -o run -- python -u bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/cfg3.log 2>&1
python tools/host_lag.py /tmp/r634 > $O/host_lag_cfg3.txt 2>&1
echo done
