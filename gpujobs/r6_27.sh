set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_27; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/cfg3 -o run -- python -u bench.py --config cfg3 --steps 30 --no-cpu-baseline --no-e2e > $O/cfg3.log 2>&1
find $O -name '*.db' -delete
echo done
