set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_19; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
TPE_ENGINE_LIB=$PWD/hyperopt_amd/libtpe_engine_exp.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/exp_trace -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 1 $P > $O/exp_trace.log 2>&1
python tools/rocpd_stats.py $O/exp_trace > $O/rocpd.log 2>&1
find $O -name '*.db' -delete
echo done
