set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_14; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
V=$PWD/hyperopt_amd/libtpe_engine_v8k.so
TPE_ENGINE_LIB=$V timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4_v8k.json 2> $O/b_cfg4_v8k.err
timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4.json 2> $O/b_cfg4.err
TPE_ENGINE_LIB=$V timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_v8k.json 2> $O/b_cfg5_v8k.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5.json 2> $O/b_cfg5.err
TPE_ENGINE_LIB=$V timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 $P > $O/b_cfg3_v8k.json 2> $O/b_cfg3_v8k.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 $P > $O/b_cfg3.json 2> $O/b_cfg3.err
TPE_ENGINE_LIB=$V timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/v8k_trace -o run -- python -u bench.py --config cfg5 --steps 1 --warmup 1 $P > $O/v8k_trace.log 2>&1
python tools/rocpd_stats.py $O/v8k_trace > $O/rocpd.log 2>&1
find $O -name '*.db' -delete
echo done
