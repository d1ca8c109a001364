set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_43; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_parallel.py tests/test_gpu_suggest.py tests/test_gpu_big.py > $O/tests.log 2>&1
tail -2 $O/tests.log
for c in cfg2 cfg3 cfg4; do
  timeout -k 10 300 python -u tools/exchange_time.py --config $c > $O/exchange_$c.json 2> $O/exchange_$c.err
  TPE_EXCHANGE_COPY=1 timeout -k 10 300 python -u tools/exchange_time.py --config $c > $O/exchange_${c}_copy.json 2> $O/exchange_${c}_copy.err
done
timeout -k 10 300 python -u bench.py --steps 5 --parallelism sharded $P > $O/b_cfg4_sharded.json 2> $O/b_cfg4_sharded.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 --parallelism sharded $P > $O/b_cfg2_sharded.json 2> $O/b_cfg2_sharded.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/x_trace -o run -- python -u tools/exchange_time.py --config cfg2 > $O/x_trace.log 2>&1
find $O -name '*.db' -delete
echo done
