set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_49; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_parallel.py tests/test_gpu_suggest.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for c in cfg2 cfg4; do timeout -k 10 300 python -u tools/exchange_time.py --config $c > $O/exchange_$c.json 2> $O/exchange_$c.err; done
for i in 1 2; do timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 --warmup 5 --parallelism sharded $P > $O/b_cfg2_sharded_$i.json 2> $O/b_cfg2_sharded_$i.err; done
echo done
