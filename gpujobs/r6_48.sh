set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_48; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u bench.py --steps 5 --parallelism sharded $P > $O/b_cfg4_sharded.json 2> $O/b_cfg4_sharded.err
timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4_single.json 2> $O/b_cfg4_single.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 --warmup 5 --parallelism sharded $P > $O/b_cfg2_sharded.json 2> $O/b_cfg2_sharded.err
timeout -k 10 300 python -u tools/exchange_time.py --config cfg4 > $O/exchange_cfg4.json 2> $O/exchange_cfg4.err
echo done
