set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_16; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
for c in cfg2 cfg3 cfg4; do timeout -k 10 300 python -u tools/exchange_time.py --config $c > $O/exchange_$c.json 2> $O/exchange_$c.err; done
timeout -k 10 300 python -u bench.py --steps 5 --parallelism sharded $P > $O/b_cfg4_sharded.json 2> $O/b_cfg4_sharded.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 --parallelism sharded $P > $O/b_cfg2_sharded.json 2> $O/b_cfg2_sharded.err
for c in cfg4 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${c}_trace -o run -- python -u bench.py --config $c --steps 1 --warmup 1 $P > $O/${c}_trace.log 2>&1
done
python tools/rocpd_stats.py $O/cfg4_trace $O/cfg5_trace > $O/rocpd.log 2>&1
find $O -name '*.db' -delete
echo done
