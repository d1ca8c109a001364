set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_44; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 --warmup 5 --parallelism sharded $P > $O/b_cfg2_sharded_$i.json 2> $O/b_cfg2_sharded_$i.err
TPE_EXCHANGE_COPY=1 timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 --warmup 5 --parallelism sharded $P > $O/b_cfg2_sharded_copy_$i.json 2> $O/b_cfg2_sharded_copy_$i.err
done
timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 --warmup 5 $P > $O/b_cfg2_single.json 2> $O/b_cfg2_single.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 --warmup 5 --parallelism sharded $P > $O/b_cfg3_sharded.json 2> $O/b_cfg3_sharded.err
TPE_EXCHANGE_COPY=1 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 --warmup 5 --parallelism sharded $P > $O/b_cfg3_sharded_copy.json 2> $O/b_cfg3_sharded_copy.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/x_trace -o run -- python -u tools/exchange_time.py --config cfg2 > $O/x_trace.log 2>&1
find $O -name '*.db' -delete
echo done
