set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_35; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
for v in base fork0 side1 graph1; do
  E=""; [ $v = fork0 ] && E="TPE_LOOKUP_FORK=0"; [ $v = side1 ] && E="TPE_SIDE_STREAMS=1"; [ $v = graph1 ] && E="TPE_GRAPH=1"
  env $E timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_$v.json 2> $O/b_cfg3_$v.err
  env $E timeout -k 10 300 python -u bench.py --config cfg2 --steps 200 $P > $O/b_cfg2_$v.json 2> $O/b_cfg2_$v.err
done
echo done
