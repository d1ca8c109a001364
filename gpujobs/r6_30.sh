set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_30; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
for v in 1 0; do
TPE_TIGHTEN=$v timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4_t$v.json 2> $O/b_cfg4_t$v.err
TPE_TIGHTEN=$v timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_t$v.json 2> $O/b_cfg5_t$v.err
TPE_TIGHTEN=$v timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 $P > $O/b_cfg3_t$v.json 2> $O/b_cfg3_t$v.err
done
echo done
