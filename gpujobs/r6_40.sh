set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_40; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3.json 2> $O/b_cfg3.err
TPE_ROW_SPLIT_MAX=65536 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_two.json 2> $O/b_cfg3_two.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_b.json 2> $O/b_cfg3_b.err
TPE_ROW_SPLIT_MAX=65536 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_two_b.json 2> $O/b_cfg3_two_b.err
echo done
