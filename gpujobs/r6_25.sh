set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_25; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
TPE_MOM16_MIN_K=500 timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_m16.json 2> $O/b_cfg5_m16.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5.json 2> $O/b_cfg5.err
TPE_MOMENT_H=0 TPE_MOM16_MIN_K=500 timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_m16noh.json 2> $O/b_cfg5_m16noh.err
echo done
