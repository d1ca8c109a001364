set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_46; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4_2048.json 2> $O/b_cfg4_2048.err
for mb in 4096 8192; do
  TPE_CHUNK_MB=$mb timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4_$mb.json 2> $O/b_cfg4_$mb.err
done
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_2048_b16.json 2> $O/b_cfg5_2048_b16.err
for mb in 4096 8192; do
  TPE_CHUNK_MB=$mb timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5_${mb}_b16.json 2> $O/b_cfg5_${mb}_b16.err
  TPE_CHUNK_MB=$mb timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 --batch 32 $P > $O/b_cfg5_${mb}_b32.json 2> $O/b_cfg5_${mb}_b32.err
done
echo done
