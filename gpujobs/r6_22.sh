set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_22; mkdir -p $O
timeout -k 10 300 python -u tools/score_stamps.py cfg5 1000000 > $O/stamps_cfg5.txt 2>&1
TPE_STAMPS_LEVEL=1 timeout -k 10 300 python -u tools/score_stamps.py cfg3 100000 > $O/stamps_cfg3.txt 2>&1
timeout -k 10 300 python -u tools/score_stamps.py cfg4 1000000 > $O/stamps_cfg4.txt 2>&1
echo done
