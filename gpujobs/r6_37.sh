set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_37; mkdir -p $O
TPE_STAMPS_SLOTS=6 timeout -k 10 300 python -u tools/fit_stamps.py cfg3 > $O/fit_stamps_cfg3.txt 2>&1
TPE_STAMPS_SLOTS=4 timeout -k 10 300 python -u tools/fit_stamps.py cfg2 > $O/fit_stamps_cfg2.txt 2>&1
echo done
