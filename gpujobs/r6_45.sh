set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_45; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/exch_trace -o run -- python -u tools/exchange_time.py --config cfg2 > $O/exch.log 2>&1
TPE_EXCHANGE_COPY=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/exch_copy_trace -o run -- python -u tools/exchange_time.py --config cfg2 > $O/exch_copy.log 2>&1
python tools/rocpd_stats.py $O/exch_trace $O/exch_copy_trace > $O/rocpd.log 2>&1
timeout -k 10 300 python -u tools/host_split.py cfg1 cfg2 > $O/host_split.txt 2>&1
find $O -name '*.db' -delete
echo done
