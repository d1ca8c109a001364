set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_41; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3.json 2> $O/b_cfg3.err
TPE_ROW_SPLIT_MAX=65536 TPE_SORT_SPLIT_MAX=262144 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_two_s4k.json 2> $O/b_cfg3_two_s4k.err
TPE_ROW_SPLIT_MAX=65536 TPE_SORT_SPLIT_MAX=262144 TPE_MOMENT=0 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_two_s4k_nomom.json 2> $O/b_cfg3_two_s4k_nomom.err
TPE_ROW_SPLIT_MAX=65536 TPE_MOMENT=0 timeout -k 10 300 python -u bench.py --config cfg3 --steps 100 $P > $O/b_cfg3_two_nomom.json 2> $O/b_cfg3_two_nomom.err
TPE_ROW_SPLIT_MAX=65536 TPE_SORT_SPLIT_MAX=262144 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/cfg3 -o run -- python -u bench.py --config cfg3 --steps 30 $P > $O/cfg3.log 2>&1
python tools/step_timeline.py $O/cfg3 > $O/cfg3_timeline.txt 2>&1
find $O -name "*.db" -delete; find $O -name "*_trace.csv" -size +4M -delete
echo done
