set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_39; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 $P > $O/b_cfg4.json 2> $O/b_cfg4.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5.json 2> $O/b_cfg5.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 $P > $O/b_cfg3.json 2> $O/b_cfg3.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 $P > $O/b_cfg2.json 2> $O/b_cfg2.err

timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/cfg3 -o run -- python -u bench.py --config cfg3 --steps 30 $P > $O/cfg3.log 2>&1
python tools/step_timeline.py $O/cfg3 > $O/cfg3_timeline.txt 2>&1
find $O -name "*.db" -delete; find $O -name "*_trace.csv" -size +4M -delete
echo done
