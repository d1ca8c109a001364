set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_42; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
timeout -k 10 600 python -u bench.py > $O/b_default.json 2> $O/b_default.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 $P > $O/b_cfg2.json 2> $O/b_cfg2.err
echo done
