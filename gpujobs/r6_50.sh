set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_50; mkdir -p $O
rc=0; timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || rc=$?
tail -1 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
echo done
