set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_01; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_cfg5.json 2> $O/b_cfg5.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 --no-cpu-baseline --no-e2e > $O/b_cfg3.json 2> $O/b_cfg3.err
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-e2e > $O/b_cfg4.json 2> $O/b_cfg4.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 --no-cpu-baseline --no-e2e > $O/b_cfg2.json 2> $O/b_cfg2.err
echo done
