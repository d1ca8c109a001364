set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_08; mkdir -p $O
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-e2e > $O/b_cfg4.json 2> $O/b_cfg4.err
TPE_MOMENT_H=0 timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-e2e > $O/b_cfg4_noh.json 2> $O/b_cfg4_noh.err
TPE_ENGINE_LIB=$PWD/hyperopt_amd/libtpe_engine_eu5.so timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-e2e > $O/b_cfg4_eu5.json 2> $O/b_cfg4_eu5.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_cfg5.json 2> $O/b_cfg5.err
TPE_ENGINE_LIB=$PWD/hyperopt_amd/libtpe_engine_eu5.so timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/b_cfg5_eu5.json 2> $O/b_cfg5_eu5.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 --no-cpu-baseline --no-e2e > $O/b_cfg3.json 2> $O/b_cfg3.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 --no-cpu-baseline --no-e2e > $O/b_cfg2.json 2> $O/b_cfg2.err
echo done
