set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_47; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
rc=0; timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || rc=$?
tail -2 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in cfg4 cfg5; do
  S="--steps 1 --warmup 1"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${c}_trace -o run -- python -u bench.py --config $c $S $P > $O/${c}_trace.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/${c}_fetch -o run -- python -u bench.py --config $c $S $P > $O/${c}_fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/${c}_write -o run -- python -u bench.py --config $c $S $P > $O/${c}_write.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $SQ -d $O/${c}_sqa -o run -- python -u bench.py --config $c $S $P > $O/${c}_sqa.log 2>&1
done
python tools/rocpd_stats.py $O/*_trace $O/*_fetch $O/*_write > $O/rocpd.log 2>&1
for c in cfg4 cfg5; do python tools/prof_summary.py --dirs rd6h $c $O/${c}_trace $O/${c}_fetch $O/${c}_write >> $O/summary.log 2>&1; done
python tools/sq_summary.py profiles/rd6h_sq.json cfg4=$O/cfg4_sqa cfg5=$O/cfg5_sqa > $O/sq.log 2>&1
timeout -k 10 600 python -u bench.py > $O/b_default.json 2> $O/b_default.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 2 --warmup 1 $P > $O/b_cfg5.json 2> $O/b_cfg5.err
timeout -k 10 300 python -u bench.py --config cfg3 --steps 50 $P > $O/b_cfg3.json 2> $O/b_cfg3.err
timeout -k 10 300 python -u bench.py --config cfg2 --steps 100 $P > $O/b_cfg2.json 2> $O/b_cfg2.err
cp traffic.json profiles/rd6h_*.json profiles/rd6h_*.csv $O/ || true
find $O -name '*.db' -size +4M -delete
echo done
