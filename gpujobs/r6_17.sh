set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_17; mkdir -p $O
P="--no-cpu-baseline --no-e2e"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/cfg4_sqa -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 1 $P > $O/cfg4_sqa.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $O/cfg4_sqb -o run -- python -u bench.py --config cfg4 --steps 1 --warmup 1 $P > $O/cfg4_sqb.log 2>&1
python tools/sq_summary.py $O/sq.json cfg4x=$O/cfg4_sqa cfg4y=$O/cfg4_sqb > $O/sq.log 2>&1
find $O -name '*.db' -delete
echo done
