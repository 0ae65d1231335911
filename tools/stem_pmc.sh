set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/stem_pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/p1 -o run --output-format csv -- python3 $ROOT/tools/stem_ab.py --modes 2 --reps 3 --rounds 1 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $ROOT/tools/stem_ab.py --modes 2 --reps 3 --rounds 1 > $OUT/p2.log 2>&1
echo done
