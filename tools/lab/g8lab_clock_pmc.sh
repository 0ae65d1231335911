# Held clock of the lab k_gemm8 schedule per diagnostic mode from GRBM_GUI_ACTIVE over each dispatch (cross-check of the s_memtime stamps).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06u
cd /tmp && export TMPDIR=/tmp
for M in 0 7 2; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r06u/m$M -o run --output-format csv -- python3 $R/tools/lab/g8lab_pmc_work.py $M 16384 4096 2048 > $R/gpurun_out/r06u/m$M.log 2>&1
done
cd $R
for M in 0 7 2; do echo "mode $M"; python3 tools/body_clock.py gpurun_out/r06u/m$M 3; done
