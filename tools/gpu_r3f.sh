# Round 3: rolling kernels after the operand-prefetch lead and the wgrad split fix:
# parity, microbench A/B, PMC of the 2-D roll (residual form) and the rolling wgrad, then the full suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3f}
timeout -k 10 400 python -u -m pytest tests/test_wgrad_roll_gpu.py tests/test_roll_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.roll.log 2>&1
rc=$?; echo "roll tests rc=$rc"; tail -5 gpurun_out/$TAG.roll.log; [ $rc -eq 0 ] || exit $rc
for C in duf64 duf224v; do
  for P in "" "wgrad_roll=0"; do
    echo "-- $C paths=$P" >> gpurun_out/$TAG.micro.txt
    timeout -k 10 200 python tools/conv_microbench.py --case $C --what wgradpro --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
for P in "" "roll=0" "" "roll=0"; do
  echo "-- edsr paths=$P" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what fwd,res,mask,relu,dgrad --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.p$i -o run --output-format csv -- python tools/conv_microbench.py --case duf64 --iters 3 --what fwdpro,dgrad,wgradpro > gpurun_out/$TAG.p$i.log 2>&1
  echo "pass $i rc=$?"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.e$i -o run --output-format csv -- python tools/conv_microbench.py --case edsr3x3 --iters 3 --what fwd,res > gpurun_out/$TAG.e$i.log 2>&1
  echo "edsr pass $i rc=$?"
done
python tools/pmc_summary.py $(find gpurun_out/$TAG.p* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc.txt
python tools/pmc_summary.py $(find gpurun_out/$TAG.e* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc_edsr.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
