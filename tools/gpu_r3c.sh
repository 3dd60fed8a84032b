# Round 3: wgrad-roll parity first, the DUF 3x3x3 microbench, the full GPU suite, then PMC passes of the roll kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3c}
timeout -k 10 300 python -u -m pytest tests/test_wgrad_roll_gpu.py tests/test_multitile_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.roll.log 2>&1
rc=$?; echo "roll tests rc=$rc"; tail -15 gpurun_out/$TAG.roll.log; [ $rc -eq 0 ] || exit $rc
for C in duf64 duf224v; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what fwdpro,dgrad,wgradpro >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.p$i -o run --output-format csv -- python tools/conv_microbench.py --case duf64 --iters 3 --what fwdpro,wgradpro > gpurun_out/$TAG.p$i.log 2>&1
  echo "pass $i rc=$?"
done
python tools/pmc_summary.py $(find gpurun_out/$TAG.p* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc.txt
grep -A 30 "roll" gpurun_out/$TAG.pmc.txt
