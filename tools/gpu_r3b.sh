# Round 3: roll kernel tests + fp16 overflow tests, microbench, then SQ PMC passes of the roll fwd.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3b}
timeout -k 10 300 python -u -m pytest tests/test_roll_gpu.py tests/test_fp16_overflow_gpu.py tests/test_predictor_gpu.py tests/test_device_batch_gpu.py tests/test_conv_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in duf64 duf224v; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what fwdpro,dgrad,wgradpro >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.p$i -o run --output-format csv -- python tools/conv_microbench.py --case duf64 --iters 3 --what fwdpro > gpurun_out/$TAG.p$i.log 2>&1
  echo "pass $i rc=$?"
done
python tools/pmc_summary.py $(find gpurun_out/$TAG.p* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc.txt
grep -A 30 conv_roll gpurun_out/$TAG.pmc.txt
