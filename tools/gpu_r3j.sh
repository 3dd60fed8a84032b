# Round 3: PMC of the rolling kernels at the DUF shapes (duf64 pad 1, duf224v depth-valid) and the EDSR 2-D roll.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3j}
for C in duf64 duf224v edsr3x3; do
  W=fwdpro,dgrad,wgradpro; [ $C = edsr3x3 ] && W=fwd,res,dgrad,wgrad
  echo "-- $C" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what $W >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for C in duf64 duf224v edsr3x3; do
    W=fwdpro,dgrad,wgradpro; [ $C = edsr3x3 ] && W=fwd,res,dgrad,wgrad
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.$C.p$i -o run --output-format csv -- python tools/conv_microbench.py --case $C --iters 3 --what $W > gpurun_out/$TAG.$C.p$i.log 2>&1
    echo "$C pass $i rc=$?"
  done
done
for C in duf64 duf224v edsr3x3; do
  python tools/pmc_summary.py $(find gpurun_out/$TAG.$C.p* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc_$C.txt
done
echo done
