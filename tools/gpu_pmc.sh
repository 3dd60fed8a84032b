# PMC counter passes (kernel-trace only; never combined with sys/runtime trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
CASE=${2:-edsr3x3}
timeout -k 10 200 python tools/conv_microbench.py --case $CASE > gpurun_out/$TAG.micro.txt 2>&1
rc=$?; cat gpurun_out/$TAG.micro.txt; [ $rc -eq 0 ] || exit $rc
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.p$i -o run --output-format csv -- python tools/conv_microbench.py --case $CASE --iters 3 > gpurun_out/$TAG.p$i.log 2>&1
  echo "pass $i rc=$?"
done
