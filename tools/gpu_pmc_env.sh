# PMC passes (kernel-trace only) over the conv microbench under an environment:
#   bash tools/gpu_pmc_env.sh TAG CASE WHAT "ENV=a ENV2=b"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CASE=$2; WHAT=$3; ENVS=$4
for kv in $ENVS; do export "$kv"; done
i=0
for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.p$i -o run --output-format csv -- python tools/conv_microbench.py --case $CASE --iters 3 --what $WHAT > gpurun_out/$TAG.p$i.log 2>&1
  echo "pass $i rc=$?"
done
python tools/pmc_summary.py $(find gpurun_out/$TAG.p* -name "*counter_collection.csv") > gpurun_out/$TAG.summary.txt
