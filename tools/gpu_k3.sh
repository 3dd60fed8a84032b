# k3 (second-generation 3x3 conv) check: conv parity tests with k3 forced on,
# then the microbench with k3 off (conv_fast) and on, then SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-k3}
VSRK_CONV_K3=1 timeout -k 10 600 python -u -m pytest tests/test_conv_kernels_gpu.py tests/test_multitile_gpu.py \
  tests/test_fullsize_gpu.py tests/test_drf_kernels_gpu.py tests/test_nets_gpu.py -m gpu -q -x --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in ${CASES:-edsr3x3 duf64 duf224v}; do
  for P in k3=0 k3=1; do
    echo "== $C $P" >> gpurun_out/$TAG.micro.txt
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwd,res,dgrad --paths $P >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG.micro.txt
if [ "${PMC:-0}" = "1" ]; then
  PASSES=" " bash tools/gpu_pmc.sh ${TAG}_pmc edsr3x3 fwd k3=1 > /dev/null 2>&1
  L=$(grep -n "conv_k3" gpurun_out/${TAG}_pmc.summary.txt | head -1 | cut -d: -f1)
  sed -n "$L,$((L+26))p" gpurun_out/${TAG}_pmc.summary.txt
fi
