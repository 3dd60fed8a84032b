# k3 (second-generation 3x3 conv) check: conv parity tests, then the
# microbench with k3 off (old fast kernel) and on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-k3}
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels_gpu.py tests/test_multitile_gpu.py \
  tests/test_fullsize_gpu.py tests/test_drf_kernels_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG.tests.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in edsr3x3 duf64 duf224v; do
  for P in k3=0 k3=1; do
    echo "== $C $P" >> gpurun_out/$TAG.micro.txt
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwd,res,dgrad --paths $P >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG.micro.txt
