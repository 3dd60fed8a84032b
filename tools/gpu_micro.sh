# Quick GPU loop: conv kernel parity tests + microbench of the conv cases.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-micro}
TESTS=${TESTS:-tests/test_conv_kernels_gpu.py}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log
[ $rc -eq 0 ] || exit $rc
for C in ${CASES:-edsr3x3 duf3x3x3}; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C ${MB_ARGS} >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
