# A/B of an experimental library build (VSRK_LIB) against the in-tree one:
# parity of the conv kernels + layout moves on the experimental build, then
# the conv microbench on both (the experimental one under each setting in
# $VARIANTS, e.g. "VSRK_FAST_WR=0 VSRK_FAST_WR=1").  Each GPU step has its
# own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
EXP=$PWD/${2:-vsr_amd/_lib/exp/libvsrk_exp.so}
CASE=${3:-edsr3x3}
VSRK_LIB=$EXP timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_conv_kernels_gpu.py tests/test_layout_gpu.py > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "exp tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
echo "== base" >> gpurun_out/$TAG.micro.txt
timeout -k 10 200 python tools/conv_microbench.py --case $CASE --what fwd,res >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
for V in ${VARIANTS:-NONE=0}; do
  echo "== exp $V" >> gpurun_out/$TAG.micro.txt
  env $V VSRK_LIB=$EXP timeout -k 10 200 python tools/conv_microbench.py --case $CASE --what fwd,res >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
