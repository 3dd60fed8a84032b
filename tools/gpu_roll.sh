# Rolling-depth conv: parity tests, then the DUF 3x3x3 microbench (roll vs conv_fast).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-roll}
timeout -k 10 300 python -u -m pytest tests/test_roll_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in ${CASES:-duf64 duf224v duf3x3x3}; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what fwdpro,dgrad >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  echo "== conv_fast (roll off)" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what fwdpro,dgrad --paths roll=0 >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
