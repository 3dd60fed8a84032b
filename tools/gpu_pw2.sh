# pw kernels: parity, then microbench A/B and ablations (VSRK_PW_ABLATE 1 = no stores, 2 = no MFMA)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pw2}
timeout -k 10 300 python -u -m pytest tests/test_pw_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG.tests.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in ${CASES:-duf1x1x1_64 duf1x1x1 duf1x1x1_224}; do
  for AB in ${ABL:-0 1 2}; do
    echo "== $C ablate=$AB" >> gpurun_out/$TAG.micro.txt
    VSRK_PW_ABLATE=$AB timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwd,fwdpro,dgrad,wgrad \
      --paths pw=1 >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG.micro.txt
