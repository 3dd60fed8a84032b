# pointwise conv check: parity tests (pw, conv kernels, nets, full-size), then
# the 1x1x1 microbench with the pw path on and off, then the DUF bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pw}
timeout -k 10 600 python -u -m pytest tests/test_pw_gpu.py tests/test_conv_kernels_gpu.py tests/test_nets_gpu.py \
  tests/test_multitile_gpu.py tests/test_fullsize_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG.tests.log 2>&1
rc=$?; tail -25 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for C in ${CASES:-duf1x1x1_64 duf1x1x1 duf1x1x1_224}; do
  for P in pw=0 pw=1; do
    echo "== $C $P" >> gpurun_out/$TAG.micro.txt
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwd,fwdpro,dgrad,wgrad --paths $P \
      >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG.micro.txt
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --models duf --steps 5 --warmup 2 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
  rc=$?; cat gpurun_out/$TAG.bench.json; tail -5 gpurun_out/$TAG.bench.err; exit $rc
fi
