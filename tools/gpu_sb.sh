# A/B of conv_fast scheduling variants (exp libs sb1, sb2) vs the in-tree build:
# parity of the conv kernels on each exp lib, then the conv microbench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sb}
OUT=gpurun_out/$TAG.micro.txt
: > $OUT
for V in sb1 sb2; do
  VSRK_LIB=$PWD/vsr_amd/_lib/exp/$V/libvsrk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_conv_kernels_gpu.py tests/test_multitile_gpu.py > gpurun_out/$TAG.$V.tests.log 2>&1
  rc=$?; echo "$V tests rc=$rc"; tail -2 gpurun_out/$TAG.$V.tests.log; [ $rc -eq 0 ] || exit $rc
done
for L in base sb1 sb2; do
  if [ $L = base ]; then LIBV=; else LIBV=VSRK_LIB=$PWD/vsr_amd/_lib/exp/$L/libvsrk.so; fi
  echo "== $L" >> $OUT
  env $LIBV timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what fwd,res,dgrad >> $OUT 2>&1 || exit $?
  env $LIBV timeout -k 10 200 python tools/conv_microbench.py --case duf64 --what fwd,fwdpro,dgrad --iters 10 >> $OUT 2>&1 || exit $?
  env $LIBV timeout -k 10 200 python tools/conv_microbench.py --case duf224v --what fwd,fwdpro,dgrad --iters 5 >> $OUT 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT
