# Thin-out forward with two stages of register prefetch: A/B microbench (HEAD
# library vs experimental builds), then the thin-channel parity tests on each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
: > gpurun_out/thinout.micro.txt
for L in base to3 to2; do
  export VSRK_LIB=vsr_amd/_lib/exp/$L/libvsrk.so
  echo "== $L" >> gpurun_out/thinout.micro.txt
  timeout -k 10 120 python tools/conv_microbench.py --case tail --what fwd --iters 20 >> gpurun_out/thinout.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/thinout.micro.txt
for L in to3 to2; do
  export VSRK_LIB=vsr_amd/_lib/exp/$L/libvsrk.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "thin or edsr or drf" tests/test_conv_kernels_gpu.py tests/test_nets_gpu.py tests/test_multitile_gpu.py > gpurun_out/thinout.$L.tests.log 2>&1
  rc=$?; echo "$L tests rc=$rc"; tail -2 gpurun_out/thinout.$L.tests.log; [ $rc -eq 0 ] || exit $rc
done
