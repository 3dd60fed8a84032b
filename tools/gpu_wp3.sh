# Pipelined wgrad: parity, then sched-interleave A/B at the DUF / EDSR shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-wp3}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_multitile_gpu.py -k "wgrad" tests/test_conv_kernels_gpu.py > gpurun_out/$TAG.tests.log 2>&1 || { tail -30 gpurun_out/$TAG.tests.log; exit 1; }
tail -2 gpurun_out/$TAG.tests.log
for c in duf64 duf224v edsr3x3; do
  for m in 1 0; do
    echo "== $c sched=$m" >> gpurun_out/$TAG.micro.txt
    VSRK_WP_SCHED=$m VSRK_WGRAD_TARGET=${TARGET:-} timeout -k 10 120 python tools/conv_microbench.py --case $c --iters 10 --what wgrad,wgradpro >> gpurun_out/$TAG.micro.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
