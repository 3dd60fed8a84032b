# Downscale/predictor tests, DUF conv microbench timings, PMC passes of the 3x3x3 wgrad.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_downscale_gpu.py tests/test_predictor_gpu.py > gpurun_out/wg3.tests.log 2>&1 || exit 1
for c in duf64 duf224v; do
  timeout -k 10 120 python tools/conv_microbench.py --case $c --iters 10 --what fwdpro,dgrad,wgrad,wgradpro >> gpurun_out/wg3.micro.txt 2>&1 || exit 1
done
cat gpurun_out/wg3.micro.txt
PASSES="SQ_WAVES" bash tools/gpu_pmc.sh wg3pmc duf64 wgradpro
