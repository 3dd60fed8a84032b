# fp16 path: parity tests, then the bench line for both models at fp16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-f16}
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels_gpu.py tests/test_pw_gpu.py tests/test_nets_gpu.py \
  -m gpu -q --timeout 300 --timeout-method thread -k "dtype2 or fp16 or f16" > gpurun_out/$TAG.tests.log 2>&1
rc=$?; tail -30 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --precision fp16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; cut -c1-400 gpurun_out/$TAG.bench.json; tail -3 gpurun_out/$TAG.bench.err; exit $rc
