# Parity of the conv/wgrad paths, then the default bench line and a rocprof
# kernel-stats profile of the DUF and EDSR steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2d}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_multitile_gpu.py tests/test_conv_kernels_gpu.py tests/test_fullsize_gpu.py > gpurun_out/$TAG.tests.log 2>&1 || { tail -30 gpurun_out/$TAG.tests.log; exit 1; }
tail -2 gpurun_out/$TAG.tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail -20 gpurun_out/$TAG.bench.err; exit 1; }
cat gpurun_out/$TAG.bench.json
for m in duf edsr; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof_$m -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --model $m --no-cpu-baseline > gpurun_out/$TAG.prof_$m.log 2>&1 || exit 1
  python tools/kstats.py $(find gpurun_out/$TAG.prof_$m -name "*kernel_stats.csv") 7 40 > gpurun_out/$TAG.$m.kernel_summary.txt 2>&1
  head -25 gpurun_out/$TAG.$m.kernel_summary.txt
done
