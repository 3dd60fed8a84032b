# Direct single-input-channel conv kernel: parity (conv, nets, DRF, ops), head / tail microbench, EDSR bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-thin1}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_kernels_gpu.py tests/test_nets_gpu.py tests/test_drf_kernels_gpu.py tests/test_ops_gpu.py tests/test_multitile_gpu.py tests/test_fullsize_gpu.py > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/$TAG.micro.txt
for C in tail head; do
  timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwd,dgrad --iters 10 >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --model edsr --steps 10 --warmup 3 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/$TAG.bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --model edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
