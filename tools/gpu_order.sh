# Depth-major tile order for the 3-D convs: parity, microbench, DUF bench, DUF conv HBM traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-order}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_kernels_gpu.py tests/test_multitile_gpu.py tests/test_fullsize_gpu.py tests/test_nets_gpu.py tests/test_bn_duf_kernels_gpu.py > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/$TAG.micro.txt
timeout -k 10 200 python tools/conv_microbench.py --case duf64 --what fwd,fwdpro,dgrad --iters 10 >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
timeout -k 10 200 python tools/conv_microbench.py --case duf224v --what fwd,fwdpro,dgrad --iters 5 >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --model duf --steps 10 --warmup 3 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/$TAG.bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
K=conv_fast_kernelILi3ELi32ELi2ELi0ELi0ELi1EDF16bLi8
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.pmc_$CNT -o run --output-format csv -- python bench.py --model duf --steps 1 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.pmc_$CNT.log 2>&1
  rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/$TAG.pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/$TAG.pmc_WRITE_SIZE/run_counter_collection.csv $K gpurun_out/$TAG.traffic_duf_bf16.json "rocprofv3 --kernel-trace --pmc FETCH_SIZE|WRITE_SIZE -- python bench.py --model duf --steps 1 --warmup 1 --no-cpu-baseline --no-peaks"
