# Deferred multi-unit bn1 apply in DUF: BN / DUF / DDP / repro parity, DUF bench + kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-multi}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_duf_kernels_gpu.py tests/test_nets_gpu.py tests/test_ddp_gpu.py tests/test_fullsize_gpu.py tests/test_repro_gpu.py tests/test_ops_gpu.py tests/test_trainer_gpu.py tests/test_abi_cpu.py > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model duf --steps 10 --warmup 3 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/$TAG.bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --model duf --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
