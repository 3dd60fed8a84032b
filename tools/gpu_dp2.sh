# N > 1 rehearsal on one GPU (two gloo ranks share the card): the spawn path
# and the torchrun path of bench.py, plus the DDP GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_gpu.py > gpurun_out/dp2.tests.log 2>&1
rc=$?; echo "ddp tests rc=$rc"; tail -2 gpurun_out/dp2.tests.log; [ $rc -eq 0 ] || exit $rc
VSR_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/dp2.spawn.json 2> gpurun_out/dp2.spawn.err
rc=$?; echo "spawn rc=$rc"; cat gpurun_out/dp2.spawn.json | head -c 600; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/dp2.spawn.err; exit $rc; }
VSR_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks --models duf > gpurun_out/dp2.trun.json 2> gpurun_out/dp2.trun.err
rc=$?; echo "torchrun rc=$rc"; grep metric gpurun_out/dp2.trun.json | head -c 600; echo; [ $rc -eq 0 ] || { tail -20 gpurun_out/dp2.trun.err; exit $rc; }
