# GPU round trip: parity tests, conv microbench, bench JSON + rocprof stats.
# Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log
[ $rc -eq 0 ] || exit $rc
for C in edsr3x3 duf3x3x3; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
