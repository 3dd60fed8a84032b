# GPU round trip: parity tests, then bench + rocprof kernel stats.  Each GPU
# step has its own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/$TAG.tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG.prof.log 2>&1
echo "prof rc=$?"
