# Re-entry check of HEAD: GPU parity suite, default bench line, rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2e}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
