# Round-2 GPU check: the whole -m gpu suite (one process), then a short bench.
# Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
SEL=${2:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --maxfail=15 --timeout 300 --timeout-method thread \
  > gpurun_out/$TAG.tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/$TAG.tests.log | tail -60
tail -3 gpurun_out/$TAG.tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
  brc=$?; echo "bench rc=$brc"; cat gpurun_out/$TAG.bench.json; tail -3 gpurun_out/$TAG.bench.err
fi
exit $rc
