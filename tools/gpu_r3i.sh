# Round 3 re-entry: full GPU suite on the current tree, then the bench line and rocprof kernel summaries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3i}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3h.sh $TAG
