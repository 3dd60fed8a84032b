# Round-end style GPU pass: parity tests, EDSR bench + rocprof kernel stats,
# DUF / DRF bench lines, wgrad path A/B.  Each GPU step has its own time
# limit; the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$TAG.bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for M in duf drf; do
  timeout -k 10 400 python bench.py --model $M --steps 5 --warmup 2 > gpurun_out/$TAG.bench_$M.json 2> gpurun_out/$TAG.bench_$M.err
  rc=$?; echo "bench $M rc=$rc"; cat gpurun_out/$TAG.bench_$M.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench_$M.err; exit $rc; }
done
for V in VSRK_WGRAD_FAST=0 VSRK_WGRAD_FAST=1; do
  for C in edsr3x3 duf3x3x3; do
    echo "$V $(env $V timeout -k 10 100 python tools/conv_microbench.py --case $C --what wgrad 2>&1 | grep $C)" >> gpurun_out/$TAG.wgrad_ab.txt || exit 1
  done
done
cat gpurun_out/$TAG.wgrad_ab.txt
# HBM traffic of the dominant kernel: two separate --pmc passes over a short bench
K=conv_fast_kernelILi3ELi64ELi2ELi0ELi0ELi0EDF16bLi8
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.pmc_$CNT -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.pmc_$CNT.log 2>&1
  rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/$TAG.pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/$TAG.pmc_WRITE_SIZE/run_counter_collection.csv $K gpurun_out/$TAG.traffic.json "rocprofv3 --kernel-trace --pmc FETCH_SIZE|WRITE_SIZE -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
