# rocprofv3 kernel statistics of the bench, one model per pass (warm-up 2,
# 5 timed steps), summarised per step.  Usage: gpu_prof.sh TAG [models]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
for M in ${2:-edsr duf}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/$M -o run --output-format csv -- \
    python bench.py --model $M --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.$M.log 2>&1 || exit $?
  S=$(find gpurun_out/$TAG/$M -name "*kernel_stats.csv" | head -1)
  cp $S gpurun_out/$TAG.$M.kernel_stats.csv
  python tools/kstats.py $S 7 30 > gpurun_out/$TAG.$M.kernel_summary.txt
  echo "== $M"; head -32 gpurun_out/$TAG.$M.kernel_summary.txt
done
