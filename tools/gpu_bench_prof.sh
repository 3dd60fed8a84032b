set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
cat gpurun_out/bench1.json
tail -5 gpurun_out/bench1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof1 -name "*stats*" | head
