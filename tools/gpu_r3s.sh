# Round 3: EDSR upsampler conv on the rolling kernel (pixel-shuffle bias order): parity, nets, EDSR bench + kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3s}
timeout -k 10 600 python -u -m pytest tests/test_roll_gpu.py tests/test_nets_gpu.py tests/test_fullsize_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --models edsr --no-cpu-baseline --no-peaks > gpurun_out/$TAG.edsr.json 2> gpurun_out/$TAG.edsr.err || exit $?
grep '^{' gpurun_out/$TAG.edsr.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('edsr', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.pe/run_kernel_stats.csv 4 12 | cut -c1-170
