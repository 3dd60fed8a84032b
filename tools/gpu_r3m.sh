# Round 3: sub-pixel tap skip in the pipelined wgrad: parity, DRF microbench, cfg3 bench; EDSR kernel summary
# (the upsampler data gradients now run on the rolling 2-D kernel's shuffled-input form).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3m}
timeout -k 10 600 python -u -m pytest tests/test_drf_kernels_gpu.py tests/test_nets_gpu.py tests/test_fullsize_cfg_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py tests/test_repro_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/drf_microbench.py --what up_wgrad,down_wgrad > gpurun_out/$TAG.micro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3.json 2> gpurun_out/$TAG.cfg3.err || exit $?
grep '^{' gpurun_out/$TAG.cfg3.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg3', d['value'], d['ms_per_step'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.pe/run_kernel_stats.csv 4 14 | cut -c1-150
