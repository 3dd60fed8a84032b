# Round 3: validation of the fused forms and the pointwise / PReLU / wgrad changes, A/B microbenches, benches
# with and without the fusions (VSRK_FUSE), cfg 3 kernel summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3o}
timeout -k 10 700 python -u -m pytest tests/test_roll_gpu.py tests/test_pw_gpu.py tests/test_bn_duf_kernels_gpu.py tests/test_drf_kernels_gpu.py tests/test_conv_kernels_gpu.py tests/test_multitile_gpu.py tests/test_fullsize_gpu.py tests/test_nets_gpu.py tests/test_fullsize_cfg_gpu.py tests/test_graph_gpu.py tests/test_repro_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
M=gpurun_out/$TAG.micro.txt
for E in 0 1; do
  for C in duf1x1x1_64 duf1x1x1_160 duf1x1x1_224; do
    echo "-- CI8=$E $C" >> $M
    VSRK_PW_WGRAD_CI8=$E timeout -k 10 120 python tools/conv_microbench.py --case $C --what wgrad,wgradpro >> $M 2>&1 || exit $?
  done
done
for C in duf_u3 duf_u4 duf_u5; do
  for P in "" "roll=0,wgrad_roll=0"; do
    echo "-- $C paths=$P" >> $M
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwdpro,dgrad,wgradpro --paths "$P" >> $M 2>&1 || exit $?
  done
done
for PR in 0 1 0 1; do
  echo "-- VSRK_ROLL_PRIO=$PR" >> $M
  VSRK_ROLL_PRIO=$PR timeout -k 10 120 python tools/conv_microbench.py --case duf64 --what fwdpro,dgrad,wgradpro >> $M 2>&1 || exit $?
  VSRK_ROLL_PRIO=$PR timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what fwd,res >> $M 2>&1 || exit $?
done
echo "-- edsr3x3 (wgrad_pipe planes padded)" >> $M
timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what wgrad,dgrad >> $M 2>&1 || exit $?
timeout -k 10 120 python tools/drf_microbench.py >> $M 2>&1 || exit $?
grep -v amdgpu.ids $M
for F in 1 0; do
  VSRK_FUSE=$F timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3_f$F.json 2> gpurun_out/$TAG.cfg3_f$F.err || exit $?
  VSRK_FUSE=$F timeout -k 10 300 python bench.py --models edsr,duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench_f$F.json 2> gpurun_out/$TAG.bench_f$F.err || exit $?
done
for f in cfg3_f1 cfg3_f0 bench_f1 bench_f0; do grep '^{' gpurun_out/$TAG.$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['models'].items()})"; done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.p3/run_kernel_stats.csv 3 14 | cut -c1-150
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd -o run -- python $GRAFT_REPO_ROOT/bench.py --models duf --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.pd/run_kernel_stats.csv 4 14 | cut -c1-150
