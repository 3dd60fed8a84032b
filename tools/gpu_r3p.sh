# Round 3 final call: the full GPU suite + smoke, the default bench line, cfg 3 / cfg 5, fused-path A/B,
# rocprof kernel summaries, PMC HBM traffic of the dominant kernels, then the A/B microbenches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3p}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.smoke.log
timeout -k 10 600 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit $?
grep '^{' gpurun_out/$TAG.bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['ms_per_step'], v['roofline']['frac']) for k, v in d['models'].items()}, d.get('north_star'))"
timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3.json 2> gpurun_out/$TAG.cfg3.err || exit $?
VSRK_FUSE=0 timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3_f0.json 2> gpurun_out/$TAG.cfg3_f0.err || exit $?
VSRK_FUSE=0 timeout -k 10 300 python bench.py --models duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.duf_f0.json 2> gpurun_out/$TAG.duf_f0.err || exit $?
timeout -k 10 400 python bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg5.json 2> gpurun_out/$TAG.cfg5.err || exit $?
for f in cfg3 cfg3_f0 duf_f0 cfg5; do grep '^{' gpurun_out/$TAG.$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['models'].items()})"; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd -o run -- python $GRAFT_REPO_ROOT/bench.py --models duf --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.p3/run_kernel_stats.csv 2 14 | cut -c1-150
python tools/kstats.py gpurun_out/$TAG.pd/run_kernel_stats.csv 3 10 | cut -c1-150
for M in edsr duf; do
  for C in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.t_${M}_$C -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --models $M --steps 1 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.t_${M}_$C.log 2>&1)
    echo "pmc $M $C rc=$?"
  done
done
M=gpurun_out/$TAG.micro.txt
for C in duf_u3 duf_u4 duf_u5; do
  for P in "" "roll=0,wgrad_roll=0"; do
    echo "-- $C paths=$P" >> $M
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what fwdpro,dgrad,wgradpro --paths "$P" >> $M 2>&1 || exit $?
  done
done
for PR in 0 1; do
  echo "-- VSRK_ROLL_PRIO=$PR" >> $M
  VSRK_ROLL_PRIO=$PR timeout -k 10 120 python tools/conv_microbench.py --case duf64 --what fwdpro,dgrad,wgradpro >> $M 2>&1 || exit $?
done
timeout -k 10 120 python tools/drf_microbench.py >> $M 2>&1 || exit $?
grep -v amdgpu.ids $M
echo done
