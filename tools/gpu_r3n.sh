# Round 3: balanced pointwise wgrad chunks (A/B vs 8-block chunks), unrolled PReLU backward, DRF concat gradients
# without zero fills: parity, microbench, DUF + cfg3 benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3n}
timeout -k 10 600 python -u -m pytest tests/test_pw_gpu.py tests/test_roll_gpu.py tests/test_bn_duf_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_drf_kernels_gpu.py tests/test_nets_gpu.py tests/test_fullsize_cfg_gpu.py tests/test_graph_gpu.py tests/test_repro_gpu.py tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for E in 0 1; do
  for C in duf1x1x1_64 duf1x1x1 duf1x1x1_160 duf1x1x1_192 duf1x1x1_224; do
    echo "-- CI8=$E $C" >> gpurun_out/$TAG.micro.txt
    VSRK_PW_WGRAD_CI8=$E timeout -k 10 200 python tools/conv_microbench.py --case $C --what wgrad,wgradpro >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
for C in duf_u3 duf_u4 duf_u5; do
  for P in "" "roll=0,wgrad_roll=0"; do
    echo "-- $C paths=$P" >> gpurun_out/$TAG.micro.txt
    timeout -k 10 200 python tools/conv_microbench.py --case $C --what fwdpro,dgrad,wgradpro --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  done
done
for PR in 0 1 0 1; do
  echo "-- VSRK_ROLL_PRIO=$PR" >> gpurun_out/$TAG.micro.txt
  VSRK_ROLL_PRIO=$PR timeout -k 10 200 python tools/conv_microbench.py --case duf64 --what fwdpro,dgrad,wgradpro >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  VSRK_ROLL_PRIO=$PR timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what fwd,res >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
echo "-- edsr3x3 (wgrad_pipe planes padded)" >> gpurun_out/$TAG.micro.txt
timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what wgrad,fwd,res,dgrad >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3.json 2> gpurun_out/$TAG.cfg3.err || exit $?
timeout -k 10 300 python bench.py --models duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.duf.json 2> gpurun_out/$TAG.duf.err || exit $?
python - <<PY
import json
for f in ("gpurun_out/$TAG.cfg3.json", "gpurun_out/$TAG.duf.json"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"])
PY
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.p3/run_kernel_stats.csv 3 12 | cut -c1-150
timeout -k 10 200 python tools/drf_microbench.py --what up_wgrad,down_wgrad > gpurun_out/$TAG.drfmicro.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/$TAG.drfmicro.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe.log 2>&1) || exit $?
python tools/kstats.py gpurun_out/$TAG.pe/run_kernel_stats.csv 4 14 | cut -c1-150
