# Round 3: staged pointwise kernel (narrow / widening / PReLU / EIN) and the rolling 2-D conv over sub-pixel views:
# parity, DRF microbench (roll on / off), cfg3 + DUF + EDSR benches, cfg3 kernel summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3l}
timeout -k 10 700 python -u -m pytest tests/test_roll_gpu.py tests/test_pw_gpu.py tests/test_drf_kernels_gpu.py tests/test_nets_gpu.py tests/test_fullsize_cfg_gpu.py tests/test_graph_gpu.py tests/test_multitile_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for P in "" "roll=0"; do
  echo "-- paths=$P" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/drf_microbench.py --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3.json 2> gpurun_out/$TAG.cfg3.err || exit $?
timeout -k 10 300 python bench.py --models edsr,duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit $?
python - <<PY
import json
for f in ("gpurun_out/$TAG.cfg3.json", "gpurun_out/$TAG.bench.json"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"], {k: v.get("ms_per_step") for k, v in d.get("models", {}).items()})
PY
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3.log 2>&1) || exit $?
echo done
