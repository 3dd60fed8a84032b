# Round 3: bench (EDSR + DUF at cfg 2, DRF at cfg 3) and their rocprof kernel summaries.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3h}
timeout -k 10 300 python bench.py --models edsr,duf --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit $?
timeout -k 10 300 python bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3.json 2> gpurun_out/$TAG.cfg3.err || exit $?
python - <<PY
import json
for f in ("gpurun_out/$TAG.bench.json", "gpurun_out/$TAG.cfg3.json"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f, d["value"], d["ms_per_step"], {k: (v.get("ms_per_step"), v.get("roofline", {}).get("frac")) for k, v in d.get("models", {}).items()})
PY
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pe.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd -o run -- python $GRAFT_REPO_ROOT/bench.py --models duf --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.pd.log 2>&1) || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.p3.log 2>&1) || exit $?
echo done
