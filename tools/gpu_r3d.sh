# Round 3: the 2-D rolling conv (EDSR body) -- parity, microbench A/B against conv_fast, EDSR/DUF bench + profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3d}
timeout -k 10 300 python -u -m pytest tests/test_roll_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.roll.log 2>&1
rc=$?; echo "roll tests rc=$rc"; tail -15 gpurun_out/$TAG.roll.log; [ $rc -eq 0 ] || exit $rc
for P in "" "roll=0"; do
  timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what fwd,relu,res,dgrad,mask,resacc --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
  echo "-- paths=$P" >> gpurun_out/$TAG.micro.txt
done
cat gpurun_out/$TAG.micro.txt
timeout -k 10 300 python bench.py --models edsr,duf --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || exit $?
python -c "
import json
for l in open('gpurun_out/$TAG.bench.json'):
    if l.startswith('{'):
        d = json.loads(l)
        print({k: (v.get('ms_per_step'), v.get('roofline', {}).get('frac')) for k, v in d.get('models', {}).items()})
"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG.prof -o run -- python $GRAFT_REPO_ROOT/bench.py --models edsr,duf --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $GRAFT_REPO_ROOT/gpurun_out/$TAG.prof.log 2>&1
echo "prof rc=$?"
