# Full GPU suite, default bench (with measured peaks), cfg3 / cfg5 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cfg}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
python -c "
import json; d=json.load(open('gpurun_out/$TAG.bench.json')); print(json.dumps(d.get('measured_peak')))
for k,v in d['models'].items(): print(k, v['ms_per_step'], v['value'], v['roofline']['frac'], v['roofline'].get('frac_of_measured_peak'))"
for C in cfg3 cfg5; do
  timeout -k 10 400 python bench.py --config $C --steps 5 --warmup 2 --no-peaks > gpurun_out/$TAG.bench_$C.json 2> gpurun_out/$TAG.bench_$C.err
  rc=$?; echo "bench $C rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench_$C.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/$TAG.bench_$C.json'))
for k,v in d['models'].items(): print('$C', k, v['ms_per_step'], v['value'], v['roofline']['frac'], v['config']['workload'])"
done
