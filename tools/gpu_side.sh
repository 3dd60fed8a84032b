# Side-stream weight gradients: full GPU suite, bench (EDSR, DUF), DRF cfg3, and the
# same with VSR_OVERLAP_WGRAD=0 for the A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-side}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
for V in 1 0; do
  VSR_OVERLAP_WGRAD=$V timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.bench$V.json 2> gpurun_out/$TAG.bench$V.err
  rc=$?; echo "bench overlap=$V rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench$V.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/$TAG.bench$V.json'))
for k,v in d['models'].items(): print('overlap=$V', k, v['ms_per_step'], v['value'], v['roofline']['frac'])"
  VSR_OVERLAP_WGRAD=$V timeout -k 10 400 python bench.py --config cfg3 --steps 4 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.cfg3_$V.json 2> gpurun_out/$TAG.cfg3_$V.err
  rc=$?; echo "cfg3 overlap=$V rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.cfg3_$V.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/$TAG.cfg3_$V.json'))
for k,v in d['models'].items(): print('overlap=$V cfg3', k, v['ms_per_step'], v['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
