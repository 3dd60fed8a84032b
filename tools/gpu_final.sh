# Round-end check: full GPU suite, default bench line (peaks + CPU baseline),
# rocprof kernel stats of the same bench, DUF dominant-conv HBM traffic (two
# separate --pmc passes), smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$TAG.smoke.log; [ $rc -eq 0 ] || exit $rc
K=conv_fast_kernelILi3ELi32ELi2ELi0ELi0ELi1EDF16bLi8
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/$TAG.pmc_$CNT -o run --output-format csv -- python bench.py --model duf --steps 1 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.pmc_$CNT.log 2>&1
  rc=$?; echo "pmc $CNT rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py gpurun_out/$TAG.pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/$TAG.pmc_WRITE_SIZE/run_counter_collection.csv $K profiles/traffic_duf_bf16.json "rocprofv3 --kernel-trace --pmc FETCH_SIZE|WRITE_SIZE -- python bench.py --model duf --steps 1 --warmup 1 --no-cpu-baseline --no-peaks" > gpurun_out/$TAG.traffic.log 2>&1
cp profiles/traffic_duf_bf16.json gpurun_out/$TAG.traffic_duf_bf16.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/$TAG.bench.err; exit $rc; }
python -c "
import json; d=json.load(open('gpurun_out/$TAG.bench.json')); print(json.dumps(d.get('measured_peak')))
for k,v in d['models'].items(): print(k, v['ms_per_step'], v['value'], v['roofline']['frac'], v['roofline'].get('frac_of_measured_peak'), v['roofline']['traffic'], v['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
