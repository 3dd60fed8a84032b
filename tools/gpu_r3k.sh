# Round 3: staged pointwise kernel for narrowing convs + mask/accumulate epilogues; DRF microbench + PMC; benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3k}
timeout -k 10 400 python -u -m pytest tests/test_pw_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.pw.log 2>&1
rc=$?; echo "pw tests rc=$rc"; tail -3 gpurun_out/$TAG.pw.log; [ $rc -eq 0 ] || exit $rc
for P in "" "pw=0"; do
  echo "-- paths=$P" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/drf_microbench.py --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/$TAG.dp1 -o run --output-format csv -- python tools/drf_microbench.py --iters 3 --what up,down,up_dgrad,down_dgrad,up_wgrad > gpurun_out/$TAG.dp1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/$TAG.dp2 -o run --output-format csv -- python tools/drf_microbench.py --iters 3 --what up,down,up_dgrad,down_dgrad,up_wgrad > gpurun_out/$TAG.dp2.log 2>&1; echo "pmc2 rc=$?"
python tools/pmc_summary.py $(find gpurun_out/$TAG.dp* -name "*counter_collection.csv") > gpurun_out/$TAG.pmc_drf.txt
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
