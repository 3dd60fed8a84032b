# One parameterised GPU script (run through gpurun from the repo root):
#
#   tools/gpu.sh TAG STEP [STEP ...]
#
# Steps run in order, each under its own time limit, and the script stops at
# the first failure (no retries).  Outputs go to gpurun_out/TAG.*.
#   tests                 the whole -m gpu suite
#   tests:FILES           named test files / node ids (comma separated)
#   smoke                 __graft_entry__.smoke()
#   bench[:CFG[:MODELS]]  bench.py line (CFG default cfg2; MODELS default the config's)
#   quick[:CFG[:MODELS]]  bench.py, 5 steps, no CPU baseline / peaks
#   prof:CFG:MODELS       rocprofv3 --kernel-trace --stats of a short bench run + top kernels
#   traffic:MODELS        separate FETCH_SIZE and WRITE_SIZE --pmc passes over a 1-step bench
#   pmc:CASE:WHAT[:PATHS] instruction / wait / LDS / HBM counter passes over tools/conv_microbench.py
#   micro:CASE[:WHAT]     tools/conv_microbench.py
#   drfmicro              tools/drf_microbench.py
# Environment variables in the gpurun command line (e.g. VSRK_FUSE=0) apply to every step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT

summary() {  # print the headline numbers of a bench JSON line
  grep '^{' "$1" | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print('value', d['value'], 'ms', round(d['ms_per_step'], 3))
for k, v in d['models'].items():
    rf = v['roofline']
    print(' ', k, round(v['ms_per_step'], 3), 'ms', 'frac', rf['frac'], 'launches', rf['launches_per_step'],
          {a: (round(b['ms_per_step'], 3), round(b['frac'] or 0, 4), b['launches_per_step']) for a, b in rf.get('by_direction', {}).items()})
"
}

for STEP in "$@"; do
  IFS=: read -r KIND A1 A2 A3 <<< "$STEP"
  echo "== $STEP"
  case $KIND in
    tests)
      if [ -z "$A1" ]; then SEL="tests -m gpu"; else SEL="${A1//,/ }"; fi
      timeout -k 10 1000 python -u -m pytest $SEL -x -q --timeout 240 --timeout-method thread > $O.tests.log 2>&1
      rc=$?; tail -4 $O.tests.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O.smoke.log 2>&1 || { tail $O.smoke.log; exit 1; }
      tail -1 $O.smoke.log ;;
    bench|quick)
      CFG=${A1:-cfg2}; EXTRA=""
      [ -n "$A2" ] && EXTRA="--models $A2"
      [ $KIND = quick ] && EXTRA="$EXTRA --steps 5 --warmup 2 --no-cpu-baseline --no-peaks"
      F=$O.$KIND.$CFG${A2:+.${A2//,/_}}
      timeout -k 10 900 python bench.py --config $CFG $EXTRA --units $F.units.txt > $F.json 2> $F.err || { tail -20 $F.err; exit 1; }
      summary $F.json ;;
    prof)
      CFG=${A1:-cfg2}; M=${A2:-duf}; D=$R/$O.prof_${CFG}_${M//,/_}
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python $R/bench.py --config $CFG --models $M --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > $D.log 2>&1) || { tail $D.log; exit 1; }
      python tools/kstats.py $D/run_kernel_stats.csv 4 16 | cut -c1-180 ;;
    traffic)
      for M in ${A1//,/ }; do
        for C in FETCH_SIZE WRITE_SIZE; do
          (cd /tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $C -d $R/$O.t_${M}_$C -o run --output-format csv -- python $R/bench.py --models $M --steps 1 --warmup 1 --no-cpu-baseline --no-peaks > $R/$O.t_${M}_$C.log 2>&1) || exit 1
          echo "pmc $M $C ok"
        done
      done ;;
    pmc)
      i=0
      for CNT in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
                 "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM" \
                 "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i+1))
        (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT -d $R/$O.pmc$i -o run --output-format csv -- python $R/tools/conv_microbench.py --case $A1 --iters 3 --what ${A2:-fwd} --paths "$A3" > $R/$O.pmc$i.log 2>&1) || exit 1
      done
      python tools/pmc_summary.py $(find $O.pmc* -name "*counter_collection.csv") > $O.pmc_summary.txt
      cat $O.pmc_summary.txt ;;
    micro)
      timeout -k 10 300 python tools/conv_microbench.py --case $A1 ${A2:+--what $A2} >> $O.micro.txt 2>&1 || { tail $O.micro.txt; exit 1; }
      tail -30 $O.micro.txt ;;
    drfmicro)
      timeout -k 10 300 python tools/drf_microbench.py >> $O.drfmicro.txt 2>&1 || { tail $O.drfmicro.txt; exit 1; }
      tail -40 $O.drfmicro.txt ;;
    *)
      echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG done"
