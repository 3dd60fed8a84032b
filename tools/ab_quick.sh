# Same-box A/B of whole bench steps over experimental libraries:
#   tools/ab_quick.sh CFG MODELS LIB1 LIB2 ...   ("-" = the in-tree library)
# two alternations, 5 steps each, ms/step per run
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
CFG=$1; M=$2; shift 2
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 600 python bench.py --config $CFG --models $M --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/abq.json 2> gpurun_out/abq.err || { tail -5 gpurun_out/abq.err; exit 1; }
    echo "[$L] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abq.json | head -2 | tr '\n' ' ')"
  done
done
