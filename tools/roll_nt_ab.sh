# A/B: non-temporal output stores in the rolling conv epilogue (tools/build_exp_multi.sh rollnt conv_roll.hip -DROLL_NT=1)
cd $GRAFT_REPO_ROOT
for A in base rollnt base rollnt; do
  if [ $A = base ]; then L=""; else L=$PWD/vsr_amd/_lib/exp/$A/libvsrk.so; fi
  echo "== $A"
  VSRK_LIB=$L timeout -k 10 300 python bench.py --models edsr,duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v['ms_per_step'],3) for k,v in d['models'].items()})" || exit 1
done
