# A/B: non-temporal output stores in the staged pointwise kernel (tools/build_exp_multi.sh pwnt conv_pw.hip -DPW_NT=2)
cd $GRAFT_REPO_ROOT
for A in base pwnt; do
  if [ $A = base ]; then L=""; else L=$PWD/vsr_amd/_lib/exp/$A/libvsrk.so; fi
  echo "== $A"
  VSRK_LIB=$L timeout -k 10 120 python tools/conv_microbench.py --case duf1x1x1_160 --what fwdpro,dgrad,dgradred 2>&1 | grep -v amdgpu.ids || exit 1
  VSRK_LIB=$L timeout -k 10 300 python bench.py --models duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('duf ms', d['models']['duf']['ms_per_step'])" || exit 1
done
