# A/B: 256-channel pointwise convs on the staged kernel in 128-channel chunks (VSRK_PW_STAGED8)
cd $GRAFT_REPO_ROOT
for st in 1 0; do
  echo "== STAGED8=$st"
  for c in duf_rn1 duf_fn1; do
    VSRK_PW_STAGED8=$st timeout -k 10 100 python tools/conv_microbench.py --case $c --what fwd,fwdpro,mask 2>&1 | grep -v amdgpu.ids || exit 1
  done
  VSRK_PW_STAGED8=$st timeout -k 10 300 python bench.py --models duf --steps 5 --warmup 2 --no-cpu-baseline --no-peaks 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('duf ms', d['models']['duf']['ms_per_step'])" || exit 1
done
