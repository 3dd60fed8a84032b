# round 4: validation of the resident-weight form and the compiler-visible prefetch, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for W in 1 0; do echo "== main WRES=$W"; VSRK_ROLL_WRES=$W timeout -k 10 200 python -m pytest tests/test_roll_gpu.py -q -x 2>&1 | tail -2 || exit 1; done
timeout -k 10 300 python -m pytest tests/test_wgrad_roll_gpu.py tests/test_multitile_gpu.py tests/test_duf_train_gpu.py -q -x 2>&1 | tail -2 || exit 1
for W in 1 0; do
  echo "== WRES=$W"
  for C in duf64 duf_u3; do VSRK_ROLL_WRES=$W timeout -k 10 120 python tools/conv_microbench.py --case $C --what dgrad,dgradred,wgradpro 2>&1 | grep -v amdgpu.ids || exit 1; done
  VSRK_ROLL_WRES=$W timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what fwd,relu,res,mask,resacc 2>&1 | grep -v amdgpu.ids || exit 1
done
