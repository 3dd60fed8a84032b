# A/B: resident workgroups per CU of the one-input-channel stencil (VSRK_STENCIL_WG)
cd $GRAFT_REPO_ROOT
for wg in 4 8 2 16; do
  echo "== WG=$wg"
  VSRK_STENCIL_WG=$wg timeout -k 10 120 python tools/conv_microbench.py --case tail --what dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
