# pointwise weight gradient at the DUF unit shapes, default chunking vs VSRK_PW_WGRAD_CI8=1
cd $GRAFT_REPO_ROOT
for ci8 in 0 1; do
  echo "== CI8=$ci8"
  for c in duf1x1x1_224 duf1x1x1_192 duf1x1x1_160 duf1x1x1 duf1x1x1_64; do
    VSRK_PW_WGRAD_CI8=$ci8 timeout -k 10 100 python tools/conv_microbench.py --case $c --what wgradpro 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
