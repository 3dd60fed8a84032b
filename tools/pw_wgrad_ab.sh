# pointwise weight gradient at the DUF shapes, default chunking vs VSRK_PW_WGRAD_CI8=1 / 0
cd $GRAFT_REPO_ROOT
for ci8 in 0 1; do
  echo "== CI8=$ci8"
  for c in duf_fn1 duf_fn2 duf_rn1; do
    VSRK_PW_WGRAD_CI8=$ci8 timeout -k 10 100 python tools/conv_microbench.py --case $c --what wgrad 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
