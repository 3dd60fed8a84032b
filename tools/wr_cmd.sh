set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh r4d tests:tests/test_roll_gpu.py,tests/test_multitile_gpu.py,tests/test_duf_train_gpu.py,tests/test_fullsize_gpu.py,tests/test_nets_gpu.py,tests/test_conv_kernels_gpu.py || exit 1
for W in 1 0 1 0; do
  echo "== WRES=$W"
  for C in duf64 duf_u3; do VSRK_ROLL_WRES=$W timeout -k 10 120 python tools/conv_microbench.py --case $C --what dgrad,dgradred 2>&1 | grep -v amdgpu.ids || exit 1; done
  VSRK_ROLL_WRES=$W timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what fwd,res,mask 2>&1 | grep -v amdgpu.ids || exit 1
done
