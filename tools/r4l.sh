# round 4: rolling weight gradient (x-row window, spread prologue): parity + microbench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_wgrad_roll_gpu.py tests/test_fullsize_gpu.py tests/test_duf_train_gpu.py -q -x 2>&1 | tail -2 || exit 1
for i in 1 2; do
  for C in duf64 duf_u3; do timeout -k 10 120 python tools/conv_microbench.py --case $C --what wgradpro,wgrad 2>&1 | grep -v amdgpu.ids || exit 1; done
done
