# Round-6 A/B of the register-transposed flush on the 2-D non-prefetch forms
# (conv_roll.hip ROLL_SWAP): roll / DRF-fused tests on the in-tree library,
# then the conv and DRF microbenches over noswap (-DROLL_SWAP=0) and in-tree
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${1:-sw}
timeout -k 10 900 python -u -m pytest tests/test_roll_gpu.py tests/test_multitile_gpu.py tests/test_prelu_fused_gpu.py tests/test_nets_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6_ab.sh $TAG "edsr3x3:fwd,relu,dgrad,resacc,res,mask" vsr_amd/_lib/exp/noswap/libvsrk.so -
for rep in 1 2; do
for L in vsr_amd/_lib/exp/noswap/libvsrk.so -; do
  if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$GRAFT_REPO_ROOT/$L; fi
  echo "== $L" >> gpurun_out/$TAG.drf.txt
  timeout -k 10 300 python tools/drf_microbench.py --what up,down,up_dgrad,down_dgrad,prelu_hr,prelu_lr >> gpurun_out/$TAG.drf.txt 2>&1 || exit 1
done
done
unset VSRK_LIB
grep -v amdgpu.ids gpurun_out/$TAG.drf.txt
