# Round-6 A/B of the deferred 2-D flush (conv_roll.hip ROLL_DEFER): roll tests on
# the in-tree library, then the conv microbench over base (HEAD~ kernel),
# nodefer (swap epilogue, -DROLL_DEFER=0) and the in-tree library
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${1:-df}
timeout -k 10 600 python -u -m pytest tests/test_roll_gpu.py tests/test_multitile_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6_ab.sh $TAG "edsr3x3:fwd,relu,dgrad,resacc,res,mask duf64:fwdpro,dgradred duf_u5:fwdpro,dgradred" vsr_amd/_lib/exp/base/libvsrk.so vsr_amd/_lib/exp/nodefer/libvsrk.so -
