# A/B of an earlier 2-D operand prefetch (ROLL_PFEARLY=1) on the EDSR residual / mask forms
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
export VSRK_LIB=$GRAFT_REPO_ROOT/vsr_amd/_lib/exp/pfe/libvsrk.so
timeout -k 10 600 python -u -m pytest tests/test_roll_gpu.py tests/test_multitile_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pfe.tests.log 2>&1; rc=$?; tail -2 gpurun_out/pfe.tests.log; [ $rc -eq 0 ] || exit $rc
unset VSRK_LIB
bash tools/r6_ab.sh pfe "edsr3x3:res,mask,relu" - vsr_amd/_lib/exp/pfe/libvsrk.so
