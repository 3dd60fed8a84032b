cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
export VSRK_LIB=$GRAFT_REPO_ROOT/vsr_amd/_lib/exp/stamp/libvsrk.so
O=gpurun_out/r6b_stamps.txt
timeout -k 10 120 python tools/conv_microbench.py --case duf64 --what fwd,fwdpro,dgrad --iters 5 --stamps >> $O 2>&1 || exit 1
VSRK_ROLL_WRES=0 timeout -k 10 120 python tools/conv_microbench.py --case duf64 --what dgrad --iters 5 --stamps >> $O 2>&1 || exit 1
timeout -k 10 120 python tools/conv_microbench.py --case duf224v --what fwd,fwdpro --iters 5 --stamps >> $O 2>&1 || exit 1
echo done
