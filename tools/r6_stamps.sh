cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
export VSRK_LIB=$GRAFT_REPO_ROOT/vsr_amd/_lib/exp/stamp/libvsrk.so
for C in "edsr3x3 fwd,res" "duf64 fwdpro,dgradred,dgrad" "duf_u3 fwdpro,dgradred" "duf_u5 dgradred"; do
  set -- $C
  timeout -k 10 120 python tools/conv_microbench.py --case $1 --what $2 --iters 5 --stamps >> gpurun_out/r6a_stamps.txt 2>&1 || exit 1
done
unset VSRK_LIB
echo stamps done
