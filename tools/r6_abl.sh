# Ablations of the rolling conv at the EDSR body shape and a DUF unit
# (tools/build_exp_multi.sh abl1|abl2|abl4 conv_roll.hip -DROLL_ABL=n; results wrong, timing only)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/abl.txt
for L in - vsr_amd/_lib/exp/abl1/libvsrk.so vsr_amd/_lib/exp/abl2/libvsrk.so vsr_amd/_lib/exp/abl4/libvsrk.so; do
  if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$GRAFT_REPO_ROOT/$L; fi
  echo "== $L" >> $O
  timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what fwd,relu,res,mask,dgrad >> $O 2>&1 || exit 1
  timeout -k 10 120 python tools/conv_microbench.py --case duf64 --what fwdpro,dgradred >> $O 2>&1 || exit 1
done
grep -v amdgpu.ids $O
