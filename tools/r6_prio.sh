# A/B of VSRK_ROLL_PRIO=1 (s_setprio 1 for waves 4-7 of the rolling convs), same box, two alternations
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/prio.txt
for rep in 1 2; do
  for P in 0 1; do
    for X in edsr3x3:fwd,relu,res,mask,dgrad duf64:fwdpro,dgradred duf_u3:fwdpro,dgradred; do
      VSRK_ROLL_PRIO=$P timeout -k 10 120 python tools/conv_microbench.py --case ${X%%:*} --what ${X#*:} 2>&1 | grep -v amdgpu.ids | sed "s|^|[prio$P] |" >> $O || exit 1
    done
  done
done
python tools/ab_summary.py $O
