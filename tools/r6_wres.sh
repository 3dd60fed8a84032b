cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6d.txt
for rep in 1 2; do
for W in 1 0; do
  for X in duf_u5:dgradred,dgrad duf_u4:dgradred duf_u3:dgradred duf64:dgradred,dgrad; do
    C=${X%%:*}; WH=${X#*:}
    VSRK_ROLL_WRES=$W timeout -k 10 120 python tools/conv_microbench.py --case $C --what $WH 2>&1 | grep -v amdgpu.ids | sed "s|^|[wres$W] |" >> $O || exit 1
  done
done
done
python tools/ab_summary.py $O
