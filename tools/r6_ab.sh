# same-box A/B of the conv microbench over libraries: tools/r6_ab.sh TAG "case:what ..." LIB...
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=$1; CW=$2; shift 2
O=gpurun_out/$TAG.ab.txt
for rep in 1 2; do
for L in "$@"; do
  for X in $CW; do
    C=${X%%:*}; W=${X#*:}
    if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what $W 2>&1 | grep -v amdgpu.ids | sed "s|^|[$L] |" >> $O || exit 1
  done
done
done
unset VSRK_LIB
python tools/ab_summary.py $O 2>/dev/null || cat $O
