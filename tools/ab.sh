# A/B microbench on one box: tools/ab.sh "CASES" "WHATS" LIB1 LIB2 ...
# (LIB "-" = the in-tree library; others are paths to an experimental libvsrk.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
CASES=$1; WHATS=$2; shift 2
for rep in 1 2; do
for L in "$@"; do
  for C in $CASES; do
    if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$L; fi
    timeout -k 10 120 python tools/conv_microbench.py --case $C --what $WHATS 2>&1 | grep -v amdgpu.ids | sed "s|^|[$L] |" || exit 1
  done
done
done
