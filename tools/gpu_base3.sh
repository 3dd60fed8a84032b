# Round-3 baseline: DUF 3x3x3 conv microbench (fwd with BN prologue, dgrad, wgrad) at the bench shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-base3}
for C in ${CASES:-duf64 duf224v duf3x3x3 edsr3x3}; do
  timeout -k 10 200 python tools/conv_microbench.py --case $C --what ${WHAT:-fwdpro,dgrad,wgradpro} >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG.micro.txt
