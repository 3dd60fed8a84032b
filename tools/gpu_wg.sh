# 3x3x3 weight-gradient A/B: generic vs LDS-DMA kernel, split targets
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-wg}
for C in ${CASES:-duf64 duf224v}; do
  for P in wgrad_fast=0 wgrad_fast=1; do
    for T in ${TARGETS:-0 256 1024}; do
      echo "== $C $P target=$T" >> gpurun_out/$TAG.txt
      if [ "$T" = "0" ]; then
        timeout -k 10 120 python tools/conv_microbench.py --case $C --what wgrad --paths $P >> gpurun_out/$TAG.txt 2>&1 || exit $?
      else
        VSRK_WGRAD_TARGET=$T timeout -k 10 120 python tools/conv_microbench.py --case $C --what wgrad --paths $P >> gpurun_out/$TAG.txt 2>&1 || exit $?
      fi
    done
  done
done
grep -v amdgpu.ids gpurun_out/$TAG.txt
