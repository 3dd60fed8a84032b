# Pipelined wgrad: split-target sweep and PMC passes at the DUF 64->32 shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-wps}
for c in duf64 duf224v; do
  for t in 512 1024 2048 4096 8192; do
    echo "== $c target=$t" >> gpurun_out/$TAG.sweep.txt
    VSRK_WGRAD_TARGET=$t timeout -k 10 120 python tools/conv_microbench.py --case $c --iters 10 --what wgradpro >> gpurun_out/$TAG.sweep.txt 2>&1 || exit 1
  done
done
cat gpurun_out/$TAG.sweep.txt
PASSES="SQ_WAVES" bash tools/gpu_pmc.sh ${TAG}pmc duf64 wgradpro
