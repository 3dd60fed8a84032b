# A/B of environment settings on the conv microbench, all in one run (one box):
#   bash tools/gpu_envab.sh TAG "case1 case2" "what" "ENV=a ENV2=b" "ENV=c" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CASES=$2; WHAT=$3; shift 3
for rep in 1 2; do
for c in $CASES; do
  for envs in "$@"; do
    echo "== rep$rep $c [$envs]" >> gpurun_out/$TAG.ab.txt
    env $envs timeout -k 10 120 python tools/conv_microbench.py --case $c --iters 10 --what $WHAT 2>&1 | grep -v amdgpu.ids >> gpurun_out/$TAG.ab.txt || exit 1
  done
done
done
cat gpurun_out/$TAG.ab.txt
