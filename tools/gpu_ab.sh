# A/B of the thin-channel and LDS-DMA wgrad kernels against the generic ones
# (env switches are read once per process, so each arm is its own process).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}.txt
: > $OUT
for ARM in "" "VSRK_CONV_THIN=0 VSRK_WGRAD_FAST=0"; do
  echo "== arm: ${ARM:-new}" >> $OUT
  env $ARM timeout -k 10 200 python tools/conv_microbench.py --case tail --what fwd,dgrad,wgrad --iters 10 >> $OUT 2>&1 || exit $?
  env $ARM timeout -k 10 200 python tools/conv_microbench.py --case head --what fwd --iters 10 >> $OUT 2>&1 || exit $?
  env $ARM timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what wgrad --iters 10 >> $OUT 2>&1 || exit $?
done
cat $OUT
