# End-of-round-6 GPU run on the final tree: full suite, smoke, cfg2 / cfg3
# bench lines, kernel-trace profiles, and the DRF re-land A/B (same box)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu.sh r6z tests smoke bench bench:cfg3 prof:cfg2:duf prof:cfg2:edsr prof:cfg3:drf || exit 1
for V in "0 0" "1 0" "1 1"; do
  set -- $V
  VSR_DRF_BATCH_IN=$1 VSR_DRF_DEFER_SLOPES=$2 bash tools/gpu.sh r6zab_$1$2 quick:cfg3 || exit 1
done
