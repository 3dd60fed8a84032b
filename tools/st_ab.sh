# A/B of the one-channel stencil builds (tools/build_exp_multi.sh stnt conv_stencil.hip -DST_NT=1)
cd $GRAFT_REPO_ROOT
for A in base stnt; do
  if [ $A = base ]; then L=""; else L=$PWD/vsr_amd/_lib/exp/$A/libvsrk.so; fi
  echo "== $A"
  VSRK_LIB=$L timeout -k 10 120 python tools/conv_microbench.py --case tail --what dgrad,fwd 2>&1 | grep -v amdgpu.ids || exit 1
done
