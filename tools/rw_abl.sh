# A/B of the rolling-row weight gradient ablation builds (tools/build_exp_multi.sh rwx<N> conv_wgrad_row.hip -DRW_ABL=<N>)
cd $GRAFT_REPO_ROOT
for A in base rwx1 rwx2 rwx3; do
  if [ $A = base ]; then L=""; else L=$PWD/vsr_amd/_lib/exp/$A/libvsrk.so; fi
  echo "== $A"
  VSRK_LIB=$L timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what wgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
