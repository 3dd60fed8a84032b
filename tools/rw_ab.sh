# A/B knobs of the rolling-row weight gradient at the EDSR body shape
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/conv_microbench.py --case edsr3x3 --what wgrad 2>&1 | grep -v amdgpu.ids || exit 1; }
run X=0
run VSRK_WGRAD_ROW_PRIO=1
run VSRK_WGRAD_ROW_BANDS=2
run VSRK_WGRAD_ROW_BANDS=8
run VSRK_WGRAD_ROW_BANDS=16
