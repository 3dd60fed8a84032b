# A/B of experimental builds of the same ABI against the in-tree library:
#   tools/abl_cmd.sh "VARIANT ..." CASE WHAT   (VARIANT: base or a vsr_amd/_lib/exp/<name> build)
set -o pipefail
cd $GRAFT_REPO_ROOT
VARS=${1:-base}; CASE=${2:-duf64}; WHAT=${3:-dgrad,dgradred,fwdpro}
for A in $VARS; do
  if [ $A = base ]; then L=""; else L=$PWD/vsr_amd/_lib/exp/$A/libvsrk.so; fi
  echo "== $A"
  for C in ${CASE//,/ }; do
    VSRK_LIB=$L timeout -k 10 120 python tools/conv_microbench.py --case $C --what $WHAT 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
