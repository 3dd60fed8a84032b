set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r2e.sh ${1:-r2e} && bash tools/gpu_sb.sh ${2:-sb}
