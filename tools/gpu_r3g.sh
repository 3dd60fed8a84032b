# Round 3: 2-D rolling conv A/B after the operand-prefetch change (quick).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3g}
timeout -k 10 300 python -u -m pytest tests/test_roll_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.roll.log 2>&1
rc=$?; echo "roll tests rc=$rc"; tail -3 gpurun_out/$TAG.roll.log; [ $rc -eq 0 ] || exit $rc
for P in "" "roll=0" "" "roll=0"; do
  echo "-- edsr paths=$P" >> gpurun_out/$TAG.micro.txt
  timeout -k 10 200 python tools/conv_microbench.py --case edsr3x3 --what fwd,res,mask,relu,dgrad --paths "$P" >> gpurun_out/$TAG.micro.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/$TAG.micro.txt
