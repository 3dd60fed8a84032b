cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_roll_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f1.tests.log 2>&1; rc=$?; tail -5 gpurun_out/f1.tests.log; [ $rc -eq 0 ] || exit $rc
for P in "roll_fold=1" "roll_fold=0,roll=1" "roll_fold=0"; do
  timeout -k 10 120 python tools/conv_microbench.py --case duf_u5 --what fwdpro,fwd --paths "$P" >> gpurun_out/f1.micro.txt 2>&1 || exit 1
  echo "$P" >> gpurun_out/f1.micro.txt
done
cat gpurun_out/f1.micro.txt
