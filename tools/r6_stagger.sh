# A/B of the staggered late flush (conv_roll.hip ROLL_STAGGER): tests on the
# in-tree library, then the conv / DRF microbenches and quick EDSR / DRF steps
# over nostag (-DROLL_STAGGER=0) and the in-tree library
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${1:-st}
timeout -k 10 900 python -u -m pytest tests/test_roll_gpu.py tests/test_multitile_gpu.py tests/test_prelu_fused_gpu.py tests/test_nets_gpu.py tests/test_graph_gpu.py tests/test_drf_seqbuf_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1; rc=$?; tail -2 gpurun_out/$TAG.tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6_ab.sh $TAG "edsr3x3:fwd,relu,dgrad,resacc" vsr_amd/_lib/exp/nostag/libvsrk.so - || exit 1
for rep in 1 2; do
for L in vsr_amd/_lib/exp/nostag/libvsrk.so -; do
  if [ "$L" = "-" ]; then unset VSRK_LIB; else export VSRK_LIB=$GRAFT_REPO_ROOT/$L; fi
  timeout -k 10 300 python tools/drf_microbench.py --what up,down > gpurun_out/$TAG.drf.tmp 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/$TAG.drf.tmp | sed "s|^|[$L] |" >> gpurun_out/$TAG.drf.txt
  for C in cfg2:edsr cfg3:drf; do
    timeout -k 10 600 python bench.py --config ${C%%:*} --models ${C##*:} --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/$TAG.q.json 2> gpurun_out/$TAG.q.err || { tail -5 gpurun_out/$TAG.q.err; exit 1; }
    echo "[$L] $C $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$TAG.q.json | head -1)" >> gpurun_out/$TAG.steps.txt
  done
done
done
unset VSRK_LIB
cat gpurun_out/$TAG.drf.txt gpurun_out/$TAG.steps.txt
