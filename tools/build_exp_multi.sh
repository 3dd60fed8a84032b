# Experimental library for A/B runs: the last full build's objects with the
# given csrc sources recompiled under extra flags.
#   tools/build_exp_multi.sh NAME "src1.hip src2.hip" -DFOO=1 ...
# -> vsr_amd/_lib/exp/NAME/libvsrk.so (load with VSRK_LIB=...)
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRCS=$2; shift 2
D=vsr_amd/_lib/exp/$NAME
mkdir -p $D
OBJS=$(ls vsr_amd/_lib/obj/*.o)
pids=""
for S in $SRCS; do
  STEM=$(basename $S .hip)
  OBJS=$(echo "$OBJS" | grep -v "/$STEM.o$")
  XF=$(python -c "import sys; sys.path.insert(0, '.'); from vsr_amd.build import SRC_FLAGS; print(' '.join(SRC_FLAGS.get('$S', [])))")
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result $XF -I include "$@" -c vsr_amd/csrc/$S -o $D/$STEM.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 $OBJS $(for S in $SRCS; do echo $D/$(basename $S .hip).o; done) -o $D/libvsrk.so
echo built $D/libvsrk.so
