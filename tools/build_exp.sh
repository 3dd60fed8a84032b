# Experimental library for A/B runs: every object of the last full build plus
# csrc/$1 recompiled with extra flags ($2...), linked to vsr_amd/_lib/exp/libvsrk_exp.so
# (load it with VSRK_LIB=vsr_amd/_lib/exp/libvsrk_exp.so).
set -e
cd "$(dirname "$0")/.."
SRC=$1; shift
STEM=$(basename $SRC .hip)
O=vsr_amd/_lib/exp/$STEM.o
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -I include "$@" -c vsr_amd/csrc/$SRC -o $O
OBJS=$(ls vsr_amd/_lib/obj/*.o | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 $OBJS $O -o vsr_amd/_lib/exp/libvsrk_exp.so
echo built vsr_amd/_lib/exp/libvsrk_exp.so
