#!/bin/bash
# Builds A/B variants of the fused bottleneck kernel as stand-alone libraries under tools/_ab/
# (each exports retr_bottleneck_s1_fwd; linked with the library's capi.o for the launch check):
#   bn_head.so   the kernel at git HEAD          bn_cur.so   the working tree
#   bn_noremap.so  the working tree with BN_XCD_REMAP=0
# then on the GPU: python tools/bn_micro.py tools/_ab/bn_*.so
set -e
cd "$(dirname "$0")/.."
make -s build/obj/capi.o
mkdir -p tools/_ab build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics"
git show HEAD:retr_amd/csrc/bottleneck.hip > build/ab/bn_head.hip
build() {  # name source extra-flags
  /opt/rocm/bin/hipcc $F -Iretr_amd/csrc $3 -c $2 -o build/ab/$1.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/ab/$1.o build/obj/capi.o -o tools/_ab/$1.so
}
build bn_head build/ab/bn_head.hip "" &
build bn_cur retr_amd/csrc/bottleneck.hip "" &
build bn_w2early retr_amd/csrc/bottleneck.hip "-DBN_W2_EARLY=1" &
build bn_diag1 retr_amd/csrc/bottleneck.hip "-DBN_DIAG=1" &
build bn_diag2 retr_amd/csrc/bottleneck.hip "-DBN_DIAG=2" &
build bn_diag9 retr_amd/csrc/bottleneck.hip "-DBN_DIAG=9" &
wait
ls -la tools/_ab/bn_*.so
