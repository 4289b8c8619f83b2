#!/bin/bash
# A/B builds of the fused stem kernel (retr_amd/csrc/stem.hip) as stand-alone libraries under
# tools/_ab/ (each exports retr_stem_pool_fwd; linked with the library's capi.o):
#   stem_head.so  the kernel at git HEAD        stem_cur.so  the working tree
#   stem_diag9.so the working tree with per-wave phase stamps (retr_stem_prof)
# then on the GPU: python tools/stem_micro.py tools/_ab/stem_*.so
set -e
cd "$(dirname "$0")/.."
make -s build/obj/capi.o
mkdir -p tools/_ab build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics"
build() {  # name source extra-flags
  /opt/rocm/bin/hipcc $F -Iretr_amd/csrc $3 -c $2 -o build/ab/$1.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/ab/$1.o build/obj/capi.o -o tools/_ab/$1.so
}
if git cat-file -e HEAD:retr_amd/csrc/stem.hip 2>/dev/null; then
  git show HEAD:retr_amd/csrc/stem.hip > build/ab/stem_head.hip
  build stem_head build/ab/stem_head.hip "" &
fi
build stem_cur retr_amd/csrc/stem.hip "" &
build stem_diag9 retr_amd/csrc/stem.hip "-DSTEM_DIAG=9" &
for v in $STEM_VARIANTS; do build stem_$v retr_amd/csrc/stem.hip "-DSTEM_$v=1" & done
wait
ls -la tools/_ab/stem_*.so
