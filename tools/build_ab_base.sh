#!/bin/bash
# Build the committed HEAD's kernel library into tools/_ab/libretr_base.so (A/B timing only:
# RETR_AB_LIB=tools/_ab/libretr_base.so makes retr_amd._lib load it instead of the working tree's).
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$REPO" archive HEAD retr_amd/csrc include | tar -x -C "$TMP"
cd "$TMP"
for f in retr_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics \
    -Wno-unused-function -c "$f" -o "${f%.hip}.o" &
done
wait
mkdir -p "$REPO/tools/_ab"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 retr_amd/csrc/*.o -o "$REPO/tools/_ab/libretr_base.so"
rm -rf "$TMP"
echo "built $REPO/tools/_ab/libretr_base.so from $(git -C "$REPO" rev-parse --short HEAD)"
