#!/bin/bash
# Builds tools/_ab/wave_reduce_check.so (tools/wave_reduce_check.hip against the library's
# common.hpp); then on the GPU: python tools/wave_reduce_check.py
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iretr_amd/csrc -shared \
  tools/wave_reduce_check.hip -o tools/_ab/wave_reduce_check.so
