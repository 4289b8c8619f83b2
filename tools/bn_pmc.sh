#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss of the fused bottleneck kernel alone (tools/bn_micro.py on one
# library), three separate rocprofv3 passes; summary per kernel: python tools/bn_pmc_sum.py <out dir>
set -e
cd "$(dirname "$0")/.."
OUT=gpurun_out/bnpmc
LIB=${1:-tools/_ab/bns_0.so}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python tools/bn_micro.py $LIB > $OUT/fetch.log 2>&1
timeout -k 10 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python tools/bn_micro.py $LIB > $OUT/write.log 2>&1
timeout -k 10 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- python tools/bn_micro.py $LIB > $OUT/hit.log 2>&1
