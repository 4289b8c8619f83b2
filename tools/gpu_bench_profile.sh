#!/bin/bash
# One GPU session: driver-style bench line, rocprofv3 kernel trace of a short bench, and the two
# PMC passes (FETCH_SIZE / WRITE_SIZE) of an eager step for roofline.traffic.
# usage: bash tools/gpu_bench_profile.sh <tag>
set -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 560 python bench.py --steps 20 --warmup 5 --probe-detail $OUT/probe_shapes.txt \
  > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
echo "bench done"; tail -c 600 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- \
  python bench.py --steps 6 --warmup 2 --no-decode --no-cpu-baseline --probe-steps 1 \
  > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed $?"; exit 1; }
echo "trace done"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python bench.py --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0 \
  > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed $?"; exit 1; }
echo "pmc fetch done"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python bench.py --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0 \
  > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed $?"; exit 1; }
echo "pmc write done"
find $OUT -name "*.csv" | head -20
