#!/bin/bash
# Round-4 measurement session: driver-style bench line, rocprofv3 kernel trace of a short bench
# (step breakdown + families), and three PMC passes of an eager step (FETCH_SIZE, WRITE_SIZE,
# MFMA busy / instruction mix).  Each GPU step has its own time limit; the first failure stops.
# usage: bash tools/gpu_profile_r4.sh <tag>
set -o pipefail
TAG=${1:-r4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --probe-detail $OUT/probe_shapes.txt \
  > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
echo "bench done"; tail -c 400 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-decode --no-cpu-baseline --probe-steps 1 \
  > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed $?"; exit 1; }
echo "trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0 \
  > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed $?"; exit 1; }
echo "pmc fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0 \
  > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed $?"; exit 1; }
echo "pmc write done"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU \
  SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_mfma -o run -- \
  python3 bench.py --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0 \
  > $OUT/pmc_mfma.log 2>&1 || { echo "pmc mfma failed $?"; exit 1; }
echo "pmc mfma done"
find $OUT -name "*.csv" -o -name "*.db" | head -20
