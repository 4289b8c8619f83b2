#!/bin/bash
# Round-6 measurement session on one MI355X, every number of the round's evidence from one tree:
#   1. cfg2 PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy / instruction mix) of an eager step
#      -> profiles/pmc_{traffic,mfma}_cfg2.json on the box, so the bench line below reads this
#      tree's counters;
#   2. the same three passes on cfg4's per-GPU slice -> profiles/pmc_{traffic,mfma}_cfg4.json
#      (bench.py reports counters only for the workload they were collected on);
#   3. the driver-style cfg2 bench line (with the per-shape probe table) and the cfg4 slice line;
#   4. a rocprofv3 kernel trace of a short graphed cfg2 bench (step breakdown + families) and
#      decode traces (bf16 greedy, fp32 parity greedy, bf16 beam 5).
# Every GPU step has its own limit; the first failure stops the script.
#   usage: bash tools/gpu_profile_r6.sh <tag> [pmc|run|all]   (two gpurun calls: pmc, then run)
set -o pipefail
TAG=${1:-r6}
PHASE=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $OUT/$name.log; exit 1; fi
}
pmc() {  # workload
  local wl=$1
  step pmc_fetch_$wl 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$wl -o run -- \
    python3 bench.py --workload $wl --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0
  step pmc_write_$wl 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$wl -o run -- \
    python3 bench.py --workload $wl --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0
  step pmc_mfma_$wl 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU \
    SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc_mfma_$wl -o run -- \
    python3 bench.py --workload $wl --eager --steps 1 --warmup 1 --no-decode --no-cpu-baseline --probe-steps 0
  local F=$(find $OUT/pmc_fetch_$wl -name "*counter_collection.csv" | head -1)
  local W=$(find $OUT/pmc_write_$wl -name "*counter_collection.csv" | head -1)
  local M=$(find $OUT/pmc_mfma_$wl -name "*counter_collection.csv" | head -1)
  python tools/pmc_traffic.py $F $W --out $OUT/pmc_traffic_$wl.json --steps 2 \
    --source "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of bench.py --workload $wl --eager --steps 1 --warmup 1 --no-decode (round 6, $TAG)" \
    > $OUT/pmc_traffic_$wl.txt 2>&1 || { echo "pmc_traffic $wl failed"; exit 1; }
  python tools/pmc_mfma.py $M --out $OUT/pmc_mfma_$wl.json --by-kernel 30 \
    --source "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_* of bench.py --workload $wl --eager --steps 1 --warmup 1 --no-decode (round 6, $TAG)" \
    > $OUT/pmc_mfma_$wl.txt 2>&1 || { echo "pmc_mfma $wl failed"; exit 1; }
  cp $OUT/pmc_traffic_$wl.json profiles/pmc_traffic_$wl.json
  cp $OUT/pmc_mfma_$wl.json profiles/pmc_mfma_$wl.json
  rm -f $F $W $M
  echo "pmc $wl done"
}
if [ "$PHASE" != run ]; then
  pmc cfg2
  pmc cfg4
fi
[ "$PHASE" = pmc ] && exit 0
step bench 420 python bench.py --steps 20 --warmup 5 --probe-detail $OUT/probe_shapes.txt
cp $OUT/bench.log $OUT/bench.json
echo "bench done"; grep -o '"value": [0-9.]*' $OUT/bench.json | head -3
step bench_cfg4 300 python bench.py --workload cfg4 --steps 10 --warmup 3 --no-decode
cp $OUT/bench_cfg4.log $OUT/bench_cfg4.json
echo "cfg4 done"
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- \
  python3 bench.py --steps 6 --warmup 2 --no-decode --no-cpu-baseline --probe-steps 1
echo "trace done"
step dec 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dec -o run -- \
  python3 tools/decode_prof.py --reps 2
step dec32 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dec32 -o run -- \
  python3 tools/decode_prof.py --reps 2 --fp32
step decb 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/decb -o run -- \
  python3 tools/decode_prof.py --reps 2 --beam 5
echo "decode traces done"
# summaries (the raw traces are large)
T=$(find $OUT/trace -name "*.db" | head -1)
python tools/rocprof_families.py $T > $OUT/rocprof_families.txt 2>&1
python tools/prof_step.py $T > $OUT/rocprof_step_breakdown.txt 2>&1
python tools/prof_summary.py $T --top 60 > $OUT/rocprof_summary.txt 2>&1
for d in dec dec32 decb; do
  D=$(find $OUT/$d -name "*kernel_trace.csv" | head -1)
  python tools/prof_summary.py $D --top 30 > $OUT/rocprof_$d.txt 2>&1
  rm -f $D
done
rm -f $T
echo "summaries done"
