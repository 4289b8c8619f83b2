#!/bin/bash
# Round-5 measurement session on one MI355X: the driver-style bench line (cfg2) with its per-shape
# probe table, the cfg4 per-GPU slice, a rocprofv3 kernel trace of a short graphed bench (step
# breakdown + families), three PMC passes of an eager step (FETCH_SIZE, WRITE_SIZE, MFMA busy /
# instruction mix; two steps each) and a decode kernel trace.  Every GPU step has its own limit;
# the first failure stops the script.   usage: bash tools/gpu_profile_r5.sh <tag>
set -o pipefail
TAG=${1:-r5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 20 --warmup 5 --probe-detail $OUT/probe_shapes.txt \
  > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; exit 1; }
echo "bench done"; tail -c 300 $OUT/bench.json
timeout -k 10 300 python bench.py --workload cfg4 --steps 10 --warmup 3 --no-decode \
  > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || { echo "cfg4 failed $?"; exit 1; }
echo "cfg4 done"
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
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dec -o run -- \
  python3 tools/decode_prof.py --reps 2 > $OUT/dec_prof.log 2>&1 || { echo "dec trace failed $?"; exit 1; }
echo "dec trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/decb -o run -- \
  python3 tools/decode_prof.py --reps 2 --beam 5 > $OUT/decb_prof.log 2>&1 || { echo "beam trace failed $?"; exit 1; }
echo "beam trace done"
# summaries here (the raw traces are large): families / step breakdown / PMC tables
T=$(find $OUT/trace -name "*.db" | head -1)
python tools/rocprof_families.py $T > $OUT/rocprof_families.txt 2>&1
python tools/prof_step.py $T > $OUT/rocprof_step_breakdown.txt 2>&1
python tools/prof_summary.py $T --top 60 > $OUT/rocprof_summary.txt 2>&1
D=$(find $OUT/dec -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $D --top 30 > $OUT/rocprof_decode.txt 2>&1
DB=$(find $OUT/decb -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $DB --top 30 > $OUT/rocprof_decode_beam.txt 2>&1
F=$(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1)
W=$(find $OUT/pmc_write -name "*counter_collection.csv" | head -1)
M=$(find $OUT/pmc_mfma -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py $F $W --out $OUT/pmc_traffic.json --steps 2 \
  --source "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of bench.py --eager --steps 1 --warmup 1 --no-decode (round 5 final tree, $TAG)" > $OUT/pmc_traffic.txt 2>&1
python tools/pmc_mfma.py $M --out $OUT/pmc_mfma.json --by-kernel 30 \
  --source "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_* of bench.py --eager --steps 1 --warmup 1 --no-decode ($TAG)" > $OUT/pmc_mfma.txt 2>&1
rm -f $T $D $DB $F $W $M
echo "summaries done"
