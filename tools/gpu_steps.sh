#!/bin/bash
# Run GPU steps in order; each step: "<seconds> <logname> <command...>" from a step file.
# A failing step (ordinary non-zero exit, e.g. a test failure) does not stop the sequence, but a
# time limit (124/137) or a signal death (>= 128: abort, segfault, FPE) does: nothing more
# touches the GPU.
# usage: bash tools/gpu_steps.sh <tag> <stepfile>
TAG=$1; STEPS=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
while IFS= read -r line; do
  [ -z "$line" ] && continue
  secs=${line%% *}; rest=${line#* }; name=${rest%% *}; cmd=${rest#* }
  echo "== $name ($secs s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -3 $OUT/$name.log
  # time limit (124, 137) or any signal death (>= 128: abort, segfault, FPE, ...): stop here
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < $STEPS
