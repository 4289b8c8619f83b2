#!/bin/bash
# Run GPU steps in order; each step: "<seconds> <logname> <command...>" from a step file.
# A failing step (ordinary non-zero exit, e.g. a test failure) does not stop the sequence, but a
# time limit (124/137), an abort (134) or a segfault (139) does: nothing more touches the GPU.
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
  case $rc in 124|137|134|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done < $STEPS
