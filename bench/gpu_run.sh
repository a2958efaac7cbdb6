#!/bin/bash
# GPU-box driver for one gpurun call: runs the given steps in order, each under its
# own time limit; stops at the first step that crashed / timed out (exit >= 2 or a
# signal), continues after plain test failures (pytest exit 1).
#   bash bench/gpu_run.sh "<name>:<seconds>:<command>" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "[gpu_run] $(date +%T) start $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_run] $(date +%T) end $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "[gpu_run] stopping after $name (rc=$rc)"; exit $rc; fi
done
