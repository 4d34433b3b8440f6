#!/bin/bash
# Runs GPU steps in order on the gpurun box.  Each step has its own time limit; an ordinary
# test failure (exit 1) lets later steps run, anything else (timeout, abort, fault) stops.
# usage: tools/gpu_steps.sh name:seconds:'command' ...
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
done
