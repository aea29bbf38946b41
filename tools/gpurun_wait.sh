#!/bin/bash
# Dev helper: gpurun, re-submitted only while the pool answers "no slot / no box free" (exit 3,
# nothing ran and nothing was charged); any other outcome is returned as is.
# Usage: tools/gpurun_wait.sh <timeout-s> '<command>'
t=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no slot (try $i), waiting 90 s" >&2
  sleep 90
done
exit 3
