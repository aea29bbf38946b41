#!/bin/bash
# heartbeat: a line every 30 s into gpurun_out/<tag>_hb.log while the given command runs (each
# command keeps its own time limit); exits with the command's status
tag=${1:?tag}; shift
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/${tag}_hb.log; sleep 30; done ) &
hb=$!
"$@"
rc=$?
kill $hb
exit $rc
