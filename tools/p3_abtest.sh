#!/bin/bash
# GPU suite, then an A/B of libekfslam.so against the listed variants on the given workloads.
# Usage: bash tools/p3_abtest.sh <tag> "<libs>" "<workload:steps:warmup> ..."
set -o pipefail
tag=${1:?tag}; libs=${2:?libs}; wls=${3:-"n1024_fp32:200:20"}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log; grep FAILED gpurun_out/${tag}_gpu_tests.log | head
[ $rc -ne 0 ] && exit $rc
for w in $wls; do
  IFS=: read wl st wu <<< "$w"
  bash tools/lib_ab.sh ${tag}_$wl "$libs" --workload $wl --steps $st --warmup $wu || exit $?
done
