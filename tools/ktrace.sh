#!/bin/bash
# The timed region under rocprofv3 --kernel-trace only (no API tracing, so the host side runs at
# its own speed), with the host clocks (EKF_BENCH_TRACE=1), for --steps 20 and 200.
# Usage: bash tools/ktrace.sh <tag> [bench args]
set -o pipefail
tag=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for K in 20 200; do
  EKF_BENCH_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d gpurun_out/${tag}_k${K} -o ${tag} -- python -u bench.py --steps $K --warmup 5 --no-cpu \
    --traffic off "$@" > gpurun_out/${tag}_k${K}.json 2> gpurun_out/${tag}_k${K}.err || exit $?
  python tools/region_timeline.py gpurun_out/${tag}_k${K} gpurun_out/${tag}_k${K}.err > gpurun_out/${tag}_k${K}_timeline.txt 2>&1
  head -30 gpurun_out/${tag}_k${K}_timeline.txt
done
