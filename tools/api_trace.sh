#!/bin/bash
# The 20-step timed region under rocprofv3 --kernel-trace --hip-trace with the host clocks
# (EKF_BENCH_TRACE=1); then tools/region_timeline.py on it. Usage: bash tools/api_trace.sh <tag> [bench args]
set -o pipefail
tag=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
EKF_BENCH_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv \
  -d gpurun_out/${tag}_trace -o ${tag} -- python -u bench.py --steps 20 --warmup 5 --no-cpu \
  --traffic off "$@" > gpurun_out/${tag}_trace.json 2> gpurun_out/${tag}_trace.err || exit $?
python tools/region_timeline.py gpurun_out/${tag}_trace gpurun_out/${tag}_trace.err > gpurun_out/${tag}_timeline.txt 2>&1
head -40 gpurun_out/${tag}_timeline.txt
