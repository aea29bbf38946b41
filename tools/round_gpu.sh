#!/bin/bash
# One GPU-box call of a round: the GPU test suite, then (unless a step crashed, hung or faulted) the
# default bench line and a rocprofv3 kernel-trace summary of the same workload.
# Usage (repo root on the box): bash tools/round_gpu.sh <tag> [tests|bench|all] [bench args...]
set -o pipefail
tag=${1:?tag}; what=${2:-all}; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${tag}_gpu_tests.log
  # 0 = green, 1 = assertion failures (the GPU is fine); anything else: stop here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  timeout -k 10 900 python -u bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
  cat gpurun_out/${tag}_bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o ${tag} -- \
    python bench.py --no-cpu --traffic off "$@" > gpurun_out/${tag}_bench_prof.json 2> gpurun_out/${tag}_bench_prof.err || exit $?
fi
