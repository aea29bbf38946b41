#!/bin/bash
# GPU suite on the current build, then an alternating A/B of two library builds on the headline
# workload (20 and 200 messages). Usage: bash tools/p3_ab2.sh <tag> <libA> <libB>
set -o pipefail
tag=${1:?tag}; la=${2:?libA}; lb=${3:?libB}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for run in a b c; do
  for lib in $la $lb; do
    for K in 20 200; do
      o=gpurun_out/${tag}_${lib%.so}_s${K}_${run}
      EKF_LIB=$lib timeout -k 10 300 python -u bench.py --steps $K --warmup 5 --no-cpu --traffic off > $o.json 2> $o.err || exit 3
      python -c "import json; d=json.load(open('$o.json')); r=d['roofline']; print('$lib $K $run', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/msg chain', round(r.get('chain_kernel_avg_us') or 0, 2))"
    done
  done
done
