#!/bin/bash
# GPU suite, then the fixed cost of a timed region: kernel-trace timelines of --steps 20 / 200 and
# plain bench lines of both shapes. Usage: bash tools/p3_fixed.sh <tag>
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/p3_ktrace.sh ${tag} > /dev/null || exit 3
for K in 20 200; do head -4 gpurun_out/${tag}_k${K}_timeline.txt; done
for run in a b; do
  for K in 20 200; do
    o=gpurun_out/${tag}_s${K}_${run}
    timeout -k 10 300 python -u bench.py --steps $K --warmup 5 --no-cpu --traffic off > $o.json 2> $o.err || exit 3
    python -c "import json; d=json.load(open('$o.json')); print('steps $K $run', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/msg')"
  done
done
