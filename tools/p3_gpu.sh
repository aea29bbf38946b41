#!/bin/bash
# Round 3 GPU call: the GPU suite, then short bench lines of the driver's shape for the workloads
# named after the tag (each under its own time limit; stops at the first crash / hang).
set -o pipefail
tag=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1
  rc=$?
  tail -4 gpurun_out/${tag}_gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
for w in "$@"; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu --traffic off \
    > gpurun_out/${tag}_${w}.json 2> gpurun_out/${tag}_${w}.err || { echo "bench $w failed"; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/${tag}_${w}.json')); print('$w', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step')"
done
