#!/bin/bash
# GPU suite, then the headline with HBM-resident inputs (default) against host inputs, 20 and 200 steps.
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log; grep FAILED gpurun_out/${tag}_gpu_tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for run in a b; do
for spec in "hbm 20 5" "host 20 5" "hbm 200 20" "host 200 20"; do
  set -- $spec
  o=gpurun_out/${tag}_${1}_s${2}_$run
  timeout -k 10 300 python -u bench.py --inputs $1 --steps $2 --warmup $3 --no-cpu --traffic off > $o.json 2> $o.err || exit 3
  python -c "import json; d=json.load(open('$o.json')); h=d.get('host_inputs') or {}; print('$1 $2 $run', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/step; host-input leg', '%.4g' % h.get('value', 0), round(h.get('ms_per_step', 0)*1e3, 2))"
done
done
