#!/bin/bash
# Σ-pass change check: the lab (product vs lab tile), the GPU suite, then bench lines (20/200).
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/pass_lab 1024 200 > gpurun_out/${tag}_pass_lab.txt 2>&1 || exit 3
grep -E "product|region wpb4" gpurun_out/${tag}_pass_lab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for run in a b; do
  for K in 20 200; do
    o=gpurun_out/${tag}_s${K}_${run}
    timeout -k 10 300 python -u bench.py --steps $K --warmup 5 --no-cpu --traffic off > $o.json 2> $o.err || exit 3
    python -c "import json; d=json.load(open('$o.json')); r=d['roofline']; print('steps $K $run', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/msg; pass', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3))"
  done
done
