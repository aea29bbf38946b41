#!/bin/bash
# dev only: the GPU suite, then the association lines of tools/profile_round.sh (CPU leg, parity,
# PMC traffic) and the rocprofv3 stats of the fp32 association command, for <tag>.
# Usage (repo root on the box): bash tools/assoc_final.sh <tag>
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${tag}_gpu_tests.log
grep FAILED gpurun_out/${tag}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in n1024_fp32_assoc n1024_fp64_assoc; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 \
    > gpurun_out/${tag}_${w}_s20.json 2> gpurun_out/${tag}_${w}_s20.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/${tag}_${w}_s20.json')); r=d['roofline']; print('$w', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/step; pass', round(r['avg_launch_us'],2), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'parity', d.get('parity',{}).get('pose_rmse_m'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_assoc -o prof --output-format csv -- \
  python -u bench.py --workload n1024_fp32_assoc --steps 20 --warmup 5 --no-cpu --traffic off \
  > gpurun_out/${tag}_prof_assoc.log 2>&1 || exit 3
f=$(find gpurun_out/${tag}_prof_assoc -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/${tag}_n1024_fp32_assoc_kernel_stats.csv
