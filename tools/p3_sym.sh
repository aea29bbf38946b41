#!/bin/bash
# GPU suite, then the Σ-pass workloads (headline, fp64, configs[1], the swarm) with the pass's
# average launch time. Usage (repo root on the box): bash tools/p3_sym.sh <tag> [skip-tests]
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log; grep FAILED gpurun_out/${tag}_gpu_tests.log | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
fi
for spec in "n1024_fp32 200 20" "n1024_fp64 200 20" "n256_fp64 200 20" "swarm_n256_fp64 50 10" "n1024_fp32 20 5"; do
  set -- $spec
  w=$1; st=$2; wu=$3
  o=gpurun_out/${tag}_${w}_s${st}
  timeout -k 10 300 python -u bench.py --workload $w --steps $st --warmup $wu --no-cpu --traffic off \
    > $o.json 2> $o.err || exit 3
  python -c "import json; d=json.load(open('$o.json')); r=d['roofline']; print('$w', '$st', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/step; pass', round(r['avg_launch_us'],2), 'us frac', round(r['frac'],3), 'chain', r.get('chain_kernel_avg_us'), 'factors', r.get('factor_kernel_avg_us'), 'flags', d['config'].get('status_flags_rank0'))"
done
