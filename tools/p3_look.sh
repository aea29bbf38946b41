#!/bin/bash
# Round 3: the factor look-back (PassArgs::fac_look) on the GPU — its bit-identity tests, the whole
# GPU suite, then the swarm bench with and without it (alternating). Usage: bash tools/p3_look.sh <tag>
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x --timeout 120 --timeout-method thread \
  -k "lookback or sync_modes or many_filters or rows_handoff" > gpurun_out/${tag}_look_tests.log 2>&1
rc=$?; tail -15 gpurun_out/${tag}_look_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for run in a b; do
  for look in 1 0; do
    o=gpurun_out/${tag}_swarm_look${look}_${run}
    EKF_FACLOOK=$look timeout -k 10 300 python -u bench.py --workload swarm_n256_fp64 --steps 20 --warmup 5 \
      --no-cpu --traffic off > $o.json 2> $o.err || exit 3
    python -c "import json; d=json.load(open('$o.json')); r=d['roofline']; print('look=$look $run', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), 'us/msg; pass', round(r['avg_launch_us'],1), 'factors', r.get('factor_kernel_avg_us'), 'chain', r.get('chain_kernel_avg_us'), 'flags', d['config'].get('status_flags_rank0'))"
  done
done
