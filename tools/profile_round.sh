#!/bin/bash
# A round's evidence (repo root on the box): full bench lines (CPU baseline, parity, PMC traffic) for
# the driver's shape (20 steps) and the steady state (200), the BASELINE.json configs, and the
# rocprofv3 --kernel-trace --stats summary of the driver-shape command.
# Usage: bash tools/profile_round.sh <tag>
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # <name> <bench args...>
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err || return 3
  python -c "import json; d=json.load(open('gpurun_out/${tag}_${name}.json')); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('${name}', '%.4g' % d['value'], round(d['ms_per_step']*1e3,2), 'us/step; kernel', r.get('kernel'), round(r['avg_launch_us'],2), 'us frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'cpu', c.get('value'), 'parity', d.get('parity',{}).get('pose_rmse_m'))"
}
line n1024_fp32_s20 --steps 20 --warmup 5 || exit 3
line n1024_fp32_s200 --steps 200 --warmup 20 || exit 3
line n1024_fp32_assoc_s20 --workload n1024_fp32_assoc --steps 20 --warmup 5 || exit 3
line n1024_fp64_assoc_s20 --workload n1024_fp64_assoc --steps 20 --warmup 5 || exit 3
line n1024_fp64_s20 --workload n1024_fp64 --steps 20 --warmup 5 || exit 3
line n256_fp64_s20 --workload n256_fp64 --steps 20 --warmup 5 || exit 3
line basic_world_s20 --workload basic_world --steps 20 --warmup 5 || exit 3
line swarm_n256_fp64_s20 --workload swarm_n256_fp64 --steps 20 --warmup 5 || exit 3
line n1024_fp32_joseph_s20 --workload n1024_fp32_joseph --steps 20 --warmup 5 || exit 3
line n1024_fp32_assoc_joseph_s20 --workload n1024_fp32_assoc_joseph --steps 20 --warmup 5 || exit 3
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in n1024_fp32 n1024_fp32_assoc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_$w -o prof --output-format csv -- \
    python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu --traffic off \
    > gpurun_out/${tag}_prof_$w.log 2>&1 || exit 3
  f=$(find gpurun_out/${tag}_prof_$w -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/${tag}_${w}_kernel_stats.csv
  head -8 gpurun_out/${tag}_${w}_kernel_stats.csv | cut -c1-160
done
