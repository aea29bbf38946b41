#!/bin/bash
# A/B of one environment switch on bench workloads, alternating (repo root on the box).
# Usage: bash tools/env_ab.sh <tag> <VAR> "<values>" "<workloads>" [bench args...]
set -o pipefail
tag=${1:?tag}; var=${2:?var}; vals=${3:?values}; wls=${4:?workloads}; shift 4
mkdir -p gpurun_out
for w in $wls; do
  for run in a b; do
    for v in $vals; do
      o=gpurun_out/${tag}_${w}_${var}${v}_${run}
      env $var=$v timeout -k 10 300 python -u bench.py --workload $w --no-cpu --traffic off "$@" > $o.json 2> $o.err || exit $?
      echo "$w $var=$v $run $(python -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print(round(d['value']), round(d['ms_per_step']*1e3,2), 'us/msg pass', round(r.get('avg_launch_us',0),2), 'chain', round(r.get('chain_kernel_avg_us',0),2), d['config'].get('status_flags_rank0'), 'parity', d.get('parity',{}).get('pose_rmse_m'))")"
    done
  done
done
