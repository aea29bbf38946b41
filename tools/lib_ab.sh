#!/bin/bash
# A/B of library builds (EKF_LIB=<name>.so) on bench workloads, alternating; prints value and
# ms per step only (any workload). Usage: bash tools/lib_ab.sh <tag> "<libs>" "<workloads>" [bench args...]
set -o pipefail
tag=${1:?tag}; libs=${2:?libs}; wls=${3:?workloads}; shift 3
mkdir -p gpurun_out
for w in $wls; do
  for run in a b; do
    for lib in $libs; do
      o=gpurun_out/${tag}_${w}_${lib%.so}_${run}
      EKF_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu --traffic off "$@" > $o.json 2> $o.err || exit $?
      echo "$w $lib $run $(python -c "import json;d=json.load(open('$o.json'));print(round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step', d['config'].get('status_flags_rank0'))")"
    done
  done
done
