#!/bin/bash
# A/B of library builds (EKF_LIB=<name>.so under ekf-slam_amd/) on one bench workload, alternating.
# Usage (repo root on the box): bash tools/lib_ab.sh <tag> "<lib1> <lib2> ..." [bench args...]
set -o pipefail
tag=${1:?tag}; libs=${2:?libs}; shift 2
mkdir -p gpurun_out
for run in a b; do
  for lib in $libs; do
    o=gpurun_out/${tag}_${lib%.so}_${run}
    EKF_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu --traffic off "$@" > $o.json 2> $o.err || exit $?
    echo "$lib $run $(python -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['config']['status_flags_rank0'], r.get('chain_kernel_avg_us'), r.get('factor_kernel_avg_us'), r['avg_launch_us'])")"
  done
done
