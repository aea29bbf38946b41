#!/bin/bash
# configs[3] swarm under different stream/CU arrangements (EKF_CU_SPLIT=<CUs per XCD for the chains>,
# EKF_DEVSYNC), alternating. Usage (repo root on the box): bash tools/swarm_split.sh <tag> [bench args...]
set -o pipefail
tag=${1:?tag}; shift
mkdir -p gpurun_out
for run in a b; do
  for v in "0 1 0" "0 1 1" "4 0 0" "8 0 0" "16 0 0"; do
    set -- $v "$@"; split=$1; ds=$2; ser=$3; shift 3
    o=gpurun_out/${tag}_s${split}_d${ds}_x${ser}_${run}
    EKF_CU_SPLIT=$split EKF_DEVSYNC=$ds EKF_SERIAL=$ser timeout -k 10 150 python -u bench.py --workload swarm_n256_fp64 \
      --no-cpu --traffic off "$@" > $o.json 2> $o.err || exit $?
    echo "split=$split devsync=$ds serial=$ser $run $(python -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['config']['status_flags_rank0'], r.get('chain_kernel_avg_us'), r.get('factor_kernel_avg_us'), r['avg_launch_us'])")"
  done
done
