#!/bin/bash
# Swarm workloads with host-replayed and device-simulated inputs (include/ekf_sim.h).
set -o pipefail
mkdir -p gpurun_out
tag=${1:-inputs}
for wl in swarm_basic_world swarm_n256_fp64; do
  for inp in device host; do
    timeout -k 10 300 python -u bench.py --workload $wl --inputs $inp --no-cpu --traffic off \
      --steps ${STEPS:-100} > gpurun_out/${tag}_${wl}_${inp}.json 2> gpurun_out/${tag}_${wl}_${inp}.err || exit $?
    echo "$wl $inp $(python -c "import json;d=json.load(open('gpurun_out/${tag}_${wl}_${inp}.json'));print(d['value'], d['ms_per_step'], d['config']['status_flags_rank0'], d['roofline'].get('kernel_corrections_per_s', d['roofline'].get('avg_launch_us')))")"
  done
done
