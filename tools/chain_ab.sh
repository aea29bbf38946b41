#!/bin/bash
# A/B of chain kernel time per chunk (HIP events) between two libraries, alternating
set -o pipefail
for r in 1 2 3; do
  for lib in libekfslam.so libekfslam_base.so; do
    o=gpurun_out/cab_${lib%.so}_$r
    EKF_LIB=$lib timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > $o.json 2> $o.err || exit $?
    python -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print('$lib', $r, round(d['value']), 'chain %.3f'%r['chain_kernel_avg_us'], 'pass %.2f'%r['avg_launch_us'])"
  done
done
