#!/bin/bash
# The headline bench under the three stream hand-off schedules (device epochs = default, events,
# one stream): value, ms per message, status flags, chain / factor / Σ-pass kernel times.
set -o pipefail
mkdir -p gpurun_out
for mode in "EKF_DEVSYNC=1" "EKF_DEVSYNC=0" "EKF_SERIAL=1"; do
  env $mode timeout -k 10 200 python -u bench.py --no-cpu --traffic off --steps 200 "$@" \
    > gpurun_out/modes_$mode.json 2> gpurun_out/modes_$mode.err || exit $?
  echo "$mode $(python -c "import json;d=json.load(open('gpurun_out/modes_$mode.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], d['config']['status_flags_rank0'], r.get('chain_kernel_avg_us'), r.get('factor_kernel_avg_us'), r['avg_launch_us'])")"
done
