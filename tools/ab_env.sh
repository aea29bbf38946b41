#!/bin/bash
# Dev A/B: alternating bench runs of two environment settings on one box (value, ms/step, chain us).
# Usage: bash tools/ab_env.sh <tag> "<env A>" "<env B>" <rounds> [bench args]
set -o pipefail
tag=$1; A=$2; B=$3; R=$4; shift 4
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for side in A B; do
    envs=$A; [ $side = B ] && envs=$B
    env $envs timeout -k 10 300 python -u bench.py --no-cpu --traffic off --no-fp64 "$@" \
      > gpurun_out/${tag}_${side}${i}.json 2> gpurun_out/${tag}_${side}${i}.err || exit $?
    python - "$side" "$i" "gpurun_out/${tag}_${side}${i}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]}{sys.argv[2]}: {d['value']:.4e} corr/s  {d['ms_per_step']*1e3:.2f} us/msg  chain {r['chain_kernel_avg_us']:.2f} us  pass {r['avg_launch_us']:.2f} us", flush=True)
PY
  done
done
