#!/bin/bash
# One GPU-box call while iterating: the GPU tests matching a pytest -k expression, then (only if
# they pass) bench lines of the headline at the driver's shape (20 messages) and at 200 messages,
# printing value, µs per message, the chain / Σ-pass kernel times and the status flags.
# Usage (repo root on the box): bash tools/quick_check.sh <tag> "<pytest -k expr>" [bench args...]
set -o pipefail
tag=${1:?tag}; expr=${2:?pytest -k expression}; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$expr" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "$expr" > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/${tag}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for K in 20 200; do
  W=$(( K == 20 ? 5 : 20 ))
  timeout -k 10 300 python -u bench.py --steps $K --warmup $W --no-cpu --traffic off "$@" \
    > gpurun_out/${tag}_s$K.json 2> gpurun_out/${tag}_s$K.err || exit $?
  python3 - "$tag" "$K" <<'EOF'
import json, sys
d = json.load(open(f"gpurun_out/{sys.argv[1]}_s{sys.argv[2]}.json"))
r = d["roofline"]
print(d["config"]["workload"], "steps", sys.argv[2], "value %.4g" % d["value"],
      "us/msg %.2f" % (d["ms_per_step"] * 1e3), "chain %.2f" % r.get("chain_kernel_avg_us", 0),
      "pass %.2f" % r.get("avg_launch_us", 0), "assoc", r.get("assoc_kernel_avg_us"),
      "flags", d["config"]["status_flags_rank0"])
EOF
done
