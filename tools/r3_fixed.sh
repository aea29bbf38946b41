#!/bin/bash
# Round 3: attribute the fixed cost of a short (--steps 20) timed replay. Two plain 20-step runs,
# one 200-step run, then a kernel + HIP API trace of the 20-step shape with host clocks around the
# timed region (EKF_BENCH_TRACE=1).
set -o pipefail
tag=${1:-r3a}
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --traffic off \
    > gpurun_out/${tag}_s20_$i.json 2> gpurun_out/${tag}_s20_$i.err || exit $?
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu --traffic off \
  > gpurun_out/${tag}_s200.json 2> gpurun_out/${tag}_s200.err || exit $?
EKF_BENCH_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv \
  -d gpurun_out/${tag}_trace -o ${tag} -- python -u bench.py --steps 20 --warmup 5 --no-cpu \
  --traffic off > gpurun_out/${tag}_trace.json 2> gpurun_out/${tag}_trace.err || exit $?
tail -c 300 gpurun_out/${tag}_s20_1.json gpurun_out/${tag}_s20_2.json gpurun_out/${tag}_s200.json
