#!/bin/bash
# Dev: kernel traces (rocpd) of the 200-message fp32 bench, two-stream and one-stream (EKF_SERIAL=1)
# schedules, for tools/bulk_timeline.py; with a workload argument, that workload's two-stream trace only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bl
if [ -n "$1" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/bl/$1 -o run -- python3 bench.py --workload $1 --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > gpurun_out/bl/$1.json 2> gpurun_out/bl/$1.err
  exit $?
fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/bl/def -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > gpurun_out/bl/def.json 2> gpurun_out/bl/def.err && \
EKF_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/bl/ser -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > gpurun_out/bl/ser.json 2> gpurun_out/bl/ser.err
