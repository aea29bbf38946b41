#!/bin/bash
# GPU-box recipe for a round's measurement artefacts: the default bench line (with PMC traffic and
# the CPU baseline) and a rocprofv3 kernel-trace summary of the same workload.
# Usage (from the repo root on the box): bash tools/profile_round.sh <tag> [bench args...]
set -eo pipefail
tag=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench.py "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o ${tag} -- \
  python bench.py --no-cpu --traffic off "$@" > gpurun_out/${tag}_bench_prof.json 2> gpurun_out/${tag}_bench_prof.err
