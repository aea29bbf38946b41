#!/bin/bash
# Calibrates FETCH_SIZE / WRITE_SIZE against known byte counts (MI355X_MICROARCH.md: other access
# widths are uncalibrated): sigma_bench's float4 copy vs the Σ pass, same buffers.
set -eo pipefail
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/calib_$c -o calib --output-format csv -- ./tools/sigma_bench 1 > gpurun_out/calib_$c.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/calibpp_$c -o calib --output-format csv -- ./tools/sigma_bench 1 1 > gpurun_out/calibpp_$c.log 2>&1
done
