#!/bin/bash
# Round 3 GPU call: GPU suite, association stamps, then driver-shape bench lines (20 steps) for the
# headline and the association workloads, and the headline at 200 steps.
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_gpu_tests.log; grep FAILED gpurun_out/${tag}_gpu_tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
EKF_LIB=libekfslam_diag.so timeout -k 10 300 python -u tools/assoc_stamps.py f32 \
  > gpurun_out/${tag}_stamps.txt 2>&1 || exit $?
head -18 gpurun_out/${tag}_stamps.txt
for w in n1024_fp32 n1024_fp32 n1024_fp32_assoc n1024_fp64_assoc n1024_fp64; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu --traffic off \
    > gpurun_out/${tag}_${w}.json 2> gpurun_out/${tag}_${w}.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/${tag}_${w}.json')); print('$w', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step')"
done
timeout -k 10 400 python -u bench.py --steps 200 --no-cpu --traffic off > gpurun_out/${tag}_s200.json \
  2> gpurun_out/${tag}_s200.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/${tag}_s200.json')); print('s200', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step')"
