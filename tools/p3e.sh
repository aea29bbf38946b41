set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-p3e}
EKF_LIB=libekfslam_diag.so timeout -k 10 300 python -u tools/assoc_stamps.py f32 > gpurun_out/${tag}_stamps.txt 2>&1 || exit $?
head -20 gpurun_out/${tag}_stamps.txt
for w in n1024_fp32_assoc n1024_fp64_assoc; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu --traffic off \
    > gpurun_out/${tag}_${w}.json 2> gpurun_out/${tag}_${w}.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/${tag}_${w}.json')); print('$w', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step', d['roofline'].get('assoc_kernel_avg_us'))"
done
