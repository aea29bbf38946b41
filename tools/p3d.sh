set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/p3d_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p3d_gpu_tests.log; grep -E "FAILED" gpurun_out/p3d_gpu_tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
EKF_LIB=libekfslam_diag.so timeout -k 10 300 python -u tools/assoc_stamps.py f32 > gpurun_out/p3d_stamps.txt 2>&1; cat gpurun_out/p3d_stamps.txt | head -40
