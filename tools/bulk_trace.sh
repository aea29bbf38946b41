set -o pipefail
# Dev: kernel traces (rocpd) of the 200-message fp32 bench, two-stream and one-stream (EKF_SERIAL=1)
# schedules, for tools/bulk_timeline.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bl
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/bl/def -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > gpurun_out/bl/def.json 2> gpurun_out/bl/def.err && \
EKF_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/bl/ser -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --traffic off --no-fp64 > gpurun_out/bl/ser.json 2> gpurun_out/bl/ser.err
