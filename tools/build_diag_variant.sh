#!/bin/bash
# dev only: libekfslam_diag_<name>.so — the stamp build (EKF_DIAG_STAMPS) with ekf_kernels.hip taken
# from <src> and extra defines; the other objects are the current diag build's. For tools/chain_stamps.py
# (EKF_LIB=libekfslam_diag_<name>.so). Usage: bash tools/build_diag_variant.sh <name> <src> [-DFOO ...]
set -e
name=${1:?name}; src=${2:?src}; shift 2
cd "$(dirname "$0")/../ekf-slam_amd"
make -s libekfslam_diag.so
tmp=build/dvar_${name}_kernels.hip
cp "$src" $tmp
HF="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -I../include -Icsrc"
/opt/rocm/bin/hipcc $HF -DEKF_DIAG_STAMPS "$@" -x hip -c $tmp -o build/dvar_${name}_kernels.o
objs=$(ls build/diag_*.o | grep -v 'diag_ekf_kernels.hip.o')
/opt/rocm/bin/hipcc $HF -shared -Wl,-rpath,/opt/rocm/lib -o libekfslam_diag_${name}.so build/dvar_${name}_kernels.o $objs
echo built libekfslam_diag_${name}.so
