#!/bin/bash
# Dev recipe: SQ counters of the chain kernel (k_chain<float>) in the headline workload, one
# rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md limits: ≤ 8 SQ counters per pass).
# EKF_SERIAL=1: counter collection serialises dispatches, so the device-epoch schedule (a persistent
# chain waiting on bulk-stream kernels) would wait out its poll timeouts; one stream, one chain
# launch per chunk instead (the same per-step code).
# Usage (repo root on the box): bash tools/chain_pmc.sh <tag>
set -o pipefail
tag=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/${tag}_avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_LEVEL_LDS"; do
  i=$((i + 1))
  EKF_SERIAL=1 timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/${tag}_pmc$i -o pmc --output-format csv -- \
    python bench.py --steps 8 --warmup 2 --no-cpu --traffic off > gpurun_out/${tag}_pmc$i.log 2>&1 || echo "pass $i rc $?"
done
