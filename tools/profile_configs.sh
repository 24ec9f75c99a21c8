#!/bin/bash
# rocprofv3 passes over tools/bench_configs.py (run ON the GPU box through
# gpurun): kernel trace + stats, then PMC passes each alone — HBM bytes
# (FETCH_SIZE, WRITE_SIZE), SQ wave states, FP64 MFMA / VALU mix, LDS.
# Usage: bash tools/profile_configs.sh <tag> <config 3|4|5> <n> [chunk]
#        (outputs under gpurun_out/prof_<tag>/; summarise with tools/pmc_summary.py)
set -o pipefail
TAG=$1
CFG=$2
N=$3
CH=${4:-$3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_configs.py $CFG $N --chunk $CH --e-sample 0"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1 || { echo "$name pass failed rc=$?"; exit 1; }
  echo "$name ok"
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
run pmc_mfma --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES
run pmc_lds --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM
