#!/bin/bash
# PMC passes over the sample-mode forecast kernels (k_predict_mc_hist /
# k_predict_mc) at the configs[3] shape, n series (run ON the GPU box).
# Usage: bash tools/profile_hist.sh <tag> [n]   (outputs under gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-hist}
N=${2:-20000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/tools/diag_mc_select.py $N 3"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 200 rocprofv3 "$@" -T --output-format csv -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1 || { echo "$name pass failed rc=$?"; exit 1; }
  echo "$name ok"
}
run trace --kernel-trace --stats
run pmc_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
run pmc_valu --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES
