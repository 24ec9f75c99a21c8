#!/bin/bash
# PMC passes over k_predict_mc in sample mode (configs[3] shape, n series; run
# ON the GPU box): wave-state and VALU / instruction-mix counters.
# Usage: bash tools/profile_mc.sh <tag> [n]   (outputs under gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-mc}
N=${2:-8000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/tools/diag_mc_select.py $N 3"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -T --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1 || { echo "sq pass failed rc=$?"; exit 1; }
echo sq ok
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES -T --output-format csv -d $OUT/pmc_valu -o run -- python3 $B > $OUT/pmc_valu.log 2>&1 || { echo "valu pass failed rc=$?"; exit 1; }
echo valu ok
