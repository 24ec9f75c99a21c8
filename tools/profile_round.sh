#!/bin/bash
# rocprofv3 passes for one round (run ON the GPU box through gpurun):
#   1. kernel trace + stats of bench.py (the committed summary)
#   2..5. PMC passes, each alone: FETCH_SIZE / WRITE_SIZE (HBM bytes), SQ
#      wave-state counters, and FP64 MFMA / VALU counters (MFMA use of the
#      polish Hessian, VALU issue of the L-BFGS row pass)
# Usage: bash tools/profile_round.sh <tag> [bench args]  (outputs under gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-r02}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-variants $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/pmc_write -o run -- python3 $B > $OUT/pmc_write.log 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo write ok
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -T --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1 || { echo "sq pass failed rc=$?"; exit 1; }
echo sq ok
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES -T --output-format csv -d $OUT/pmc_mfma -o run -- python3 $B > $OUT/pmc_mfma.log 2>&1 || { echo "mfma pass failed rc=$?"; exit 1; }
echo mfma ok
