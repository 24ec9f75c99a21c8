#!/bin/bash
# PMC passes over the tiled fit (configs[2] shape, n series; run ON the GPU
# box through gpurun): kernel trace + SQ wave-state, instruction-mix and
# FP64 MFMA counters, each pass alone.
# Usage: bash tools/profile_tile.sh <tag> [n]   (outputs under gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-tile}
N=${2:-16384}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_configs.py 3 $N"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo trace ok
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -T --output-format csv -d $OUT/pmc_sq -o run -- python3 $B > $OUT/pmc_sq.log 2>&1 || { echo "sq pass failed rc=$?"; exit 1; }
echo sq ok
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES -T --output-format csv -d $OUT/pmc_mfma -o run -- python3 $B > $OUT/pmc_mfma.log 2>&1 || { echo "mfma pass failed rc=$?"; exit 1; }
echo mfma ok
if [ -n "$PF_EXTRA_PMC" ]; then
  timeout -k 10 200 rocprofv3 --pmc $PF_EXTRA_PMC -T --output-format csv -d $OUT/pmc_extra -o run -- python3 $B > $OUT/pmc_extra.log 2>&1 || { echo "extra pass failed rc=$?"; exit 1; }
  echo extra ok
fi
