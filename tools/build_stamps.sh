#!/bin/sh
# Diagnostic library for tools/stamps*.py (-DPF_STAMPS); never loaded by the product.
# Extra -D flags are passed through (experiment variants): build_stamps.sh [OUT [-DX ...]]
cd "$(dirname "$0")/.." || exit 1
out="${1:-diag_exp/libprophet_hip_stamps.so}"
[ $# -gt 0 ] && shift
exec python distributed-forecasting_amd/build.py --out "$out" -DPF_STAMPS "$@"
