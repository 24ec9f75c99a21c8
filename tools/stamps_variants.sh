#!/bin/sh
# Run tools/stamps.py on every diag_exp/libstamps_*.so variant + the base stamps lib.
# usage: tools/stamps_variants.sh OUTPREFIX
p="${1:-gpurun_out/stamps}"
for lib in diag_exp/libprophet_hip_stamps.so diag_exp/libstamps_*.so; do
  n=$(basename "$lib" .so)
  echo "== $n" >> "$p.log"
  PF_STAMPS_LIB="$lib" timeout -k 10 120 python tools/stamps.py 500 >> "$p.log" 2>&1 || exit 1
done
