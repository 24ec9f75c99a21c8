#!/bin/sh
# Diagnostic library for tools/stamps.py (-DPF_STAMPS); never loaded by the product.
cd "$(dirname "$0")/.." && exec /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -DPF_STAMPS -Iinclude -Idistributed-forecasting_amd/csrc \
  -o diag_exp/libprophet_hip_stamps.so distributed-forecasting_amd/csrc/pf_engine.hip
