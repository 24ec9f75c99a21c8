#!/bin/bash
# Pre-flight + gpurun: rebuild the in-tree library if its build id does not
# match the sources (a stale .so is refused on the box), then run the command
# on the GPU box, retrying only while no box is free (exit 3: nothing ran).
cd "$(dirname "$0")/.." || exit 1
python distributed-forecasting_amd/build.py >/dev/null 2>&1 || { echo "build failed"; exit 1; }
python -c "import sys; sys.path.insert(0, '.'); from distributed_forecasting_amd import _lib; _lib.check_build_id()" || exit 1
exec bash tools/gpurun_retry.sh "$@"
