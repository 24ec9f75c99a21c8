#!/bin/bash
# End-of-round measurement on the GPU box (run through gpurun):
# GPU tests, the full bench.py line, the other BASELINE configs, then the
# rocprofv3 trace + PMC passes of the headline.  Outputs: gpurun_out/<tag>_*.
set -o pipefail
TAG=${1:-r03z}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "tests failed"; tail -5 $O/${TAG}_gpu_tests.log; exit 1; }
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
echo bench ok
timeout -k 10 300 python tools/bench_configs.py 3 > $O/${TAG}_configs2.json 2> /dev/null || { echo "configs2 failed"; exit 1; }
echo configs2 ok
timeout -k 10 400 python tools/bench_configs.py 4 --e-sample 0 > $O/${TAG}_configs3.json 2> /dev/null || { echo "configs3 failed"; exit 1; }
echo configs3 ok
timeout -k 10 500 python tools/bench_configs.py 5 --chunk 50000 > $O/${TAG}_configs4.json 2> /dev/null || { echo "configs4 failed"; exit 1; }
echo configs4 ok
bash tools/profile_round.sh $TAG || exit 1
