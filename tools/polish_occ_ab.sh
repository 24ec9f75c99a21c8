# A/B: standalone k_polish at 2 workgroups / CU (diag_exp/lib_w2.so) vs 1 (the build), configs[2] and configs[3]
set -o pipefail
summ() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernels_ms_total']; print(d['config_index'], round(d['value']), 'polish', round(k.get('k_polish',0),1), 'cert', d['map_certified'])"; }
for lib in diag_exp/lib_w2.so distributed-forecasting_amd/libprophet_hip.so; do
  timeout -k 10 200 python tools/bench_configs.py 3 --e-sample 0 --lib $lib 2>/dev/null | summ || exit 1
  timeout -k 10 200 python tools/bench_configs.py 4 250000 --e-sample 0 --lib $lib 2>/dev/null | summ || exit 1
done
