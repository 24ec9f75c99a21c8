set -o pipefail
summ() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernels_ms_total']; print(d['config_index'], d['opt'], round(d['value']), 'polish', round(k.get('k_polish',0),1), 'tile', round(k.get('k_fit_tile',0),1), 'cert', d['map_certified'])"; }
for o in "" "--opt polish_lag_ratio=0.1" "--opt polish_lag_ratio=0.3 --opt polish_max_lag=8" "--opt polish_lag_ratio=0.5 --opt polish_max_lag=16"; do
  timeout -k 10 200 python tools/bench_configs.py 5 20000 --e-sample 0 $o 2>/dev/null | summ || exit 1
done
for o in "" "--opt polish_lag_ratio=0.3 --opt polish_max_lag=8"; do
  timeout -k 10 200 python tools/bench_configs.py 3 --e-sample 0 $o 2>/dev/null | summ || exit 1
done
