"""Summarise a tools/profile_round.sh output directory into profiles/.

    python tools/pmc_summary.py gpurun_out/prof_r01 r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of
bench.py), profiles/<tag>_pmc.json (per-kernel averages of every counter) and
profiles/pmc_k_fit.json (the HBM bytes per launch of the headline's dominant
kernel — k_fit_forecast, else k_fit_polish — bench.py reports as
roofline.traffic).  HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on
gfx950 FETCH_SIZE counts half of a wide coalesced read stream
(MI355X_MICROARCH.md §HBM)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def read_counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(src, tag):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    keep_fit = len(sys.argv) < 4 or sys.argv[3] != "--no-fit-traffic"
    out = defaultdict(dict)
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            out[row["Name"]]["avg_ns"] = float(row["AverageNs"])
            out[row["Name"]]["calls"] = int(row["Calls"])
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_mfma", "pmc_lds", "pmc_valu"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for k, cs in read_counters(p).items():
            for c, v in cs.items():
                out[k][c] = sum(v) / len(v)
    for k, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            if "avg_ns" in d:
                d["hbm_GBps"] = d["hbm_bytes_per_launch"] / d["avg_ns"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"] > 0:
            w = d["SQ_WAVE_CYCLES"]
            d["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / w
            d["frac_wait_inst_any"] = d.get("SQ_WAIT_INST_ANY", 0) / w
            d["frac_active_inst_any"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
            if "SQ_ACTIVE_INST_VALU" in d:
                # ACTIVE_INST_* and WAVE_CYCLES are both quad-cycle counts
                d["frac_active_inst_valu"] = d["SQ_ACTIVE_INST_VALU"] / w
        if "SQ_INSTS_VALU_MFMA_MOPS_F64" in d:
            # one MOP = 512 FLOP (gfx9 MFMA MOPS unit); 16x16x4 f64 = 2048 FLOP = 4 MOPS
            d["mfma_f64_flops_per_launch"] = 512.0 * d["SQ_INSTS_VALU_MFMA_MOPS_F64"]
        if d.get("SQ_ACTIVE_INST_LDS", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in d:
            d["lds_bank_conflict_per_active_lds"] = d["SQ_LDS_BANK_CONFLICT"] / d["SQ_ACTIVE_INST_LDS"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("SQ_BUSY_CU_CYCLES", 0) > 0:
            d["mfma_busy_per_cu_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / d["SQ_BUSY_CU_CYCLES"]
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    kf = next((k for k in ("k_fit_forecast", "k_fit_polish", "k_fit") if k in out), "k_fit")
    if keep_fit and kf in out and "hbm_bytes_per_launch" in out[kf]:
        with open(os.path.join(prof, "pmc_k_fit.json"), "w") as f:
            json.dump({"tag": tag, "kernel": kf,
                       "hbm_bytes_per_launch": out[kf]["hbm_bytes_per_launch"],
                       "FETCH_SIZE_KiB": out[kf]["FETCH_SIZE"],
                       "WRITE_SIZE_KiB": out[kf]["WRITE_SIZE"],
                       "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)"},
                      f, indent=1)
    if keep_fit and "SQ_INSTS_VALU" in out.get("k_predict_mc", {}):
        # the headline's K5 instruction count (bench.py forecast_roofline:
        # the default bench shape, 500 series, 90-day horizon)
        d = out["k_predict_mc"]
        with open(os.path.join(prof, "pmc_k_predict_mc.json"), "w") as f:
            json.dump({"tag": tag, "kernel": "k_predict_mc", "n_series": 500, "horizon": 90,
                       "SQ_INSTS_VALU": d["SQ_INSTS_VALU"], "avg_ns": d.get("avg_ns"),
                       "SQ_WAVES": d.get("SQ_WAVES")}, f, indent=1)
    for k in ("k_fit", "k_fit_polish", "k_fit_forecast", "k_fit_tile", "k_polish", "k_predict_det",
              "k_predict_mc"):
        if k in out:
            print(k, {a: (round(b, 4) if isinstance(b, float) else b) for a, b in out[k].items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
