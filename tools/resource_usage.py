"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (dev tool).
    python tools/resource_usage.py [TU] [-DFLAG ...]   (TU = split unit, default 1: reference layout)"""
import re, subprocess, sys
tu = next((a for a in sys.argv[1:] if not a.startswith("-")), "1")
defs = [a for a in sys.argv[1:] if a.startswith("-D")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", f"-DPF_TU={tu}", *defs,
       "-Iinclude", "-Idistributed-forecasting_amd/csrc", "-o", "/tmp/_res.o",
       "distributed-forecasting_amd/csrc/pf_engine.hip", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for n, r in rows.items():
    print(f"{n[:58]:58s} VGPR={r.get('VGPRs', '?'):>4} AGPR={r.get('AGPRs', '?'):>3} "
          f"spillV={r.get('VGPRs Spill', '?'):>4} spillS={r.get('SGPRs Spill', '?'):>4} "
          f"scratch={r.get('ScratchSize [bytes/lane]', '?'):>5} occ={r.get('Occupancy [waves/SIMD]', '?')}")
