"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (dev tool)."""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "distributed-forecasting_amd/csrc/pf_engine.hip"
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Iinclude",
       "-Idistributed-forecasting_amd/csrc", "-o", "/tmp/_res.so", src, "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)([^\[]+?)\s*\[-Rpass", line)
    if not m: continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = txt.split(":", 1)[1].strip(); rows[cur] = {}
    elif cur and ":" in txt:
        k, v = txt.split(":", 1); rows[cur][k.strip()] = v.strip()
for n, r in rows.items():
    dm = subprocess.run(["llvm-cxxfilt", n], capture_output=True, text=True).stdout.strip() if False else n
    print(f"{dm[:60]:60s} VGPR={r.get('VGPRs','?'):>4} AGPR={r.get('AGPRs','?'):>3} SGPR={r.get('SGPRs','?'):>4} LDS={r.get('LDS Size [bytes/block]','?'):>5} "
          f"spillV={r.get('VGPRs Spill','?'):>4} spillS={r.get('SGPRs Spill','?'):>4} scratch={r.get('ScratchSize [bytes/lane]','?'):>4} occ={r.get('Occupancy [waves/SIMD]','?')}")
