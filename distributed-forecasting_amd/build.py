"""Build the gfx950 engine library in-tree (hipcc, no cmake)."""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
SOURCES = [os.path.join(_HERE, "csrc", "pf_engine.hip")]
DEPS = SOURCES + [os.path.join(_HERE, "csrc", "pf_common.h"),
                  os.path.join(_HERE, "csrc", "pf_polish.h"),
                  os.path.join(_HERE, "csrc", "pf_cv.h"),
                  os.path.join(_HERE, "csrc", "pf_ostat.h"),
                  os.path.join(_HERE, "csrc", "pf_mc.h"),
                  os.path.join(_HERE, "csrc", "pf_tile.h"),
                  os.path.join(_ROOT, "include", "prophet_hip.h")]
OUT = os.path.join(_HERE, "libprophet_hip.so")
ARCH = os.environ.get("PF_OFFLOAD_ARCH", "gfx950")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(_ROOT, "include"), "-I", os.path.join(_HERE, "csrc"),
           "-o", OUT + ".tmp", *SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
