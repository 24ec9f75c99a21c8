"""Build the gfx950 engine library in-tree (hipcc, no cmake).

The library carries a build id: a SHA-256 over every file under csrc/ and
include/ plus the compile flags, baked in as ``PF_BUILD_ID`` and returned by
``pf_build_id()``.  ``build()`` recompiles whenever the id embedded in the
existing .so differs from the id of the sources on disk (not on mtimes: a
pushed tree may carry a prebuilt .so with any timestamp), and ``_lib.load()``
refuses a library whose id does not match the sources next to it.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
CSRC = os.path.join(_HERE, "csrc")
INCLUDE = os.path.join(_ROOT, "include")
SOURCES = [os.path.join(CSRC, "pf_engine.hip")]
OUT = os.path.join(_HERE, "libprophet_hip.so")
ARCH = os.environ.get("PF_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared"]
_ID_RE = re.compile(rb"PF_BUILD_ID:([0-9a-f]{32})")


def source_files(csrc: str = CSRC, include: str = INCLUDE) -> list:
    """Every file the library is compiled from (sorted, absolute)."""
    out = []
    for d in (csrc, include):
        if os.path.isdir(d):
            out += [os.path.join(d, f) for f in sorted(os.listdir(d))
                    if f.endswith((".h", ".hip", ".hpp"))]
    return out


def source_hash(csrc: str = CSRC, include: str = INCLUDE) -> str | None:
    """Build id of the sources on disk (None when they are absent)."""
    files = source_files(csrc, include)
    if not files:
        return None
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    for p in files:
        h.update(b"\0" + os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:32]


def embedded_id(so_path: str = OUT) -> str | None:
    """The build id baked into a built library (read from its bytes: no
    dlopen, so it works without a GPU runtime)."""
    if not os.path.exists(so_path):
        return None
    with open(so_path, "rb") as f:
        m = _ID_RE.search(f.read())
    return m.group(1).decode() if m else None


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    return embedded_id(OUT) != source_hash()


# pf_engine.hip compiles as N_TU translation units (PF_TU = 0: host API and
# non-fit kernels; 1..7: groups of fit-kernel instantiations) in parallel,
# then links into one shared library
N_TU = 8
OBJ_DIR = os.path.join(_ROOT, "build", "pf_objs")


def build(force: bool = False, verbose: bool = True, jobs: int | None = None,
          out: str | None = None, defines=()) -> str:
    """Compile the library (in-tree ``OUT`` by default).  ``out`` + ``defines``
    build a diagnostic variant (e.g. -DPF_STAMPS) elsewhere; it is never the
    library ``_lib.load()`` checks."""
    if out is None and not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    bid = source_hash()
    target = OUT if out is None else os.path.abspath(out)
    obj_dir = OBJ_DIR if out is None else target + ".objs"
    os.makedirs(obj_dir, exist_ok=True)
    jobs = jobs or min(N_TU, max(1, os.cpu_count() or 1), 16)
    compile_flags = [f for f in FLAGS if f != "-shared"]
    cmds = [[hipcc, *compile_flags, "-c", f"-DPF_TU={k}", f'-DPF_BUILD_ID="{bid}"', *defines,
             "-I", INCLUDE, "-I", CSRC, "-o", os.path.join(obj_dir, f"pf_tu{k}.o"), *SOURCES]
            for k in range(N_TU)]
    pending, running = list(cmds), []
    while pending or running:
        while pending and len(running) < jobs:
            c = pending.pop(0)
            if verbose:
                print(" ".join(c), file=sys.stderr)
            running.append((c, subprocess.Popen(c)))
        c, pr = running.pop(0)
        if pr.wait() != 0:
            for _, q in running:
                q.wait()
            raise subprocess.CalledProcessError(pr.returncode, c)
    link = [hipcc, *FLAGS, "-o", target + ".tmp"] + [os.path.join(obj_dir, f"pf_tu{k}.o") for k in range(N_TU)]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.check_call(link)
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    # python build.py [--force] [--out PATH] [-DNAME ...]
    args = sys.argv[1:]
    o = args[args.index("--out") + 1] if "--out" in args else None
    build(force="--force" in args, out=o, defines=[a for a in args if a.startswith("-D")])
