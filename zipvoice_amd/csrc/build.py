#!/usr/bin/env python3
"""Build libzipvoice_hip.so (gfx950) in-tree with hipcc.  No torch involvement:
the library is a plain C-ABI shared object loaded with ctypes."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT = os.path.join(PKG, "libzipvoice_hip.so")
SRC = os.path.join(HERE, "zv_engine.hip")
DEPS = [os.path.join(HERE, f) for f in os.listdir(HERE)
        if f.endswith((".hip", ".inc", ".h"))] + [
    os.path.join(os.path.dirname(PKG), "include", "zipvoice_hip.h")]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True, out=None, defines=()):
    if out is None and not force and up_to_date():
        return OUT
    out = out or OUT
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-munsafe-fp-atomics", "-Wno-unused-result", *[f"-D{d}" for d in defines],
           "-o", out + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # build.py [--force] [--out PATH] [-DNAME ...]   (alternative builds for A/B runs)
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else None
    build(force="--force" in args, out=out,
          defines=[a[2:] for a in args if a.startswith("-D")])
