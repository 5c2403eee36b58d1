#!/usr/bin/env python3
"""Build libzipvoice_hip.so (gfx950) in-tree with hipcc.  No torch involvement:
the library is a plain C-ABI shared object loaded with ctypes."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT = os.path.join(PKG, "libzipvoice_hip.so")
# the same sources with fp16 MFMA operands (the parity-grade fast mode's library)
OUT_F16 = os.path.join(PKG, "libzipvoice_hip_f16.so")
VARIANTS = ((OUT, ()), (OUT_F16, ("ZV_OPERAND_F16",)))
SRC = os.path.join(HERE, "zv_engine.hip")
DEPS = [os.path.join(HERE, f) for f in os.listdir(HERE)
        if f.endswith((".hip", ".inc", ".h"))] + [
    os.path.join(os.path.dirname(PKG), "include", "zipvoice_hip.h")]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def source_hash(defines=()):
    """sha256 over every source the library is built from (+ the extra defines): embedded
    in the library (zv_version) so a prebuilt .so can be checked against the tree."""
    import hashlib
    h = hashlib.sha256()
    for d in sorted(DEPS):
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    for d in defines:
        h.update(d.encode())
    return h.hexdigest()[:16]


def library_hash(path=OUT):
    """The source hash a built library carries (None if absent / unreadable)."""
    import ctypes
    if not os.path.exists(path):
        return None
    try:
        v = ctypes.CDLL(path).zv_version
        v.restype = ctypes.c_char_p
        s = v().decode()
    except OSError:
        return None
    return s.split("src=")[1].split()[0] if "src=" in s else None


def up_to_date(out=OUT, defines=()):
    """Rebuild unless the in-tree library was built from exactly these sources."""
    if not os.path.exists(out):
        return False
    stamp = out + ".src"
    return os.path.exists(stamp) and open(stamp).read().strip() == source_hash(defines)


def _cmd(out, defines):
    digest = source_hash(defines)
    # ZV_EXTRA_FLAGS: extra compiler flags for alternative builds (A/B runs with --out)
    extra = os.environ.get("ZV_EXTRA_FLAGS", "").split()
    return digest, [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-munsafe-fp-atomics", "-Wno-unused-result", "-Wl,-Bsymbolic", *extra,
                    *[f"-D{d}" for d in defines], f'-DZV_SRC_HASH="{digest}"', "-o", out + ".tmp",
                    SRC]


def build(force=False, verbose=True, out=None, defines=()):
    """Build the engine libraries (both operand formats, compiled in parallel); with `out`,
    one alternative build (A/B runs)."""
    jobs = [(out, tuple(defines))] if out else list(VARIANTS)
    jobs = [(o, d) for o, d in jobs if force or out or not up_to_date(o, d)]
    procs = []
    for o, d in jobs:
        digest, cmd = _cmd(o, d)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((o, digest, subprocess.Popen(cmd)))
    for o, digest, pr in procs:
        if pr.wait() != 0:
            raise subprocess.CalledProcessError(pr.returncode, "hipcc " + o)
        os.replace(o + ".tmp", o)
        with open(o + ".src", "w") as f:
            f.write(digest + "\n")
    return out or OUT


if __name__ == "__main__":
    # build.py [--force] [--out PATH] [-DNAME ...]   (alternative builds for A/B runs)
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else None
    build(force="--force" in args, out=out,
          defines=[a[2:] for a in args if a.startswith("-D")])
