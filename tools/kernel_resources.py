#!/usr/bin/env python3
"""Per-kernel register / LDS / spill usage of the built gfx950 code object
(libzipvoice_hip.so): unbundles .hip_fatbin and reads the AMDGPU metadata notes."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zipvoice_amd", "libzipvoice_hip.so")
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
with tempfile.TemporaryDirectory() as d:
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")])
    tgt = [t for t in subprocess.check_output([f"{LLVM}/clang-offload-bundler", "--list", "--type=o",
                                               f"--input={fb}"]).decode().split() if "gfx950" in t][0]
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           f"--targets={tgt}", f"--output={co}"])
    notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co]).decode()
recs, cur = [], None
for line in notes.splitlines():
    s = line.strip()
    if s.startswith("- .agpr_count:") or s.startswith("- .args:"):
        if cur:
            recs.append(cur)
        cur = {}
    m = re.match(r"-?\s*\.(\w+):\s*(\S+)", s)
    if m and cur is not None and m.group(1) in ("agpr_count", "vgpr_count", "sgpr_count", "name",
                                                 "group_segment_fixed_size", "vgpr_spill_count",
                                                 "private_segment_fixed_size"):
        cur[m.group(1)] = m.group(2)
if cur:
    recs.append(cur)
dem = subprocess.run(["c++filt"], input="\n".join(r.get("name", "?") for r in recs), text=True,
                     capture_output=True).stdout.splitlines()
print(f"{'kernel':70s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'lds':>7s} {'spill':>5s} {'scratch':>7s}")
for r, n in zip(recs, dem):
    n = n.split("(")[0]
    if pat and not pat.search(n):
        continue
    print(f"{n[:70]:70s} {r.get('vgpr_count','?'):>5s} {r.get('agpr_count','?'):>5s} "
          f"{r.get('sgpr_count','?'):>5s} {r.get('group_segment_fixed_size','?'):>7s} "
          f"{r.get('vgpr_spill_count','?'):>5s} {r.get('private_segment_fixed_size','?'):>7s}")
