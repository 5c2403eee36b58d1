#!/usr/bin/env python3
"""Disassemble one kernel of the built gfx950 code object and summarise its loops.

usage: disasm.py LIB SYMBOL_REGEX [--dump]

Unbundles .hip_fatbin (as kernel_resources.py), runs llvm-objdump on the gfx950 object,
keeps the first function whose demangled name matches SYMBOL_REGEX, and prints the
instruction mix of every backward branch's body (the loops), by class: MFMA, transcendental
VALU (v_exp/v_log/v_rcp/...), other VALU, LDS, global/buffer, SALU, waitcnt/barrier.
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(lib, d):
    fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib,
                           os.path.join(d, "x")])
    tgt = [t for t in subprocess.check_output([f"{LLVM}/clang-offload-bundler", "--list", "--type=o",
                                               f"--input={fb}"]).decode().split() if "gfx950" in t][0]
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           f"--targets={tgt}", f"--output={co}"])
    return co


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
        return "valu_trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_barrier")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    lib, rx = sys.argv[1], re.compile(sys.argv[2])
    with tempfile.TemporaryDirectory() as d:
        co = code_object(lib, d)
        txt = subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--demangle", co]).decode()
    funcs = re.split(r"\n(?=[0-9a-f]{16} <)", txt)
    f = next((x for x in funcs if x[:400].find("<") >= 0 and rx.search(x.split("\n", 1)[0])), None)
    if f is None:
        sys.exit("no match")
    head, body = f.split("\n", 1)
    print(head)
    ins = []
    for line in body.splitlines():
        m = re.match(r"\s*([a-z_0-9]+)\b(.*?)//\s*([0-9A-F]+):", line)
        if m:
            ins.append((int(m.group(3), 16), m.group(1), m.group(2).strip(), line))
    if "--dump" in sys.argv:
        for a, op, args, _ in ins:
            print(f"{a:6x} {op} {args}")
    print(f"{len(ins)} instructions; total mix {dict(Counter(klass(o) for _, o, _, _ in ins))}")
    addr = {a: i for i, (a, _, _, _) in enumerate(ins)}
    for i, (a, op, args, line) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.match(r"(-?\d+)", args)
            if not m:
                continue
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off      # simm16, dwords after PC + 4
            j = addr.get(a + 4 + 4 * off)
            if j is not None and j < i:
                c = Counter(klass(o) for _, o, _, _ in ins[j:i + 1])
                print(f"loop {ins[j][0]:x}..{a:x}: {i - j + 1} instructions {dict(c)}")


if __name__ == "__main__":
    main()
