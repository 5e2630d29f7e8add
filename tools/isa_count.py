#!/usr/bin/env python3
"""Instruction mix of one kernel's loop bodies in a hipcc -S listing.

    hipcc --offload-arch=gfx950 ... --cuda-device-only -S -o x.s csrc/screen32.hip
    python tools/isa_count.py x.s <symbol substring> [--all]

Prints, per basic block that holds an MFMA (or every block with --all), the
count of VALU / MFMA / LDS / VMEM / SALU instructions and the top mnemonics.
"""
import collections
import re
import sys


def blocks(path, sym):
    body, on = [], False
    with open(path) as fh:
        for line in fh:
            if not on and re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", line):
                on = True
                continue
            if on:
                if line.startswith(".Lfunc_end"):
                    break
                body.append(line.rstrip())
    cur, name = [], "entry"
    for line in body:
        m = re.match(r"^(\.LBB\S+):", line)
        if m:
            yield name, cur
            cur, name = [], m.group(1)
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s.split()[0])
    yield name, cur


def kind(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    every = "--all" in sys.argv
    for name, ops in blocks(path, sym):
        c = collections.Counter(kind(o) for o in ops)
        if not ops or (not every and not c["mfma"]):
            continue
        top = collections.Counter(o for o in ops if kind(o) == "valu").most_common(14)
        print(f"{name}: {len(ops)} instr  " + "  ".join(f"{k}={v}" for k, v in sorted(c.items())))
        print("   " + ", ".join(f"{o}:{n}" for o, n in top))


if __name__ == "__main__":
    main()
