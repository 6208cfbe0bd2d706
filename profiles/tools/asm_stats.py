"""Instruction mix of hipcc-generated gfx950 kernels (static, from `-S --cuda-device-only` output).

Usage: python3 profiles/tools/asm_stats.py file.s [kernel-substring ...]
For each matching kernel: total instructions, f64 / f32 VALU, LDS, VMEM counts, and the same for
every loop body (a label that a later s_cbranch / s_branch jumps back to).
"""
import collections
import re
import sys


def kernels(txt):
    for m in re.finditer(r"^(_Z\S+):\s*;", txt, re.M):
        name = m.group(1)
        end = txt.index(".Lfunc_end", m.end())
        yield name, txt[m.end():end].split("\n")


def classify(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def mix(lines):
    c = collections.Counter()
    for l in lines:
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":"):
            continue
        c[classify(l.split()[0])] += 1
    return c


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    txt = open(path).read()
    for name, body in kernels(txt):
        if pats and not any(p in name for p in pats):
            continue
        print(name[:70])
        print("  kernel", dict(mix(body)))
        labels = {}
        for i, l in enumerate(body):
            s = l.strip()
            if re.match(r"^\.LBB\S+:", s):
                labels[s[:-1].split(":")[0]] = i
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\S+)", s)
            if m and m.group(2) in labels and labels[m.group(2)] < i:
                c = mix(body[labels[m.group(2)]:i + 1])
                print("  loop %s (%d lines)" % (m.group(2), i - labels[m.group(2)]), dict(c))


if __name__ == "__main__":
    main()
