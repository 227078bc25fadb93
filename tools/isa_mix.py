#!/usr/bin/env python3
"""Instruction mix of one kernel in a `hipcc --cuda-device-only -S` listing (static counts).

usage: tools/isa_mix.py <file.s> <kernel-name-substring> [top]
"""
import collections
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    pat, top = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN\S*:", l) and pat in l.split(":")[0])
    body = []
    for l in lines[start + 1:]:
        if l.strip().startswith("s_endpgm"):
            break
        m = re.match(r"^\s+([a-z][a-z0-9_]*)", l)
        if m and not l.strip().startswith("."):
            body.append(m.group(1))
    c = collections.Counter(body)
    kinds = collections.Counter(op.split("_")[0] for op in body)
    print(f"{pat}: {len(body)} instructions; " + ", ".join(f"{k} {v}" for k, v in kinds.most_common(8)))
    for op, n in c.most_common(top):
        print(f"  {n:6d} {op}")


if __name__ == "__main__":
    main()
