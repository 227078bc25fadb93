#!/usr/bin/env python3
"""VGPR / spill / LDS figures per kernel from a `hipcc --cuda-device-only -S` listing (AMDGPU metadata).

usage: tools/kernel_regs.py <file.s> [name-substring]
"""
import re
import sys


def main():
    t = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = t[t.find("amdhsa.kernels:"):]
    for blk in re.split(r"\n  - \.", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", "." + blk)
        if not name or pat not in name.group(1):
            continue
        f = {k: re.search(rf"\.{k}:\s+(\d+)", "." + blk) for k in
             ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size",
              "private_segment_fixed_size")}
        print(name.group(1)[:70], {k: int(v.group(1)) if v else None for k, v in f.items()})


if __name__ == "__main__":
    main()
