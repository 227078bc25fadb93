"""Build-time check of K2V's register fence (semi-direct-visual-odometry_amd/csrc/align_refv.hip).

K2V keeps rows 0..87 of each pair's residual vector in the VGPRs v80..v255, written and read only by its
inline-asm blocks.  The compiler is not told about them outside those blocks, so this check reads the
generated assembly of every K2V kernel and fails when an instruction outside an ;;#ASMSTART / ;;#ASMEND
block names a VGPR >= the fence (or M0, which the indexed row moves set), when a compiler-chosen operand
of those blocks is >= the fence, or when a kernel's VGPR count is not 256 (the data registers must be
allocated) or it allocates AGPRs.

usage: python3 tools/check_vreg_fence.py <device assembly .s> [fence]
"""
import re
import sys

KERNELS = ("align_scale_refv_kernel", "debug_robust_scale_v_kernel")
REG = re.compile(r"\bv\[?(\d+)(?::(\d+))?\]?")
# the indexed data operands the asm blocks name (rows r..r+3 of an index session)
DATA_OPERANDS = {f"v{i}" for i in range(80, 88)} | {f"v[{i}:{i + 1}]" for i in range(80, 88, 2)}
# the fixed data operands of the MAD pass's in-place |x - med| block (every row's pair and its high word) and of
# the LDS reads of wave 0's staged rows
MAD_OPERANDS = {f"v[{i}:{i + 1}]" for i in range(80, 256, 2)} | {f"v{i}" for i in range(81, 256, 2)}


def check(path, fence=80):
    text = open(path).read().splitlines()
    errors = []
    for k in KERNELS:
        start = next((i for i, l in enumerate(text) if re.match(r"^_ZN3svo\d+" + k + r"\w*:", l)), None)
        if start is None:
            errors.append(f"{k}: not found in {path}")
            continue
        in_asm, top = False, -1
        for l in text[start:]:
            s = l.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if s.startswith("s_endpgm"):
                break
            if not s or s.startswith(";") or s.startswith("."):
                continue
            code = s.split(";")[0].strip()
            if not in_asm and re.search(r"\bm0\b", code):
                errors.append(f"{k}: compiler code uses M0, which the row moves overwrite: {code}")
            parts = code.split(None, 1)
            ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
            for j, o in enumerate(ops):
                # inside the asm blocks the data registers appear only as the indexed operands of the row
                # moves / compares / selects (v80, v81, v[80:81]), as the destinations of the row loads and as
                # the fixed rows of the MAD transform;
                # every other operand is the compiler's and must stay below the fence
                if in_asm and ((code.startswith(("v_mov_b32", "v_cndmask_b32", "v_cmp_")) and o in DATA_OPERANDS) or
                               (code.startswith("buffer_load_dwordx2") and j == 0) or
                               (code.startswith(("v_add_f64", "v_and_b32")) and o in MAD_OPERANDS) or
                               (code.startswith("ds_read_b64") and j == 0 and o in MAD_OPERANDS)):
                    continue
                for m in REG.finditer(o):
                    hi = int(m.group(2) or m.group(1))
                    top = max(top, hi)
                    if hi >= fence:
                        errors.append(f"{k}: compiler-chosen register v{hi} (fence v{fence}): {code}")
        print(f"{k}: compiler-owned VGPRs up to v{top} (fence v{fence})")
    # the kernel descriptors: all 256 VGPRs allocated, no AGPRs
    entries = re.split(r"\n  - ", "\n".join(text))
    for k in KERNELS:
        seg = next((e for e in entries if re.search(r"\.name:\s+_ZN3svo\d+" + k, e)), None)
        if seg is None:
            errors.append(f"{k}: metadata not found")
            continue
        ag = re.search(r"\.agpr_count:\s+(\d+)", seg)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", seg)
        if ag is None or int(ag.group(1)) != 0:
            errors.append(f"{k}: agpr_count {ag.group(1) if ag else '?'} != 0")
        if vg is None or int(vg.group(1)) != 256:
            errors.append(f"{k}: vgpr_count {vg.group(1) if vg else '?'} != 256")
    if errors:
        print("\n".join(errors[:20]), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(check(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 80))
