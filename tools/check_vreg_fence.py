"""Build-time check of K2V's register fences (semi-direct-visual-odometry_amd/csrc/align_refv.hip).

K2V keeps the register rows of each pair's residual vector in the VGPRs above its layout's fence (v80..v255 for
LayA, v72..v255 for LayB, v64..v255 for LayC), written and read only by its inline-asm blocks.  The compiler is not told about them
outside those blocks, so this check reads the generated assembly of every K2V kernel instantiation, from its
entry label to its .Lfunc_end label, takes the fence from the kernel's `;@vfence B` marker, and fails when

  * an instruction outside an ;;#ASMSTART / ;;#ASMEND block names a VGPR >= the fence, or M0 (which the
    indexed row moves set);
  * an operand of an asm-block instruction is >= the fence and is not one of the fixed data operands that
    instruction's `;@vfix i[,j..]` tag lists (operand positions after the mnemonic, 0-based): every data-register
    operand in the asm templates carries such a tag (the templates in align_refv.hip and the generated
    refv_rows.h), so a compiler-chosen operand (a %N the compiler filled in) that strays above the fence is
    caught even inside the blocks;
  * a tagged operand is below the fence (a stale tag);
  * the kernel's VGPR count is not 256 (the data registers must be allocated) or it allocates AGPRs;
  * a kernel has no `;@vfence` marker.

usage: python3 tools/check_vreg_fence.py <device assembly .s>
"""
import re
import sys

KERNELS = ("align_scale_refv_kernel", "debug_robust_scale_v_kernel", "plain_robust_scale_v_kernel")
REG = re.compile(r"\bv\[?(\d+)(?::(\d+))?\]?")
TAG = re.compile(r";@vfix\s+([\d,]+)")


def operands(code):
    parts = code.split(None, 1)
    return [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []


def top_reg(o):
    hi = -1
    for m in REG.finditer(o):
        hi = max(hi, int(m.group(2) or m.group(1)))
    return hi


def check(path):
    text = open(path).read().splitlines()
    errors = []
    found = {k: 0 for k in KERNELS}
    starts = []
    for i, l in enumerate(text):
        m = re.match(r"^(_ZN3svo\d+(" + "|".join(KERNELS) + r")\w*):", l)
        if m:
            starts.append((i, m.group(1), m.group(2)))
            found[m.group(2)] += 1
    for k, c in found.items():
        if c == 0:
            errors.append(f"{k}: not found in {path}")
    names = []
    for start, name, k in starts:
        names.append(name)
        fm = None
        end = next((i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end") and name in text[i]),
                   None)
        if end is None:  # (the label is "<.Lfunc_endN>:"; the symbol size directive after it names the kernel)
            end = next((i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end")), len(text))
        for l in text[start + 1:end]:
            mm = re.search(r";@vfence\s+(\d+)", l)
            if mm:
                fm = int(mm.group(1))
                break
        if fm is None:
            errors.append(f"{name}: no ;@vfence marker")
            continue
        fence = fm
        in_asm, top, tagged = False, -1, 0
        for l in text[start + 1:end]:
            s = l.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not s or s.startswith(";") or s.startswith("."):
                continue
            code = s.split(";")[0].strip()
            if not code:
                continue
            if not in_asm and re.search(r"\bm0\b", code):
                errors.append(f"{name}: compiler code uses M0, which the row moves overwrite: {code}")
            tag = TAG.search(s) if in_asm else None
            fixed = {int(x) for x in tag.group(1).split(",") if x} if tag else set()
            tagged += 1 if tag else 0
            for j, o in enumerate(operands(code)):
                hi = top_reg(o)
                if j in fixed:
                    if hi < fence:
                        errors.append(f"{name}: tagged data operand {j} below the fence: {code}")
                    continue
                top = max(top, hi)
                if hi >= fence:
                    errors.append(f"{name}: compiler-chosen register v{hi} (fence v{fence}): {code}")
        print(f"{name}: compiler-owned VGPRs up to v{top} (fence v{fence}), {tagged} tagged data-register instructions")
    # the kernel descriptors: all 256 VGPRs allocated, no AGPRs
    entries = re.split(r"\n  - ", "\n".join(text))
    for k in names:
        seg = next((e for e in entries if re.search(r"\.name:\s+" + re.escape(k) + r"\s", e)), None)
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
    sys.exit(check(sys.argv[1]))
