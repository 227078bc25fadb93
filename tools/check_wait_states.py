"""Build-time check of five gfx9 wait-state rules (R1-R5 below) around K2V's inline-asm blocks.

Scope: only the five rules listed below are modelled.  Hazards outside them -- among others the gfx940 / gfx950 rules
for a VALU write of EXEC followed by v_readlane / v_writelane, the s_set_gpr_idx_on / s_set_gpr_idx_off mode
switches, and transcendental-op forwarding -- are not checked, so a clean pass means "no R1-R5 violation", not
"hazard-free" (ADVICE r5).

hipcc inserts the wait states gfx9 needs between its own instructions, but nothing inside an inline-asm block, and
an asm block's first instructions may follow a compiler instruction that needs them (round 4's GPU fault: a
compiler v_readfirstlane wrote the buffer descriptor's SGPR two instructions before the block's buffer_load,
DESIGN.md 17.2).  This check reads the generated device assembly and fails when, on any path (fall-through or
branch into a label), a consumer comes fewer wait states after its producer than the rule needs, for every pair
in which the producer or the consumer is an inline-asm instruction:

  R1  VALU write of an SGPR          -> a VMEM instruction reading that SGPR            5 wait states
  R2  VALU write of VCC              -> a VALU reading VCC as a constant (not as the     1
                                        implicit carry-in / mask of the e32 forms)
  R3  VALU write of a VGPR           -> v_readlane / v_readfirstlane reading that VGPR   1
  R4  VALU write of an SGPR or VCC   -> v_readlane / v_writelane using it as the lane    4
                                        select
  R5  VALU write of VCC              -> v_div_fmas                                        4

A wait state is one instruction; `s_nop N` provides N + 1.  Comments, labels and directives provide none.

usage: python3 tools/check_wait_states.py <device assembly .s> [...]
"""
import re
import sys

NEED = {"R1": 5, "R2": 1, "R3": 1, "R4": 4, "R5": 4}
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b|\b(vcc_lo|vcc_hi|vcc)\b")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("buffer_", "global_", "flat_", "scratch_", "image_", "tbuffer_")
# VALU whose operand 1 is a second (carry / scale) destination when it names an SGPR pair or VCC
CARRY_DST = ("v_add_co_", "v_sub_co_", "v_subrev_co_", "v_addc_co_", "v_subb_co_", "v_subbrev_co_", "v_div_scale_",
             "v_mad_u64_u32", "v_mad_i64_i32")
# e32 forms whose last operand VCC is the implicit carry-in / mask (0 wait states)
IMPLICIT_VCC = ("v_cndmask_b32", "v_addc_co_u32", "v_subb_co_u32", "v_subbrev_co_u32")
UNCOND = ("s_branch", "s_setpc_b64", "s_endpgm", "s_trap")


def sregs(op):
    out = set()
    for m in SREG.finditer(op):
        if m.group(4):
            out |= {"vcc_lo", "vcc_hi"} if m.group(4) == "vcc" else {m.group(4)}
        elif m.group(1):
            out |= {f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)}
        else:
            out.add(f"s{m.group(3)}")
    return out


def vregs(op):
    out = set()
    for m in VREG.finditer(op):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


class Ins:
    __slots__ = ("line", "mn", "ops", "asm", "label", "nops")

    def __init__(self, line, mn, ops, asm):
        self.line, self.mn, self.ops, self.asm = line, mn, ops, asm
        self.nops = int(ops[0], 0) + 1 if mn == "s_nop" and ops else 1

    def valu(self):
        return self.mn.startswith("v_")

    def writes(self):
        """(sgprs, vgprs) written (VALU only)."""
        if not self.valu() or not self.ops:
            return set(), set()
        dst = [self.ops[0]]
        if self.mn.startswith(CARRY_DST) and len(self.ops) > 1 and sregs(self.ops[1]):
            dst.append(self.ops[1])
        if self.mn.startswith("v_cmpx"):
            dst.append("exec")
        s, v = set(), set()
        for d in dst:
            s |= sregs(d)
            v |= vregs(d)
        return s, v


def parse(path):
    funcs, cur, in_asm = [], None, False
    for n, raw in enumerate(open(path), 1):
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^([\w.$]+):", s)
        if m and not raw.startswith((" ", "\t")):
            name = m.group(1)
            if not name.startswith(".L") or cur is None:
                if not name.startswith(".L"):
                    cur = {"name": name, "ins": [], "labels": {}}
                    funcs.append(cur)
                    continue
            if cur is not None:
                cur["labels"][name] = len(cur["ins"])
            continue
        if cur is None or not s or s.startswith((";", ".")):
            continue
        code = s.split(";")[0].strip()
        if not code:
            continue
        parts = code.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        cur["ins"].append(Ins(n, parts[0], ops, in_asm))
    return funcs


def preds(f, i, branch_srcs):
    """Predecessor instruction indices of instruction i."""
    ins = f["ins"]
    out = []
    if i > 0 and not ins[i - 1].mn.startswith(UNCOND):
        out.append(i - 1)
    out += branch_srcs.get(i, [])
    return out


def consumers(c):
    """[(rule, needed sgprs, needed vgprs)] the instruction consumes under each rule."""
    out = []
    if c.mn.startswith(VMEM):
        s = set()
        for o in c.ops:
            s |= sregs(o)
        s -= {"vcc_lo", "vcc_hi"}
        if s:
            out.append(("R1", s, set()))
    if c.valu():
        srcs = c.ops[1:]
        if c.mn.startswith(CARRY_DST) and len(c.ops) > 1 and sregs(c.ops[1]):
            srcs = c.ops[2:]
        if c.mn.startswith(IMPLICIT_VCC) and "_e64" not in c.mn and srcs and srcs[-1] == "vcc":
            srcs = srcs[:-1]
        if any(sregs(o) & {"vcc_lo", "vcc_hi"} for o in srcs):
            out.append(("R2", {"vcc_lo", "vcc_hi"}, set()))
        if c.mn.startswith("v_div_fmas"):
            out.append(("R5", {"vcc_lo", "vcc_hi"}, set()))
    if c.mn in ("v_readlane_b32", "v_readfirstlane_b32") and len(c.ops) > 1:
        out.append(("R3", set(), vregs(c.ops[1])))
    if c.mn in ("v_readlane_b32", "v_writelane_b32") and len(c.ops) > 2:
        ls = sregs(c.ops[2])
        if ls:
            out.append(("R4", ls, set()))
    return out


def check_func(f):
    ins = f["ins"]
    branch_srcs = {}
    for j, x in enumerate(ins):
        if x.mn.startswith(("s_branch", "s_cbranch")) and x.ops:
            t = f["labels"].get(x.ops[-1])
            if t is not None:
                branch_srcs.setdefault(t, []).append(j)
    errors = []
    for i, c in enumerate(ins):
        for rule, sneed, vneed in consumers(c):
            need = NEED[rule]
            # walk back over every path until `need` wait states lie between the producer and c
            stack = [(p, 0) for p in preds(f, i, branch_srcs)]
            seen = set()
            while stack:
                j, ws = stack.pop()
                if (j, ws) in seen:
                    continue
                seen.add((j, ws))
                p = ins[j]
                ws_s, ws_v = p.writes()
                hit = (ws_s & sneed) or (ws_v & vneed)
                if rule in ("R2", "R5") and hit and not (ws_s & {"vcc_lo", "vcc_hi"}):
                    hit = False
                if hit:
                    if p.asm or c.asm:
                        errors.append(f"{f['name']}: {rule} needs {need} wait states, {ws} between line {p.line} "
                                      f"({p.mn} {', '.join(p.ops)}) and line {c.line} ({c.mn} {', '.join(c.ops)})")
                    continue  # (an earlier producer of the same register is shadowed on this path)
                nws = ws + p.nops
                if nws < need:
                    stack += [(q, nws) for q in preds(f, j, branch_srcs)]
    return errors


def check(paths):
    errors, n = [], 0
    for path in paths:
        for f in parse(path):
            n += sum(1 for x in f["ins"] if x.asm)
            errors += check_func(f)
    if errors:
        print("\n".join(errors[:30]), file=sys.stderr)
        print(f"check_wait_states: {len(errors)} violation(s)", file=sys.stderr)
        return 1
    print(f"check_wait_states: {n} inline-asm instructions, every R1-R5 wait state present")
    return 0


if __name__ == "__main__":
    sys.exit(check(sys.argv[1:]))
