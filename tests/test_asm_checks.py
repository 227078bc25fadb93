"""CPU: the build-time checks that guard K2V's inline asm.

* tools/check_wait_states.py flags each wait-state rule it enforces (R1-R5) on a seeded violation, on a straight
  path and across a branch into a label, and accepts the same code once the wait states are there;
* a seeded violation compiled by hipcc fails `make hazard-check` (the rule the K2V build runs on align_refv.s);
* the committed generated header csrc/refv_rows.h is exactly what tools/gen_refv_rows.py writes now.
"""
import filecmp
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_wait_states as W  # noqa: E402

PKG = os.path.join(ROOT, "semi-direct-visual-odometry_amd")


def _s(tmp_path, body, name="k.s"):
    p = tmp_path / name
    p.write_text("\t.text\nkern:\n" + body + "\ts_endpgm\n.Lfunc_end0:\n")
    return str(p)


def _asm(*lines):
    return "\t;;#ASMSTART\n" + "".join(f"\t{l}\n" for l in lines) + "\t;;#ASMEND\n"


CASES = {
    # rule: (producer, consumer, padding that satisfies the rule)
    "R1": ("v_readfirstlane_b32 s24, v1", "buffer_load_dwordx2 v[80:81], v40, s[24:27], 0 offen", "s_nop 4"),
    "R2": ("v_cmp_ngt_f64_e32 vcc, s[0:1], v[80:81]", "v_writelane_b32 v3, vcc_lo, 5", "s_nop 0"),
    "R3": ("v_mov_b32 v5, v6", "v_readlane_b32 s0, v5, 3", "s_nop 0"),
    "R4": ("v_readfirstlane_b32 s7, v1", "v_readlane_b32 s0, v5, s7", "s_nop 3"),
    "R5": ("v_div_scale_f64 v[0:1], vcc, v[2:3], v[2:3], v[4:5]", "v_div_fmas_f64 v[0:1], v[0:1], v[2:3], v[4:5]",
           "s_nop 3"),
}


@pytest.mark.parametrize("rule", sorted(CASES))
def test_each_rule_flags_a_seeded_violation(tmp_path, rule, capsys):
    prod, cons, pad = CASES[rule]
    # producer is compiler code, consumer inside an asm block (round 4's fault had this shape)
    bad = _s(tmp_path, f"\t{prod}\n" + _asm(cons))
    assert W.check([bad]) == 1
    assert rule in capsys.readouterr().err
    good = _s(tmp_path, f"\t{prod}\n" + _asm(pad, cons), "good.s")
    assert W.check([good]) == 0
    # both inside one block, one wait state short (s_nop N gives N + 1)
    n = W.NEED[rule]
    short = _s(tmp_path, _asm(prod, f"s_nop {n - 2}" if n >= 2 else "", cons).replace("\t\n", ""), "short.s")
    assert W.check([short]) == 1
    # compiler code on both sides is hipcc's to pad: not this check's business
    assert W.check([_s(tmp_path, f"\t{prod}\n\t{cons}\n", "cc.s")]) == 0


def test_a_violation_across_a_branch(tmp_path):
    body = ("\tv_readfirstlane_b32 s24, v1\n\ts_cbranch_scc1 .LBB0_2\n\ts_nop 7\n.LBB0_2:\n" +
            _asm("buffer_load_dwordx2 v[80:81], v40, s[24:27], 0 offen"))
    assert W.check([_s(tmp_path, body)]) == 1  # the taken branch reaches the load 1 wait state after the write
    body_ok = body.replace("\ts_cbranch_scc1 .LBB0_2\n", "\ts_nop 4\n\ts_cbranch_scc1 .LBB0_2\n")
    assert W.check([_s(tmp_path, body_ok, "ok.s")]) == 0


def test_the_built_k2v_assembly_passes():
    s = os.path.join(PKG, "build", "align_refv.s")
    if not os.path.exists(s):
        pytest.skip("not built")
    assert W.check([s]) == 0


SEEDED = r"""
#include <hip/hip_runtime.h>
// a VALU write of the descriptor's base SGPR one wait state before the buffer load that reads it (R1: five needed)
__global__ void seeded(const double* p, double* o, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    uint32_t lo, hi;
    asm volatile("s_mov_b32 s41, %3\n\ts_mov_b32 s42, %4\n\ts_mov_b32 s43, 0x20000\n\t"
                 "v_readfirstlane_b32 s40, %2\n\ts_nop 0\n\tbuffer_load_dwordx2 v[0:1], %5, s[40:43], 0 offen\n\t"
                 "s_waitcnt vmcnt(0)\n\tv_mov_b32 %0, v0\n\tv_mov_b32 %1, v1"
                 : "=v"(lo), "=v"(hi)
                 : "v"((uint32_t)a), "s"((uint32_t)(a >> 32) & 0xFFFFu), "s"(bytes), "v"(threadIdx.x * 8u)
                 : "s40", "s41", "s42", "s43", "v0", "v1", "memory");
    o[threadIdx.x] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
"""


def test_a_seeded_violation_fails_make(tmp_path):
    src = tmp_path / "seeded.hip"
    src.write_text(SEEDED)
    r = subprocess.run(["make", "-s", "-C", PKG, "hazard-check", f"SRC={src}", f"OUT={tmp_path / 'seeded.s'}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "R1" in r.stderr, r.stdout + r.stderr
    fixed = tmp_path / "fixed.hip"
    fixed.write_text(SEEDED.replace(r"s_nop 0\n\tbuffer", r"s_nop 4\n\tbuffer"))
    r = subprocess.run(["make", "-s", "-C", PKG, "hazard-check", f"SRC={fixed}", f"OUT={tmp_path / 'fixed.s'}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_generated_rows_header_is_current(tmp_path):
    out = tmp_path / "refv_rows.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_refv_rows.py"), str(out)], check=True,
                   capture_output=True, timeout=120)
    assert filecmp.cmp(str(out), os.path.join(PKG, "csrc", "refv_rows.h"), shallow=False), \
        "csrc/refv_rows.h differs from tools/gen_refv_rows.py's output: regenerate and commit it"
