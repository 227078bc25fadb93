"""CPU: the occupancy budgets the reference-mode throughput depends on, read from the
built gfx950 code object (tools/kernel_resources.py).  K2R's 8-wave instantiation must keep two workgroups
per CU: at most 128 VGPRs per lane (2 workgroups x 8 waves = 4 waves per SIMD) and at most 80 KB of LDS;
a change that crossed 128 VGPRs cut the headline from 89.2k to 67.7k pairs/s.  The 16-wave
instantiation runs one workgroup per CU: 128 VGPRs (4 waves per SIMD) and at most 160 KB."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
PKG = os.path.join(ROOT, "semi-direct-visual-odometry_amd")
OBJ = os.path.join(PKG, "build", "align_ref.o")
OBJ_V = os.path.join(PKG, "build", "align_refv.o")
LIB = os.path.join(PKG, "build", "libsvo_hip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# skipped only when the library is not built; a built library whose objects or metadata cannot be read fails
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libsvo_hip.so not built")


def load(obj):
    assert os.path.exists(READELF), READELF
    assert os.path.exists(obj), f"{obj} missing although {LIB} is built"
    import kernel_resources
    res = kernel_resources.resources(obj)
    assert res, f"no kernel metadata read from {obj}"
    return res


def k2r(res, nb, tw):
    name = f"_ZN3svo22align_scale_ref_kernelILi{nb}ELi{tw}EEEvNS_9AlignArgsEi"
    assert name in res, sorted(res)
    return res[name]


def test_k2r_occupancy_budgets():
    res = load(OBJ)
    r8 = k2r(res, 2, 8)  # the headline's instantiation (config 2: <= 65536 slots)
    assert r8["vgpr_count"] + r8["agpr_count"] <= 128, r8
    assert r8["vgpr_spill_count"] == 0, r8
    assert 2 * r8["group_segment_fixed_size"] <= 160 * 1024, r8
    r16 = k2r(res, 2, 16)  # launches of <= 128 pairs: one workgroup per CU
    assert r16["vgpr_count"] + r16["agpr_count"] <= 128, r16
    assert r16["group_segment_fixed_size"] <= 160 * 1024, r16


def test_k2v_register_residency():
    """K2V (align_refv.hip) keeps rows 0..87 of the vector in v80..v255: every VGPR allocated, no AGPRs,
    no spills, one 512-thread workgroup per CU within 160 KB of LDS (tools/check_vreg_fence.py checks the
    fence itself at build time)."""
    res = load(OBJ_V)
    names = [n for n in res if "align_scale_refv_kernel" in n]
    assert names, sorted(res)
    for n in names:
        r = res[n]
        assert r["vgpr_count"] == 256 and r["agpr_count"] == 0, r
        assert r["vgpr_spill_count"] == 0, r
        assert r["group_segment_fixed_size"] <= 160 * 1024, r
