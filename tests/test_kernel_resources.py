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
OBJ = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "align_ref.o")

pytestmark = pytest.mark.skipif(not os.path.exists(OBJ) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readelf"),
                                reason="needs the built objects and the ROCm llvm tools")


def k2r(res, nb, tw):
    name = f"_ZN3svo22align_scale_ref_kernelILi{nb}ELi{tw}EEEvNS_9AlignArgsEi"
    assert name in res, sorted(res)
    return res[name]


def test_k2r_occupancy_budgets():
    import kernel_resources
    res = kernel_resources.resources(OBJ)
    r8 = k2r(res, 2, 8)  # the headline's instantiation (config 2: <= 65536 slots)
    assert r8["vgpr_count"] + r8["agpr_count"] <= 128, r8
    assert r8["vgpr_spill_count"] == 0, r8
    assert 2 * r8["group_segment_fixed_size"] <= 160 * 1024, r8
    r16 = k2r(res, 2, 16)  # launches of <= 128 pairs: one workgroup per CU
    assert r16["vgpr_count"] + r16["agpr_count"] <= 128, r16
    assert r16["group_segment_fixed_size"] <= 160 * 1024, r16
