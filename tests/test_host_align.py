"""The C++ drop-in ImageAlignment (host/svo.hpp, libsvo_host.so, driven by build/svo_host_check align)
against the oracle: ImageAlignment::align (src/image_alignment.cpp:25-67) through the class surface the
reference's System calls (src/system.cpp:313), in both median modes, twice on one object (the second call
reuses the object's grow-only batch and must repeat the first bit for bit)."""
import os
import subprocess

import numpy as np
import pytest

import svo_amd.synth as synth
from common import canon, oracle_align

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build", "svo_host_check")


write_align_problem = synth.write_align_problem


def test_align_problem_file_layout(tmp_path):
    """CPU: the data file holds the header and one 9-double row per feature, as svo_host_check reads it."""
    s = synth.make_pair(n_features=20)
    paths = write_align_problem(s, str(tmp_path))
    v = np.fromfile(paths[0])
    assert v.size == 6 + 21 + 2 + 9 * len(s.px)
    assert (v[27], v[28]) == (s.n_ref, s.n_kf)
    np.testing.assert_array_equal(v[29:29 + 2], s.px[0])


@pytest.mark.gpu
@pytest.mark.parametrize("median", [1, 0])
def test_gpu_cpp_mirror_image_alignment(tmp_path, median):
    s = synth.make_pair(n_features=400)
    paths = write_align_problem(s, str(tmp_path))
    out = subprocess.run([EXE, "align", *paths, "5", "0", "4", str(median)], capture_output=True, text=True,
                         timeout=120, check=True)
    lines = out.stdout.splitlines()
    assert len(lines) == 2 and lines[0] == lines[1]  # the reused batch repeats the first call exactly
    v = [float(x) for x in lines[0].split()]
    err, st, pose = v[0], int(v[1]), np.array(v[2:9])
    # oracle median_mode 0 = the reference's nth_element (GPU SVO_MEDIAN_REFERENCE = 1); 1 = exact
    pc, ec, stc, _ = oracle_align(s, 5, 0, 4, mode=0 if median == 1 else 1)
    assert st == stc
    assert np.abs(canon(pose) - canon(pc)).max() <= 1e-9
    assert abs(err - ec) <= 1e-9 * ec
