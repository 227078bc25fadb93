"""The INTEGRATION.md adapter compiled and run.

tests/cpp/adapter.cpp holds the adapter bodies a maintainer puts behind the reference's ImageAlignment /
ImagePyramid / FeatureAlignment (src/image_alignment.cpp:25-67, src/image_pyramid.cpp:36-52,
src/feature_alignment.cpp:25-62); tests/cpp/ref_types.hpp gives it the shapes of the reference's Frame / Feature /
Point / camera types.  CPU: the blocks appear verbatim in INTEGRATION.md, the file compiles and links against
libsvo_hip.so, and a call that cannot get a context leaves the pose and the pixel position bit-unchanged and returns
NaN (the reference never throws), and the ImagePyramid getters (include/image_pyramid.hpp:75-140) give
no levels, (0, 0) sizes and empty Mats.  GPU: the compiled adapter aligns a config-2 pair to the oracle's
pose (reference median semantics, 1e-9), FeatureAlignment(7) matches the oracle bit for bit, and every pyramid level
of both stacks read through the getters equals the oracle's bytes."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as O
import svo_amd.synth as synth
from common import canon, oracle_align

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
BUILD = os.path.join(ROOT, "semi-direct-visual-odometry_amd", "build")


def _blocks():
    src = open(os.path.join(CPP, "adapter.cpp")).read()
    return re.findall(r"// >>> (.+?)\n(.*?)// <<< \1\n", src, re.S)


def test_adapter_blocks_are_the_integration_doc():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    names = [n for n, _ in _blocks()]
    assert names == ["context", "ImageAlignment::align", "ImagePyramid", "ImagePyramid getters",
                     "FeatureAlignment::align"]
    for name, body in _blocks():
        assert body in doc, f"INTEGRATION.md lacks the compiled block {name!r} (tests/cpp/adapter.cpp)"


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("adapter") / "adapter_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), "-I" + CPP,
                    "-o", out, os.path.join(CPP, "adapter.cpp"), os.path.join(CPP, "adapter_check.cpp"),
                    "-L" + BUILD, "-lsvo_hip", "-Wl,-rpath," + BUILD], check=True, timeout=120)
    return out


def _input(path, s, levels=5, patch=5, n_fa=64, seed=3):
    cam = s.camera
    rng = np.random.default_rng(seed)
    fa_ref = s.px[:n_fa].copy()
    fa_init = fa_ref + rng.uniform(-1.5, 1.5, fa_ref.shape)
    with open(path, "wb") as f:
        f.write(np.array([cam["width"], cam["height"], levels, patch, 0, levels - 1], np.int32).tobytes())
        f.write(np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float64).tobytes())
        for im in (s.ref_img, s.kf_img, s.cur_img):
            f.write(np.ascontiguousarray(im, np.uint8).tobytes())
        f.write(np.concatenate([s.ref_pose, s.kf_pose, s.cur_init_pose]).astype(np.float64).tobytes())
        f.write(np.array([s.n_ref, s.n_kf], np.int32).tobytes())
        for a in (s.px, s.bearing, s.point):
            f.write(np.ascontiguousarray(a, np.float64).tobytes())
        f.write(np.ascontiguousarray(s.has_point, np.uint8).tobytes())
        f.write(np.array([n_fa], np.int32).tobytes())
        f.write(fa_ref.astype(np.float64).tobytes())
        f.write(fa_init.astype(np.float64).tobytes())
    return fa_ref, fa_init


def _run(exe, path, mode):
    r = subprocess.run([exe, path, mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = {"fa": [], "lvl": []}
    for line in r.stdout.splitlines():
        k, *v = line.split()
        if k == "fa":
            out["fa"].append([float(x) for x in v[1:]])
        elif k == "lvl":
            out["lvl"].append([int(x) for x in v])
        elif k in ("pyr", "all"):
            out[k] = [int(x) for x in v]
        else:
            out[k] = [float(x) for x in v]
    out["fa"] = np.array(out["fa"]).reshape(-1, 3)
    return out


def _fnv1a(a):
    x = 1469598103934665603
    for b in np.ascontiguousarray(a, np.uint8).tobytes():
        x = ((x ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return x


def _check_untouched(o, s, fa_init, levels=5):
    # the pyramid getters without a set: no levels, (0, 0) sizes, empty Mats at every level, no crash
    assert o["pyr"] == [0, 0, 0] and o["all"] == [0, 1]
    empty = _fnv1a(np.zeros(0, np.uint8))
    assert o["lvl"] == [[l, 0, 0, 0, 0, empty, empty] for l in range(levels + 1)]
    assert np.isnan(o["err"][0])
    assert o["unchanged"] == [1.0] and np.array_equal(np.array(o["pose"]), s.cur_init_pose)
    assert o["again"] == [1.0]
    assert np.array_equal(o["fa"][:, :2], fa_init) and np.all(np.isnan(o["fa"][:, 2]))


def test_adapter_failure_leaves_the_pose_untouched(exe, tmp_path):
    """No context (a device index that does not exist): NaN, pose and pixel positions bit-unchanged."""
    s = synth.make_pair(n_features=300)
    path = str(tmp_path / "in.bin")
    _, fa_init = _input(path, s)
    _check_untouched(_run(exe, path, "fail"), s, fa_init)


def test_adapter_without_a_gpu(exe, tmp_path):
    import ctypes
    from svo_amd import _capi
    n = ctypes.c_int32(-1)
    assert _capi.lib().svo_device_count(ctypes.byref(n)) == 0
    if n.value > 0:
        pytest.skip("a GPU is visible (test_gpu_adapter_matches_oracle runs instead)")
    s = synth.make_pair(n_features=300)
    path = str(tmp_path / "in.bin")
    _, fa_init = _input(path, s)
    _check_untouched(_run(exe, path, "run"), s, fa_init)


@pytest.mark.gpu
def test_gpu_adapter_matches_oracle(exe, tmp_path):
    s = synth.make_pair(n_features=2000)
    path = str(tmp_path / "in.bin")
    fa_ref, fa_init = _input(path, s)
    o = _run(exe, path, "run")
    pc, ec, stc, _ = oracle_align(s, 5, 0, 4, mode=0)
    assert o["unchanged"] == [0.0] and o["again"] == [1.0]
    assert np.abs(canon(np.array(o["pose"])) - canon(pc)).max() <= 1e-9
    assert abs(o["err"][0] - ec) <= 1e-9 * ec
    # the ImagePyramid getters: level count, sizes, and every level of both stacks byte-equal to the oracle's
    # pyramid (hashed); one level past the last gives (0, 0) and an empty Mat
    h, w = s.ref_img.shape
    oi, og = O.build_pyramid(s.ref_img, 5)
    li, lg = O.unpack_levels(oi, w, h, 5), O.unpack_levels(og, w, h, 5)
    assert o["pyr"] == [5, w, h] and o["all"] == [5, 1]
    for l in range(5):
        lh, lw = li[l].shape
        assert o["lvl"][l] == [l, lw, lh, lh, lw, _fnv1a(li[l]), _fnv1a(lg[l])], l
    empty = _fnv1a(np.zeros(0, np.uint8))
    assert o["lvl"][5] == [5, 0, 0, 0, 0, empty, empty]
    g_ref, g_cur = O.build_pyramid(s.ref_img, 1)[1], O.build_pyramid(s.cur_img, 1)[1]
    px_c, err_c, _ = O.feature_align(s.camera, 7, g_ref, g_cur, fa_ref, fa_init)
    assert np.array_equal(o["fa"][:, :2], px_c)
    ok = ~np.isnan(err_c)
    assert np.array_equal(np.isnan(o["fa"][:, 2]), ~ok) and np.array_equal(o["fa"][ok, 2], err_c[ok])
