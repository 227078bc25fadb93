"""CPU checks of the round-6 measurement tools (no GPU): the timeline's interval arithmetic, the kernel-trace split
by launch shape, the 4-byte key of tools/k2v_round_table.py, and bench.py's dominant-kernel figure."""
import csv
import importlib.util
import io
import os
import sys
from contextlib import redirect_stdout

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, rel))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_union_len():
    tl = _load("tl_tool", "tools/timeline.py")
    assert tl.union_len([]) == 0
    assert tl.union_len([(0, 10)]) == 10
    assert tl.union_len([(0, 10), (5, 15), (20, 25)]) == 20  # overlap merged, gap kept
    assert tl.union_len([(20, 25), (0, 10), (10, 12)]) == 17  # unsorted, touching


def test_headline_kernel_stats_split_by_shape(tmp_path):
    hk = _load("hk_tool", "tools/headline_kernel_stats.py")
    p = tmp_path / "trace.csv"
    rows = [("void svo::align_scale_refv_kernel<X>(svo::AlignArgs, int)", 65536, 100, 300),
            ("void svo::align_scale_refv_kernel<X>(svo::AlignArgs, int)", 65536, 400, 600),
            ("void svo::align_scale_refv_kernel<X>(svo::AlignArgs, int)", 131072, 0, 1000),
            ("svo::pyr_l01_kernel(unsigned char*)", 2304, 0, 50)]
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Workgroup_Size_X", "Start_Timestamp",
                    "End_Timestamp"])
        for k, g, s, e in rows:
            w.writerow([k, g, 1, 1, 512 if "refv" in k else 256, s * 1000, e * 1000])
    buf = io.StringIO()
    with redirect_stdout(buf):
        hk.main(str(p))
    out = list(csv.DictReader(io.StringIO(buf.getvalue())))
    k2v = {int(r["grid_x"]): r for r in out if r["kernel"].startswith("void align_scale_refv_kernel")}
    assert k2v[65536]["count"] == "2" and float(k2v[65536]["median_us"]) == 200.0 and k2v[65536]["pairs"] == "128"
    assert k2v[131072]["count"] == "1" and float(k2v[131072]["median_us"]) == 1000.0 and k2v[131072]["pairs"] == "256"
    assert any(r["kernel"] == "pyr_l01_kernel" and r["pairs"] == "" for r in out)


def test_key32_order_preserving():
    """The 4-byte key of the two-pairs-per-CU capacity study: a < b implies key(a) <= key(b), and
    distinct keys always order their doubles exactly."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    rt = _load("rt_tool", "tools/k2v_round_table.py")
    rng = np.random.default_rng(3)
    v = np.concatenate([rng.normal(0, 20, 5000), [0.0, -0.0, 1e-300, -1e-300, 255.0, -255.0, np.finfo(float).max]])
    v.sort()
    k = rt.key32(v)
    assert np.all(np.diff(k.astype(np.int64)) >= 0)
    a, b = rng.normal(0, 20, 2000), rng.normal(0, 20, 2000)
    ka, kb = rt.key32(a), rt.key32(b)
    d = ka != kb
    assert np.array_equal((ka < kb)[d], (a < b)[d])


def test_dominant_kernel_from_stats(tmp_path):
    b = _load("bench_tool", "bench.py")
    p = tmp_path / "stats.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "workgroup_x", "pairs", "count", "median_us", "mean_us", "p10_us",
                    "p90_us", "min_us", "max_us", "total_ms"])
        w.writerow(["void align_scale_refv_kernel<Lay<RowsA, 98, 12288u, true, 2048u> >", 65536, 1, 1, 512, 128, 10, 250.0,
                    260.0, 200.0, 300.0, 190.0, 400.0, 2.6])
    d = b.dominant_kernel(str(p), 512, 4, 1993406, 5)
    assert d["pairs_per_launch"] == 128 and d["launch_median_us"] == 250.0
    assert d["algorithmic_bytes_per_launch"] == round(128 * 1993406 / 5)
    assert abs(d["frac_chip"] - 2 * d["frac"]) <= 2e-5  # (both rounded to 5 digits)
    assert b.dominant_kernel(str(tmp_path / "missing.csv"), 512, 4, 1993406, 5) is None
