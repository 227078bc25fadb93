"""Trajectory and feature-dump text formats of the reference.

  write_in_file             System::writeInFile (src/system.cpp:635-640): one KITTI line per processed
                            image, the ref frame's camera->world pose m_absPose.inverse().matrix3x4(),
                            12 numbers at stream precision 6 (utils::eigenFormatIO, src/utils.cpp:10-13);
  write_failed              main's "Failed" line for an image addImage rejected (src/main.cpp:118-121);
  read_trajectory           the inverse of the two above (not in the reference; for replaying and comparing
                            trajectories): one (3, 4) matrix per line, None for "Failed";
  write_all_info_file       utils::writeAllInfoFile (src/utils.cpp:62-71): "rx ry cx cy X Y Z" per feature;
  write_features_info_file  utils::writeFeaturesInfoFile (:73-81): "rx ry cx cy";
  read_all_from_file /      utils::readAllFromFile / readFeaturesFromFile (:83-117), including their quirk:
  read_features_from_file   both clear the frames' features first and then loop to numberObservation(),
                            which is now 0, so they read nothing;
  read_all_info             parses a writeAllInfoFile dump into arrays (the reading the reference meant).

Numbers are printed as `std::ostream << std::setprecision(6)` prints a double, i.e. printf "%.6g"; the pose
line comes from the C ABI (svo_format_kitti_pose) so the C++ host mirror and Python write the same bytes.
"""
import ctypes

import numpy as np

from ._capi import check, lib, ptr


def _g6(v):
    return "%.6g" % float(v)


def pose_matrix3x4_inverse(pose):
    """m_absPose.inverse().matrix3x4() for a world->camera pose in Sophus params order."""
    p = np.ascontiguousarray(pose, np.float64)
    out = np.zeros(12)
    check(lib().svo_pose_matrix3x4_inverse(ptr(p), ptr(out)))
    return out.reshape(3, 4)


def kitti_line(pose):
    p = np.ascontiguousarray(pose, np.float64)
    buf = ctypes.create_string_buffer(256)
    check(lib().svo_format_kitti_pose(ptr(p), buf, 256))
    return buf.value.decode()


def write_in_file(ref_frame, f):
    f.write(kitti_line(ref_frame.abs_pose) + "\n")


def write_failed(f):
    f.write("Failed\n")


def read_trajectory(f):
    out = []
    for line in f:
        line = line.strip()
        if not line:
            continue
        if line == "Failed":
            out.append(None)
            continue
        v = np.array([float(x) for x in line.split()], np.float64)
        if v.size != 12:
            raise ValueError(f"trajectory line with {v.size} numbers: {line!r}")
        out.append(v.reshape(3, 4))
    return out


def write_all_info_file(ref_frame, cur_frame, f):
    for i in range(len(ref_frame.features)):
        r = ref_frame.features[i].pixel_position
        c = cur_frame.features[i].pixel_position
        p = ref_frame.features[i].point.position
        f.write(" ".join(_g6(v) for v in (r[0], r[1], c[0], c[1], p[0], p[1], p[2])) + "\n")


def write_features_info_file(ref_frame, cur_frame, f):
    for i in range(len(ref_frame.features)):
        r = ref_frame.features[i].pixel_position
        c = cur_frame.features[i].pixel_position
        f.write(" ".join(_g6(v) for v in (r[0], r[1], c[0], c[1])) + "\n")


def read_all_from_file(ref_frame, cur_frame, f):
    ref_frame.features.clear()
    cur_frame.features.clear()
    for _ in range(len(ref_frame.features)):  # 0 iterations, as in the reference (:87-89)
        raise AssertionError("unreachable")


def read_features_from_file(ref_frame, cur_frame, f):
    ref_frame.features.clear()
    cur_frame.features.clear()
    for _ in range(len(ref_frame.features)):  # 0 iterations (:104-106)
        raise AssertionError("unreachable")


def read_all_info(f):
    """(ref_px (n, 2), cur_px (n, 2), points (n, 3)) from a writeAllInfoFile dump."""
    rows = [[float(x) for x in line.split()] for line in f if line.strip()]
    a = np.array(rows, np.float64).reshape(-1, 7)
    return a[:, 0:2].copy(), a[:, 2:4].copy(), a[:, 4:7].copy()
