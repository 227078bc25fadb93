"""Map reprojection: Map::reprojectMap / reprojectCell / addCandidateToFrame
(src/map.cpp:260-634) as a batched FeatureAlignment caller.

CPU: the oracle restatement (oracle/svo_oracle.cpp, one alignment per candidate in the reference's order)
on hand-built maps with known answers.  Flat gradient images make FeatureAlignment leave the pixel where
it starts, so the expected new features are the projections themselves.
GPU: svo_amd.Map (svo_map_reproject_plan + one svo_feature_align_multi launch per call) against the
oracle on synthetic maps: the same new features in the same order (aligned pixels bit-exact), the same
point states, counters and visited cells.
"""
import math

import numpy as np
import pytest

import oracle as O
import svo_amd.synth as synth

CAM = dict(fx=300.0, fy=300.0, cx=160.0, cy=48.0, width=320, height=96)
GOOD, DELETED, CANDIDATE, UNKNOWN = 0, 1, 2, 3
IDENT = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
NO_FRAME = np.uint64(2 ** 64 - 1)


def point_at(u, v, z=10.0, cam=CAM):
    return np.array([(u - cam["cx"]) / cam["fx"] * z, (v - cam["cy"]) / cam["fy"] * z, z])


def grid(cam, cell=30):
    return math.ceil(cam["width"] / cell), math.ceil(cam["height"] / cell)


def run_oracle(cam, feats_per_kf, feat_point, pos, ptype, psucc, cell_order=None, cur_id=7):
    flat = np.zeros((cam["height"], cam["width"]), np.uint8)
    cols, rows = grid(cam)
    order = np.arange(cols * rows, dtype=np.int32) if cell_order is None else cell_order
    off = np.cumsum([0] + feats_per_kf).astype(np.int32)
    n = off[-1]
    ptype = np.array(ptype, np.uint32)
    psucc = np.array(psucc, np.uint32)
    plast = np.full(len(pos), NO_FRAME, np.uint64)
    visited = np.zeros(cols * rows, np.uint8)
    out = O.reproject_map(cam, 30, order, IDENT, cur_id, flat, [flat] * len(feats_per_kf), off,
                          np.full((n, 2), 100.0), np.array(feat_point, np.int32), np.array(pos), ptype, psucc, plast,
                          visited)
    return out, ptype, psucc, plast, visited


def cell_of(px, cam=CAM, cell=30):
    cols, _ = grid(cam)
    return int(px[1]) // cell * cols + int(px[0]) // cell


def test_reproject_cell_order_types_and_bookkeeping():
    # cell A (u 65, v 40): GOOD, DELETED, UNKNOWN -> sorted by type descending, UNKNOWN is taken
    # cell B (u 200, v 70): only DELETED -> a trial, no match
    # cell C (u 250, v 10): UNKNOWN with 10 successes -> accepted, promoted to GOOD
    # P5 projects to u = 2 < 3: outside the frame; the last keyframe's feature re-observes P0
    pos = [point_at(65.5, 40.5), point_at(66.5, 41.5), point_at(67.5, 42.5), point_at(200.5, 70.5),
           point_at(250.25, 10.75), point_at(2.0, 50.0)]
    ptype = [GOOD, DELETED, UNKNOWN, DELETED, UNKNOWN, UNKNOWN]
    psucc = [0, 0, 3, 0, 10, 0]
    feat_point = [0, 1, 2, 3, 4, 5, 0, -1]  # ref: 6 features; last keyframe: P0 again, one without a point
    (overlap, new_px, new_point, new_feat, m, t), ptype, psucc, plast, visited = run_oracle(
        CAM, [6, 2], feat_point, pos, ptype, psucc)
    assert list(overlap) == [5, 0]                     # P5 outside; P0 already projected for this frame
    assert list(plast) == [7] * 6                      # every point with a feature was projected once
    cA, cB, cC = cell_of((65.5, 40.5)), cell_of((200.5, 70.5)), cell_of((250.25, 10.75))
    assert cC < cA < cB                                # identity cell order: C (row 0), A, then B
    assert list(new_point) == [4, 2] and list(new_feat) == [4, 2]
    assert np.allclose(new_px, [[250.25, 10.75], [67.5, 42.5]], rtol=0, atol=1e-9)  # projection round trip
    assert (m, t) == (2, 2 + 1)                        # A: one trial, C: one, B: one (deleted)
    assert list(psucc) == [0, 0, 4, 0, 11, 0] and list(ptype) == [GOOD, DELETED, UNKNOWN, DELETED, GOOD, UNKNOWN]
    assert set(np.nonzero(visited)[0]) == {cA, cC}


def test_reproject_stops_after_151_matches():
    cam = dict(fx=721.5377, fy=721.5377, cx=609.5593, cy=172.854, width=1241, height=376)
    cols, rows = grid(cam)
    cells = [(c, r) for r in range(rows) for c in range(cols - 1)][:200]  # the last column lies partly outside
    pos = [point_at(30 * c + 15.5, 30 * r + 15.5, cam=cam) for c, r in cells]
    (overlap, new_px, new_point, _, m, t), *_ = run_oracle(cam, [len(pos)], list(range(len(pos))), pos,
                                                          [UNKNOWN] * len(pos), [0] * len(pos))
    assert overlap[0] == 200 and (m, t) == (151, 151) and len(new_point) == 151
    assert list(new_point) == list(range(151))        # identity order: cell k holds point k


def test_add_candidates_first_match_per_cell_wins():
    flat = np.zeros((CAM["height"], CAM["width"]), np.uint8)
    cols, rows = grid(CAM)
    visited = np.zeros(cols * rows, np.uint8)
    visited[cell_of((200.5, 70.5))] = 1
    cand_pos = np.array([point_at(65.5, 40.5), point_at(66.5, 41.5), point_at(200.5, 70.5), point_at(1.0, 40.0),
                         point_at(120.5, 20.5)])
    matched, new_px = O.add_candidates(CAM, 30, visited, IDENT, flat, [flat] * 5, np.full((5, 2), 100.0), cand_pos)
    assert list(matched) == [True, False, False, False, True]  # same cell / visited cell / outside
    assert np.allclose(new_px[[0, 4]], [[65.5, 40.5], [120.5, 20.5]], rtol=0, atol=1e-9)
    assert visited[cell_of((65.5, 40.5))] and visited[cell_of((120.5, 20.5))]


# ---------------------------------------------------------------- GPU parity
def oracle_side(p, cell_order, cur_id):
    g = {k: O.unpack_levels(O.build_pyramid(img, 1)[1], p.camera["width"], p.camera["height"], 1)[0]
         for k, img in (("ref", p.ref_img), ("kf", p.kf_img), ("cur", p.cur_img))}
    ptype, psucc = p.point_type.copy(), p.point_succ.copy()
    plast = np.full(len(p.point_pos), NO_FRAME, np.uint64)
    visited = np.zeros(len(cell_order), np.uint8)
    off = np.array([0, p.n_ref, p.n_ref + p.n_kf], np.int32)
    rep = O.reproject_map(p.camera, p.cell_size, cell_order, p.cur_pose, cur_id, g["cur"], [g["ref"], g["kf"]], off,
                          p.feat_px, p.feat_point, p.point_pos, ptype, psucc, plast, visited)
    visited_after_reproject = visited.copy()
    cand = O.add_candidates(p.camera, p.cell_size, visited, p.cur_pose, g["cur"], [g["kf"]] * len(p.cand_feat),
                            p.feat_px[p.cand_feat], p.cand_pos)
    return rep, ptype, psucc, plast, visited_after_reproject, cand, visited


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [synth.SEED_BASE, synth.SEED_BASE + 5])
def test_gpu_map_matches_oracle(seed):
    p = synth.make_map_problem(seed=seed)
    m, ref, kf, cur, points, feats = synth.map_objects(p, seed=seed)
    (overlap, new_px, new_point, new_feat, matches, trials), ptype, psucc, plast, vis1, (cmatch, cpx), vis2 = \
        oracle_side(p, m.cell_orders, cur.id)
    overlap_kf = []
    m.reproject_map(ref, cur, overlap_kf)
    assert [c for _, c in overlap_kf] == list(overlap) and overlap_kf[0][0] is ref and overlap_kf[1][0] is kf
    assert (m.matches, m.trials) == (matches, trials) and matches > 100
    assert len(cur.features) == len(new_px)
    got_px = np.array([f.pixel_position for f in cur.features])
    assert np.array_equal(got_px, new_px)                              # FeatureAlignment bit-exact
    assert [points.index(f.point) for f in cur.features] == list(new_point)
    assert [p.type for p in points] == list(ptype) and [p.succeeded_projection for p in points] == list(psucc)
    assert [p.last_projected_kf_id for p in points] == [int(x) for x in plast]
    assert np.array_equal(m.cell_visited, vis1.astype(bool))
    n_before = len(cur.features)
    cands = [c[0] for c in m.candidates]
    m.add_candidate_to_frame(cur)
    added = cur.features[n_before:]
    assert len(added) == int(cmatch.sum()) and len(added) > 0
    assert np.array_equal(np.array([f.pixel_position for f in added]), cpx[cmatch])
    assert np.array_equal(m.cell_visited, vis2.astype(bool))
    assert len(m.candidates) == len(cands) - len(added)                 # removeMatchedCandidate
    for f in added:
        assert f.point.features[-1] is f and f.point.features[-2].point is f.point


@pytest.mark.gpu
def test_gpu_map_needs_last_keyframe():
    p = synth.make_map_problem(n_features=200)
    m, ref, kf, cur, _, _ = synth.map_objects(p)
    ref.last_keyframe = None
    with pytest.raises(ValueError):
        m.reproject_map(ref, cur, [])


@pytest.mark.gpu
def test_gpu_cpp_mirror_map(tmp_path):
    """host/svo.hpp Map (libsvo_host.so via build/svo_host_check map): reprojectMap + addCandidateToFrame on a
    config-2 map against the sequential oracle: the same new features, bit-exact, in the same order."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    mp = synth.make_map_problem()
    c = mp.camera
    W, H = c["width"], c["height"]
    ncells = math.ceil(W / mp.cell_size) * math.ceil(H / mp.cell_size)
    order = np.random.default_rng(5).permutation(ncells).astype(np.int32)
    paths = synth.write_map_problem(mp, str(tmp_path), order)
    out = subprocess.run([exe, "map", *paths], capture_output=True, text=True, timeout=60, check=True)
    lines = out.stdout.splitlines()
    got = np.array([[float(v) for v in l.split()[1:]] for l in lines[1:]]).reshape(-1, 2)
    grad = {k: O.unpack_levels(O.build_pyramid(img, 1)[1], W, H, 1)[0]
            for k, img in (("ref", mp.ref_img), ("kf", mp.kf_img), ("cur", mp.cur_img))}
    ptype, psucc = mp.point_type.copy(), mp.point_succ.copy()
    plast = np.full(len(mp.point_pos), np.uint64(2 ** 64 - 1), np.uint64)
    visited = np.zeros(ncells, np.uint8)
    rep = O.reproject_map(mp.camera, mp.cell_size, order, mp.cur_pose, 7, grad["cur"], [grad["ref"], grad["kf"]],
                          np.array([0, mp.n_ref, mp.n_ref + mp.n_kf], np.int32), mp.feat_px, mp.feat_point,
                          mp.point_pos, ptype, psucc, plast, visited)
    cm, cpx = O.add_candidates(mp.camera, mp.cell_size, visited, mp.cur_pose, grad["cur"], [grad["kf"]] * len(mp.cand_feat),
                               mp.feat_px[mp.cand_feat], mp.cand_pos)
    expect = np.concatenate([rep[1], cpx[cm]])
    assert lines[0] == f"counts {rep[4]} {rep[5]}"
    np.testing.assert_array_equal(got, expect)


@pytest.mark.gpu
def test_gpu_cpp_mirror_add_candidates_twice(tmp_path):
    """host/svo.hpp Map::addCandidateToFrame removes its matched candidates (src/map.cpp:626, 629-634): a
    second call, on a frame 5 cm further along x, aligns only the candidates the first call left, against
    the sequential oracle (same cells visited, same remaining list, same new features bit for bit)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "semi-direct-visual-odometry_amd", "build", "svo_host_check")
    mp = synth.make_map_problem()
    c = mp.camera
    W, H = c["width"], c["height"]
    ncells = math.ceil(W / mp.cell_size) * math.ceil(H / mp.cell_size)
    order = np.random.default_rng(5).permutation(ncells).astype(np.int32)
    paths = synth.write_map_problem(mp, str(tmp_path), order)
    out = subprocess.run([exe, "map", *paths, "0", "twice"], capture_output=True, text=True, timeout=60, check=True)
    lines = out.stdout.splitlines()
    grad = {k: O.unpack_levels(O.build_pyramid(img, 1)[1], W, H, 1)[0]
            for k, img in (("ref", mp.ref_img), ("kf", mp.kf_img), ("cur", mp.cur_img))}
    ptype, psucc = mp.point_type.copy(), mp.point_succ.copy()
    plast = np.full(len(mp.point_pos), np.uint64(2 ** 64 - 1), np.uint64)
    visited = np.zeros(ncells, np.uint8)
    O.reproject_map(mp.camera, mp.cell_size, order, mp.cur_pose, 7, grad["cur"], [grad["ref"], grad["kf"]],
                    np.array([0, mp.n_ref, mp.n_ref + mp.n_kf], np.int32), mp.feat_px, mp.feat_point,
                    mp.point_pos, ptype, psucc, plast, visited)
    nc = len(mp.cand_feat)
    cm, _ = O.add_candidates(mp.camera, mp.cell_size, visited, mp.cur_pose, grad["cur"], [grad["kf"]] * nc,
                             mp.feat_px[mp.cand_feat], mp.cand_pos)
    keep = ~cm
    assert cm.any() and keep.any()
    pose2 = np.array(mp.cur_pose, np.float64).copy()
    pose2[4] += 0.05
    cm2, cpx2 = O.add_candidates(mp.camera, mp.cell_size, visited, pose2, grad["cur"], [grad["kf"]] * int(keep.sum()),
                                 mp.feat_px[mp.cand_feat][keep], mp.cand_pos[keep])
    counts = [ln for ln in lines if ln.startswith("candidates ")]
    assert counts == [f"candidates {int(keep.sum())}", f"candidates {int(keep.sum() - cm2.sum())}"], counts
    got2 = np.array([[float(v) for v in ln.split()[1:]] for ln in lines if ln.startswith("px2 ")]).reshape(-1, 2)
    np.testing.assert_array_equal(got2, cpx2[cm2])
