"""Regression check: a process that exits with Frame <-> Feature cycles still holding device pyramids
(and its context) must exit cleanly (their finalizers may run after the context's)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import svo_amd  # noqa: E402
import svo_amd.synth as synth  # noqa: E402

ctx = svo_amd.Context(0)
p = synth.make_map_problem(n_features=400)
graphs = [synth.map_objects(p, ctx=ctx) for _ in range(3)]
m, ref, kf, cur, _, _ = graphs[0]
m.reproject_map(ref, cur, [])
m.add_candidate_to_frame(cur)
print("new features", len(cur.features))
