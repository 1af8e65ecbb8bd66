"""The Box.Intersect gate's plane order (kernels.hip box_gate): on the driver's
frame the far-first order needs at most ~3 exact plane evaluations per 64-ray wave, about half
of the order it replaced (tests/gate_order_model.py; the oracle traces the rays)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def test_far_first_plane_order_is_cheaper():
    from gate_order_model import model
    m = model(240, 136)
    for name, (face, obj) in m.items():
        for old, new in (face, obj):
            assert new <= old, (name, face, obj)
            assert new <= 3.05, (name, face, obj)
    assert m["primary"][0][1] < 0.7 * m["primary"][0][0]
