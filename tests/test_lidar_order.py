"""The lidar's child visit order.

The product's k_lidar walks each node's children in the octant order of
scene.h octantNodeImages; the oracle follows it when lidar_order="octant"
(the default, so GPU parity stays bit-exact) and follows the slot order of
mesh_bvh.inl:160-204 as written when lidar_order="slot".  Closest hits can
only differ where two distinct coplanar triangles tie (simple_map holds
overlapping coplanar faces): this pins that the difference is at most one
ulp of lidar depth and never reaches a discrete channel or another output.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import lidar_order_check  # noqa: E402


def test_octant_order_matches_slot_order_up_to_coplanar_ties():
    rays, diff, max_ulp, disc, other = lidar_order_check.main(W=24, steps=150, ts=6)
    assert rays == 24 * 12 * 80 * 150
    assert max_ulp <= 1
    assert diff <= rays * 1e-4
    assert disc == 0 and other == 0
