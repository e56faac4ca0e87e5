"""The reference's own known-answer tests, ported verbatim against the oracle.

Every test here cites the `test` block of /root/reference/src/linalg.zig it
restates.  These are the ONLY reference-owned golden vectors for the hot path
(SURVEY.md §4, §8c c3); they pin the oracle's vector, slab and DDA code.
"""
import math

import numpy as np
import pytest


def norm(v):
    v = np.asarray(v, np.float32)
    inv = np.float32(1.0) / np.sqrt(np.float32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return v * inv


def test_rgb_size_is_3():
    # linalg.zig:9-11 -- our RGB8 output is packed 3 bytes per pixel
    assert np.dtype([("r", "u1"), ("g", "u1"), ("b", "u1")]).itemsize == 3


def test_cross_product(oracle_mod):
    # linalg.zig:231-236
    r = oracle_mod.cross([1, -8, 12], [4, 6, 3])
    assert list(r) == [-96, 45, 38]


def test_vector_length(oracle_mod):
    # linalg.zig:238-241
    assert abs(oracle_mod.length([1.5, 100.0, -21.1]) - 102.21281720019266) <= 1e-4


@pytest.mark.parametrize("bmin,bmax,orig,d,hit,t", [
    # linalg.zig:352-364
    ((-1, -1, -1), (1, 1, 1), (0, 0, 5), (0, 0, -1), True, 4.0),
    # linalg.zig:366-378
    ((1, 1, 1), (2, 2, 2), (0, 0, 0), "n111", True, math.sqrt(3)),
    # linalg.zig:380-392 (origin inside bbox -> t < 0)
    ((-1, -1, -1), (3, 3, 3), (0, 0, 0), "n110", True, -math.sqrt(2)),
    # linalg.zig:394-405 (miss)
    ((-1, -1, -1), (3, 3, 3), (5, 5, 5), "n110", False, None),
])
def test_bbox_ray_intersection(oracle_mod, bmin, bmax, orig, d, hit, t):
    if d == "n111":
        d = norm([1, 1, 1])
    elif d == "n110":
        d = norm([1, 1, 0])
    h, tt = oracle_mod.bbox_ray(bmin, bmax, orig, d)
    assert h == hit
    if hit:
        assert abs(tt - t) <= 1e-4


def test_decrement_via_add():
    # linalg.zig:565-569: the DDA steps -1 as a wrapping +0xFFFFFFFF
    assert (5 + 0xFFFFFFFF) & 0xFFFFFFFF == 4


def test_grid_get_cell_bbox(oracle_mod):
    # linalg.zig:571-581
    mn, mx = oracle_mod.grid_cell_bbox((0, 0, 0), (5, 5, 5), (5, 5, 5), 0, 1, 4)
    assert list(mn) == [0, 1, 4]
    assert list(mx) == [1, 2, 5]


GRID_CASES = {
    # linalg.zig:583-607
    "traceRay 1": ((0.5, 0.5, 0.5), "n210", (0, 0, 0), [
        ((1, 0, 0), 0.559017002), ((1, 1, 0), 1.11803400), ((2, 1, 0), 1.67705106),
        ((3, 1, 0), 2.79508495), ((3, 2, 0), 3.35410213), ((4, 2, 0), 3.91311883)]),
    # linalg.zig:609-629
    "traceRay 2": ((0.5, 10.0, 0.5), (0, -1, 0), (0, 4, 0), [
        ((0, 3, 0), 6), ((0, 2, 0), 7), ((0, 1, 0), 8), ((0, 0, 0), 9)]),
    # linalg.zig:631-651
    "traceRay 3": ((0.5, -5.0, 0.5), (0, 1, 0), (0, 0, 0), [
        ((0, 1, 0), 6), ((0, 2, 0), 7), ((0, 3, 0), 8), ((0, 4, 0), 9)]),
    # linalg.zig:653-681 (45-degree tie case)
    "traceRay 4": ((0.5, 0.5, 0.5), "n110", (0, 0, 0), [
        ((0, 1, 0), 0.707106769), ((1, 1, 0), 0.707106769), ((1, 2, 0), 2.12132024),
        ((2, 2, 0), 2.12132024), ((2, 3, 0), 3.53553390), ((3, 3, 0), 3.53553390),
        ((3, 4, 0), 4.94974756), ((4, 4, 0), 4.94974756)]),
}


@pytest.mark.parametrize("name", sorted(GRID_CASES))
def test_grid_trace_ray(oracle_mod, name):
    orig, d, first, seq = GRID_CASES[name]
    if d == "n210":
        d = norm([2, 1, 0])
    elif d == "n110":
        d = norm([1, 1, 0])
    out = oracle_mod.grid_trace((0, 0, 0), (5, 5, 5), (5, 5, 5), orig, d)
    assert out is not None
    f, cells, ts = out
    assert f == first
    assert len(ts) == len(seq) + 1
    for k, (cell, t) in enumerate(seq):
        assert abs(ts[k] - t) <= 1e-4, (k, ts[k], t)
        assert tuple(int(c) for c in cells[k]) == cell
    # after the last cell next() returns +inf (exit reached)
    assert ts[-1] == np.inf
