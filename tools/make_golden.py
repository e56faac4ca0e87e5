#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz from the CPU oracle (oracle/zrt_oracle.c).

Small, deterministic inputs -> outputs: renders (build-mode counter RNG and
the reference's REF-mode Xoshiro schedule), Moller-Trumbore, DDA, slab,
toRGB, texture sampling and RNG streams.  tests/test_golden.py checks the
oracle still reproduces them (CPU) and that the HIP path does (GPU).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402

from zig_raytracing_contest_amd import scenes  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def _norm(v):
    v = np.asarray(v, np.float32)
    return v * (np.float32(1) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))


def renders():
    for name, cam_name, w, h, spp in (("sphere", None, 32, 32, 2), ("cornell", None, 24, 24, 3),
                                      ("contest", "Camera 1", 48, 27, 2)):
        soup = scenes.get_scene(name)
        c = soup.camera(cam_name)
        cam = orc.camera_from_matrix(c.matrix, c.yfov, c.aspect, None if c.aspect else w, h)
        sc = orc.OracleScene(soup)
        rgb, lin, ctr = sc.render(cam, spp, 4, orc.RNG_PATH, 0, 8)
        rgb_ref, lin_ref, ctr_ref = sc.render(cam, spp, 4, orc.RNG_REF, 0, 4)
        np.savez_compressed(os.path.join(OUT, f"render_{name}.npz"), w=cam.w, h=cam.h, spp=spp,
                            max_bounce=4, seed=0, camera=cam_name or "", rgb=rgb, linear=lin,
                            counters=ctr, rgb_ref4=rgb_ref, linear_ref4=lin_ref, counters_ref4=ctr_ref)


def vectors():
    rng = np.random.default_rng(20241115)
    n = 512
    tri = rng.uniform(-1, 1, (n, 9)).astype(np.float32)
    o = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    cen = (tri[:, :3] + tri[:, 3:6] + tri[:, 6:]) / 3
    d = np.stack([_norm(x) for x in (cen - o)]).astype(np.float32)
    d[::3] = np.stack([_norm(x) for x in rng.uniform(-1, 1, (len(d[::3]), 3))])
    hit = np.zeros(n, np.uint8)
    tuv = np.zeros((n, 3), np.float32)
    for i in range(n):
        h, r = orc.tri_intersect(tri[i, :3], tri[i, 3:6], tri[i, 6:], o[i], d[i])
        hit[i], tuv[i] = h, r
    # DDA on a 5x7x3 grid over random boxes
    m = 128
    box = np.concatenate([lo := rng.uniform(-3, 0, (m, 3)), lo + rng.uniform(0.5, 4, (m, 3))], 1).astype(np.float32)
    ro = rng.uniform(-6, 6, (m, 3)).astype(np.float32)
    rd = np.stack([_norm(rng.uniform(box[i, :3], box[i, 3:]) - ro[i]) for i in range(m)]).astype(np.float32)
    steps = np.full(m, -1, np.int32)
    cells = np.zeros((m, 64, 3), np.uint32)
    ts = np.zeros((m, 64), np.float32)
    for i in range(m):
        r = orc.grid_trace(box[i, :3], box[i, 3:], (5, 7, 3), ro[i], rd[i], 64)
        if r is not None:
            steps[i] = len(r[2])
            cells[i, :steps[i]] = r[1]
            ts[i, :steps[i]] = r[2]
    vals = np.concatenate([rng.uniform(0, 1.2, (300, 3)),
                           np.array([[0, 1, 2], [np.nan, np.inf, -1], [1e-40, 0.999999, 1e30]])]).astype(np.float32)
    rgb = np.stack([orc.to_rgb(v) for v in vals])
    keys = np.array([[0, p, s] for p in (0, 1, 777, 2 ** 22 + 3) for s in (0, 1, 65535)], np.uint32)
    f32 = np.stack([orc.path_f32(int(k[0]), int(k[1]), int(k[2]), 16) for k in keys])
    nrm = np.stack([orc.path_norm(int(k[0]), int(k[1]), int(k[2]), 16) for k in keys])
    np.savez_compressed(os.path.join(OUT, "vectors.npz"), tri=tri, tri_o=o, tri_d=d, tri_hit=hit,
                        tri_tuv=tuv, dda_box=box, dda_o=ro, dda_d=rd, dda_res=np.array([5, 7, 3], np.uint32),
                        dda_steps=steps, dda_cells=cells, dda_t=ts, rgb_in=vals, rgb_out=rgb,
                        rng_keys=keys, rng_f32=f32, rng_norm=nrm)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    renders()
    vectors()
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
