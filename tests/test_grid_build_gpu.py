"""GPU grid build (csrc/grid_build.hip) against the host
build (geometry.cpp, itself pinned to the oracle by test_build_parity.py):
grid, cells, ref order and every baked array, bit for bit."""
import time

import numpy as np
import pytest

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,res", [("sphere", (128, 128, 128)), ("sphere", (5, 7, 3)),
                                      ("cornell", (128, 128, 128)), ("cornell555", (128, 128, 128)),
                                      ("contest", (128, 128, 128)), ("contest", (1, 1, 1)),
                                      ("sponza", (128, 128, 128)), ("sponza", (200, 64, 97))])
def test_device_build_bitexact(name, res):
    soup = scenes.get_scene(name)
    t0 = time.perf_counter()
    h = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, res, num_threads=16)
    t1 = time.perf_counter()
    d = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, res, device=0)
    t2 = time.perf_counter()
    print(f"{name} {res}: host {1e3 * (t1 - t0):.1f} ms, device {1e3 * (t2 - t1):.1f} ms, "
          f"{h.num_refs} refs")
    assert bytes(h.scene.grid) == bytes(d.scene.grid)
    assert h.num_refs == d.num_refs
    assert np.array_equal(h.cells(), d.cells())
    assert np.array_equal(h.indices(), d.indices())
    assert np.array_equal(h.tri_pos().view(np.uint32), d.tri_pos().view(np.uint32))
    assert np.array_equal(h.tri_data().view(np.uint32), d.tri_data().view(np.uint32))
    assert np.array_equal(h.tri_material(), d.tri_material())


def test_device_build_rejects_bad_args():
    soup = scenes.get_scene("sphere")
    with pytest.raises(native.ZrtError):
        native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, (0, 128, 128), device=0)
    with pytest.raises(native.ZrtError):
        native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, (8, 8, 8), device=99)


# zrt_context_create_built: the device build feeding the render context
# directly renders exactly what the host-built context renders (image, linear
# radiance and the traversal counters), timed kernels and counting build.
@pytest.mark.parametrize("name,res", [("cornell", (128, 128, 128)), ("contest", (128, 128, 128)),
                                      ("sponza", (200, 64, 97)), ("sphere", (1, 1, 1))])
@pytest.mark.parametrize("stats", [False, True])
def test_context_built_on_device_renders_identically(name, res, stats):
    soup = scenes.get_scene(name)
    cam = camera_for(soup, None, None if soup.camera(None).aspect else 96, 54)
    h = RenderScene(soup, res)
    d = RenderScene(soup, res, device_build=True)
    try:
        cells = h.geometry.cells()
        k = cells[:, 1] - cells[:, 0]
        want = (h.geometry.num_refs, int((k == 0).sum()),
                int(k[k > 0].min()) if (k > 0).any() else 0xFFFFFFFF, int(k.max()))
        assert h.context.grid_info() == want
        assert d.context.grid_info() == want
        ih, rh = h.render(cam, num_samples=2, max_bounce=4, stats=stats, linear=True)
        idv, rd = d.render(cam, num_samples=2, max_bounce=4, stats=stats, linear=True)
        assert np.array_equal(ih, idv)
        assert np.array_equal(rh["linear"].view(np.uint32), rd["linear"].view(np.uint32))
        if stats:
            ks = [k for k in rh["stats"] if not k.endswith("_ms")]
            assert {k: rh["stats"][k] for k in ks} == {k: rd["stats"][k] for k in ks}
    finally:
        h.close()
        d.close()


def test_context_built_rejects_bad_args():
    soup = scenes.get_scene("sphere")
    mats = native.Scene()
    keep = []
    native.attach_materials(mats, soup.tex_desc, soup.texels, keep)
    with pytest.raises(native.ZrtError):
        native.Context.built(soup.pos, soup.nrm, soup.uv, soup.mat, mats, (0, 8, 8), 0)
    with pytest.raises(native.ZrtError):
        native.Context.built(soup.pos, soup.nrm, soup.uv, soup.mat + 1000, mats, (8, 8, 8), 0)
    with pytest.raises(native.ZrtError):
        native.Context.built(soup.pos, soup.nrm, soup.uv, soup.mat, mats, (8, 8, 8), 99)
