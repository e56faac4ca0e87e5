"""Scene-to-context wall clock on one GPU: host build +
upload (zrt_geometry_build + zrt_context_create), device build with the host
round trip (zrt_geometry_build_device + zrt_context_create) and the device
build straight into the context (zrt_context_create_built)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
from zig_raytracing_contest_amd import RenderScene, native, scenes  # noqa: E402


def ms(t):
    return (time.perf_counter() - t) * 1e3


for name in sys.argv[1:] or ["contest", "sponza"]:
    soup = scenes.get_scene(name)
    t = time.perf_counter()
    native.lib().zrt_device_warmup(0)
    print(f"warmup {ms(t):.1f} ms")
    for k in range(3):
        t = time.perf_counter()
        g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, num_threads=16)
        t1 = ms(t)
        keep = []
        native.attach_materials(g.scene, soup.tex_desc, soup.texels, keep)
        c = native.Context(g.scene, 0)
        print(f"{name} host build {t1:.1f} ms + upload -> {ms(t):.1f} ms")
        c.close()
        t = time.perf_counter()
        g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, device=0)
        t1 = ms(t)
        native.attach_materials(g.scene, soup.tex_desc, soup.texels, keep)
        c = native.Context(g.scene, 0)
        print(f"{name} device build {t1:.1f} ms + upload -> {ms(t):.1f} ms")
        c.close()
        t = time.perf_counter()
        r = RenderScene(soup, device=0, device_build=True)
        print(f"{name} built into context -> {ms(t):.1f} ms")
        r.close()
