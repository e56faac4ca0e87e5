import time, sys, os
sys.path.insert(0, os.getcwd())
from zig_raytracing_contest_amd import native, scenes
import ctypes as C
soup = scenes.get_scene("contest")
L = native.lib()
t=time.perf_counter(); L.zrt_device_warmup(0); print("warmup %.1f ms" % ((time.perf_counter()-t)*1e3))
for k in range(3):
    t=time.perf_counter(); g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, device=0); print("device build %d: %.1f ms" % (k, (time.perf_counter()-t)*1e3))
t=time.perf_counter(); g = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, num_threads=16); print("host build: %.1f ms" % ((time.perf_counter()-t)*1e3))
