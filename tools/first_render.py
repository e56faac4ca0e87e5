import sys, time, os, json
sys.path.insert(0, os.getcwd())
from zig_raytracing_contest_amd import RenderScene, camera_for, scenes
soup = scenes.get_scene("contest")
cam = camera_for(soup, "Camera 1", None, 1080)
rs = RenderScene(soup, device=0, device_build=True)
for k in range(3):
    t0 = time.perf_counter()
    img, r = rs.render(cam, num_samples=3, max_bounce=4)
    dt = time.perf_counter() - t0
    print(json.dumps({"render": k, "ms": round(dt * 1e3, 2), "kernel_ms": round(r["stats"]["trace_kernel_ms"], 2),
                      "render_ms": round(r["stats"].get("render_ms", 0), 2)}), flush=True)
