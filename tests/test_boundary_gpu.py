"""The drop-in boundary on the GPU, exactly as its callers use it.

* zrt_render -- the one-shot export INTEGRATION.md binds in place of
  Scene.render (stage3.zig:247, called at main.zig:126): upload, render,
  download, free -- against the committed golden renders (tests/golden/,
  tools/make_golden.py), no oracle at run time.
* bench.py's multi-GPU step (dist.render_gathered): render into a torch
  device buffer through zrt_outputs.device_rgb_packed, then the gather of
  packed RGB8 tiles to rank 0 -- over a real "nccl" (RCCL) process group at
  world size 1, and over gloo with two ranks sharing the GPU; both must equal
  the single-process host-copy image.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import torch  # noqa: F401  (first: libzrt then binds to torch's HIP runtime, as in bench.py)

from zig_raytracing_contest_amd import RenderScene, camera_for, native, scenes
from zig_raytracing_contest_amd import dist as zdist

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name", ["sphere", "cornell", "contest"])
def test_oneshot_zrt_render_matches_golden(name):
    g = np.load(os.path.join(GOLD, f"render_{name}.npz"), allow_pickle=False)
    soup = scenes.get_scene(name)
    cname = str(g["camera"]) or None
    c = soup.camera(cname)
    cam = camera_for(soup, cname, None if c.aspect else int(g["w"]), int(g["h"]))
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat)
    keep = []
    native.attach_materials(geo.scene, soup.tex_desc, soup.texels, keep)
    img, st = native.render_oneshot(geo.scene, cam, int(g["spp"]), int(g["max_bounce"]), seed=int(g["seed"]))
    assert np.array_equal(img.reshape(-1, 3), g["rgb"])
    assert st["samples"] == cam.w * cam.h * int(g["spp"])
    assert st["segments"] == int(g["counters"][0])


def _golden_scene(name):
    g = np.load(os.path.join(GOLD, f"render_{name}.npz"), allow_pickle=False)
    soup = scenes.get_scene(name)
    cname = str(g["camera"]) or None
    c = soup.camera(cname)
    cam = camera_for(soup, cname, None if c.aspect else int(g["w"]), int(g["h"]))
    return g, soup, cam


@pytest.mark.parametrize("name,devices", [("contest", [0, 0]), ("cornell", [0, 0, 0]), ("sphere", [0, 0])])
def test_oneshot_zrt_render_device_list_matches_golden(name, devices):
    """zrt_render with a device list (zrt_render_config.devices): the tiles
    split over one context per entry (two or three contexts sharing GPU 0
    here; the 8-GPU node is the driver's), gathered on the first device,
    equal the golden one-device image bit for bit (stage3.zig:247-256 spawns
    and joins every worker inside the one call)."""
    g, soup, cam = _golden_scene(name)
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat)
    keep = []
    native.attach_materials(geo.scene, soup.tex_desc, soup.texels, keep)
    img, st = native.render_oneshot(geo.scene, cam, int(g["spp"]), int(g["max_bounce"]), seed=int(g["seed"]),
                                    devices=devices)
    assert np.array_equal(img.reshape(-1, 3), g["rgb"])
    assert st["samples"] == cam.w * cam.h * int(g["spp"])
    assert st["segments"] == int(g["counters"][0])


def test_group_built_and_rank_share():
    """zrt_group_create_built (the grid built on every device of the group)
    renders the golden image; with num_ranks 2 the group renders only this
    process's tiles (rank 1), each device a sub-rank, and leaves the other
    pixels of the caller's image untouched."""
    g, soup, cam = _golden_scene("contest")
    mats = native.Scene()
    keep = []
    native.attach_materials(mats, soup.tex_desc, soup.texels, keep)
    grp = native.Group.built(soup.pos, soup.nrm, soup.uv, soup.mat, mats, [0, 0])
    try:
        img, st = grp.render(cam, int(g["spp"]), int(g["max_bounce"]), seed=int(g["seed"]))
        assert np.array_equal(img.reshape(-1, 3), g["rgb"])
        assert st["segments"] == int(g["counters"][0])
        part = np.full((cam.h, cam.w, 3), 7, np.uint8)
        grp.render(cam, int(g["spp"]), int(g["max_bounce"]), seed=int(g["seed"]), rank=1, num_ranks=2, image=part)
    finally:
        grp.close()
    mine = native.tile_pixels(cam.w, cam.h, 32, 1, 2)       # 32x32 tiles: the default over several devices
    assert 0 < mine.size < cam.w * cam.h
    flat = part.reshape(-1, 3)
    assert np.array_equal(flat[mine], g["rgb"][mine])
    other = np.ones(cam.w * cam.h, bool)
    other[mine] = False
    assert (flat[other] == 7).all()


def test_oneshot_zrt_render_rejects_bad_input():
    soup = scenes.get_scene("sphere")
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat, resolution=(8, 8, 8))
    keep = []
    native.attach_materials(geo.scene, soup.tex_desc, soup.texels, keep)
    cam = camera_for(soup, None, 16, 16)
    with pytest.raises(native.ZrtError) as e:
        native.render_oneshot(geo.scene, cam, 0, 4)
    assert e.value.status == -1
    with pytest.raises(native.ZrtError) as e:
        native.render_oneshot(geo.scene, cam, 1, 4, device=99)
    assert e.value.status == -2
    with pytest.raises(native.ZrtError) as e:
        native.render_oneshot(geo.scene, cam, 1, 4, devices=[0, 99])
    assert e.value.status == -2
    # a one-entry list names the device: [99] fails, [0] renders on 0 whatever
    # cfg.device says (it used to fall back to cfg.device)
    with pytest.raises(native.ZrtError) as e:
        native.render_oneshot(geo.scene, cam, 1, 4, devices=[99])
    assert e.value.status == -2
    one, _ = native.render_oneshot(geo.scene, cam, 1, 4, device=99, devices=[0])
    ref, _ = native.render_oneshot(geo.scene, cam, 1, 4, device=0)
    assert np.array_equal(one, ref)
    # num_devices 1 without a list keeps cfg.device (ABI-1 callers)
    null1, _ = native.render_oneshot(geo.scene, cam, 1, 4, device=0, num_devices=1)
    assert np.array_equal(null1, ref)
    with pytest.raises(native.ZrtError) as e:
        native.render_oneshot(geo.scene, cam, 1, 4, device=99, num_devices=1)
    assert e.value.status == -2


def _visible_gpus():
    import torch      # device_count() does not initialise HIP on this image
    return torch.cuda.device_count()


@pytest.mark.skipif(_visible_gpus() < 2, reason="needs two distinct GPUs (the peer-copy gather)")
@pytest.mark.parametrize("name", ["contest", "cornell"])
def test_oneshot_zrt_render_distinct_devices_matches_golden(name):
    """The cross-GPU branch of the group's gather (hipDeviceEnablePeerAccess
    + hipMemcpyPeerAsync, group.hip) on two DIFFERENT ordinals: the golden
    image bit for bit.  Skipped on one-GPU boxes (until it
    has run, DESIGN/INTEGRATION say the peer path is unverified)."""
    g, soup, cam = _golden_scene(name)
    geo = native.Geometry(soup.pos, soup.nrm, soup.uv, soup.mat)
    keep = []
    native.attach_materials(geo.scene, soup.tex_desc, soup.texels, keep)
    img, st = native.render_oneshot(geo.scene, cam, int(g["spp"]), int(g["max_bounce"]), seed=int(g["seed"]),
                                    devices=[1, 0])
    assert np.array_equal(img.reshape(-1, 3), g["rgb"])
    assert st["segments"] == int(g["counters"][0])


def test_bench_gather_path_nccl_world1():
    import torch
    import torch.distributed as dist
    soup = scenes.get_scene("contest")
    cam = camera_for(soup, "Camera 1", None, 90)
    rs = RenderScene(soup, device=0)
    ref, _ = rs.render(cam, num_samples=2, max_bounce=4)              # host copy
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        buf = torch.zeros(zdist.max_packed(cam.w, cam.h, 1) * 3, dtype=torch.uint8, device="cuda:0")
        img, res = zdist.render_gathered(rs.context, cam, 2, 4, 0, 1, dist, buf)
        torch.cuda.synchronize()
        assert np.array_equal(img.cpu().numpy(), ref)
        assert res["stats"]["samples"] == cam.w * cam.h * 2
    finally:
        dist.destroy_process_group()
        rs.close()


_RANK_SCRIPT = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["ZRT_ROOT"])
from zig_raytracing_contest_amd import RenderScene, camera_for, scenes
from zig_raytracing_contest_amd import dist as zdist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
soup = scenes.get_scene("contest")
cam = camera_for(soup, "Camera 1", None, 180)
rs = RenderScene(soup, device=0)
res = rs.context.render(cam, 2, 4, rank=rank, num_ranks=world, packed=True, tile=zdist.TILE)
buf = torch.zeros(zdist.max_packed(cam.w, cam.h, world) * 3, dtype=torch.uint8)
buf[: res["packed"].size] = torch.from_numpy(res["packed"].reshape(-1))
img = zdist.gather_image(buf, cam.w, cam.h, rank, world, dist)
if rank == 0:
    np.save(os.environ["ZRT_OUT"], img.numpy())
dist.barrier()
dist.destroy_process_group()
rs.close()
"""


def test_two_ranks_on_one_gpu_gather_gloo(tmp_path):
    soup = scenes.get_scene("contest")
    cam = camera_for(soup, "Camera 1", None, 180)
    rs = RenderScene(soup, device=0)
    ref, _ = rs.render(cam, num_samples=2, max_bounce=4)
    rs.close()
    port, out = _free_port(), str(tmp_path / "img.npy")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   ZRT_ROOT=ROOT, ZRT_OUT=out)
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK_SCRIPT], env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    assert np.array_equal(np.load(out), ref)


def _bench_json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, stdout[-2000:]
    import json
    return json.loads(lines[0])


def test_bench_entry_two_ranks_gloo_matches_one():
    """bench.py's own N > 1 entry, end to end, as the driver launches it
    (torch.distributed.run, one process per rank, rank 0 prints ONE line):
    two gloo ranks sharing device 0 (--backend gloo is test-only; the driver's
    8-GPU run uses RCCL).  The line says n_gpus 2 and its img_sha1 (the whole
    gathered frame) equals the N = 1 run's."""
    common = ["--config", "cfg2", "--spp", "4", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
              "--no-wall-clock"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + common, cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr[-3000:]
    j1 = _bench_json(one.stdout)
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo"] + common,
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert two.returncode == 0, two.stderr[-3000:]
    j2 = _bench_json(two.stdout)
    assert j1["n_gpus"] == 1 and j2["n_gpus"] == 2
    assert j1["img_sha1"] and j2["img_sha1"] == j1["img_sha1"]
    assert j2["config"]["segments_per_step"] == j1["config"]["segments_per_step"]
    # the driver's plain form, no launcher: bench.py starts its own 2 ranks
    env.pop("WORLD_SIZE", None)
    own = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo"]
                         + common, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert own.returncode == 0, own.stderr[-3000:]
    j3 = _bench_json(own.stdout)
    assert j3["n_gpus"] == 2 and j3["img_sha1"] == j1["img_sha1"]
    assert j3["config"]["parallelism"] == "tiles2"
