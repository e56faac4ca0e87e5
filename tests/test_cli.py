"""The `zrt` CLI end to end: the drop-in for the reference executable
(src/main.zig:73-143): same flags (main.zig:33-39), the same config.json
(main.zig:56-69), the same phase log lines, glTF in and PNG out.  On the GPU
the written image must equal the CPU oracle's render of the same scene, bit
for bit."""
import dataclasses
import json
import os
import subprocess

import numpy as np
import pytest

from zig_raytracing_contest_amd import native, pngio, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ZRT = os.path.join(ROOT, "zig_raytracing_contest_amd", "bin", "zrt")
CFG = {"grid_resolution": [128, 128, 128], "num_threads": None, "num_samples": 3, "max_bounce": 4}

pytestmark = pytest.mark.skipif(not os.path.exists(ZRT), reason="zrt CLI not built")


def _run(args, cwd, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([ZRT] + args, cwd=cwd, capture_output=True, text=True, timeout=180, env=e)


def test_cli_argument_and_config_errors(tmp_path):
    """main.zig's failure modes, before any GPU work: zig-args errors,
    std.json's missing file / unknown field, a missing input file."""
    r = _run(["--bogus", "x"], tmp_path)
    assert r.returncode == 1 and "unknown option --bogus" in r.stderr
    r = _run(["--width", "70000"], tmp_path)
    assert r.returncode == 1 and "u16" in r.stderr
    r = _run([], tmp_path)
    assert r.returncode == 1 and "FileNotFound: config.json" in r.stderr
    (tmp_path / "config.json").write_text(json.dumps(dict(CFG, extra=1)))
    r = _run([], tmp_path)
    assert r.returncode == 1 and "UnknownField: extra" in r.stderr
    (tmp_path / "config.json").write_text(json.dumps(CFG))
    r = _run(["--in", "missing.gltf"], tmp_path)
    assert r.returncode == 1 and "loadGltfFile" in r.stderr
    assert "info: Num samples: 3, max bounce 4" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"ZRT_DEVICE_BUILD": "0"}, {"ZRT_DEVICE_BUILD": "1"},
                                 {"ZRT_DEVICES": "0,0"}],
                         ids=["built-into-context", "host-build", "device-build", "two-ranks"])
def test_cli_render_matches_oracle(tmp_path, oracle_mod, env):
    soup = scenes.get_scene("cornell")
    scenes.write_gltf(soup, str(tmp_path / "c.gltf"))
    (tmp_path / "config.json").write_text(json.dumps(CFG))
    r = _run(["--in", "c.gltf", "--out", "o.png", "--width", "64", "--height", "48"], tmp_path, env)
    assert r.returncode == 0, r.stderr
    for phase in ("Loaded in", "Preprocessed in", "Compiled in", "Rendered in", "Saved in", "Done in"):
        assert f"info: {phase}" in r.stderr
    img = pngio.read(str(tmp_path / "o.png"))[..., :3]
    assert img.shape == (48, 64, 3)
    # the loader normalizes normals (stage1.zig:246): the oracle renders that soup
    loaded = dataclasses.replace(soup, nrm=scenes.f32_normalize(soup.nrm.reshape(-1, 3)).reshape(-1, 9))
    c = soup.camera(None)
    ocam = oracle_mod.camera_from_matrix(c.matrix, c.yfov, c.aspect, 64, 48)
    rgb, _, _ = oracle_mod.OracleScene(loaded).render(ocam, 3, 4, oracle_mod.RNG_PATH, 0, 16)
    assert np.array_equal(img.reshape(-1, 3), rgb)
    # the grid log line (main.zig:117-118 path) on every build path agrees
    # with the host build's cells (pinned to the oracle, test_build_parity.py)
    g = native.Geometry(loaded.pos, loaded.nrm, loaded.uv, loaded.mat, tuple(CFG["grid_resolution"]))
    k = g.cells()[:, 1] - g.cells()[:, 0]
    ne = int((k > 0).sum())
    assert (f"Empty cells: {k.size - ne}/{k.size} ({100.0 * (k.size - ne) / k.size:.2f}%) min triangles: "
            f"{int(k[k > 0].min())} max triangles: {int(k.max())} mean_triangles: {g.num_refs // ne}") \
        in r.stderr
