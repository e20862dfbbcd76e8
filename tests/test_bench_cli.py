"""bench.py's command line (driver contract) and its workloads against
BASELINE.json's configs; no GPU needed."""
import argparse
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _parse(argv):
    import bench

    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_defaults_are_the_headline_on_one_gpu():
    import bench

    a = _parse([])
    assert a.gpus == 1 and a.workload == "headline" and a.mode == "curved" and a.percent_black < 0
    assert bench.WORKLOADS["headline"] == (1920, 1080, 2000)
    assert a.steps >= 1 and a.warmup >= 0 and a.inflight == 0


def test_driver_flags_parse():
    a = _parse(["--gpus", "8", "--steps", "5", "--warmup", "2"])
    assert (a.gpus, a.steps, a.warmup) == (8, 5, 2)


def test_workloads_match_baseline_configs():
    import bench

    configs = json.loads((ROOT / "BASELINE.json").read_text())["configs"]
    sizes = []
    for c in configs:
        m = re.search(r"(\d+)x(\d+)[^,]*, (\d+) steps", c)
        if m:
            sizes.append(tuple(int(v) for v in m.groups()))
    assert sorted(sizes) == sorted(bench.WORKLOADS.values())
    metric = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
    assert "1920x1080" in metric and "2000" in metric


def test_help_runs_without_a_gpu():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--workload" in r.stdout and "--inflight" in r.stdout


def test_frames_per_launch_by_rank_share():
    import bench

    # about eight headline frames' worth of a rank's share per launch, 1..16
    assert [bench.frames_per_launch(1920, 1080, n) for n in (1, 2, 4, 8)] == [16, 16, 16, 16]
    # at most half of the timed window per launch (two launches overlap their tails)
    assert [bench.frames_per_launch(1920, 1080, n, 20) for n in (1, 2, 4, 8)] == [16, 10, 10, 10]
    assert bench.frames_per_launch(1920, 1080, 1, 5) == 3 and bench.frames_per_launch(1920, 1080, 1, 1) == 1
    assert bench.frames_per_launch(1920, 1080, 1, 8) == 4 and bench.frames_per_launch(1920, 1080, 1, 96) == 16
    assert bench.frames_per_launch(640, 360, 1) == 16  # config 2
    assert bench.frames_per_launch(3840, 2160, 1) == 2 and bench.frames_per_launch(3840, 2160, 8) == 16
    assert bench.frames_per_launch(7680, 4320, 1) == 1 and bench.frames_per_launch(7680, 4320, 8) == 4
    assert bench.launches_in_flight(4) == 3 and bench.launches_in_flight(1) == 4
    # one GPU at the headline's scale: 16 frames per launch, two in flight
    assert bench.launches_in_flight(16, 1920, 1080, 1) == 2 and bench.launches_in_flight(16, 1920, 1080, 2) == 3
    assert bench.launches_in_flight(16, 640, 360, 1) == 3 and bench.launches_in_flight(4, 1920, 1080, 1) == 3
    a = _parse(["--batch", "2", "--split", "32:4:1000"])
    assert a.batch == 2 and a.split == "32:4:1000"


def test_cpu_baseline_sweeps_the_full_frame():
    """`value` is the wall time over the full frame (every
    row), the like-for-like SwiftShader figure is quoted beside it."""
    import bench
    import srpkg

    cam = srpkg.load_package().abi.default_camera()
    out = bench.cpu_baseline(cam, 48, 27, 60, 0, sweeps=(("48x27/60", 48, 27, 60),), rays=())
    assert out["sample"].startswith("full frame") and "all 27 rows" in out["sample"]
    assert out["value"] > 0 and out["kind"] == "port" and out["cores"] >= 1
    assert out["configs"]["48x27/60"]["same_as"] == "value"
    assert out["like_for_like"]["value"] == 0.00225
    part = bench.cpu_baseline(cam, 48, 27, 60, 9, sweeps=(), rays=())
    assert part["sample"].startswith("sample: ") and "rows [9,18)" in part["sample"]


def _bench(args, env_extra=None, timeout=120):
    import os

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_world_size_must_equal_gpus():
    """A launcher's WORLD_SIZE that differs from --gpus is an error (before
    any torch or HIP import), not a mislabelled line."""
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=30)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and "--gpus 1" in r.stderr
    r = _bench(["--gpus", "4"], {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}, timeout=30)
    assert r.returncode != 0 and "--gpus 4" in r.stderr
    r = _bench(["--gpus", "0"], timeout=30)
    assert r.returncode != 0


def test_spawned_ranks_need_a_gpu_each_for_nccl():
    """--gpus 2 without a launcher spawns two ranks (launch_contract); with
    the nccl backend and fewer visible GPUs than local ranks (none here) every
    rank exits non-zero at once with the reason, and so does the parent."""
    import time

    t = time.monotonic()
    r = _bench(["--gpus", "2", "--dist-backend", "nccl", "--steps", "2"], {"HIP_VISIBLE_DEVICES": ""}, timeout=120)
    assert r.returncode != 0
    assert r.stderr.count("needs one GPU per rank: 2 local ranks") == 2, r.stderr[-2000:]
    assert time.monotonic() - t < 60


def test_spawn_ranks_env_and_status(tmp_path):
    """spawn_ranks gives each rank the env:// rendezvous of
    torch.distributed.run and returns the first failure's status."""
    import bench

    probe = tmp_path / "probe.py"
    probe.write_text("import json, os, sys\n"
                     "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
                     f"open(r'{tmp_path}/rank' + os.environ['RANK'], 'w').write(json.dumps({{k: os.environ[k] for k in keys}}))\n"
                     "sys.exit(int(sys.argv[1]) if os.environ['RANK'] == sys.argv[2] else 0)\n")
    old = bench.__file__
    try:
        bench.__file__ = str(probe)
        assert bench.spawn_ranks(3, ["0", "-1"]) == 0
        envs = [json.loads((tmp_path / f"rank{r}").read_text()) for r in range(3)]
        assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
        assert all(e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1"
                   for e in envs)
        assert len({e["MASTER_PORT"] for e in envs}) == 1
        assert bench.spawn_ranks(2, ["7", "1"], grace_s=5) == 7
    finally:
        bench.__file__ = old


def test_spawn_ranks_retries_a_taken_port(tmp_path):
    """free_port() releases its socket before rank 0's store binds
    the port. A rank 0 that finds it taken exits with EXIT_PORT_TAKEN and
    spawn_ranks starts every rank again on a new port; the real store's error
    on a held port is what `port_taken` recognises."""
    import os
    import socket

    import bench

    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys\n"
                     f"d = r'{tmp_path}'\n"
                     "n = len([f for f in os.listdir(d) if f.startswith('try')])\n"
                     "if os.environ['RANK'] == '0':\n"
                     "    open(os.path.join(d, 'try%d_' % n + os.environ['MASTER_PORT']), 'w').close()\n"
                     "    sys.exit(98 if n == 0 else 0)\n")
    old = bench.__file__
    try:
        bench.__file__ = str(probe)
        assert bench.spawn_ranks(2, [], grace_s=60) == 0
    finally:
        bench.__file__ = old
    tries = sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("try"))
    assert len(tries) == 2 and tries[0].split("_")[1] != tries[1].split("_")[1]
    # the store's own message for a port another socket holds
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        code = ("import datetime, os, torch.distributed as d\n"
                "try:\n"
                "    d.init_process_group('gloo', timeout=datetime.timedelta(seconds=5))\n"
                "except Exception as e:\n"
                "    print(str(e))\n")
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), RANK="0",
                   WORLD_SIZE="2")
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert bench.port_taken(RuntimeError(out.stdout)), out.stdout + out.stderr
    assert not bench.port_taken(RuntimeError("connection refused"))


def test_roofline_steps_per_frame_and_launch():
    """roofline.steps_per_frame is one frame's executed ray-steps of the
    rank's rows, and steps_per_frame x frames_per_launch the launch's (a
    static camera: B equal frames), checked against the oracle's step map of a
    small config rendered B times."""
    import argparse

    import numpy as np

    import bench
    import srpkg

    pkg, oracle = srpkg.load_package(), srpkg.load_oracle()
    sc, abi = pkg.scenes, pkg.abi
    W, H, N, B = 48, 32, 300, 3
    scene, cam = sc.scene_default(textured=False), abi.default_camera()
    params = abi.default_params(max_steps=N, percent_black=-1.0)
    tex = oracle.TextureSet(sc.skybox(64, 32), sc.default_texture_array()[0])
    launch_steps = sum(int(oracle.render(scene, cam, params, W, H, tex)[2].astype(np.int64).sum()) for _ in range(B))
    frame_steps = launch_steps // B
    args = argparse.Namespace(pmc_json="/nonexistent", traffic_json="/nonexistent", camera="static",
                              scene="default", test_ray="off")
    rf = bench.make_roofline(args, W, H, N, 1, 2, B, 0.1, [[0.1, 0.01, 0.0]], [B], 0.3, frame_steps, frame_steps, H,
                             None, None)
    assert rf["steps_per_frame"] == frame_steps and rf["frames_per_launch"] == B
    assert rf["steps_per_frame"] * rf["frames_per_launch"] == rf["steps_per_launch"] == launch_steps
    args.camera = "flyby"
    assert bench.make_roofline(args, W, H, N, 1, 2, B, 0.1, [[0.1, 0.01, 0.0]], [B], 0.3, frame_steps, frame_steps,
                               H, None, None)["steps_per_launch"] is None


def test_launch_accounting_unequal_launches():
    """The driver's 20-frame window in launches of 16 is [16, 4] (two
    launches in flight): kernel_ms is the plain mean of the two durations (as
    rocprofv3 --stats averages them), each size is reported apart, and
    overlap is the total integrate duration over the window."""
    import bench

    ms_per_step = 0.8
    kt = [[11.9, 0.9, 0.02], [3.6, 0.25, 0.01]]  # 16 frames, 4 frames (integrate, shade, resume)
    acc = bench.launch_accounting(kt, [16, 4], ms_per_step)
    assert acc["kernel_ms"] == round((11.9 + 3.6) / 2, 4)
    assert acc["kernel_ms_by_launch_frames"] == {"16": 11.9, "4": 3.6}
    assert acc["kernel_ms_per_frame"] == round((11.9 + 3.6) / 20, 4)
    assert acc["overlap"] == round((11.9 + 3.6) / (20 * ms_per_step), 3)
    assert acc["launch_frames"] == [16, 4]
    assert acc["pipeline_ms_per_frame"]["shade"] == round(1.15 / 20, 4)
    # the window's launches as bench.main orders ktimes: context k's launches j = k, k + F, ...
    sizes = [min(16, 20 - f) for f in range(0, 20, 16)]
    F = 2
    assert [sizes[j] for k in range(F) for j in range(k, len(sizes), F)] == [16, 4]


def test_counter_records_keyed_by_scene_variant(tmp_path):
    """A PMC / traffic record counts for a bench line only when it was taken
    on the same config, kernel source and scene variant (default, stress,
    testray): the stress and test-ray lines read their own files."""
    import bench

    args = argparse.Namespace(scene="stress", test_ray="off")
    assert bench.scene_variant(args) == "stress"
    assert bench.scene_variant(argparse.Namespace(scene="default", test_ray="on")) == "testray"
    assert bench.profile_record("", "pmc", "default").name == "pmc_latest.json"
    assert bench.profile_record("", "traffic", "stress").name == "traffic_latest_stress.json"
    assert bench.profile_record(str(tmp_path / "x.json"), "pmc", "stress") == tmp_path / "x.json"
    rec = {"width": 640, "height": 360, "max_steps": 1000, "kernel_sha": bench.kernel_sha(), "variant": "stress"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(rec))
    assert bench.load_matching(p, 640, 360, 1000, 1, "stress") == rec
    assert bench.load_matching(p, 640, 360, 1000, 1, "default") is None
    assert bench.load_matching(p, 640, 360, 1000, 1, "testray") is None
    assert bench.load_matching(p, 1920, 1080, 2000, 1, "stress") is None
    del rec["variant"]  # records from before the variant key: the default scene
    p.write_text(json.dumps(rec))
    assert bench.load_matching(p, 640, 360, 1000, 1) == rec
    # options that change the kernel's work per frame never read the default's counters
    base = dict(scene="default", test_ray="off", mode="curved", percent_black=-1.0, no_cull=False, camera="static")
    assert bench.counter_variant(argparse.Namespace(**base)) == "default"
    for k, v, key in (("mode", "half_width", "default_half_width"), ("percent_black", 0.75, "default_noise"),
                      ("no_cull", True, "default_nocull"), ("camera", "flyby", "default_flyby")):
        key_got = bench.counter_variant(argparse.Namespace(**{**base, k: v}))
        assert key_got == key
        assert bench.load_matching(p, 640, 360, 1000, 1, key_got) is None
    assert bench.counter_variant(argparse.Namespace(**{**base, "scene": "stress"})) == "stress"
    assert bench.load_matching(p, 640, 360, 1000, 1, "stress") is None
