"""The multi-rank bench path on the GPU box: bench.py under torchrun with two,
three or eight ranks (the driver's largest world: padded block lists) sharing
the one leased GPU (gloo backend, tiles staged through host memory), three
frames in flight, a flyby camera (every frame different).
Every gathered frame must equal, byte for byte, the frame the single-rank
run of the same command renders. This executes the distributed init, the
cost-balanced sr_render_block_list shares (and the block-cyclic
sr_render_blocks_batch ones), FrameGather, the in-flight pipeline and
the max-over-ranks timing of bench.py (the 8-GPU run uses the same code with
the nccl backend). Both runs are child processes: this test process never
touches the GPU."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
ARGS = ["--width", "320", "--height", "180", "--max-steps", "800", "--steps", "12", "--warmup", "2",
        "--inflight", "3", "--camera", "flyby", "--cpu-baseline", "off", "--critical-path", "off",
        "--reference-loop", "off"]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(cmd, out):
    r = subprocess.run(cmd + ARGS + ["--dump-frames", str(out)], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("world,balance", [(2, "cost"), (3, "cost"), (2, "cyclic"), (8, "cost"), (8, "auto")])
def test_multi_rank_bench_frames_equal_single_rank(tmp_path, world, balance):
    try:
        import torch
    except ImportError:
        pytest.skip("torch missing")
    single = run([sys.executable, "bench.py", "--gpus", "1"], tmp_path / "one")
    multi = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                 "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(world),
                 "--dist-backend", "gloo", "--balance", balance], tmp_path / "multi")
    assert multi["n_gpus"] == world and single["n_gpus"] == 1
    bal = multi["config"]["balance"]
    if balance == "cost":
        assert bal["max_over_mean"] <= bal["cyclic_max_over_mean"] + 1e-9, bal
    else:  # auto with the flyby: cyclic rows (dist.REPRICE_MARGIN)
        assert bal is None
    assert multi["config"]["balance_policy"]["used"] == ("cost" if balance == "cost" else "cyclic")
    assert multi["config"]["dist_backend"] == "gloo" and multi["config"]["launches_in_flight"] == 3
    ranks = multi["config"]["ranks"]  # the N-rank line documents every rank
    assert [r["rank"] for r in ranks] == list(range(world)) and all(r["world_size"] == world for r in ranks)
    assert all(r["share_ms_per_frame"] > 0 and r["gather_ms_per_frame"] >= 0 for r in ranks)
    lc = multi["config"]["last_camera_max_over_mean"]
    assert lc["lists_in_use"] >= 1.0 and lc["cyclic"] >= 1.0
    if balance == "cost":  # the flyby re-prices the lists while frames are in flight
        assert bal["lists_from"] == "rank 0 (broadcast)" and bal["repriced"] >= 1, bal
        assert set(bal["reprice_choices"]) <= {"priced", "cyclic"} and len(bal["reprice_choices"]) == bal["repriced"]
        assert lc["frame0_lists"] >= 1.0
    else:
        assert lc["lists_in_use"] == lc["cyclic"]
    one = sorted((tmp_path / "one").glob("frame_*.npy"))
    many = sorted((tmp_path / "multi").glob("frame_*.npy"))
    assert len(one) == len(many) == 12
    distinct = set()
    for a, b in zip(one, many):
        assert a.name == b.name
        fa, fb = np.load(a), np.load(b)
        assert fa.shape == fb.shape == (180, 320, 4)
        assert np.array_equal(fa, fb), a.name
        distinct.add(fa.tobytes())
    assert len(distinct) == 12  # the flyby moves the camera every frame


def test_bench_gpus_2_without_a_launcher(tmp_path):
    """The driver's BENCH command shape with N = 2 and no torchrun: bench.py
    spawns its two ranks itself (launch_contract; gloo here, both on the one
    GPU), labels the line with them, and its last timed headline frame matches
    the oracle's frame hashes."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--steps", "4",
                        "--warmup", "2", "--cpu-baseline", "off", "--critical-path", "off", "--reference-loop", "off"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0's line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size"] == 2
    assert [x["rank"] for x in d["config"]["ranks"]] == [0, 1]
    assert d["parity"]["frame_sha_match"] is True, d["parity"]


def test_bench_nccl_refuses_two_ranks_on_one_gpu():
    """--gpus 2 with RCCL on a one-GPU box: a clear, quick failure instead of
    two RCCL ranks on one device."""
    import time

    try:
        import torch
        n = torch.cuda.device_count()
    except ImportError:
        pytest.skip("torch missing")
    if n >= 2:
        pytest.skip("more than one GPU visible")
    t = time.monotonic()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "nccl", "--steps", "2"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "needs one GPU per rank" in r.stderr, r.stderr[-2000:]
    assert time.monotonic() - t < 60
