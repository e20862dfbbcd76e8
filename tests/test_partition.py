"""The multi-GPU frame partition behind the C-ABI (csrc/host/partition.cpp:
sr_block_costs, sr_balanced_blocks, sr_assemble_blocks) against the Python
statement of the same rules (dist.block_costs_py, balanced_blocks_py,
assemble_lists): bit for bit, on CPU (the library's host functions need no
GPU)."""
import numpy as np
import pytest


def ring_costs(rng, nb):
    """Block costs shaped like a frame's: a photon-ring bump over a floor, integer-valued."""
    y = np.arange(nb)
    base = 400.0 + 1600.0 * np.exp(-((y - nb * 0.55) / (nb * 0.12)) ** 2)
    return np.floor(base * rng.uniform(0.8, 1.2, nb) + 8 * rng.integers(0, 200, nb))


@pytest.mark.parametrize("seed", range(12))
def test_balanced_blocks_cpp_equals_python(pkg, seed):
    D = pkg.dist
    rng = np.random.default_rng(seed)
    for nb in (1, 7, 45, 135, 270, 540):
        for world in (1, 2, 3, 4, 8):
            costs = ring_costs(rng, nb) if seed % 3 else rng.uniform(0, 1e4, nb)  # integer and fractional
            a = D.balanced_blocks(costs, world)
            b = D.balanced_blocks_py(costs, world)
            assert a == b, (seed, nb, world)
            assert sorted(x for l in a for x in l if x >= 0) == list(range(nb))


def test_balanced_blocks_ties_and_pads(pkg):
    D = pkg.dist
    for costs, world in (([5.0, 1.0, 3.0], 8), ([0.0] * 5, 2), ([10.0] + [1.0] * 10, 2), ([2.0] * 16, 4),
                         ([3.0, 3.0, 1.0, 1.0, 2.0], 3)):
        assert D.balanced_blocks(costs, world) == D.balanced_blocks_py(costs, world)


def test_block_costs_cpp_equals_python(pkg):
    D = pkg.dist
    rng = np.random.default_rng(3)
    for nb, nc in ((135, 240), (270, 480), (3, 1), (1, 7)):
        w = np.stack([rng.integers(0, 2001, (nb, nc)), rng.integers(0, 300, (nb, nc))], axis=-1).astype(np.int32)
        a = D.block_costs(w)
        b = D.block_costs_py(w)
        assert a.dtype == np.float64 and np.array_equal(a, b)
        assert np.array_equal(D.block_costs(w, 0.0), D.block_costs_py(w, 0.0))


@pytest.mark.parametrize("world,B", [(1, 1), (2, 3), (3, 1), (8, 2)])
def test_assemble_blocks_host_equals_assemble_lists(pkg, world, B):
    D = pkg.dist
    rng = np.random.default_rng(world * 10 + B)
    for H in (180, 1080, 37):
        nb = D.nblocks(H, 8)
        lists = D.balanced_blocks(ring_costs(rng, nb), world)
        per = len(lists[0])
        stacked = rng.integers(0, 256, (world, B, per * 8, 24, 4), dtype=np.uint8)
        want = D.assemble_lists(stacked, lists, H, 8)
        got = D.assemble_blocks_abi(stacked, lists, H, 8)
        assert got.shape == want.shape == (B, H, 24, 4)
        assert np.array_equal(got, want)
        assert np.array_equal(D.assemble_blocks_abi(stacked[:, 0].copy(), lists, H, 8), want[0])


def test_partition_abi_rejects_bad_arguments(pkg):
    import ctypes as C

    lib = pkg.abi.load()
    per = C.c_int()
    out = (C.c_int * 4)()
    cost = (C.c_double * 8)(*range(8))
    assert lib.sr_balanced_blocks(cost, 8, 0, out, 4, C.byref(per)) == pkg.abi.SR_E_INVALID
    assert lib.sr_balanced_blocks(cost, 8, 3, out, 4, C.byref(per)) == pkg.abi.SR_E_CAPACITY  # 3 x 3 > 4
    assert lib.sr_block_costs(None, 1, 1, 8.0, None) == pkg.abi.SR_E_INVALID
    assert lib.sr_assemble_blocks(None, 0, 0, None, 1, 1, 8, 8, 4, None, 0, 1, 0, None) == pkg.abi.SR_E_INVALID


def test_cpp_multi_gpu_driver_builds_and_runs_help():
    """examples/sr_multi_gpu links libsr.so and RCCL (built by build()); --help needs no GPU."""
    import subprocess
    from pathlib import Path

    exe = Path(__file__).resolve().parents[1] / "examples" / "bin" / "sr_multi_gpu"
    if not exe.exists():
        pytest.skip("examples/bin/sr_multi_gpu not built (make -C schwarzschild-raytracer_amd)")
    r = subprocess.run([str(exe), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--gpus" in r.stdout and "WORLD_SIZE" in r.stdout


def test_list_schedule_every_context_adopts_repriced_lists(pkg):
    """bench.py --reprice (dist.ListSchedule): after a re-pricing every context
    renders the new lists from its next launch on, and a launch's render and
    gather always use the same lists (its context switches only between its
    own launches)."""
    D = pkg.dist
    for F, every, B in ((3, 3, 10), (3, 1, 8), (2, 2, 16), (4, 3, 1)):
        sched = D.ListSchedule("L0", F, every, B)
        versions = ["L0"]
        seen = {}  # context -> lists of its last launch
        for j, first in enumerate(range(B * F, B * F + 40 * B, B)):  # after warmup, launches of B frames
            new = None
            if sched.due(first):
                new = f"L{len(versions)}"
                versions.append(new)
            lst, changed = sched.adopt(j, new)
            k = j % F
            assert lst == versions[-1]  # the newest lists, from this launch on
            assert changed == (seen.get(k, "L0") != lst)
            seen[k] = lst
        assert sched.count == len(versions) - 1 and sched.count >= 40 // every - 1
    never = D.ListSchedule("L0", 3, 0, 8)
    assert not any(never.due(f) for f in range(0, 400, 8))
    assert never.adopt(5) == ("L0", False)


def test_reprice_falls_back_to_cyclic_rows(pkg):
    """A re-pricing keeps the priced lists only when they beat block-cyclic
    rows by more than the inter-frame drift margin (dist.REPRICE_MARGIN) under
    the map they were priced from; otherwise every rank gets its cyclic rows
    (padded to the lists' length). bench.py --camera flyby --balance auto uses
    cyclic rows outright."""
    D = pkg.dist
    H, rows, world = 1080, 8, 8
    nb = D.nblocks(H, rows)
    rng = np.random.default_rng(5)
    flat = rng.uniform(1.0, 1.001, nb)  # priced lists cannot beat cyclic by 2 % here
    lists, how = D.choose_lists(D.balanced_blocks(flat, world), flat, world, H, rows)
    assert how == "cyclic"
    assert [[b for b in l if b >= 0] for l in lists] == [D.blocks_of(k, world, H, rows) for k in range(world)]
    assert len({len(l) for l in lists}) == 1  # equal-length lists (pads)
    skew = np.where(np.arange(nb) % world == 0, 50.0, 1.0)  # cyclic rows put every heavy block on rank 0
    priced = D.balanced_blocks(skew, world)
    lists, how = D.choose_lists(priced, skew, world, H, rows)
    assert how == "priced" and lists == priced
    assert D.max_over_mean(priced, skew) < D.max_over_mean(
        [D.blocks_of(k, world, H, rows) for k in range(world)], skew) / (1 + D.REPRICE_MARGIN)
