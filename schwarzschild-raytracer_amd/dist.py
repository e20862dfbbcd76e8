"""Row-band tiling of one frame over the ranks of a node and the gather of the
tiles to rank 0. One process per GPU; torch.distributed with
backend "nccl" is RCCL over xGMI on ROCm ("gloo" for CPU tests).

Partition: the frame's rows are cut into blocks of `block_rows`; block b goes
to rank b % world (block-cyclic). Rows through the photon ring cost ~2x the
edge rows, so contiguous bands are imbalanced (max/mean 1.14 at 8 ranks);
interleaving 8-row blocks keeps every rank within a few % of the mean while
each 8-row block still maps onto whole 8x8 wave tiles.

Cost-balanced lists (balanced_blocks): the same 8-row blocks, assigned from
a per-wave cost map of the frame (sr_wave_costs: each 8x8 wave's longest
ray's steps and its budget events; block_costs) so that every rank gets the
same number of blocks and about the same cost (sr_render_block_list renders
a list). Block-cyclic rows leave the slowest of 8 ranks 3.6 % above the mean
(profiles/r02/s9_*); balancing on steps alone missed the events (a share's
time fits steps + ~8 x events, profiles/r02/s15_*).

Exchange: every rank packs its blocks densely into an equal-size tile
(padded to the largest share; sr_render_blocks writes exactly that layout)
and one `gather` brings all tiles to rank 0 into one [world, tile_rows, W, 4]
buffer. Because block b = k*world + rank sits at slot (rank, k), the frame is
that buffer transposed to (k, rank) — a single device copy. With RCCL each
peer's tile travels over its own xGMI link into rank 0.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def nblocks(height: int, block_rows: int) -> int:
    return (height + block_rows - 1) // block_rows


def blocks_of(rank: int, world: int, height: int, block_rows: int) -> list[int]:
    return list(range(rank, nblocks(height, block_rows), world))


def rows_of(rank: int, world: int, height: int, block_rows: int) -> list[int]:
    rows = []
    for b in blocks_of(rank, world, height, block_rows):
        rows.extend(range(b * block_rows, min(height, (b + 1) * block_rows)))
    return rows


def tile_rows(world: int, height: int, block_rows: int) -> int:
    """Rows of the equal-size tile every rank contributes to the gather."""
    return ((nblocks(height, block_rows) + world - 1) // world) * block_rows


def wave_costs(steps, block_rows: int = 8, wave: int = 8):
    """Per-block cost from a [H, W] map of executed steps: the sum over the
    block's wave tiles (block_rows x wave pixels) of their longest ray's steps
    (a wave runs until its last lane is done). numpy or torch -> numpy float64."""
    s = steps.cpu().numpy() if hasattr(steps, "cpu") else np.asarray(steps)
    H, W = s.shape
    hb, wb = nblocks(H, block_rows), (W + wave - 1) // wave
    pad = np.zeros((hb * block_rows, wb * wave), dtype=np.int64)
    pad[:H, :W] = s
    return pad.reshape(hb, block_rows, wb, wave).max(axis=(1, 3)).sum(axis=1).astype(np.float64)


EVENT_STEPS = 8.0  # one budget event costs about as much as this many wave steps (profiles/r02/s15_*)


def block_costs_py(wave_cost, event_steps: float = EVENT_STEPS):
    """Per 8-row block cost from sr_wave_costs' [rows / 8, cols / 8, 2] map:
    the sum over the block's waves of steps + event_steps x events (the
    statement of the rule; block_costs runs the library's sr_block_costs)."""
    w = wave_cost.cpu().numpy() if hasattr(wave_cost, "cpu") else np.asarray(wave_cost)
    w = w.astype(np.float64)
    return (w[..., 0] + event_steps * w[..., 1]).sum(axis=1)


def block_costs(wave_cost, event_steps: float = EVENT_STEPS):
    """block_costs_py through the C-ABI (sr_block_costs, csrc/host/partition.cpp):
    the C++ a multi-GPU caller of libsr uses."""
    w = wave_cost.cpu().numpy() if hasattr(wave_cost, "cpu") else np.asarray(wave_cost)
    w = np.ascontiguousarray(w, dtype=np.int32)
    nb, nc = w.shape[0], w.shape[1]
    out = np.zeros(nb, dtype=np.float64)
    abi.check(abi.load().sr_block_costs(w.ctypes.data, nb, nc, float(event_steps), out.ctypes.data), "sr_block_costs")
    return out


def balanced_blocks(costs, world: int) -> list[list[int]]:
    """balanced_blocks_py through the C-ABI (sr_balanced_blocks,
    csrc/host/partition.cpp): the same lists, computed by the library."""
    c = np.ascontiguousarray(np.asarray(costs, dtype=np.float64))
    nb = int(c.shape[0])
    per = (nb + world - 1) // world
    out = np.empty(max(1, world * per), dtype=np.int32)
    got = C.c_int()
    abi.check(abi.load().sr_balanced_blocks(c.ctypes.data, nb, int(world), out.ctypes.data, int(out.size),
                                            C.byref(got)), "sr_balanced_blocks")
    assert got.value == per
    return [[int(b) for b in out[r * per:(r + 1) * per]] for r in range(world)]


def balanced_blocks_py(costs, world: int) -> list[list[int]]:
    """Equal-length block lists (padded with -1) of about equal total cost:
    blocks by descending cost, each to the rank with the least cost so far
    among those with room (ties: lowest rank), then pairwise swaps (a pad
    counts as a block of cost 0) that lower the most loaded rank's cost. The
    block-cyclic lists are returned instead when they are at least as even.
    Deterministic: every rank computes the same lists from the same costs."""
    costs = [float(c) for c in costs]
    nb = len(costs)
    per = (nb + world - 1) // world
    cost = lambda b: costs[b] if b >= 0 else 0.0  # noqa: E731
    load = [0.0] * world
    lists: list[list[int]] = [[] for _ in range(world)]
    for b in sorted(range(nb), key=lambda i: (-costs[i], i)):
        r = min((k for k in range(world) if len(lists[k]) < per), key=lambda k: (load[k], k))
        lists[r].append(b)
        load[r] += costs[b]
    for l in lists:
        l.extend([-1] * (per - len(l)))
    for _ in range(4 * nb):  # swaps out of the most loaded rank while one lowers the pair's maximum
        hi = max(range(world), key=lambda k: (load[k], -k))
        best = None
        for r in range(world):
            if r == hi:
                continue
            for i, a in enumerate(lists[hi]):
                for j, b in enumerate(lists[r]):
                    d = cost(a) - cost(b)
                    if d <= 0:
                        continue
                    m = max(load[hi] - d, load[r] + d)
                    if m < load[hi] - 1e-9 and (best is None or m < best[0]):
                        best = (m, r, i, j, d)
        if best is None:
            break
        _, r, i, j, d = best
        lists[hi][i], lists[r][j] = lists[r][j], lists[hi][i]
        load[hi] -= d
        load[r] += d
    cyc = [[b for b in range(k, nb, world)] for k in range(world)]
    cyc = [l + [-1] * (per - len(l)) for l in cyc]
    cyc_max = max(sum(cost(b) for b in l) for l in cyc)
    if cyc_max <= max(load):
        return cyc
    return [sorted(b for b in l if b >= 0) + [-1] * l.count(-1) for l in lists]


def rows_of_list(blocks, height: int, block_rows: int) -> list[int]:
    rows = []
    for b in blocks:
        if b >= 0:
            rows.extend(range(b * block_rows, min(height, (b + 1) * block_rows)))
    return rows


def list_sources(lists, height: int, block_rows: int):
    """Frame block b -> its slot r * per + s in the stacked tiles (lists[r][s] == b)."""
    per = len(lists[0])
    nb = nblocks(height, block_rows)
    src = np.full(nb, -1, dtype=np.int64)
    for r, l in enumerate(lists):
        for s_, b in enumerate(l):
            if b >= 0:
                src[b] = r * per + s_
    assert (src >= 0).all(), "every block of the frame must be on some rank"
    return src


def assemble_lists(stacked, lists, height: int, block_rows: int, src=None):
    """Gathered tiles of sr_render_block_list ranks -> frames: [world, tile_rows,
    W, C] -> [height, W, C], or [world, B, tile_rows, W, C] -> [B, height, W, C];
    frame block b is slot s of rank r where lists[r][s] == b. src: list_sources
    (for torch, a tensor on the tiles' device: no host copy per call)."""
    world, per = len(lists), len(lists[0])
    nb = nblocks(height, block_rows)
    if src is None:
        src = list_sources(lists, height, block_rows)
    batched = stacked.ndim == 5
    rest = tuple(stacked.shape[3 if batched else 2:])
    if isinstance(stacked, np.ndarray):
        if batched:
            v = stacked.reshape((world, stacked.shape[1], per, block_rows) + rest).swapaxes(0, 1)
            v = v.reshape((stacked.shape[1], world * per, block_rows) + rest)[:, src]
            return np.ascontiguousarray(v.reshape((stacked.shape[1], nb * block_rows) + rest)[:, :height])
        v = stacked.reshape((world * per, block_rows) + rest)[src]
        return np.ascontiguousarray(v.reshape((nb * block_rows,) + rest)[:height])
    import torch

    idx = src if isinstance(src, torch.Tensor) else torch.as_tensor(src, device=stacked.device)
    if batched:
        B = stacked.shape[1]
        v = stacked.reshape((world, B, per, block_rows) + rest).transpose(0, 1)
        v = v.reshape((B, world * per, block_rows) + rest).index_select(1, idx)
        return v.reshape((B, nb * block_rows) + rest)[:, :height]
    v = stacked.reshape((world * per, block_rows) + rest).index_select(0, idx)
    return v.reshape((nb * block_rows,) + rest)[:height]


def assemble_blocks_abi(stacked, lists, height: int, block_rows: int, out=None, dev_lists=None, stream=None):
    """assemble_lists through the C-ABI (sr_assemble_blocks): gathered tiles
    [world, B, tile_rows, W, C] (or [world, tile_rows, W, C]) -> frames
    [B, height, W, C] (or [height, W, C]). Torch tensors on a device: the
    library's copy kernel on `stream` (dev_lists: the flattened lists as an
    int32 tensor on that device); numpy arrays: the host copy."""
    world, per = len(lists), len(lists[0])
    batched = stacked.ndim == 5
    B = stacked.shape[1] if batched else 1
    tile_rows, W, ch = stacked.shape[-3], stacked.shape[-2], stacked.shape[-1]
    is_torch = type(stacked).__module__.startswith("torch")
    row_bytes = W * ch * (stacked.element_size() if is_torch else stacked.itemsize)
    in_frame = tile_rows * row_bytes
    rank_stride = B * in_frame
    lib = abi.load()
    if is_torch and stacked.device.type == "cuda":
        import torch

        assert stacked.is_contiguous()
        if out is None:
            out = torch.empty((B, height, W, ch), dtype=stacked.dtype, device=stacked.device)
        if dev_lists is None:
            dev_lists = torch.tensor([b for l in lists for b in l], dtype=torch.int32, device=stacked.device)
        s = stream if stream is not None else torch.cuda.current_stream(stacked.device)
        abi.check(lib.sr_assemble_blocks(C.c_void_p(stacked.data_ptr()), rank_stride, in_frame,
                                         C.c_void_p(dev_lists.data_ptr()), world, per, height, block_rows, row_bytes,
                                         C.c_void_p(out.data_ptr()), height * row_bytes, B, 1,
                                         C.c_void_p(s.cuda_stream)), "sr_assemble_blocks")
        return out if batched else out[0]
    a = stacked.numpy() if hasattr(stacked, "numpy") else np.asarray(stacked)
    a = np.ascontiguousarray(a)
    res = np.zeros((B, height, W, ch), dtype=a.dtype) if out is None else out
    flat = np.ascontiguousarray([b for l in lists for b in l], dtype=np.int32)
    abi.check(lib.sr_assemble_blocks(a.ctypes.data, rank_stride, in_frame, flat.ctypes.data, world, per, height,
                                     block_rows, row_bytes, res.ctypes.data, height * row_bytes, B, 0, None),
              "sr_assemble_blocks")
    return res if batched else res[0]


def assemble(stacked, world: int, height: int, block_rows: int):
    """[world, tile_rows, W, C] gathered tiles (rank order) -> [height, W, C]
    frame. numpy arrays or torch tensors. Batched tiles [world, B, tile_rows,
    W, C] -> [B, height, W, C] frames."""
    if stacked.ndim == 5:
        B = stacked.shape[1]
        if isinstance(stacked, np.ndarray):
            return np.stack([assemble(stacked[:, b], world, height, block_rows) for b in range(B)])
        tr, rest = stacked.shape[2], tuple(stacked.shape[3:])
        per = tr // block_rows
        v = stacked.reshape((world, B, per, block_rows) + rest).permute((1, 2, 0, 3) + tuple(range(4, 4 + len(rest))))
        return v.reshape((B, per * world * block_rows) + rest)[:, :height]
    w, tr = stacked.shape[0], stacked.shape[1]
    assert w == world and tr % block_rows == 0
    rest = tuple(stacked.shape[2:])
    per = tr // block_rows
    v = stacked.reshape((world, per, block_rows) + rest)
    if isinstance(v, np.ndarray):
        v = v.transpose((1, 0, 2) + tuple(range(3, v.ndim)))
        return np.ascontiguousarray(v.reshape((per * world * block_rows,) + rest)[:height])
    v = v.permute((1, 0, 2) + tuple(range(3, v.dim())))
    return v.reshape((per * world * block_rows,) + rest)[:height]


def max_over_mean(lists, costs) -> float:
    """The most loaded rank's cost over the mean (pads, -1, cost nothing)."""
    loads = [sum(float(costs[b]) for b in lst if b >= 0) for lst in lists]
    mean = sum(loads) / max(1, len(loads))
    return max(loads) / mean if mean > 0 else 1.0


# Block costs change from frame to frame of a moving camera by more than a
# priced list gains over block-cyclic rows: over the bench's 8-rank flyby,
# lists priced from the full-resolution map of one re-price camera scored
# 1.018-1.031 max/mean on the cameras they were then used for, cyclic rows
# 1.015-1.018 (profiles/r05/s2_reprice_*.jsonl, tools/reprice_eval.py).
REPRICE_MARGIN = 0.02


def choose_lists(priced, costs, world: int, height: int, block_rows: int, margin: float = REPRICE_MARGIN):
    """Lists for the frames after a re-pricing: the newly priced lists only
    when, under the map they were priced from, they beat block-cyclic rows by
    more than `margin` (the map's own drift to the next frames); otherwise the
    cyclic rows. Returns (lists, "priced" | "cyclic")."""
    cyclic = [blocks_of(k, world, height, block_rows) for k in range(world)]
    per = len(priced[0])
    cyc = [c + [-1] * (per - len(c)) for c in cyclic]  # the same equal-length form
    if max_over_mean(priced, costs) * (1.0 + margin) < max_over_mean(cyc, costs):
        return priced, "priced"
    return cyc, "cyclic"


class ListSchedule:
    """The rank lists each launch renders when a moving camera re-prices them
    (bench.py --reprice). Launch j runs on context j % contexts; a launch whose
    first frame starts a new group of `every` launches (first // B % every ==
    0) gets new lists (priced by the caller for its first camera), and every
    context adopts the newest lists at its next launch: its previous launch was
    gathered in launch order, so that launch's render and gather switch
    together."""

    def __init__(self, lists, contexts: int, every: int, frames_per_launch: int):
        self.current = lists
        self.ctx = [lists] * contexts
        self.every = every
        self.B = frames_per_launch
        self.count = 0  # re-pricings so far

    def due(self, first: int) -> bool:
        return bool(self.every) and first > 0 and (first // self.B) % self.every == 0

    def adopt(self, j: int, new=None):
        """(lists for launch j, whether its context switched to them)"""
        if new is not None:
            self.current = new
            self.count += 1
        k = j % len(self.ctx)
        changed = self.ctx[k] is not self.current
        self.ctx[k] = self.current
        return self.current, changed


class FrameGather:
    """Preallocated gather of equal-size tiles to rank 0 (collective). A tile
    of [B, tile_rows, W, C] holds B frames (a batched launch); __call__(n)
    gathers the first n of them and returns the [n, H, W, C] frames.

    On device tiles with block lists the returned frames live in a buffer
    this gather keeps and reuses: the next call overwrites them (clone to
    keep one)."""

    def __init__(self, tile, world: int, rank: int, height: int, block_rows: int, group=None, lists=None):
        self.world, self.rank, self.height, self.block_rows, self.group = world, rank, height, block_rows, group
        self.lists = lists  # balanced_blocks lists (sr_render_block_list tiles), else block-cyclic
        self._src = None  # the lists' block sources on the tiles' device (made once; host tiles)
        self._dev_lists = None  # the flattened lists on the tiles' device (sr_assemble_blocks)
        self._frames = None  # rank 0's reassembled frames (device tiles)
        self.tile = tile
        self.stacked = None
        self.views = None
        if rank == 0 and world > 1:
            self.stacked = tile.new_empty((world,) + tuple(tile.shape))
            self.views = [self.stacked[i] for i in range(world)]
        if lists is not None:
            self.set_lists(lists)  # checks the lists cover the frame (list_sources)

    def set_lists(self, lists):
        """Switch to balanced_blocks lists; their block sources go to the tiles'
        device now, outside any launch."""
        src = list_sources(lists, self.height, self.block_rows)  # asserts the lists cover the frame
        self.lists = lists
        self._src = None
        self._dev_lists = None
        if type(self.tile).__module__.startswith("torch"):
            import torch

            self._src = torch.as_tensor(src, device=self.tile.device)
            if self.tile.device.type == "cuda":
                self._dev_lists = torch.tensor([b for l in lists for b in l], dtype=torch.int32,
                                               device=self.tile.device)

    def __call__(self, n: int | None = None, assemble_frame: bool = True):
        import torch.distributed as dist

        tile, views, stacked = self.tile, self.views, self.stacked
        if n is not None:  # batched tile: its first n frames
            tile = tile[:n]
            views = None if views is None else [v[:n] for v in views]
            stacked = None if stacked is None else stacked[:, :n]
        if self.world == 1:
            stacked = tile[None]
        else:
            dist.gather(tile, views if self.rank == 0 else None, dst=0, group=self.group)
        if self.rank != 0:
            return None
        if not assemble_frame:
            return stacked
        if self.lists is not None:
            if type(stacked).__module__.startswith("torch") and stacked.device.type == "cuda":
                # the library's reassembly kernel on the launch's stream, into
                # this gather's frame buffer (valid until its next call)
                if self._dev_lists is None or self._dev_lists.device != stacked.device:
                    import torch

                    # built once: a per-call host-to-device copy of the lists
                    # would wait for the launch's stream (the whole render)
                    self._dev_lists = torch.tensor([b for l in self.lists for b in l], dtype=torch.int32,
                                                   device=stacked.device)
                nf = stacked.shape[1] if stacked.ndim == 5 else 1
                if self._frames is None or self._frames.shape[0] < nf:
                    self._frames = stacked.new_empty((nf, self.height) + tuple(stacked.shape[-2:]))
                out = assemble_blocks_abi(stacked if stacked.is_contiguous() else stacked.contiguous(), self.lists,
                                          self.height, self.block_rows, out=self._frames[:nf],
                                          dev_lists=self._dev_lists)
                return out
            if self._src is None or self._src.device != stacked.device:
                import torch

                self._src = torch.as_tensor(list_sources(self.lists, self.height, self.block_rows),
                                            device=stacked.device)
            return assemble_lists(stacked, self.lists, self.height, self.block_rows, self._src)
        return assemble(stacked, self.world, self.height, self.block_rows)
