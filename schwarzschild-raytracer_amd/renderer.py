"""GPU renderer: a thin Python handle over the C-ABI (libsr.so).

PyTorch only provides device memory and the HIP stream; every pixel is
computed by the gfx950 kernel in libsr.so. There is no CPU fallback: without a
HIP device `Renderer()` raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class Renderer:
    """One sr_ctx bound to one HIP device (the reference's single GL program)."""

    def __init__(self, device: int = 0, lib=None):
        """lib: a loaded library (abi.load(path)) other than the package's
        libsr.so, e.g. the test-only 7-wave build (tests/test_gpu_allocation.py)."""
        import torch

        self.torch = torch
        self.lib = lib if lib is not None else abi.load()
        self.device = int(device)
        self.tdev = torch.device("cuda", self.device)
        ctx = C.c_void_p()
        abi.check(self.lib.sr_create(C.byref(ctx), self.device), "sr_create")
        self.ctx = ctx
        self._keep = []

    # ---- uploads (src/main.cpp:205-274 equivalents) ----------------------------
    def set_scene(self, scene: abi.Scene) -> None:
        abi.check(self.lib.sr_set_scene(self.ctx, C.byref(scene)), "sr_set_scene")

    def set_test_ray(self, test_ray: abi.TestRay) -> None:
        abi.check(self.lib.sr_set_test_ray(self.ctx, C.byref(test_ray)), "sr_set_test_ray")

    def set_background(self, img: np.ndarray) -> None:
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w, ch = img.shape
        abi.check(self.lib.sr_set_background(self.ctx, img.ctypes.data, w, h, ch), "sr_set_background")

    def set_texture_array(self, arr: np.ndarray) -> None:
        arr = np.ascontiguousarray(arr, dtype=np.uint8)
        layers, h, w, ch = arr.shape
        abi.check(self.lib.sr_set_texture_array(self.ctx, arr.ctypes.data, w, h, layers, ch), "sr_set_texture_array")

    def set_culling(self, enabled: bool) -> None:
        abi.check(self.lib.sr_debug_set_culling(self.ctx, 1 if enabled else 0), "sr_debug_set_culling")

    def set_split(self, max_tiles: int, lanes_per_wave: int = 16, min_steps: int = 1) -> None:
        """Run the costliest tiles of the previous frame as sparse waves (sr_set_split; 0 tiles: off)."""
        abi.check(self.lib.sr_set_split(self.ctx, int(max_tiles), int(lanes_per_wave), int(min_steps)), "sr_set_split")

    # ---- rendering -------------------------------------------------------------
    def set_latency_mode(self, on: bool) -> None:
        """sr_set_latency_mode: a 2-step fast loop for one frame at a time (pixels unchanged)."""
        abi.check(self.lib.sr_set_latency_mode(self.ctx, 1 if on else 0), "sr_set_latency_mode")

    def set_timing(self, capacity: int) -> None:
        """Record per-kernel HIP events for the next `capacity` frames (0: off)."""
        abi.check(self.lib.sr_debug_set_timing(self.ctx, int(capacity)), "sr_debug_set_timing")

    def kernel_times(self, max_frames: int = 4096) -> np.ndarray:
        """[frames, 3] ms of (integrate, shade, resume) for the recorded frames."""
        buf = (C.c_float * (3 * max_frames))()
        n = C.c_int()
        abi.check(self.lib.sr_debug_kernel_times(self.ctx, buf, max_frames, C.byref(n)), "sr_debug_kernel_times")
        k = min(n.value, max_frames)
        return np.frombuffer(buf, dtype=np.float32, count=3 * k).reshape(k, 3).copy()

    def diag_counters(self) -> dict:
        """sr_diag_counters after this context's frames: opaque-classified hits
        whose shaded alpha was not 1 (must stay 0) and failed stream-ordered frees."""
        buf = (C.c_int64 * 2)()
        abi.check(self.lib.sr_diag_counters(self.ctx, buf, 2), "sr_diag_counters")
        return {"hit_not_opaque": int(buf[0]), "free_errors": int(buf[1])}

    def last_order(self) -> np.ndarray:
        """The launch codes the last frame left for the next one (tile << 8, | 0x80 | sub when split, -1 unused)."""
        n = C.c_int()
        abi.check(self.lib.sr_debug_last_order(self.ctx, None, 0, C.byref(n)), "sr_debug_last_order")
        buf = (C.c_int * max(1, n.value))()
        abi.check(self.lib.sr_debug_last_order(self.ctx, buf, n.value, C.byref(n)), "sr_debug_last_order")
        return np.frombuffer(buf, dtype=np.int32, count=n.value).copy()

    def pixel_state(self) -> np.ndarray:
        """The integrate -> shade hand-off after the last frame (post-mortems):
        float32 [SR_PS_FIELDS * n] in geodesic.hip's PS layout, n pixel ids."""
        n = C.c_size_t()
        abi.check(self.lib.sr_debug_pixel_state(self.ctx, None, 0, C.byref(n)), "sr_debug_pixel_state")
        buf = np.empty(max(1, n.value * abi.PS_FIELDS), dtype=np.float32)
        abi.check(self.lib.sr_debug_pixel_state(self.ctx, buf.ctypes.data_as(C.POINTER(C.c_float)),
                                                n.value * abi.PS_FIELDS, C.byref(n)), "sr_debug_pixel_state")
        return buf[:n.value * abi.PS_FIELDS]

    def _stream(self, stream):
        if stream is None:
            stream = self.torch.cuda.current_stream(self.tdev)
        return C.c_void_p(stream.cuda_stream)

    def render(self, cam: abi.Camera, params: abi.Params, width: int, height: int, row_begin: int = 0,
               row_end: int | None = None, out=None, stream=None):
        """RGBA8 rows [row_begin, row_end) (GL order, row 0 = bottom) into a
        uint8 tensor [rows, width, 4] on this device. Asynchronous."""
        row_end = height if row_end is None else row_end
        rows = row_end - row_begin
        if out is None:
            out = self.torch.empty((max(rows, 0), width, 4), dtype=self.torch.uint8, device=self.tdev)
        assert out.is_contiguous() and out.dtype == self.torch.uint8 and out.numel() >= rows * width * 4
        abi.check(
            self.lib.sr_render(self.ctx, C.byref(cam), C.byref(params), width, height, row_begin, row_end,
                               C.c_void_p(out.data_ptr()), width * 4, self._stream(stream)),
            "sr_render",
        )
        return out

    def render_blocks(self, cam: abi.Camera, params: abi.Params, width: int, height: int, block_rows: int,
                      block_first: int, block_step: int, out=None, stream=None):
        """Block-cyclic row bands (multi-GPU tiling), packed densely."""
        rows = self.lib.sr_blocks_row_count(height, block_rows, block_first, block_step)
        nblocks = -(-rows // block_rows) if rows else 0
        cap = nblocks * block_rows
        if out is None:
            out = self.torch.empty((cap, width, 4), dtype=self.torch.uint8, device=self.tdev)
        assert out.is_contiguous() and out.numel() >= cap * width * 4
        abi.check(
            self.lib.sr_render_blocks(self.ctx, C.byref(cam), C.byref(params), width, height, block_rows,
                                      block_first, block_step, C.c_void_p(out.data_ptr()), width * 4,
                                      self._stream(stream)),
            "sr_render_blocks",
        )
        return out, rows

    def render_blocks_batch(self, cams, params: abi.Params, width: int, height: int, block_rows: int,
                            block_first: int, block_step: int, out=None, stream=None):
        """sr_render_blocks' rows of len(cams) frames in one launch -> ([B, tile_rows, W, 4], rows)."""
        rows = self.lib.sr_blocks_row_count(height, block_rows, block_first, block_step)
        nblocks = -(-rows // block_rows) if rows else 0
        cap = nblocks * block_rows
        B = len(cams)
        arr = (abi.Camera * B)(*cams)
        if out is None:
            out = self.torch.empty((B, cap, width, 4), dtype=self.torch.uint8, device=self.tdev)
        assert out.is_contiguous() and out.dtype == self.torch.uint8 and tuple(out.shape[:1]) == (B,)
        assert out[0].numel() >= cap * width * 4
        abi.check(
            self.lib.sr_render_blocks_batch(self.ctx, arr, B, C.byref(params), width, height, block_rows, block_first,
                                            block_step, C.c_void_p(out.data_ptr()), width * 4,
                                            out[0].numel(), self._stream(stream)),
            "sr_render_blocks_batch",
        )
        return out, rows

    def wave_costs(self, cam: abi.Camera, params: abi.Params, width: int, height: int, stream=None):
        """sr_wave_costs: int32 [ceil(H / 8), ceil(W / 8), 2] per 8x8 wave tile of
        the frame: {longest ray's steps, budget events}. Asynchronous."""
        out = self.torch.zeros(((height + 7) // 8, (width + 7) // 8, 2), dtype=self.torch.int32, device=self.tdev)
        abi.check(self.lib.sr_wave_costs(self.ctx, C.byref(cam), C.byref(params), width, height,
                                         C.c_void_p(out.data_ptr()), self._stream(stream)), "sr_wave_costs")
        return out

    def render_block_list(self, cams, params: abi.Params, width: int, height: int, block_rows: int, blocks,
                          out=None, stream=None):
        """Rows of an explicit block list (sr_render_block_list; -1 = padding)
        for len(cams) frames in one launch -> [B, len(blocks) * block_rows, W, 4]."""
        blocks = [int(b) for b in blocks]
        B = len(cams)
        arr = (abi.Camera * B)(*cams)
        lst = (C.c_int * len(blocks))(*blocks)
        rows = len(blocks) * block_rows
        if out is None:
            out = self.torch.empty((B, rows, width, 4), dtype=self.torch.uint8, device=self.tdev)
        assert out.is_contiguous() and out.dtype == self.torch.uint8 and tuple(out.shape[:1]) == (B,)
        assert out[0].numel() >= rows * width * 4
        abi.check(
            self.lib.sr_render_block_list(self.ctx, arr, B, C.byref(params), width, height, block_rows, lst,
                                          len(blocks), C.c_void_p(out.data_ptr()), width * 4, out[0].numel(),
                                          self._stream(stream)),
            "sr_render_block_list",
        )
        return out

    def render_debug(self, cam: abi.Camera, params: abi.Params, width: int, height: int, row_begin: int = 0,
                     row_end: int | None = None, stream=None):
        """(float RGBA FragColor, RGBA8, executed steps) for rows [row_begin, row_end)."""
        t = self.torch
        row_end = height if row_end is None else row_end
        rows = row_end - row_begin
        f = t.empty((rows, width, 4), dtype=t.float32, device=self.tdev)
        b = t.empty((rows, width, 4), dtype=t.uint8, device=self.tdev)
        s = t.empty((rows, width), dtype=t.int32, device=self.tdev)
        abi.check(
            self.lib.sr_render_debug(self.ctx, C.byref(cam), C.byref(params), width, height, row_begin, row_end,
                                     C.c_void_p(f.data_ptr()), C.c_void_p(b.data_ptr()), C.c_void_p(s.data_ptr()),
                                     self._stream(stream)),
            "sr_render_debug",
        )
        return f, b, s

    def close(self) -> None:
        if self.ctx:
            self.lib.sr_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
