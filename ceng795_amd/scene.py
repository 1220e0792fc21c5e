"""Scene: the reference's Scene interface (HW2/Scene.h) over the C ABI."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import check, lib

# rt_render_device tile_major flags (include/ceng795_rt.h)
RT_TILE_MAJOR, RT_TILE_BLOCKS, RT_TILE_RECORDS = 1, 2, 4
RT_UNTILE_BLOCKS, RT_UNTILE_SKIP_ROOT = 1, 2  # rt_untile_device flags


@dataclass
class CameraInfo:
    width: int
    height: int
    num_samples: int
    image_name: str
    e: tuple
    top_left: tuple
    s_u: tuple
    s_v: tuple


class Scene:
    """HW2 ``Scene``: parse an XML scene and render its cameras on the GPU.

    ``render_image(camera_index, result, starting_row, height_increase)`` has the reference's
    argument meaning (HW2/Scene.cpp:16-31): rows ``starting_row + k*height_increase`` of
    ``result`` (an ``(h, w, 3)`` float32 array standing for ``Pixel[w*h]``) receive the fp32
    radiance ``Pixel::color``; other rows are untouched.  Errors raise ``RTError`` (the
    reference throws ``std::runtime_error`` from the loader, HW2/Scene.cpp:204,208).

    ``devices`` (a list of GPU ordinals) makes one scene over several GPUs of this process
    (rt_scene_load_xml_multi): every frame's tiles are dealt over them and gathered onto
    ``devices[0]`` with RCCL.
    """

    def __init__(self, file_name: str, device: int = -1, traversal: str = "fast",
                 devices: Optional[list] = None):
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devices))(*devices)
            check(lib().rt_scene_load_xml_multi(str(file_name).encode(), len(devices), arr,
                                                C.byref(h)))
        else:
            check(lib().rt_scene_load_xml(str(file_name).encode(), device, C.byref(h)))
        self._h = h
        self.set_traversal(traversal)

    @classmethod
    def _from_handle(cls, h: C.c_void_p) -> "Scene":
        s = cls.__new__(cls)
        s._h = h
        return s

    # ------------------------------------------------------------------ lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().rt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------------ queries
    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def num_cameras(self) -> int:
        return lib().rt_scene_num_cameras(self._h)

    @property
    def num_lights(self) -> int:
        return lib().rt_scene_num_lights(self._h)

    @property
    def device_count(self) -> int:
        return lib().rt_scene_device_count(self._h)

    @property
    def bvh_depth(self) -> int:
        return lib().rt_scene_bvh_depth(self._h)

    def camera(self, i: int) -> CameraInfo:
        c = _lib.rt_camera()
        check(lib().rt_scene_camera(self._h, i, C.byref(c)))
        name = lib().rt_scene_image_name(self._h, i).decode()
        return CameraInfo(c.width, c.height, c.num_samples, name, tuple(c.e),
                          tuple(c.top_left), tuple(c.s_u), tuple(c.s_v))

    def set_traversal(self, mode: str) -> None:
        m = {"fast": _lib.RT_TRAVERSAL_FAST, "reference": _lib.RT_TRAVERSAL_REFERENCE}[mode]
        check(lib().rt_set_traversal(self._h, m))

    def set_msaa_seed(self, seed: int) -> None:
        """Seed of the per-pixel MSAA generators (the reference uses the wall clock)."""
        check(lib().rt_set_msaa_seed(self._h, int(seed)))

    def dump_bvh(self, path: str) -> None:
        check(lib().rt_scene_dump_bvh(self._h, str(path).encode()))

    # ------------------------------------------------------------------ rendering
    def new_image(self, camera_index: int) -> np.ndarray:
        c = self.camera(camera_index)
        return np.zeros((c.height, c.width, 3), np.float32)

    def render_image(self, camera_index: int, result: Optional[np.ndarray] = None,
                     starting_row: int = 0, height_increase: int = 1):
        """Scene::render_image (HW2/Scene.h:34-35).  Returns (result, rt_stats).

        NumSamples > 1: whole frames only; result is Pixel::color / Pixel::weight."""
        if result is None:
            result = self.new_image(camera_index)
        c = self.camera(camera_index)
        if result.dtype != np.float32 or not result.flags.c_contiguous or \
                result.size != c.width * c.height * 3:
            raise ValueError("result must be a C-contiguous float32 array of h*w*3 values")
        st = _lib.rt_stats()
        check(lib().rt_render(self._h, camera_index, starting_row, height_increase,
                              result.ctypes.data, C.byref(st)))
        return result, st

    def num_tiles(self, camera_index: int, starting_row: int = 0, row_stride: int = 1) -> int:
        return check(lib().rt_num_tiles(self._h, camera_index, starting_row, row_stride))

    def render_device(self, camera_index: int, out_ptr: int, *, starting_row: int = 0,
                      row_stride: int = 1, tile_begin: int = 0, tile_step: int = 1,
                      tile_major: bool = False, blocks: bool = False, stream: int = 0,
                      tile_count: int = -1, records: bool = False) -> None:
        """Asynchronous render into device memory at ``out_ptr`` on HIP stream ``stream``
        (deal units tile_begin + k*tile_step, k < tile_count; tile_count < 0: all of them; a
        unit is a tile, or with ``blocks`` a 2x2 block of tiles in deal order —
        RT_TILE_BLOCKS of include/ceng795_rt.h).  ``records`` (with ``tile_major``): 64
        32-bit pixel records per tile instead of RGB (RT_TILE_RECORDS)."""
        flags = ((RT_TILE_MAJOR if tile_major else 0) | (RT_TILE_BLOCKS if blocks else 0) |
                 (RT_TILE_RECORDS if records else 0))
        check(lib().rt_render_device_range(self._h, camera_index, starting_row, row_stride,
                                           tile_begin, tile_step, tile_count, flags,
                                           C.c_void_p(out_ptr), C.c_void_p(stream)))

    def untile_device(self, camera_index: int, devices: int, slot: int, gathered_ptr: int,
                      out_ptr: int, *, tile_offset: int = 0, blocks: bool = False,
                      skip_root: bool = False, stream: int = 0) -> None:
        """rt_untile_device: the gathered [devices][slot][64][3] tile shares of a round-robin
        deal (unit u to rank (u + tile_offset) mod devices; units are tiles, or 2x2 blocks in
        deal order with ``blocks``) into the row-major frame; ``skip_root``: rank 0's units
        are left as they are (rendered in place)."""
        flags = (RT_UNTILE_BLOCKS if blocks else 0) | (RT_UNTILE_SKIP_ROOT if skip_root else 0)
        check(lib().rt_untile_device(self._h, camera_index, 0, 1, devices, slot, tile_offset,
                                     flags, C.c_void_p(gathered_ptr), C.c_void_p(out_ptr),
                                     C.c_void_p(stream)))

    def tile_costs(self, stream: int, capacity: int) -> "np.ndarray":
        """rt_tile_costs: every tile's measured time (100 MHz ticks) in the last frame enqueued on
        HIP stream ``stream``, in that call's selection order (waits for the stream)."""
        out = np.zeros(max(1, capacity), dtype=np.uint32)
        n = check(lib().rt_tile_costs(self._h, C.c_void_p(stream),
                                      out.ctypes.data_as(C.c_void_p), capacity))
        return out[:n]

    def resolve_rows(self, camera_index: int, row_begin: int, row_end: int, records_ptr: int,
                     out_ptr: int, *, stream: int = 0) -> None:
        """rt_resolve_rows: row-major pixel records (one 32-bit word per pixel of the frame)
        shaded into rows [row_begin, row_end) of the row-major frame at ``out_ptr``."""
        check(lib().rt_resolve_rows(self._h, camera_index, row_begin, row_end,
                                    C.c_void_p(records_ptr), C.c_void_p(out_ptr),
                                    C.c_void_p(stream)))

    def records_ok(self, camera_index: int) -> bool:
        """rt_scene_records_ok: may this camera's shares travel as pixel records?"""
        return bool(check(lib().rt_scene_records_ok(self._h, camera_index)))

    def resolve_device(self, camera_index: int, devices: int, slot: int, gathered_ptr: int,
                       out_ptr: int, *, tile_offset: int = 0, blocks: bool = False,
                       skip_root: bool = False, stream: int = 0) -> None:
        """rt_resolve_device: gathered pixel records [devices][slot][64] (RT_TILE_RECORDS
        shares) shaded into the row-major frame (the layout and flags of untile_device)."""
        flags = (RT_UNTILE_BLOCKS if blocks else 0) | (RT_UNTILE_SKIP_ROOT if skip_root else 0)
        check(lib().rt_resolve_device(self._h, camera_index, 0, 1, devices, slot, tile_offset,
                                      flags, C.c_void_p(gathered_ptr), C.c_void_p(out_ptr),
                                      C.c_void_p(stream)))

    def release_stream(self, stream: int) -> None:
        """Frees the scratch the library keeps for HIP stream ``stream`` (after waiting for it)."""
        check(lib().rt_release_stream_scratch(self._h, C.c_void_p(stream)))

    def set_kernel_timing(self, enable: bool) -> None:
        check(lib().rt_set_kernel_timing(self._h, int(enable)))

    def read_kernel_times(self):
        """(ms summed {frame kernel, order kernel, other, total}, launches) since the last read."""
        ms = (C.c_double * 4)()
        n = C.c_longlong()
        check(lib().rt_read_kernel_times(self._h, ms, C.byref(n)))
        keys = ("frame", "order", "other", "total")
        return dict(zip(keys, list(ms))), n.value

    DIAG_NAMES = ["primary_rays", "shadow_rays", "secondary_rays", "primary_hits",
                  "prim_node_visits", "prim_node_lanes", "prim_leaf_visits", "prim_leaf_lanes",
                  "shad_node_visits", "shad_node_lanes", "shad_leaf_visits", "shad_leaf_lanes",
                  "exact_box_fallbacks", "guard_tests", "prim_wide_visits",
                  "shad_wide_visits"]

    def debug_counters(self) -> dict:
        """All device counters (diagnostic columns only in the CENG795_LIB=diag build)."""
        arr = (C.c_longlong * 16)()
        diag = check(lib().rt_debug_counters(self._h, arr))
        d = dict(zip(self.DIAG_NAMES, list(arr)))
        d["diag_build"] = bool(diag)
        return d

    def collect_stats(self) -> "_lib.rt_stats":
        st = _lib.rt_stats()
        check(lib().rt_collect_stats(self._h, C.byref(st)))
        return st


def write_png(path: str, rgb: np.ndarray) -> None:
    """HW2/main.cpp:43-57: clamp(int(c), 0, 255) per channel."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    check(lib().rt_write_png(str(path).encode(), rgb.ctypes.data, w, h))


def host_dump_bvh(xml_path: str, out_path: str) -> None:
    """Host-only: parse + build + flatten the BVH and dump it (no GPU needed)."""
    check(lib().rt_host_dump_bvh_xml(str(xml_path).encode(), str(out_path).encode()))
