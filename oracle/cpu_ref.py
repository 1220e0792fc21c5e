"""ORACLE TEST INFRASTRUCTURE — ctypes view of oracle/libcpu_ref.so (the CPU restatement).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as
the checker / CPU baseline.  The product (ceng795_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Stats(C.Structure):
    _fields_ = [("primary_rays", C.c_longlong), ("shadow_rays", C.c_longlong),
                ("secondary_rays", C.c_longlong), ("primary_hits", C.c_longlong),
                ("box_tests", C.c_longlong * 3), ("prim_tests", C.c_longlong * 3)]

    def as_dict(self):
        return {"primary_rays": self.primary_rays, "shadow_rays": self.shadow_rays,
                "secondary_rays": self.secondary_rays, "primary_hits": self.primary_hits,
                "box_tests": list(self.box_tests), "prim_tests": list(self.prim_tests)}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcpu_ref.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        L.cpuref_load.restype = C.c_void_p
        L.cpuref_load.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.cpuref_free.argtypes = [C.c_void_p]
        L.cpuref_num_cameras.argtypes = [C.c_void_p]
        L.cpuref_num_lights.argtypes = [C.c_void_p]
        L.cpuref_camera_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                         C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.cpuref_render.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_void_p, C.POINTER(Stats)]
        L.cpuref_render_msaa.argtypes = [C.c_void_p, C.c_int, C.c_ulonglong, C.c_int,
                                         C.c_void_p, C.POINTER(Stats)]
        L.cpuref_minstd_uniform.argtypes = [C.c_ulonglong, C.c_int, C.c_void_p]
        L.cpuref_msaa_seed.argtypes = [C.c_ulonglong, C.c_ulonglong]
        L.cpuref_msaa_seed.restype = C.c_ulonglong
        L.cpuref_dump_bvh.argtypes = [C.c_void_p, C.c_char_p]
        L.cpuref_primary_records.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _LIB = L
    return _LIB


def minstd_uniform(seed: int, count: int) -> np.ndarray:
    """The oracle's restatement of uniform_real_distribution<float>(0,1) over
    std::default_random_engine(seed) (libstdc++)."""
    out = np.zeros(count, np.float32)
    lib().cpuref_minstd_uniform(seed, count, out.ctypes.data)
    return out


@dataclass
class CameraInfo:
    width: int
    height: int
    num_samples: int


class OracleScene:
    """CPU restatement of HW2 Scene (HW2/Scene.h)."""

    def __init__(self, xml_path: str):
        err = C.create_string_buffer(512)
        h = lib().cpuref_load(xml_path.encode(), err, 512)
        if not h:
            raise RuntimeError(err.value.decode())
        self._h = h

    def close(self):
        if self._h:
            lib().cpuref_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_cameras(self) -> int:
        return lib().cpuref_num_cameras(self._h)

    @property
    def num_lights(self) -> int:
        return lib().cpuref_num_lights(self._h)

    def camera(self, i: int) -> CameraInfo:
        w, h, n = C.c_int(), C.c_int(), C.c_int()
        if lib().cpuref_camera_info(self._h, i, C.byref(w), C.byref(h), C.byref(n)):
            raise IndexError(i)
        return CameraInfo(w.value, h.value, n.value)

    def render(self, cam: int = 0, starting_row: int = 0, row_stride: int = 1,
               threads: int = 0, out: np.ndarray | None = None):
        info = self.camera(cam)
        if out is None:
            out = np.zeros((info.height, info.width, 3), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous
        assert out.size == info.width * info.height * 3
        threads = threads or (os.cpu_count() or 1)
        st = Stats()
        rc = lib().cpuref_render(self._h, cam, starting_row, row_stride, threads,
                                 out.ctypes.data, C.byref(st))
        if rc:
            raise RuntimeError(f"cpuref_render failed ({rc})")
        return out, st

    def render_msaa(self, cam: int = 0, seed: int = 0, threads: int = 0):
        info = self.camera(cam)
        out = np.zeros((info.height, info.width, 3), np.float32)
        st = Stats()
        rc = lib().cpuref_render_msaa(self._h, cam, seed, threads or (os.cpu_count() or 1),
                                      out.ctypes.data, C.byref(st))
        if rc:
            raise RuntimeError(f"cpuref_render_msaa failed ({rc})")
        return out, st

    def dump_bvh(self, path: str):
        if lib().cpuref_dump_bvh(self._h, path.encode()):
            raise RuntimeError("dump failed")

    def primary_records(self, cam: int = 0) -> np.ndarray:
        info = self.camera(cam)
        out = np.zeros((info.height, info.width, 8), np.float32)
        lib().cpuref_primary_records(self._h, cam, out.ctypes.data)
        return out
