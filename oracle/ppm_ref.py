"""ORACLE TEST INFRASTRUCTURE — ctypes view of oracle/libppm_ref.so (CPU restatement of the
reference's photon-mapping path, see oracle/ppm_ref.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as
the checker / CPU baseline.  The product (ceng795_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class PPMStats(C.Structure):
    _fields_ = [("photons", C.c_longlong), ("photon_rays", C.c_longlong),
                ("deposits", C.c_longlong), ("updates", C.c_longlong),
                ("eye_rays", C.c_longlong), ("hit_points", C.c_longlong)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libppm_ref.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        vp, i, ip = C.c_void_p, C.c_int, C.POINTER(C.c_int)
        L.ppmref_load.restype = vp
        L.ppmref_load.argtypes = [C.c_char_p, C.c_char_p, i]
        L.ppmref_free.argtypes = [vp]
        L.ppmref_num_cameras.argtypes = [vp]
        L.ppmref_camera_info.argtypes = [vp, i, ip, ip, ip]
        L.ppmref_settings.argtypes = [vp, ip, ip, ip]
        L.ppmref_eye_pass.argtypes = [vp, i, C.c_ulonglong, C.POINTER(PPMStats)]
        L.ppmref_build_hash_grid.argtypes = [vp, i, i, C.POINTER(C.c_double)]
        L.ppmref_num_hit_points.argtypes = [vp]
        L.ppmref_hit_points.argtypes = [vp, vp]
        L.ppmref_hit_state.argtypes = [vp, vp]
        L.ppmref_trace_photons.argtypes = [vp, C.c_ulonglong, C.c_longlong, C.c_longlong,
                                           C.POINTER(PPMStats)]
        L.ppmref_density.argtypes = [vp, C.c_longlong, vp]
        L.ppmref_render.argtypes = [vp, i, C.c_ulonglong, i, vp, C.POINTER(PPMStats)]
        for f in ("sinf", "cosf", "asinf"):
            getattr(L, "ppmref_" + f).restype = C.c_float
            getattr(L, "ppmref_" + f).argtypes = [C.c_float]
        L.ppmref_powf.restype = C.c_float
        L.ppmref_powf.argtypes = [C.c_float, C.c_float]
        _LIB = L
    return _LIB


class OraclePPM:
    """CPU restatement of the PPM Scene (PPM/include/Scene.h)."""

    def __init__(self, xml_path: str):
        err = C.create_string_buffer(512)
        h = lib().ppmref_load(xml_path.encode(), err, 512)
        if not h:
            raise RuntimeError(err.value.decode())
        self._h = h

    def close(self):
        if self._h:
            lib().ppmref_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def camera(self, cam=0):
        w, h, n = C.c_int(), C.c_int(), C.c_int()
        if lib().ppmref_camera_info(self._h, cam, C.byref(w), C.byref(h), C.byref(n)):
            raise IndexError(cam)
        return w.value, h.value, n.value

    def settings(self):
        p, it, d = C.c_int(), C.c_int(), C.c_int()
        lib().ppmref_settings(self._h, C.byref(p), C.byref(it), C.byref(d))
        return p.value, it.value, d.value

    def eye_pass(self, cam=0, seed=0):
        st = PPMStats()
        if lib().ppmref_eye_pass(self._h, cam, seed, C.byref(st)):
            raise RuntimeError("eye pass failed")
        return st

    def build_hash_grid(self, width, height):
        info = (C.c_double * 8)()
        lib().ppmref_build_hash_grid(self._h, width, height, info)
        return list(info)

    def hit_points(self) -> np.ndarray:
        n = lib().ppmref_num_hit_points(self._h)
        out = np.zeros((n, 16), np.float32)
        lib().ppmref_hit_points(self._h, out.ctypes.data)
        return out

    def hit_state(self) -> np.ndarray:
        n = lib().ppmref_num_hit_points(self._h)
        out = np.zeros((n, 5), np.float32)
        lib().ppmref_hit_state(self._h, out.ctypes.data)
        return out

    def trace_photons(self, seed, first, count):
        st = PPMStats()
        if lib().ppmref_trace_photons(self._h, seed, first, count, C.byref(st)):
            raise RuntimeError("photon pass failed")
        return st

    def density(self, total, cam=0):
        w, h, _ = self.camera(cam)
        out = np.zeros((h, w, 3), np.float32)
        if lib().ppmref_density(self._h, total, out.ctypes.data):
            raise RuntimeError("density estimation failed")
        return out

    def render(self, cam=0, seed=0, threads=8):
        w, h, _ = self.camera(cam)
        out = np.zeros((h, w, 3), np.float32)
        st = PPMStats()
        if lib().ppmref_render(self._h, cam, seed, threads, out.ctypes.data, C.byref(st)):
            raise RuntimeError("render failed")
        return out, st
