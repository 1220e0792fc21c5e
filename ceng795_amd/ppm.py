"""Progressive photon mapping (BASELINE config C5) — Python mirror of the reference's PPM
Scene interface (PPM/include/Scene.h:44-56), backed by libceng795_ppm.so
(include/ceng795_ppm.h).  Every pass runs in gfx950 kernels; there is no CPU path.

    scene = PhotonScene("cornell.xml")        # Scene::Scene(file_name)
    scene.reset_hash_grid(); scene.eye_trace_lines(0)
    scene.build_hash_grid(width, height)
    scene.trace_n_photons(n, iterations)      # photons [k, k + n*iterations) of the sequence
    image = scene.density_estimation(total_num_of_photons)
or, the whole of PPM/src/main.cpp for one camera:
    image, stats = scene.render(0, reference_threads=8)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from ._lib import RTError, _share_torch_hip_runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
# CENG795_PPM_LIB=<variant> picks lib/libceng795_ppm_<variant>.so (timing experiments only)
_VARIANT = os.environ.get("CENG795_PPM_LIB", "")
LIB_PATH = os.path.join(_HERE, "lib", f"libceng795_ppm_{_VARIANT}.so" if _VARIANT else
                        "libceng795_ppm.so")
ABI_VERSION = 6  # CENG795_PPM_ABI_VERSION

_lib = None


class ppm_stats(C.Structure):
    _fields_ = [("photons", C.c_longlong), ("photon_rays", C.c_longlong),
                ("deposits", C.c_longlong), ("updates", C.c_longlong),
                ("eye_rays", C.c_longlong), ("hit_points", C.c_longlong),
                ("eye_ms", C.c_double), ("grid_ms", C.c_double), ("photon_ms", C.c_double),
                ("density_ms", C.c_double), ("update_deposit_visits", C.c_longlong),
                ("update_candidates", C.c_longlong), ("update_launches", C.c_longlong),
                ("update_ms", C.c_double), ("update_compacted_segments", C.c_longlong),
                ("update_compaction_fallbacks", C.c_longlong),
                ("update_compacted_deposits", C.c_longlong)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_VP, _I, _IP = C.c_void_p, C.c_int, C.POINTER(C.c_int)
SIGNATURES = {
    "ppm_abi_version": (_I, []),
    "ppm_last_error": (C.c_char_p, []),
    "ppm_scene_load_xml": (_I, [C.c_char_p, _I, C.POINTER(_VP)]),
    "ppm_scene_destroy": (None, [_VP]),
    "ppm_num_cameras": (_I, [_VP]),
    "ppm_camera_info": (_I, [_VP, _I, _IP, _IP, _IP]),
    "ppm_image_name": (C.c_char_p, [_VP, _I]),
    "ppm_settings": (_I, [_VP, _IP, _IP, _IP]),
    "ppm_set_seed": (_I, [_VP, C.c_ulonglong]),
    "ppm_set_batching": (_I, [_VP, C.c_longlong, C.c_longlong]),
    "ppm_set_update_compaction": (_I, [_VP, C.c_longlong]),
    "ppm_set_update_segment": (_I, [_VP, _I]),
    "ppm_eye_pass": (_I, [_VP, _I]),
    "ppm_build_hash_grid": (_I, [_VP, _I, _I, C.POINTER(C.c_double)]),
    "ppm_num_hit_points": (_I, [_VP]),
    "ppm_read_hit_points": (_I, [_VP, _VP]),
    "ppm_read_hit_state": (_I, [_VP, _VP]),
    "ppm_trace_photons": (_I, [_VP, C.c_longlong, C.c_longlong]),
    "ppm_density_estimation": (_I, [_VP, C.c_longlong, _VP]),
    "ppm_render": (_I, [_VP, _I, _I, _VP, C.POINTER(ppm_stats)]),
    "ppm_collect_stats": (_I, [_VP, C.POINTER(ppm_stats)]),
    "ppm_write_png": (_I, [C.c_char_p, _VP, _I, _I]),
    "ppm_scene_load_xml_multi": (_I, [C.c_char_p, _I, _IP, C.POINTER(_VP)]),
    "ppm_scene_device_count": (_I, [_VP]),
    "ppm_set_update_shard": (_I, [_VP, _I, _I]),
    "ppm_hit_point_shards": (_I, [_VP, _VP]),
    "ppm_write_hit_state": (_I, [_VP, _VP]),
}


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"ceng795_amd photon-mapping library not built: {LIB_PATH} is "
                              "missing (run `python -c 'import __graft_entry__ as g; g.build()'`)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.ppm_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: C ABI version {L.ppm_abi_version()}, expected "
                              f"{ABI_VERSION} (rebuild the library)")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise RTError(rc, lib().ppm_last_error().decode(errors="replace"))
    return rc


@dataclass
class PPMCamera:
    width: int
    height: int
    num_samples: int
    image_name: str


class PhotonScene:
    """PPM Scene on one GPU (device index ``device``), or — ``devices=[...]`` — one scene over
    several GPUs of this process: every pass runs on each, the update pass is sharded by hit
    point and the shards' state is gathered onto ``devices[0]`` (ppm_scene_load_xml_multi)."""

    def __init__(self, xml_path: str, device: int = 0, seed: int = 0, devices=None):
        h = C.c_void_p()
        if devices is None:
            check(lib().ppm_scene_load_xml(str(xml_path).encode(), device, C.byref(h)))
        else:
            ids = (C.c_int * len(devices))(*[int(d) for d in devices])
            check(lib().ppm_scene_load_xml_multi(str(xml_path).encode(), len(devices), ids,
                                                 C.byref(h)))
        self._h = h
        self.set_seed(seed)

    def close(self):
        if getattr(self, "_h", None):
            lib().ppm_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def num_cameras(self) -> int:
        return lib().ppm_num_cameras(self._h)

    def camera(self, i: int = 0) -> PPMCamera:
        w, h, n = C.c_int(), C.c_int(), C.c_int()
        check(lib().ppm_camera_info(self._h, i, C.byref(w), C.byref(h), C.byref(n)))
        return PPMCamera(w.value, h.value, n.value, lib().ppm_image_name(self._h, i).decode())

    def settings(self):
        """(PhotonCountPerIteration, NumberOfIterations, MaxRecursionDepth)"""
        p, it, d = C.c_int(), C.c_int(), C.c_int()
        check(lib().ppm_settings(self._h, C.byref(p), C.byref(it), C.byref(d)))
        return p.value, it.value, d.value

    def set_seed(self, seed: int) -> None:
        check(lib().ppm_set_seed(self._h, int(seed)))

    def set_batching(self, slot_bytes: int = 0, max_updates: int = 0) -> None:
        """Photon-pass batch sizing (results do not depend on it); 0 = defaults."""
        check(lib().ppm_set_batching(self._h, int(slot_bytes), int(max_updates)))

    def set_update_compaction(self, min_list: int = -1) -> None:
        """Update-pass tile-list compaction threshold (results do not depend on it):
        -1 = default, 0 = off, n = compact tiles whose deposit list holds >= n deposits."""
        check(lib().ppm_set_update_compaction(self._h, int(min_list)))

    def set_update_segment(self, seg_len: int = 0) -> None:
        """Deposits per compaction segment of the update pass (results do not depend on it):
        0 = default (32768)."""
        check(lib().ppm_set_update_segment(self._h, int(seg_len)))

    @property
    def device_count(self) -> int:
        return lib().ppm_scene_device_count(self._h)

    def set_update_shard(self, shard: int, shards: int) -> None:
        """Apply only update shard ``shard`` of ``shards`` (one process per GPU); takes effect
        at the next build_hash_grid."""
        check(lib().ppm_set_update_shard(self._h, int(shard), int(shards)))

    def hit_point_shards(self) -> np.ndarray:
        """Per hit point, the shard whose update tiles own it (after build_hash_grid)."""
        out = np.zeros(lib().ppm_num_hit_points(self._h), np.int32)
        check(lib().ppm_hit_point_shards(self._h, out.ctypes.data))
        return out

    def write_hit_state(self, state: np.ndarray) -> None:
        """Overwrite the hit-point state (n x 5: flux xyz, radius^2, n)."""
        st = np.ascontiguousarray(state, np.float32)
        if st.shape != (lib().ppm_num_hit_points(self._h), 5):
            raise ValueError(f"hit state must be ({lib().ppm_num_hit_points(self._h)}, 5)")
        check(lib().ppm_write_hit_state(self._h, st.ctypes.data))

    # ------------------------------------------------------------------ reference passes
    def reset_hash_grid(self) -> None:
        """Scene::reset_hash_grid — folded into eye_trace_lines (which rebuilds the points)."""

    def eye_trace_lines(self, camera_index: int = 0) -> int:
        check(lib().ppm_eye_pass(self._h, camera_index))
        return lib().ppm_num_hit_points(self._h)

    def build_hash_grid(self, width: int, height: int):
        info = (C.c_double * 8)()
        check(lib().ppm_build_hash_grid(self._h, width, height, info))
        return list(info)

    def trace_photons(self, first: int, count: int) -> None:
        check(lib().ppm_trace_photons(self._h, first, count))

    def trace_n_photons(self, n: int, iteration_count: int, first: int = 0) -> None:
        self.trace_photons(first, n * iteration_count)

    def density_estimation(self, total_num_of_photons: int, camera_index: int = 0) -> np.ndarray:
        c = self.camera(camera_index)
        out = np.zeros((c.height, c.width, 3), np.float32)
        check(lib().ppm_density_estimation(self._h, total_num_of_photons, out.ctypes.data))
        return out

    def hit_points(self) -> np.ndarray:
        n = lib().ppm_num_hit_points(self._h)
        out = np.zeros((n, 16), np.float32)
        check(lib().ppm_read_hit_points(self._h, out.ctypes.data))
        return out

    def hit_state(self) -> np.ndarray:
        n = lib().ppm_num_hit_points(self._h)
        out = np.zeros((n, 5), np.float32)
        check(lib().ppm_read_hit_state(self._h, out.ctypes.data))
        return out

    def collect_stats(self) -> ppm_stats:
        st = ppm_stats()
        check(lib().ppm_collect_stats(self._h, C.byref(st)))
        return st

    def render(self, camera_index: int = 0, reference_threads: int = 8):
        c = self.camera(camera_index)
        out = np.zeros((c.height, c.width, 3), np.float32)
        st = ppm_stats()
        check(lib().ppm_render(self._h, camera_index, reference_threads, out.ctypes.data,
                               C.byref(st)))
        return out, st


def merge_shard_states(states, owners: np.ndarray) -> np.ndarray:
    """The merged hit-point state of a sharded update pass: hit point h takes row h of the
    state of the shard that owns it (``owners`` = hit_point_shards())."""
    states = np.stack([np.asarray(s, np.float32) for s in states])
    owners = np.asarray(owners)
    if owners.shape != states.shape[1:2] or (owners.size and (owners.min() < 0 or
                                                              owners.max() >= len(states))):
        raise ValueError("owners must name one of the shards for every hit point")
    return states[owners, np.arange(owners.size)]


def write_ppm_png(path: str, rgb: np.ndarray) -> None:
    """PPM/src/main.cpp:142-156 tone curve + PNG."""
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w, _ = rgb.shape
    check(lib().ppm_write_png(str(path).encode(), rgb.ctypes.data, w, h))
