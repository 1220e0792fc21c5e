"""ctypes binding of libceng795_rt.so (include/ceng795_rt.h).

The library is built in-tree (``make -C ceng795_amd/csrc`` or ``__graft_entry__.build()``).
There is no fallback: if the library is missing, importing the renderer fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CENG795_LIB=<variant> selects lib/libceng795_rt_<variant>.so: "diag" is the RT_DIAG build
# (packet-level work counters); other variants are timing experiments (tools/experiments.sh).
_VARIANT = os.environ.get("CENG795_LIB", "")
LIB_PATH = os.path.join(_HERE, "lib", f"libceng795_rt_{_VARIANT}.so" if _VARIANT else
                        "libceng795_rt.so")

RT_OK = 0
RT_E_INVALID = -1
RT_E_HIP = -2
RT_E_IO = -3
RT_E_PARSE = -4
RT_E_UNSUPPORTED = -5

RT_TRAVERSAL_FAST = 0
RT_TRAVERSAL_REFERENCE = 1

F3 = C.c_float * 3


class rt_material(C.Structure):
    _fields_ = [("ambient", F3), ("diffuse", F3), ("specular", F3), ("mirror", F3),
                ("transparency", F3), ("refraction_index", C.c_float),
                ("phong_exponent", C.c_float)]


class rt_point_light(C.Structure):
    _fields_ = [("position", F3), ("intensity", F3)]


class rt_camera(C.Structure):
    _fields_ = [("e", F3), ("top_left", F3), ("s_u", F3), ("s_v", F3), ("width", C.c_int),
                ("height", C.c_int), ("num_samples", C.c_int)]


class rt_scene_desc(C.Structure):
    _fields_ = [
        ("background", F3), ("shadow_ray_epsilon", C.c_float), ("max_recursion_depth", C.c_int),
        ("ambient_light", F3),
        ("vertices", C.POINTER(C.c_float)), ("num_vertices", C.c_int),
        ("materials", C.POINTER(rt_material)), ("num_materials", C.c_int),
        ("lights", C.POINTER(rt_point_light)), ("num_lights", C.c_int),
        ("cameras", C.POINTER(rt_camera)), ("num_cameras", C.c_int),
        ("num_meshes", C.c_int), ("mesh_material", C.POINTER(C.c_int)),
        ("mesh_face_count", C.POINTER(C.c_int)), ("mesh_faces", C.POINTER(C.c_int)),
        ("num_triangles", C.c_int), ("triangle_indices", C.POINTER(C.c_int)),
        ("triangle_material", C.POINTER(C.c_int)),
        ("num_spheres", C.c_int), ("sphere_center", C.POINTER(C.c_int)),
        ("sphere_radius", C.POINTER(C.c_float)), ("sphere_material", C.POINTER(C.c_int)),
        # ABI 7: the caller's own BVH (zero = the library builds the reference's)
        ("bvh_num_nodes", C.c_int), ("bvh_children", C.POINTER(C.c_int)),
        ("bvh_boxes", C.POINTER(C.c_float)), ("bvh_num_leaves", C.c_int),
        ("bvh_leaf_object", C.POINTER(C.c_int)), ("bvh_leaf_normals", C.POINTER(C.c_float)),
    ]


class rt_stats(C.Structure):
    _fields_ = [("primary_rays", C.c_longlong), ("shadow_rays", C.c_longlong),
                ("secondary_rays", C.c_longlong), ("primary_hits", C.c_longlong),
                ("kernel_ms", C.c_double)]

    def rays(self) -> int:
        return self.primary_rays + self.shadow_rays + self.secondary_rays


# name -> (restype, argtypes); mirrors include/ceng795_rt.h one to one
SIGNATURES = {
    "rt_scene_create": (C.c_int, [C.POINTER(rt_scene_desc), C.c_int, C.POINTER(C.c_void_p)]),
    "rt_scene_destroy": (None, [C.c_void_p]),
    "rt_scene_load_xml": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    "rt_scene_create_multi": (C.c_int, [C.POINTER(rt_scene_desc), C.c_int, C.POINTER(C.c_int),
                                        C.POINTER(C.c_void_p)]),
    "rt_scene_load_xml_multi": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_int),
                                          C.POINTER(C.c_void_p)]),
    "rt_scene_device_count": (C.c_int, [C.c_void_p]),
    "rt_release_stream_scratch": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_untile_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_scene_num_cameras": (C.c_int, [C.c_void_p]),
    "rt_scene_camera": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(rt_camera)]),
    "rt_scene_image_name": (C.c_char_p, [C.c_void_p, C.c_int]),
    "rt_scene_num_lights": (C.c_int, [C.c_void_p]),
    "rt_scene_dump_bvh": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rt_scene_bvh_depth": (C.c_int, [C.c_void_p]),
    "rt_set_traversal": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_set_msaa_seed": (C.c_int, [C.c_void_p, C.c_ulonglong]),
    "rt_render": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                            C.POINTER(rt_stats)]),
    "rt_render_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_void_p, C.c_void_p]),
    "rt_render_device_range": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "rt_scene_records_ok": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_tile_costs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "rt_resolve_rows": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p]),
    "rt_resolve_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_set_kernel_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_read_kernel_times": (C.c_int, [C.c_void_p, C.POINTER(C.c_double),
                                       C.POINTER(C.c_longlong)]),
    "rt_num_tiles": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "rt_collect_stats": (C.c_int, [C.c_void_p, C.POINTER(rt_stats)]),
    "rt_write_png": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "rt_camera_from_view": (C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_float),
                                      C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_float,
                                      C.c_int, C.c_int, C.c_int, C.POINTER(rt_camera)]),
    "rt_last_error": (C.c_char_p, []),
    "rt_abi_version": (C.c_int, []),
    "rt_host_dump_bvh_xml": (C.c_int, [C.c_char_p, C.c_char_p]),
    "rt_host_dump_bvh_desc": (C.c_int, [C.POINTER(rt_scene_desc), C.c_char_p]),
    "rt_host_alloc": (C.c_void_p, [C.c_size_t]),
    "rt_host_free": (None, [C.c_void_p]),
    "rt_host_check_accel_xml": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_longlong)]),
    "rt_debug_counters": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong)]),
    "rt_debug_timeline": (C.c_longlong, [C.POINTER(C.c_ulonglong), C.c_longlong]),
    "rt_debug_phases": (C.c_longlong, [C.POINTER(C.c_ulonglong), C.c_longlong]),
    "rt_debug_quotient_check": (C.c_int, [C.c_int, C.c_ulonglong, C.c_longlong,
                                          C.POINTER(C.c_longlong)]),
}

_lib = None


class RTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _share_torch_hip_runtime() -> None:
    """torch (2.10+rocm7.0) ships its own libamdhip64 / libhsa-runtime64 with the same
    sonames as /opt/rocm's.  Two HIP runtimes in one process cannot both own the GPU, so when
    torch is importable we load it first: the dynamic loader then binds our library's
    NEEDED libamdhip64.so.7 to the copy torch already mapped, and torch tensors, streams and
    torch.distributed (RCCL) share one runtime with our kernels."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


ABI_VERSION = 7  # CENG795_RT_ABI_VERSION of include/ceng795_rt.h


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"ceng795_amd native library not built: {LIB_PATH} is missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                if not _VARIANT:  # the shipping library must export the whole header
                    raise
                continue  # an older experiment build (CENG795_LIB): bind what it has
            fn.restype = res
            fn.argtypes = args
        if L.rt_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: C ABI version {L.rt_abi_version()}, this binding "
                              f"expects {ABI_VERSION} (rebuild the library)")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise RTError(rc, lib().rt_last_error().decode(errors="replace"))
    return rc
