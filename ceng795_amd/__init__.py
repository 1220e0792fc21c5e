"""ceng795_amd — MI355X-native ray-trace hot path of kadircet/ceng795 HW2.

Python mirror of the reference's render interface (HW2/Scene.h:30-43):

    scene = Scene("scene.xml")                       # Scene::Scene(file_name)
    pixels = scene.new_image(camera_index)           # Pixel[w*h]  (fp32 RGB radiance)
    scene.render_image(camera_index, pixels, starting_row, height_increase)
    write_png(name, pixels)                          # HW2/main.cpp:43-57

Rendering runs in libceng795_rt.so's gfx950 kernels; there is no CPU path.
"""
from .scene import Scene, CameraInfo, write_png  # noqa: F401
from ._lib import RTError, RT_TRAVERSAL_FAST, RT_TRAVERSAL_REFERENCE  # noqa: F401

__all__ = ["Scene", "CameraInfo", "write_png", "RTError", "RT_TRAVERSAL_FAST",
           "RT_TRAVERSAL_REFERENCE"]
