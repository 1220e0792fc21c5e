"""Scene catalogue for the tests: deterministic XML from tools/gen_scene.py.

Each entry names what it covers from SURVEY.md appendix A (parity hazards)."""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_scene as G  # noqa: E402

# name -> (factory, what it exercises)
CATALOGUE = {
    # C1: 3 triangles + 1 sphere, Phong exponent 10 on one material (double pow)
    "c1": (lambda: G.simple_scene(400, 400), "C1 plumbing scene; misses -> background"),
    "hf_small": (lambda: G.heightfield_scene(32, 64, 48), "shared mesh edges (equal-t ties)"),
    "hf_side": (lambda: G.heightfield_scene(48, 96, 64, view="side"),
                "partial coverage, oblique + grazing rays, silhouettes"),
    "soup1": (lambda: G.soup_scene(1, 96, 96),
              "meshes + loose tris + spheres, 4 lights, back-lit faces, grazing camera"),
    "soup2": (lambda: G.soup_scene(2, 80, 64), "second seed"),
    "soup3": (lambda: G.soup_scene(3, 64, 72, n_mesh_tris=2000), "bigger mesh"),
    "single_sphere": (lambda: G.single_sphere_scene(64, 64),
                      "root is a sphere: negative-t hits shaded (Sphere.h:43-45)"),
    "single_triangle": (lambda: G.single_triangle_scene(64, 64), "root is a triangle"),
    "c2": (lambda: G.heightfield_scene(187, 800, 800, name="c2.png"), "C2 69k tris 800x800"),
    # grazing rays: the fp32 triangle test's t is ill-conditioned (exactness of any culling)
    "graze_plane": (lambda: G.grazing_plane_scene(64, 96, 64),
                    "flat grid, rays 1e-7..1e-4 rad above its plane"),
    "graze_hf": (lambda: G.grazing_heightfield_scene(187, 256, 64),
                 "C2 height field skimmed at < 1e-3 rad"),
}

# Scenes whose MaxRecursionDepth > 0 with mirror / dielectric materials.
RECURSIVE = {
    "soup_depth3": (lambda: G.soup_scene(4, 96, 96, depth=3, mirror=True, glass=True),
                    "mirror + dielectric recursion depth 3"),
    "soup_depth1": (lambda: G.soup_scene(5, 64, 64, depth=1, mirror=True, glass=True),
                    "depth 1: one bounce, misses below max depth return black"),
    "soup_depth6": (lambda: G.soup_scene(6, 48, 40, depth=6, mirror=True, glass=True,
                                         n_spheres=10),
                    "depth 6: total internal reflection, exiting rays, Beer absorption"),
    "mirror_only": (lambda: G.soup_scene(7, 64, 48, depth=4, mirror=True, glass=False),
                    "mirrors only"),
}

# Cameras with NumSamples > 1: jittered MSAA + Gaussian 3x3 splat.
MSAA = {
    "msaa4": (lambda: G.soup_scene(8, 48, 40, num_samples=4), "n = 2, depth 0"),
    "msaa5": (lambda: G.soup_scene(9, 33, 27, num_samples=5),
              "NumSamples 5 -> n = (int)sqrt(5) = 2; ragged tiles"),
    "msaa9_depth2": (lambda: G.soup_scene(10, 40, 32, depth=2, mirror=True, glass=True,
                                          num_samples=9), "n = 3 with mirror + dielectric"),
    "msaa16": (lambda: G.soup_scene(11, 32, 24, num_samples=16), "n = 4"),
}

# The multi-GPU split paths (row bands, pixel records) on a frame whose sides are no multiple of
# the 8x8 tile: partial tile rows and columns, pixels outside the frame in the last tiles.
SPLIT = {
    "ragged": (lambda: G.soup_scene(12, 75, 53), "75x53: ragged tiles, 4 lights, spheres"),
}

SMALL = ["c1", "hf_small", "hf_side", "soup1", "soup2", "soup3", "single_sphere",
         "single_triangle", "graze_plane", "graze_hf"]


def write(name: str, directory: str) -> str:
    table = {**CATALOGUE, **RECURSIVE, **MSAA, **SPLIT}
    path = os.path.join(directory, f"{name}.xml")
    if not os.path.exists(path):
        text = table[name][0]().to_xml()
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)
    return path


def write_c3(directory: str, cameras: int = 1) -> str:
    path = os.path.join(directory, f"c3_{cameras}.xml")
    if not os.path.exists(path):
        spec = G.heightfield_scene(708, 1920, 1080, name="c3.png", cameras=cameras)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(spec.to_xml())
        os.replace(tmp, path)
    return path


# PPM (photon mapping) scenes in the PPM XML dialect (tools/gen_ppm_scene.py).
import gen_ppm_scene as GP  # noqa: E402

PPM = {
    "ppm_box": (lambda: GP.cornell(64, 64, photons=10000, iterations=10),
                "C5 Cornell box at 64x64, 1e5 photons: mirror + glass spheres"),
    "ppm_xform": (lambda: GP.cornell(64, 64, photons=10000, iterations=10, variant="transforms"),
                  "scaled sphere, rotated smooth-shaded mesh + MeshInstance"),
    "ppm_msaa": (lambda: GP.cornell(48, 40, photons=8000, iterations=10, num_samples=4),
                 "NumSamples 4: 2x2 jittered eye samples per pixel"),
    "ppm_shallow": (lambda: GP.cornell(40, 40, photons=6000, iterations=10, max_depth=3),
                    "MaxRecursionDepth 3 cuts eye and photon paths"),
}

# GPU-vs-oracle only (no reference goldens): a mesh BVH deeper than the kernels' LDS traversal
# stacks, so the eye and photon kernels take their scratch-stack variants.
PPM_DEEP = {
    "ppm_deep": (lambda: GP.cornell(40, 40, photons=6000, iterations=10, variant="deep"),
                 "4,608-triangle floor mesh: BVH deeper than the LDS stacks (scratch stacks)"),
}


def write_ppm(name: str, directory: str) -> str:
    path = os.path.join(directory, f"{name}.xml")
    if not os.path.exists(path):
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write({**PPM, **PPM_DEEP}[name][0]())
        os.replace(tmp, path)
    return path


def write_c5(directory: str) -> str:
    path = os.path.join(directory, "c5.xml")
    if not os.path.exists(path):
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(GP.cornell(256, 256, photons=10000, iterations=1000))
        os.replace(tmp, path)
    return path


def write_c4(directory: str) -> str:
    """C4: the C3 mesh at 3840x2160 (BASELINE.json configs[3])."""
    path = os.path.join(directory, "c4.xml")
    if not os.path.exists(path):
        spec = G.heightfield_scene(708, 3840, 2160, name="c4.png")
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(spec.to_xml())
        os.replace(tmp, path)
    return path
