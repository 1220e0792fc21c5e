#!/usr/bin/env python3
"""Deterministic synthetic scene generator (HW2 XML dialect).

The reference ships no scenes (its .gitignore drops *.xml and scenes/), so every
parity and timing input is synthesised here, following SURVEY.md §8(d):

* ``heightfield``: an n x n vertex grid over x in [-3, 3], z in [-8, -2] with
  y = -1.5 + 0.15 sin(5x) cos(4z) + 0.02 U[0,1) (random.seed(795), row-major j then i),
  two faces per quad, one Mesh, one point light.  C2 = n 187 at 800x800,
  C3 = n 708 at 1920x1080, C4 = n 708 at 3840x2160.
* ``simple``: the C1 plumbing scene (3 triangles + 1 sphere, 400x400).
* ``soup``: a seeded mix of meshes, loose triangles, spheres, several materials and
  lights, and camera placements that produce grazing rays, back-lit faces and misses.
  It exists to cover the hazards listed in SURVEY.md appendix A.
* ``single_sphere`` / ``single_triangle``: one-object scenes, where the BVH root is the
  primitive itself (HW2/Bounding_volume_hierarchy.h:13-14).

The XML follows the tags and defaults read by HW2/Scene.cpp:198-451 (appendix B).  The
file starts with ``<Scene>`` and has no XML declaration, because the reference takes
``file.FirstChild()`` as the root (HW2/Scene.cpp:206).
"""
from __future__ import annotations

import argparse
import math
import random
import sys
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

Vec = Tuple[float, float, float]


def _v(v: Sequence[float]) -> str:
    return " ".join(_num(x) for x in v)


def _num(x) -> str:
    if isinstance(x, int):
        return str(x)
    s = repr(float(x))
    return s[:-2] if s.endswith(".0") else s


@dataclass
class Camera:
    position: Vec
    gaze: Vec
    up: Vec
    near_plane: Tuple[float, float, float, float]
    near_distance: float
    width: int
    height: int
    image_name: str
    num_samples: Optional[int] = None


@dataclass
class Material:
    ambient: Vec = (0, 0, 0)
    diffuse: Vec = (0, 0, 0)
    specular: Vec = (0, 0, 0)
    mirror: Optional[Vec] = None
    phong: Optional[float] = None
    transparency: Optional[Vec] = None
    refraction_index: Optional[float] = None


@dataclass
class SceneSpec:
    cameras: List[Camera]
    ambient: Vec
    lights: List[Tuple[Vec, Vec]]
    materials: List[Material]
    vertex_text: str
    meshes: List[Tuple[int, str]] = field(default_factory=list)  # (material, faces text)
    triangles: List[Tuple[int, Tuple[int, int, int]]] = field(default_factory=list)
    spheres: List[Tuple[int, int, float]] = field(default_factory=list)  # (mat, center idx, r)
    background: Optional[Vec] = (0, 0, 0)
    shadow_eps: Optional[float] = 1e-3
    max_depth: Optional[int] = 0

    def to_xml(self) -> str:
        out = ["<Scene>"]
        if self.background is not None:
            out.append(f"  <BackgroundColor>{_v(self.background)}</BackgroundColor>")
        if self.shadow_eps is not None:
            out.append(f"  <ShadowRayEpsilon>{_num(self.shadow_eps)}</ShadowRayEpsilon>")
        if self.max_depth is not None:
            out.append(f"  <MaxRecursionDepth>{self.max_depth}</MaxRecursionDepth>")
        out.append("  <Cameras>")
        for i, c in enumerate(self.cameras):
            out.append(f'    <Camera id="{i + 1}">')
            out.append(f"      <Position>{_v(c.position)}</Position>")
            out.append(f"      <Gaze>{_v(c.gaze)}</Gaze>")
            out.append(f"      <Up>{_v(c.up)}</Up>")
            out.append(f"      <NearPlane>{_v(c.near_plane)}</NearPlane>")
            out.append(f"      <NearDistance>{_num(c.near_distance)}</NearDistance>")
            out.append(f"      <ImageResolution>{c.width} {c.height}</ImageResolution>")
            if c.num_samples is not None:
                out.append(f"      <NumSamples>{c.num_samples}</NumSamples>")
            out.append(f"      <ImageName>{c.image_name}</ImageName>")
            out.append("    </Camera>")
        out.append("  </Cameras>")
        out.append("  <Lights>")
        out.append(f"    <AmbientLight>{_v(self.ambient)}</AmbientLight>")
        for i, (p, inten) in enumerate(self.lights):
            out.append(f'    <PointLight id="{i + 1}">')
            out.append(f"      <Position>{_v(p)}</Position>")
            out.append(f"      <Intensity>{_v(inten)}</Intensity>")
            out.append("    </PointLight>")
        out.append("  </Lights>")
        out.append("  <Materials>")
        for i, m in enumerate(self.materials):
            out.append(f'    <Material id="{i + 1}">')
            out.append(f"      <AmbientReflectance>{_v(m.ambient)}</AmbientReflectance>")
            out.append(f"      <DiffuseReflectance>{_v(m.diffuse)}</DiffuseReflectance>")
            out.append(f"      <SpecularReflectance>{_v(m.specular)}</SpecularReflectance>")
            if m.mirror is not None:
                out.append(f"      <MirrorReflectance>{_v(m.mirror)}</MirrorReflectance>")
            if m.phong is not None:
                out.append(f"      <PhongExponent>{_num(m.phong)}</PhongExponent>")
            if m.transparency is not None:
                out.append(f"      <Transparency>{_v(m.transparency)}</Transparency>")
            if m.refraction_index is not None:
                out.append(f"      <RefractionIndex>{_num(m.refraction_index)}</RefractionIndex>")
            out.append("    </Material>")
        out.append("  </Materials>")
        out.append("  <VertexData>")
        out.append(self.vertex_text)
        out.append("  </VertexData>")
        out.append("  <Objects>")
        for i, (mat, faces) in enumerate(self.meshes):
            out.append(f'    <Mesh id="{i + 1}">')
            out.append(f"      <Material>{mat}</Material>")
            out.append("      <Faces>")
            out.append(faces)
            out.append("      </Faces>")
            out.append("    </Mesh>")
        for i, (mat, idx) in enumerate(self.triangles):
            out.append(f'    <Triangle id="{i + 1}">')
            out.append(f"      <Material>{mat}</Material>")
            out.append(f"      <Indices>{idx[0]} {idx[1]} {idx[2]}</Indices>")
            out.append("    </Triangle>")
        for i, (mat, c, r) in enumerate(self.spheres):
            out.append(f'    <Sphere id="{i + 1}">')
            out.append(f"      <Material>{mat}</Material>")
            out.append(f"      <Center>{c}</Center>")
            out.append(f"      <Radius>{_num(r)}</Radius>")
            out.append("    </Sphere>")
        out.append("  </Objects>")
        out.append("</Scene>")
        return "\n".join(out) + "\n"


# --------------------------------------------------------------------------- grazing rays
def grazing_plane_scene(n: int, width: int, height: int, cam_height: float = 1e-3,
                        rows_angle: Tuple[float, float] = (1e-7, 1e-4)) -> SceneSpec:
    """A flat n x n vertex grid on y = 0 (x in [-50, 50], z in [-2000, 0]) seen by a camera
    cam_height above it looking along -z: row angles below the horizon run over rows_angle
    (radians), so rays meet the triangles' plane at grazing angles down to ~1e-7, where the
    fp32 Cramer quotients of Triangle::intersect (HW2/Triangle.cpp:35-65) are ill-conditioned
    and a hit's computed t can be far from its true distance."""
    lines = []
    for j in range(n):
        z = -2000.0 + 2000.0 * j / (n - 1)
        for i in range(n):
            x = -50.0 + 100.0 * i / (n - 1)
            lines.append("%.6f %.6f %.6f" % (x, 0.0, z))
    lo, hi = rows_angle
    cam = Camera((0, cam_height, 0), (0, 0, -1), (0, 1, 0), (-0.5, 0.5, -hi, -lo), 1,
                 width, height, "graze_plane.png")
    return SceneSpec(
        cameras=[cam], ambient=(25, 25, 25), lights=[((0, 10, -50), (5e5, 5e5, 5e5))],
        materials=[Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1), phong=1)],
        vertex_text="\n".join(lines), meshes=[(1, "\n".join(heightfield_faces(n)))])


def grazing_heightfield_scene(n: int, width: int, height: int) -> SceneSpec:
    """The height field of SURVEY §8(d) seen from just above its highest point, looking along
    -z with row angles 0..1e-3 rad below the horizon: rays skim the bumps."""
    spec = heightfield_scene(n, width, height)
    spec.cameras = [Camera((0, -1.42, -1.9), (0, 0, -1), (0, 1, 0), (-0.6, 0.6, -1e-3, 0.0), 1,
                           width, height, "graze_hf.png")]
    return spec


# --------------------------------------------------------------------------- heightfield
def heightfield_vertices(n: int, seed: int = 795) -> List[str]:
    rng = random.Random(seed)
    lines = []
    for j in range(n):
        z = -8.0 + 6.0 * j / (n - 1)
        for i in range(n):
            x = -3.0 + 6.0 * i / (n - 1)
            y = -1.5 + 0.15 * math.sin(5.0 * x) * math.cos(4.0 * z) + 0.02 * rng.random()
            lines.append("%.6f %.6f %.6f" % (x, y, z))
    return lines


def heightfield_faces(n: int) -> List[str]:
    lines = []
    for j in range(n - 1):
        for i in range(n - 1):
            a = j * n + i + 1
            b = a + 1
            c = a + n
            d = c + 1
            lines.append(f"{a} {c} {b}")
            lines.append(f"{b} {c} {d}")
    return lines


def heightfield_scene(n: int, width: int, height: int, view: str = "top",
                      near_plane=None, name: str = "heightfield.png",
                      cameras: int = 1) -> SceneSpec:
    verts = heightfield_vertices(n)
    faces = heightfield_faces(n)
    cams = []
    for k in range(cameras):
        # extra cameras (multi-frame bench) are shifted along z; coverage stays ~100 %
        dz = 0.1 * (k - (cameras - 1) / 2.0)
        if view == "top":
            if near_plane is None:
                aspect = width / height
                near_plane = (-1, 1, -1, 1) if abs(aspect - 1) < 1e-9 else (-0.9, 0.9, -0.5, 0.5)
            cams.append(Camera((0, 1.5, -5 + dz), (0, -1, 0), (0, 0, -1), tuple(near_plane), 1,
                               width, height, name if cameras == 1 else f"{k}_{name}"))
        elif view == "side":
            np_ = near_plane or (-1, 1, -1, 1)
            cams.append(Camera((0, 0.5, 1.0 + dz), (0, -0.35, -1), (0, 1, 0), tuple(np_), 1,
                               width, height, name if cameras == 1 else f"{k}_{name}"))
        else:
            raise ValueError(view)
    return SceneSpec(
        cameras=cams,
        ambient=(25, 25, 25),
        lights=[((0, 4, -5), (1000, 1000, 1000))],
        materials=[Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1), phong=1)],
        vertex_text="\n".join(verts),
        meshes=[(1, "\n".join(faces))],
    )


# --------------------------------------------------------------------------- C1 simple
def simple_scene(width: int = 400, height: int = 400) -> SceneSpec:
    verts = [(-1.0, -0.5, -3.0), (1.0, -0.5, -3.0), (0.0, 0.8, -3.5),
             (-2.0, -1.0, -2.0), (2.0, -1.0, -2.0), (2.0, -1.0, -6.0), (-2.0, -1.0, -6.0),
             (0.6, 0.2, -2.2)]
    return SceneSpec(
        cameras=[Camera((0, 0, 0), (0, 0, -1), (0, 1, 0), (-1, 1, -1, 1), 1, width, height,
                        "simple.png")],
        background=(0, 0, 0),
        ambient=(25, 25, 25),
        lights=[((0, 2, 0), (800, 800, 800))],
        materials=[Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1), phong=1),
                   Material(ambient=(1, 0, 0), diffuse=(1, 0, 0), specular=(1, 1, 1), phong=10)],
        vertex_text="\n".join("%.6f %.6f %.6f" % v for v in verts),
        triangles=[(1, (1, 2, 3)), (2, (4, 5, 6)), (2, (4, 6, 7))],
        spheres=[(1, 8, 0.3)],
    )


# --------------------------------------------------------------------------- soup
def soup_scene(seed: int, width: int = 96, height: int = 96, n_mesh_tris: int = 400,
               n_loose: int = 12, n_spheres: int = 6, n_lights: int = 3,
               depth: int = 0, mirror: bool = False, glass: bool = False,
               num_samples: Optional[int] = None) -> SceneSpec:
    rng = random.Random(seed)
    verts: List[Vec] = []

    def add(v: Vec) -> int:
        verts.append(v)
        return len(verts)  # 1-based

    mats = [
        Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1), phong=1),
        Material(ambient=(0.1, 0.2, 0.3), diffuse=(0.6, 0.3, 0.2), specular=(0.9, 0.9, 0.9),
                 phong=rng.choice([3, 17.5, 64, 100])),
        Material(ambient=(0.5, 0.5, 0.5), diffuse=(0.2, 0.8, 0.4), specular=(0.3, 0.3, 0.3),
                 phong=7),
    ]
    if mirror:
        mats.append(Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.2, 0.2, 0.2),
                             specular=(0.5, 0.5, 0.5), mirror=(0.6, 0.6, 0.6), phong=20))
    if glass:
        mats.append(Material(ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0.8, 0.8, 0.8),
                             transparency=(0.3, 0.6, 0.9), refraction_index=1.5, phong=50))
    nm = len(mats)
    # a bumpy mesh patch (shared edges -> equal-t ties) + a vertical wall (grazing rays)
    g = max(2, int(math.sqrt(n_mesh_tris / 2)) + 1)
    base = len(verts)
    for j in range(g):
        for i in range(g):
            x = -2 + 4 * i / (g - 1)
            z = -6 + 4 * j / (g - 1)
            y = -1 + 0.3 * math.sin(3 * x + seed) * math.cos(2 * z) + 0.05 * rng.random()
            add((round(x, 6), round(y, 6), round(z, 6)))
    faces = []
    for j in range(g - 1):
        for i in range(g - 1):
            a = base + j * g + i + 1
            b, c = a + 1, a + g
            d = c + 1
            faces.append(f"{a} {c} {b}")
            faces.append(f"{b} {c} {d}")
    wall = []
    w0 = len(verts)
    for j in range(3):
        for i in range(3):
            add((round(-2 + 2 * i, 6), round(-1 + 1.2 * j, 6), -6.0))
    for j in range(2):
        for i in range(2):
            a = w0 + j * 3 + i + 1
            b, c = a + 1, a + 3
            d = c + 1
            wall.append(f"{a} {b} {c}")
            wall.append(f"{b} {d} {c}")
    loose = []
    for _ in range(n_loose):
        cx, cy, cz = rng.uniform(-1.5, 1.5), rng.uniform(-0.8, 1.2), rng.uniform(-5.5, -2.5)
        ids = tuple(add((round(cx + rng.uniform(-0.6, 0.6), 6), round(cy + rng.uniform(-0.6, 0.6), 6),
                         round(cz + rng.uniform(-0.6, 0.6), 6))) for _ in range(3))
        loose.append((rng.randrange(nm) + 1, ids))
    spheres = []
    for _ in range(n_spheres):
        c = add((round(rng.uniform(-1.5, 1.5), 6), round(rng.uniform(-0.5, 1.0), 6),
                 round(rng.uniform(-5.5, -2.5), 6)))
        spheres.append((rng.randrange(nm) + 1, c, round(rng.uniform(0.1, 0.5), 4)))
    lights = []
    for k in range(n_lights):
        lights.append(((round(rng.uniform(-3, 3), 3), round(rng.uniform(0.5, 4), 3),
                        round(rng.uniform(-6, 0), 3)),
                       (rng.choice([300, 600, 1000]), rng.choice([300, 600, 1000]), 500)))
    # one light below the floor: back-lit faces (negative, unclamped diffuse cos)
    lights.append(((0.3, -3.0, -4.0), (400, 400, 400)))
    cams = [Camera((0.2, 0.4, 0.5), (0, -0.15, -1), (0, 1, 0), (-0.8, 0.8, -0.8, 0.8), 1,
                   width, height, "soup_front.png", num_samples),
            Camera((0, 3.0, -4.0), (0, -1, 0.001), (0, 0, -1), (-1, 1, -1, 1), 1,
                   width, height, "soup_top.png", num_samples),
            # nearly edge-on to the mesh patch: grazing rays
            Camera((-3.5, -0.95, -4.0), (1, 0.003, 0), (0, 1, 0), (-0.6, 0.6, -0.3, 0.3), 1,
                   width, height, "soup_grazing.png", num_samples)]
    return SceneSpec(
        cameras=cams,
        background=(7, 13, 29),
        ambient=(20, 20, 20),
        lights=lights,
        materials=mats,
        vertex_text="\n".join("%.6f %.6f %.6f" % v for v in verts),
        meshes=[(1, "\n".join(faces)), (3, "\n".join(wall))],
        triangles=loose,
        spheres=spheres,
        max_depth=depth,
    )


def single_sphere_scene(width: int = 64, height: int = 64) -> SceneSpec:
    # camera *inside* the sphere region on one axis so negative-t roots occur
    return SceneSpec(
        cameras=[Camera((0, 0, 0), (0, 0, -1), (0, 1, 0), (-1, 1, -1, 1), 1, width, height,
                        "sphere.png"),
                 Camera((0, 0, -2.5), (0, 0, -1), (0, 1, 0), (-1, 1, -1, 1), 1, width, height,
                        "sphere_inside.png")],
        ambient=(25, 25, 25),
        lights=[((1, 2, 0), (700, 700, 700))],
        materials=[Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1), phong=5)],
        vertex_text="0 0 -3",
        spheres=[(1, 1, 1.0)],
        background=(3, 2, 1),
    )


def single_triangle_scene(width: int = 64, height: int = 64) -> SceneSpec:
    return SceneSpec(
        cameras=[Camera((0, 0, 0), (0, 0, -1), (0, 1, 0), (-1, 1, -1, 1), 1, width, height,
                        "tri.png")],
        ambient=(25, 25, 25),
        lights=[((0, 1, 0), (700, 700, 700)), ((0, 0, -5), (500, 500, 500))],
        materials=[Material(ambient=(1, 1, 1), diffuse=(1, 1, 1), specular=(1, 1, 1))],
        vertex_text="-1 -1 -2\n1 -1 -2\n0 1 -2.5",
        triangles=[(1, (1, 2, 3))],
    )


CONFIGS = {
    "c1": lambda: simple_scene(400, 400),
    "c2": lambda: heightfield_scene(187, 800, 800, name="c2.png"),
    "c3": lambda: heightfield_scene(708, 1920, 1080, name="c3.png"),
    "c4": lambda: heightfield_scene(708, 3840, 2160, name="c4.png"),
}


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("kind", choices=["c1", "c2", "c3", "c4", "heightfield", "simple", "soup",
                                    "single_sphere", "single_triangle"])
    p.add_argument("-o", "--out", default="-")
    p.add_argument("--n", type=int, default=32)
    p.add_argument("--width", type=int, default=128)
    p.add_argument("--height", type=int, default=128)
    p.add_argument("--view", default="top")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--depth", type=int, default=0)
    p.add_argument("--cameras", type=int, default=1)
    a = p.parse_args(argv)
    if a.kind in CONFIGS:
        spec = CONFIGS[a.kind]()
    elif a.kind == "heightfield":
        spec = heightfield_scene(a.n, a.width, a.height, view=a.view, cameras=a.cameras)
    elif a.kind == "simple":
        spec = simple_scene(a.width, a.height)
    elif a.kind == "soup":
        spec = soup_scene(a.seed, a.width, a.height, depth=a.depth, mirror=a.depth > 0,
                          glass=a.depth > 0)
    elif a.kind == "single_sphere":
        spec = single_sphere_scene(a.width, a.height)
    else:
        spec = single_triangle_scene(a.width, a.height)
    text = spec.to_xml()
    if a.out == "-":
        sys.stdout.write(text)
    else:
        with open(a.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
