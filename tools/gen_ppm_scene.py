#!/usr/bin/env python3
"""Deterministic synthetic scenes in the PPM XML dialect (PPM/src/Scene.cpp:373-501).

The reference ships no scenes.  Config C5 is a Cornell box: five walls of
two triangles each (floor, ceiling, back, left, right; the front is open), a mirror sphere
and a glass sphere of radius 0.35, one PointLight at (0, 0.9, 0) with intensity 1,
PhotonCountPerIteration 10000, NumberOfIterations 1000, 256x256.

Tags and defaults follow the PPM loaders: Camera.cpp:4-99 (Position, Up, NearDistance,
ImageResolution, NumSamples, ImageName, Gaze, NearPlane), Material.cpp:3-75,
Transformation.cpp:95-134, Point_light.cpp:32-51, Sphere.cpp:84-144, Mesh.cpp:5-206.
Triangles are wound so that (v1-v0)x(v2-v0) faces into the box: PPM culls triangles whose
normal points along the ray (Mesh_triangle.cpp:70-72).

``variant`` adds loader / traversal coverage on top of the box: ``"transforms"`` puts the
glass sphere under a scaling + translation and adds a rotated, smooth-shaded MeshInstance
of a small prism.
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional, Sequence


def _num(x) -> str:
    if isinstance(x, int):
        return str(x)
    s = repr(float(x))
    return s[:-2] if s.endswith(".0") else s


def _v(v: Sequence[float]) -> str:
    return " ".join(_num(x) for x in v)


def cornell(width: int = 256, height: int = 256, photons: int = 10000, iterations: int = 1000,
            max_depth: Optional[int] = None, num_samples: Optional[int] = None,
            variant: str = "plain", image_name: str = "cornell.png",
            light=(0.0, 0.9, 0.0), intensity=(1.0, 1.0, 1.0)) -> str:
    verts: List[Sequence[float]] = []

    def add(v) -> int:
        verts.append(v)
        return len(verts)  # 1-based

    # box corners: x, y, z in [-1, 1]
    c = {}
    for x in (-1, 1):
        for y in (-1, 1):
            for z in (-1, 1):
                c[(x, y, z)] = add((x, y, z))
    walls = {  # quad a b c d (counter-clockwise seen from inside) -> (a,b,c), (a,c,d)
        "floor": ((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)),
        "ceiling": ((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)),
        "back": ((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)),
        "left": ((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)),
        "right": ((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)),
    }
    mirror_center = add((-0.45, -0.65, -0.35))
    glass_center = add((0.45, -0.65, 0.25))
    lines = ["<Scene>"]
    if max_depth is not None:
        lines.append(f"  <MaxRecursionDepth>{max_depth}</MaxRecursionDepth>")
    lines += [f"  <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>",
              f"  <PhotonCountPerIteration>{photons}</PhotonCountPerIteration>",
              f"  <NumberOfIterations>{iterations}</NumberOfIterations>",
              "  <Cameras>", "    <Camera id=\"1\">",
              "      <Position>0 0 3.2</Position>", "      <Gaze>0 0 -1</Gaze>",
              "      <Up>0 1 0</Up>", "      <NearPlane>-0.5 0.5 -0.5 0.5</NearPlane>",
              "      <NearDistance>1.5</NearDistance>",
              f"      <ImageResolution>{width} {height}</ImageResolution>"]
    if num_samples is not None:
        lines.append(f"      <NumSamples>{num_samples}</NumSamples>")
    lines += [f"      <ImageName>{image_name}</ImageName>", "    </Camera>", "  </Cameras>",
              "  <Lights>", "    <PointLight id=\"1\">",
              f"      <Position>{_v(light)}</Position>",
              f"      <Intensity>{_v(intensity)}</Intensity>", "    </PointLight>",
              "  </Lights>", "  <Materials>"]
    mats = [  # id: (diffuse, specular, mirror, phong, transparency, refraction)
        ((0.75, 0.75, 0.75), None, None, None, None, None),      # 1 white
        ((0.75, 0.25, 0.25), None, None, None, None, None),      # 2 red
        ((0.25, 0.25, 0.75), None, None, None, None, None),      # 3 blue
        ((0, 0, 0), None, (1, 1, 1), None, None, None),          # 4 mirror
        ((0, 0, 0), None, None, None, (1, 1, 1), 1.5),           # 5 glass
        ((0.6, 0.6, 0.2), (0.3, 0.3, 0.3), None, 20, None, None),  # 6 glossy (variant)
    ]
    for k, (kd, ks, km, ph, kt, eta) in enumerate(mats, 1):
        lines.append(f"    <Material id=\"{k}\">")
        lines.append(f"      <DiffuseReflectance>{_v(kd)}</DiffuseReflectance>")
        if ks is not None:
            lines.append(f"      <SpecularReflectance>{_v(ks)}</SpecularReflectance>")
        if km is not None:
            lines.append(f"      <MirrorReflectance>{_v(km)}</MirrorReflectance>")
        if ph is not None:
            lines.append(f"      <PhongExponent>{ph}</PhongExponent>")
        if kt is not None:
            lines.append(f"      <Transparency>{_v(kt)}</Transparency>")
        if eta is not None:
            lines.append(f"      <RefractionIndex>{eta}</RefractionIndex>")
        lines.append("    </Material>")
    lines.append("  </Materials>")
    prism = []
    if variant == "transforms":
        lines += ["  <Transformations>",
                  "    <Translation id=\"1\">0.1 0.05 0</Translation>",
                  "    <Translation id=\"2\">-0.3 0.2 0.3</Translation>",
                  "    <Scaling id=\"1\">1.2 0.8 1.2</Scaling>",
                  "    <Rotation id=\"1\">30 0 1 0</Rotation>",
                  "    <Rotation id=\"2\">-15 1 0 0.5</Rotation>",
                  "  </Transformations>"]
        base = [add((-0.15, -0.3, -0.15)), add((0.15, -0.3, -0.15)), add((0.0, -0.3, 0.15)),
                add((0.0, 0.05, 0.0))]
        prism = [(base[0], base[1], base[2]), (base[0], base[3], base[1]),  # outward normals
                 (base[1], base[3], base[2]), (base[2], base[3], base[0])]
    grid = []
    if variant == "deep":  # the floor as a 48 x 48 grid of quads: a mesh BVH of 13+ levels
        n = 48
        idx = {}
        for j in range(n + 1):
            for i in range(n + 1):
                idx[(i, j)] = add((-1 + 2 * i / n, -1.0, 1 - 2 * j / n))
        for j in range(n):
            for i in range(n):
                a, b, cc, d = idx[(i, j)], idx[(i + 1, j)], idx[(i + 1, j + 1)], idx[(i, j + 1)]
                grid += [(a, b, cc), (a, cc, d)]
    lines.append("  <VertexData>")
    lines += ["    " + _v(v) for v in verts]
    lines.append("  </VertexData>")
    lines.append("  <Objects>")
    wall_mat = {"floor": 1, "ceiling": 1, "back": 1, "left": 2, "right": 3}
    mesh_id = 0
    for name, quad in walls.items():
        a, b, cc, d = (c[q] for q in quad)
        mesh_id += 1
        if name == "floor" and grid:
            lines += [f"    <Mesh id=\"{mesh_id}\">", f"      <Material>{wall_mat[name]}</Material>",
                      "      <Faces>"]
            lines += [f"        {x} {y} {z}" for x, y, z in grid]
            lines += ["      </Faces>", "    </Mesh>"]
            continue
        lines += [f"    <Mesh id=\"{mesh_id}\">", f"      <Material>{wall_mat[name]}</Material>",
                  "      <Faces>", f"        {a} {b} {cc}", f"        {a} {cc} {d}",
                  "      </Faces>", "    </Mesh>"]
    if prism:
        mesh_id += 1
        lines += [f"    <Mesh id=\"{mesh_id}\" shadingMode=\"smooth\">",
                  "      <Material>6</Material>",
                  "      <Transformations>r1 t1</Transformations>", "      <Faces>"]
        lines += [f"        {a} {b} {cc}" for a, b, cc in prism]
        lines += ["      </Faces>", "    </Mesh>",
                  f"    <MeshInstance id=\"1\" baseMeshId=\"{mesh_id}\">",
                  "      <Material>6</Material>",
                  "      <Transformations>r2 t2</Transformations>", "    </MeshInstance>"]
    glass_tf = "      <Transformations>s1 t1</Transformations>" if variant == "transforms" else None
    lines += ["    <Sphere id=\"1\">", "      <Material>4</Material>",
              f"      <Center>{mirror_center}</Center>", "      <Radius>0.35</Radius>",
              "    </Sphere>", "    <Sphere id=\"2\">", "      <Material>5</Material>",
              f"      <Center>{glass_center}</Center>", "      <Radius>0.35</Radius>"]
    if glass_tf:
        lines.append(glass_tf)
    lines += ["    </Sphere>", "  </Objects>", "</Scene>"]
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("out")
    ap.add_argument("--size", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--photons", type=int, default=10000)
    ap.add_argument("--iterations", type=int, default=1000)
    ap.add_argument("--variant", default="plain", choices=["plain", "transforms", "deep"])
    ap.add_argument("--num-samples", type=int, default=None)
    a = ap.parse_args(argv)
    with open(a.out, "w") as f:
        f.write(cornell(a.size[0], a.size[1], a.photons, a.iterations,
                        num_samples=a.num_samples, variant=a.variant))
    return 0


if __name__ == "__main__":
    sys.exit(main())
