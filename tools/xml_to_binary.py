#!/usr/bin/env python3
"""Rewrite an HW2 scene so its bulk lists use HW7's binary format:
<VertexData binaryFile="x.vertices"/> and <Faces binaryFile="x.faces<k>"/>, each file an int32
count N followed by N float32 (vertex) or int32 (face, 1-based as in the text, unless
<ZeroBasedIndexing>true</ZeroBasedIndexing>) triples — HW7/src/Scene.cpp:1839-1904.

The numbers are parsed exactly as the reference parses the text (std::stringstream >> float
is strtof; Python's float() is correctly rounded, and numpy rounds it to float32 once), so the
binary scene loads to the same bits.  usage: xml_to_binary.py in.xml out.xml
"""
import os
import re
import sys

import numpy as np


def convert(src: str, dst: str, zero_based: bool = False) -> None:
    text = open(src).read()
    base = os.path.splitext(os.path.basename(dst))[0]
    outdir = os.path.dirname(os.path.abspath(dst))

    def vertices(m):
        vals = np.array([float(t) for t in m.group(1).split()], np.float32).reshape(-1, 3)
        name = f"{base}.vertices"
        with open(os.path.join(outdir, name), "wb") as f:
            np.array([len(vals)], np.int32).tofile(f)
            vals.tofile(f)
        return f'<VertexData binaryFile="{name}"/>'

    text = re.sub(r"<VertexData>(.*?)</VertexData>", vertices, text, flags=re.S)
    count = [0]

    def faces(m):
        idx = np.array([int(t) for t in m.group(1).split()], np.int32).reshape(-1, 3)
        if zero_based:
            idx = idx - 1
        name = f"{base}.faces{count[0]}"
        count[0] += 1
        with open(os.path.join(outdir, name), "wb") as f:
            np.array([len(idx)], np.int32).tofile(f)
            idx.tofile(f)
        return f'<Faces binaryFile="{name}"/>'

    text = re.sub(r"<Faces>(.*?)</Faces>", faces, text, flags=re.S)
    if zero_based:
        text = text.replace("<Scene>", "<Scene>\n  <ZeroBasedIndexing>true</ZeroBasedIndexing>", 1)
    with open(dst, "w") as f:
        f.write(text)


if __name__ == "__main__":
    convert(sys.argv[1], sys.argv[2], zero_based="--zero-based" in sys.argv)
