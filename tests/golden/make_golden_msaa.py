#!/usr/bin/env python3
"""Golden fixtures for MSAA cameras, from the REFERENCE ITSELF.

The reference seeds every pixel's std::default_random_engine from the wall clock
(HW2/Scene.cpp:35-37), so its MSAA frames are not reproducible and cannot be compared bit
for bit.  This script records, for every camera of tests/scenes.MSAA, TWO independent
reference renders (oracle/_ref/ref_harness `resolved`: Pixel::color / Pixel::weight, one
thread), which the tests use as a statistical pin: the oracle's (deterministically seeded)
frame must sit as close to each reference frame as the two reference frames sit to each
other.

It also pins the random-number pieces exactly: a tiny program compiled here against the
system libstdc++ (the reference's own <random>) prints uniform_real_distribution<float>(0,1)
draws of default_random_engine for a set of seeds; tests compare the oracle's restatement
bit for bit.

Output: tests/golden/golden_msaa.npz.   usage: python tests/golden/make_golden_msaa.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import scenes  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
SEEDS = [0, 1, 2, 16807, 2147483646, 2147483647, 2147483648, 12345678901234567,
         1760000000123456789, 2**64 - 1]
DRAWS = 64

STDLIB_PROBE = r"""
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
int main(int argc, char** argv) {
  const int n = std::atoi(argv[1]);
  for (int a = 2; a < argc; a++) {
    std::default_random_engine g;
    g.seed(std::strtoull(argv[a], nullptr, 10));
    std::uniform_real_distribution<float> d(0.0, 1);
    for (int k = 0; k < n; k++) {
      float f = d(g);
      unsigned u;
      std::memcpy(&u, &f, 4);
      std::printf("%08x\n", u);
    }
  }
}
"""


def stdlib_draws(d):
    src = os.path.join(d, "probe.cpp")
    exe = os.path.join(d, "probe")
    with open(src, "w") as f:
        f.write(STDLIB_PROBE)
    subprocess.run(["g++", "-O2", "-std=c++14", src, "-o", exe], check=True)
    out = subprocess.run([exe, str(DRAWS)] + [str(s) for s in SEEDS], check=True,
                         capture_output=True, text=True).stdout.split()
    bits = np.array([int(x, 16) for x in out], np.uint32).reshape(len(SEEDS), DRAWS)
    return bits.view(np.float32)


def camera_sizes(xml):
    import re
    text = open(xml).read()
    return [tuple(int(v) for v in m.split()) for m in
            re.findall(r"<ImageResolution>(.*?)</ImageResolution>", text)]


def main():
    if not os.path.exists(HARNESS):
        sys.exit("reference harness missing: run `make -C oracle ref` first")
    arrays = {}
    with tempfile.TemporaryDirectory() as d:
        arrays["stdlib_seeds"] = np.array(SEEDS, np.uint64)
        arrays["stdlib_draws"] = stdlib_draws(d)
        for name in scenes.MSAA:
            xml = scenes.write(name, d)
            for cam, (w, h) in enumerate(camera_sizes(xml)):
                for r in range(2):
                    out = os.path.join(d, f"{name}_{cam}_{r}.f32")
                    subprocess.run([HARNESS, "resolved", xml, str(cam), out, "1"], check=True)
                    arrays[f"{name}__{cam}__ref{r}"] = np.fromfile(out, np.float32).reshape(h, w, 3)
                print(name, cam, w, h, flush=True)
    np.savez_compressed(os.path.join(HERE, "golden_msaa.npz"), **arrays)


if __name__ == "__main__":
    main()
