#!/usr/bin/env python3
"""Does a device-to-host copy of one C3 frame overlap a render kernel on this box?  Times, one
at a time and then together on two streams: the 24.9 MB D2H copy into pinned memory, and a C3
frame (rt_render_device).  Prints one JSON object (ms)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import ceng795_amd
    with ceng795_amd.Scene(bench.scene_path("c3", 1), device=0) as s:
        c = s.camera(0)
        frame = torch.empty((c.height, c.width, 3), device="cuda")
        src = torch.rand((c.height, c.width, 3), device="cuda")
        host = torch.empty((c.height, c.width, 3), pin_memory=True)
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

        def render():
            s.render_device(0, frame.data_ptr(), stream=sa.cuda_stream)

        def copy():
            with torch.cuda.stream(sb):
                host.copy_(src, non_blocking=True)

        def timed(fn, reps=20):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
                torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        out = {"copy_ms": timed(copy), "render_ms": timed(render)}
        out["both_ms"] = timed(lambda: (render(), copy()))
        out["copy_GBps"] = host.numel() * 4 / out["copy_ms"] / 1e6
        print(json.dumps({k: round(v, 4) for k, v in out.items()}))


if __name__ == "__main__":
    main()
