bash tools/gpu_probe_prof.sh r03d && bash tools/gpu_timeline.sh r03d_tl
