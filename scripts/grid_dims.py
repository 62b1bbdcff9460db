"""Grid layout (cells per axis, cells, references) of the canonical scene at the default and two
other cell scales (rt_debug_scene 9)."""
import sys
sys.path.insert(0, "ray-tracing-gpu-vulkan_amd")
import rtvk
r = rtvk.Renderer(0)
for K in (11,):
    r.set_scene(rtvk.generateRandomScene(0.0, K))
    print("canonical host grid", r.scene_array(9))
    for s in (1.6, 1.7):
        r.tune(grid_scale=s)
        r.set_scene(rtvk.generateRandomScene(0.0, K))
        print("scale", s, r.scene_array(9))
