import os, sys
sys.path.insert(0, os.getcwd())
import bench
pkg = bench.load_package()
opts = pkg.RenderOptions.from_cli("-w 1920 -r 5 -O r -A 4".split())
host = pkg.HostScene("scenes/trimesh2.ray")
dev = pkg.DeviceScene(host, 0)
st = dev.render(opts, want_f64=False, stats=True)["stats"]
print(os.environ.get("RTX_HIP_LIB", "default"), st["kernel_ms"])
