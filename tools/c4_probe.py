import os, sys, time
sys.path.insert(0, os.getcwd())
import bench
pkg = bench.load_package()
host = pkg.HostScene("scenes/trimesh2.ray")
dev = pkg.DeviceScene(host, 0)
opts = pkg.RenderOptions.from_cli("-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05".split())
dev.render(opts, want_f64=False)
t = time.time(); dev.render(opts, want_f64=False); print(os.environ.get("RTX_MEGAKERNEL", "wf"), os.environ.get("RTX_SLOTS", "-"), "ms", (time.time() - t) * 1e3, flush=True)
