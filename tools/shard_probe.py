#!/usr/bin/env python3
"""Per-rank frame time of the tile-sharded headline frame, measured on ONE
GPU (back-to-back frames, which overlap on the scene's frame contexts,
and one frame alone): rank r of N renders tiles t % N == r (what bench.py --gpus N runs on
each GPU).  The slowest shard's time bounds the N-GPU frame (plus the RCCL
gather of a few MB).  Prints one JSON line per N.
usage (GPU box): python tools/shard_probe.py [--scene NAME.ray] [--flags "-w 1920 ..."] [--rank R] [--tile T] [N ...]
(--rank R: only rank R of each N > 1, e.g. for a kernel trace of one shard;
 --own-stream: a created stream, not the default one)
(dragon.ray, C5's scene, is generated when missing: tools/gen_scenes.py --dragon)"""
import json
import os

# frame contexts: 2 x 3 slot-group streams want their own hardware queues; the
# environment may hold HIP's default of 4 (the GPU box does), so raise it
import sys  # (before the queue override below)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    if os.environ.get("GPU_MAX_HW_QUEUES"):
        print(f"{os.path.basename(__file__)}: GPU_MAX_HW_QUEUES={os.environ['GPU_MAX_HW_QUEUES']} raised to 16",
              file=sys.stderr)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch

    pkg = bench.load_package()
    args = sys.argv[1:]
    flags = "-w 1920 -r 5 -O r -A 4"
    scene = "trimesh2.ray"
    only_rank = None
    own_stream = False
    tile_px = 16  # bench.py's default
    while args and args[0] in ("--flags", "--scene", "--rank", "--own-stream", "--tile"):
        if args[0] == "--own-stream":  # render on a created stream instead of torch's default (null) stream
            own_stream = True
            args = args[1:]
            continue
        if args[0] == "--flags":
            flags = args[1]
        elif args[0] == "--rank":
            only_rank = int(args[1])
        elif args[0] == "--tile":
            tile_px = int(args[1])
        else:
            scene = args[1]
        args = args[2:]
    if scene == "dragon.ray" and not os.path.exists(os.path.join(ROOT, "scenes", scene)):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_scenes.py"), "--dragon"], check=True,
                       stdout=subprocess.DEVNULL)
    ns = [int(a) for a in args] or [1, 2, 4, 8]
    opts = pkg.RenderOptions.from_cli(flags.split())
    host = pkg.HostScene(os.path.join(ROOT, "scenes", scene))
    dev = pkg.DeviceScene(host, 0)
    h = host.height_for(opts.width)
    ts = torch.cuda.Stream() if own_stream else torch.cuda.current_stream()
    stream = ts.cuda_stream
    free0 = torch.cuda.mem_get_info()[0]
    for n in ns:
        times, lat = [], []
        for r in range(n):
            if only_rank is not None and n > 1 and r != only_rank:
                continue
            tile = tile_px if n > 1 else 0
            npix = pkg.shard_pixels(opts, h, tile, r, n, n > 1)
            out = torch.zeros(npix * 3, dtype=torch.uint8, device="cuda")
            for _ in range(4):  # warm both frame contexts (buffers, bucket-pool sizes)
                dev.render_device(opts, out.data_ptr(), 0, stream, tile=tile, shard=r, nshards=n, packed=n > 1)
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(6):  # back to back (consecutive frames overlap: frame contexts)
                dev.render_device(opts, out.data_ptr(), 0, stream, tile=tile, shard=r, nshards=n, packed=n > 1)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) / 6 * 1e3)
            one = []
            for _ in range(3):  # one frame alone
                t0 = time.perf_counter()
                dev.render_device(opts, out.data_ptr(), 0, stream, tile=tile, shard=r, nshards=n, packed=n > 1)
                torch.cuda.synchronize()
                one.append((time.perf_counter() - t0) * 1e3)
            lat.append(sorted(one)[1])
        # HBM the library holds beyond the scene (frame buffers grown so far)
        held = (free0 - torch.cuda.mem_get_info()[0]) / 2**30
        print(json.dumps({"scene": scene, "flags": flags, "n": n, "shard_ms": [round(t, 2) for t in times],
                          "max_ms": round(max(times), 2), "latency_ms": [round(t, 2) for t in lat],
                          "max_latency_ms": round(max(lat), 2), "frame_buffers_gb": round(held, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
