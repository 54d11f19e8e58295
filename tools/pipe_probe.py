#!/usr/bin/env python3
"""Frame pipelining estimate on ONE GPU: consecutive frames of the same shard
rendered by two device contexts (two DeviceScenes = two sets of frame
buffers and group streams) on two streams, so frame k + 1's throughput phase
can overlap frame k's latency-bound last iterations.  Prints, per N, the
slowest rank's per-frame time with and without the overlap.
usage (GPU box): python tools/pipe_probe.py [--scene S] [--flags F] [--frames K] [N ...]"""
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
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch

    pkg = bench.load_package()
    args = sys.argv[1:]
    flags, scene, K = "-w 1920 -r 5 -O r -A 4", "trimesh2.ray", 6
    while args and args[0] in ("--flags", "--scene", "--frames"):
        if args[0] == "--flags":
            flags = args[1]
        elif args[0] == "--scene":
            scene = args[1]
        else:
            K = int(args[1])
        args = args[2:]
    ns = [int(a) for a in args] or [1, 8]
    opts = pkg.RenderOptions.from_cli(flags.split())
    host = pkg.HostScene(os.path.join(ROOT, "scenes", scene))
    devs = [pkg.DeviceScene(host, 0), pkg.DeviceScene(host, 0)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    h = host.height_for(opts.width)
    for n in ns:
        seq, pipe = [], []
        for r in range(n):
            tile = 16 if n > 1 else 0
            npix = pkg.shard_pixels(opts, h, tile, r, n, n > 1)
            outs = [torch.zeros(npix * 3, dtype=torch.uint8, device="cuda") for _ in range(2)]

            def frame(k):
                dev, s, o = devs[k & 1], streams[k & 1], outs[k & 1]
                dev.render_device(opts, o.data_ptr(), 0, s.cuda_stream, tile=tile, shard=r, nshards=n, packed=n > 1)

            for k in range(2):  # warm both contexts
                frame(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):  # one context, frame after frame
                devs[0].render_device(opts, outs[0].data_ptr(), 0, streams[0].cuda_stream, tile=tile, shard=r,
                                      nshards=n, packed=n > 1)
            torch.cuda.synchronize()
            seq.append((time.perf_counter() - t0) / K * 1e3)
            t0 = time.perf_counter()
            for k in range(K):  # two contexts alternating: frames overlap
                frame(k)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) / K * 1e3)
        print(json.dumps({"scene": scene, "flags": flags, "n": n, "seq_max_ms": round(max(seq), 3),
                          "pipe_max_ms": round(max(pipe), 3), "seq_ms": [round(x, 2) for x in seq],
                          "pipe_ms": [round(x, 2) for x in pipe]}), flush=True)


if __name__ == "__main__":
    main()
