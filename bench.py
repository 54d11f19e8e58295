#!/usr/bin/env python3
"""Benchmark: Mrays/s + frame ms of the headline config (BASELINE.json):
trimesh2.ray (stand-in, tools/gen_scenes.py) at 1920x1080, depth 5, 4x4
regular AA (`ray -w 1920 -r 5 -O r -A 4`).

One step = one frame.  On N GPUs (one process per GPU, torch.distributed over
RCCL) the frame is cut into 16x16 tiles dealt round-robin along rotated rows
(diagonal stripes, deal index % N == rank),
each rank renders its tiles into a packed HBM buffer and rank 0 gathers them
over xGMI (dist.gather) — total work is fixed, so scaling is strong.
`python3 bench.py --gpus N` starts the N ranks itself (launch_ranks: child
processes, rendezvous on 127.0.0.1, the first failing rank ends the job);
under `torch.distributed.run --nproc-per-node N ... bench.py --gpus N` the
launcher's ranks are used as they are.

value = rays of the whole frame (camera + reflection/refraction + shadow
queries) / frame wall time, taken as the max over ranks between
barrier+synchronize brackets.  roofline.achieved = algorithmic bytes of one
frame / the frame's GPU time (HIP events on the render stream bracketing all
of the frame's kernels, rtx_kernel_time).  cpu_baseline = the CPU restatement (oracle/, "port") timed on this
host's cores over row bands of the same frame.
"""
import argparse
import hashlib
import importlib.util
import json
import os
import subprocess
import sys
import time

# The CPU leg's OpenMP threads stay on their cores (one per core, packed):
# set before any OpenMP runtime (torch's or the oracle's) initialises
# (the affinity mask as the job got it: once an OpenMP runtime binds the
# initial thread to its first place, sched_getaffinity reports that place)
_AFFINITY0 = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
os.environ.setdefault("OMP_PROC_BIND", "close")
os.environ.setdefault("OMP_PLACES", "cores")
# Consecutive frames overlap on the scene's frame contexts (three on frames
# of at most 10 M units, two above), each with its slot groups on streams of
# its own (rtx_render, DESIGN.md "Frame contexts"): with HIP's default of 4
# hardware queues per process, the contexts' group streams share queues and frame k + 1 queues behind frame k's tail
# (kernel trace, profiles/r04i_timeline_q4.txt).  The environment may hold the
# default explicitly (the GPU box does), so a lower value is raised.  Read
# when HIP initialises.
_HWQ_ENV = os.environ.get("GPU_MAX_HW_QUEUES")  # as the job got it (reported in the line)
if int(_HWQ_ENV or 0) < 16:
    if _HWQ_ENV:
        print(f"bench.py: GPU_MAX_HW_QUEUES={_HWQ_ENV} in the environment raised to 16 (the frame contexts' "
              "nine group streams need queues of their own)", file=sys.stderr)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "Mrays/sec + frame ms, trimesh2.ray 1920×1080 depth-5 4×AA; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per unit: ray in + hit out, BVH node, object
# record, triangle record, material record per shade
# (a BVH box test reads one 32-B entry of a 128-B 4-wide float record)
B_RAY, B_NODE, B_OBJ, B_TRI, B_SHADE = 48 + 72, 32, 224, 96, 176
# VALU issue ceiling (MI355X_MICROARCH.md: 256 CUs x 4 SIMDs at 2.4 GHz).  A
# CDNA4 SIMD is 32 lanes wide (MI355X_MICROARCH.md "Terms", "Wave
# scheduling", per-instruction table: v_fma_f32 wave64 2 cycles of
# throughput), so a wave64 VALU instruction occupies its SIMD for 2 cycles;
# FP64 runs at half the FP32 rate (78.6 vs 157.3 TFLOP/s vector), 4 cycles.
# The ceiling is priced in SIMD cycles: 2 per non-FP64 and 4 per FP64
# wave-instruction (the FP64 share from the PMC classes ADD/MUL/FMA/TRANS_F64).
N_CU, SIMD_PER_CU, CLOCK_HZ = 256, 4, 2.4e9
SIMD_CYCLES_PER_S = N_CU * SIMD_PER_CU * CLOCK_HZ
VALU_CYC, VALU_CYC_F64 = 2, 4
VALU_PEAK = SIMD_CYCLES_PER_S / VALU_CYC  # non-FP64 wave-instructions per second


def kernel_bytes(w):
    """algorithmic bytes of one kernel class's work (rtx_last_work)"""
    return (B_RAY * w["queries"] + B_NODE * w["node_visits"] + B_OBJ * w["object_tests"] +
            B_TRI * w["tri_tests"] + B_SHADE * w["shades"])
LIB = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "lib", "librtx_hip.so")


def load_package():
    name = "cs378hgraphics_raytracer_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "cs378hgraphics-raytracer_amd",
                                                                     "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def ensure_built(pkg_dir):
    if not os.path.exists(os.path.join(pkg_dir, "lib", "librtx_hip.so")):
        subprocess.run(["make", "-C", pkg_dir, "-j8", "all"], check=True)


def file_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def build_id():
    """git head the libraries were built from (lib/BUILD_ID, written by make)"""
    p = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "lib", "BUILD_ID")
    return open(p).read().strip() if os.path.exists(p) else None


def host_cpu():
    """CPU model, logical CPUs of the host, and the share this job may use
    (affinity mask, cgroup CPU quota)."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ncpu = os.cpu_count() or 1
    aff = _AFFINITY0
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    share = aff if quota is None else max(1, min(aff, int(quota)))
    return model, ncpu, aff, quota, share


def cpu_baseline(pkg, path, opts, height, budget_s=10.0, repeats=3, o0=False):
    """Time the CPU restatement (oracle/, OpenMP over pixels, every core this
    job may use) on the same frame: the whole frame when one render fits in
    ~budget_s of CPU time (median of 3 full renders), else row
    bands spread over the image with the band height calibrated to ~budget_s;
    the median of `repeats` runs is reported.  o0: the restatement built at
    the reference's own -O0 (ray/cmake/env.cmake:9) — BASELINE.md's labelled
    context row, never the denominator."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg

    libp = oracle.LIB_O0 if o0 else oracle.LIB
    if not os.path.exists(libp):
        oracle.build()
    model, ncpu, aff, quota, share = host_cpu()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or share
    w = opts.width
    nb = 4
    y_centres = [int(height * (k + 0.5) / nb) for k in range(nb)]

    def bands(band):
        if band >= height:  # the whole frame
            r = oracle.render(pkg, path, opts, threads=threads, want_hits=False, lib_path=libp)
            return r["stats"]["rays"], r["stats"]["kernel_ms"] * 1e-3
        rays, secs = 0, 0.0
        for yc in y_centres:
            y0 = max(0, min(height - band, yc - band // 2))
            r = oracle.render(pkg, path, opts, rect=(0, y0, w, y0 + band), threads=threads, want_hits=False,
                              lib_path=libp)
            secs += r["stats"]["kernel_ms"] * 1e-3  # render loop only, parse excluded
            rays += r["stats"]["rays"]
        return rays, secs

    band = 2
    while True:  # calibrate: whole frame if it fits the budget, else the band height
        rays, secs = bands(band)
        full_est = secs * height / (nb * band)
        if full_est <= budget_s:
            band = height
            break
        if secs >= budget_s * 0.5 or band >= height // nb:
            break
        band = min(height // nb, max(band + 1, int(band * min(8.0, budget_s / max(secs, 1e-3)))))
    runs = [bands(band) for _ in range(repeats)]
    rates = sorted(r / s / 1e6 for r, s in runs)
    med = rates[len(rates) // 2]
    what = (f"the whole frame ({runs[0][0]} rays per run)" if band >= height else
            f"{nb} bands of {band} rows x {w} px of the same frame ({runs[0][0]} rays per run)")
    return {"value": med, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpus": ncpu, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "runs_mrays_s": [round(x, 3) for x in rates], "full_frame": band >= height,
            "spread": round((rates[-1] - rates[0]) / med, 4),
            "omp": {"proc_bind": os.environ.get("OMP_PROC_BIND"), "places": os.environ.get("OMP_PLACES")},
            "sample": (f"CPU restatement (oracle/, g++ {'-O0, the reference build flags (ray/cmake/env.cmake:9): a context row, never the denominator' if o0 else '-O2'}, "
                       f"OpenMP {threads} threads) on {what}, median of {repeats} runs"),
            "_band": band, "_threads": threads}


def parity_block(pkg, dev, path, opts, height, band, threads, timed_rgb8=None):
    """Parity of the benchmarked frame (untimed, after the CPU leg): the frame
    rendered again into host buffers with its per-sample hit records, against
    the CPU restatement's under the north-star bar of tests/parity.py — over
    the whole frame when the CPU leg rendered it whole, else over the CPU
    leg's row bands.  timed_rgb8: the last timed frame itself (rendered into
    HBM on the overlapping frame contexts), compared byte for byte with that
    host-buffer render over the whole frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle  # test infrastructure: the checker
    from parity import RGB_TOL, measure

    gpu = dev.render(opts, want_f64=True, want_hits=True)
    if band >= height:
        rows = [(0, height)]
    else:
        nb = 4
        rows = []
        for k in range(nb):
            yc = int(height * (k + 0.5) / nb)
            y0 = max(0, min(height - band, yc - band // 2))
            rows.append((y0, y0 + band))
    sel = np.concatenate([np.arange(a, b) for a, b in rows])
    ref_rgb = np.zeros_like(gpu["rgb"])
    ref_rgb8 = np.zeros_like(gpu["rgb8"])
    ref_hits = None
    for a, b in rows:
        r = oracle.render(pkg, path, opts, rect=(0, a, opts.width, b) if (a, b) != (0, height) else None,
                          threads=threads, want_hits=True)
        ref_rgb[a:b], ref_rgb8[a:b] = r["rgb"][a:b], r["rgb8"][a:b]
        if ref_hits is None:
            ref_hits = np.zeros_like(gpu["hits"])
        ref_hits[a:b] = r["hits"][a:b]
        del r
    m = measure(gpu["rgb"][sel], gpu["rgb8"][sel], ref_rgb[sel], ref_rgb8[sel], gpu["hits"][sel], ref_hits[sel])
    m["rows"] = "whole frame" if band >= height else [list(x) for x in rows]
    m["tolerance_rgb"] = RGB_TOL
    ok_timed = True
    if timed_rgb8 is not None:
        t8 = timed_rgb8.reshape(gpu["rgb8"].shape)
        m["timed_frame_rgb8_mismatch"] = int(np.count_nonzero(np.any(t8 != gpu["rgb8"], axis=-1)))
        m["timed_frame_pixels"] = int(t8.shape[0] * t8.shape[1])
        ok_timed = m["timed_frame_rgb8_mismatch"] == 0
    m["pass"] = bool(m["max_abs_rgb"] <= RGB_TOL and m["rgb8_mismatch"] == 0 and m["hit_mismatch"] == 0 and
                     m["t_mismatch"] == 0 and m["nan_mismatch"] == 0 and ok_timed)
    return m


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rehearsal():
    """RTX_BENCH_REHEARSAL=1: every rank on device 0 and the gather over gloo
    through host memory — the N-rank path (launch, shards, gather, timing
    over ranks, the JSON line) exercised on a one-GPU box, where RCCL cannot
    put two ranks on one device.  Its numbers are not an N-GPU measurement
    (the ranks share one GPU) and its line says so."""
    return os.environ.get("RTX_BENCH_REHEARSAL", "0") == "1"


def launch_ranks(n, argv, probe=False, grace_s=10.0):
    """`bench.py --gpus N` without an external launcher: start N rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    rendezvous on 127.0.0.1) and return the job's exit code.  The parent
    touches neither HIP nor torch.cuda beyond counting devices (which does not
    initialise the runtime) and never execs: the ranks are children.  The
    first rank to fail ends the others (SIGTERM, then SIGKILL after
    `grace_s`), and its exit code is the job's — the counterpart of the
    product driver's failure path (csrc/host/multi_gpu.cpp)."""
    import signal

    if not probe and not _rehearsal():
        import torch

        ndev = torch.cuda.device_count()
        if ndev < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, {ndev} visible", file=sys.stderr, flush=True)
            return 3
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))

    def stop_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_term(signum, _frame):  # the job's own time limit: take the ranks along
        stop_all(signal.SIGKILL)
        sys.exit(128 + signum)

    old = signal.signal(signal.SIGTERM, on_term)
    rc = 0
    try:
        live = set(range(n))
        while live and rc == 0:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0:
                    print(f"bench.py: rank {r} of {n} exited with {c}; ending the other ranks", file=sys.stderr,
                          flush=True)
                    rc = c if c > 0 else 128 - c
                    break
            time.sleep(0.05)
        if rc != 0:
            stop_all(signal.SIGTERM)
            t_end = time.monotonic() + grace_s
            while any(p.poll() is None for p in procs) and time.monotonic() < t_end:
                time.sleep(0.05)
            stop_all(signal.SIGKILL)
        for p in procs:
            p.wait()
    finally:
        signal.signal(signal.SIGTERM, old)
    return rc


def launch_probe(args):
    """Rank body of `--launch-probe` (CPU test of launch_ranks): report the
    rendezvous environment, run one gloo all-reduce over the ranks, and fail
    on request — no device is touched."""
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if rank == args.launch_probe_fail:
        sys.exit(7)
    if args.launch_probe_fail >= 0:
        time.sleep(600)  # another rank fails: the launcher must end this one
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "rank_sum": int(t.item()), "master": os.environ["MASTER_ADDR"],
                          "local_ranks": world}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one rank each (default 1; under torch.distributed.run: WORLD_SIZE)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-probe-fail", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "trimesh2.ray"))
    ap.add_argument("--flags", default="-w 1920 -r 5 -O r -A 4")
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU work per baseline run")
    ap.add_argument("--no-parity", action="store_true", help="skip the parity block of the timed frame")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-measured HBM bytes per launch (tools/profile_traffic.sh output)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        # no launcher around us: --gpus N > 1 starts the N ranks itself
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            print("bench.py: --gpus must be >= 1", file=sys.stderr)
            sys.exit(2)
        if n > 1 or args.launch_probe:
            if not args.launch_probe:  # host-only preparation, before any rank starts
                ensure_built(os.path.join(ROOT, "cs378hgraphics-raytracer_amd"))
                if not os.path.exists(args.scene):
                    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_scenes.py")], check=True,
                                   stdout=subprocess.DEVNULL)
            sys.exit(launch_ranks(n, sys.argv[1:], probe=args.launch_probe))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
        sys.exit(2)
    if args.launch_probe:
        launch_probe(args)
        return
    pkg_dir = os.path.join(ROOT, "cs378hgraphics-raytracer_amd")
    if rank == 0 or world == 1:
        ensure_built(pkg_dir)
    import torch
    import torch.distributed as dist

    rehearsal = _rehearsal() and world > 1
    if rehearsal:
        local_rank = 0
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    # (under an external launcher the scenes may not exist yet: rank 0 makes
    # them, the others wait at the barrier; launch_ranks made them already)
    if not os.path.exists(args.scene) and rank == 0:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_scenes.py")], check=True,
                       stdout=subprocess.DEVNULL)
    if world > 1:
        dist.barrier()
    pkg = load_package()
    opts = pkg.RenderOptions.from_cli(args.flags.split())
    host = pkg.HostScene(args.scene)
    height = host.height_for(opts.width)
    dev = pkg.DeviceScene(host, local_rank)
    cdev = "cpu" if rehearsal else "cuda"  # where the collectives' tensors live (gloo: host memory)
    tile = args.tile if world > 1 else 0
    packed = world > 1
    npix = pkg.shard_pixels(opts, height, tile, rank, world, packed)
    rgb8 = torch.zeros(npix * 3, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    # counting pass (untimed): rays and traversal work of this rank's share
    st = dev.render(opts, want_f64=False, stats=True, tile=tile, shard=rank, nshards=world, packed=packed)["stats"]
    dev.kernel_time()  # drop the counting launch's events
    gather_list = None
    if world > 1 and rank == 0:
        gather_list = [torch.zeros(pkg.shard_pixels(opts, height, tile, r, world, True) * 3, dtype=torch.uint8,
                                   device=cdev) for r in range(world)]
        # dist.gather needs equal sizes: pad to the largest shard
        mx = max(g.numel() for g in gather_list)
        gather_list = [torch.zeros(mx, dtype=torch.uint8, device=cdev) for _ in range(world)]
    if world > 1:
        mx = torch.tensor([rgb8.numel()], device=cdev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        send = torch.zeros(int(mx.item()), dtype=torch.uint8, device=cdev)

    def step():
        dev.render_device(opts, rgb8.data_ptr(), 0, stream, tile=tile, shard=rank, nshards=world, packed=packed)
        if world > 1:
            send[: rgb8.numel()].copy_(rgb8)
            dist.gather(send, gather_list, dst=0)

    # settle (untimed, before the W warmups): a frame's first render on each
    # frame context sizes its buffers for the default slot pool, and the
    # renders after it resize them once to the frame's fork history (a
    # hipMalloc / hipFree that waits for the device) — 3 frames cover both
    # contexts
    for _ in range(3):
        step()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dev.kernel_time()
    dev.frame_status()  # (raises if a frame so far came out wrong: rtx_frame_status)
    dev.overlap_count()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the frames' GPU time: HIP events on the render stream (where every
    # frame's work joins, for its reduce) around the K frames — consecutive
    # frames overlap on the frame contexts, so one frame's own event span
    # (rtx_kernel_time) would count the overlap twice
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    kms, nlaunch = dev.kernel_time()
    # every timed frame came out right (a wrong one raises: the line is not
    # printed), and how many of them ran on the alternating frame contexts
    frame_check = dev.frame_status()
    pipelined, renders = dev.overlap_count()
    n_ctx = dev.frame_contexts()
    # the last timed frame, for the byte comparison in the parity block
    timed_rgb8 = rgb8.cpu().numpy() if world == 1 else None
    # one frame alone (the frame before it finished, no overlap): the
    # latency of a frame, beside the throughput of back-to-back frames
    lat = []
    for _ in range(3):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t1) * 1e3)
    frame_latency_ms = sorted(lat)[1]
    dev.kernel_time()  # (not part of the roofline's frames)
    if world > 1:
        t = torch.tensor([frame_latency_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        frame_latency_ms = float(t.item())
    dev.frame_status()  # (the latency frames too)
    # N > 1: the gathered frame (the last one: every rank rendered its tiles
    # into HBM on the overlapping frame contexts, rank 0 gathered them) against
    # rank 0's own host-buffer render of the whole frame, byte for byte
    gather_check = None
    if world > 1 and rank == 0:
        import numpy as np

        full = np.zeros((height, opts.width, 3), np.uint8)
        for r in range(world):
            n = pkg.shard_pixels(opts, height, tile, r, world, True) * 3
            pkg.unpack_tiles(gather_list[r][:n].cpu().numpy(), opts.width, height, tile, r, world, full)
        ref = dev.render(opts, want_f64=False)["rgb8"].reshape(full.shape)
        gather_check = {"rgb8_mismatch_pixels": int(np.count_nonzero(np.any(full != ref, axis=-1))),
                        "pixels": int(height * opts.width),
                        "against": "rank 0's host-buffer render of the whole frame"}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([st["rays"]], dtype=torch.int64, device=cdev)
        dist.all_reduce(tot)
        frame_rays = int(tot.item())
    else:
        frame_rays = st["rays"]
    shadow_skipped = st["shadow_rays"] - st["shadow_traced"]
    if world > 1:
        t = torch.tensor([shadow_skipped], dtype=torch.int64, device=cdev)
        dist.all_reduce(t)
        shadow_skipped = int(t.item())
    traced_rays = frame_rays - shadow_skipped
    ms_per_step = elapsed / args.steps * 1e3
    value = frame_rays * args.steps / elapsed / 1e6

    if rank == 0:
        # the default wavefront path renders a frame as a few dozen iterations
        # of advance_fused_kernel + trace_kernel<closest, fused> (closest hit +
        # shading) + trace_kernel<next, fused> (whole shadow walks) on 3
        # streams, then tail_fused_kernel and reduce_kernel (launches_per_frame:
        # the library's count of its kernel launches, rtx_kernel_time), so the
        # roofline is priced per frame: algorithmic bytes of
        # one frame / GPU time of one frame (the event pair around the K
        # timed frames on the render stream, / K; frame_span_ms is one
        # frame's own span, rtx_kernel_time, which overlaps the frames
        # beside it).  With RTX_MEGAKERNEL=1 the frame is one render_kernel
        # launch.
        launches_per_frame = nlaunch / max(1, args.steps)
        mega = os.environ.get("RTX_MEGAKERNEL", "0") not in ("", "0")
        avg_kernel_ms = gpu_ms / max(1, args.steps)
        frame_span_ms = kms / max(1, args.steps)  # one frame's own first-to-last-kernel span (overlaps its neighbours)
        algo_bytes = (B_RAY * st["rays"] + B_NODE * st["node_visits"] + B_OBJ * st["object_tests"] +
                      B_TRI * st["tri_tests"] + B_SHADE * st["shades"])
        achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
        # PMC-measured HBM bytes of one frame (tools/profile_traffic.sh): only
        # from a pass over this very library build, flags and GPU count
        traffic, traffic_src, totals = None, None, {}
        lib_hash = file_sha256(LIB)
        if os.path.exists(args.traffic):
            try:
                with open(args.traffic) as f:
                    tr = json.load(f)
                if (tr.get("flags") == args.flags and tr.get("n_gpus", 1) == world and
                        tr.get("lib_sha256") == lib_hash):
                    traffic = tr.get("hbm_bytes_per_launch")
                    totals = tr.get("totals", {})
                    traffic_src = {"file": os.path.relpath(args.traffic, ROOT), "tag": tr.get("tag"),
                                   "build_id": tr.get("build_id")}
            except (OSError, ValueError):
                traffic = None
        # VALU issue ceiling (SURVEY 8(d)'s FP64-VALU secondary bound), from
        # the same stamped PMC passes: VALU wave-instructions of one frame /
        # the frame's GPU time / the issue peak = the measured share of VALU
        # issue cycles
        valu = totals.get("SQ_INSTS_VALU")
        f64 = sum(totals.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                                 "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
        valu_cycles = (VALU_CYC * (valu - f64) + VALU_CYC_F64 * f64) if valu else None
        frac_valu = round(valu_cycles / (avg_kernel_ms * 1e-3) / SIMD_CYCLES_PER_S, 4) if valu else None
        frac_hbm = round(traffic / (avg_kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None
        # the ceiling the frame is closer to, by the measured fractions
        # the roofline priced is HBM's (north star: achieved HBM GB/s against
        # the gfx950 peak; no MFMA on this path).  What limits the frame is
        # named beside it from the measured fractions: a ceiling past half its
        # peak, else dependent-load latency (neither is)
        bound = "hbm"
        fr = {"valu": frac_valu or 0.0, "hbm": frac_hbm or 0.0}
        top = max(fr, key=fr.get)
        limiter = top if fr[top] >= 0.5 else "latency"
        kernels = st.get("kernels") or {}
        for w in kernels.values():
            w["algorithmic_bytes"] = kernel_bytes(w)
        cpu, parity, cpu_o0 = None, None, None
        if not args.no_cpu and world == 1:
            cpu = cpu_baseline(pkg, args.scene, opts, height, args.cpu_budget)
            band, threads = cpu.pop("_band"), cpu.pop("_threads")
            # BASELINE.md's optional context row: the restatement at the
            # reference's -O0, a bounded sample (a few row bands), one run
            cpu_o0 = cpu_baseline(pkg, args.scene, opts, height, min(args.cpu_budget, 5.0), repeats=1, o0=True)
            cpu_o0.pop("_band"), cpu_o0.pop("_threads")
            if not args.no_parity:
                parity = parity_block(pkg, dev, args.scene, opts, height, band, threads, timed_rgb8)
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (procedural trimesh2 stand-in scene, tools/gen_scenes.py seed 2; reference scene absent)",
            "config": {"workload": f"trimesh2 {opts.width}x{height} {args.flags}", "scene": os.path.basename(args.scene),
                       "triangles": host.info.n_faces, "rays_per_frame": frame_rays, "tile": tile or None,
                       "parallelism": ((f"REHEARSAL: {world} ranks sharing one GPU, gloo gather through host memory"
                                        " (not an N-GPU measurement)") if rehearsal else
                                       f"tile-shard x{world} + RCCL gather" if world > 1 else "single GPU")},
            "roofline": {"bound": bound, "limiter": limiter if (frac_valu or frac_hbm) else None, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         # measured: PMC HBM bytes of a frame / the frame's GPU time / peak
                         "frac_hbm": frac_hbm,
                         # measured: SIMD cycles the frame's VALU instructions occupy (2 per
                         # wave64 instruction on a 32-lane SIMD, 4 for FP64) / GPU time /
                         # SIMD cycles available (256 CUs x 4 SIMDs x 2.4 GHz)
                         "frac_valu": frac_valu,
                         "valu_insts": valu, "valu_f64_insts": f64 or None, "valu_simd_cycles": valu_cycles,
                         "valu_cycles_per_inst": {"non_f64": VALU_CYC, "f64": VALU_CYC_F64},
                         "simd_cycles_per_s": SIMD_CYCLES_PER_S,
                         "traffic_source": traffic_src,
                         "kernel": ("render_kernel<false,false> (megakernel, 1 launch per frame)" if mega else
                                    "frame: trace_kernel<false,1,true,*,true> (first camera rays), then "
                                    "advance_fused_kernel + trace_kernel<false,1,true,*> (closest hit + shading) + "
                                    "trace_kernel<false,2,true> (shadow walks) iterations on 3 streams, "
                                    "tail_fused_kernel, reduce_kernel; GPU time = HIP events on the render stream "
                                    "around the K frames / K"),
                         "avg_kernel_ms": round(avg_kernel_ms, 3), "frame_span_ms": round(frame_span_ms, 3),
                         "launches_per_frame": launches_per_frame,
                         "algorithmic_bytes_per_launch": algo_bytes},
            "cpu_baseline": cpu,
            "cpu_baseline_O0": cpu_o0,
            # the timed frame against the CPU restatement (tests/parity.py bar)
            "parity": parity,
            # traversal work of one frame (the counting pass of the same kernels)
            "work": dict({k: st[k] for k in ("rays", "camera_rays", "secondary_rays", "shadow_rays",
                                             "shadow_traced", "node_visits", "object_tests", "tri_tests",
                                             "shades")},
                         # per kernel class (rtx_last_work): closest-hit, next-hit (walk) and tail
                         # launches, with their algorithmic bytes (tools/kernel_roofline.py
                         # divides them by the rocprof kernel times)
                         kernels=kernels),
            # rays counted as the reference traces them vs rays the GPU traced
            # (dark-light shadow rays are counted, not traced: DESIGN.md §2)
            "rays_traced_per_frame": traced_rays,
            # frames are rendered back to back: frame k + 1 starts on the
            # other frame context while frame k finishes; ms_per_step is the
            # throughput, frame_latency_ms one frame rendered alone (render
            # + gather, max over ranks)
            "frame_latency_ms": round(frame_latency_ms, 3),
            # timed frames that ran pipelined on the frame contexts (how many
            # contexts: rtx_frame_contexts; rtx_overlap_count), and the frame
            # check of the timed frames
            # (rtx_frame_status: first wrong frame, wrong frames)
            "frame_contexts": n_ctx if pipelined == renders and renders > 0 else (1 if pipelined == 0 else "mixed"),
            "pipelined_frames": [pipelined, renders],
            "frame_check": {"first_bad": frame_check[0], "bad_frames": frame_check[1]},
            "gather_check": gather_check,
            "gpu_max_hw_queues": {"effective": os.environ.get("GPU_MAX_HW_QUEUES"), "environment": _HWQ_ENV},
            "mrays_traced_per_s": round(traced_rays * args.steps / elapsed / 1e6, 3),
            "build": {"build_id": build_id(), "lib_sha256": lib_hash},
        }
        if cpu:
            line["gpu_over_cpu"] = round(value / cpu["value"], 2)
            line["gpu_traced_over_cpu"] = round(line["mrays_traced_per_s"] / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
