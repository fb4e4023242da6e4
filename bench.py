#!/usr/bin/env python3
"""Benchmark: BASELINE.json's headline metric on MI355X.

Workload (BASELINE.json configs[2], the metric's config): the 07_specular_BRDF
scene (reference Main.cu:39-67), 1920x1080, 8 spp (= 8 progressive frames,
accumulatedFrames 1..8), maxBounces 4.  One "step" renders that full 8-spp
frame from scratch (accumulation reset, RNG streams continuing like the
reference's controls() reset) with inputs already resident in HBM, and — for
N > 1 — includes the RCCL gather of the RGBA8 image to rank 0 and the
de-interleave kernel.  The frame is fixed, so N GPUs split it by interleaved
pixel rows: strong scaling.

Metric: Msamples/s (nominal) = W*H*spp*bounces / t / 1e6,
ms/frame = ms_per_step.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
                  [--no-cpu-baseline] [--cpu-threads T] [--dist] [--no-overlap]
The CPU baseline is the library's scalar C++ fallback (rt_render_cpu) on
every CPU of the process's affinity (or --cpu-threads), timed on rank 0 at
N = 1 after the GPU steps, and checked bit-exact against the GPU; in the same
leg the oracle (oracle/, the checker) renders the bench frame (config 4: a
row sample; config 5: none) and the GPU's frame, frameSum and RNG state
must equal it bit for bit ("oracle_check", "verified").
--dist takes the multi-rank code path (process group, gather, de-interleave,
verify) at N = 1 too.
N > 1: one rank per GPU over RCCL.  Under torch.distributed.run (WORLD_SIZE
set) each process is one rank; a plain `python bench.py --gpus N` starts
torch.distributed.run itself (N child ranks on 127.0.0.1) before touching
the GPU, forwards their output and exits with their status.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]

import torch  # noqa: E402  (import torch BEFORE libbwrt: one shared HIP runtime)
import torch.distributed as dist  # noqa: E402

from bwrt import Renderer, abi, scenes  # noqa: E402
from bwrt.dist import ShardPlan, gather_rows  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# closest-hit queries (traced ray segments) per full frame, SURVEY.md §8(d)'s
# "actual segments".  The paths are a deterministic function of the scene and
# the RNG streams (bit-exact with the oracle): c2 / c3 are the oracle's count
# for the first frame from the y*W+x seeds (tests/test_oracle.py checks
# them), c4 / c5 the diagnostic build's count (-DRT_STAMPS,
# tools/stamps_run.py, stamps[16]) for the stream's second frame.  Each bench
# step continues the streams, so a step's count differs by < 0.1 % (c3:
# 32,340,255 first frame, 32,347,861 second).
QUERIES_PER_FRAME = {"c2": 6619930, "c3": 32340255, "c4": 261860320, "c5": 346188412}
BYTES_PER_PIXEL_PASS = 76  # rng 24+24, frameSum 12+12, RGBA8 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(scenes.CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true",
                    help="also at N = 1: re-render from fresh seeds and check the frame against the CPU fallback's "
                         "rows (N > 1 always checks the gathered frame against rank 0's single-GPU render)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: gather each frame before the next render starts (no frame pipelining)")
    ap.add_argument("--dist", action="store_true",
                    help="take the multi-rank path even at N = 1: process group (RCCL unless BWRT_DIST_BACKEND), "
                         "rooted gather of the row blocks, de-interleave kernel, verify against a solo render")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic-json", default=None,
                    help="PMC record of this workload (default: profiles/traffic_<config>.json, then "
                         "profiles/traffic_latest.json; used only when its workload key matches)")
    return ap.parse_args()


SCENE_NAMES = {"01": "01_red_circle", "04": "04_path_tracing", "07": "07_specular_BRDF", "stress": "stress_10k"}
SCENE_DATA = {
    "01": "reference scene 01 (one red sphere)",
    "04": "reference scene 04 (07 spheres 0,1,4,5 + floor)",
    "07": "reference scene 07 (Main.cu:39-67)",
    "stress": "stress scene (10,000 triangles + 256 spheres + floor, xorshift32 seed, bwrt/scenes.py)",
}


# CPU-baseline sample: a row shard (every k-th row) of the bench frame, so
# the scalar fallback's run stays within seconds on the big configs
CPU_SAMPLE_ROW_STRIDE = {"c1": 1, "c2": 1, "c3": 1, "c4": 4, "c5": 27}
CPU_MIN_REPS, CPU_MIN_S = 3, 2.0  # the CPU-baseline sample: repeated, median reported


def cpu_quota():
    """CPUs of this process's cgroup quota (cpu.max), or None if unlimited."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if quota == "max" else float(quota) / float(period)
    except (OSError, ValueError):
        return None


def cpu_baseline(lib, config, scene_key, w, h, spp, mb, threads, gpu_renderer=None):
    """The product's scalar C++ CPU fallback (rt_create_cpu / rt_render_cpu:
    the kernels' per-ray arithmetic compiled for the host, one pixel per loop
    iteration, std::thread pool) timed on the host cores — the reported CPU
    baseline ("fallback"), never the measured product.  With gpu_renderer the
    sample is also rendered on the GPU from the same seeds and compared."""
    stride = CPU_SAMPLE_ROW_STRIDE.get(config, 1)
    aff = len(os.sched_getaffinity(0))
    threads = threads if threads > 0 else lib.rt_cpu_threads()  # affinity capped by the cgroup quota
    scene = scenes.SCENES[scene_key]()
    with Renderer.cpu(threads, lib=lib) as c:
        c.set_scene(scene)
        c.init_rand(w, h, 0, stride)
        c.render(w, h, 1, mb, first_frame=1, row_stride=stride)  # warm (pages, threads)
        # the sample rendered again from the same seeds until CPU_MIN_S of
        # wall time (at least CPU_MIN_REPS times): the median rep is reported
        times, t_all = [], time.perf_counter()
        while len(times) < CPU_MIN_REPS or time.perf_counter() - t_all < CPU_MIN_S:
            c.init_rand(w, h, 0, stride)
            t0 = time.perf_counter()
            img = c.render(w, h, spp, mb, first_frame=1, row_stride=stride)
            times.append(time.perf_counter() - t0)
        dt = sorted(times)[len(times) // 2]
    rows = img.shape[0]
    out = {"value": round(rows * w * spp * mb / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads,
           # a port of the reference's algorithm to scalar C++ (north_star's
           # "scalar C++ CPU fallback of the same kernel"): the product's
           # rt_render_cpu, bit-exact with the GPU and with the oracle
           "kind": "port", "impl": "libbwrt.so rt_render_cpu (csrc/rt_cpu.cpp over csrc/rt_path.h)",
           "ms_per_sample": round(dt * 1e3, 2), "reps": len(times),
           "ms_per_sample_min_max": [round(min(times) * 1e3, 2), round(max(times) * 1e3, 2)],
           "sample": f"{'one full' if stride == 1 else f'rows y = 0 mod {stride} of one'} {w}x{h} {spp}-spp "
                     f"{mb}-bounce frame of scene {scene_key} ({rows} rows; libbwrt.so rt_render_cpu, "
                     f"{threads} threads; sched affinity {aff} CPUs, cgroup quota "
                     f"{cpu_quota() or 'none'})"}
    if stride == 1:
        out["ms_per_frame"] = out["ms_per_sample"]
    if gpu_renderer is not None:
        gpu_renderer.init_rand(w, h, 0, stride)
        g = gpu_renderer.render(w, h, spp, mb, first_frame=1, row_stride=stride)
        out["bit_exact_vs_gpu"] = bool((g == img).all())
    return out


# Oracle check in the CPU-baseline leg (the checker, never the measured
# path): the bench frame (config 4: every 4th row) rendered by the oracle (oracle/,
# the C restatement of the reference, OpenMP) and by the GPU from the same
# seeds, compared bit for bit — RGBA8, frameSum and RNG state.  Config 5 is
# left out: the oracle's brute-force loop over 10,256 primitives takes
# minutes per row there (the GPU suite checks it against committed digests).
ORACLE_ROW_STRIDE = {"c1": 1, "c2": 1, "c3": 1, "c4": 4}


def oracle_check(config, scene_key, w, h, spp, mb, gpu_renderer):
    stride = ORACLE_ROW_STRIDE.get(config)
    if not stride:
        return None
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # the checker only (oracle/oracle.py)
    scene = scenes.SCENES[scene_key]()
    t0 = time.perf_counter()
    st = O.render_image(scene, w, h, spp, mb, 0, stride)
    dt = time.perf_counter() - t0
    gpu_renderer.set_scene(scene)
    gpu_renderer.init_rand(w, h, 0, stride)
    img = gpu_renderer.render(w, h, spp, mb, first_frame=1, row_stride=stride)
    rng, acc = gpu_renderer.get_state(st.rows, w)
    exact = (bool(np.array_equal(img, st.rgba)) and bool(np.array_equal(rng, st.rng))
             and bool(np.array_equal(acc, st.accum, equal_nan=True)))
    return {"rows": st.rows, "row_stride": stride, "bit_exact": exact,
            "compared": "RGBA8, frameSum and RNG state after all frames",
            "oracle_ms": round(dt * 1e3, 1), "oracle": "oracle/oracle.c (C restatement of Main.cu:111-315, OpenMP)"}


def load_traffic(paths, workload_key):
    """The first PMC record (tools/make_traffic_json.py) among `paths` whose
    workload key is this run's."""
    for path in paths:
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload_key:
            return t
    return None


def traffic_paths(explicit, config):
    if explicit:
        return [explicit]
    return [os.path.join(REPO, "profiles", f"traffic_{config}.json"),
            os.path.join(REPO, "profiles", "traffic_latest.json")]


# L1 (vector cache) line throughput per CU, tools/micro/ta_gather.hip:
# dependent per-lane 16-byte gathers, 64 distinct 128-byte lines per
# wave-load, cycles per wave-load per CU at 2.4 GHz / 64 — L1-resident lines
# (16 KB footprint: hits, 64.14 cycles) and L2-served lines (4 MB footprint:
# every line an L1 miss, 146.81 cycles) (profiles/r06a/ta_gather_micro.txt)
L1_HIT_CYCLES_PER_LINE = 64.14 / 64
L1_MISS_CYCLES_PER_LINE = 146.81 / 64
L1_MICRO = "profiles/r06a/ta_gather_micro.txt"


RANK_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
            "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")


def self_launch_command(argv, nproc, port):
    """The command and environment that run this script as `nproc` ranks of
    torch.distributed.run on this node (rendezvous on 127.0.0.1:port), with
    the same arguments; each rank then reads RANK / LOCAL_RANK / WORLD_SIZE."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    # a rank identity left in the caller's environment (this process under
    # another launcher) must not leak into the children: torch.distributed.run
    # sets every one of these itself
    env = {k: v for k, v in os.environ.items() if k not in RANK_ENV}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL needs it on this driver
    env.setdefault("OMP_NUM_THREADS", "1")  # torch.distributed.run would print a warning and set it
    return cmd, env


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    args = parse()
    if (args.gpus > 1 or args.dist) and "WORLD_SIZE" not in os.environ:
        # a plain launch for N GPUs: start the N ranks as children.  Nothing
        # here has touched the GPU (importing torch does not), and this
        # process only waits for them: no exec, no retry
        cmd, env = self_launch_command(sys.argv[1:], args.gpus, free_port())
        print(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
        raise SystemExit(subprocess.run(cmd, env=env).returncode)
    scene_key, W, H, SPP, MB, _ = scenes.CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU (LOCAL_RANK); the modulo only matters when ranks
    # are rehearsed on fewer GPUs than ranks (BWRT_DIST_BACKEND=gloo)
    dev_index = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    backend = os.environ.get("BWRT_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
    # the multi-rank path: every N > 1 run, and N = 1 under --dist (the same
    # process group, gather, de-interleave and verify with one rank)
    distributed = world > 1 or args.dist
    if distributed:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    lib = abi.load()
    hip_libs = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
    if len(hip_libs) != 1:
        print(f"warning: {len(hip_libs)} HIP runtimes loaded: {hip_libs}", file=sys.stderr)
    r = Renderer(dev_index, lib=lib)
    # no per-launch start marker inside the library (a marker packet the GPU
    # drains between two launches: 5-7 us per step, tools/ev_ab.sh); the bench
    # brackets its whole timed region with one event pair instead
    # (BENCH_KTIMING=1: library timing on, for that A/B)
    r.set_kernel_timing(os.environ.get("BENCH_KTIMING") == "1")
    scene = scenes.SCENES[scene_key]()
    r.set_scene(scene)
    plan = ShardPlan(H, world, rank)
    rows_per = plan.rows_per_shard
    my_rows = lib.rt_shard_rows(H, plan.row_offset, plan.row_stride)
    assert my_rows == plan.rows
    r.init_rand(W, H, plan.row_offset, plan.row_stride)
    # N > 1: frames are pipelined — frame k's gather + de-interleave run on a
    # second stream while frame k+1 renders (double-buffered row blocks);
    # the timed region still covers every render and every gather
    overlap = distributed and not args.no_overlap
    nbuf = 2 if overlap else 1
    local_imgs = [torch.zeros(rows_per * W, dtype=torch.int32, device=dev) for _ in range(nbuf)]
    full_img = torch.empty(H * W, dtype=torch.int32, device=dev) if rank == 0 else None
    # the gather's landing buffers exist on the root only
    gathered = ([torch.empty((world, rows_per * W), dtype=torch.int32, device=dev) for _ in range(nbuf)]
                if distributed and rank == 0 else [None] * nbuf)
    torch.cuda.synchronize(dev)  # (the zero fills ran on torch's default stream, unordered with the renders)
    # the context's own stream (rt_get_stream), wrapped for torch: the
    # kernel, the bench's timing events and the RCCL gather are all ordered
    # on it, and renders on the context's stream defer the library's end
    # event, so back-to-back steps carry no marker packet between them
    # (BENCH_CALLER_STREAM=1: a torch-created stream instead, for that A/B)
    stream = (torch.cuda.Stream(dev) if os.environ.get("BENCH_CALLER_STREAM") == "1"
              else torch.cuda.ExternalStream(r.stream_handle(), device=dev))
    comm = torch.cuda.Stream(dev) if overlap else stream
    torch.cuda.set_stream(stream)
    ev_rendered = [torch.cuda.Event() for _ in range(nbuf)]
    ev_sent = [torch.cuda.Event() for _ in range(nbuf)]  # block b's last gather has read it
    params = r.params(W, H, SPP, MB, first_frame=1, row_offset=plan.row_offset, row_stride=plan.row_stride)
    counter = [0]

    def step():
        b = counter[0] % nbuf
        counter[0] += 1
        local_img = local_imgs[b]
        if overlap:
            stream.wait_event(ev_sent[b])  # no-op until the event is first recorded
        r.render_device(params, local_img.data_ptr() if distributed else full_img.data_ptr(),
                        stream.cuda_stream)
        if distributed:
            ev_rendered[b].record(stream)
            with torch.cuda.stream(comm):
                comm.wait_event(ev_rendered[b])
                gather_rows(local_img, plan, out=gathered[b])
                if rank == 0:
                    r.deinterleave_device(gathered[b].data_ptr(), full_img.data_ptr(), W, H, world, rows_per,
                                          comm.cuda_stream)
                ev_sent[b].record(comm)

    for _ in range(args.warmup):
        step()
    # HIP events on the launch stream bracket the K timed launches (one pair:
    # events between the steps would put marker packets, ~5 us each, between
    # the launches); the average launch = their span / K, which also covers
    # the order-sort kernel and the launch gaps of each step
    ev_start, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev_start.record(stream)
    for _ in range(args.steps):
        step()
    ev_end.record(stream)
    t_issued = time.perf_counter()  # host time to enqueue the steps (must stay below the GPU time)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_span = ev_start.elapsed_time(ev_end) / args.steps
    launched = r.last_kernel_name()  # the render kernel the launch policy picked for this rank's work
    t = torch.tensor([elapsed, kern_span, t_issued - t0], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_avg_ms, issue_s = float(t[0]), float(t[1]), float(t[2])
    kernel_timing = "event pair around the timed launches on the render stream, / steps"
    if distributed:
        # the timed region's span on the render stream also holds its waits
        # for the gather stream (and, with --no-overlap, the gather itself):
        # the render kernel's own time comes from render-only launches after
        # the timed region (same shard, no gather), max over ranks
        kreps = min(args.steps, 10)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(kreps):
            r.render_device(params, local_imgs[0].data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        k = torch.tensor([e0.elapsed_time(e1) / kreps], dtype=torch.float64, device=dev)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        kern_avg_ms = float(k[0])
        kernel_timing = f"render-only pass of {kreps} launches after the timed region (no gather), max over ranks"

    # parity of the measured path: N > 1 always (the sharded + gathered frame
    # from fresh seeds against rank 0 rendering the whole frame alone); N = 1
    # with --verify (a fresh frame against the CPU fallback on a row sample)
    verified, verify_how = None, None
    if distributed:
        r.init_rand(W, H, plan.row_offset, plan.row_stride)
        step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        if rank == 0:
            got = full_img.cpu()
            solo_r = Renderer(dev_index, lib=lib)
            solo_r.set_scene(scene)
            solo = torch.empty(H * W, dtype=torch.int32, device=dev)
            solo_r.init_rand(W, H)
            solo_r.render_device(solo_r.params(W, H, SPP, MB, first_frame=1), solo.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize(dev)
            solo_r.close()
            verified = bool(torch.equal(got, solo.cpu()))
            verify_how = f"{world}-rank gathered frame (fresh y*W+x seeds) vs rank 0's 1-GPU render, bit for bit"
    elif args.verify:
        verify_rows = CPU_SAMPLE_ROW_STRIDE.get(args.config, 1) * 8
        with Renderer.cpu(0, lib=lib) as c, Renderer(dev_index, lib=lib) as g:
            c.set_scene(scene)
            g.set_scene(scene)
            c.init_rand(W, H, 0, verify_rows)
            g.init_rand(W, H, 0, verify_rows)
            a = c.render(W, H, SPP, MB, first_frame=1, row_stride=verify_rows)
            b = g.render(W, H, SPP, MB, first_frame=1, row_stride=verify_rows)
        verified = bool((a == b).all())
        verify_how = f"rows y = 0 mod {verify_rows} (fresh seeds): GPU vs the CPU fallback, bit for bit"

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        samples = W * H * SPP * MB * args.steps
        value = samples / elapsed / 1e6
        # roofline of the dominant kernel (rank 0's render kernel, as the
        # library reports it: the sorted kernel on full frames, the pair
        # kernel on small shards, the BVH refill kernel for the stress
        # scene), per launch
        units = my_rows * W * SPP  # pixel-passes in one launch on this rank
        alg_bytes = units * BYTES_PER_PIXEL_PASS
        achieved = alg_bytes / (kern_avg_ms * 1e-3) / 1e9
        workload_key = f"{scene_key}-{W}x{H}-{SPP}spp-{MB}b-rows{world}"
        traffic = load_traffic(traffic_paths(args.traffic_json, args.config), workload_key)
        out = {
            "metric": f"Msamples/sec (W*H*spp*bounces/t), {W}x{H} {SPP}spp {MB}-bounce, {SCENE_NAMES[scene_key]}",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: {SCENE_DATA[scene_key]}, per-pixel RNG seeded y*W+x",
            "config": {"workload": f"07_specular_BRDF {W}x{H} {SPP}spp {MB}-bounce (BASELINE configs[2])"
                       if args.config == "c3" else f"{args.config}: scene {scene_key} {W}x{H} {SPP}spp {MB}-bounce",
                       "scene": scene_key, "width": W, "height": H, "spp": SPP, "max_bounces": MB,
                       "parallelism": f"pixel-rows/{world}" + (f" + {'rccl' if backend == 'nccl' else backend} gather" if distributed else "")
                       + (" (frames pipelined: gather of frame k overlaps render of k+1)" if overlap else "")},
            "world_size": world,
            "backend": (("rccl" if backend == "nccl" else backend) if distributed else None),
            "verified": verified,
            "verify": verify_how,
            "ms_per_frame": round(ms_step, 4),
            "kernel_ms_avg": round(kern_avg_ms, 4),
            "kernel_timing": kernel_timing,
            # host time to enqueue one step (render + gather calls), max over ranks
            "host_issue_ms_per_step": round(issue_s / args.steps * 1e3, 4),
            "queries_per_frame": QUERIES_PER_FRAME.get(args.config),
            "actual_Msegments_per_s": (round(QUERIES_PER_FRAME[args.config] * args.steps / elapsed / 1e6, 1)
                                       if args.config in QUERIES_PER_FRAME else None),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": (round(traffic["hbm_bytes_per_launch"]) if traffic else None),
                         "kernel": launched,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "bytes_per_unit": BYTES_PER_PIXEL_PASS, "units_per_launch": units},
        }
        if traffic and traffic.get("valu"):
            # the binding roofline of this branchy fp32 path: VALU issue.
            # peak: 256 CUs x 4 SIMD x 64 lanes / 2 cycles x 2.4 GHz
            v = traffic["valu"]
            ks = kern_avg_ms * 1e-3
            lane_peak = 256 * 4 * 64 / 2 * 2.4e9
            inst_peak = 256 * 4 / 2 * 2.4e9
            out["valu_roofline"] = {
                "bound": "valu", "unit": "lane-ops/s", "peak": lane_peak,
                "achieved": round(v["lane_ops_per_launch"] / ks, 1),
                "frac": round(v["lane_ops_per_launch"] / ks / lane_peak, 4),
                "issue_frac": round(v["insts_valu_per_launch"] / ks / inst_peak, 4),
                "active_lanes_per_valu": round(v["active_lanes_per_valu"], 2),
                "counters": traffic.get("source")}
        if traffic and traffic.get("l1") and "bvh" in (launched or ""):
            # the BVH walk's bound: the L1's line throughput.
            # achieved = the launch's L1 tag accesses (one per distinct line
            # per wave-load) / the kernel's time; peak = 256 CUs x the
            # micro-benchmark's L1-hit rate (1 line per cycle) x 2.4 GHz.
            # model_floor_ms: the launch's hits and misses (L1->L2 requests)
            # each at the micro-benchmark's cycles per line
            l1 = traffic["l1"]
            tags, miss = l1["tag_accesses_per_launch"], l1["l2_requests_per_launch"]
            peak = 256 * 2.4e9 / L1_HIT_CYCLES_PER_LINE
            achieved = tags / (kern_avg_ms * 1e-3)
            floor_ms = ((tags - miss) * L1_HIT_CYCLES_PER_LINE + miss * L1_MISS_CYCLES_PER_LINE) / (256 * 2.4e9) * 1e3
            out["l1_line_roofline"] = {
                "bound": "l1_lines", "unit": "lines/s", "achieved": round(achieved), "peak": round(peak),
                "frac": round(achieved / peak, 4), "tag_accesses_per_launch": round(tags),
                "l2_requests_per_launch": round(miss), "cycles_per_hit_line": round(L1_HIT_CYCLES_PER_LINE, 3),
                "cycles_per_miss_line": round(L1_MISS_CYCLES_PER_LINE, 3), "model_floor_ms": round(floor_ms, 3),
                "model_floor_frac": round(floor_ms / kern_avg_ms, 4), "counters": traffic.get("source"),
                "micro": L1_MICRO}
        if not distributed and not args.no_cpu_baseline:
            torch.cuda.synchronize(dev)
            with Renderer(dev_index, lib=lib) as check:
                check.set_scene(scene)
                out["cpu_baseline"] = cpu_baseline(lib, args.config, scene_key, W, H, SPP, MB, args.cpu_threads,
                                                   gpu_renderer=check)
                oc = oracle_check(args.config, scene_key, W, H, SPP, MB, check)
            if oc is not None:
                out["oracle_check"] = oc
            if out["verified"] is None:
                fb = out["cpu_baseline"]["bit_exact_vs_gpu"]
                if oc is not None:
                    out["verified"] = fb and oc["bit_exact"]
                    out["verify"] = (f"rows y = 0 mod {oc['row_stride']} (fresh seeds): GPU vs the oracle, bit for bit "
                                     "(RGBA8, frameSum, RNG); and the CPU baseline's sample: GPU vs the CPU fallback")
                else:
                    out["verified"] = fb
                    out["verify"] = "the CPU baseline's sample: GPU vs the CPU fallback from the same seeds, bit for bit"
        print(json.dumps(out), flush=True)
    ok = torch.tensor([0 if verified is False else 1], dtype=torch.int32, device=dev)
    if distributed:
        dist.broadcast(ok, 0)
    torch.cuda.synchronize(dev)
    torch.cuda.set_stream(torch.cuda.default_stream(dev))  # the context's stream goes with it
    r.close()
    if distributed:
        dist.destroy_process_group()
    if int(ok[0]) == 0 or (rank == 0 and world == 1 and out.get("verified") is False):
        print("verify FAILED: the measured path's frame differs", file=sys.stderr, flush=True)
        raise SystemExit(1)


if __name__ == "__main__":
    main()
