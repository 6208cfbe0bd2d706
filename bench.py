#!/usr/bin/env python3
"""Benchmark: scans/s of TSDF integration (128x1024 Ouster scans, 5 cm voxels) on N MI355X.

A step integrates one batch of synthetic scans that are already resident in HBM (the C1/M1
workload of SURVEY.md §8d: OS-1-128 1024x10 beams, analytic scene, circular trajectory at 10 Hz,
5 cm voxels, 15 cm truncation, no carving), scan after scan, through libtsdf_hip.so's
tsdf_integrate_batch_device.  Multi-GPU (one process per GPU, torch.distributed over RCCL): rank k
integrates sector k of every scan of the step into its own partial field (tsdf_params.n_sectors /
sector; weak scaling: a step of N GPUs holds N * batch scans, each rank's share is `batch` scans'
worth of rays).  The default sector rule (ABI v10) is the index rule: sector k is the
contiguous k-th 1/N of each scan's points -- the scans are in DLIO's time order, so a column
(azimuth) range of the spin -- and the rank's kernels read only that share; `--sector-rule world`
runs the world-frame pseudo-angle rule, where every rank reads every point and its walk kernels
drop the other sectors' rays.  No collective runs on the data path — the device-resident
border-brick reduce over RCCL (tsdf_map.distributed.border_reduce) is a read-out operation, timed
separately (readout_merge_ms).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "noetic-slam_amd"))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
PROFILE_PERIOD = 8  # non-dominant kernels are timed on every 8th batch of the timed region


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64,
                    help="scans per GPU per step: with N sector shards a step holds N x batch full "
                         "scans, integrated by every rank as ONE GPU batch (<= 512 scans; the field "
                         "does not depend on batching)")
    ap.add_argument("--voxel", type=float, default=0.05)
    ap.add_argument("--trunc", type=float, default=0.15)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of each CPU-oracle baseline leg (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the multi-threaded oracle leg (capped by the CPU affinity set; "
                         "16 = one GPU's CPU share on the box)")
    ap.add_argument("--cpu-threads-full", type=int, default=0,
                    help="also time the oracle on this many threads (0: off; the box's rules size "
                         "worker pools to one GPU's 16-core share, so the whole host is projected, "
                         "not run)")
    ap.add_argument("--no-cpu", action="store_true",
                    help="skip the CPU baseline and the parity check (both use the CPU oracle)")
    ap.add_argument("--parity-steps", type=int, default=2,
                    help="timed steps re-integrated by a fresh context and compared bit for bit "
                         "with the CPU oracle after the timed region (0: off)")
    ap.add_argument("--pipeline", type=int, nargs="?", const=1, default=2, choices=(0, 1, 2),
                    help="tsdf_params.pipeline: 2 (default) overlaps batch b+1's k_count / "
                         "k_compact with batch b's k_integrate on a second HIP stream, k_place "
                         "always runs alone; 1 overlaps count / compact / place of b+1 with place / "
                         "integrate of b; 0 runs batches one after another")
    ap.add_argument("--sensor", default="os1_128_1024", choices=("os1_128_1024", "os1_128_2048"),
                    help="beam table of the synthetic scans (os1_128_2048 + --voxel 0.02 --trunc "
                         "0.06 --hz 20: the C4 workload); the headline metric is os1_128_1024")
    ap.add_argument("--hz", type=float, default=10.0)
    ap.add_argument("--max-bricks", type=int, default=1 << 20,
                    help="brick pool capacity (4 KiB per brick)")
    ap.add_argument("--semantics", default="vdbfusion_f64",
                    choices=("vdbfusion", "voxblox", "vdbfusion_f64"),
                    help="fusion rule (tsdf_params.semantics); the headline is vdbfusion_f64, "
                         "VDBFusion at upstream's own precisions (the mode that meets SURVEY §8c's "
                         "per-voxel bar against literal VDBFusion, DESIGN.md §2c)")
    ap.add_argument("--method", default="simple", choices=("simple", "merged"),
                    help="with --semantics voxblox: voxblox's integrator (tsdf_params.voxblox_method;"
                         " voxblox_ros' default is merged, DESIGN.md §2d)")
    ap.add_argument("--const-weight", action="store_true",
                    help="with --semantics voxblox: use_const_weight (w = 1); the default is "
                         "voxblox's 1/z^2 weight from each scan's pose")
    ap.add_argument("--rank-rehearsal", type=int, default=0, metavar="N",
                    help="one process plays rank 0 of an N-GPU run (sector 0 of N, N x batch full "
                         "scans per step): its time per step is one rank's; value = N x batch "
                         "scans / step time, the N-GPU throughput if every rank took as long "
                         "(rehearsal of the scaling runs on a one-GPU box)")
    ap.add_argument("--rehearsal-sector", type=int, default=0, metavar="K",
                    help="with --rank-rehearsal N: play rank K (sector K of N) instead of rank 0")
    ap.add_argument("--sector-rule", default="index", choices=("index", "world"),
                    help="tsdf_params.sector_rule with N > 1 shards: index (default; contiguous "
                         "1/N of each scan's points, i.e. sensor-frame column sectors) or world "
                         "(world-frame pseudo-angle sectors, every rank reads every point)")
    ap.add_argument("--walk", default="two", choices=("two", "single"),
                    help="front end (tsdf_params.walk): two = k_count + k_place (default); single = "
                         "every ray walked once (k_walk + k_spans) when the band allows it")
    ap.add_argument("--no-profile", action="store_true",
                    help="do not record per-kernel HIP events in the timed region")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_r06.json"),
                    help="PMC-measured HBM bytes per launch (from a separate rocprofv3 --pmc run)")
    return ap.parse_args()


def launch_ranks(n, script=None, argv=None):
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment): start N rank
    processes of this script, one per GPU, before this process touches any GPU, and exit with
    their status.  Rank 0 prints the JSON line.  If a rank fails, the others are stopped (by their
    PIDs) so no rank waits forever at a barrier."""
    import signal
    import socket
    import subprocess

    with socket.socket() as sk:  # a free rendezvous port on the loopback interface
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmd = [sys.executable, script or os.path.abspath(__file__)]
        procs.append(subprocess.Popen(cmd + list(sys.argv[1:] if argv is None else argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def bench_parity(args, steps, make_volume):
    """The driver-timed workload under parity: a fresh context with the bench's settings integrates
    the first `parity_steps` timed steps (the same resident TorchOusterSim tensors, the same
    tsdf_integrate_batch_device calls), and its field is compared bit for bit (touched voxels,
    weights, sdf bits) with the CPU oracle's on the same scans and semantics."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    t0 = time.perf_counter()
    sel = list(range(args.warmup, min(len(steps), args.warmup + args.parity_steps)))
    g = make_volume()
    for i in sel:
        x, offs, org = steps[i]
        g.integrate_batch_device(x.data_ptr(), offs, org)
    gi, gs, gw = g.export_voxels()
    g.close()
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(args.cpu_threads, share or 1))
    ov = oracle.OracleTSDFVolume(args.voxel, args.trunc, semantics=args.semantics, threads=threads,
                                 method=args.method, use_const_weight=args.const_weight)
    n_scans = 0
    for i in sel:
        x, offs, org = steps[i]
        xs = x.cpu().numpy()
        for j in range(len(org)):
            ov.integrate(xs[offs[j]:offs[j + 1]], org[j])
            n_scans += 1
    oi, os_, ow = ov.export_voxels()
    same_set = gi.shape == oi.shape and bool(np.array_equal(gi, oi))
    w_eq = same_set and bool(np.array_equal(gw.view(np.uint32), ow.view(np.uint32)))
    s_eq = same_set and bool(np.array_equal(gs.view(np.uint32), os_.view(np.uint32)))
    out = {"scans": n_scans, "voxels": int(gi.shape[0]), "oracle_voxels": int(oi.shape[0]),
           "bitwise": bool(same_set and w_eq and s_eq), "same_voxels": same_set,
           "weights_equal": w_eq, "sdf_bits_equal": s_eq,
           "settings": "fresh context, semantics %s%s, pipeline %d, %d-scan device batches" % (
               args.semantics, (" %s %s" % (args.method, "const weight" if args.const_weight
                                            else "1/z^2")) if args.semantics == "voxblox" else "",
               args.pipeline, args.batch),
           "oracle": "oracle/tsdf_oracle.c scan-fused, %d threads" % threads,
           "seconds": round(time.perf_counter() - t0, 2)}
    if same_set and not (w_eq and s_eq):
        out["sdf_mismatch_voxels"] = int(np.count_nonzero(gs.view(np.uint32) != os_.view(np.uint32)))
        out["max_abs_dsdf"] = float(np.max(np.abs(gs - os_)))
    return out


def lib_sha16():
    """First 16 hex digits of the sha256 of the loaded kernel library (the build the PMC traffic
    file must have been measured on)."""
    import hashlib
    from tsdf_map._lib import HIP_LIB
    p = os.environ.get("TSDF_HIP_LIB") or HIP_LIB
    with open(p, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def read_traffic(path, kernel):
    """roofline.traffic: PMC HBM bytes per launch of `kernel` from a separate rocprofv3 --pmc run
    (profiles/collect_pmc.sh), only when that run measured THIS build of the library."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, {"file": os.path.relpath(path, REPO), "error": "unreadable"}
    cur = lib_sha16()
    src = {"file": os.path.relpath(path, REPO), "lib_sha16": tj.get("lib_sha16"),
           "this_build_sha16": cur, "matches_build": tj.get("lib_sha16") == cur}
    if not src["matches_build"]:
        return None, src  # stale: measured on another build of the kernels
    return tj.get("bytes_per_launch", {}).get("k_" + kernel), src


def serial_kernel_times(args, steps, make_volume):
    """Every kernel's duration alone: a fresh context with pipeline 0 integrates the warmup steps,
    then the timed steps with every launch of every kernel timed (dispatch timestamps).  Returns
    ({kernel: mean ms per launch}, {kernel: launches})."""
    v = make_volume(pipeline=0)
    for i in range(args.warmup):
        x, offs, org = steps[i]
        v.integrate_batch_device(x.data_ptr(), offs, org)
    v.sync()
    v.reset_stats()
    v.set_profiling(True)
    for i in range(args.warmup, len(steps)):
        x, offs, org = steps[i]
        v.integrate_batch_device(x.data_ptr(), offs, org)
    v.sync()
    st = v.stats()
    v.close()
    n = st["kernel_launches"]
    return ({k: st["kernel_ms"][k] / n[k] for k in st["kernel_ms"] if n[k] > 0},
            {k: n[k] for k in n if n[k] > 0})


def check_world(n_gpus, world):
    """The printed line's n_gpus must be the ranks that actually ran."""
    if n_gpus != world:
        raise SystemExit("refusing to report n_gpus=%d from a world of %d rank(s)" % (n_gpus, world))


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_world(args.gpus, world)
    # TSDF_BENCH_SHARED_GPU=1 (rehearsal only, never the driver's runs): every rank on device
    # local % device_count, collectives over gloo on host tensors -- exercises the N-rank path
    # (sector sharding, max-over-ranks timing, read-out merge) on a one-GPU box
    shared = os.environ.get("TSDF_BENCH_SHARED_GPU") == "1"
    if shared:
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if shared else dev  # where collective tensors live
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from tsdf_map import HipTSDFVolume
    from tsdf_map.scan_gen import TorchOusterSim, pose_on_circle

    # ---- synthesize every (full) scan of every step, resident in HBM ----------------------------
    sim = TorchOusterSim(dev, beams=args.sensor, hz=args.hz)
    n_steps = args.warmup + args.steps
    n_shards = args.rank_rehearsal if (args.rank_rehearsal > 1 and world == 1) else world
    scans_per_step = n_shards * args.batch
    steps = []
    t_gen = time.time()
    for s in range(n_steps):
        parts, offs, origins = [], [0], []
        for j in range(scans_per_step):
            k = s * scans_per_step + j
            pts, org = sim.scan(k)
            parts.append(pts)
            offs.append(offs[-1] + pts.shape[0])
            if args.semantics == "voxblox":
                # the full pose (x, y, z, qx, qy, qz, qw): Voxblox's 1/z^2 weight needs the sensor
                # axes (the yaw of pose_on_circle; tsdf_integrate_batch_device_pose)
                yaw = pose_on_circle(k, hz=args.hz)[1]
                org = np.concatenate([org, [0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2)]])
            origins.append(org)
        steps.append((torch.cat(parts).contiguous(), np.array(offs, np.uint64),
                      np.stack(origins)))
    torch.cuda.synchronize()
    t_gen = time.time() - t_gen
    max_pts = max(int(np.diff(o).max()) for _, o, _ in steps)

    def make_volume(pipeline=None):
        return HipTSDFVolume(args.voxel, args.trunc, max_points=max(max_pts, 1 << 17),
                             max_bricks=args.max_bricks, device_id=local,
                             max_batch=min(scans_per_step, 512),  # one launch per step (all shards)
                             pipeline=args.pipeline if pipeline is None else pipeline,
                             semantics=args.semantics,
                             method=args.method, use_const_weight=args.const_weight,
                             n_sectors=n_shards,  # this rank's azimuth sector of every scan
                             sector=(args.rehearsal_sector % n_shards if world == 1 and n_shards > 1
                                     else rank),
                             walk=args.walk, sector_rule=args.sector_rule)

    vol = make_volume()

    def run_step(i):
        x, offs, org = steps[i]
        vol.integrate_batch_device(x.data_ptr(), offs, org)

    # Kernel times.  The roofline kernel is ranked and timed ALONE: a serial leg
    # (a fresh context with pipeline 0, the same steps; serial_kernel_times, after the timed
    # region) times every kernel on every launch, where no kernel shares the GPU with another
    # batch's.  The timed region itself samples every kernel on every 8th batch only (a timed
    # launch costs the stream ~10 us): those are the pipelined durations (kernel_ms_per_launch),
    # which under pipeline 1 / 2 include the other batch's kernels running beside them.
    for i in range(args.warmup):
        run_step(i)
    vol.sync()
    timing = None
    if not args.no_profile:
        vol.set_profiling(True)
        vol.set_profiling_period([], PROFILE_PERIOD)
        timing = {"every_launch": [], "all_kernels_every_nth_batch": PROFILE_PERIOD,
                  "method": "dispatch timestamps (hipExtLaunchKernel start/stop events)",
                  "roofline_kernel_times": "serial leg (pipeline 0, every launch timed)"}
    vol.reset_stats()

    # ---- timed region ---------------------------------------------------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, n_steps):
        run_step(i)
    torch.cuda.synchronize()
    vol.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = vol.stats()

    # every rank's time (reported), the step time is the slowest rank's
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        all_el = [torch.zeros_like(el) for _ in range(world)]
        dist.all_gather(all_el, el)
        rank_elapsed = [float(t.item()) for t in all_el]
    else:
        rank_elapsed = [elapsed]
    elapsed = max(rank_elapsed)
    total_scans = args.steps * scans_per_step
    value = total_scans / elapsed

    # ---- roofline of the dominant kernel (per-launch means, this rank) -------------------------
    # One launch = one batch of scans.  Algorithmic bytes: per scan
    # B_scan = 12 N_valid + 16 U_vox (every valid ray's xyz read once, every voxel the scan updates
    # read and written once as (S, W) f32), times the scans one launch integrates.  Also reported:
    # the batch-deduplicated figure (a voxel updated by several scans of one batch counted once),
    # which is what the batched pipeline must move at minimum.
    n_batches = max(1, st["n_batches"])
    n_scans_rank = max(1, st["n_scans"])
    rays_per_scan = st["n_rays_total"] / n_scans_rank
    uvox_per_scan = st["n_voxels_total"] / n_scans_rank
    bytes_per_scan = 12.0 * rays_per_scan + 16.0 * uvox_per_scan  # SURVEY.md §8d B_scan
    scans_per_launch = n_scans_rank / n_batches
    bytes_per_launch = bytes_per_scan * scans_per_launch
    dedup_bytes_per_launch = (12.0 * st["n_rays_total"] + 16.0 * st["n_dirty_total"]) / n_batches
    kms = st["kernel_ms"]
    roofline = None
    kernel_ms_per_launch = {k: (kms[k] / st["kernel_launches"][k]) for k in kms
                            if st["kernel_launches"][k] > 0}
    serial = None
    if not args.no_profile:
        vol_serial_ms, serial_launches = serial_kernel_times(args, steps, make_volume)
        serial = {k: round(v, 5) for k, v in vol_serial_ms.items()}
        # the dominant kernel: the largest of the kernels' durations ALONE
        dom = max(vol_serial_ms, key=vol_serial_ms.get)
        t_launch = vol_serial_ms[dom] * 1e-3
        achieved = bytes_per_launch / t_launch / 1e9
        traffic, traffic_src = read_traffic(args.traffic_json, dom) if world == 1 else (None, None)
        roofline = {"bound": "hbm", "kernel": "k_" + dom, "achieved": round(achieved, 2),
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 5),
                    "traffic": traffic, "traffic_source": traffic_src,
                    "algorithmic_bytes_per_launch": round(bytes_per_launch),
                    "dedup_bytes_per_launch": round(dedup_bytes_per_launch),
                    "scans_per_launch": round(scans_per_launch, 2),
                    "avg_launch_ms": round(vol_serial_ms[dom], 5),
                    "launches_timed": serial_launches[dom],
                    "timed_in": "serial leg: a fresh context with pipeline 0 integrating the same "
                                "warmup + timed steps, every launch of the timed steps timed, so "
                                "every kernel's duration is its own (the headline runs pipeline %d)"
                                % args.pipeline}
        # the whole path: the same algorithmic bytes over the step time (pipelined kernels overlap,
        # so their summed times would overstate it)
        path_ms = (sum(kernel_ms_per_launch.values()) if args.pipeline == 0
                   else elapsed * 1e3 / args.steps)
        roofline["path_achieved"] = round(bytes_per_launch / (path_ms * 1e-3) / 1e9, 2)
        roofline["path_frac"] = round(bytes_per_launch / (path_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)
    launch_ms = (sum(kernel_ms_per_launch.values()) if args.pipeline == 0
                 else elapsed * 1e3 / max(1, args.steps))  # pipelined: the step time
    path_ms_per_scan = launch_ms * n_batches / n_scans_rank

    # ---- read-out merge of border bricks (not in the timed region) ----------------------------
    merge_ms = merge_info = None
    if world > 1:
        from tsdf_map.distributed import border_reduce
        dist.barrier()
        tm = time.perf_counter()
        try:
            merge_info = border_reduce(vol, comm_device=cdev)
        except Exception as e:  # a read-out failure is reported in the line, not lost with it
            merge_info = {"error": "%s: %s" % (type(e).__name__, e)}
            print("border_reduce failed on rank %d: %s" % (rank, merge_info["error"]),
                  file=sys.stderr)
        dist.barrier()
        merge_ms = (time.perf_counter() - tm) * 1e3

    # ---- parity of the timed workload: the first timed steps, integrated by a fresh context with
    # the bench's exact settings (semantics, pipeline, batch size, device batch API), against the
    # CPU oracle on the same scans (rank 0, N=1; after the timed region, never inside it) ---------
    parity = None
    if rank == 0 and world == 1 and n_shards == 1 and not args.no_cpu and args.parity_steps > 0:
        parity = bench_parity(args, steps, make_volume)

    # ---- CPU baseline: the oracle on a bounded sample of the same workload (rank 0, N=1) --------
    # Two legs: the partitioned multi-threaded oracle on the box's CPU share (the
    # reported value) and the serial oracle (VDBFusion's serial Integrate loop), same scans.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle

        def oracle_leg(threads):
            ov = oracle.OracleTSDFVolume(args.voxel, args.trunc, semantics=args.semantics,
                                         threads=threads, method=args.method,
                                         use_const_weight=args.const_weight)
            n_done, tc, busy = 0, time.perf_counter(), 0.0
            for i in range(args.warmup, n_steps):  # the timed steps' scans, in order, until the budget
                x, offs, org = steps[i]
                xs = x.cpu().numpy()
                t1 = time.perf_counter()
                for j in range(len(org)):
                    ov.integrate(xs[offs[j]:offs[j + 1]], org[j])
                    n_done += 1
                    if time.perf_counter() - tc > args.cpu_seconds:
                        break
                busy += time.perf_counter() - t1
                if time.perf_counter() - tc > args.cpu_seconds:
                    break
            return n_done, busy

        share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
        threads = max(1, min(args.cpu_threads, share or 1))
        n_mt, t_mt = oracle_leg(threads)
        n_1, t_1 = oracle_leg(1)
        host = os.cpu_count() or 1
        cpu = {"value": round(n_mt / t_mt, 4), "unit": "scans/s", "cores": threads, "kind": "port",
               "host_nproc": host, "affinity_cpus": share,
               "sample": "the first %d scans of the timed steps (%.1f s), C oracle in its partitioned "
                         "multi-threaded scan-fused mode (%d threads: one GPU's CPU share of the "
                         "box), same inputs, same semantics" % (n_mt, t_mt, threads),
               "serial": {"value": round(n_1 / t_1, 4), "cores": 1,
                          "sample": "the first %d scans (%.1f s), serial scan-fused oracle "
                                    "(VDBFusion's serial Integrate loop)" % (n_1, t_1)},
               # the whole host at the measured per-thread rate of the share leg (linear scaling:
               # an upper bound for the CPU); not run, the box's rules size worker pools to 16
               "full_host_projection": {"value": round(n_mt / t_mt * host / threads, 2),
                                        "cores": host,
                                        "note": "share-leg rate x host_nproc / cores (perfect "
                                                "scaling assumed: an upper bound, not a run)"}}
        if args.cpu_threads_full > 0:
            tf = min(args.cpu_threads_full, share or 1)
            n_f, t_f = oracle_leg(tf)
            cpu["full"] = {"value": round(n_f / t_f, 4), "cores": tf,
                           "sample": "the first %d scans (%.1f s), %d threads" % (n_f, t_f, tf)}

    if rank == 0:
        check_world(args.gpus, world)
        out = {
            "metric": "scans/sec TSDF integration (128x1024 pts, 5 cm voxel)",
            "value": round(value, 2),
            "unit": "scans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "rank_ms_per_step": [round(e / args.steps * 1e3, 4) for e in rank_elapsed],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"vdbfusion": "f32", "voxblox": "f32",
                      "vdbfusion_f64": "f64+f32"}[args.semantics],  # f64 SDF, f32 DDA (upstream's)
            "data": "synthetic (OS-1-128 1024x10 beam angles from the reference's metadata "
                    "fixture; analytic scene; resident in HBM)",
            "config": {"workload": ("C1/M1 ouster_os1_128_1024x10_synthetic_5cm"
                                    if args.sensor == "os1_128_1024" else
                                    "C4/M4 ouster_%s_synthetic_%gcm_%ghz" % (args.sensor,
                                                                            args.voxel * 100,
                                                                            args.hz)),
                       "voxel_size_m": args.voxel, "sdf_trunc_m": args.trunc,
                       "scans_per_step": scans_per_step, "global_batch": scans_per_step,
                       "points_per_scan": int(round(rays_per_scan * n_shards)),
                    "scans_per_gpu_batch": args.batch, "pipelined_batches": args.pipeline,
                       "semantics": args.semantics,
                       "voxblox": ({"method": args.method, "weight": "const" if args.const_weight
                                    else "1/z^2"} if args.semantics == "voxblox" else None),
                       "parallelism": ("%s-sector x%d" % (args.sector_rule, world) if world > 1 else
                                       "rank-%d rehearsal of %s-sector x%d" % (
                                           args.rehearsal_sector % n_shards, args.sector_rule,
                                           n_shards)
                                       if n_shards > 1 else "single"),
                       "sector_rule": args.sector_rule if n_shards > 1 else None,
                       "sector_split": (None if n_shards <= 1 else
                                        "index share: the rank reads only its contiguous 1/N of "
                                        "each resident scan (timed)" if args.sector_rule == "index"
                                        else "in-kernel world-frame filter (timed)"),
                       "front_end": ("single walk (k_walk + k_spans)" if "walk" in kernel_ms_per_launch
                                     else "two walks (k_count + k_place)")},
            "roofline": roofline,
            "parity": parity,
            "cpu_baseline": cpu,
            "path_ms_per_scan": round(path_ms_per_scan, 5),
            "kernel_ms_per_launch": {k: round(v, 5) for k, v in kernel_ms_per_launch.items()},
            "serial_kernel_ms_per_launch": serial,
            "kernel_timing": timing,
            "uvox_per_scan": round(uvox_per_scan),
            "dirty_voxels_per_batch": round(st["n_dirty_total"] / n_batches),
            "survey_bytes_per_scan": round(bytes_per_scan),
            "survey_gbs": round(bytes_per_scan / (path_ms_per_scan * 1e-3) / 1e9, 2)
            if path_ms_per_scan else None,
            "bricks": st["n_bricks"],
            "readout_merge_ms": merge_ms,
            "readout_merge": merge_info,
            "gen_seconds": round(t_gen, 2),
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
