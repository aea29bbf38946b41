#!/usr/bin/env python3
"""EKF-SLAM correction throughput on MI355X (BASELINE.json metric).

Default workload = BASELINE.json configs[2], the north-star target: N = 1024 synthetic landmarks,
one filter per GPU, Σ in fp32, known association, 16 markers per sensor message.
A "step" is one sensor message = predict + 16 corrections + posterior (slam.cpp:180-316) through
the C-ABI (ekf_replay → ekf_batch_sensor). value = corrections/s summed over ranks.

Inputs: filter g (global index over all ranks) is seeded --seed + g (its own map,
slip and sensor noise); an untimed survey drive sights every landmark before the timed circle
drive, so the timed messages update a fully populated, correlated Σ.

Multi-GPU: `bench.py --gpus N` starts N ranks itself (torch.distributed.run as a child process,
before anything touches a GPU), or runs as one rank under an external launcher. Every rank runs its
own independent filters (weak scaling, no data-path collective); the final poses are all-gathered
once over RCCL. configs[3] (N=256 × 4096 filters over 8 GPUs) is
`bench.py --workload swarm_n256_fp64 --gpus 8` (512 filters per rank).

Also reported: the Σ-pass roofline (HIP events on the library's stream), the CPU baseline (the
literal dense restatement of slam.cpp through numpy's OpenBLAS dgemm on the host cores, rank 0 at
N=1 only; the C oracle's literal and O(n²) legs beside it) and pose parity of the first timed
messages against the fp64 oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# dense MFMA peaks: fp32 157.3 TF (MI355X_MICROARCH.md); fp64 78.6 TF (AMD MI355X spec sheet)
MFMA_PEAK_TF = {"f32": 157.3, "f64": 78.6}
WORKLOADS = {
    # name: (N landmarks, dtype, filters per GPU, markers per message, BASELINE config)
    "n1024_fp32": (1024, "f32", 1, 16, "configs[2]: N=1024 synthetic landmarks, 1 filter, fp32"),
    "n256_fp64": (256, "f64", 1, 16, "configs[1]: N=256 synthetic landmarks, 1 filter, fp64"),
    "swarm_n256_fp64": (256, "f64", 512, 16,
                        "configs[3]: N=256 landmarks x 512 independent filters per GPU, fp64"),
    "basic_world": (50, "f64", 1, 4, "configs[0]: basic_world 4 landmarks in 50 slots, fp64"),
    # Monte-Carlo swarm at the reference's own map size (resident path, one CU-resident filter
    # per workgroup): configs[0]'s filter × 1024 seeded runs per GPU
    "swarm_basic_world": (50, "f64", 1024, 4,
                          "configs[0] x 1024 Monte-Carlo runs per GPU (basic_world, fp64)"),
    # configs[2] at the reference's own precision (slam.cpp is fp64 throughout)
    "n1024_fp64": (1024, "f64", 1, 16, "configs[2] at fp64: N=1024 synthetic landmarks, 1 filter"),
    # unknown association (sensor_cb, slam.cpp:318-530): ids stripped, every marker scored against
    # the 960 mapped landmarks (64 slots left for new ones)
    "n1024_fp32_assoc": (1024, "f32", 1, 16, "configs[2] with unknown association (sensor_cb): "
                                              "N=1024 slots, 960 mapped landmarks, fp32"),
    "n1024_fp64_assoc": (1024, "f64", 1, 16, "configs[2] with unknown association (sensor_cb): "
                                              "N=1024 slots, 960 mapped landmarks, fp64"),
    # the Joseph-form covariance update (BASELINE.json north_star, ekf_set_joseph): one chunk per
    # 16-marker message, one Σ pass of rank 2 + 4m
    "n1024_fp32_joseph": (1024, "f32", 1, 16, "configs[2] with the Joseph-form Sigma update "
                                               "(north_star): N=1024, 1 filter, fp32"),
    "n1024_fp32_assoc_joseph": (1024, "f32", 1, 16, "configs[2] with unknown association "
                                                     "(sensor_cb) in the Joseph form: N=1024 "
                                                     "slots, 960 mapped landmarks, fp32"),
}
JOSEPH_CHUNK = 16  # markers per Joseph-form chunk (kMaxJoseph, ekf_device.hpp)
ASSOC_FREE_SLOTS = 64  # association workloads map N − 64 landmarks (room for new ones)


def is_assoc(workload):
    return workload.endswith("_assoc") or workload.endswith("_assoc_joseph")


def is_joseph(workload):
    return workload.endswith("_joseph")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--workload", default="n1024_fp32",
                   choices=sorted(WORKLOADS) + ["frontend", "rosbag_surrogate"],
                   help="frontend: the landmark front-end (include/landmarks.h), scans/s; "
                        "rosbag_surrogate: configs[4]'s shape, scans → detect → slam node")
    p.add_argument("--seed", type=int, default=20240317,
                   help="filter g (global index over ranks) uses seed + g (SURVEY.md §8d)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and parity legs")
    p.add_argument("--inputs", choices=["auto", "host", "hbm", "device"], default="auto",
                   help="hbm: the pyekf.synth marker arrays uploaded to HBM before the timed region "
                        "and planned on the GPU (ekf_replay_device); device: odometry, slip and the "
                        "fake sensor simulated on the GPU inside the timed region, descriptors "
                        "written there too (include/ekf_sim.h); host: the marker arrays replayed "
                        "through ekf_replay (host planning + PCIe inside the timed region); auto: "
                        "device for the fp64 swarm workloads, hbm for the other known-id pipeline "
                        "workloads, host otherwise (association, the resident N = 50)")
    p.add_argument("--parity-messages", type=int, default=10)
    p.add_argument("--traffic", choices=["auto", "off"], default="auto",
                   help="auto: measure the Σ pass's HBM bytes with two rocprofv3 --pmc child runs")
    p.add_argument("--no-fp64", action="store_true",
                   help="skip the n1024_fp32 line's fp64 leg (configs[2] at slam.cpp's arithmetic)")
    return p.parse_args(argv)


def _pmc_pass(args, counters):
    """One rocprofv3 --pmc pass (its own child bench run, every kernel on one stream so each
    dispatch's counters are its own) → {counter: mean over k_sigma_pass dispatches}, or an error
    string. Child runs happen before this process touches the GPU."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 not found"
    # the workload's own instantiation (the fp32 workload's fp64 warm-up lap is excluded)
    kname = "k_sigma_pass<float," if WORKLOADS[args.workload][1] == "f32" else "k_sigma_pass<double,"
    d = tempfile.mkdtemp(prefix="ekf_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [exe, "--pmc", *counters, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--workload", args.workload,
           "--steps", "8", "--warmup", "2", "--no-cpu", "--traffic", "off", "--no-fp64"]
    env = dict(os.environ, EKF_SERIAL="1")
    name = " ".join(counters)
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
    except subprocess.TimeoutExpired:
        return None, f"rocprofv3 --pmc {name} timed out"
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if r.returncode != 0 or not files:
        return None, f"rocprofv3 --pmc {name} failed (rc {r.returncode})"
    per = {c: {} for c in counters}
    with open(files[0]) as fh:
        for row in csv.DictReader(fh):
            c = row.get("Counter_Name")
            if kname in row.get("Kernel_Name", "") and c in per:
                key = row.get("Dispatch_Id", row.get("Correlation_Id", len(per[c])))
                per[c][key] = per[c].get(key, 0.0) + float(row["Counter_Value"])
    shutil.rmtree(d, ignore_errors=True)
    if not all(per[c] for c in counters):
        return None, f"no k_sigma_pass dispatches with {name}"
    return {c: float(np.mean(list(per[c].values()))) for c in counters}, None


def pmc_traffic(args):
    """HBM-side bytes per k_sigma_pass launch from PMC counters (MI355X_MICROARCH.md, HBM):
    FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not fit one pass), FETCH_SIZE
    doubled on gfx950; then MFMA-busy cycles beside GRBM_GUI_ACTIVE in a third pass. Any failure
    gives None with the reason (a measurement gap, never a different compute path)."""
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        v, err = _pmc_pass(args, [counter])
        if v is None:
            return None, err
        vals.update(v)
    # counters are in KB (rocprofv3 derived FETCH_SIZE / WRITE_SIZE)
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    out = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
           "note": "FETCH_SIZE x2 (gfx950 correction, calibrated for this kernel's loads in "
                   "profiles/r1/pmc_calibration.md) + WRITE_SIZE; separate --pmc passes over a "
                   "short child run with every kernel on one stream (EKF_SERIAL=1); mean over "
                   "k_sigma_pass dispatches"}
    v, err = _pmc_pass(args, ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"])
    if v is None:
        out["mfma_busy"] = err
    else:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md); the MFMA-busy cycles
        # over every SIMD: busy ÷ (kernel cycles × 256 CUs × 4 SIMDs)
        # (GRBM_GUI_ACTIVE spans the whole counter-collection window of a dispatch, several times
        # the kernel; main() divides the busy cycles by the event-timed duration instead)
        out["mfma_busy"] = {"SQ_VALU_MFMA_BUSY_CYCLES": v["SQ_VALU_MFMA_BUSY_CYCLES"],
                            "GRBM_GUI_ACTIVE": v["GRBM_GUI_ACTIVE"],
                            "note": "SQ_VALU_MFMA_BUSY_CYCLES summed over the SIMDs, per "
                                    "k_sigma_pass dispatch; one --pmc pass, same child run shape"}
    return out, None


def frontend_main(args):
    """Landmark front-end (landmarks.cpp laserCallback, include/landmarks.h): one step = one batch
    of 4096 scans (one per filter of the configs[3] swarm) of 360 beams, basic_world obstacles
    plus 20 clutter cylinders. value = scans/s of the detect kernel with the ranges resident in
    HBM (HIP events around each dispatch); the host-inclusive call rate (ranges over PCIe, markers
    back) is reported beside it. N=1 only (scans are independent: replicas across ranks)."""
    import pyekf  # noqa: F401
    from pyekf import synth
    from pyekf.landmarks import Detector
    S, B = 4096, 360
    rng = np.random.default_rng(20240317)
    obs = [(-0.5, -0.7, 0.038), (0.8, -0.8, 0.038), (0.4, 0.8, 0.038), (-0.6, 0.65, 0.038)]
    obs += [(rng.uniform(-4.5, 4.5), rng.uniform(-2.2, 2.2), rng.uniform(0.03, 0.1))
            for _ in range(20)]
    poses = np.stack([rng.uniform(-np.pi, np.pi, S), rng.uniform(-1.5, 1.5, S),
                      rng.uniform(-1.0, 1.0, S)], 1)
    ranges = synth.lidar_scans(poses, obs, n_beams=B, sigma=0.001)
    inc = float(np.float32(2 * np.pi / B))
    amin, ainc = np.zeros(S), np.full(S, inc)
    det = Detector(max_scans=S, max_beams=B)
    for _ in range(max(args.warmup, 1)):
        cnt, _ = det.detect(ranges, amin, ainc)
    kern = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        det.detect(ranges, amin, ainc)
        kern.append(det.last_kernel_us())
    wall = time.perf_counter() - t0
    k_us = float(np.mean(kern))
    in_bytes = S * B * 4 + S * 16
    result = {
        "metric": "landmark front-end scans/sec (laserCallback: cluster, classify, Hyper fit)",
        "value": S / (k_us * 1e-6), "unit": "scans/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": k_us / 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic lidar scans",
        "config": {"workload": "frontend", "scans_per_step": S, "beams": B,
                   "obstacles": len(obs), "markers_per_scan_mean": float(np.mean(cnt)),
                   "parallelism": "one wavefront per scan"},
        "roofline": {"kernel": "k_detect", "bound": "latency (per-lane f64 fits)",
                     "achieved": in_bytes / (k_us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": in_bytes / (k_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                     "traffic": None, "algorithmic_bytes_per_launch": in_bytes,
                     "avg_launch_us": k_us},
        "host_inclusive": {"scans_per_s": S * args.steps / wall,
                           "note": "lm_detect call: ranges H2D, kernel, markers D2H, sync"},
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import landmarks_numpy as L  # noqa: E402  (cpu_baseline leg only)
        n_cpu = 64
        t0 = time.perf_counter()
        for k in range(n_cpu):
            L.laser_callback(ranges[k], 0.0, inc)
        dt = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": n_cpu / dt, "unit": "scans/s", "cores": 1,
                                  "kind": "port", "sample": f"numpy/LAPACK restatement "
                                  f"(oracle/landmarks_numpy.py), {n_cpu} scans in {dt:.2f} s"}
    print(json.dumps(result))
    det.close()


def rosbag_main(args):
    """BASELINE configs[4] surrogate (the bag's .mcap payload is missing from the reference
    snapshot; synth.lidar_world has its shape: 426 scans at 5 Hz, 20 odometry ticks per scan,
    20 obstacles): one step = the whole 87 s drive — lm_detect over the 426 scans (one batch) and
    the slam node's loop (joint states, unknown-association MarkerArrays) natively (slam_replay),
    fp64, N = 50 slots. value = corrections/s; parity = pose trace vs the CPU pipeline
    (landmarks_numpy.laser_callback → the C oracle's node loop); the CPU pipeline's time is the
    cpu_baseline."""
    import math as _m
    import pyekf
    from pyekf import synth
    from pyekf.landmarks import Detector
    sc, obs, scans = synth.lidar_world()
    T = len(scans)
    inc = float(np.float32(2 * _m.pi / 360))
    det = Detector(max_scans=T, max_beams=360)

    s = pyekf.Slam(n_landmarks=50, source=pyekf.SOURCE_ASSOC)

    def gpu_run(trace):
        s.reset()  # a fresh node per drive (Σ₀, odometry at the origin) on the same handle
        cnt, mk = det.detect(scans, np.zeros(T), np.full(T, inc))
        c = np.clip(cnt, 0, mk.shape[1])  # LM_NO_BREAK (the reference throws): no markers
        keep = np.arange(mk.shape[1])[None, :] < c[:, None]
        rel = np.stack([np.where(keep, mk["x"], 0.0), np.where(keep, mk["y"], 0.0)], -1)
        scg = synth.Scenario(sc.n_landmarks, sc.landmarks, sc.wheel,
                             np.full(keep.shape, -1, np.int32), np.zeros(keep.shape, np.int32),
                             rel, c.astype(np.int32), sc.truth, sc.track, sc.radius)
        # no trace: the drive's messages are planned on the host and run as one submission
        _, poses, _ = s.replay(scg, poses=trace)
        s.filter_state(sigma=False)               # the drive's end: synchronises
        return scg, poses
    for _ in range(max(args.warmup, 1)):
        gpu_run(False)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        scg, _ = gpu_run(False)
    dt = (time.perf_counter() - t0) / args.steps
    # device time of the EKF kernels over one more (untimed) drive, HIP events per launch
    s.profile(True)
    gpu_run(False)
    dev = {k: s.profile_read(k) for k in (4, 1, 2, 3, 0)}
    s.profile(False)
    scg, poses = gpu_run(True)  # the pose trace for parity, untimed
    det.close()
    s.close()
    corr = int(scg.count.sum())
    tr = sc.truth.copy()
    tr[:, 1] -= 1.0  # the map frame starts at the drive's start pose (θ0 = 0, x0 = 1)
    result = {
        "metric": "EKF correction steps/sec at N landmarks; pose RMSE vs reference",
        "value": corr / dt, "unit": "corrections/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic surrogate of rosbag2_2024_03_17-18_35_57 (payload missing)",
        "config": {"workload": "rosbag_surrogate", "baseline_config": "configs[4] (surrogate)",
                   "scans": T, "obstacles": len(obs), "n_landmarks": 50,
                   "markers": corr, "association": "unknown (sensor_cb)",
                   "step": "slam_reset + lm_detect batch + 426 slam_markers messages with "
                           "wheel ticks (one deferred submission) + state read-back",
                   "device_path": "resident" if s.path == pyekf.EKF_PATH_RESIDENT else "pipeline"},
        "ekf_device_ms_per_step": sum(v[1] for v in dev.values()),
        "ekf_device_launches_per_step": {
            {4: "k_resident", 1: "k_chain", 2: "k_assoc", 3: "k_factors", 0: "k_sigma_pass"}[k]: v[0]
            for k, v in dev.items() if v[0]},
        "pose_rmse_vs_truth_m": float(np.sqrt(np.mean(np.sum((poses[:, 1:] - tr[:, 1:]) ** 2,
                                                               1)))),
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import landmarks_numpy as L  # noqa: E402  (cpu_baseline / parity legs only)
        orc = _oracle()
        t0 = time.perf_counter()
        cpu_mk = [[(w[1], w[2]) for w in L.laser_callback(scans[t], 0.0, inc)] for t in range(T)]
        o = orc.run_scenario(synth.with_markers(sc, cpu_mk), True)
        cdt = time.perf_counter() - t0
        d = poses - o["poses"]
        result["parity"] = {"pose_rmse_m": float(np.sqrt(np.mean(d[:, 1] ** 2 + d[:, 2] ** 2))),
                            "heading_rmse_rad": float(np.sqrt(np.mean(np.arctan2(
                                np.sin(d[:, 0]), np.cos(d[:, 0])) ** 2))),
                            "messages": T, "vs": "laser_callback (numpy) → C oracle node loop"}
        result["cpu_baseline"] = {"value": corr / cdt, "unit": "corrections/s", "cores": 1,
                                  "kind": "port", "sample": f"the whole drive: numpy front-end + "
                                  f"C oracle (O(n^2)), {corr} corrections in {cdt:.2f} s"}
    print(json.dumps(result))


def launch_ranks(args, argv):
    """`bench.py --gpus N` outside a launcher: start N ranks (one process per GPU) with
    torch.distributed.run as a CHILD process — this process never touches the GPU — relay
    rank 0's output and exit with the launcher's status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


class HipBackend:
    """The product: libekfslam.so's HIP path on this rank's GPU, RCCL for the final gather."""
    dist_backend = "nccl"
    device = "cuda"

    def __init__(self, local):
        import torch
        import pyekf
        self.torch = torch
        self.EKF = pyekf.EKF
        self.F32, self.F64 = pyekf.EKF_F32, pyekf.EKF_F64
        if os.environ.get("EKF_BENCH_SHARE_GPU") == "1":
            # dev rehearsal of the N > 1 path on a one-GPU box: every rank on the GPUs there are,
            # the rank reductions over gloo (RCCL wants one GPU per rank)
            local = local % torch.cuda.device_count()
            self.dist_backend, self.device = "gloo", "cpu"
        self.local = local
        torch.cuda.set_device(local)

    def sync(self):
        self.torch.cuda.synchronize()

    def device_info(self):
        """This rank's GPU as the runtime sees it (the line's rank map: which GPU each rank ran)."""
        torch = self.torch
        d = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(d)
        info = {"device": d, "name": p.name}
        for k in ("pci_bus_id", "pci_device_id", "uuid"):
            v = getattr(p, k, None)
            if v is not None:
                info[k] = str(v)
        return info


def build_inputs(N, F, T, seed, m, rank, n_map=None):
    """SURVEY.md §8d inputs for this rank's F filters: global filter g = rank·F + f is seeded
    seed + g (its own map, slip and sensor noise); the survey warm-up (every landmark sighted)
    precedes T messages of the circle drive. N = 50 is configs[0]'s basic_world (4 landmarks,
    every one in view, no survey needed). n_map < N landmarks are placed (association workloads:
    the rest of the slots stay free for new landmarks). Returns the synth.Swarm (its drive, maps and
    the host restatement of every marker) and the odometry."""
    from pyekf import synth
    import pyekf
    if N == 50:
        drive = synth.circle_drive(T, 0.3, sense=synth.SENSE_ALL)
        sw = synth._generate(50, drive, np.uint64(seed + rank * F) + np.arange(F, dtype=np.uint64),
                             synth.BASIC_WORLD_LANDMARKS,
                             start_pose=(synth.BASIC_WORLD_THETA0, 0.0, 0.0))
        n_target = 4
    else:
        sw = synth.swarm(N, F, T, seed=seed + rank * F, max_markers=m,
                         **({} if n_map is None else {"n_map": n_map}))
        n_target = N if n_map is None else n_map
    odo = pyekf.odometry(sw.scenario(0))  # encoders report the commanded drive: every filter's
    return sw, np.repeat(odo[:, None], F, 1), n_target


def main(argv=None, backend=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.workload == "frontend":
        return frontend_main(args)
    if args.workload == "rosbag_surrogate":
        return rosbag_main(args)
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = max(world, 1)
    if args.gpus not in (1, world) and backend is None:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return run(args, rank, world, local, backend)[0]


def run(args, rank, world, local, backend=None):
    """One rank: its own filters (weak scaling, no collective on the data path), the timed K
    messages between barriers, the slowest rank's time (MAX), corrections of all ranks (SUM), one
    all_gather of the final poses (the path's only collective)."""
    N, dt, F, m, cfgname = WORKLOADS[args.workload]
    assoc = is_assoc(args.workload)
    n_map = N - ASSOC_FREE_SLOTS if assoc else None
    traffic, traffic_err = None, "not measured (--traffic off or N>1)"
    resident = dt == "f64" and 3 + 2 * N <= 128 and os.environ.get("EKF_RESIDENT") != "0"
    if resident:
        traffic_err = "resident path: Σ crosses HBM once per launch (no Σ pass to count)"
    if args.traffic == "auto" and world == 1 and not resident and backend is None:
        traffic, traffic_err = pmc_traffic(args)  # child runs, before this process uses the GPU
    import torch.distributed as dist
    be = backend if backend is not None else HipBackend(local)
    local = getattr(be, "local", local)  # (EKF_BENCH_SHARE_GPU: the GPU this rank shares)
    if world > 1:
        dist.init_process_group(be.dist_backend)
    # which rank ran where, gathered once before any timing (so the line shows that the collective
    # saw N ranks, each on its own GPU)
    me = {"rank": rank, "local_rank": local, "pid": os.getpid()}
    if hasattr(be, "device_info"):
        me.update(be.device_info())
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        dist_info = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                     "ranks": ranks}
    else:
        dist_info = {"world_size": 1, "backend": None, "ranks": [me]}
    dtype = be.F32 if dt == "f32" else be.F64
    W, K = args.warmup, args.steps
    t_gen = time.perf_counter()
    inputs = args.inputs
    if inputs == "auto":
        if F > 1 and dt == "f64" and backend is None:
            inputs = "device"
        elif not assoc and not resident and backend is None:
            inputs = "hbm"
        else:
            inputs = "host"
    if inputs == "device" and (dt != "f64" or assoc):
        raise SystemExit("--inputs device: fp64 known-id workloads (fp32 takes its survey on an "
                         "fp64 handle; the device planner writes known-id chunks)")
    if inputs == "hbm" and (assoc or resident or backend is not None):
        raise SystemExit("--inputs hbm: known-id workloads on the HBM pipeline (ekf_replay_device)")
    # hbm: a third span of K messages times the same path with host inputs (PCIe-inclusive)
    sw, odom, n_init_target = build_inputs(N, F, W + (3 if inputs == "hbm" else 2) * K, args.seed,
                                           m, rank, n_map)
    n_warm, counts, ids, act, rel = sw.n_warm, sw.count, sw.ids, sw.actions, sw.rel
    t_gen = time.perf_counter() - t_gen
    ekf = be.EKF(n_landmarks=N, n_filters=F, dtype=dtype, device=local)
    joseph = is_joseph(args.workload)
    if joseph and ekf.set_joseph(True) != 0:
        raise SystemExit("ekf_set_joseph failed")
    sim = None
    if inputs == "device":
        import pyekf
        tpm = sw.wheel.shape[1]
        sim = pyekf.Sim(ekf, sw.landmarks, seed=int(args.seed), f0=rank * F, ticks_per_msg=tpm,
                        max_markers=min(m, sw.landmarks.shape[1]), marker_stride=ids.shape[2],
                        start_theta=sw.start_pose[0], start_x=sw.start_pose[1],
                        start_y=sw.start_pose[2])

    gpu_in = None
    if inputs == "hbm":  # every message's markers in HBM before anything is timed
        import torch
        dev = torch.device("cuda", local)
        gpu_in = [torch.from_numpy(np.ascontiguousarray(a, dtype=d)).to(dev) for a, d in
                  ((counts, np.int32), (ids, np.int32), (act, np.int32), (rel, np.float64),
                   (odom, np.float64))]
        torch.cuda.synchronize()
        gpu_rows = [(g.data_ptr(), g[0].numel() * g.element_size()) for g in gpu_in]

    def msgs(a, b, e=None, known=False, host=False):
        if sim is not None and e is None:  # the GPU simulates, senses and plans these messages
            sim.run(sw.cmd[a * tpm:b * tpm], sw.sense[a:b])
            return
        if gpu_in is not None and e is None and not host:  # planned on the GPU from HBM
            # message a's rows by address (no tensor slicing on the timed path)
            pc, pi, pa, pr, po = (base + a * rb for base, rb in gpu_rows)
            ekf.replay_device_raw(b - a, ids.shape[2], pc, pr, po, pi, pa)
            return
        sl = slice(a, b)
        un = assoc and not known  # the survey sights with known ids; the drive's ids are stripped
        (e or ekf).replay(counts[sl], rel[sl], odom[sl], ids=None if un else ids[sl],
                          actions=act[sl], assoc=un)

    # ---- untimed warm-up: the survey (every landmark initialised), then W messages ----
    # fp32 cannot take first sightings against the 1e7 prior (slam.cpp:130): the survey runs on an
    # fp64 handle whose state seeds the fp32 one
    # (association: the survey sights with known ids on an fp64 handle, then counter_obstacles =
    # the mapped landmarks, numbered 0..n_map−1 as slam.cpp:351-356 would have numbered them)
    warm_state = None
    if (dtype == be.F32 or assoc) and n_warm:
        e64 = be.EKF(n_landmarks=N, n_filters=F, device=local)
        msgs(0, n_warm, e64, known=True)
        warm_state = []
        for f in range(F):
            x, S, cnt = e64.state(f)
            tmo = e64.map_odom(f)
            cnt = n_map if assoc else cnt
            ekf.set_state(x, S, tmo=tmo, counter=cnt, f=f)
            warm_state.append((x, S, tmo, cnt))
        e64.close()
    elif n_warm:
        msgs(0, n_warm)
    # the state reads below leave the GPU idle for milliseconds (a whole Σ crosses PCIe), and an idle
    # GPU enters the timed region at low clocks: the last two warm-up messages run after them
    W1 = max(W - 2, 0)
    if W1:
        msgs(n_warm, n_warm + W1)
    ekf.sync()
    # landmarks initialised (state slot ≠ (0, 0), slam.cpp:213) in every filter of this rank
    n_init = min(int(np.count_nonzero(np.any(ekf.state(f, sigma=False)[0][3:].reshape(-1, 2)
                                             != 0.0, 1))) for f in range(F))
    status = [ekf.status(f) for f in range(F)]
    x0, S0, c0 = ekf.state(0)
    ws0 = (x0, S0, ekf.map_odom(0), c0)  # the state before message t_ws (parity's start)
    t_ws = n_warm + W1
    if W > W1:
        msgs(n_warm + W1, n_warm + W)

    # ---- timed region: exactly K messages ----
    t0s = n_warm + W
    if world > 1:
        dist.barrier()
    be.sync()
    trace = os.environ.get("EKF_BENCH_TRACE") == "1"  # dev: host clocks around the timed region
    t0 = time.perf_counter()
    if trace:
        clk = [("t0", time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                time.clock_gettime_ns(time.CLOCK_BOOTTIME))]
    msgs(t0s, t0s + K)
    if trace:
        clk.append(("enqueued", time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                    time.clock_gettime_ns(time.CLOCK_BOOTTIME)))
    ekf.flush()  # everything planned is submitted (ekf_flush: no wait)
    if trace:
        clk.append(("flushed", time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                    time.clock_gettime_ns(time.CLOCK_BOOTTIME)))
    be.sync()   # device-wide (torch.cuda.synchronize on the GPU): waits for the library's streams too
    # this rank's own region (its K messages, enqueue to device-wide sync); the closing barrier
    # aligns the ranks, and reduce_ranks takes the MAX of these over ranks
    elapsed = time.perf_counter() - t0
    # the library's own sync after the region: its errors / timeouts, and the check that the
    # device-wide sync left nothing of it running (it returns at once then)
    t_ls = time.perf_counter()
    ekf.sync()
    lib_sync_after_us = (time.perf_counter() - t_ls) * 1e6
    if world > 1:
        dist.barrier()
    if trace:
        clk.append(("synced", time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                    time.clock_gettime_ns(time.CLOCK_BOOTTIME)))
        print(json.dumps({"trace_clocks": clk}), file=sys.stderr, flush=True)
    live = np.arange(act.shape[2]) < counts[t0s:t0s + K][..., None]
    corrections = int(np.count_nonzero(live & (act[t0s:t0s + K] != 2)))  # slam.cpp:205
    poses = np.stack([ekf.pose(f) for f in range(F)])
    status = [s | ekf.status(f) for f, s in enumerate(status)]
    if world > 1:
        elapsed, total_corr, all_poses = reduce_ranks(elapsed, corrections, poses, be.device)
    else:
        total_corr, all_poses = float(corrections), poses

    # ---- roofline pass: same work, Σ-pass launches bracketed by HIP events ----
    ps = slice(t0s + K, t0s + 2 * K)
    ekf.profile(True)
    msgs(ps.start, ps.stop)
    n_sig, ms_sig = ekf.profile_read(0)
    n_gain, ms_gain = ekf.profile_read(1)
    n_fac, ms_fac = ekf.profile_read(3)
    n_res, ms_res = ekf.profile_read(4)
    n_asc, ms_asc = ekf.profile_read(2)
    ekf.profile(False)
    live = np.arange(act.shape[2]) < counts[ps][..., None]
    res_corr = int(np.count_nonzero(live & (act[ps] != 2)))
    host_rate = None
    if inputs == "hbm":  # the same path fed host arrays (ekf_replay): host planning and PCIe timed
        hs = slice(t0s + 2 * K, t0s + 3 * K)
        ekf.sync()  # (the planning state comes back from the device first: not this span's cost)
        if world > 1:
            dist.barrier()
        be.sync()
        t1 = time.perf_counter()
        msgs(hs.start, hs.stop, host=True)
        be.sync()
        el_h = time.perf_counter() - t1
        if world > 1:
            dist.barrier()
        live_h = np.arange(act.shape[2]) < counts[hs][..., None]
        corr_h = int(np.count_nonzero(live_h & (act[hs] != 2)))
        if world > 1:
            el_h, corr_h, _ = reduce_ranks(el_h, corr_h, poses, be.device)
        host_rate = {"value": corr_h / el_h, "unit": "corrections/s", "ms_per_step": el_h / K * 1e3,
                     "note": "PCIe-inclusive: the same messages handed over as host arrays "
                             "(ekf_replay: host planning, one descriptor upload, launches), "
                             f"messages {hs.start}..{hs.stop - 1}; not the value"}
    bytes_per_launch = ekf.sigma_pass_bytes()
    avg_sig_s = ms_sig / max(n_sig, 1) / 1e3
    achieved = bytes_per_launch / avg_sig_s / 1e9 if n_sig else 0.0

    if traffic and isinstance(traffic.get("mfma_busy"), dict) and n_sig:
        # busy SIMD-cycles over what 1024 SIMDs offer in the event-timed launch at the 2.4 GHz
        # maximum clock (the chip runs slower under load, so this is a lower bound)
        mb = traffic["mfma_busy"]
        mb["busy_frac_at_max_clock"] = mb["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg_sig_s * 2.4e9 * 1024)
    result = None
    if rank == 0:
        value = total_corr / elapsed
        wsz = 4 if dt == "f32" else 8
        n = 3 + 2 * N
        # the rank-(2+2m) update's useful flops (fp64: the upper triangle, the symmetric pass);
        # Joseph: rank 2 + 4m per pass, ⌈m/16⌉ = 1 pass per message
        rank_k = 2 + 4 * min(m, JOSEPH_CHUNK) if joseph else 2 + 2 * m
        passes = -(-m // JOSEPH_CHUNK) if joseph else 1
        mfma_flops = 2.0 * rank_k * (n * n if wsz == 4 else n * (n + 1) / 2) * F
        result = {
            "metric": "EKF correction steps/sec at N landmarks; pose RMSE vs reference",
            "value": value,
            "unit": "corrections/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if dt == "f32" else "f64",
            "data": "synthetic (seeded map per filter, survey warm-up sighting every landmark, "
                    "then the circle drive with a nusim-style fake sensor)" + (
                        "; odometry, slip and sensing simulated on the GPU inside the timed "
                        "region (ekf_sim)" if inputs == "device" else
                        "; host-generated markers uploaded to HBM before the timed region, planned "
                        "on the GPU (ekf_replay_device)" if inputs == "hbm" else
                        "; host-generated markers replayed through ekf_replay"),
            "config": {"workload": args.workload, "baseline_config": cfgname,
                       "n_landmarks": N, "state_dim": n, "filters_per_gpu": F,
                       "filters_total": F * world, "markers_per_message": m,
                       "association": "unknown (sensor_cb)" if assoc else "known",
                       "seeds": f"{args.seed} + global filter index",
                       "survey_messages": n_warm,
                       "landmarks_initialised_min": n_init,
                       "landmarks_initialised_target": n_init_target,
                       "status_flags_rank0": sorted(set(status)),
                       "host_input_generation_s": t_gen,
                       "inputs": inputs,
                       "parallelism": f"independent filters x{world} ranks",
                       "distributed": dist_info},
            "roofline": {
                "kernel": "k_sigma_pass", "bound": "hbm", "achieved": achieved,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "traffic_detail": traffic if traffic else traffic_err,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "bytes_formula": (f"2*n^2*w*F = 2*{n}^2*{wsz}*{F}" if wsz == 4 else
                                  f"(n(n+1)/2 + n^2)*w*F = ({n}*{n + 1}/2 + {n}^2)*{wsz}*{F} "
                                  "(the symmetric fp64 pass reads the upper triangle of Sigma_in)"),
                "avg_launch_us": avg_sig_s * 1e6, "launches": n_sig,
                "mfma": {"flops_per_launch": mfma_flops,
                         "achieved_tflops": mfma_flops / avg_sig_s / 1e12 if n_sig else 0.0,
                         "peak_tflops": MFMA_PEAK_TF[dt],
                         "frac": mfma_flops / avg_sig_s / 1e12 / MFMA_PEAK_TF[dt] if n_sig else 0.0,
                         "formula": (f"2*k*n^2*F = 2*{rank_k}*{n}^2*{F}" if wsz == 4 else
                                     f"2*k*n(n+1)/2*F = 2*{rank_k}*{n}*{n + 1}/2*{F}") +
                                    f", k = {'2+4m (Joseph)' if joseph else '2+2m'}",
                         "pmc": traffic.get("mfma_busy") if traffic else traffic_err},
                "chain_kernel_avg_us": ms_gain / max(n_gain, 1) * 1e3,
                "factor_kernel_avg_us": ms_fac / max(n_fac, 1) * 1e3,
                # the whole step against the rank-2m ceiling: one Σ pass per
                # message is the algorithmic minimum, sigma_pass_bytes per step (the Joseph form
                # too: one pass of rank 2 + 4m per message)
                "end_to_end": {
                    "bytes_per_step": passes * bytes_per_launch,
                    "passes_per_step": passes,
                    "achieved": passes * bytes_per_launch / (elapsed / K) / 1e9,
                    "frac": passes * bytes_per_launch / (elapsed / K) / 1e9 / HBM_PEAK_GBS,
                    "ceiling_corrections_per_s": (HBM_PEAK_GBS * 1e9 / (passes * bytes_per_launch) * (
                        total_corr / world / K)) if bytes_per_launch else None,
                },
            },
        }
        result["roofline"]["end_to_end_frac"] = result["roofline"]["end_to_end"]["frac"]
        result["region_end"] = {
            "timed_until": "ekf_flush, then torch.cuda.synchronize (device-wide: the library's "
                           "streams included)",
            "library_sync_after_us": lib_sync_after_us}
        if host_rate is not None:
            result["host_inputs"] = host_rate
        if n_asc:
            result["roofline"]["assoc_kernel_avg_us"] = ms_asc / n_asc * 1e3
            result["roofline"]["assoc_launches"] = n_asc
        if world > 1:
            result["gathered_poses"] = {"filters": int(all_poses.shape[0]),
                                        "all_finite": bool(np.all(np.isfinite(all_poses)))}
        if n_res:
            # resident path (ekf_resident.hip): one launch runs the whole replay, Σ in registers;
            # its bound is the sequential f64 chain of one CU per filter, priced against that
            # CU's share of the fp64 vector peak (78.6 TF / 256 CUs)
            flops = 4.0 * n * n * res_corr  # Σ ← Σ − K·(HΣ): 2 FMAs per element per correction
            sec = ms_res / 1e3  # every launch of the profiled replay (res_corr spans them all)
            cu_peak = MFMA_PEAK_TF["f64"] / 256 * min(F, 256)
            result["roofline"] = {
                "kernel": "k_resident", "bound": "fp64-valu, one CU per filter (latency chain)",
                "achieved": flops / sec / 1e12, "peak": cu_peak, "unit": "TFLOP/s",
                "frac": flops / sec / 1e12 / cu_peak, "traffic": None,
                "traffic_detail": traffic_err,
                "flops_formula": f"4*n^2*corrections = 4*{n}^2*{res_corr}",
                "avg_launch_us": sec * 1e6 / n_res, "launches": n_res,
                "us_per_correction": sec * 1e6 / max(res_corr, 1),
                "hbm_bytes_per_launch": 2.0 * n * n * 8 * F,
                "kernel_corrections_per_s": res_corr / sec,
            }
            result["config"]["device_path"] = "resident"
    # ---- parity (rank 0) and the CPU baseline (rank 0, N=1 only) ----
    # parity and the CPU leg start from a state the host holds: the survey's (fp32 / association
    # handles, then messages t0s..) or the one read before the last warm-up messages (t_ws..)
    ws = warm_state[0] if warm_state else ws0
    tp = t0s if warm_state else t_ws
    if rank == 0 and not args.no_cpu:
        result["parity"] = parity(args, N, ekf_first_poses(args, be, N, dtype, ws, counts, ids,
                                                           act, rel, odom, tp, local,
                                                           gpu_in=gpu_in),
                                  ws, counts, ids, act, rel, odom, tp)
        if world == 1:
            result["cpu_baseline"] = cpu_baseline(args, N, ws, counts, ids, act, rel, odom, tp)
    if (rank == 0 and world == 1 and args.workload == "n1024_fp32" and gpu_in is not None
            and warm_state and not args.no_fp64):
        result["fp64"] = fp64_leg(args, be, N, warm_state[0], gpu_rows, ids.shape[2], n_warm, W, K,
                                  local, counts, ids, act, rel, odom, gpu_in)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if sim is not None:
        sim.close()
    ekf.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result, all_poses


def fp64_leg(args, be, N, ws, gpu_rows, M, n_warm, W, K, local, counts, ids, act, rel, odom,
             gpu_in):
    """configs[2] at the reference's own arithmetic (slam.cpp is fp64 throughout), after the
    fp32 line's timed region: a fresh fp64 handle from the same survey state replays the same
    warm-up and the same K timed messages from the same HBM inputs through the same entry point
    (ekf_replay_device), timed the same way; then one more span with HIP events per launch (chain,
    Σ pass) and, unless --no-cpu, pose parity of the first messages against the fp64 oracle."""
    x, S, tmo, cnt = ws
    e = be.EKF(n_landmarks=N, dtype=be.F64, device=local)
    e.set_state(x, S, tmo=tmo, counter=cnt)

    def span(a, b):
        pc, pi, pa, pr, po = (base + a * rb for base, rb in gpu_rows)
        e.replay_device_raw(b - a, M, pc, pr, po, pi, pa)
    t0s = n_warm + W
    if W > 2:
        span(n_warm, t0s - 2)
    e.sync()
    span(max(t0s - 2, n_warm), t0s)
    be.sync()
    t0 = time.perf_counter()
    span(t0s, t0s + K)
    e.sync()
    be.sync()
    el = time.perf_counter() - t0
    live = np.arange(act.shape[2]) < counts[t0s:t0s + K][..., None]
    corr = int(np.count_nonzero(live[:, :1] & (act[t0s:t0s + K, :1] != 2)))
    e.profile(True)
    span(t0s + K, t0s + 2 * K)
    n_sig, ms_sig = e.profile_read(0)
    n_ch, ms_ch = e.profile_read(1)
    e.profile(False)
    st = e.status(0)
    byt = e.sigma_pass_bytes()
    e.close()
    sig_us = ms_sig / max(n_sig, 1) * 1e3
    out = {"value": corr / el, "unit": "corrections/s", "ms_per_step": el / K * 1e3,
           "steps": K, "dtype": "f64", "status_flags": st,
           "chain_kernel_avg_us": ms_ch / max(n_ch, 1) * 1e3,
           "sigma_pass_avg_us": sig_us,
           "sigma_pass_frac": byt / (sig_us * 1e-6) / 1e9 / HBM_PEAK_GBS if n_sig else None,
           "note": "same survey state, warm-up, messages and entry point as the fp32 value, "
                   "on an fp64 handle (Σ and its pass in fp64), timed after it; not the value"}
    if not args.no_cpu:
        out["parity"] = parity(args, N, ekf_first_poses(args, be, N, be.F64, ws, counts, ids, act,
                                                        rel, odom, t0s, local, gpu_in=gpu_in),
                               ws, counts, ids, act, rel, odom, t0s)
    return out


def reduce_ranks(elapsed, corrections, poses, device):
    """Whole-job numbers across ranks: the slowest rank's time (MAX), the corrections of all ranks
    (SUM), and every filter's final pose gathered to all ranks — the path's one collective (RCCL on
    the GPU box; gloo in tests/test_multirank.py)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(corrections)], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    p = torch.tensor(poses, dtype=torch.float64, device=device)
    gathered = [torch.zeros_like(p) for _ in range(dist.get_world_size())]
    dist.all_gather(gathered, p)
    return float(t.item()), float(c.item()), np.concatenate([g.cpu().numpy() for g in gathered])


def ekf_first_poses(args, be, N, dtype, ws, counts, ids, act, rel, odom, t0s, device,
                    gpu_in=None):
    """Posterior poses of the first timed messages of filter 0 from the same warm state, through
    the path the timed region took (gpu_in: ekf_replay_device on the HBM inputs, a message at a
    time)."""
    k = args.parity_messages
    x, S, tmo, cnt = ws
    e = be.EKF(n_landmarks=N, dtype=dtype, device=device)
    e.set_state(x, S, tmo=tmo, counter=cnt)
    if is_joseph(args.workload):
        e.set_joseph(True)
    sl = slice(t0s, t0s + k)
    un = is_assoc(args.workload)
    if gpu_in is not None:
        p = []
        for t in range(t0s, t0s + k):
            gc, gi, ga, gr, go = (g[t:t + 1, :1].contiguous() for g in gpu_in)
            e.replay_device(gc, gr, go, gi, ga)
            p.append(e.pose(0))
        e.close()
        return np.stack(p)
    p = e.replay(counts[sl, :1], rel[sl, :1], odom[sl, :1], ids=None if un else ids[sl, :1],
                 actions=act[sl, :1], poses=True, assoc=un)[:, 0]
    e.close()
    return p


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc  # noqa: E402  (bench's cpu_baseline / parity legs only)
    orc.build()
    return orc


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max((p.get("num_threads", 1) for p in threadpool_info()
                    if p.get("user_api") == "blas"), default=1)
    except Exception:  # noqa: BLE001
        return None


def cpu_baseline(args, N, ws, counts, ids, act, rel, odom, t0s):
    """The reference's own algorithm on the host cores, over a bounded sample of the same
    messages from the same warm state:
      value       literal dense slam.cpp (At·Σ·Atᵀ, (I−KH)·Σ: O(n³) per correction) through numpy's
                  OpenBLAS dgemm (oracle/ekf_numpy.py) — the reference's Armadillo→BLAS path;
      c_literal   the same dense algebra in the C oracle (a blocked OpenMP GEMM, no BLAS);
      structured  the O(n²) rank-2 restatement (the GPU's algorithm) in the C oracle."""
    orc = _oracle()
    import ekf_numpy  # noqa: E402  (cpu_baseline leg only)
    x, S, tmo, cnt = ws
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    avail = counts.shape[0] - t0s

    def timed(step, k_min, budget):
        ncorr, nmsg = 0, 0
        t0 = time.perf_counter()
        for t in range(t0s, t0s + avail):
            if nmsg >= k_min and time.perf_counter() - t0 >= budget:
                break
            c = int(counts[t, 0])
            step(t, c)
            ncorr += int(np.count_nonzero(act[t, 0, :c] != 2))
            nmsg += 1
        return ncorr, nmsg, time.perf_counter() - t0

    # numpy / OpenBLAS literal (the DenseEKF members of slam.cpp:657-676 set to the warm state)
    jos = is_joseph(args.workload)
    d = ekf_numpy.DenseEKF(n_landmarks=N, joseph=jos)
    d.state, d.sigma, d.counter = x.copy(), S.copy(), int(cnt)
    d.t_map_odom, d.prev = tuple(tmo), tuple(x[:3])

    un = is_assoc(args.workload)

    def np_step(t, c):
        d.t_odom_robot = tuple(odom[t, 0])
        if un:
            d.sensor_cb(rel[t, 0, :c])
        else:
            d.fake_sensor_cb(ids[t, 0, :c], act[t, 0, :c], rel[t, 0, :c])
    nb, kb, tb = timed(np_step, 1, 10.0)
    out = {}
    for literal, k_min, budget in ((True, 1, 10.0), (False, args.steps, 0.0)):
        ref = orc.OracleEKF(n_landmarks=N, literal=literal, joseph=jos)
        ref.set(x, S, tmo, x[:3], cnt)

        def c_step(t, c, ref=ref):
            ref.set_odom(odom[t, 0])
            if un:
                ref.sensor_cb(rel[t, 0, :c])
            else:
                ref.fake_sensor_cb(ids[t, 0, :c], act[t, 0, :c], rel[t, 0, :c])
        out[literal] = timed(c_step, k_min, budget)
    lc, lk, lt = out[True]
    sc_, sk, st = out[False]
    return {"value": nb / tb, "unit": "corrections/s", "cores": _blas_threads() or cores,
            "kind": "port",
            "sample": f"literal dense restatement of slam.cpp{' sensor_cb' if un else ''}"
                      f"{' in Joseph form' if jos else ''} "
                      f"(numpy + OpenBLAS dgemm, fp64, "
                      f"oracle/ekf_numpy.py): {kb} message(s) = {nb} corrections in {tb:.2f} s",
            "c_literal": {"value": lc / lt, "cores": cores,
                          "sample": f"C oracle, dense O(n^3) with a blocked OpenMP GEMM: {lk} "
                                    f"message(s) = {lc} corrections in {lt:.2f} s"},
            "structured": {"value": sc_ / st, "cores": cores,
                           "sample": f"C oracle, O(n^2) rank-2 restatement: {sk} messages = "
                                     f"{sc_} corrections in {st:.2f} s"}}


def parity(args, N, gpu_poses, ws, counts, ids, act, rel, odom, t0s):
    orc = _oracle()
    x, S, tmo, cnt = ws
    ref = orc.OracleEKF(n_landmarks=N, joseph=is_joseph(args.workload))
    ref.set(x, S, tmo, x[:3], cnt)
    k = len(gpu_poses)
    ref_p = np.zeros((k, 3))
    for i, t in enumerate(range(t0s, t0s + k)):
        ref.set_odom(odom[t, 0])
        c = int(counts[t, 0])
        if is_assoc(args.workload):
            ref.sensor_cb(rel[t, 0, :c])
        else:
            ref.fake_sensor_cb(ids[t, 0, :c], act[t, 0, :c], rel[t, 0, :c])
        ref_p[i] = ref.get(sigma=False)[0][:3]
    d = gpu_poses - ref_p
    dth = np.arctan2(np.sin(d[:, 0]), np.cos(d[:, 0]))
    return {"pose_rmse_m": float(np.sqrt(np.mean(d[:, 1] ** 2 + d[:, 2] ** 2))),
            "heading_rmse_rad": float(np.sqrt(np.mean(dth ** 2))),
            "messages": k, "vs": "oracle structured fp64 (CPU), filter 0, same warm state" + (
                ", Joseph mode" if is_joseph(args.workload) else "")}


if __name__ == "__main__":
    main()
