"""bench.py's multi-rank path (weak scaling over independent filters) on gloo, world size 2.

The GPU box runs `bench.py --gpus N` (N ranks over RCCL, each owning its own filters); here the same
`bench.run()` runs end to end on the CPU in two processes, as SURVEY.md §8(e) prescribes for the N>1
path: per-rank seeded inputs (filter g = rank·F + f uses seed + g), the survey warm-up, the timed
region between barriers, MAX/SUM over ranks and the all_gather of every filter's final pose. The
filters of this CPU test are the C oracle (test infrastructure, injected as bench's backend); the
product path itself needs the GPU and is exercised by the `-m gpu` tests and bench runs.
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = (24, "f64", 3, 6, "test: N=24 x 3 filters per rank, fp64")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleSwarm:
    """bench's EKF interface over one C-oracle filter per index (CPU, fp64)."""

    def __init__(self, n_landmarks, n_filters=1, dtype=0, device=0):
        import orc
        self.N, self.F = n_landmarks, n_filters
        self.f = [orc.OracleEKF(n_landmarks=n_landmarks) for _ in range(n_filters)]

    def replay(self, counts, rel, odom, ids=None, actions=None, poses=False, assoc=False):
        T = counts.shape[0]
        out = np.zeros((T, self.F, 3))
        for t in range(T):
            for f, e in enumerate(self.f):
                c = int(counts[t, f])
                e.set_odom(odom[t, f])
                if assoc:
                    e.sensor_cb(rel[t, f, :c])
                else:
                    e.fake_sensor_cb(ids[t, f, :c], actions[t, f, :c], rel[t, f, :c])
                out[t, f] = e.get(sigma=False)[0][:3]
        return out if poses else None

    def state(self, f=0, sigma=True):
        x, S, _, cnt = self.f[f].get(sigma=sigma)
        return x, S, cnt

    def map_odom(self, f=0):
        return self.f[f].get(sigma=False)[2]

    def set_state(self, state, sigma=None, tmo=None, counter=0, f=0):
        self.f[f].set(state, sigma, tmo, state[:3], counter)

    def pose(self, f=0):
        return self.f[f].get(sigma=False)[0][:3]

    def status(self, f=0):
        return 0

    def sync(self):
        pass

    def flush(self):
        pass

    def profile(self, on=True):
        pass

    def profile_read(self, k):
        return 0, 0.0

    def sigma_pass_bytes(self, filters=None):
        return 0.0

    def close(self):
        pass


class CpuBackend:
    dist_backend = "gloo"
    device = "cpu"
    F32, F64 = 1, 0
    EKF = OracleSwarm

    def sync(self):
        pass


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    bench.WORKLOADS["tiny"] = TINY
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    args = bench.parse(["--workload", "tiny", "--gpus", str(world), "--steps", "3",
                        "--warmup", "2", "--traffic", "off", "--parity-messages", "2"])
    try:
        result, poses = bench.run(args, rank, world, 0, CpuBackend())
    except BaseException as e:  # report at once instead of leaving the parent to time out
        q.put((rank, repr(e), None))
        raise
    q.put((rank, result, poses))



def test_bench_run_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {r: (res, poses) for r, res, poses in (q.get(timeout=300) for _ in procs)}
    for r, (res, _) in out.items():
        assert not isinstance(res, str), f"rank {r}: {res}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res, poses = out[0]
    assert out[1][0] is None  # only rank 0 reports
    assert res["n_gpus"] == 2 and res["config"]["filters_total"] == 6
    di = res["config"]["distributed"]  # the line records what the process group saw
    assert di["world_size"] == 2 and di["backend"] == "gloo"
    assert [r["rank"] for r in di["ranks"]] == [0, 1] and di["ranks"][0]["pid"] != di["ranks"][1]["pid"]
    assert res["config"]["landmarks_initialised_min"] == 24  # the survey sighted every landmark
    assert res["value"] > 0 and res["gathered_poses"]["filters"] == 6
    assert res["parity"]["pose_rmse_m"] == 0.0
    np.testing.assert_array_equal(poses, out[1][1])  # all_gather: every rank holds all poses
    # the gathered poses are those of global filters 0..5 seeded seed + g, in rank order
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    N, _, F, m, _ = TINY
    sw, odom, _ = bench.build_inputs(N, 2 * F, 2 + 2 * 3, 20240317, m, 0)
    n_warm, counts, ids, act, rel = sw.n_warm, sw.count, sw.ids, sw.actions, sw.rel
    ref = OracleSwarm(N, 2 * F)
    ref.replay(counts[:n_warm + 2 + 3], rel[:n_warm + 5], odom[:n_warm + 5], ids=ids[:n_warm + 5],
               actions=act[:n_warm + 5])
    want = np.stack([ref.pose(g) for g in range(2 * F)])
    np.testing.assert_allclose(poses, want, rtol=0, atol=1e-12)


def _reduce_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = 3  # filters per rank; rank r owns filters [3r, 3r+3)
    poses = np.arange(F * 3, dtype=np.float64).reshape(F, 3) + 100 * rank
    elapsed, total, gathered = bench.reduce_ranks(0.5 + rank, 10 * (rank + 1), poses, "cpu")
    q.put((rank, elapsed, total, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, total, gathered in out:
        assert elapsed == 1.5            # MAX over ranks
        assert total == 30.0             # SUM of corrections
        assert gathered.shape == (6, 3)  # contiguous filter blocks, rank order
        np.testing.assert_array_equal(gathered[:3], np.arange(9.0).reshape(3, 3))
        np.testing.assert_array_equal(gathered[3:], np.arange(9.0).reshape(3, 3) + 100)


def test_gpus_flag_launches_ranks(monkeypatch):
    """`bench.py --gpus N` without a launcher starts N ranks through torch.distributed.run as a
    child process (this process never initialises a GPU) and returns the launcher's status."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []

    class R:
        returncode = 0

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr("subprocess.run", lambda cmd, **kw: calls.append(cmd) or R())
    try:
        bench.main(["--gpus", "4", "--workload", "swarm_n256_fp64", "--steps", "5"])
    except SystemExit as e:
        assert e.code == 0
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[-6:] == ["--gpus", "4", "--workload", "swarm_n256_fp64", "--steps", "5"]
