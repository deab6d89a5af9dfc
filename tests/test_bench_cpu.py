"""bench.py's JSON line without a GPU: the fields the driver's multi-GPU scaling run reads
are built from the measurements the way a torchrun launch builds them.  Two gloo ranks
stand in for two GPUs: each reports its own batch times and kernel times, ``reduce_max``
takes the max over ranks, and rank 0 builds the line with ``make_line``."""
import argparse
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _fake_result(world, rank, model="wholebody", K=8192, H=64, native=False, backend="gloo"):
    rng = np.random.default_rng(rank)
    return {"batches_s": list(20 * 20e-6 * (1 + 0.05 * rng.random(7)) * (1 + rank)), "dt": None,
            "enqueue_s": list(20 * 8e-6 * np.ones(7)),
            "tim": {"rollout_us": 12.5 + rank, "finalize_us": 4.8, "pair_us": 17.4 + rank,
                    "rollout_in_step_us": 12.6 + rank, "method": "fake"},
            "lat": [3e-5] * 10, "K": K, "H": H, "A": 10, "V": 1, "strong": True,
            "bytes": K * H * 88 + 4 * K, "ess": 1.0, "model": model, "state_f64": False, "native": native,
            "exchange": "rccl" if native else "torch", "native_error": None, "world": world, "backend": backend,
            "rccl_nranks": world if native else None, "rccl_rank": rank if native else None}


def _args(steps=20):
    return argparse.Namespace(steps=steps, warmup=5)


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = _fake_result(world, rank, K=65536 // world)
        r["batches_s"] = bench.reduce_max(r["batches_s"], dist, "cpu")
        r["dt"] = float(np.median(r["batches_s"]))
        t = r["tim"]
        t["rollout_us_max_over_ranks"], t["rollout_in_step_us_max_over_ranks"] = bench.reduce_max(
            [t["rollout_us"], t["rollout_in_step_us"]], dist, "cpu")
        q.put((rank, bench.make_line("c4", r, _args()) if rank == 0 else None, r["batches_s"]))
    finally:
        dist.destroy_process_group()


def test_bench_line_two_gloo_ranks():
    """The SCALE line of a 2-rank gloo rehearsal: no RCCL communicator is claimed
    (rccl_nranks null, backend gloo), the batch times are the max over ranks, the roofline
    is the rank's own launch shape (K = 65536/2) with traffic of that shape only, and the
    step-level fraction is N*bytes/step/(N*8 TB/s)."""
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    line = res[0][1]
    assert res[0][2] == res[1][2], "every rank holds the max-over-ranks batch times"
    worst = [max(a, b) for a, b in zip(_fake_result(2, 0)["batches_s"], _fake_result(2, 1)["batches_s"])]
    assert np.allclose(res[0][2], worst)
    mg = line["multi_gpu"]
    assert mg["rccl_nranks"] is None and mg["backend"] == "gloo" and mg["world_size"] == 2
    assert "gloo" in mg["collective"]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["samples_per_gpu"] == 32768 and line["config"]["samples_total"] == 65536
    step = float(np.median(worst)) / 20
    assert line["ms_per_step"] == pytest.approx(step * 1e3)
    assert line["value"] == pytest.approx(2 * 32768 * 64 / step)
    assert line["timing"]["timed_batches"] == 7
    rf = line["roofline"]
    assert rf["launch_shape"] == "wholebody_k32768_h64"
    assert rf["bytes_per_launch"] == 32768 * 64 * 88 + 4 * 32768
    bytes_ = rf["bytes_per_launch"]
    assert rf["frac_step"] == pytest.approx(2 * bytes_ / step / (2 * 8e12))
    if rf["traffic"] is not None:   # counters of exactly this shape, never another shape's
        assert 1.0 <= rf["traffic_over_algorithmic"] < 1.1
        assert "wholebody_k32768_h64" in rf["traffic_source"]
    assert line["kernels"]["rollout_in_step_us_max_over_ranks"] == pytest.approx(13.6)


def test_bench_line_native_one_rank_and_traffic_by_shape():
    """A 1-rank RCCL run names the communicator's own rank count; traffic is looked up by
    launch shape (the N=8 c4 rank shape has counters; a shape without any gets null)."""
    r = _fake_result(1, 0, native=True, backend=None)
    r["dt"] = float(np.median(r["batches_s"]))
    line = bench.make_line("c4_shard_native1", r, _args())
    assert line["multi_gpu"]["rccl_nranks"] == 1
    assert "ncclCommCount" in line["multi_gpu"]["rccl_nranks_source"]
    rf = line["roofline"]
    assert rf["launch_shape"] == "wholebody_k8192_h64"
    assert rf["traffic"] is not None and 1.0 <= rf["traffic_over_algorithmic"] < 1.1
    r = _fake_result(1, 0, K=1000)
    r["dt"] = float(np.median(r["batches_s"]))
    assert bench.make_line("wholebody_c4", r, _args())["roofline"]["traffic"] is None
    assert bench.load_traffic("wholebody_k1000_h64") == (None, None)


def test_auto_batches():
    assert bench.auto_batches(20) == 7 and bench.auto_batches(500) == 3 and bench.auto_batches(5000) == 1


def test_primary_weak_and_c4_secondary_at_two_ranks():
    """Under torchrun the primary stays the metric's arm_c3 shape, weak-scaled (K=4096 per
    rank, total 4096*N), so a scaling curve's N=1 point measures what its N>1 points do; the
    north-star c4 (K=65536 split over the ranks) is reported beside it as secondary.c4 with
    the whole job's rollout-steps/s."""
    r = _fake_result(2, 0, model="arm", K=4096, H=32)
    r.update(A=7, strong=False, bytes=4096 * 32 * 76 + 4 * 4096, state_f64=True, exchange="peer", native=True,
             rccl_nranks=None, rccl_rank=None)
    r["dt"] = float(np.median(r["batches_s"]))
    line = bench.make_line("arm_c3", r, _args())
    step = r["dt"] / 20
    assert line["scaling"] == "weak" and line["n_gpus"] == 2
    assert line["config"]["samples_per_gpu"] == 4096 and line["config"]["samples_total"] == 8192
    assert line["value"] == pytest.approx(2 * 4096 * 32 / step)
    assert "peer exchange" in line["config"]["parallelism"] and line["multi_gpu"]["exchange"] == "peer"
    s = _fake_result(2, 0, K=32768)
    s["dt"] = float(np.median(s["batches_s"]))
    s["tim"]["rollout_in_step_us_max_over_ranks"] = 13.6
    e = bench.secondary_entry(s, 20)
    assert e["n_gpus"] == 2 and e["scaling"] == "strong" and e["samples_total"] == 65536
    assert e["value"] == pytest.approx(65536 * 64 / (s["dt"] / 20))
    assert e["rollout_us_max_over_ranks"] == 13.6 and e["exchange"] == "torch"


# ------------------------------------------------------------ bench.py --gpus N without a launcher
_STUB = r"""
import json, os, sys
rank = int(os.environ.get("RANK", "0"))
print("a rank's stray stdout line", flush=True)
if rank == 0:
    print(json.dumps({"metric": "m", "value": 1.0, "argv": sys.argv[1:],
                      "world": os.environ.get("WORLD_SIZE"), "spawned": os.environ.get("MPPI_BENCH_SPAWNED")}),
          flush=True)
sys.exit(int(os.environ.get("STUB_RC", "0")))
"""


def test_spawn_ranks_relays_one_line_and_the_child_rc(tmp_path, capsys):
    """``bench.py --gpus N`` without WORLD_SIZE runs the ranks as a CHILD
    (spawn_ranks) and relays exactly one bench line -- rank 0's; other stdout lines go to stderr --
    and returns the child's exit code.  Stub child: a script that prints what it was given."""
    import io
    import sys
    stub = tmp_path / "stub.py"
    stub.write_text(_STUB)
    for rc in (0, 3):
        out = io.StringIO()
        env_rc = {"STUB_RC": str(rc)}
        os.environ.update(env_rc)
        try:
            got = bench.spawn_ranks([sys.executable, str(stub), "--gpus", "2", "--steps", "7"], out=out)
        finally:
            del os.environ["STUB_RC"]
        lines = [ln for ln in out.getvalue().splitlines() if ln.strip()]
        assert got == rc and len(lines) == 1, (got, lines)
        d = json.loads(lines[0])
        assert d["argv"] == ["--gpus", "2", "--steps", "7"] and d["spawned"] == "1"
    assert "stray stdout line" in capsys.readouterr().err
    # a child that prints no bench line and exits 0 is a failure, not a silent empty run
    quiet = tmp_path / "quiet.py"
    quiet.write_text("print('nothing to relay')\n")
    out = io.StringIO()
    assert bench.spawn_ranks([sys.executable, str(quiet)], out=out) == 1 and out.getvalue() == ""


def test_spawn_through_torch_distributed_run(tmp_path):
    """The launcher command itself (torch.distributed.run, static rendezvous on 127.0.0.1): two ranks
    of a stub, every argument forwarded after the script, WORLD_SIZE = 2 in the ranks, rank 0's line
    relayed alone, the launcher's exit code returned."""
    import io
    stub = tmp_path / "stub.py"
    stub.write_text(_STUB)
    argv = ["--gpus", "2", "--steps", "20", "--warmup", "5", "--secondary", ""]
    cmd = bench.launcher_cmd(2, argv, script=str(stub))
    assert cmd[cmd.index(str(stub)) + 1:] == argv and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert bench.launcher_cmd(8, argv)[-len(argv) - 1] == os.path.abspath(bench.__file__)
    out = io.StringIO()
    rc = bench.spawn_ranks(cmd, out=out)
    lines = [ln for ln in out.getvalue().splitlines() if ln.strip()]
    assert rc == 0 and len(lines) == 1, (rc, lines)
    d = json.loads(lines[0])
    assert d["argv"] == argv and d["world"] == "2"


def test_main_spawns_without_a_launcher(monkeypatch):
    """main() with --gpus 2 and no WORLD_SIZE goes to spawn_ranks with its own argv, before any GPU
    call, and exits with the child's code; under a launcher (WORLD_SIZE set) it never spawns."""
    import sys
    seen = {}

    def fake_spawn(cmd, out=None):
        seen["cmd"] = cmd
        return 5
    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("MPPI_BENCH_SPAWNED", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "9"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 5
    assert seen["cmd"][-4:] == ["--gpus", "2", "--steps", "9"] and "--nproc-per-node=2" in seen["cmd"]
    monkeypatch.setenv("MPPI_BENCH_SPAWNED", "1")
    with pytest.raises(SystemExit, match="own launcher"):
        bench.main()


# ------------------------------------------------------------ a failed secondary does not cost the line
def test_secondary_failure_is_reported_not_fatal(monkeypatch):
    """At N = 1 a secondary that raises (any exception) becomes {"error": ...} in the line and the
    next secondary still runs; at N > 1 only StepsGivenUp (raised on every rank together) is
    caught, anything else ends the run.  The engine is closed either way (run_workload's finally)."""
    monkeypatch.setattr(bench, "log", lambda *a: None)
    calls = []

    def fake_run(name, ns, warmup, world, dist, lat_steps, batches=1):
        calls.append(name)
        if name == "bad":
            raise RuntimeError("boom")
        if name == "given_up":
            raise bench.StepsGivenUp("given up")
        r = _fake_result(world, 0, K=8192)
        r["dt"] = float(np.median(r["batches_s"]))
        return r

    out = bench.run_secondaries(["bad", "good", "given_up"], 500, 1, None, 1, run=fake_run)
    assert calls == ["bad", "good", "given_up"]
    assert out["bad"] == {"error": "RuntimeError: boom"}
    assert out["given_up"]["error"].startswith("StepsGivenUp")
    assert out["good"]["value"] > 0 and out["good"]["samples"] == 8192
    out = bench.run_secondaries(["given_up", "good"], 500, 2, None, 1, run=fake_run)
    assert "error" in out["given_up"] and "value" in out["good"]
    with pytest.raises(RuntimeError, match="boom"):
        bench.run_secondaries(["bad"], 500, 2, None, 1, run=fake_run)


def test_guarded_reports_the_error():
    assert bench.guarded("x", lambda: 3) == 3
    g = bench.guarded("x", lambda: 1 / 0)
    assert g["error"].startswith("ZeroDivisionError")


_MAIN_STUB = r"""
import sys, numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, TESTS)
import bench
from test_bench_cpu import _fake_result

def fake_run(name, steps_n, warmup, world, dist, lat_steps, timing=True, batches=1, lat_rate_calls=0):
    if name == "drone_c2":
        raise RuntimeError("secondary boom")
    r = _fake_result(1, 0, model="arm", K=4096, H=32)
    r.update(A=7, strong=False, bytes=4096 * 32 * 76 + 4 * 4096, state_f64=True, exchange=None, native=False)
    r["dt"] = float(np.median(r["batches_s"]))
    return r

def boom():
    raise OSError("no host sampling here")

bench.run_workload = fake_run
bench.dropin_latency = lambda n: boom()
bench.cpu_baseline = lambda w, b: boom()
bench.measured_hbm = lambda local: {"fill_GBps": 5000.0}
sys.argv = ["bench.py", "--steps", "20", "--warmup", "5", "--no-numa-bind", "--secondary", "drone_c2,wholebody_c4"]
bench.main()
"""


def test_main_prints_one_line_when_parts_fail(tmp_path):
    """bench.main() at N = 1 with a secondary, the drop-in latency and the CPU baseline all failing
    (stand-ins for the GPU workloads, run in a child: main() re-points fd 1): still exactly one JSON
    line on stdout, the failures named in it, the primary's numbers intact."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = f"ROOT = {os.path.dirname(here)!r}\nTESTS = {here!r}\n" + _MAIN_STUB
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(here))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["config"]["workload"] == "arm_c3" and line["value"] > 0
    assert line["secondary"]["drone_c2"] == {"error": "RuntimeError: secondary boom"}
    assert line["secondary"]["wholebody_c4"]["value"] > 0
    assert line["dropin_latency"]["error"].startswith("OSError")
    assert line["cpu_baseline"]["error"].startswith("OSError") and line["cpu_baseline_all"] is None
    assert line["roofline"]["peak_measured"] == {"fill_GBps": 5000.0}


_RUN_STUB = r"""
import sys, types, numpy as np
sys.path.insert(0, ROOT)
import torch
torch.cuda.synchronize = lambda *a, **k: None   # (no device here: the fake engine below stands in)
import bench
import quadrotor_manipulator_mppi_amd.distributed as D

class Stat:
    ess = 123.0

class FakeEngine:
    def __init__(self, model, K, H, V):
        self.K, self.H, self.V = K, H, V
        self.A = {"arm": 7, "drone": 3, "wholebody": 10, "quadrotor": 4}[model]
        self.cfg = types.SimpleNamespace(state_f64=model == "arm", quad_mass=1.0, quad_gravity=9.81)
        self.closed = 0
        self.steps = 0
    def set_target(self, *a, **k): pass
    def set_u_prev(self, u): pass
    def set_state(self, s): assert s.shape[0] == self.V
    def kernel_timing_ex(self, n): return (5.0, 4.0, 9.0)
    def exchange_timing(self, n): return 2.0
    def set_prewarm(self, us): pass
    def prewarm(self): return (0, 7)
    def dispatch_info(self): return "fake"
    def read_outputs(self): return np.zeros((self.V, 14)), np.zeros((self.V, self.A)), [Stat()]
    def comm_info(self): return (1, 0)
    def peer_info(self): return (1, 0, 0)
    def rollout_bytes(self): return self.K * self.H * 76
    def synchronize(self): pass
    def close(self):
        self.closed += 1
        CLOSED.append(self)

CLOSED = []

class FakeSharded:
    def __init__(self, seed, native, mode, model, n_samples, n_horizon, n_vehicles=1, **kw):
        self.engine = FakeEngine(model, n_samples, n_horizon, n_vehicles)
        self.vehicles = range(0, n_vehicles)
        self.mode, self.native, self.native_error, self.agree_every = mode or "torch", bool(native), None, None
        self.give_up = FAIL == model
    def run_steps(self, n): self.engine.steps += n
    def synchronize(self): return self.give_up and self.engine.steps > 100
    def step(self, state): return None

D.ShardedEngine = FakeSharded
r = bench.run_workload("arm_c3", 20, 5, 1, None, 3, batches=2, lat_rate_calls=2)
assert r["K"] == 4096 and r["H"] == 32 and len(r["batches_s"]) == 2 and r["ess"] == 123.0, r
assert r["tim"]["rollout_in_step_us"] == 5.0 and len(r["lat"]) == 3 and len(r["lat100"]) == 2
assert [e.closed for e in CLOSED] == [1]
FAIL = "wholebody"
try:
    bench.run_workload("wholebody_c4", 20, 5, 1, None, 0, batches=1)
    raise SystemExit("no StepsGivenUp")
except bench.StepsGivenUp:
    pass
assert [e.closed for e in CLOSED] == [1, 1], "the engine is closed when a step is given up"
print("RUN_OK")
"""


def test_run_workload_with_a_stand_in_engine():
    """run_workload's own logic on the CPU (the GPU engine replaced by a stand-in, torch.cuda's
    synchronize stubbed): batches, kernel timing, latency legs and results; a given-up peer step
    raises StepsGivenUp and the engine is still closed."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = f"ROOT = {os.path.dirname(here)!r}\nFAIL = None\n" + _RUN_STUB
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(here))
    assert p.returncode == 0 and "RUN_OK" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])
