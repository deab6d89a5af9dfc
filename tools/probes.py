"""GPU diagnostics for the control step (tools/, not shipped; none of it is on the product path).

    python tools/probes.py <probe> [args]

probes:
  timeline <workload> [trials]   wall-clock timeline of one step (kernel spans and the gaps between
                                 them); needs a timeline build: MPPI_HIP_LIB=<lib built with
                                 MPPI_HIPCC_EXTRA="-DMPPI_STAMPS -DMPPI_TIMELINE"> MPPI_STAMPS=1
                                 MPPI_EVENT_WAIT=1 MPPI_DEBUG_NO_FLAG=1
  batch                          short-batch cost, native vs HIP dispatch: run_steps(n)+synchronize
                                 for n = 1..200 -> per-batch intercept and per-step slope
  fences                         C3 step rate and bit-exactness vs HIP under MPPI_AQL_FENCES
  calls [modes]                  control-call latency p50/p90/p99, native vs HIP (comma list)
  sequence                       (rollout, X) pair costs; MPPI_PROBE builds only
  stamps <model> <K> <H> [threads] [nb]
                                 per-wave phase timelines of the last rollout (stamps build,
                                 MPPI_STAMPS=1): shader clock, wave lifetimes, per-XCD / per-CU ends
  latency [model] [K] [H]        control-call latency split: enqueue vs read_outputs, flag vs event wait
  rate [model] [K] [H] [calls]   control-call latency vs the idle gap before each call (100 Hz node):
                                 back to back, 10 ms sleep, 10 ms host spin, 1 ms, 0.1 ms
  store_floor [sizes] [launches] write-only floor (torch fill_) at the rollouts' per-launch bytes
  noise_src [model] [K] [H] [n]  rollout with device Philox vs noise read from HBM (run under a kernel trace)
  geom [model] [K] [H] [bpvs] [threads]
                                 rollout / finalize / pair times per blocks-per-vehicle choice
  peer_soak [model] [K] [H] [G] [batches] [steps]
                                 G in-process peer-exchange ranks for batches x steps: no timeout, ranks
                                 bit-identical after every batch
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]
STATES = {"arm": [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 7,
          "drone": [0, 0, 1, 0, 0, 0],
          "wholebody": [0, 0, 1, 0, 0, 0, 1] + HOME + [0.0] * 10}
ARM_T = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])


def _engine(model="arm", K=4096, H=32, dispatch=None, **kw):
    from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
    if dispatch is not None:
        os.environ["MPPI_DISPATCH"] = dispatch
    e = Engine(make_config(model, device=0, n_samples=K, n_horizon=H, state_f64=(model == "arm"), **kw))
    e.set_target(*ARM_T)
    e.set_state(np.array(STATES[model], np.float64))
    return e


def probe_timeline(name, trials="30"):
    """Every rollout wave and finalize block of a timeline build stores s_memrealtime (100 MHz) at
    its start and end; per trial the engine runs back-to-back steps and the stamps of the LAST step
    are read: rollout first wave start .. last wave end, [PACK ..,] FINAL .., relative to the
    rollout's first wave start.  Medians over the trials: kernel spans and launch gaps."""
    import bench
    from quadrotor_manipulator_mppi_amd.distributed import ShardedEngine
    trials = int(trials)
    w = dict(bench.WORKLOADS[name])
    w.pop("desc")
    w.pop("strong", None)
    native = w.pop("native", None)
    se = ShardedEngine(seed=1234, native=native, **w)
    eng = se.engine
    V = w.get("n_vehicles", 1)
    bench.set_targets(eng, w["model"], se.vehicles)
    eng.set_state(bench.make_state(w["model"], V))
    L = eng._L
    L.mppi_debug_stamps.restype = C.c_int64
    L.mppi_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    L.mppi_debug_fstamps.restype = C.c_int64
    L.mppi_debug_fstamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
    rb = np.zeros((1 << 18, 16), np.uint64)
    fb = np.zeros((4096, 16), np.uint64)
    se.run_steps(50)
    eng.synchronize()
    periods = []   # the step period of this build (the stamps' own cost included)
    for _ in range(5):
        t0 = time.perf_counter()
        se.run_steps(500)
        eng.synchronize()
        periods.append((time.perf_counter() - t0) / 500 * 1e9)
    rows = []
    for _ in range(trials):
        se.run_steps(10)
        eng.synchronize()
        n = L.mppi_debug_stamps(eng._h, rb.ctypes.data, rb.shape[0])
        r = rb[:n].astype(np.int64)
        t0 = r[:, 13].min()
        xcc = (r[:, 15] >> 32) & 0xF
        row = {"roll_last_start": (r[:, 13].max() - t0) * 10.0, "roll_first_end": (r[:, 14].min() - t0) * 10.0,
               "roll_end": (r[:, 14].max() - t0) * 10.0,
               "roll_life_med": float(np.median(r[:, 14] - r[:, 13])) * 10.0,
               # phases per wave: prologue (loads, LDS staging, barrier), the rollout groups, the
               # block combine + record (slots 1 and 5 of the timeline build)
               "roll_prologue_med": float(np.median(r[:, 1] - r[:, 13])) * 10.0,
               "roll_philox_med": float(np.median(r[:, 10] - r[:, 13])) * 10.0,
               "roll_staging_med": float(np.median(r[:, 1] - r[:, 10])) * 10.0,
               "roll_groups_med": float(np.median(r[:, 5] - r[:, 1])) * 10.0,
               "roll_combine_med": float(np.median(r[:, 14] - r[:, 5])) * 10.0}
        if (r[:, 3] > 0).all():   # a -DMPPI_TIMELINE_FINE=1 build: every phase boundary stamped
            chain = [(13, "start"), (9, "loads_issued"), (10, "philox"), (8, "staging_stores"), (1, "barrier"),
                     (2, "noise"), (3, "integrator"), (4, "fk_cost_stores"), (5, "cost_sum_softmin"),
                     (11, "lds_deposit"), (6, "combine_barrier"), (12, "cost_stores_fw"), (7, "record_body"),
                     (14, "end")]
            for (a, _), (b, nm) in zip(chain, chain[1:]):
                row[f"phase_{nm}_med"] = float(np.median(r[:, b] - r[:, a])) * 10.0
        for c in range(8):
            m = xcc == c
            if m.any():
                row[f"roll_xcd{c}_start"] = (r[m, 13].min() - t0) * 10.0
                row[f"roll_xcd{c}_end"] = (r[m, 14].max() - t0) * 10.0
        for which, key in ((1, "pack"), (0, "final")):
            m = L.mppi_debug_fstamps(eng._h, fb.ctypes.data, fb.shape[0], which)
            f = fb[:m].astype(np.int64)
            f = f[(f[:, 13] > 0) & (f[:, 14] >= f[:, 13])]
            if len(f) and (f[:, 13].min() >= t0 or key == "final"):
                row[key + "_start"] = (f[:, 13].min() - t0) * 10.0
                row[key + "_end"] = (f[:, 14].max() - t0) * 10.0
                row[key + "_life_med"] = float(np.median(f[:, 14] - f[:, 13])) * 10.0
                row[key + "_last_start"] = (f[:, 13].max() - t0) * 10.0
                row[key + "_records_med"] = float(np.median(f[:, 1] - f[:, 13])) * 10.0
                row[key + "_issue_med"] = float(np.median(f[:, 7] - f[:, 13])) * 10.0
                row[key + "_tail_med"] = float(np.median(f[:, 14] - f[:, 1])) * 10.0
                fx = f[:, 15] & 0xF
                for c in range(8):
                    m = fx == c
                    if m.any():   # per XCD: first block start, last records-combined, last end
                        row[f"{key}_xcd{c}_start"] = (f[m, 13].min() - t0) * 10.0
                        row[f"{key}_xcd{c}_records"] = (f[m, 1].max() - t0) * 10.0
                        row[f"{key}_xcd{c}_end"] = (f[m, 14].max() - t0) * 10.0
        rows.append(row)
    med = {k: float(np.median([r[k] for r in rows if k in r])) for k in rows[0].keys()}
    out = {"workload": name, "trials": trials, "dispatch": eng.dispatch_info(),
           "ns_median": {k: round(v) for k, v in med.items()}}
    if "final_start" in med:
        gaps = {"rollout_span": med["roll_end"]}
        prev = med["roll_end"]
        if "pack_start" in med:
            gaps["gap_rollout_pack"] = med["pack_start"] - prev
            gaps["pack_span"] = med["pack_end"] - med["pack_start"]
            prev = med["pack_end"]
        gaps["gap_to_final"] = med["final_start"] - prev
        gaps["final_span"] = med["final_end"] - med["final_start"]
        gaps["step_to_final_end"] = med["final_end"]
        gaps["step_period"] = float(np.median(periods))
        gaps["gap_final_to_next_rollout"] = gaps["step_period"] - med["final_end"]
        out["us"] = {k: round(v / 1e3, 3) for k, v in gaps.items()}
    print(json.dumps(out), flush=True)
    eng.close()


def probe_batch():
    """Median wall time of run_steps(n); synchronize() after an untimed priming batch each time:
    the intercept is the per-batch bracket (first kernel start + completion wake-up), the slope
    the per-step time."""
    import torch
    engines = {}
    for m in ("hip", "aql"):
        engines[m] = _engine(dispatch=m, seed=3)
        engines[m].run_steps(50)
        engines[m].synchronize()
    ns = [1, 2, 5, 10, 20, 50, 200]
    # "aql_t": the same native engine with torch's synchronize ahead of the engine's (bench.py's
    # bracket since round 4: torch's idle-device cost overlaps the running batch)
    variants = [("hip", "hip", False), ("aql", "aql", False), ("aql_t", "aql", True)]
    res = {m: {} for m, _, _ in variants}
    for _ in range(15):
        for m, em, torch_first in variants:
            e = engines[em]
            for n in ns:
                e.run_steps(10)   # priming, untimed
                e.synchronize()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e.run_steps(n)
                t1 = time.perf_counter()
                if torch_first:
                    torch.cuda.synchronize()
                    ts = time.perf_counter()
                    e.synchronize()
                else:
                    e.synchronize()
                    ts = time.perf_counter()
                    torch.cuda.synchronize()
                t2 = time.perf_counter()
                e.synchronize()          # both again, idle: the bracket's own host cost
                ti = time.perf_counter()
                torch.cuda.synchronize()
                tj = time.perf_counter()
                res[m].setdefault(n, []).append(((t2 - t0) * 1e6, (t1 - t0) * 1e6, (ts - t1) * 1e6,
                                                 (t2 - ts) * 1e6, (ti - t2) * 1e6, (tj - ti) * 1e6))
    for m in res:
        tot = [np.median([x[0] for x in res[m][n]]) for n in ns]
        enq = [np.median([x[1] for x in res[m][n]]) for n in ns]
        slope, icpt = np.polyfit(ns, tot, 1)
        print(f"{m}: " + "  ".join(f"n={n}: {t:.1f} us (enq {q:.1f})" for n, t, q in zip(ns, tot, enq)) +
              f"  | fit: {slope:.2f} us/step + {icpt:.1f} us per batch; n=20 -> {tot[ns.index(20)] / 20:.2f} us/step")
        for n in (1, 20):
            med = np.median(np.array(res[m][n]), axis=0)
            print(f"  {m} n={n}: run_steps call {med[1]:.1f}, first sync {med[2]:.1f}, second sync {med[3]:.1f} us; "
                  f"idle: engine sync {med[4]:.1f}, torch sync {med[5]:.1f} us")


def probe_fences():
    """Native dispatch under MPPI_AQL_FENCES (diagnostic packet fence scopes)."""
    h, a = _engine(dispatch="hip", seed=3), _engine(dispatch="aql", seed=3)
    for e in (h, a):
        e.run_steps(300)
        e.synchronize()
    ok = np.array_equal(h.get_u_prev(), a.get_u_prev()) and np.array_equal(h.get_costs(), a.get_costs())
    rates = []
    for _ in range(5):
        a.run_steps(50)
        a.synchronize()
        t0 = time.perf_counter()
        a.run_steps(1000)
        a.synchronize()
        rates.append((time.perf_counter() - t0) / 1000 * 1e6)
    print(f"fences={os.environ.get('MPPI_AQL_FENCES', 'default 0000')} bit-exact vs HIP after 300 steps: {ok}  "
          f"us/step (1000-step batches): median {np.median(rates):.2f}  all {[round(x, 2) for x in rates]}")


def probe_calls(modes="hip,aql"):
    """Engine.step latency at C3 with a changing state, modes interleaved in blocks of 200."""
    import torch  # noqa: F401  (the bench's process shape)
    modes = modes.split(",")
    eng = {m: _engine(dispatch=m, seed=3) for m in modes}
    st0 = np.array(STATES["arm"], np.float64)
    rng = np.random.default_rng(0)
    lat = {m: [] for m in modes}
    for _ in range(10):
        for m, e in eng.items():
            for i in range(220):
                st = st0.copy()
                st[7:14] += rng.normal(0, 0.01, 7)
                t0 = time.perf_counter()
                e.step(st)
                if i >= 20:
                    lat[m].append((time.perf_counter() - t0) * 1e6)
    for m in modes:
        x = np.array(lat[m])
        print(f"{m}: calls {eng[m].dispatch_info()!r}  p50 {np.median(x):.2f} us  p10 {np.percentile(x, 10):.2f}  "
              f"p90 {np.percentile(x, 90):.2f}  p99 {np.percentile(x, 99):.2f}")


def probe_sequence():
    """What a (rollout, X) pair costs for X = an empty kernel, a one-block rollout, the finalize."""
    names = ["rollout+empty", "rollout+rollout(1 block)", "rollout+finalize", "empty", "rollout(1 block)", "rollout"]
    for model, K, H in (("arm", 4096, 32), ("wholebody", 8192, 64)):
        e = _engine(model, K, H)
        e.run_steps(100)
        e.synchronize()
        fn = e._L.mppi_probe_sequence
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_double)]
        res = {}
        for _ in range(5):
            for m in range(6):
                us = C.c_double()
                fn(e._h, 200, m, C.byref(us))
                res.setdefault(m, []).append(us.value)
        print(model, K, H, "  ".join(f"{names[m]} {np.median(v):.2f}" for m, v in res.items()), flush=True)
        e.close()


def probe_stamps(model, K, H, bt="0", nb="0"):
    """Raw stamps of the last rollout launch: s_memtime and s_memrealtime at each wave's start and
    end give the shader clock, the wave lifetimes and the grid timeline (ramp, body, drain)."""
    K, H, bt, nb = int(K), int(H), int(bt), int(nb)
    e = _engine(model, K, H, block_threads=bt, blocks_per_vehicle=nb)
    for _ in range(30):
        e.step(np.array(STATES[model], np.float64))
    print(model, K, H, "block_threads", bt or "default", "nb", nb or "auto", flush=True)
    fn = e._L.mppi_debug_stamps
    fn.restype = C.c_int64
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    buf = np.zeros((1 << 20, 16), np.uint64)
    n = fn(e._h, buf.ctypes.data, buf.shape[0])
    if n > 0:
        x = buf[:n].astype(np.int64)
        clk = x[:, 7] - x[:, 0]                 # shader clock ticks, STAMP(0) .. STAMP(7)
        rt0, rt1 = x[:, 13], x[:, 14]
        life_ns = (rt1 - rt0) * 10.0
        ok = life_ns > 0
        ghz = np.median(clk[ok] / life_ns[ok])
        t0 = rt0.min()
        start_ns, end_ns = (rt0 - t0) * 10.0, (rt1 - t0) * 10.0
        span = end_ns.max()
        print(f"waves {n}: shader clock {ghz:.2f} GHz; grid span {span / 1e3:.2f} us; wave life "
              f"median {np.median(life_ns) / 1e3:.2f} us (p10 {np.percentile(life_ns, 10) / 1e3:.2f}, "
              f"p90 {np.percentile(life_ns, 90) / 1e3:.2f}); last wave start {start_ns.max() / 1e3:.2f} us, "
              f"first wave end {end_ns.min() / 1e3:.2f} us")
        edges = np.linspace(0, span, 21)
        act = [int(((start_ns <= t) & (end_ns > t)).sum()) for t in edges[:-1] + (edges[1] - edges[0]) / 2]
        print("waves resident per 5% of the span:", act, flush=True)
        hw = x[:, 15] & 0xFFFFFFFF
        xcc = (x[:, 15] >> 32) & 0xF
        cu, se, simd = (hw >> 8) & 0xF, (hw >> 13) & 0x7, (hw >> 4) & 0x3
        for c in range(int(xcc.max()) + 1):
            m = xcc == c
            if m.any():
                print(f"  xcc {c}: waves {int(m.sum()):5d}  life median {np.median(life_ns[m]) / 1e3:6.2f} us  "
                      f"end max {end_ns[m].max() / 1e3:6.2f} us  end median {np.median(end_ns[m]) / 1e3:6.2f} us")
        key = (xcc * 8 + se) * 16 + cu
        u, cnt = np.unique(key, return_counts=True)
        per_cu_end = np.array([end_ns[key == k].max() for k in u])
        print(f"  CUs used {len(u)}; waves per CU min {cnt.min()} max {cnt.max()}; per-CU last end "
              f"p10 {np.percentile(per_cu_end, 10) / 1e3:.2f} p50 {np.median(per_cu_end) / 1e3:.2f} "
              f"max {per_cu_end.max() / 1e3:.2f} us; simd ids {np.bincount(simd).tolist()}", flush=True)
    e.close()


def probe_latency(model="arm", K="4096", H="32"):
    """Host-inclusive control-call latency: enqueue (set_state + rollout + finalize) vs wait
    (read_outputs), for the completion-flag poll (default) and MPPI_EVENT_WAIT=1."""
    K, H = int(K), int(H)
    state = np.array(STATES[model], np.float64)
    n = 400
    for mode in ("flag", "event"):
        if mode == "event":
            os.environ["MPPI_EVENT_WAIT"] = "1"
        else:
            os.environ.pop("MPPI_EVENT_WAIT", None)
        e = _engine(model, K, H)
        for _ in range(50):
            e.step(state)
        full, enq, wait = [], [], []
        for _ in range(n):
            t0 = time.perf_counter()
            e.step(state)
            full.append(time.perf_counter() - t0)
        for _ in range(n):
            t0 = time.perf_counter()
            e.set_state(state)
            e.rollout()
            e.finalize()
            t1 = time.perf_counter()
            e.read_outputs()
            t2 = time.perf_counter()
            enq.append(t1 - t0)
            wait.append(t2 - t1)
        q = lambda x, p: np.percentile(np.array(x) * 1e6, p)  # noqa: E731
        print(f"{model} K={K} H={H} wait={mode}: step p50 {q(full, 50):6.1f} us p99 {q(full, 99):6.1f} | split: "
              f"enqueue p50 {q(enq, 50):5.1f} us, read_outputs p50 {q(wait, 50):5.1f} us", flush=True)
        e.close()


def probe_ramp(model="arm", K="4096", H="32"):
    """Per-step time against how long the GPU has been busy: 20-step batches after an idle pause
    and right after sustained bursts of different lengths; then one long run timed in chunks of
    100 steps.  A per-step time that falls with the length of the preceding burst is the GPU's
    clock/power state ramping under sustained load, not the step itself."""
    import torch
    e = _engine(model=model, K=int(K), H=int(H), seed=3)
    e.run_steps(200)
    e.synchronize()

    def batch20():
        torch.cuda.synchronize()
        e.synchronize()
        t0 = time.perf_counter()
        e.run_steps(20)
        torch.cuda.synchronize()
        e.synchronize()
        return (time.perf_counter() - t0) / 20 * 1e6

    res = {}
    for _ in range(5):
        for pre in (0, 200, 1000, 5000, 20000):
            if pre:
                e.run_steps(pre)   # a sustained burst right before the timed batch
            else:
                time.sleep(0.05)   # idle
            res.setdefault(pre, []).append(batch20())
    for pre, v in res.items():
        print(f"{model} K={K} H={H}: 20-step batch after {'50 ms idle' if not pre else f'{pre}-step burst'}: "
              f"median {np.median(v):.2f} us/step  {[round(x, 2) for x in v]}", flush=True)
    time.sleep(0.05)
    chunks = []
    t_prev = time.perf_counter()
    for i in range(60):   # 60 x 100 steps, synchronised per chunk (no idle beyond the sync)
        e.run_steps(100)
        e.synchronize()
        t = time.perf_counter()
        chunks.append((t - t_prev) / 100 * 1e6)
        t_prev = t
    print(f"{model}: per-step time of consecutive 100-step chunks after 50 ms idle: "
          f"{[round(x, 2) for x in chunks]}", flush=True)
    e.close()


def probe_peer_ranks(model="arm", K="512", H="32", Gs="1,2,4,8"):
    """Per-step time of G peer-exchange ranks as engines of this one process (mppi_peer_connect_ptrs),
    every engine's 200-step native batch in flight together, K samples per engine: with small K the
    rollouts hardly contend and the G-rank step over the 1-engine step is the exchange's cost on
    one GPU (G = 1: a plain engine).  Median of 7 batches after a 15 ms heat-up per batch."""
    import torch
    for G in [int(g) for g in Gs.split(",")]:
        es = [_engine(model=model, K=int(K), H=int(H), seed=3, shard_rank=r, shard_count=G) for r in range(G)]
        if G > 1:
            for e in es:
                e.peer_open()
            addrs = [e.peer_region() for e in es]
            for e in es:
                e.peer_connect_ptrs(addrs)
        for e in es:
            e.run_steps(200)
        for e in es:
            e.synchronize()
        ts = []
        for _ in range(7):
            for e in es:
                e.run_steps(2000)   # heat-up
            for e in es:
                e.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for e in es:
                e.run_steps(200)
            for e in es:
                e.synchronize()
            ts.append((time.perf_counter() - t0) / 200 * 1e6)
        bad = sum(bool(e.read_outputs()[2][0].nonfinite) for e in es)
        print(f"{model} K={K}/engine H={H} G={G}: {np.median(ts):.2f} us/step (batches {[round(x, 2) for x in ts]})"
              f"{'  NONFINITE/TIMEOUT on %d engines' % bad if bad else ''}", flush=True)
        for e in es:
            e.close()


def probe_geom(model="wholebody", K="8192", H="64", bpvs="256,512,1024", threads="0"):
    """Rollout / finalize / pair times (HIP events, kernel_timing_ex, median of 7) for each
    blocks-per-vehicle choice (the grid's groups per wave follow from it: K / (bpv * rollouts per
    block)); one engine per choice, created in turn, both orders."""
    res = {}
    bl = [int(b) for b in bpvs.split(",")]
    for order in (bl, bl[::-1]):
        for b in order:
            e = _engine(model, int(K), int(H), blocks_per_vehicle=b, block_threads=int(threads))
            for _ in range(3):
                e.kernel_timing_ex(400)
            xs = [e.kernel_timing_ex(400) for _ in range(7)]
            r = tuple(float(np.median([x[i] for x in xs])) for i in range(3))
            res.setdefault(b, []).append(r)
            print(f"{model} K={K} H={H} blocks/vehicle {b}: rollout {r[0]:.2f} us, finalize {r[1]:.2f}, "
                  f"pair {r[2]:.2f}  [{e.dispatch_info()}]", flush=True)
            e.close()


def probe_peer_soak(model="wholebody", K="8192", H="64", G="2", batches="20", steps="1000"):
    """Soak of the peer exchange: G in-process ranks (mppi_peer_connect_ptrs) run `batches` native
    batches of `steps` steps together; after every batch each rank's sticky timeout word must be 0
    and every rank's u_prev bit-identical to rank 0's.  Prints one line per batch and a verdict."""
    G, nb, ns = int(G), int(batches), int(steps)
    es = [_engine(model=model, K=int(K), H=int(H), seed=3, shard_rank=r, shard_count=G) for r in range(G)]
    for e in es:
        e.peer_open()
    addrs = [e.peer_region() for e in es]
    for e in es:
        e.peer_connect_ptrs(addrs)
    ok = True
    t_all = time.perf_counter()
    for b in range(nb):
        t0 = time.perf_counter()
        for e in es:
            e.run_steps(ns)
        for e in es:
            e.synchronize()
        dt = (time.perf_counter() - t0) / ns * 1e6
        sticky = [e.peer_status(reports=False)[0] for e in es]
        u0 = es[0].get_u_prev()
        same = all(np.array_equal(u0, e.get_u_prev()) for e in es[1:])
        fin = bool(np.isfinite(u0).all())
        ok &= (not any(sticky)) and same and fin
        print(f"batch {b}: {ns} steps, {dt:.2f} us/step, sticky {sticky}, ranks bit-identical {same}, finite {fin}",
              flush=True)
    print(f"{model} K={K} H={H} G={G}: {nb * ns} steps in {time.perf_counter() - t_all:.1f} s: "
          f"{'OK' if ok else 'FAILED'}", flush=True)
    for e in es:
        e.close()
    if not ok:
        sys.exit(1)


def probe_rate(model="arm", K="4096", H="32", calls="200"):
    """Control-call latency against the idle time before each call (bench.py latency_100hz: the
    node ticks at 100 Hz, kinova.py:101).  Phases, in order: back to back; 10 ms sleeps (rospy.Rate);
    10 ms of host spinning (the host thread stays awake, only the GPU idles); 1 ms and 0.1 ms sleeps.
    Sleep-gap latency well above spin-gap latency = the host's wake-up; spin-gap above back-to-back =
    the GPU's idle state.  Each phase prints p50/p90/p99 and its call count, so a rocprofv3 kernel
    trace of this probe splits into the phases by launch order (kernel durations cold vs warm)."""
    K, H, n = int(K), int(H), int(calls)
    state = np.array(STATES[model], np.float64)
    e = _engine(model, K, H)
    for _ in range(100):
        e.step(state)

    import torch
    touch_buf = torch.zeros(16, device="cuda:0")
    touch_stream = torch.cuda.Stream(device=0)

    def touch():   # a tiny kernel on another stream, not waited for: the GPU's queues and link stay busy
        with torch.cuda.stream(touch_stream):
            touch_buf.add_(1.0)

    def run(gap_s, spin, touch_every=0.0, touch_before=0.0):
        lat = []
        for _ in range(n):
            if gap_s:
                if spin or touch_every:
                    t_end = time.perf_counter() + gap_s
                    t_touch = time.perf_counter()
                    while time.perf_counter() < t_end - touch_before:
                        if touch_every and time.perf_counter() >= t_touch:
                            touch()
                            t_touch += touch_every
                        if not spin:
                            time.sleep(min(touch_every, max(0.0, t_end - touch_before - time.perf_counter())))
                else:
                    time.sleep(gap_s - touch_before)
                if touch_before:
                    touch()
                    t_end = time.perf_counter() + touch_before
                    while time.perf_counter() < t_end:
                        pass
            t0 = time.perf_counter()
            e.step(state)
            lat.append(time.perf_counter() - t0)
        return np.array(lat) * 1e6

    for name, gap, spin, te, tb in (("back-to-back", 0.0, False, 0, 0), ("sleep 10 ms", 0.01, False, 0, 0),
                                    ("spin 10 ms", 0.01, True, 0, 0), ("sleep 1 ms", 0.001, False, 0, 0),
                                    ("sleep 0.1 ms", 0.0001, False, 0, 0),
                                    ("spin 10 ms, touch /1ms", 0.01, True, 0.001, 0),
                                    ("spin 10 ms, touch -50us", 0.01, True, 0, 5e-5),
                                    ("sleep 10 ms, touch /1ms", 0.01, False, 0.001, 0),
                                    ("sleep 10 ms, prewarm 100", 0.01, False, 0, 100),
                                    ("sleep 10 ms, prewarm 200", 0.01, False, 0, 200),
                                    ("sleep 10 ms, prewarm 500", 0.01, False, 0, 500),
                                    ("spin 10 ms, prewarm 200", 0.01, True, 0, 200),
                                    ("back-to-back (again)", 0.0, False, 0, 0)):
        pw = tb if tb >= 50 else 0    # rows with an integer >= 50 there: the engine's prewarm window, us
        e.set_prewarm(pw)
        x = run(gap, spin, te, 0 if pw else tb)
        e.set_prewarm(0)
        print(f"{model} K={K} H={H} {name:22s}: calls {x.size}  p50 {np.percentile(x, 50):6.1f} us  "
              f"p90 {np.percentile(x, 90):6.1f}  p99 {np.percentile(x, 99):6.1f}  mean {x.mean():6.1f}", flush=True)
    print(f"dispatch: {e.dispatch_info()}", flush=True)
    e.close()


def probe_rate_split(model="arm", K="4096", H="32", calls="200"):
    """Where the ~7 us between a spin-gap call and a back-to-back call goes (probe_rate: the host
    thread stays awake, only the device side idles 10 ms).  Every row spins 10 ms, then before the
    timed call does one of: nothing; a torch kernel on another stream 5 us before; torch kernels
    every 20 us through the gap; a control call on a second engine (its own AQL queue, same kernels)
    50 us / 5 us before; a control call on the same engine 50 us before (its own queue warm, the
    call's outputs and arguments just touched).  Rows that recover back-to-back latency name the
    state that went cold."""
    K, H, n = int(K), int(H), int(calls)
    state = np.array(STATES[model], np.float64)
    e, e2 = _engine(model, K, H), _engine(model, K, H)
    for _ in range(100):
        e.step(state)
        e2.step(state)

    import torch
    buf = torch.zeros(16, device="cuda:0")
    side = torch.cuda.Stream(device=0)

    def torch_touch():
        with torch.cuda.stream(side):
            buf.add_(1.0)

    L = e._L
    L.mppi_debug_queue_touch.restype = C.c_int32
    L.mppi_debug_queue_touch.argtypes = [C.c_void_p]

    L.mppi_debug_queue_ring.restype = C.c_int32
    L.mppi_debug_queue_ring.argtypes = [C.c_void_p]

    def qring():    # the doorbell again with the last packet's index (mppi_aql step_ring)
        assert L.mppi_debug_queue_ring(e._h) == 0

    def qtouch():   # two one-wave packets on the engine's own AQL queue (mppi_aql step_touch)
        assert L.mppi_debug_queue_touch(e._h) == 0

    def spin(t_end, every=0.0, fn=None):
        t_next = time.perf_counter()
        while time.perf_counter() < t_end:
            if every and time.perf_counter() >= t_next:
                fn()
                t_next += every

    def run(before_s=0.0, fn=None, every=0.0):
        lat = []
        for _ in range(n):
            t_end = time.perf_counter() + 0.01
            if every:
                spin(t_end, every, fn)
            else:
                spin(t_end - before_s)
                if fn:
                    fn()
                spin(t_end)
            t0 = time.perf_counter()
            e.step(state)
            lat.append(time.perf_counter() - t0)
        return np.array(lat) * 1e6

    rows = (("back-to-back", None),
            ("spin 10 ms", dict()),
            ("spin, torch touch -5us", dict(before_s=5e-6, fn=torch_touch)),
            ("spin, torch touch /20us", dict(every=2e-5, fn=torch_touch)),
            ("spin, engine2 call -50us", dict(before_s=5e-5, fn=lambda: e2.step(state))),
            ("spin, engine2 call -5us", dict(before_s=5e-6, fn=lambda: e2.step(state))),
            ("spin, same-engine call -50us", dict(before_s=5e-5, fn=lambda: e.step(state))),
            ("spin, queue touch -20us", dict(before_s=2e-5, fn=qtouch)),
            ("spin, queue touch -50us", dict(before_s=5e-5, fn=qtouch)),
            ("spin, queue touch -100us", dict(before_s=1e-4, fn=qtouch)),
            ("spin, queue touch -200us", dict(before_s=2e-4, fn=qtouch)),
            ("spin, queue touch -300us", dict(before_s=3e-4, fn=qtouch)),
            ("spin, queue touch -500us", dict(before_s=5e-4, fn=qtouch)),
            ("spin, queue touch -0us", dict(before_s=1e-9, fn=qtouch)),
            ("spin, doorbell -50us", dict(before_s=5e-5, fn=qring)),
            ("spin, doorbell -20us", dict(before_s=2e-5, fn=qring)),
            ("spin, doorbell -5us", dict(before_s=5e-6, fn=qring)),
            ("spin, doorbell -0us", dict(before_s=1e-9, fn=qring)),
            ("spin, queue touch /1ms", dict(every=1e-3, fn=qtouch)),
            ("back-to-back (again)", None))
    for name, kw in rows:
        if kw is None:
            lat = []
            for _ in range(n):
                t0 = time.perf_counter()
                e.step(state)
                lat.append(time.perf_counter() - t0)
            x = np.array(lat) * 1e6
        else:
            x = run(**kw)
        print(f"{model} K={K} H={H} {name:30s}: calls {x.size}  p50 {np.percentile(x, 50):6.1f} us  "
              f"p90 {np.percentile(x, 90):6.1f}  p99 {np.percentile(x, 99):6.1f}  mean {x.mean():6.1f}", flush=True)
    e2.close()
    e.close()


def probe_rate_prewarm(model="arm", K="4096", H="32", calls="200", rounds="3", windows="200"):
    """bench.py's 100 Hz loop (latency_at_rate) with the prewarm off and on (mppi_set_prewarm),
    alternating blocks of `calls` for `rounds` rounds per window, so that box noise falls on both:
    per block p50/p90/p99/max, then the pooled percentiles per setting and the touches per call."""
    import bench
    K, H, n, R = int(K), int(H), int(calls), int(rounds)
    state = np.array(STATES[model], np.float64)
    e = _engine(model, K, H)
    for _ in range(100):
        e.step(state)
    wins = [w for w in windows.split(",")]   # "200" sleep between touches, "200s" spin through the window
    pooled = {w: [] for w in ["0"] + wins}
    for r in range(R):
        for w in ["0"] + wins:
            os.environ["MPPI_PREWARM_SPIN"] = "1" if w.endswith("s") else "0"
            e.set_prewarm(int(w.rstrip("s")))
            t0 = e.prewarm()[1]
            x = np.array(bench.latency_at_rate(e, state, n, idle_s=0.02)) * 1e6
            t1 = e.prewarm()[1]
            e.set_prewarm(0)
            pooled[w].append(x)
            print(f"round {r} prewarm {w:>5s}: p50 {np.percentile(x, 50):6.1f} us  p90 {np.percentile(x, 90):6.1f}  "
                  f"p99 {np.percentile(x, 99):6.1f}  max {x.max():6.1f}  touches/call {(t1 - t0) / n:.1f}", flush=True)
    for w, xs in pooled.items():
        x = np.concatenate(xs)
        print(f"pooled prewarm {w:>5s}: calls {x.size}  p50 {np.percentile(x, 50):6.1f} us  p90 {np.percentile(x, 90):6.1f}  "
              f"p99 {np.percentile(x, 99):6.1f}  p99.9 {np.percentile(x, 99.9):6.1f}  mean {x.mean():6.1f}", flush=True)
    e.close()


def probe_store_floor(sizes="1589248,9981952,46170112,369360896", launches="400"):
    """Write-only floor at the rollout's per-launch byte counts (drone C2, arm C3, whole-body C4
    share, fleet C5 share): torch fill_ of a buffer of that many bytes, `launches` back to back
    between one event pair (steps-only, like the rollout's rocprof average), median of 7.  A store
    kernel of the same size cannot finish faster on this box, so rollout_us / floor_us is how far the
    rollout sits from its own store floor (the 8 TB/s peak is not reachable by a write stream)."""
    import torch
    n = int(launches)
    for nbytes in (int(s) for s in sizes.split(",")):
        buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda:0")
        for _ in range(50):
            buf.fill_(1.0)
        torch.cuda.synchronize()
        us = []
        for trial in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(n):
                buf.fill_(float(i))
            b.record()
            b.synchronize()
            us.append(a.elapsed_time(b) * 1e3 / n)
        m = float(np.median(us))
        print(f"store floor {nbytes / 1e6:8.2f} MB: {m:7.2f} us/launch  {nbytes / m / 1e3:7.1f} GB/s  "
              f"(median of 7 x {n} launches)", flush=True)
        del buf


def probe_noise_src(model="arm", K="4096", H="32", n="2000"):
    """Rollout with the noise drawn on the device (Philox + Box-Muller in the prologue) against the
    same rollout reading its noise from HBM (the injected-noise path): n rollouts of each, back to
    back, Philox first.  Run under `rocprofv3 --kernel-trace`: the two halves of the k_rollout
    dispatches are the two modes (same kernel symbol).  Tells what drawing the next step's noise
    off the critical path could save at most."""
    import torch
    K, H, n = int(K), int(H), int(n)
    state = np.array(STATES[model], np.float64)
    for mode in ("philox", "injected"):
        e = _engine(model, K, H, noise=mode)
        e.set_state(state)
        A = e.A
        eps = torch.randn(K * H * A, device="cuda:0", dtype=torch.float32) * 0.1 if mode == "injected" else None
        torch.cuda.synchronize()
        ptr = eps.data_ptr() if eps is not None else 0
        for _ in range(50):
            e.rollout(ptr)
        e.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            e.rollout(ptr)
        e.synchronize()
        print(f"{model} K={K} H={H} {mode:8s}: {n} rollouts, {(time.perf_counter() - t0) / n * 1e6:.2f} us each "
              f"(host-paced; the kernel trace has the device time)", flush=True)
        e.close()


PROBES = {"timeline": probe_timeline, "noise_src": probe_noise_src, "peer_soak": probe_peer_soak, "geom": probe_geom, "batch": probe_batch, "fences": probe_fences, "calls": probe_calls,
          "sequence": probe_sequence, "stamps": probe_stamps, "latency": probe_latency,
          "ramp": probe_ramp, "peer_ranks": probe_peer_ranks, "rate": probe_rate, "rate_split": probe_rate_split, "rate_prewarm": probe_rate_prewarm,
          "store_floor": probe_store_floor}

if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in PROBES:
        sys.exit(__doc__)
    PROBES[sys.argv[1]](*sys.argv[2:])
