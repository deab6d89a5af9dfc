"""Per-phase wave timelines of the rollout / finalize kernels (stamps build).
   MPPI_HIP_LIB=.../libmppi_hip_stamps.so MPPI_STAMPS=1 python tools/stamp_probe.py drone 256 32 [threads] [nb]

Besides the averaged phase cycles (printed by the library at close), it reads the raw
stamps of the last rollout launch: s_memtime (shader clock) and s_memrealtime (100 MHz)
at each wave's start and end give the shader clock, the wall-clock wave lifetimes and
the grid timeline (launch ramp, body, drain)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config

model, K, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
bt = int(sys.argv[4]) if len(sys.argv) > 4 else 0
nb = int(sys.argv[5]) if len(sys.argv) > 5 else 0
e = Engine(make_config(model, n_samples=K, n_horizon=H, block_threads=bt, blocks_per_vehicle=nb,
                       state_f64=(model == "arm")))
sd = {"arm": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7,
      "drone": [0, 0, 1, 0, 0, 0], "wholebody": [0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 10}[model]
e.set_target([0.1, 0.4, 1.6], [-0.5, -0.5, 0.5, -0.5])
for i in range(30):
    e.step(np.array(sd, np.float64))
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
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    simd = (hw >> 4) & 0x3
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
