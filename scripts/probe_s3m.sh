export TMPDIR=/tmp
timeout -k 10 100 python tools/geom_sweep.py arm 4096 32 0 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/geom_sweep.py drone 4096 32 0 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/geom_sweep.py wholebody 8192 64 0 0 2>&1 | grep -v amdgpu.ids || exit 1
GEOM_V=8 timeout -k 10 100 python tools/geom_sweep.py wholebody 8192 64 0 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 100 python tools/geom_sweep.py quadrotor 4096 32 0 0 2>&1 | grep -v amdgpu.ids || exit 1
