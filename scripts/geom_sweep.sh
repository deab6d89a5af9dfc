export TMPDIR=/tmp
timeout -k 10 200 python tools/geom_sweep.py wholebody 8192 64 1024,512,256,128 512,256 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/geom_sweep.py arm 4096 32 256,128,64 512,256 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/geom_sweep.py drone 4096 32 256,128,64 512,256 2>&1 | grep -v amdgpu.ids || exit 1
