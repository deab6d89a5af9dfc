export TMPDIR=/tmp
GEOM_V=8 timeout -k 10 200 python tools/geom_sweep.py wholebody 8192 64 128,64,32 512 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/geom_sweep.py wholebody 65536 64 4096,2048,1024,512 512 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/geom_sweep.py wholebody 8192 64 512,384,256 512 2>&1 | grep -v amdgpu.ids || exit 1
