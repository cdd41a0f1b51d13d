set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-poolocc}; mkdir -p $O
WGT_DEBUG=1 WGT_POOL=6 timeout -k 10 120 python scripts/pool_probe.py sponza 16 > $O/p6.log 2>&1; cat $O/p6.log | grep -v Warning | tail -3
python - <<'PY'
import ctypes
h=ctypes.CDLL("libamdhip64.so")
class P(ctypes.Structure): _fields_=[("b",ctypes.c_byte*4096)]
for name,attr in [("maxSharedMemoryPerMultiProcessor",74),("sharedMemPerBlock",8)]:
    pass
v=ctypes.c_int()
# hipDeviceAttributeMaxSharedMemoryPerMultiprocessor / hipDeviceAttributeSharedMemPerBlockOptin
for a in range(0,120):
    r=h.hipDeviceGetAttribute(ctypes.byref(v), a, 0)
    if r==0 and v.value in (65536,163840,167936,160*1024): print("attr",a,v.value)
PY
