"""hipMalloc / hipFree / hipHostMalloc cost on the box for add_tracks-sized buffers (ctypes on
libamdhip64, no torch)."""
import ctypes as C
import time

hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipFree.argtypes = [C.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
p = C.c_void_p()
assert hip.hipMalloc(C.byref(p), 1 << 20) == 0
hip.hipFree(p)
for mb in (1, 4, 16, 64, 128):
    ts, tf = [], []
    for _ in range(10):
        t = time.perf_counter()
        assert hip.hipMalloc(C.byref(p), mb << 20) == 0
        ts.append(time.perf_counter() - t)
        t = time.perf_counter()
        hip.hipFree(p)
        tf.append(time.perf_counter() - t)
    ts.sort(); tf.sort()
    print(f"{mb:4d} MiB hipMalloc median {ts[5]*1e6:8.1f} us  hipFree median {tf[5]*1e6:8.1f} us")
