"""Probe: create / destroy CU-masked HIP streams in a loop (does queue creation stall?)."""
import ctypes as C, time, sys
h = C.CDLL("libamdhip64.so")
n = C.c_int()
print("count", h.hipGetDeviceCount(C.byref(n)), n.value, flush=True)
h.hipSetDevice(0)
ncu = C.c_int()
h.hipDeviceGetAttribute(C.byref(ncu), 16, 0)  # hipDeviceAttributeMultiprocessorCount
print("cus", ncu.value, flush=True)
words = (ncu.value + 31) // 32
mask = (C.c_uint32 * words)(*([0xFFFFFFFF] * words))
mask[0] &= ~1
t = time.time()
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 300):
    s = C.c_void_p()
    rc = h.hipExtStreamCreateWithCUMask(C.byref(s), words, mask)
    s2 = C.c_void_p()
    rc2 = h.hipStreamCreateWithFlags(C.byref(s2), 1)
    h.hipStreamSynchronize(s); h.hipStreamSynchronize(s2)
    h.hipStreamDestroy(s); h.hipStreamDestroy(s2)
    if i % 50 == 0:
        print(i, rc, rc2, round(time.time() - t, 3), flush=True)
print("done", round(time.time() - t, 3), flush=True)
