"""Diagnostic: the host's per-call cost of the Python -> ctypes path of a step, against a trivial C
function with mppi_step's signature (so no GPU work is timed), and with torch imported and CUDA
initialised as in bench.py.  Usage: python profiles/ubench/callcost.py"""
import ctypes as C
import os
import subprocess
import sys
import tempfile
import time

src = "#include <stdint.h>\nint triv(void* c, int p, uint64_t s, void* o) { return p == 7 ? 1 : 0; }\n"
d = tempfile.mkdtemp()
open(os.path.join(d, "t.c"), "w").write(src)
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", os.path.join(d, "t.c"), "-o", os.path.join(d, "t.so")], check=True)
lib = C.CDLL(os.path.join(d, "t.so"))
f = lib.triv
f.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_void_p]
f.restype = C.c_int
ctx = C.c_void_p(1234)
out = C.byref(C.c_int(0))
PROJ = {"3d": 3, "2d": 2}


class E:
    def __init__(s):
        s._f, s.ctx, s._o = f, ctx, out

    def step(s, proj="3d", step=0, copy=True):
        rc = s._f(s.ctx, PROJ[proj], int(step), s._o)
        if rc != 0:
            raise RuntimeError
        return None


def run(tag):
    e = E()
    n = 200000
    t = time.perf_counter()
    for i in range(n):
        e.step("3d", i, copy=False)
    a = (time.perf_counter() - t) / n * 1e6
    t = time.perf_counter()
    for i in range(n):
        f(ctx, 3, i, out)
    b = (time.perf_counter() - t) / n * 1e6
    print(f"{tag}: Engine.step path {a:.2f} us/call, bare ctypes {b:.2f} us/call")


run("plain python")
if len(sys.argv) < 2:
    import torch
    torch.cuda.init()
    x = torch.ones(4, device="cuda")
    torch.cuda.synchronize()
    run("torch + CUDA initialised")
    hip = C.CDLL("libamdhip64.so")
    n = 100000
    t = time.perf_counter()
    for i in range(n):
        hip.hipSetDevice(0)
    a = (time.perf_counter() - t) / n * 1e6
    dev = C.c_int(0)
    t = time.perf_counter()
    for i in range(n):
        hip.hipGetDevice(C.byref(dev))
    b = (time.perf_counter() - t) / n * 1e6
    print(f"hipSetDevice(0) {a:.2f} us/call, hipGetDevice {b:.2f} us/call (ctypes included)")
