"""Probe: how does the HIP runtime run hipLaunchHostFunc callbacks?

Enqueues one host function on each of two streams; each sleeps 0.4 s and
records its OS thread id and start/end time.  If the two callbacks overlap
in time the runtime runs host functions of different streams concurrently
(one callback thread per stream / a pool); if they serialise, a host
function that blocks on a peer process stalls every other stream's host
functions in this process (what a host-staged collective must respect).
Run: python scripts/probe_hostfn.py"""
import ctypes
import os
import threading
import time

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
log = []


def fn(arg):
    t0 = time.time()
    time.sleep(0.4)
    log.append((int(arg or 0), threading.get_native_id(), t0, time.time()))


cb = CB(fn)
lib.hipLaunchHostFunc.argtypes = [ctypes.c_void_p, CB, ctypes.c_void_p]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
t = time.time()
for i, s in enumerate((s1, s2)):
    r = lib.hipLaunchHostFunc(ctypes.c_void_p(s.cuda_stream), cb, ctypes.c_void_p(i + 1))
    assert r == 0, r
torch.cuda.synchronize()
time.sleep(0.1)
main_tid = threading.get_native_id()
for a, tid, t0, t1 in sorted(log):
    print(f"cb{a}: tid={tid} (main {main_tid}) start={t0 - t:.3f}s end={t1 - t:.3f}s")
ov = len(log) == 2 and min(log[0][3], log[1][3]) > max(log[0][2], log[1][2])
print("HOSTFN_CONCURRENT" if ov else "HOSTFN_SERIAL", f"total={time.time() - t:.3f}s")
