"""Load order of the HIP runtime in one Python process: the library first
(its backend loads /opt/rocm's runtime), then torch -- or torch first, then
the library (whose backend then binds to torch's, same soname).  Prints what
each sees and which runtimes the process mapped.  The library is loaded
through ctypes directly, so the package's own torch-first step
(sha1chunk._one_hip_runtime) does not hide the lib-first case.

    python3 tools/order_probe.py lib-first|torch-first
"""
import ctypes
import os
import sys

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "congestion-control-with-bittorren_amd", "libsha1chunk.so")


def lib_devices():
    return ctypes.CDLL(LIB).sha1chunk_device_count()


order = sys.argv[1]
if order == "lib-first":
    print("lib devices", lib_devices(), flush=True)
    import torch
    print("torch available", torch.cuda.is_available(), flush=True)
else:
    import torch
    print("torch available", torch.cuda.is_available(), flush=True)
    print("lib devices", lib_devices(), flush=True)
maps = open("/proc/self/maps").read()
print(sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "hsa-runtime" in l}))
