"""Diagnose HIP runtime sharing between torch and librtamd.so in one process."""
import re
import sys

order = sys.argv[1]
def libs():
    maps = open('/proc/self/maps').read()
    return sorted(set(l for l in re.findall(r'(/\S+\.so[\.\d]*)', maps) if re.search('amdhip|hsa-runtime', l)))
if order == "torch_first":
    import torch
    print("torch count", torch.cuda.device_count(), flush=True)
    x = torch.zeros(4, device="cuda:0")
    import ctypes
    L = ctypes.CDLL('raytracert_amd/librtamd.so')
    n = ctypes.c_int32(); L.rt_device_count(ctypes.byref(n)); print("rt count", n.value)
    print(libs())
    y = torch.ones(4, device="cuda:0"); print("torch ok", float(y.sum()))
elif order == "torch_import_only":
    import torch
    import ctypes
    L = ctypes.CDLL('raytracert_amd/librtamd.so')
    n = ctypes.c_int32(); L.rt_device_count(ctypes.byref(n)); print("rt count", n.value)
    print(libs())
    y = torch.ones(4, device="cuda:0"); print("torch ok", float(y.sum()))
else:
    import ctypes
    L = ctypes.CDLL('raytracert_amd/librtamd.so')
    n = ctypes.c_int32(); L.rt_device_count(ctypes.byref(n)); print("rt count", n.value)
    import torch
    print(libs())
    y = torch.ones(4, device="cuda:0"); print("torch ok", float(y.sum()))
