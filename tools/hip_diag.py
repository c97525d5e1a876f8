"""Tiny diagnostic: which HIP runtime the process maps, and a context create."""
import ctypes
import torch

print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
x = torch.zeros(4, device="cuda")
from multilinear_amd import device as D  # noqa: E402

L = D.lib()
h = ctypes.c_void_p()
rc = L.mlh_context_create(0, None, ctypes.byref(h))
print("mlh_context_create rc", rc)
for line in open("/proc/self/maps"):
    if "amdhip" in line or "hsa-runtime" in line:
        print(line.split()[-1])
