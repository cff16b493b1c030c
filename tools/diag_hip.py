"""Diagnose HIP runtime / device visibility from the library (GPU box)."""
import ctypes, os, sys
order = sys.argv[1] if len(sys.argv) > 1 else "lib-first"
lib_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "leveldb-kv-separation_amd", "liblvkv_crc32c.so")
if order == "torch-first":
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
L = ctypes.CDLL(lib_path)
L.lvkv_device_groups.restype = ctypes.c_int
L.lvkv_last_hip_error.restype = ctypes.c_int
g = L.lvkv_device_groups()
print(order, "groups", g, "hip err", L.lvkv_last_hip_error())
if order == "lib-first":
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
    g = L.lvkv_device_groups()
    print("after torch: groups", g, "hip err", L.lvkv_last_hip_error())
for ln in open("/proc/self/maps"):
    if "amdhip64" in ln or "hsa-runtime" in ln:
        print(ln.split()[-1])
print({k: v for k, v in os.environ.items() if "HIP" in k or "ROCR" in k or "HSA" in k or "CUDA" in k})
