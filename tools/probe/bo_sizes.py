"""(probe) dmabuf fd size vs hipMemGetAddressRange size for hipMalloc / torch allocations of
several sizes: do allocations with a buffer object of their own export exactly their size?"""
import ctypes
import os
import json
import torch

hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipMemGetAddressRange.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(sz), vp]
hip.hipMemGetHandleForAddressRange.argtypes = [ctypes.POINTER(ctypes.c_int), vp, sz, ctypes.c_int, ctypes.c_ulonglong]


def probe(p, tag):
    base, size = vp(), sz()
    assert hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), vp(p)) == 0
    fd = ctypes.c_int(-1)
    rc = hip.hipMemGetHandleForAddressRange(ctypes.byref(fd), base, size, 1, 0)
    end = -1
    if rc == 0:
        end = os.lseek(fd.value, 0, os.SEEK_END)
        os.close(fd.value)
    print(json.dumps({"tag": tag, "ptr": hex(p), "base": hex(base.value), "range": size.value, "fd_size": end,
                      "rc": rc}), flush=True)


torch.cuda.init()
for b in (4 << 10, 64 << 10, 1 << 20, (1 << 20) + 4096, 2 << 20, 3 << 20, (5 << 20) + 12345, 64 << 20):
    p = vp()
    assert hip.hipMalloc(ctypes.byref(p), b) == 0
    probe(p.value, f"hipMalloc {b}")
for k in range(6):
    n = (1 << 18) + k * (1 << 19)
    t = torch.empty(n, dtype=torch.float32, device="cuda")
    probe(t.data_ptr(), f"torch f32 x {n}")

# ROCr's view of the same allocations (the identity the engine's export check uses)
hsa = ctypes.CDLL("libhsa-runtime64.so")


class PtrInfo(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_int), ("agentBaseAddress", ctypes.c_void_p),
                ("hostBaseAddress", ctypes.c_void_p), ("sizeInBytes", ctypes.c_size_t), ("userData", ctypes.c_void_p),
                ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32), ("registered", ctypes.c_bool)]


hsa.hsa_amd_pointer_info.argtypes = [vp, ctypes.POINTER(PtrInfo), vp, vp, vp]
for b in (4 << 10, 64 << 10, 1 << 20, 3 << 20):
    p = vp()
    assert hip.hipMalloc(ctypes.byref(p), b) == 0
    info = PtrInfo()
    info.size = ctypes.sizeof(PtrInfo)
    rc = hsa.hsa_amd_pointer_info(p, ctypes.byref(info), None, None, None)
    fd = ctypes.c_int(-1)
    hip.hipMemGetHandleForAddressRange(ctypes.byref(fd), p, b, 1, 0)
    end = os.lseek(fd.value, 0, os.SEEK_END)
    os.close(fd.value)
    print(json.dumps({"tag": f"hsa hipMalloc {b}", "ptr": hex(p.value), "rc": rc, "type": info.type,
                      "agent_base": hex(info.agentBaseAddress or 0), "hsa_size": info.sizeInBytes, "fd_size": end,
                      "names_itself": (info.agentBaseAddress == p.value and end == info.sizeInBytes)}), flush=True)
