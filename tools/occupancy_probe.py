import ctypes, torch
import os
lib = ctypes.CDLL(os.environ.get("GWN_LIB") or "graph-wavenet_amd/gwn_amd/libgwn.so")
torch.cuda.init()
p = torch.cuda.get_device_properties(0)
print(p)
for attr in ["multi_processor_count", "max_threads_per_multi_processor", "shared_memory_per_multiprocessor", "shared_memory_per_block_optin", "regs_per_multiprocessor"]:
    print(attr, getattr(p, attr, None))
for n in (207, 325, 128, 64):
    print("n", n, "fwd blocks/CU", lib.gwn_fused_occupancy(n, 0, 1), "bwd", lib.gwn_fused_occupancy(n, 1, 1))
