"""c3 device-output path with DPF_AMD_TRACE_HOST phase marks (GPU box):
    DPF_AMD_TRACE_HOST=1 python tools/trace_c3.py 2> trace.log"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_configs as B  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(B.c3(dev, 4), flush=True)
