"""Diagnostic: does torch's HIP runtime initialise after an lb_ctx exists?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
order = sys.argv[1] if len(sys.argv) > 1 else "ctx_first"
import torch  # noqa: E402

from lodestar_amd.native import Device  # noqa: E402

if order == "torch_first":
    x = torch.zeros(4, device="cuda")
    print("torch ok first", x.sum().item(), flush=True)
    d = Device(0)
    print("ctx ok", flush=True)
else:
    d = Device(0)
    print("ctx ok", flush=True)
    try:
        x = torch.zeros(4, device="cuda")
        print("torch ok after ctx", x.sum().item(), flush=True)
    except Exception as e:
        print("torch FAILED after ctx:", e, flush=True)
d.close()
