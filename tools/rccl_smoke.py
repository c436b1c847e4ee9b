"""RCCL world-size-1 smoke: init the nccl process group on cuda:0 and run one all_reduce and
one all_gather_into_tensor, printing each step (debug aid for tests/test_gpu_rccl.py)."""
import os
import sys
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
t0 = time.time()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
print(f"[{time.time() - t0:.1f}s] init nccl", flush=True)
kw = {"device_id": dev} if os.environ.get("RS_DEVICE_ID", "1") == "1" else {}
dist.init_process_group("nccl", rank=0, world_size=1, **kw)
print(f"[{time.time() - t0:.1f}s] init done, backend {dist.get_backend()}", flush=True)
x = torch.arange(16, device=dev, dtype=torch.float32)
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"[{time.time() - t0:.1f}s] all_reduce ok {x[:4].tolist()}", flush=True)
y = torch.empty(1, 16, device=dev, dtype=torch.uint8)
dist.all_gather_into_tensor(y, x.to(torch.uint8))
torch.cuda.synchronize()
print(f"[{time.time() - t0:.1f}s] all_gather ok", flush=True)
dist.destroy_process_group()
print(f"[{time.time() - t0:.1f}s] done", flush=True)
sys.exit(0)
