"""Host enqueue cost of the bench's train step (config 2, bf16): how long the
Python + ctypes side of one Trainer.train_step takes when the GPU is far
behind (a long sleep kernel queued first, so no call ever waits on the
device), against the step's GPU time.  If the two are close, GPU idle gaps
open wherever the host falls behind.  Usage (GPU): python tools/host_time.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = yaml.safe_load(open(os.path.join(root, "vae_npvc_amd", "conf", "vcc20.yaml")))
cfg.update(compute_dtype="bf16", batch_size=64)
from vae_npvc_amd.trainer.basic import Trainer  # noqa: E402

torch.manual_seed(777)
np.random.seed(777)
tr = Trainer(cfg)
dev = torch.device("cuda", 0)
x = torch.randn(64, 80, 256, device=dev)
y = torch.randint(0, cfg["y_num"], (64, 1), device=dev)
for _ in range(5):
    _, det = tr.train_step((x, y))
dict(det)
torch.cuda.synchronize()

# GPU-bound timing (as bench.py)
t0 = time.perf_counter()
for _ in range(steps):
    _, det = tr.train_step((x, y))
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / steps * 1e3

# host-only: the device is held ~steps x 8 ms behind by a sleep kernel
torch.cuda._sleep(int(steps * 8e-3 * 2.0e9))
host = []
for _ in range(steps):
    t = time.perf_counter()
    _, det = tr.train_step((x, y))
    host.append((time.perf_counter() - t) * 1e3)
t_enq = time.perf_counter()
torch.cuda.synchronize()
print(f"step wall (GPU-bound) {gpu_ms:.3f} ms; host enqueue per step: median {np.median(host):.3f} ms, "
      f"min {min(host):.3f}, max {max(host):.3f}; device still busy {1e3 * (time.perf_counter() - t_enq):.1f} ms "
      f"after the last enqueue (> 0: the host never waited)")
