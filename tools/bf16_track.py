"""Print the bf16 engine's loss dict next to the fp32 oracle's for 3 steps
(the test_bf16_step_tracks_oracle setting)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.helpers import cfg_of, make_trainer  # noqa: E402
from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict  # noqa: E402

for dt in ("bf16", "fp32"):
    cfg = cfg_of("vcc20", compute_dtype=dt)
    B, T = 4, 128
    tr = make_trainer(cfg, 78)
    orc = OracleTrainer(dict(cfg), seeded_state_dict(cfg, 78))
    torch.manual_seed(3)
    np.random.seed(3)
    for s in range(3):
        x, y = seeded_batch(cfg, B, T, 100 + s)
        torch.manual_seed(10 + s)
        _, do = orc.train_step((x, y))
        torch.manual_seed(10 + s)
        _, dg = tr.train_step((x.cuda(), y.cuda()))
        dg = dict(dg)
        print(dt, s, {k: round(v, 4) for k, v in dg.items()}, {k: round(v, 4) for k, v in do.items()}, flush=True)
