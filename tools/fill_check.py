#!/usr/bin/env python3
"""Where the product fill differs from the oracle's (diagnostic): config 2 through cts_fill, first differing bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import oracle
from ctstraffic_amd import Engine, workload as W

with Engine(0) as e:
    for n, hint in ((4096, 65536), (64, 65536), (5, 65536), (4096, 0)):
        w = W.tcp_resident(n_buffers=n, corrupt_rate=0)
        arena = torch.zeros(w.arena_bytes, dtype=torch.uint8, device="cuda")
        d = torch.from_numpy(w.descs.view(np.uint8).copy()).cuda()
        e.fill(arena, d, max_length_hint=hint)
        torch.cuda.synchronize()
        got = arena.cpu().numpy()
        exp = np.zeros_like(got)
        oracle.fill(exp, w.descs)
        bad = np.nonzero(got != exp)[0]
        print(n, hint, "bad bytes", bad.size, "first", bad[:4].tolist(), "bufs", np.unique(bad // 65536)[:10].tolist(),
              "got", got[bad[:4]].tolist(), "exp", exp[bad[:4]].tolist(), flush=True)
