#!/usr/bin/env python3
"""Can two RCCL ranks share one GPU? (bench.py's N > 1 collectives could then be rehearsed on a 1-GPU box.)
Two spawned ranks init "nccl" on cuda:0 and all-reduce one int64; prints one JSON line with what happened.
usage: timeout -k 10 90 python tools/rccl_same_gpu_probe.py"""
import json
import os
import socket
import sys

import torch.multiprocessing as mp


def rank_main(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2", RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        import datetime

        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=2, timeout=datetime.timedelta(seconds=40),
                                device_id=torch.device("cuda:0"))
        t = torch.tensor([rank + 1], dtype=torch.int64, device="cuda:0")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        q.put((rank, "ok", int(t.item())))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, "error", repr(e)[:400]))


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = []
    for _ in range(2):
        try:
            out.append(q.get(timeout=70))
        except Exception as e:
            out.append(("?", "timeout", repr(e)))
            break
    for p in ps:
        p.join(10)
        if p.is_alive():
            p.kill()
    print(json.dumps({"results": out, "exitcodes": [p.exitcode for p in ps]}))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
