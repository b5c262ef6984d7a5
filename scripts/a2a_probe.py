"""Is a one-rank RCCL all_to_all_single an exact copy at the engine's region sizes? Fills a send
buffer with a pattern, moves it with all_to_all_single (sync and async), compares.
usage: python scripts/a2a_probe.py MB [MB ...]"""
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29581")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
for mb in [int(x) for x in sys.argv[1:]]:
    n = mb << 20
    send = torch.randint(0, 256, (n + 4096,), dtype=torch.uint8, device="cuda")
    for async_op in (False, True):
        recv = torch.zeros(n + 8192, dtype=torch.uint8, device="cuda")
        w = dist.all_to_all_single(recv[:n], send[:n], [n], [n], async_op=async_op)
        if w is not None:
            w.wait()
        torch.cuda.synchronize()
        bad = (recv[:n] != send[:n]).nonzero()
        first = int(bad[0]) if len(bad) else -1
        print(f"{mb} MB async={async_op}: mismatched bytes {len(bad)} first at {first}, tail untouched "
              f"{bool((recv[n:] == 0).all())}", flush=True)
    del send, recv
    torch.cuda.empty_cache()
dist.destroy_process_group()
