"""Worker of test_gpu_cluster's chunked-exchange test: a one-rank nccl group moves byte regions
with raftd_amd.cluster.all_to_all_bytes — small forced chunks over ragged regions, then one
1.5 GB region at the default chunk (RCCL 2.26.6's single all_to_all_single corrupted it)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from raftd_amd.cluster import a2a_chunks, all_to_all_bytes, exchange_sizes, p2p_regions  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
torch.cuda.set_stream(torch.cuda.Stream())
for n, chunk, async_op in ((3_000_001, 1 << 20, False), (3_000_001, 1 << 20, True), (0, 1 << 20, False),
                           (1_500 << 20, None, True)):
    send = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device="cuda")
    recv = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    rs, biggest = exchange_sizes([n])
    kw = dict(chunk=chunk) if chunk else {}
    k = a2a_chunks(biggest, **kw)
    h = all_to_all_bytes(send, [n], recv, rs, async_op=async_op, nchunks=k, **kw)
    if h is not None:
        h.wait()
    torch.cuda.synchronize()
    assert rs == [n] and biggest == n
    assert torch.equal(recv[:n], send[:n]) and bool((recv[n:] == 0).all()), (n, chunk, async_op)
    print(f"ok {n} bytes in {k} calls", flush=True)
    del send, recv
# the exchange's point-to-point path (cluster.p2p_regions, what DistEngine runs on nccl at N > 1), its
# region to this rank forced through isend / irecv pieces: a region laid out past the receive regions
# (send_offs, as _Half packs them), ragged piece counts, sync and async
for n, chunk, async_op in ((3_000_001, 1 << 20, False), (5_000_000, 1 << 21, True), (16, 1 << 20, False)):
    base = torch.randint(0, 256, (2 * n + 4096,), dtype=torch.uint8, device="cuda")
    so = ((n + 255) // 256 * 256 + 512,)  # the send region after the receive area
    recv = base  # one buffer: receive regions at the front
    want = base[so[0]:so[0] + n].clone()
    h = p2p_regions(base, [n], recv, [n], async_op=async_op, chunk=chunk, send_offs=so, self_p2p=True)
    if h is not None:
        h.wait()
    torch.cuda.synchronize()
    assert torch.equal(recv[:n], want), (n, chunk, async_op)
    print(f"ok p2p {n} bytes in pieces of {chunk}", flush=True)
dist.destroy_process_group()
print("a2a chunks ok", flush=True)
