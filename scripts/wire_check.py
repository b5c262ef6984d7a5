"""Probe: pack a large exchange on a wire_all engine and check the buffer's structure on the host
before the tick consumes it. usage: wire_check.py G P L SE ticks"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raftd_amd import Engine  # noqa: E402

G, P, L, SE, T = (int(x) for x in sys.argv[1:6])
R, E = 3, 64
b = Engine(wire_all=1, groups=G, replicas=R, log_capacity=L, payload_bytes=P, max_entries_per_msg=E,
           snapshot_entries=SE)
b.bootstrap()
camp = np.zeros(G * R, np.uint8)
camp[0::R] = 1
pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
buf = None
for t in range(T):
    ins = dict(campaign=camp) if t == 1 else (dict(prop_target=pt, prop_count=pc) if t >= 6 else {})
    sizes = b.wire_plan()
    n = sum(sizes)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 1 << 20) * 3 // 2, dtype=torch.uint8, device="cuda")
    b.wire_pack(buf.data_ptr(), buf.numel())
    b.sync()
    if n > (1 << 30):
        h = buf[:n].cpu().numpy()
        U = 6 * G
        tab = h[:U * 8].view(np.uint64)
        off, cnt = (tab >> 8).astype(np.int64), (tab & 0xFF).astype(np.int64)
        tb = (U * 8 + 255) & ~255
        pos, maxoff, bad = 0, 0, 0
        for u in range(U):
            if off[u] != pos // 16:
                bad += 1
                if bad < 5:
                    print("unit", u, "table off16", off[u], "expected", pos // 16, flush=True)
            p = tb + off[u] * 16
            for k in range(cnt[u]):
                w0 = int(h[p:p + 8].view(np.uint64)[0])
                nn = (w0 >> 32) if (w0 & 0xFF) == 12 else 0
                if nn > 64 or (w0 & 0xFF) not in (4, 7, 12, 13, 14, 15, 16, 17, 18):
                    bad += 1
                    if bad < 5:
                        print("unit", u, "msg", k, "bad header", hex(w0), flush=True)
                    break
                maxoff = max(maxoff, p + 64 + 16 * nn + P * nn)
                p += 64 + nn * (16 + P)
            pos = (p - tb)
        print(f"tick {t}: {n} B, data end {pos + tb}, max payload end {maxoff}, bad {bad}", flush=True)
    b.wire_recv(buf.data_ptr(), sizes)
    b.sync()
    b.tick(**ins)
    b.sync()
    print("tick", t, "ok", n, flush=True)
