"""VERDICT r05 item 5 (r04f's misrouted header): for every inlined `send` of control_slow_kernel<5> in the
optimized device IR of a build variant, check that the outbox plane index (dst) in the header's store
address is the header's own `to` - 1 (raftgpu_control.h `send`: one variable gives both).
Usage (CPU only; the r05h diagnostic sources, commit d7502dd):
  hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -DRG_CTL_R=5 -DRG_AB_CTL2D -DRG_AB_SV_SEND \
        --cuda-device-only -S -emit-llvm raftgpu_ctl.hip -o sv_send.ll
  awk '/^define.*control_slow_kernelILi5/{f=1} f{print} f&&/^}/{exit}' sv_send.ll > slow.ll
  python3 scripts/ir_send_check.py slow.ll
A site is the `v_mov_b32 $0, $0` that launders the slot (RG_AB_SV_SEND) followed by the plane address
(slot * 5 + dst) and the first header store. Sites whose word 0 or dst is a phi over several sends
(merged tails, loop-carried destinations) are reported as not parsed. A "to=X+256" line is the reject
bit (1 << 24) of a reply, not a destination: those are consistent too.
Prints one line per send site and a summary."""
import re, sys
lines = open(sys.argv[1]).read().split("\n")
defs = {}
for i, ln in enumerate(lines):
    m = re.match(r"\s+(%[\w.]+) = (.*)", ln)
    if m:
        defs[m.group(1)] = (i, m.group(2))

def canon(v, depth=0):
    """A canonical form: through zext/trunc/phis whose incomings agree."""
    if depth > 12 or not v.startswith("%"):
        return v
    d = defs.get(v)
    if not d:
        return v
    e = d[1]
    m = re.match(r"(zext|trunc|sext)( nneg| nuw| nsw)* \w+ ([%\w.]+) to \w+", e)
    if m:
        return canon(m.group(3), depth + 1)
    m = re.match(r"phi \w+ (.*)", e)
    if m:
        inc = re.findall(r"\[ ([^,]+), %[\w.]+ \]", m.group(1))
        cs = {canon(x.strip(), depth + 1) for x in inc}
        if len(cs) == 1:
            return cs.pop()
        return v
    return v

ok = bad = unk = 0
for i, ln in enumerate(lines):
    if 'v_mov_b32 $0, $0' not in ln:
        continue
    L = ln.split("=")[0].strip()
    win = lines[i:i + 40]
    txt = "\n".join(win)
    # zext of the laundered slot, * R (5), + dst
    mz = re.search(r"(%[\w.]+) = zext i32 " + re.escape(L) + r" to i64", txt)
    if not mz:
        unk += 1; print(i + 1, "no zext"); continue
    mm = re.search(r"(%[\w.]+) = mul nuw nsw i64 " + re.escape(mz.group(1)) + r", 5", txt)
    if not mm:
        unk += 1; print(i + 1, "no mul"); continue
    ma = re.search(r"= add nuw nsw i64 (?:" + re.escape(mm.group(1)) + r", ([%\w.\-]+)|([%\w.\-]+), " + re.escape(mm.group(1)) + ")", txt)
    if not ma:
        unk += 1; print(i + 1, "no add"); continue
    dst = ma.group(1) or ma.group(2)
    # the header word 0: the first store after the launder
    ms = re.search(r"store i64 ([%\w.\-]+), ptr addrspace\(1\) (%[\w.]+)", txt)
    w0 = ms.group(1)
    # find `to`: walk the or-chain of w0 for a shl by 16 or a constant with bits 16..23
    to = None
    stack = [w0]
    seen = set()
    while stack and to is None:
        v = stack.pop()
        if v in seen:
            continue
        seen.add(v)
        if not v.startswith("%"):
            c = int(v)
            if (c >> 16) & 0xFF:
                to = ("const", (c >> 16) & 0xFF)
            continue
        d = defs.get(v)
        if not d:
            continue
        e = d[1]
        m = re.match(r"shl (?:nuw |nsw )*i\d+ ([%\w.]+), 16", e)
        if m:
            to = ("var", m.group(1), 0)
            break
        m = re.match(r"(?:or|add)(?: disjoint| nuw| nsw)* i\d+ ([%\w.\-]+), ([%\w.\-]+)", e)
        if m:
            a, b = m.group(1), m.group(2)
            # (x << 16) + k·65536 + type: to = x + k
            for x, y in ((a, b), (b, a)):
                if x.startswith("%") and re.match(r"shl (?:nuw |nsw )*i\d+ ([%\w.]+), 16", defs.get(x, (0, ""))[1]) and not y.startswith("%"):
                    to = ("var", re.match(r"shl (?:nuw |nsw )*i\d+ ([%\w.]+), 16", defs[x][1]).group(1), (int(y) >> 16) & 0xFF)
            stack += [a, b]
            continue
        m = re.match(r"zext (?:nneg )*i\d+ ([%\w.]+) to i64", e)
        if m:
            stack.append(m.group(1))
    if to is None:
        unk += 1; print(i + 1, "to?", w0); continue
    if to[0] == "const":
        good = canon(dst) == str(to[1] - 1)
        desc = f"to={to[1]} dst={canon(dst)}"
    else:
        # to = X + k  ⇒ dst must be X + k - 1
        X, k = to[1], to[2]
        cx = canon(X)
        if k == 1:
            good = canon(dst) == cx
        else:
            dd = defs.get(canon(dst), (0, ""))[1]
            good = bool(re.match(r"add (?:nuw |nsw )*i\d+ " + re.escape(cx) + r", " + str(k - 1) + "$", dd)) or (k - 1 == 0 and canon(dst) == cx)
        desc = f"to={cx}+{k} dst={canon(dst)}"
    print(i + 1, "OK " if good else "BAD", desc)
    ok += good; bad += not good
print(f"sends: {ok} consistent, {bad} inconsistent, {unk} not parsed")
