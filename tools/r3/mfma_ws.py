"""Wait states between an MFMA and the next VALU/VMEM/DS read of its result
(diagnostic).  Counts issued instructions along the layout order inside each
basic block (s_nop N = N+1), the way the compiler's hazard recognizer does.
usage: python tools/r3/mfma_ws.py <listing.s> <kernel symbol>"""
import re
import sys
from collections import Counter


def regs(tok):
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"-?\|?([va])(\d+)\|?", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def main(path, sym):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    last = {}          # reg -> (ws counter at mfma issue, text)
    ws = 0
    hist = Counter()
    low = []
    for l in lines[st + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB"):
                last.clear()          # block boundary: be conservative, restart
            continue
        op, _, rest = s.partition(" ")
        ops = [t.strip() for t in rest.split(",")] if rest else []
        if op.startswith("s_nop"):
            ws += int(ops[0]) + 1
            continue
        if op.startswith("v_mfma"):
            # srcC chaining into another MFMA is hardware-forwarded: skip reads by MFMAs
            for r in regs(ops[0]):
                last[r] = (ws, s)
            ws += 1
            continue
        srcs = set()
        first = 0 if op.startswith(("ds_write", "global_store", "buffer_store")) else 1
        for t in ops[first:]:
            srcs |= regs(t)
        for r in srcs:
            if r in last:
                d = ws - last[r][0] - 1
                hist[d] += 1
                if d <= 8:
                    low.append((d, s, last[r][1]))
                del last[r]
        if op.startswith(("v_", "ds_read", "buffer_load", "global_load")) and ops:
            for r in regs(ops[0]):
                last.pop(r, None)
        ws += 1
    print("wait states MFMA -> first read of its result (histogram, first 20 bins):")
    print(sorted(hist.items())[:20])
    print(f"{len(low)} reads at <= 8 wait states")
    for d, a, b in low[:12]:
        print(f"  {d}: {a}   <- {b}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
