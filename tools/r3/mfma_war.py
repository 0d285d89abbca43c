"""WAR distances: wait states from an MFMA that READS a VGPR (srcA/B/C) to the
next non-MFMA instruction that WRITES it (diagnostic; layout order inside
basic blocks, s_nop N = N+1).
usage: python tools/r3/mfma_war.py <listing.s> <kernel symbol> [max_print]"""
import re
import sys
from collections import Counter

from mfma_ws import regs


def main(path, sym, nprint=10):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    rd = {}            # reg -> (ws at MFMA issue, text)
    ws = 0
    hist = Counter()
    low = []
    for l in lines[st + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB"):
                rd.clear()
            continue
        op, _, rest = s.partition(" ")
        ops = [t.strip() for t in rest.split(",")] if rest else []
        if op.startswith("s_nop"):
            ws += int(ops[0]) + 1
            continue
        if op.startswith("v_mfma"):
            for t in ops[1:]:
                for r in regs(t):
                    if r[0] == "v":
                        rd[r] = (ws, s)
            ws += 1
            continue
        if ops and (op.startswith(("v_", "ds_read", "buffer_load", "global_load"))
                    and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane"))):
            for r in regs(ops[0]):
                if r in rd:
                    d = ws - rd[r][0] - 1
                    hist[d] += 1
                    low.append((d, s, rd[r][1]))
                    del rd[r]
        ws += 1
    low.sort(key=lambda x: x[0])
    print("MFMA source read -> overwrite, wait states (first 16 bins):", sorted(hist.items())[:16])
    for d, a, b in low[:nprint]:
        print(f"  {d}: {a}   <- {b}")


if __name__ == "__main__":
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 10)
